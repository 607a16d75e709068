#!/bin/bash
# One GPU-box pass: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash / timeout stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
STEPS=${STEPS:-50}
run() {  # run <name> <timeout> cmd...; aborts on crash/timeout
    local name=$1 to=$2; shift 2
    echo "== $name"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abort after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps "$STEPS" --warmup 10 --cpu-seconds 8
if [ "${PROFILE:-1}" = "1" ]; then
  run rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
fi
echo done

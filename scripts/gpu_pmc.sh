#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only; no sys/runtime trace).
#   TAG=x [PROG="python scripts/kbench.py --steps 5"] bash scripts/gpu_pmc.sh "C1 C2" "C3 C4" ...
# PROG is run directly after `--` (no env/bash hops); set MBOTS_LIB in the
# environment to profile an A/B build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pmc}
PROG=${PROG:-python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-kernel-timing}
i=0
for counters in "$@"; do
  i=$((i+1))
  echo "== pass $i: $counters"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters --output-format csv \
      -d gpurun_out/${TAG}_p$i -o run -- $PROG > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/${TAG}_p$i.log; exit $rc; fi
done
echo done

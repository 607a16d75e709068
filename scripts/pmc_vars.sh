#!/bin/bash
# One PMC pass per build_var/libmbots_*.so variant (instruction mix of each).
#   bash scripts/pmc_vars.sh "C1 C2 ..." [kbench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
counters=$1; shift
for lib in build_var/libmbots_*.so; do
  v=$(basename $lib .so); v=${v#libmbots_}
  MBOTS_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters --output-format csv \
      -d gpurun_out/pv_${v}_p1 -o run -- python scripts/run_variant.py scripts/kbench.py --steps 5 --warmup 20 --no-kernel-timing "$@" \
      > gpurun_out/pv_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/pv_$v.log; exit 1; }
  echo "== $v"; python scripts/pmc_summary.py gpurun_out/pv_$v | grep -A12 "^${KGREP:-sensor}"
done

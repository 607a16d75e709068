#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only; no sys/runtime trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pmc}
ARGS=${ARGS:---steps 10 --warmup 5 --no-cpu-baseline --no-kernel-timing}
i=0
for counters in "$@"; do
  i=$((i+1))
  echo "== pass $i: $counters"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters --output-format csv \
      -d gpurun_out/${TAG}_p$i -o run -- python bench.py $ARGS > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/${TAG}_p$i.log; exit $rc; fi
done
echo done

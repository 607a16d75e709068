#!/bin/bash
# GPU box: the -m gpu suite (one process), then a short bench.  Each GPU step
# has its own limit; a failure or timeout ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${SEL:-}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread $SEL \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
  rc=$?; tail -3 gpurun_out/bench.log; exit $rc
fi

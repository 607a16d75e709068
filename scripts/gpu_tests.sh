#!/bin/bash
# The -m gpu suite on one MI355X (K: optional -k expression), log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=()
[ -n "${K:-}" ] && ARGS=(-k "$K")
timeout -k 10 ${LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${ARGS[@]}" \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -${SHOW:-15}
tail -3 gpurun_out/pytest_gpu.log
exit $rc

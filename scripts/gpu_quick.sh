#!/bin/bash
# Quick GPU iteration: parity tests, then kbench of the default build (overlapped
# schedule, per-kernel timing off and on) and of every build_var/*.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 120 python scripts/kbench.py --no-kernel-timing || exit 1
timeout -k 10 120 python scripts/kbench.py || exit 1
shopt -s nullglob
for lib in build_var/*.so; do
  MBOTS_LIB=$lib timeout -k 10 120 python scripts/kbench.py "$@" || exit 1
done

#!/bin/bash
# Quick GPU iteration: selected parity tests (SEL, default the sensor-heavy
# ones), then an interleaved A/B of the default build vs build_var/*.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SEL=${SEL:-"tests/test_parity_gpu.py tests/test_parity_large.py"}
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert" gpurun_out/pytest_iter.log | head -30; exit $rc; fi
timeout -k 10 120 python scripts/kbench.py || exit 1
bash scripts/ab.sh ${ROUNDS:-3} "$@"

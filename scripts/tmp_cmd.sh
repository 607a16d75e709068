#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert|FAILED" gpurun_out/pytest_q.log | head -20; exit $rc; fi
scripts/ab_libs.sh 4 build_var/libmbots_cur.so build_var/libmbots_w.so -- --stream-priority -1

#!/bin/bash
# GPU box (one MI355X): rehearse bench.py's self-spawned multi-rank path --
# `python bench.py --gpus 2` with no launcher starts two ranks itself; on a
# one-GPU box they share cuda:0 over gloo (--same-device).  Config 5 (rollout
# records gathered to rank 0) runs by default with several ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --same-device --steps 40 --warmup 10 \
    --worlds ${WORLDS:-32768} --no-secondary --no-cpu-baseline > gpurun_out/${TAG}_multi2.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_multi2.log; exit $rc

#!/bin/bash
# GPU box (one MI355X): rehearse bench.py's self-spawned multi-rank path --
# `python bench.py --gpus N` with no launcher starts N ranks itself; on a
# one-GPU box they share cuda:0 over gloo (--same-device).  Config 5 (the
# learner round trip: records gathered to rank 0, actions scattered back) runs
# by default with several ranks.  Then the real `--gpus 2` path on one GPU,
# which must end with the ranks' own error (the parent makes no GPU call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r04}
for n in ${RANKS:-2 4}; do
  timeout -k 10 300 python -u bench.py --gpus $n --backend gloo --same-device --steps 40 --warmup 10 \
      --worlds ${WORLDS:-16384} $([ -z "${SECONDARY:-}" ] && echo --no-secondary) --no-cpu-baseline > gpurun_out/${TAG}_multi$n.log 2>&1 \
      || { tail -5 gpurun_out/${TAG}_multi$n.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_multi$n.log | tail -1 > gpurun_out/${TAG}_rehearsal_${n}rank_same_device.json
  python -c "import json; d = json.load(open('gpurun_out/${TAG}_rehearsal_${n}rank_same_device.json')); c = d.get('config5', {}); print($n, 'ranks:', round(d['ms_per_step'], 4), 'ms/step; config5', c.get('ms_per_step'), c.get('error'))"
done
timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline \
    > gpurun_out/${TAG}_spawn_dry.log 2>&1
rc=$?
echo "--gpus 2 on one GPU: rc=$rc"; grep -m1 "needs 2 devices" gpurun_out/${TAG}_spawn_dry.log || exit 1

#!/bin/bash
# GPU box: worlds-per-wave sweep of the caller chain's per-world kernels
# (K3a export_rows, the synthetic writer), interleaved kbench at 65536 worlds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L="madrona-bots_amd/madrona_bots/libmbots.so $LIBS"
bash scripts/ab_libs.sh ${ROUNDS:-3} $L -- --warmup 5 --steps 20 --stream-priority -1 > gpurun_out/wpw_drv.log 2>&1 || exit 1
bash scripts/ab_libs.sh ${SS_ROUNDS:-2} $L -- --warmup 250 --steps 100 --stream-priority -1 > gpurun_out/wpw_ss.log 2>&1 || exit 1
python - <<'PY'
import json, collections
for f in ("gpurun_out/wpw_drv.log", "gpurun_out/wpw_ss.log"):
    r = collections.defaultdict(list)
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); r[d["lib"]].append(d["ms_per_step"])
    print(f)
    for k, v in r.items():
        print(f"  {k:28s} " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")
PY

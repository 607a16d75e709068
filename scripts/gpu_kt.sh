#!/bin/bash
# Per-kernel event times (kbench with kernel timing) of the tree's library and
# every build_var/libmbots_*.so at the WORLDS sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for W in ${WORLDS:-4096}; do
  for lib in madrona-bots_amd/madrona_bots/libmbots.so $(ls build_var/libmbots_*.so 2>/dev/null); do
    MBOTS_LIB=$lib timeout -k 10 120 python scripts/run_variant.py scripts/kbench.py --worlds $W --steps ${STEPS:-100} \
        --warmup ${WARM:-200} > gpurun_out/kt_tmp.json 2>/dev/null || exit 1
    python - $W <<'PY'
import json, sys
d = json.loads(open("gpurun_out/kt_tmp.json").read().strip().splitlines()[-1])
print(f"W={sys.argv[1]} {d['lib']:24s} ms/step {d['ms_per_step']:.4f} " + " ".join(f"{k}={v*1e3:.1f}" for k, v in d["kernel_ms"].items()))
PY
  done
done

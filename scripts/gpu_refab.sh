#!/bin/bash
# GPU box: interleaved A/B of the reference-loop line (scripts/refloop.py) over
# build_var/libmbots_*.so at 4096 and 65536 worlds; prints the min per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/refab.log
for r in $(seq ${ROUNDS:-3}); do
  for l in build_var/libmbots_*.so; do
    for wv in ${WORLDS:-4096 65536}; do
      MBOTS_LIB=$l timeout -k 10 120 python scripts/run_variant.py scripts/refloop.py --worlds $wv --steps ${STEPS:-200} \
          >> gpurun_out/refab.log 2>&1 || { tail -5 gpurun_out/refab.log; exit 1; }
    done
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/refab.log"):
    if line.startswith("{"):
        d = json.loads(line); r[(d["lib"], d["worlds"])].append(d["ms_per_step"])
for k in sorted(r):
    print(f"{k[0]:28s} {k[1]:6d}  " + " ".join(f"{x:.4f}" for x in r[k]) + f"   min {min(r[k]):.4f}")
PY

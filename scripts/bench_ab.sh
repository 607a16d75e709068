#!/bin/bash
# Interleaved A/B of build_var/libmbots_*.so with bench.py itself (the driver's
# line: high-priority caller stream, seed 69), ROUNDS rounds, min per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/bench_ab.log
for r in $(seq ${ROUNDS:-3}); do
  for l in build_var/libmbots_*.so; do
    MBOTS_LIB=$l timeout -k 10 180 python scripts/run_variant.py bench.py --no-cpu-baseline --no-secondary --no-kernel-timing \
        --steps ${STEPS:-200} ${BENCH_ARGS:-} 2>/dev/null | grep '^{' | \
        python -c "import sys, json; d = json.loads(sys.stdin.read()); print(json.dumps({'lib': '$l', 'ms': d['ms_per_step']}))" \
        >> gpurun_out/bench_ab.log || exit 1
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/bench_ab.log"):
    d = json.loads(line); r[d["lib"]].append(d["ms"])
for k, v in r.items():
    print(f"{k:36s} " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")
PY

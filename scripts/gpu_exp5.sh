#!/bin/bash
# Round-5 experiment call: optional -m gpu selection (K), A/B of build_var
# libraries at 65536 and 4096 worlds, kernel times early vs steady state.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${K:-}" ]; then
  timeout -k 10 ${LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "$K" \
      > gpurun_out/pytest_k.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/pytest_k.log | head -20; tail -3 gpurun_out/pytest_k.log; exit 1; }
  grep -E "PASSED|FAILED" gpurun_out/pytest_k.log; tail -1 gpurun_out/pytest_k.log
fi
libs="madrona-bots_amd/madrona_bots/libmbots.so $(ls build_var/libmbots_*.so 2>/dev/null)"
for W in ${WORLDS:-65536 4096}; do
  bash scripts/ab_libs.sh ${ROUNDS:-3} $libs -- --worlds $W --steps ${STEPS:-100} --warmup ${WARM:-200} ${KB_EXTRA:-} > gpurun_out/ab_${TAG:-a}_$W.log 2>&1 || { tail -5 gpurun_out/ab_${TAG:-a}_$W.log; exit 1; }
  python - $W ${TAG:-a} <<'PY'
import json, collections, sys
r = collections.defaultdict(list); hr = collections.defaultdict(list)
for line in open(f"gpurun_out/ab_{sys.argv[2]}_{sys.argv[1]}.log"):
    if line.startswith("{"):
        d = json.loads(line); r[d["lib"]].append(d["ms_per_step"]); hr[d["lib"]].append(d.get("host_ms_per_step", 0))
for k, v in r.items():
    print(f"W={sys.argv[1]} {k:28s} ms/step " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}  host {min(hr[k]):.4f}")
PY
done
if [ -n "${PHASES:-}" ]; then
  for w in 20 250; do
    timeout -k 10 120 python scripts/kbench.py --worlds 65536 --warmup $w --steps 30 > gpurun_out/kb_phase_$w.json || exit 1
    cat gpurun_out/kb_phase_$w.json
  done
fi

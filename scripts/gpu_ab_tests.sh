#!/bin/bash
# GPU box: the -m gpu suite, then an interleaved A/B (scripts/kbench.py) of the
# tree's library against the build_var/libmbots_*.so given in LIBS, in the
# driver's window (steps 5-24) and at steady state (steps 250-349).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:warnings \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
fi
L="madrona-bots_amd/madrona_bots/libmbots.so $LIBS"
bash scripts/ab_libs.sh ${ROUNDS:-3} $L -- --warmup 5 --steps 20 > gpurun_out/ab_drv.log 2>&1 || { tail -5 gpurun_out/ab_drv.log; exit 1; }
bash scripts/ab_libs.sh ${SS_ROUNDS:-2} $L -- --warmup 250 --steps 100 > gpurun_out/ab_ss.log 2>&1 || { tail -5 gpurun_out/ab_ss.log; exit 1; }
python - <<'PY'
import json, collections
for f in ("gpurun_out/ab_drv.log", "gpurun_out/ab_ss.log"):
    r = collections.defaultdict(list)
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); r[d["lib"]].append(d["ms_per_step"])
    print(f)
    for k, v in r.items():
        print(f"  {k:28s} ms/step " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")
PY

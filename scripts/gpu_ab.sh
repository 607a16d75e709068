#!/bin/bash
# GPU box: the -m gpu suite, then an interleaved A/B of the tree's library
# against every build_var/libmbots_*.so (scripts/kbench.py, 65536 worlds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
fi
libs="madrona-bots_amd/madrona_bots/libmbots.so $(ls build_var/libmbots_*.so 2>/dev/null)"
bash scripts/ab_libs.sh ${ROUNDS:-3} $libs -- ${KB_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/ab.log"):
    if line.startswith("{"):
        d = json.loads(line); r[d["lib"]].append(d["ms_per_step"])
for k, v in r.items():
    print(f"{k:28s} ms/step " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")
PY

#!/bin/bash
# One experiment call on the GPU box: the -m gpu suite on the tree's library,
# an interleaved A/B against build_var/libmbots_*.so (scripts/kbench.py), and
# any probe commands given in $PROBES (each under its own limit).
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
if [ "${AB:-1}" = "1" ]; then
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
fi
if [ -n "${PROBES:-}" ]; then
  timeout -k 10 300 bash -c "$PROBES" > gpurun_out/probes.log 2>&1 || { tail -5 gpurun_out/probes.log; exit 1; }
  tail -20 gpurun_out/probes.log
fi

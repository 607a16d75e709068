#!/bin/bash
# Round evidence on one MI355X: the -m gpu suite, the default bench line, the
# rocprofv3 summaries (kernel stats, FETCH/WRITE traffic, VALU mix, timeline)
# and the smoke check.  Each GPU step has its own limit; the script stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench_full.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_full.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_full.log | tail -1 > gpurun_out/${TAG}_bench.json
if [ "${PROFILE:-1}" = "1" ]; then
  TAG=$TAG bash scripts/gpu_profile.sh > gpurun_out/${TAG}_prof_steps.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_steps.log; exit 1; }
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
python - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_bench.json"))
print("ms/step", round(d["ms_per_step"], 4), "G agent-steps/s", round(d["value"] / 1e9, 3),
      "frac", round(d["roofline"]["frac"], 4), "span", round(d["roofline"]["avg_launch_ms"], 4),
      "wall frac", round(d["roofline"]["wall_clock"]["frac"], 4))
for k in ("secondary", "reference_loop"):
    if k in d: print(k, round(d[k]["ms_per_step"], 4), round(d[k]["value"] / 1e9, 3))
if "cpu_baseline" in d: print("cpu", d["cpu_baseline"]["value"] / 1e6, d["cpu_baseline"]["cores"])
PY

#!/bin/bash
# GPU box: (TESTS=1) the -m gpu suite, then the driver's exact bench command,
# ROUNDS times, interleaved with extra variants given as env assignments in
# VARIANTS (e.g. "MBOTS_SWAP=0").
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
: > gpurun_out/drv.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in default $VARIANTS; do
    if [ "$v" = default ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/drv_one.log 2>&1 \
        || { tail -5 gpurun_out/drv_one.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/drv_one.log | tail -1)" >> gpurun_out/drv.log
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/drv.log"):
    v, j = line.split(" ", 1)
    d = json.loads(j)
    print(v, "ms", round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 4), "span", round(d["roofline"]["avg_launch_ms"], 4),
          "steady", round(d["steady_state"]["ms_per_step"], 4), "cfg2", round(d["config2"]["ms_per_step"], 4))
PY

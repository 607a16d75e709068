#!/bin/bash
# the driver's exact bench command beside longer lines on
# the same lease, plus a per-step trace from the first step on, to attribute
# the gap between the driver's 20-step / 5-warmup line and a 100-step one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
O=gpurun_out/${TAG}_gap
mkdir -p $O
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 -u bench.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 4), "span", round(d["roofline"]["avg_launch_ms"], 4),
      "agents/world", round(d["config"]["mean_agents_per_world"], 3), "frac", round(d["roofline"]["frac"], 4),
      "wall frac", round(d["roofline"]["wall_clock"]["frac"], 4),
      "config2", round(d["config2"]["ms_per_step"], 4) if "config2" in d else "-")
PY
}
run driver1 --gpus 1 --steps 20 --warmup 5
timeout -k 10 120 python3 -u scripts/steptrace.py --steps 300 > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
run s20w5 --steps 20 --warmup 5 --no-secondary --no-cpu-baseline
run s100w20 --steps 100 --warmup 20 --no-secondary --no-cpu-baseline
run s20w100 --steps 20 --warmup 100 --no-secondary --no-cpu-baseline
run s20w5_nospan --steps 20 --warmup 5 --no-secondary --no-cpu-baseline
run s100w5 --steps 100 --warmup 5 --no-secondary --no-cpu-baseline
run driver2 --gpus 1 --steps 20 --warmup 5

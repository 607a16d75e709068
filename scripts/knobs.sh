#!/bin/bash
# GPU side of the occupancy-knob experiment (MB_KNOBS build): one kbench per setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build_var/libmbots_knobs.so
: > gpurun_out/knobs.jsonl
run() {  # run "<env assignments>" extra-args...
  local envs=$1; shift
  env $envs MBOTS_LIB=$L timeout -k 10 120 python scripts/kbench.py --no-kernel-timing --stream-priority 0 "$@" > gpurun_out/knobs_one.json 2>> gpurun_out/knobs_err.log || { echo "abort: $envs"; tail -5 gpurun_out/knobs_err.log; exit 1; }
  echo "$envs $(cat gpurun_out/knobs_one.json)" | tee -a gpurun_out/knobs.jsonl
}
run "X=0"
run "MBOTS_SENSOR_LDS_PAD=4096"
run "MBOTS_SENSOR_LDS_PAD=7400"
run "MBOTS_SENSOR_LDS_PAD=12000"
run "MBOTS_SENSOR_CUS=240"
run "MBOTS_SENSOR_CUS=224"
run "MBOTS_SENSOR_CUS=192"
run "X=0"

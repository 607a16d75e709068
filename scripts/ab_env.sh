#!/bin/bash
# GPU side of an env-knob A/B: kbench of the default build once per value.
#   VAR=MBOTS_SENSOR_LDS_PAD bash scripts/ab_env.sh 0 4096 7400 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_env.jsonl
for v in "$@"; do
  env_line="$VAR=$v"
  export $env_line
  timeout -k 10 240 python scripts/kbench.py >> gpurun_out/ab_env.jsonl 2> gpurun_out/ab_err.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "abort: $env_line rc=$rc"; tail -5 gpurun_out/ab_err.log; exit $rc; fi
  echo "$env_line $(tail -1 gpurun_out/ab_env.jsonl)"
done

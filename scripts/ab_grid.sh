#!/bin/bash
# fork-mode kbench of the default build over (move grid, shift grid) pairs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pair in "$@"; do
  mg=${pair%,*}; sg=${pair#*,}
  r=$(MBOTS_MOVE_GRID=$mg MBOTS_SHIFT_GRID=$sg timeout -k 10 240 python scripts/kbench.py 2> gpurun_out/ab_err.log) || { echo "abort $pair"; tail -3 gpurun_out/ab_err.log; exit 1; }
  echo "$pair $r"
done

#!/bin/bash
# Same-box A/B: the default build vs build_var/libmbots_*.so, interleaved, N rounds.
#   ab.sh [rounds] [kbench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=${1:-2}; shift
for r in $(seq $n); do
  timeout -k 10 120 python scripts/kbench.py --no-kernel-timing "$@" || exit 1
  for lib in build_var/libmbots_*.so; do
    MBOTS_LIB=$lib timeout -k 10 120 python scripts/run_variant.py scripts/kbench.py --no-kernel-timing "$@" || exit 1
  done
done

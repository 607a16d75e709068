#!/bin/bash
# Per-variant kernel times (kernel timing on) then step times (off), build_var/libmbots_*.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in build_var/libmbots_*.so; do
  MBOTS_LIB=$lib timeout -k 10 120 python scripts/kbench.py "$@" || exit 1
done
for r in 1 2; do
  for lib in build_var/libmbots_*.so; do
    MBOTS_LIB=$lib timeout -k 10 120 python scripts/kbench.py --no-kernel-timing "$@" || exit 1
  done
done

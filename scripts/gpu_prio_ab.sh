#!/bin/bash
# GPU box: interleaved kbench runs with the caller's stream at high (-1) and
# normal (0) priority, driver's window and steady state.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for args in "--warmup 5 --steps 20" "--warmup 250 --steps 100"; do
  for r in 1 2 3; do
    for p in -1 0; do
      echo "prio=$p $args"
      timeout -k 10 120 python scripts/kbench.py --no-kernel-timing --stream-priority $p $args 2>/dev/null | grep '^{' || exit 1
    done
  done
done

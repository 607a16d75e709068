#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3 4 5; do for lib in build_var/libmbots_r0.so build_var/libmbots_cur.so; do
  MBOTS_LIB=$lib timeout -k 10 120 python scripts/refloop.py --steps 400 || exit 1
done; done

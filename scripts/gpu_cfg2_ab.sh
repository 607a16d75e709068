#!/bin/bash
# GPU box: small-world schedule sizing -- interleaved kbench runs of the
# tree's library and build_var variants at 2048 / 4096 / 8192 worlds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L="madrona-bots_amd/madrona_bots/libmbots.so $LIBS"
for w in ${WORLDS:-2048 4096 8192}; do
  for r in 1 2 3; do
    for lib in $L; do
      echo "W=$w $(basename $lib)"
      MBOTS_LIB=$lib timeout -k 10 120 python scripts/run_variant.py scripts/kbench.py --no-kernel-timing \
          --stream-priority -1 --worlds $w --warmup 50 --steps 200 2>/dev/null | grep '^{' || exit 1
    done
  done
done

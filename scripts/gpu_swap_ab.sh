#!/bin/bash
# GPU box: interleaved kbench runs of the default schedule and MBOTS_SWAP=1
# (K1 / K2 / the sensor on the internal stream) in the driver's window and at
# steady state.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "--warmup 5 --steps 20" "--warmup 250 --steps 100"; do
  for r in 1 2 3; do
    for sw in 0 1; do
      echo -n "swap=$sw $args: "
      MBOTS_SWAP=$sw timeout -k 10 120 python scripts/kbench.py --no-kernel-timing --stream-priority -1 $args || exit 1
    done
  done
done

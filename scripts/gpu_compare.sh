#!/bin/bash
# GPU box: per-kernel event times (kbench, kernel timing on) and the sensor's
# instruction mix (one PMC pass) for every build_var/libmbots_*.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in build_var/libmbots_*.so; do
  MBOTS_LIB=$lib timeout -k 10 120 python scripts/run_variant.py scripts/kbench.py ${KB_ARGS:-} || exit 1
done
bash scripts/pmc_vars.sh "${COUNTERS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES}" ${KB_ARGS:-}

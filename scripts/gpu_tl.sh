#!/bin/bash
# Kernel-trace timelines (rocprofv3 --kernel-trace, scripts/timeline.py) of the
# tree's library and every build_var/libmbots_*.so at WORLDS worlds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
W=${WORLDS:-4096}
for lib in madrona-bots_amd/madrona_bots/libmbots.so $(ls build_var/libmbots_*.so 2>/dev/null); do
  n=$(basename $lib .so)
  MBOTS_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$n -o run -- \
      python scripts/run_variant.py scripts/kbench.py --worlds $W --steps 300 --warmup 100 --no-kernel-timing \
      > gpurun_out/tl_$n.log 2>&1 || { tail gpurun_out/tl_$n.log; exit 1; }
  python scripts/timeline.py gpurun_out/tl_$n/run_kernel_trace.csv 100 > gpurun_out/tl_${n}_$W.txt
  echo "== $n"; cat gpurun_out/tl_${n}_$W.txt
done

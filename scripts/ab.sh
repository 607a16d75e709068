#!/bin/bash
# GPU side of an A/B run: time every build_var/*.so (and the default build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
shopt -s nullglob
for lib in madrona-bots_amd/madrona_bots/libmbots.so build_var/*.so; do
  MBOTS_LIB=$lib timeout -k 10 240 python scripts/kbench.py "$@" >> gpurun_out/ab.jsonl 2> gpurun_out/ab_err.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "abort: $lib rc=$rc"; tail -5 gpurun_out/ab_err.log; exit $rc; fi
done
cat gpurun_out/ab.jsonl

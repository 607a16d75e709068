#!/bin/bash
# stream-priority A/B of the default build: the caller's (main) stream at each
# priority given (none = default stream), kernel timing off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/prio.jsonl
for p in "$@"; do
  if [ "$p" = none ]; then a=""; else a="--stream-priority $p"; fi
  timeout -k 10 240 python scripts/kbench.py --no-kernel-timing --steps 300 --warmup 200 $a >> gpurun_out/prio.jsonl 2> gpurun_out/prio_err.log \
    || { echo "abort $p"; tail -5 gpurun_out/prio_err.log; exit 1; }
done
cat gpurun_out/prio.jsonl

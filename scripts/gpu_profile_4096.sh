#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p4096 -o run -- python scripts/kbench.py --worlds 4096 --steps 300 --warmup 100 --no-kernel-timing > gpurun_out/p4096.log 2>&1 || { tail gpurun_out/p4096.log; exit 1; }
python scripts/timeline.py gpurun_out/p4096/run_kernel_trace.csv 100 > gpurun_out/${TAG:-r05}_timeline_4096.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d gpurun_out/p4096v -o run -- python scripts/kbench.py --worlds 4096 --steps 6 --warmup 2 --no-kernel-timing > gpurun_out/p4096v.log 2>&1 || { tail gpurun_out/p4096v.log; exit 1; }
python scripts/valu.py gpurun_out/p4096v 4096 gpurun_out/${TAG:-r05}_valu_4096.json
cat gpurun_out/${TAG:-r05}_timeline_4096.txt; cat gpurun_out/${TAG:-r05}_valu_4096.json

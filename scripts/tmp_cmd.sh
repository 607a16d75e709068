#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r02 bash scripts/gpu_profile.sh > gpurun_out/prof_steps.log 2>&1 || { tail -5 gpurun_out/prof_steps.log; exit 1; }
cp gpurun_out/r02_traffic.json gpurun_out/r02_valu.json gpurun_out/r02_kernel_stats.csv profiles/
timeout -k 10 400 python -u bench.py > gpurun_out/r02_bench_full.log 2>&1 || exit 1
tail -1 gpurun_out/r02_bench_full.log > gpurun_out/r02_bench.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
python -c "import json; d=json.load(open('gpurun_out/r02_bench.json')); print(d['ms_per_step'], d['value']/1e9, d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['wall_clock']['frac'], d['secondary']['ms_per_step'], d['reference_loop']['ms_per_step'])"

#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats + FETCH/WRITE PMC passes
# of the bench command (65536 worlds).  Copies summaries to profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
mkdir -p gpurun_out
B="bench.py --steps 30 --warmup 100 --no-cpu-baseline --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
    -- python $B > gpurun_out/prof_$TAG.log 2>&1 || { echo "stats pass failed"; tail gpurun_out/prof_$TAG.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_$c -o run \
      -- python $B --no-kernel-timing > gpurun_out/pmc_${TAG}_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
# sensor VALU issue (secondary roofline): instructions per launch
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv \
    -d gpurun_out/pmc_${TAG}_valu -o run -- python $B --no-kernel-timing > gpurun_out/pmc_${TAG}_valu.log 2>&1 \
    || { echo "pmc valu failed"; exit 1; }
python scripts/valu.py gpurun_out/pmc_${TAG}_valu 65536 gpurun_out/${TAG}_valu.json
mkdir -p gpurun_out/traffic_$TAG
i=0; for c in FETCH_SIZE WRITE_SIZE; do i=$((i+1)); rm -rf gpurun_out/traffic_${TAG}_p$i; cp -r gpurun_out/pmc_${TAG}_$c gpurun_out/traffic_${TAG}_p$i; done
python scripts/traffic.py gpurun_out/traffic_$TAG 65536 gpurun_out/${TAG}_traffic.json
cp gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
python scripts/timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv 100 > gpurun_out/${TAG}_timeline.txt
grep '^{' gpurun_out/prof_$TAG.log | tail -1 > gpurun_out/${TAG}_bench_under_rocprof.json
echo done
# (run locally afterwards: cp gpurun_out/${TAG}_{traffic.json,valu.json,kernel_stats.csv,bench_under_rocprof.json,timeline.txt} profiles/)

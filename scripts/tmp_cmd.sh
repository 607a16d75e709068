cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 50 --warmup 20 --cpu-seconds 8 > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
TAG=r02 bash scripts/gpu_profile.sh

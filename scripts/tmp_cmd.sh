cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in build_var/libmbots_wpb8.so build_var/libmbots_wpb16.so; do
  MBOTS_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "small or 64_worlds or 4096 or edge or capacity" --timeout 200 --timeout-method thread > gpurun_out/pt_$(basename $lib).log 2>&1 || { tail -20 gpurun_out/pt_$(basename $lib).log; exit 1; }
  tail -1 gpurun_out/pt_$(basename $lib).log
done
for r in 1 2; do
for lib in build_var/libmbots_*.so; do MBOTS_LIB=$lib timeout -k 10 120 python scripts/kbench.py || exit 1; done
done
bash scripts/ab.sh 1 --worlds 4096 --steps 200

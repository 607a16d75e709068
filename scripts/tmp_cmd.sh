cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SEL="tests/test_parity_gpu.py tests/test_parity_large.py tests/test_checkpoint.py" ROUNDS=3 bash scripts/gpu_iter.sh || exit 1
bash scripts/ab.sh 2 --worlds 4096 --steps 200 || exit 1

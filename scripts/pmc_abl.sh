set -o pipefail
cd "${GRAFT_REPO_ROOT}"
for v in 0 8 16 32 48 56; do
  MBOTS_LIB=build_var/libmbots_abl$v.so TAG=abl$v PROG="python scripts/kbench.py --steps 5 --warmup 50" bash scripts/gpu_pmc.sh "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" > /dev/null || exit 1
done
bash scripts/ab.sh > /dev/null && cat gpurun_out/ab.jsonl

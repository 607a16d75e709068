#!/bin/bash
# GPU box: the K1-finder prev-sensor race test against a single-buffered
# obsrow_out build (expected to fail) and the tree's library, then the
# small-world schedule sizing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/ubench/valu_rate > gpurun_out/valu_rate.jsonl 2>&1 || exit 1
cat gpurun_out/valu_rate.jsonl
PYTHONPATH=scripts MBOTS_LIB=build_var/libmbots_single.so timeout -k 10 300 python -u -m pytest -p _variant \
    tests/test_parity_gpu.py -k "k1_finder_step_only" -v --timeout 200 --timeout-method thread -p no:warnings \
    > gpurun_out/race_single.log 2>&1
echo "single-buffer build rc=$? (1: the test caught the race)"
grep -E "PASSED|FAILED" gpurun_out/race_single.log | head
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "k1_finder_step_only" -v --timeout 200 \
    --timeout-method thread -p no:warnings > gpurun_out/race_tree.log 2>&1 || { tail -20 gpurun_out/race_tree.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/race_tree.log | head
LIBS="build_var/libmbots_f8192.so build_var/libmbots_f8192lazy.so build_var/libmbots_flazy.so" \
    bash scripts/gpu_cfg2_ab.sh > gpurun_out/cfg2_ab.log 2>&1 || exit 1
python scripts/ab_parse.py gpurun_out/cfg2_ab.log
# worlds per wave of the caller chain's per-world kernels, 65536 worlds
L="madrona-bots_amd/madrona_bots/libmbots.so build_var/libmbots_act4.so build_var/libmbots_exp4.so build_var/libmbots_both4.so"
bash scripts/ab_libs.sh 3 $L -- --warmup 5 --steps 20 --stream-priority -1 > gpurun_out/wpw_drv.log 2>&1 || exit 1
bash scripts/ab_libs.sh 2 $L -- --warmup 250 --steps 100 --stream-priority -1 > gpurun_out/wpw_ss.log 2>&1 || exit 1
python - <<'PY'
import json, collections
for f in ("gpurun_out/wpw_drv.log", "gpurun_out/wpw_ss.log"):
    r = collections.defaultdict(list)
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); r[d["lib"]].append(d["ms_per_step"])
    print(f)
    for k, v in r.items():
        print(f"  {k:28s} " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")
PY

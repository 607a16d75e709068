set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTHONPATH=scripts MBOTS_LIB=build_var/libmbots_single.so timeout -k 10 300 python -u -m pytest -p _variant tests/test_parity_gpu.py -k "k1_finder_step_only" -v --timeout 120 --timeout-method thread -p no:warnings > gpurun_out/single.log 2>&1
echo "single rc=$?"
grep -E "PASSED|FAILED|differ" gpurun_out/single.log | head -12
L="madrona-bots_amd/madrona_bots/libmbots.so build_var/libmbots_shifth.so build_var/libmbots_shiftpsem.so build_var/libmbots_shiftnone.so"
bash scripts/ab_libs.sh 3 $L -- --warmup 5 --steps 20 > gpurun_out/ab_drv.log 2>&1 || exit 1
bash scripts/ab_libs.sh 2 $L -- --warmup 250 --steps 100 > gpurun_out/ab_ss.log 2>&1 || exit 1
python - <<'PY'
import json, collections
for f in ("gpurun_out/ab_drv.log", "gpurun_out/ab_ss.log"):
    r = collections.defaultdict(list)
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); r[d["lib"]].append(d["ms_per_step"])
    print(f)
    for k, v in r.items():
        print(f"  {k:28s} ms/step " + " ".join(f"{x:.4f}" for x in v) + f"   min {min(v):.4f}")
PY

#!/bin/bash
# GPU box: the config-5 tests, then the config-5 line with slim and with full
# learner records (one rank: pack + unpack locally).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_learner_roundtrip.py tests/test_gather.py -m gpu -x -q --timeout 400 \
    --timeout-method thread -p no:warnings > gpurun_out/c5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/c5_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/c5_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --gather --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    --no-kernel-timing > gpurun_out/c5_slim.json 2> gpurun_out/c5_slim.err || { tail -5 gpurun_out/c5_slim.err; exit 1; }
timeout -k 10 300 python -u bench.py --gather --full-records --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    --no-kernel-timing > gpurun_out/c5_full.json 2> gpurun_out/c5_full.err || { tail -5 gpurun_out/c5_full.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/c5_slim.json", "gpurun_out/c5_full.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c = d["config5"]
    print(f, {k: c[k] for k in ("ms_per_step", "gather_ms_per_step", "bytes_per_agent", "records")},
          json.dumps(c.get("roundtrip_roofline")))
PY

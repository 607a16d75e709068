#!/usr/bin/env python3
"""More seeds of tests/test_parity_gpu.py::test_random_call_sequences on the
GPU (random step / shift / action-write / column-read / construct_obs /
checkpoint hand-over sequences against the oracle; seeds % 4 == 0 at 4100
worlds, the others at 21+ worlds in K1-finder mode):
    python scripts/fuzz_calls.py FIRST_SEED END_SEED [WORLDS]
(WORLDS: every seed at that world count, e.g. 16400 for the swapped schedule)"""
import sys, os, time
sys.path[:0] = ["madrona-bots_amd", "oracle", "tests"]
import test_parity_gpu as t
lo, hi = int(sys.argv[1]), int(sys.argv[2])
W = int(sys.argv[3]) if len(sys.argv) > 3 else None
t0 = time.time()
for s in range(lo, hi):
    t.test_random_call_sequences(s, W)
    print("seed", s, "ok", round(time.time() - t0, 1), flush=True)

#!/usr/bin/env python3
"""Host microseconds per call of the bench's bare loop (step, shift, action
write) at a given world count, and the loop's wall ms/step: whether the host or
the device sets the pace (a device-bound loop lets the host run ahead).
    python scripts/barehost.py [--worlds 4096] [--steps 400]"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import _variant  # noqa: E402,F401  (MBOTS_LIB: A/B builds)
import torch
import madrona_bots as mb

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=4096)
ap.add_argument("--steps", type=int, default=400)
a = ap.parse_args()
torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
m = mb.SimManager(0, a.worlds, 69, 32)
m.write_synthetic_actions(1234, 0)
for t in range(50):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
acc = {"step": 0.0, "shift": 0.0, "write": 0.0}
w0 = time.perf_counter()
for t in range(50, 50 + a.steps):
    t0 = time.perf_counter(); m.step()
    t1 = time.perf_counter(); m.shift_observations()
    t2 = time.perf_counter(); m.write_synthetic_actions(1234, t + 1)
    t3 = time.perf_counter()
    acc["step"] += t1 - t0; acc["shift"] += t2 - t1; acc["write"] += t3 - t2
torch.cuda.synchronize()
wall = (time.perf_counter() - w0) / a.steps * 1e3
print(json.dumps({"lib": os.path.basename(os.environ.get("MBOTS_LIB", "libmbots.so")), "worlds": a.worlds,
                  "host_us_per_call": {k: round(v / a.steps * 1e6, 2) for k, v in acc.items()},
                  "ms_per_step": round(wall, 5)}), flush=True)

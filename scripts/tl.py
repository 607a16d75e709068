#!/usr/bin/env python3
"""Kernel timeline of an MB_TL build without a profiler in the process: per
step, each kernel's first-wave start and last-wave end (100 MHz realtime clock).

    MBOTS_LIB=build_var/libmbots_tl.so python scripts/tl.py [--worlds W] [--steps K]
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
import torch
import madrona_bots as mb

NAMES = ["world_step", "scan", "export", "sensor", "move", "shift", "actions"]
ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=65536)
ap.add_argument("--steps", type=int, default=32)
ap.add_argument("--warmup", type=int, default=100)
a = ap.parse_args()
m = mb.SimManager(0, a.worlds, 69, 32)
fn = mb._lib.mbots_debug_timeline
buf = (ctypes.c_ulonglong * (64 * 8 * 2))()
m.write_synthetic_actions(1234, 0)
for t in range(a.warmup):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
fn(buf)
for t in range(a.warmup, a.warmup + a.steps):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
fn(buf)
v = list(buf)
steps = []
for s in range(64):
    ev = {}
    for k, nm in enumerate(NAMES):
        st, en = v[(s * 8 + k) * 2], v[(s * 8 + k) * 2 + 1]
        if en and st != 2**64 - 1:
            ev[nm] = (st, en)
    if "world_step" in ev:
        steps.append(ev)
steps.sort(key=lambda e: e["world_step"][0])
# step s spans [K1 start of s, K1 start of s+1)
rows = []
for s in range(len(steps) - 1):
    t0 = steps[s]["world_step"][0]
    t1 = steps[s + 1]["world_step"][0]
    rows.append({"step_us": (t1 - t0) / 100.0,
                 **{nm: [round((b - t0) / 100.0, 1), round((e - t0) / 100.0, 1)]
                    for nm, (b, e) in steps[s].items()}})
mean = {"step_us": sum(r["step_us"] for r in rows) / len(rows)}
for nm in NAMES:
    xs = [r[nm] for r in rows if nm in r]
    if xs:
        mean[nm] = [round(sum(x[0] for x in xs) / len(xs), 1), round(sum(x[1] for x in xs) / len(xs), 1)]
print(json.dumps({"lib": os.path.basename(os.environ.get("MBOTS_LIB", "default")),
                  "worlds": a.worlds, "mean_us_from_K1_start": mean}), flush=True)

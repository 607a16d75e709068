#!/usr/bin/env python3
"""Per-phase sensor clocks of an MB_PROF build (A/B experiments).

    MBOTS_LIB=build_var/libmbots_prof.so python scripts/sprof.py [--worlds W]
Prints mean shader-clock cycles per world for each sensor phase."""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
import torch
import madrona_bots as mb

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=65536)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--warmup", type=int, default=100)
a = ap.parse_args()
m = mb.SimManager(0, a.worlds, 69, 32)
lib = mb._lib
fn = lib.mbots_debug_sensor_prof
buf = (ctypes.c_ulonglong * 16)()
m.write_synthetic_actions(1234, 0)
for t in range(a.warmup):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
m.sensor_index_tensor()   # joins the sensor
fn(buf)
for t in range(a.warmup, a.warmup + a.steps):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
m.sensor_index_tensor()
fn(buf)
v = list(buf)
nw = v[7]
names = ["staging", "p1_excl", "survivors", "output", "total", "n_survivors", "pairs"]
out = {k: v[i] / nw for i, k in enumerate(names) if i not in (1,)}
out["n_wide"] = v[1] / nw
out["p1_excl"] = (v[4] - v[0] - v[2] - v[3]) / nw
k = v[8:]
kn = k[7] or 1
out["k1"] = {nm: round(k[i] / kn, 1) for i, nm in enumerate(
    ["stage", "addfood", "action", "health", "surround_respawn", "compact", "n0"])}
out["lib"] = os.path.basename(os.environ.get("MBOTS_LIB", "default"))
print(json.dumps({k: (round(x, 1) if isinstance(x, float) else x) for k, x in out.items()}), flush=True)

#!/usr/bin/env python3
"""Config-2 latency probe: the steady-state bench loop
(step + shift + action write) at small world counts, eager on the current
build vs captured as a HIP graph of two steps (the table halves alternate, so
two steps return the manager to the same buffers) and replayed.  Prints one
JSON line per mode.  A replay repeats the captured action-stream step numbers,
so this is a latency measurement, not a bench line.

    MBOTS_LIB=... python scripts/graph_probe.py [--worlds 4096] [--steps 400]
"""
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
lib = os.path.basename(os.environ.get("MBOTS_LIB", "default"))
m = mb.SimManager(0, a.worlds, 69, 32)
m.write_synthetic_actions(1234, 0)
t = 0
def one():
    global t
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1); t += 1
for _ in range(100):
    one()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    one()
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / a.steps * 1e3
print(json.dumps({"lib": lib, "mode": "eager", "worlds": a.worlds, "ms_per_step": eager}), flush=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.stream(s):
        one(); one()            # settle the deferred-move state on this stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            one(); one(); m.join()
    torch.cuda.synchronize()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps // 2):
        g.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / (2 * (a.steps // 2)) * 1e3
    print(json.dumps({"lib": lib, "mode": "graph", "worlds": a.worlds, "ms_per_step": gr}), flush=True)
except Exception as e:   # capture not supported by this build's launches
    print(json.dumps({"lib": lib, "mode": "graph", "worlds": a.worlds, "error": repr(e)[:300]}), flush=True)

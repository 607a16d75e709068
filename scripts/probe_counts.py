#!/usr/bin/env python3
"""Counting-probe builds (build_var/probe_*.so: the sensor adds a per-world
counter into the overflow column): counter total / (worlds x steps)."""
import glob, os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WINDOWS = os.environ.get("WINDOWS", "200-220")
code = "WINDOWS = [" + ", ".join("(%s, %s)" % tuple(w.split("-")) for w in WINDOWS.split()) + "]\n" + r'''
import sys, json; sys.path.insert(0, "madrona-bots_amd"); sys.path.insert(0, "scripts"); import _variant
import torch, madrona_bots as mb
W = 65536
m = mb.SimManager(0, W, 69, 32)
m.write_synthetic_actions(1234, 0)
out = {}
t = 0
for lo, hi in WINDOWS:
    while t < lo:
        m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1); t += 1
    torch.cuda.synchronize()
    a = m.overflow()
    n0 = m.agent_steps()
    while t < hi:
        m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1); t += 1
    torch.cuda.synchronize()
    out[f"steps {lo}-{hi - 1}"] = {"per_world_step": round((m.overflow() - a) / (W * (hi - lo)), 3),
                                   "agents_per_world": round((m.agent_steps() - n0) / (W * (hi - lo)), 3)}
print(json.dumps(out))
'''
for lib in sorted(glob.glob(os.path.join(ROOT, "build_var", "probe_*.so"))):
    env = dict(os.environ, MBOTS_LIB=lib)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, timeout=120)
    print(os.path.basename(lib), r.stdout.strip() or r.stderr[-300:], flush=True)

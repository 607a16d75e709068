#!/usr/bin/env python3
"""CPU-mode throughput of libmbots builds (MBOTS_LIB) at several thread
counts, interleaved: python scripts/cpu_ab.py lib1.so lib2.so ... """
import os, subprocess, sys, json
code = r'''
import sys, time, os; sys.path.insert(0, "madrona-bots_amd"); sys.path.insert(0, "scripts"); import _variant
import madrona_bots as mb
W = int(os.environ["W"])
s = mb.SimManager(0, W, 69, 32, exec_mode="cpu")
s.write_synthetic_actions(1234, 0); s.step(); s.shift_observations()
a0 = s.agent_steps(); t0 = time.perf_counter(); k = 0
while time.perf_counter() - t0 < 4:
    s.write_synthetic_actions(1234, k + 1); s.step(); s.shift_observations(); k += 1
dt = time.perf_counter() - t0
print((s.agent_steps() - a0) / dt / 1e6)
'''
for rnd in range(2):
    for th, W in ((16, 4096), (256, 16384)):
        for lib in sys.argv[1:]:
            env = dict(os.environ, MBOTS_LIB=lib, MBOTS_CPU_THREADS=str(th), W=str(W))
            r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
            print(os.path.basename(lib), th, r.stdout.strip() or r.stderr[-200:], flush=True)

#!/usr/bin/env python3
"""Per-kernel timing of one libmbots build (A/B experiments).

    MBOTS_LIB=build_var/libmbots_x.so python scripts/kbench.py [--worlds W] [--steps K]
"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import _variant  # noqa: E402,F401  (MBOTS_LIB: A/B builds)
import torch
import madrona_bots as mb

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=65536)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--warmup", type=int, default=200)
ap.add_argument("--stream-priority", type=int, default=None,
                help="run on a new torch stream of this priority (lower = higher priority)")
ap.add_argument("--no-kernel-timing", action="store_true")
ap.add_argument("--capacity", default="128", help='agent_capacity (kernel class 128 / 256 / 512 / 1024 / 2048 / 4096, or "auto")')
a = ap.parse_args()
if a.stream_priority is not None:
    torch.cuda.set_stream(torch.cuda.Stream(priority=a.stream_priority))
m = mb.SimManager(0, a.worlds, 69, 32, agent_capacity=a.capacity if a.capacity == "auto" else int(a.capacity))
m.write_synthetic_actions(1234, 0)
for t in range(a.warmup):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
m.enable_kernel_timing(not a.no_kernel_timing)
s0 = m.agent_steps()
t0 = time.perf_counter()
for t in range(a.warmup, a.warmup + a.steps):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
th = time.perf_counter() - t0   # the host's enqueue time (= dt when host-bound)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
kt = m.kernel_times()
out = {"lib": os.path.basename(os.environ.get("MBOTS_LIB", "default")), "capacity": a.capacity,
       "stream_priority": a.stream_priority,
       "agent_steps_per_s": (m.agent_steps() - s0) / dt, "ms_per_step": dt / a.steps * 1e3,
       "host_ms_per_step": th / a.steps * 1e3,
       "kernel_ms": {k: round(v[0] / v[1], 4) for k, v in kt.items() if v[1]}}
print(json.dumps(out), flush=True)

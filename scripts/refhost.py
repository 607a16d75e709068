#!/usr/bin/env python3
"""Host time per call of bench.py's reference-loop sequence (the
learn/training_loop.py call sequence), to tell host-bound from device-bound:
    python scripts/refhost.py [--worlds 4096] [--steps 200]"""
import argparse, collections, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
import torch
import madrona_bots as mb

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=4096)
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
m = mb.SimManager(0, a.worlds, 69, 32)
acc = collections.defaultdict(float)


def one(t, rec):
    stamps = [("start", time.perf_counter())]

    def mark(k):
        stamps.append((k, time.perf_counter()))
    m.step(); mark("step")
    ends = m.species_count_tensor().to_torch().sum(dim=0).cumsum(dim=0); mark("species_count+sum")
    m.action_tensor(False).to_torch(); mark("action view")
    m.hidden_state_tensor(False).to_torch(); mark("hidden view")
    rew = m.reward_tensor(False).to_torch().clone(); mark("reward clone")
    hp = m.health_tensor(False).to_torch().clone(); mark("health clone")
    prev = m.construct_obs(True); mark("obs prev")
    obs = m.construct_obs(False); mark("obs cur")
    ph = m.hidden_state_tensor(True).to_torch(); mark("prev hidden view")
    m.shift_observations(); mark("shift")
    m.write_synthetic_actions(1234, t + 1, True); mark("write")
    if rec:
        for (k0, t0), (k1, t1) in zip(stamps, stamps[1:]):
            acc[k1] += t1 - t0
    return ends, rew, hp, obs, prev, ph


m.write_synthetic_actions(1234, 0, True)
for t in range(20):
    one(t, False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(20, 20 + a.steps):
    one(t, True)
torch.cuda.synchronize()
el = time.perf_counter() - t0
out = {"worlds": a.worlds, "ms_per_step": el / a.steps * 1e3,
       "host_us_per_call": {k: round(v / a.steps * 1e6, 1) for k, v in acc.items()},
       "host_us_total": round(sum(acc.values()) / a.steps * 1e6, 1)}
print(json.dumps(out), flush=True)

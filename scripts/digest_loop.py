#!/usr/bin/env python3
"""Digest of every exported column (current and Prev) after K steps of the
bench's loop (step, shift_observations, synthetic actions) for one library
build (MBOTS_LIB, scripts/_variant.py): an A/B build that changes the schedule
or fuses kernels must print the digest the tree's library prints.

    MBOTS_LIB=build_var/libmbots_x.so python scripts/digest_loop.py [--worlds W] [--steps K]
"""
import argparse, hashlib, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import _variant  # noqa: E402,F401
import torch  # noqa: E402
import madrona_bots as mb  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=4096)
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--write-hidden", action="store_true")
a = ap.parse_args()
m = mb.SimManager(0, a.worlds, 69, 32)
m.write_synthetic_actions(1234, 0, a.write_hidden)
for t in range(a.steps):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1, a.write_hidden)
torch.cuda.synchronize()
h = hashlib.sha256()
names = ["species_tensor", "position_tensor", "health_tensor", "surrounding_tensor", "reward_tensor",
         "action_tensor", "stats_tensor", "hidden_state_tensor", "semantic_tensor", "depth_tensor"]
for name in names:
    for prev in (False, True):
        h.update(getattr(m, name)(prev).to_torch().cpu().numpy().tobytes())
h.update(m.species_count_tensor().to_torch().cpu().numpy().tobytes())
print(os.path.basename(os.environ.get("MBOTS_LIB", "default")), a.worlds, a.steps, m.num_agents(), h.hexdigest()[:16])

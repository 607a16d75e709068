#!/usr/bin/env python3
"""Regenerates the committed fixtures under tests/golden/.

1. reference_shapes.json -- facts the reference itself pins at the boundary
   (read here from /root/reference, which is not on the GPU box):
     * learner checkpoints (checkpoints/universe_violence/species_*/...pt,
       loaded with torch.load(weights_only=True)): observation width 69 and
       action width 6 (learn/env.py:19, learn/util.py:23-28);
     * mesh extents (data/agent_render.obj, data/cube_render.obj, read as text)
       behind the sensor objects, and the agent mesh's cross-section in the
       rays' plane (agents: discs of radius 0.92; food: the +-1 cube as a
       rotated square).
2. oracle_w4_a32_s69.npz / oracle_w8_a4_s7_fixed.npz -- golden vectors of the
   CPU oracle (oracle/mbots_oracle.c, the parity checker): per-step SHA-256
   digests of every exported column after step() and after
   shift_observations(), and the full final tables.  The HIP path is checked
   against these in tests/test_parity_gpu.py, the oracle itself in
   tests/test_golden.py.
3. oracle_w4096_a32_s69_h120.npz -- the bench's horizon:
   BASELINE config 2's 4096 worlds driven for 120 steps by bench.py's loop
   (identity-keyed one-hot actions, seed 1234, no memory writes; step, shift),
   per-step digests only (the tables themselves would be ~35 MB).  Checked
   against the HIP path in tests/test_parity_horizon.py.

    python tests/golden/make_golden.py
"""
import glob
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402

REF = "/root/reference"

NAMES = ["species", "pos", "health", "surround", "reward", "action", "stats", "hidden",
         "semantic", "depth"]

FIXTURES = [
    # name, worlds, agents, seed, steps, reward_fixed, cap
    ("oracle_w4_a32_s69", 4, 32, 69, 16, False, 128),
    ("oracle_w8_a4_s7_fixed", 8, 4, 7, 24, True, 16),
]


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def table_digests(sim):
    out = {}
    for i, nm in enumerate(NAMES):
        out[nm] = digest(sim.column(i))
        out["prev_" + nm] = digest(sim.column(i, True))
    out["species_count"] = digest(sim.species_count())
    return out


def run_fixture(W, A, seed, steps, reward_fixed, cap):
    sim = pyoracle.OracleSim(W, seed, A, cap=cap, reward_fixed=reward_fixed)
    log = [("init", sim.num_agents(), table_digests(sim))]
    for t in range(steps):
        sim.write_synthetic_actions(1234, t, True)
        sim.step()
        log.append((f"step{t}", sim.num_agents(), table_digests(sim)))
        sim.shift_observations()
        log.append((f"shift{t}", sim.num_agents(), table_digests(sim)))
    return sim, log


def save_fixture(name, W, A, seed, steps, reward_fixed, cap):
    sim, log = run_fixture(W, A, seed, steps, reward_fixed, cap)
    arrays = {nm: sim.column(i).copy() for i, nm in enumerate(NAMES)}
    arrays.update({"prev_" + nm: sim.column(i, True).copy() for i, nm in enumerate(NAMES)})
    arrays["species_count"] = sim.species_count().copy()
    meta = {"worlds": W, "agents": A, "seed": seed, "steps": steps, "reward_fixed": reward_fixed,
            "cap": cap, "action_seed": 1234, "write_hidden": True, "log": log}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **arrays)
    print(f"{name}: {sim.num_agents()} agents after {steps} steps")


HORIZON = ("oracle_w4096_a32_s69_h120", 4096, 32, 69, 120)


def save_horizon(name, W, A, seed, steps, threads=8):
    sim = pyoracle.OracleSim(W, seed, A, num_threads=threads)
    log = [("init", sim.num_agents(), table_digests(sim))]
    for t in range(steps):
        sim.write_synthetic_actions(1234, t, False)   # bench.py: write_synthetic_actions(ACTION_SEED, t)
        sim.step()
        log.append((f"step{t}", sim.num_agents(), table_digests(sim)))
        sim.shift_observations()
        log.append((f"shift{t}", sim.num_agents(), table_digests(sim)))
    meta = {"worlds": W, "agents": A, "seed": seed, "steps": steps, "reward_fixed": False, "cap": 128,
            "action_seed": 1234, "write_hidden": False, "overflow": int(sim.overflow()), "log": log}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta))
    print(f"{name}: {sim.num_agents()} agents after {steps} steps")


def obj_extent(path):
    xs = []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                xs.append([float(v) for v in line.split()[1:4]])
    xs = np.array(xs)
    return float(np.abs(xs).max())


def obj_section_radii(path, z=0.0):
    """Radii (min, max) of the mesh's cross-section with the plane Z = z: the
    outline horizontal sensor rays at the camera's height meet (cameras sit at
    the agent's centre, sim.cpp:220-221; every agent and food entity stands at
    z = 1 with scale 1, sim.cpp:204-211, :332-345)."""
    V, F = [], []
    with open(path) as f:
        for line in f:
            t = line.split()
            if not t:
                continue
            if t[0] == "v":
                V.append([float(v) for v in t[1:4]])
            elif t[0] == "f":
                F.append([int(x.split("/")[0]) - 1 for x in t[1:]])
    V = np.array(V)
    pts = []
    for face in F:
        for i in range(len(face)):
            a, b = V[face[i]], V[face[(i + 1) % len(face)]]
            if (a[2] - z) * (b[2] - z) < 0 or (a[2] == z) != (b[2] == z):
                t = (z - a[2]) / (b[2] - a[2])
                pts.append(a + (b - a) * t)
    r = np.linalg.norm(np.array(pts)[:, :2], axis=1)
    return [round(float(r.min()), 6), round(float(r.max()), 6)]


def reference_shapes():
    import torch
    out = {"source": "read from /root/reference by tests/golden/make_golden.py"}
    species = {}
    for f in sorted(glob.glob(f"{REF}/checkpoints/universe_violence/species_*/latest_model_epoch_*.pt")):
        d = torch.load(f, weights_only=True, map_location="cpu")
        mc = d["model_config"]
        sd = d["model_state_dict"]
        species[os.path.basename(os.path.dirname(f))] = {
            "obs_dim": int(mc["layers"][0]["in_features"]),
            "action_dim": int(mc["actor"][-1]["out_features"]),
            "recurrent": mc["recurrent"]["type"],
            "feature0_weight_shape": list(sd["a2c_nets.feature.0.weight"].shape),
        }
    out["checkpoints"] = species
    out["obs_dim"] = sorted({v["obs_dim"] for v in species.values()})
    out["action_dim"] = sorted({v["action_dim"] for v in species.values()})
    out["mesh_abs_extent"] = {m: obj_extent(f"{REF}/data/{m}")
                             for m in ("agent_render.obj", "cube_render.obj")}
    # the agent disc of the sensor spec: radius 0.92 covers this
    out["agent_section_z0_radii"] = obj_section_radii(f"{REF}/data/agent_render.obj")
    return out


def main():
    pyoracle.build()
    if os.path.isdir(REF):
        with open(os.path.join(HERE, "reference_shapes.json"), "w") as f:
            json.dump(reference_shapes(), f, indent=1, sort_keys=True)
        print("reference_shapes.json written")
    for fx in FIXTURES:
        save_fixture(*fx)
    save_horizon(*HORIZON)


if __name__ == "__main__":
    main()

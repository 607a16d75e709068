"""Helpers for the committed golden fixtures (tests/golden/*.npz)."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = ["species", "pos", "health", "surround", "reward", "action", "stats", "hidden",
         "semantic", "depth"]
FIXTURES = [
    ("oracle_w4_a32_s69", 4, 32, 69, 16, False, 128),
    ("oracle_w8_a4_s7_fixed", 8, 4, 7, 24, True, 16),
]


def load_fixture(name):
    z = np.load(os.path.join(HERE, "golden", name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    arrays = {k: z[k] for k in z.files if k != "meta"}
    return meta, arrays


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def table_digests(get, species_count):
    """get(name, is_prev) -> numpy array in the oracle's dtypes."""
    out = {}
    for nm in NAMES:
        out[nm] = digest(get(nm, False))
        out["prev_" + nm] = digest(get(nm, True))
    out["species_count"] = digest(species_count)
    return out


def run_digests(sim, meta):
    """Drive the oracle through the fixture's call sequence."""
    def get(nm, prev):
        return sim.column(NAMES.index(nm), prev)
    log = [["init", sim.num_agents(), table_digests(get, sim.species_count())]]
    for t in range(meta["steps"]):
        sim.write_synthetic_actions(meta["action_seed"], t, meta["write_hidden"])
        sim.step()
        log.append([f"step{t}", sim.num_agents(), table_digests(get, sim.species_count())])
        sim.shift_observations()
        log.append([f"shift{t}", sim.num_agents(), table_digests(get, sim.species_count())])
    return log

"""CPU: the oracle reproduces the committed golden vectors, and the boundary
shapes match what the reference's own files pin (tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest

import pyoracle as po
from golden_util import FIXTURES, load_fixture, run_digests

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("name", [f[0] for f in FIXTURES])
def test_oracle_reproduces_golden(name):
    meta, arrays = load_fixture(name)
    sim = po.OracleSim(meta["worlds"], meta["seed"], meta["agents"], cap=meta["cap"],
                       reward_fixed=meta["reward_fixed"])
    log = run_digests(sim, meta)
    for (tag, n, dg), (tag2, n2, dg2) in zip(meta["log"], log):
        assert tag == tag2 and n == n2, (tag, n, n2)
        bad = [k for k in dg if dg[k] != dg2[k]]
        assert not bad, f"{name} {tag}: columns differ: {bad}"


def test_reference_boundary_shapes():
    ref = json.load(open(os.path.join(HERE, "golden", "reference_shapes.json")))
    # learn/env.py:19 obs = depth 32 + health 1 + position 2 + semantic 32 + surrounding 2
    assert ref["obs_dim"] == [32 + 1 + 2 + 32 + 2]
    assert ref["action_dim"] == [6]
    sim = po.OracleSim(2, 69, 32)
    widths = {c: sim.column(c).shape[1] for c in range(10)}
    assert widths[po.COL_DEPTH] + widths[po.COL_HEALTH] + widths[po.COL_POS] + \
        widths[po.COL_SEMANTIC] + widths[po.COL_SURROUND] == ref["obs_dim"][0]
    assert widths[po.COL_ACTION] == ref["action_dim"][0]
    # sensor objects: food the +-1 cube; agents the agent mesh's cross-section
    # in the rays' plane (z = 0 of the mesh: the camera sits at the agent's
    # centre), radii 0.910-0.921 -> the spec's disc of radius 0.92, which the
    # near sphere 1.1 (mgr.cpp:133) clears, so a camera never sees its own body
    ext = ref["mesh_abs_extent"]
    assert 1.0 <= ext["agent_render.obj"] <= 1.2 and ext["cube_render.obj"] == 1.0
    lo, hi = ref["agent_section_z0_radii"]
    assert lo <= 0.92 and abs(hi - 0.92) < 1e-3 and hi < 1.1


def test_golden_final_tables_consistent():
    meta, arrays = load_fixture("oracle_w4_a32_s69")
    sc = arrays["species_count"]
    assert sc.sum() == arrays["species"].shape[0]
    assert (np.diff(arrays["species"].ravel()) >= 0).all()

"""GPU parity: HIP product vs the CPU oracle, bitwise on every exported column.

The oracle (oracle/mbots_oracle.c) restates src/sim/sim.cpp; both sides run the
same seeds and the identity-keyed synthetic action stream, so
integer columns must be bit-exact and float columns bit-exact too (the float
tolerance the north star allows, 1e-5, is not needed: both sides round
identically with -ffp-contract=off)."""
import numpy as np
import pytest

import pyoracle
from simpair import compare

pytestmark = pytest.mark.gpu


def _pair(W, seed=69, A=32, steps=12, cap=128, reward_fixed=False, depth_fixed=False,
          write_hidden=True, world_offset=0):
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, seed, A, agent_capacity=cap, reward_fixed=reward_fixed,
                        fix_depth_alias=depth_fixed, world_offset=world_offset)
    orc = pyoracle.OracleSim(W, seed, A, cap=cap, reward_fixed=reward_fixed,
                             world_offset=world_offset, num_threads=8)
    errs = compare(mgr, orc, "init", depth_fixed=depth_fixed)
    assert not errs, errs[:5]
    for t in range(steps):
        mgr.write_synthetic_actions(1234, t, write_hidden)
        orc.write_synthetic_actions(1234, t, write_hidden)
        mgr.step()
        orc.step()
        errs = compare(mgr, orc, f"step {t}", depth_fixed=depth_fixed)
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
        errs = compare(mgr, orc, f"shift {t}", depth_fixed=depth_fixed)
        assert not errs, errs[:5]
    return mgr, orc


def test_parity_small():
    _pair(4, steps=24)


def test_parity_64_worlds():
    _pair(64, steps=40)


def test_parity_reward_fixed_and_depth():
    _pair(32, steps=16, reward_fixed=True, depth_fixed=True)


def test_parity_seed_and_offset():
    _pair(48, seed=7, steps=16, world_offset=1000)


def test_parity_small_population():
    # A=4 -> one agent per species; respawn path exercised constantly
    _pair(64, A=4, steps=30, cap=16)


def test_parity_4096_worlds():
    _pair(4096, steps=6)

"""Parity at the bench's horizon: BASELINE config 2's
4096 worlds driven by bench.py's own loop -- identity-keyed one-hot actions
(seed 1234, no memory writes), step(), shift_observations() -- for 120 steps,
against the oracle's per-step digests of every exported column
(tests/golden/oracle_w4096_a32_s69_h120.npz, tests/golden/make_golden.py).
By step 120 the population has drifted from 32 to ~33 agents per world
through breeding, shooting, starvation and respawns (sim.cpp:505-581,
:791-838), the paths short runs barely reach.

* every step: every column after every step() and every shift (each read
  materialises the step's deferred moves);
* the bench path: nothing read in between (the lazy shift, the aliased
  Action / HiddenState and the deferred moves stay as the bench leaves them),
  the tables compared after steps 30, 60, 90 and 120.
"""
import numpy as np
import pytest

from golden_util import load_fixture, table_digests

NAME = "oracle_w4096_a32_s69_h120"
ACC = {"species": "species_tensor", "pos": "position_tensor", "health": "health_tensor",
       "surround": "surrounding_tensor", "reward": "reward_tensor", "action": "action_tensor",
       "stats": "stats_tensor", "hidden": "hidden_state_tensor", "semantic": "semantic_tensor"}


def _digests(mgr):
    def get(nm, prev):
        if nm == "depth":   # depth aliases the semantic column (B.1): not compared twice
            return np.zeros(0)
        a = getattr(mgr, ACC[nm])(prev).to_torch().cpu().numpy()
        return a.view(np.int32) if nm == "health" else a
    return table_digests(get, mgr.species_count_tensor().to_torch().cpu().numpy())


def _check(entry, mgr):
    tag, n, want = entry
    assert mgr.num_agents() == n, (tag, mgr.num_agents(), n)
    got = _digests(mgr)
    bad = [k for k in want if "depth" not in k and want[k] != got[k]]
    assert not bad, f"{tag}: columns differ from the oracle: {bad}"


def test_oracle_reproduces_horizon_head():
    """The fixture pinned by its generator: the oracle's first 6 steps."""
    import pyoracle
    meta, _ = load_fixture(NAME)
    sim = pyoracle.OracleSim(meta["worlds"], meta["seed"], meta["agents"], num_threads=8)
    log = meta["log"]

    def dg():
        return {k: v for k, v in table_digests(lambda nm, p: sim.column(["species", "pos", "health", "surround",
                                                                         "reward", "action", "stats", "hidden",
                                                                         "semantic", "depth"].index(nm), p),
                                               sim.species_count()).items()}
    assert log[0][2] == dg()
    for t in range(6):
        sim.write_synthetic_actions(meta["action_seed"], t, meta["write_hidden"])
        sim.step()
        assert [sim.num_agents(), dg()] == log[1 + 2 * t][1:], f"step{t}"
        sim.shift_observations()
        assert [sim.num_agents(), dg()] == log[2 + 2 * t][1:], f"shift{t}"


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_hip_horizon_every_step():
    import madrona_bots as mb
    meta, _ = load_fixture(NAME)
    log = meta["log"]
    mgr = mb.SimManager(0, meta["worlds"], meta["seed"], meta["agents"])
    _check(log[0], mgr)
    for t in range(meta["steps"]):
        mgr.write_synthetic_actions(meta["action_seed"], t, meta["write_hidden"])
        mgr.step()
        _check(log[1 + 2 * t], mgr)
        mgr.shift_observations()
        _check(log[2 + 2 * t], mgr)
    assert mgr.overflow() == meta["overflow"] == 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_hip_horizon_bench_path():
    import madrona_bots as mb
    meta, _ = load_fixture(NAME)
    log = meta["log"]
    mgr = mb.SimManager(0, meta["worlds"], meta["seed"], meta["agents"])
    for t in range(meta["steps"]):
        mgr.write_synthetic_actions(meta["action_seed"], t, meta["write_hidden"])
        mgr.step()
        mgr.shift_observations()
        if (t + 1) % 30 == 0:
            _check(log[2 + 2 * t], mgr)

"""The reference training loop's own view pattern on the GPU, against the oracle
(VERDICT r5 item 1): learn/training_loop.py:43-48 fetches the Action and
HiddenState views once right after step(), :135 shifts once per species, and
:136-137 then writes the new actions and memory through those pre-shift views.
Whether the writes reach the next K1 depends on the manager's deferred-move
state machine (the alias / pending flags and the eager-vs-fused shift), so
harness/rollout.learner_rollout runs that exact pattern on the HIP manager and
on tests/oracle_adapter.OracleSimManager with the same CPU generator, and every
tensor the loop reads (observations, previous observations, rewards, health,
memory, PrevHiddenState, previous actions) must be bitwise equal, step after
step.  `observe=True` also compares every table column, current and Prev,
after each step's writes (the accessors then copy the deferred columns out,
another path through the state machine); `observe=False` leaves the loop's
own reads as the only ones until the end.

Crossed with the schedule modes: MBOTS_SWAP=1 at 16384
worlds carries the learner pattern, a checkpoint hand-over in the middle of
it and a graph-captured pair of steps."""
import os
import sys

import numpy as np
import pytest
import torch

import pyoracle
from simpair import compare
from oracle_adapter import OracleSimManager

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd", "harness"))
import rollout  # noqa: E402

pytestmark = pytest.mark.gpu


def _bits(t):
    a = np.ascontiguousarray(t.detach().cpu().numpy())
    return a.view(np.uint32) if a.dtype.itemsize == 4 else a.view(np.uint8)


class _Log:
    """Every tensor the loop reads, as host copies keyed (step, species, name)."""

    def __init__(self):
        self.d = {}

    def __call__(self, t, sp, name, x):
        self.d[(t, sp, name)] = x.detach().cpu().clone()


def _diff(a, b, where):
    errs = []
    if a.d.keys() != b.d.keys():
        return [f"{where}: read sets differ: {sorted(set(a.d) ^ set(b.d))[:4]}"]
    for k in sorted(a.d):
        x, y = a.d[k], b.d[k]
        if x.shape != y.shape or x.dtype != y.dtype or not np.array_equal(_bits(x), _bits(y)):
            errs.append(f"{where}: {k} differs (shape {tuple(x.shape)} vs {tuple(y.shape)})")
    return errs


def _run(W, steps, per_species, fused, seed=1234):
    """The whole HIP loop, then the whole oracle loop: no read but the loop's
    own until the end."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32)
    ref = OracleSimManager(0, W, 69, 32, num_threads=8)
    lg, lo = _Log(), _Log()
    rollout.learner_rollout(mgr, steps, seed=seed, shift_per_species=per_species, fused=fused, record=lg)
    rollout.learner_rollout(ref, steps, seed=seed, shift_per_species=per_species, record=lo)
    errs = _diff(lg, lo, f"W={W}")
    assert not errs, errs[:5]
    errs = compare(mgr, ref._s, f"W={W} end")
    assert not errs, errs[:5]
    return mgr, ref


@pytest.mark.parametrize("observe", [False, True])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("per_species", [True, False])
@pytest.mark.parametrize("W", [64, 4096])
def test_learner_pattern_matches_oracle(W, per_species, fused, observe):
    """64 worlds run in K1-finder mode, 4096 on the joined schedule with its
    value waits; 8 steps of the training loop's call pattern each."""
    if observe:
        _side_by_side(W, 8, per_species, fused)
    else:
        _run(W, 8, per_species, fused)


def _side_by_side(W, steps, per_species, fused, gen_seed=1234):
    """The two loops in lockstep (one step each, same generator state), every
    table column compared after each step's writes."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32)
    ref = OracleSimManager(0, W, 69, 32, num_threads=8)
    gg = torch.Generator().manual_seed(gen_seed)
    go = torch.Generator().manual_seed(gen_seed)
    for t in range(steps):
        lg, lo = _Log(), _Log()
        rollout.learner_rollout(mgr, 1, shift_per_species=per_species, fused=fused, record=lg, gen=gg)
        rollout.learner_rollout(ref, 1, shift_per_species=per_species, record=lo, gen=go)
        errs = _diff(lg, lo, f"W={W} step {t}")
        errs += compare(mgr, ref._s, f"W={W} step {t}")
        assert not errs, errs[:5]
    return mgr, ref


def test_learner_pattern_long_horizon_4096():
    """20 steps of the loop's pattern at config 2's size (per-species shifts,
    fused observation rows), compared only at the end: the deferred moves and
    aliases stay on the loop's own path the whole way."""
    _run(4096, 20, True, True, seed=77)


@pytest.mark.parametrize("swap", ["1", "0"])
def test_learner_pattern_swap_schedule_16384(monkeypatch, swap):
    """Both large-world schedules -- K1 / K2 / the sensor on the internal
    stream (MBOTS_SWAP=1, the default above 8192 worlds) and the sensor forked
    off the caller's stream (MBOTS_SWAP=0) -- under the training loop's
    pattern, then a checkpoint hand-over in the middle of the loop into a
    fresh manager of the same schedule, then more of the pattern: every read
    and every column equal the oracle's."""
    import madrona_bots as mb
    W = 16384
    monkeypatch.setenv("MBOTS_SWAP", swap)   # read when a manager is created
    mgr = mb.SimManager(0, W, 69, 32)
    assert mgr.schedule_info()["swap"] == (swap == "1")
    ref = OracleSimManager(0, W, 69, 32, num_threads=16)
    gg = torch.Generator().manual_seed(5)
    go = torch.Generator().manual_seed(5)

    def steps(m, n, fused):
        for t in range(n):
            lg, lo = _Log(), _Log()
            rollout.learner_rollout(m, 1, shift_per_species=True, fused=fused, record=lg, gen=gg)
            rollout.learner_rollout(ref, 1, shift_per_species=True, record=lo, gen=go)
            errs = _diff(lg, lo, f"swap step {t}")
            assert not errs, errs[:5]
    steps(mgr, 4, fused=True)
    blob = mgr.save_checkpoint()
    mgr2 = mb.SimManager(0, W, 69, 32)
    mgr2.load_checkpoint(blob)
    del mgr
    steps(mgr2, 4, fused=False)
    monkeypatch.delenv("MBOTS_SWAP", raising=False)
    errs = compare(mgr2, ref._s, "swap end")
    assert not errs, errs[:5]


@pytest.mark.parametrize("swap", ["1", "0"])
def test_swap_schedule_graph_capture_16384(monkeypatch, swap):
    """A graph-captured pair of steps (with the synthetic writer) replayed on
    a manager of either large-world schedule, after eager steps: the replays
    equal the same sequence on the oracle, bitwise."""
    import madrona_bots as mb
    W = 16384
    monkeypatch.setenv("MBOTS_SWAP", swap)
    mgr = mb.SimManager(0, W, 69, 32)
    assert mgr.schedule_info()["swap"] == (swap == "1")
    monkeypatch.delenv("MBOTS_SWAP", raising=False)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for t in range(3):
            mgr.write_synthetic_actions(1234, t, True)
            orc.write_synthetic_actions(1234, t, True)
            mgr.step(); orc.step()
            mgr.shift_observations(); orc.shift_observations()
        mgr.write_synthetic_actions(1234, 3, True)
        orc.write_synthetic_actions(1234, 3, True)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 4, True)
            mgr.step(); mgr.shift_observations(); mgr.write_synthetic_actions(1234, 5, True)
            mgr.join()
    for _ in range(2):
        g.replay()
        for t in (4, 5):
            orc.step(); orc.shift_observations(); orc.write_synthetic_actions(1234, t, True)
    errs = compare(mgr, orc, "swap graph")
    assert not errs, errs[:5]
    # and eager swap-schedule steps after the replays
    for t in range(6, 9):
        mgr.write_synthetic_actions(1234, t, True)
        orc.write_synthetic_actions(1234, t, True)
        mgr.step(); orc.step()
        mgr.shift_observations(); orc.shift_observations()
    errs = compare(mgr, orc, "swap after graph")
    assert not errs, errs[:5]

"""Checkpoint / restore and the per-world debug dump (SURVEY 8f items 3-4;
not in the reference).  A manager restored from a checkpoint continues
bit-exactly; world_state matches the oracle's world state."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

ACCESSORS = ["depth_tensor", "semantic_tensor", "reward_tensor", "position_tensor",
             "health_tensor", "surrounding_tensor", "action_tensor", "stats_tensor",
             "hidden_state_tensor", "species_tensor"]


def _snap(sim):
    out = {"species_count": sim.species_count_tensor().to_torch().cpu().clone()}
    for name in ACCESSORS:
        for prev in (False, True):
            t = getattr(sim, name)(prev).to_torch().cpu().contiguous()
            out[(name, prev)] = t.view(torch.uint8).clone()
    return out


def _run(sim, t0, t1, write_hidden=True):
    for t in range(t0, t1):
        sim.write_synthetic_actions(1234, t, write_hidden=write_hidden)
        sim.step()
        sim.shift_observations()


@pytest.mark.gpu
@pytest.mark.parametrize("fix_depth", [False, True])
def test_checkpoint_continues_bit_exactly(tmp_path, fix_depth):
    import madrona_bots as mb
    kw = dict(fix_depth_alias=fix_depth, world_offset=3)
    a = mb.SimManager(0, 96, 11, 24, **kw)
    _run(a, 0, 6)
    path = str(tmp_path / "ck.bin")
    blob = a.save_checkpoint(path)
    _run(a, 6, 11)
    ref = _snap(a)
    b = mb.SimManager(0, 96, 11, 24, **kw)
    b.load_checkpoint(path)
    _run(b, 6, 11)
    got = _snap(b)
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
    c = mb.SimManager(0, 96, 11, 24, **kw)
    c.load_checkpoint(blob.tobytes())
    _run(c, 6, 8)
    assert c.num_agents() > 0


@pytest.mark.gpu
def test_checkpoint_with_aliased_action_hidden(tmp_path):
    """Saved right after a fused shift while HiddenState was never written
    (write_hidden=False): the current Action / HiddenState columns are views of
    their Prev copies (DESIGN.md "Aliased current Action / HiddenState") and the
    save copies them out; the restored manager continues bit-exactly."""
    import madrona_bots as mb
    a = mb.SimManager(0, 64, 13, 24)
    _run(a, 0, 3)                        # nonzero HiddenState first
    _run(a, 3, 5, write_hidden=False)
    blob = a.save_checkpoint()
    _run(a, 5, 9, write_hidden=False)
    ref = _snap(a)
    b = mb.SimManager(0, 64, 13, 24)
    b.load_checkpoint(blob.tobytes())
    _run(b, 5, 9, write_hidden=False)
    got = _snap(b)
    for k in ref:
        assert torch.equal(ref[k], got[k]), k


@pytest.mark.gpu
def test_checkpoint_rejects_other_config():
    import madrona_bots as mb
    a = mb.SimManager(0, 32, 5, 16)
    a.step()
    blob = a.save_checkpoint()
    b = mb.SimManager(0, 32, 6, 16)
    with pytest.raises(RuntimeError):
        b.load_checkpoint(blob.tobytes())


@pytest.mark.gpu
def test_world_state_matches_oracle():
    import madrona_bots as mb
    import pyoracle as po
    sim = mb.SimManager(0, 8, 69, 32)
    orc = po.OracleSim(8, 69, 32, cap=128)
    for t in range(5):
        sim.write_synthetic_actions(1234, t)
        orc.write_synthetic_actions(1234, t)
        sim.step(); orc.step()
        sim.shift_observations(); orc.shift_observations()
    for w in range(8):
        g, o = sim.world_state(w), orc.world_state(w)
        assert np.array_equal(g["position"].view(np.int32), o["xy"].view(np.int32))
        assert np.array_equal(g["rotation_wz"].view(np.int32), o["rot"].view(np.int32))
        assert np.array_equal(g["species"], o["species"])
        assert np.array_equal(g["health"], o["health"])
        assert np.array_equal(g["finder"], o["finder"])
        assert len(g["food"]) <= 30
        assert np.array_equal(g["food"], o["food"])   # (chunk, x, y, box rotation)


@pytest.mark.gpu
def test_checkpoint_between_step_and_shift(tmp_path):
    """A save right after step() (every deferred Prev move and the Action /
    HiddenState move still pending) restores to the same state: both managers
    then shift and step on identically."""
    import madrona_bots as mb
    a = mb.SimManager(0, 48, 5, 24)
    _run(a, 0, 4)
    a.write_synthetic_actions(1234, 4, write_hidden=True)
    a.step()                                 # no accessor, no shift
    path = str(tmp_path / "mid.bin")
    a.save_checkpoint(path)
    b = mb.SimManager(0, 48, 5, 24)
    b.load_checkpoint(path)
    for sim in (a, b):
        sim.shift_observations()
        _run(sim, 5, 8)
    ra, rb = _snap(a), _snap(b)
    for k in ra:
        assert torch.equal(ra[k], rb[k]), k


@pytest.mark.gpu
def test_set_action_after_step_then_shift():
    """set_action between step() and shift_observations() lands in the row the
    shift copies to PrevAction (the deferred Action move runs first)."""
    import madrona_bots as mb
    m = mb.SimManager(0, 16, 69, 32)
    m.write_synthetic_actions(1234, 0)
    m.step()
    before = m.action_tensor(False).to_torch().clone()
    m.step()
    m.set_action(3, 1, 0, 1, 0, 1, 0)
    m.shift_observations()
    prev = m.action_tensor(True).to_torch()
    cur = m.action_tensor(False).to_torch()
    assert prev[3].tolist() == [1, 0, 1, 0, 1, 0]
    assert torch.equal(prev, cur)
    assert before.shape[1] == 6


@pytest.mark.gpu
@pytest.mark.parametrize("ghost", [False, True])
def test_checkpoint_load_then_save_before_stepping(ghost):
    """a restored manager saved again before any step writes the
    same blob (the table's row count -- every row, the shard ghost's included,
    kCkptVersion 3+ -- comes back with the state), and an older version's blob
    is refused."""
    import madrona_bots as mb
    kw = dict(shard_ghost=ghost)
    a = mb.SimManager(0, 64, 5, 32, **kw)
    _run(a, 0, 7)
    blob = a.save_checkpoint()
    b = mb.SimManager(0, 64, 5, 32, **kw)
    b.load_checkpoint(blob)
    assert b.num_rows() == a.num_rows() > b.num_agents() if ghost else b.num_rows() == a.num_rows()
    again = b.save_checkpoint()
    assert np.array_equal(blob, again)
    old = blob.copy()
    old[8:12] = np.frombuffer(np.uint32(2).tobytes(), np.uint8)   # header version field
    c = mb.SimManager(0, 64, 5, 32, **kw)
    with pytest.raises(RuntimeError, match="version"):
        c.load_checkpoint(old)


@pytest.mark.gpu
def test_checkpoint_with_bad_totals_leaves_manager_intact():
    """a blob whose saved row count disagrees with its header is
    refused before anything is overwritten (the target keeps its own state)."""
    import madrona_bots as mb
    a = mb.SimManager(0, 64, 5, 32)
    _run(a, 0, 5)
    blob = a.save_checkpoint()
    b = mb.SimManager(0, 64, 5, 32)
    _run(b, 0, 2)
    mine = b.save_checkpoint()
    # header (56 B), 11 agent columns of 64 x 128 slots, the per-world arrays
    # (n, ctr, key, food, food_rot, cur_food, sreward, scount, row_base,
    # world_off, overflow: 1420 B per world), then totals[8]
    tot = 56 + 11 * 64 * 128 * 4 + 64 * 1420
    assert int(np.frombuffer(blob[tot + 20:tot + 24].tobytes(), np.uint32)[0]) == a.num_rows()
    bad = blob.copy()
    bad[tot + 20:tot + 24] = np.frombuffer(np.uint32(a.num_rows() + 1).tobytes(), np.uint8)
    with pytest.raises(RuntimeError, match="disagrees"):
        b.load_checkpoint(bad)
    assert np.array_equal(b.save_checkpoint(), mine)

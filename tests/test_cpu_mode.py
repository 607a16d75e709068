"""CPU execution mode (exec_mode="cpu", the reference Manager's ExecMode::CPU;
BASELINE config 1: "64 worlds, ExecMode::CPU via learn/env.py, runs without a
GPU").  The product's host path (madrona-bots_amd/csrc/mbots_cpu.cpp, inside
libmbots.so) against the oracle, bitwise on every exported column -- no GPU
needed, so these run in the CPU suite."""
import numpy as np
import pytest
import torch

import pyoracle
from simpair import compare


def _mgr(W, seed=69, A=32, **kw):
    import madrona_bots as mb
    return mb.SimManager(0, W, seed, A, exec_mode="cpu", **kw)


def _pair(W, seed=69, A=32, steps=10, cap=128, reward_fixed=False, depth_fixed=False,
          world_offset=0, write_hidden=True):
    mgr = _mgr(W, seed, A, agent_capacity=cap, reward_fixed=reward_fixed,
               fix_depth_alias=depth_fixed, world_offset=world_offset)
    orc = pyoracle.OracleSim(W, seed, A, cap=cap, reward_fixed=reward_fixed,
                             world_offset=world_offset, num_threads=4)
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


def test_config1_64_worlds_matches_oracle():
    _pair(64, steps=25)


def test_reward_fixed_depth_seed_offset():
    _pair(16, seed=7, steps=12, reward_fixed=True, depth_fixed=True, world_offset=1000)


def test_small_population_and_capacity_overflow():
    mgr, orc = _pair(32, A=4, steps=20, cap=8)
    assert mgr.overflow() == orc.overflow()


def test_views_are_host_zero_copy_and_writable():
    mgr = _mgr(8)
    mgr.step()
    n = mgr.num_agents()
    a = mgr.action_tensor(False).to_torch()
    assert a.device.type == "cpu" and tuple(a.shape) == (n, 6) and a.dtype == torch.int32
    a.zero_()
    a[3, 5] = 1
    assert int(mgr.action_tensor(False).to_torch()[3, 5]) == 1
    mgr.set_action(4, 1, 0, 0, 0, 0, 0)
    assert mgr.action_tensor(False).to_torch()[4].tolist() == [1, 0, 0, 0, 0, 0]
    h = mgr.health_tensor(False).to_torch()
    assert h.dtype == torch.float32 and int(h.view(torch.int32).max()) <= 200
    assert tuple(mgr.species_count_tensor().to_torch().shape) == (8, 4)
    assert tuple(mgr.done_tensor().to_torch().shape) == (n, 1)


def test_offsets_sensor_index_and_world_state():
    mgr, orc = _pair(24, steps=6)
    counts, offsets = orc.world_counts()
    assert [mgr.agent_offset_for_world(w) for w in range(24)] == offsets.tolist()
    si = mgr.sensor_index_tensor().to_torch().numpy().ravel()
    assert np.array_equal(si, orc.sensor_index())
    for w in (0, 11, 23):
        g, o = mgr.world_state(w), orc.world_state(w)
        assert np.array_equal(g["position"].view(np.int32), o["xy"].view(np.int32))
        assert np.array_equal(g["finder"], o["finder"])
        assert np.array_equal(g["food"], o["food"])


def test_construct_obs_matches_torch_cat():
    mgr, _ = _pair(8, steps=3)
    for prev in (False, True):
        want = torch.cat((mgr.depth_tensor(prev).to_torch(), mgr.health_tensor(prev).to_torch(),
                          mgr.position_tensor(prev).to_torch(), mgr.semantic_tensor(prev).to_torch(),
                          mgr.surrounding_tensor(prev).to_torch()), dim=1)
        got = mgr.construct_obs(prev)
        assert got.device.type == "cpu"
        assert torch.equal(got.view(torch.int32), want.view(torch.int32))


def test_checkpoint_continues_bit_exactly(tmp_path):
    a = _mgr(16)
    for t in range(5):
        a.write_synthetic_actions(1234, t, True)
        a.step()
        a.shift_observations()
    blob = a.save_checkpoint(tmp_path / "ck.bin")
    b = _mgr(16)
    b.load_checkpoint(tmp_path / "ck.bin")
    for t in range(5, 9):
        for m in (a, b):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            m.shift_observations()
    for name in ("position_tensor", "reward_tensor", "semantic_tensor", "hidden_state_tensor"):
        for prev in (False, True):
            assert torch.equal(getattr(a, name)(prev).to_torch(), getattr(b, name)(prev).to_torch())
    with pytest.raises(RuntimeError):
        _mgr(8).load_checkpoint(blob.tobytes())


def test_bad_exec_mode_rejected():
    import madrona_bots as mb
    with pytest.raises(ValueError):
        mb.SimManager(0, 4, 69, 32, exec_mode="tpu")


@pytest.mark.gpu
def test_cpu_mode_equals_hip_mode():
    """The two execution modes of one library: the same stream leaves the same
    bits in every column (config 1 size)."""
    g = _pair_modes(64, steps=12)
    assert g


def _pair_modes(W, steps):
    import madrona_bots as mb
    h = mb.SimManager(0, W, 69, 32)
    c = _mgr(W)
    for t in range(steps):
        for m in (h, c):
            m.write_synthetic_actions(1234, t, True)
            m.step()
        _same(h, c, f"step {t}")
        for m in (h, c):
            m.shift_observations()
        _same(h, c, f"shift {t}")
    return True


def _same(h, c, where):
    assert h.num_agents() == c.num_agents(), where
    for name in ("species_tensor", "position_tensor", "health_tensor", "surrounding_tensor",
                 "reward_tensor", "action_tensor", "stats_tensor", "hidden_state_tensor",
                 "semantic_tensor", "depth_tensor"):
        for prev in (False, True):
            a = getattr(h, name)(prev).to_torch().cpu()
            b = getattr(c, name)(prev).to_torch()
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)), (where, name, prev)


def test_breed_heavy_to_capacity_256():
    """A breed-heavy stream fills worlds to 256 slots; births past it are
    dropped and counted exactly as the oracle does."""
    import madrona_bots as mb
    W = 16
    mgr = _mgr(W, agent_capacity=256)
    orc = pyoracle.OracleSim(W, 69, 32, cap=256, num_threads=4)
    with pytest.warns(mb.CapacityWarning, match=f"at most {mb.MAX_CAPACITY}"):
        _breed_steps(mgr, orc, 40)
    assert mgr.overflow() == orc.overflow() > 0


@pytest.mark.parametrize("cap,W,steps", [(512, 16, 70), (1024, 8, 110)])
def test_breed_heavy_large_capacity_classes(cap, W, steps):
    """The 512- and 1024-slot classes (64-bit sensor keys: agent orders past
    511) under the breed-heavy stream until the cap binds: every column and
    the dropped-birth count equal the oracle's."""
    import madrona_bots as mb
    mgr = _mgr(W, agent_capacity=cap)
    orc = pyoracle.OracleSim(W, 69, 32, cap=cap, num_threads=4)
    with pytest.warns(mb.CapacityWarning):
        peak = _breed_steps(mgr, orc, steps)
    assert peak == cap
    assert mgr.overflow() == orc.overflow() > 0


def test_auto_capacity_grows_without_drops():
    """agent_capacity="auto": the breed-heavy stream grows the worlds through
    the capacity classes (the state moved by a cross-capacity checkpoint before
    each step that could overflow) and every column stays bitwise equal to an
    oracle that never drops an agent -- the reference's unbounded tables, up to
    1024 per world."""
    import madrona_bots as mb
    W = 8
    mgr = _mgr(W, agent_capacity="auto")
    orc = pyoracle.OracleSim(W, 69, 32, cap=1024, num_threads=4)
    assert mgr.agent_capacity == 128
    seen = {mgr.agent_capacity}
    peak = 0
    for t in range(80):
        peak = max(peak, _breed_steps(mgr, orc, 1, t0=t))
        seen.add(mgr.agent_capacity)
    assert {128, 256, 512} <= seen and peak > 256
    assert mgr.overflow() == orc.overflow() == 0


def test_auto_capacity_failed_growth_keeps_the_run(monkeypatch):
    """A growth whose checkpoint load fails raises and leaves the manager in
    its old class with its state (not a fresh world); the run then carries on,
    grows once loads work again and stays equal to the oracle."""
    import madrona_bots as mb
    W = 8
    mgr = _mgr(W, agent_capacity="auto")
    orc = pyoracle.OracleSim(W, 69, 32, cap=1024, num_threads=4)
    real = mb._lib.mbots_load_checkpoint
    monkeypatch.setattr(mb._lib, "mbots_load_checkpoint", lambda *a: -1)
    t = 0
    with pytest.raises(RuntimeError):
        while t < 80:
            _breed_steps(mgr, orc, 1, t0=t)
            t += 1
    assert mgr.agent_capacity == 128 and mgr.num_agents() == orc.num_agents()
    monkeypatch.setattr(mb._lib, "mbots_load_checkpoint", real)
    _breed_steps(mgr, orc, 20, t0=t)
    assert mgr.agent_capacity > 128
    assert mgr.overflow() == orc.overflow() == 0


def test_auto_capacity_old_views_keep_their_storage():
    _old_views_keep_storage("cpu")


@pytest.mark.gpu
def test_auto_capacity_old_views_keep_their_storage_gpu():
    _old_views_keep_storage("hip")


def _old_views_keep_storage(exec_mode):
    """A view (Tensor) taken before a growth still reads the storage it was
    taken from, alive and unchanged, after the manager moved on (on the device
    its to_torch() does not go through the new storage's view cache)."""
    import madrona_bots as mb
    mgr = mb.SimManager(0, 4, 69, 32, exec_mode=exec_mode, agent_capacity="auto")
    old = mgr.position_tensor()
    before = old.to_torch().clone()
    mgr._grow_if_needed = lambda: None   # (only the forced growth below)
    blob = mgr.save_checkpoint()
    keep = mgr._hd
    mgr._open(256)
    import ctypes
    mb._check(mb._lib.mbots_load_checkpoint(mgr._h, ctypes.c_void_p(blob.ctypes.data), blob.size))
    del keep
    assert mgr.agent_capacity == 256
    assert torch.equal(old.to_torch(), before)
    assert torch.equal(mgr.position_tensor().to_torch(), before)
    mgr.step()
    assert torch.equal(old.to_torch(), before)
    assert old.to_torch().data_ptr() != mgr.position_tensor().to_torch().data_ptr()


def test_checkpoint_across_capacities():
    """A checkpoint restores into a manager of another capacity when every
    world fits (the per-slot columns re-laid out); a world that does not fit
    is refused before anything is overwritten."""
    a = _mgr(16, agent_capacity=128)
    for t in range(6):
        a.write_synthetic_actions(1234, t, True)
        a.step()
        a.shift_observations()
    blob = a.save_checkpoint()
    for cap in (512, 64):
        b = _mgr(16, agent_capacity=cap)
        b.load_checkpoint(blob.tobytes())
        for t in range(6, 10):
            for m in (a, b) if cap == 512 else (b,):
                m.write_synthetic_actions(1234, t, True)
                m.step()
                m.shift_observations()
        if cap == 512:
            for name in ("position_tensor", "reward_tensor", "semantic_tensor", "hidden_state_tensor"):
                for prev in (False, True):
                    assert torch.equal(getattr(a, name)(prev).to_torch(), getattr(b, name)(prev).to_torch())
    with pytest.raises(RuntimeError, match="more than agent_capacity"):
        _mgr(16, agent_capacity=32).load_checkpoint(blob.tobytes())


def _breed_steps(mgr, orc, steps, t0=0):
    peak = 0
    for t in range(t0, t0 + steps):
        g = torch.Generator().manual_seed(1000 + t)
        n = mgr.num_agents()
        r = torch.randint(0, 8, (n,), generator=g)
        a = torch.zeros((n, 6), dtype=torch.int32)
        a[r < 4, 5] = 1
        a[(r >= 4) & (r < 6), 0] = 1
        a[r == 6, 2] = 1
        a[r == 7, 3] = 1
        mgr.action_tensor(False).to_torch().copy_(a)
        orc.column(pyoracle.COL_ACTION)[:] = a.numpy()
        mgr.step()
        orc.step()
        errs = compare(mgr, orc, f"step {t}")
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
        peak = max(peak, int(mgr.species_count_tensor().to_torch().sum(1).max()))
    return peak


@pytest.mark.gpu
def test_shard_ghost_learner_actions_cpu_equals_hip():
    """A shard with a ghost world (MBOTS_FLAG_SHARD_GHOST) driven by a learner
    writing Action / HiddenState through the exported views (the reference
    loop, learn/training_loop.py:136-137): the ghost's rows are never written
    by the learner (it only sees rows [0, N)), so they carry their last actions
    through the row moves and the shift -- identically in both execution modes
    (the HIP moves used to stop at row N)."""
    import madrona_bots as mb
    W = 48
    h = mb.SimManager(0, W, 69, 32, shard_ghost=True)
    c = _mgr(W, shard_ghost=True)
    for m in (h, c):
        m.write_synthetic_actions(1234, 0, True)   # every row, the ghost's included
    for t in range(10):
        for m in (h, c):
            m.step()
        _same(h, c, f"step {t}")
        for m in (h, c):
            m.shift_observations()
        n = h.num_agents()
        g = torch.Generator().manual_seed(77 + t)
        a = torch.zeros((n, 6), dtype=torch.int32)
        a[torch.arange(n), torch.randint(0, 6, (n,), generator=g)] = 1
        hid = torch.rand((n, 16), generator=g)
        for m in (h, c):
            m.action_tensor(False).to_torch().copy_(a)
            m.hidden_state_tensor(False).to_torch().copy_(hid)
        _same(h, c, f"write {t}")

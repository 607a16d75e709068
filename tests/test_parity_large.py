"""GPU parity at the BASELINE sizes.

* config 3: 65536 worlds, bitwise against the oracle after every step and
  every shift (the one-wave-per-world sensor path, which only world counts
  above the split threshold take, is also covered at 8192 worlds);
* config 4: 262144 worlds as 8 x 32768 world_offset shards on one device,
  every species segment bit-exact against one 262144-world manager (world RNG
  keys are split from the global world index, sim.cpp:1238-1239);
* config 5: the learner-rank reassembly of the rollout gather
  (harness/gather.py) on device, two shard managers against one manager.
"""
import os

import numpy as np
import pytest
import torch

import pyoracle
from simpair import COLUMNS, compare

pytestmark = pytest.mark.gpu


def oracle_threads():
    """Host threads the oracle may use: the CPUs this process may run on,
    capped at the GPU box's per-GPU share (16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _pair(W, steps, **kw):
    import madrona_bots as mb
    mgr = mb.SimManager(0, W, 69, 32, **kw)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=oracle_threads(),
                             reward_fixed=kw.get("reward_fixed", False),
                             world_offset=kw.get("world_offset", 0))
    errs = compare(mgr, orc, "init")
    assert not errs, errs[:5]
    for t in range(steps):
        mgr.write_synthetic_actions(1234, t, True)
        orc.write_synthetic_actions(1234, t, True)
        mgr.step()
        orc.step()
        errs = compare(mgr, orc, f"step {t}")
        assert not errs, errs[:5]
        mgr.shift_observations()
        orc.shift_observations()
        errs = compare(mgr, orc, f"shift {t}")
        assert not errs, errs[:5]
    return mgr, orc


def test_parity_8192_worlds_one_wave_sensor():
    # above MB_SENSOR_SPLIT_MAX (4096): sensor_kernel<*, 1>, the config-3 path
    _pair(8192, steps=4)


@pytest.mark.timeout(900)
def test_parity_config3_65536_worlds():
    # 20 steps: every column after every step and shift
    mgr, orc = _pair(65536, steps=20)
    assert mgr.overflow() == orc.overflow() == 0


def _segments(counts):
    """species-major row ranges of a table: [(start, end)] per species."""
    tot = counts.sum(0)
    ends = np.cumsum(tot)
    return [(int(e - t), int(e)) for t, e in zip(tot, ends)]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("reward_fixed", [True, False])
def test_config4_eight_shards_equal_one_manager(reward_fixed):
    """262144 worlds = 8 x 32768 (world_offset = r * 32768) on one device vs one
    262144-world manager: per species, the full table's segment is the
    concatenation of the shards' segments (rows (species, world, slot)).  In
    the faithful B.3 mode shards 0..6 step a ghost of the next shard's first
    world (shard_ghost), as bench.py's ranks do."""
    import madrona_bots as mb
    R, WS = 8, 32768
    steps = 5
    cols = ("species_tensor", "position_tensor", "health_tensor", "surrounding_tensor",
            "reward_tensor", "action_tensor", "stats_tensor", "hidden_state_tensor",
            "semantic_tensor")

    def run(m):
        for t in range(steps):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            m.shift_observations()
        torch.cuda.synchronize()

    full = mb.SimManager(0, R * WS, 69, 32, reward_fixed=reward_fixed)
    run(full)
    shards = []
    for r in range(R):
        s = mb.SimManager(0, WS, 69, 32, reward_fixed=reward_fixed, world_offset=r * WS,
                          shard_ghost=(not reward_fixed) and r < R - 1)
        run(s)
        shards.append(s)
    fcnt = full.species_count_tensor().to_torch().cpu().numpy()
    scnt = [s.species_count_tensor().to_torch().cpu().numpy() for s in shards]
    assert np.array_equal(fcnt, np.concatenate(scnt))
    fseg = _segments(fcnt)
    sseg = [_segments(c) for c in scnt]
    assert full.num_agents() == sum(s.num_agents() for s in shards)
    for nm in cols:
        for prev in (False, True):
            f = getattr(full, nm)(prev).to_torch()
            parts = [getattr(s, nm)(prev).to_torch() for s in shards]
            for sp in range(4):
                a, b = fseg[sp]
                want = torch.cat([parts[r][sseg[r][sp][0]:sseg[r][sp][1]] for r in range(R)])
                assert torch.equal(f[a:b].view(torch.uint8), want.view(torch.uint8)), (nm, prev, sp)
    assert full.overflow() == 0


def test_config5_gather_reassembly_on_device():
    """harness/gather.py's learner-side reassembly (the part of gather_rollout
    after the RCCL gather) on device: two shards' padded row buffers
    reassembled == the rows of one manager holding both shards' worlds."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "madrona-bots_amd", "harness"))
    import gather
    import madrona_bots as mb
    W = 1024

    def run(m):
        for t in range(6):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            if t < 5:
                m.shift_observations()

    full = mb.SimManager(0, 2 * W, 69, 32, reward_fixed=True)
    run(full)
    shards = [mb.SimManager(0, W, 69, 32, reward_fixed=True, world_offset=r * W) for r in range(2)]
    for s in shards:
        run(s)
    rows = [gather.species_rows(s.species_count_tensor().to_torch()) for s in shards]
    all_cnt = torch.stack([r.cpu() for r in rows])
    n_max = int(all_cnt.sum(1).max())
    want = {"obs": full.construct_obs(False), "reward": full.reward_tensor(False).to_torch(),
            "prev_obs": full.construct_obs(True)}
    for name in want:
        bufs = []
        for s in shards:
            t = {"obs": lambda: s.construct_obs(False), "reward": lambda: s.reward_tensor(False).to_torch(),
                 "prev_obs": lambda: s.construct_obs(True)}[name]()
            pad = torch.zeros((n_max,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            pad[:t.shape[0]] = t
            bufs.append(pad)
        got = gather.reassemble(bufs, all_cnt)
        assert torch.equal(got.view(torch.uint8), want[name].view(torch.uint8)), name


@pytest.mark.parametrize("fix_depth", [False, True])
def test_config5_rollout_records_two_shards_equal_one(fix_depth):
    """Config 5 payload: two HIP shards (faithful B.3 rewards, the
    first with the shard ghost) pack 64-B (96-B) rollout records on device;
    the learner-side reassembly + unpack_rollout kernel rebuild [N, 69] rows,
    rewards and stats bit-identical to one manager holding both shards."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "madrona-bots_amd", "harness"))
    import gather
    import madrona_bots as mb
    W = 1024

    def run(m):
        for t in range(6):
            m.write_synthetic_actions(1234, t, True)
            m.step()
            if t < 5:
                m.shift_observations()

    full = mb.SimManager(0, 2 * W, 69, 32, fix_depth_alias=fix_depth)
    run(full)
    shards = [mb.SimManager(0, W, 69, 32, fix_depth_alias=fix_depth, world_offset=r * W,
                            shard_ghost=r == 0) for r in range(2)]
    for s in shards:
        run(s)
    rows = [gather.species_rows(s.species_count_tensor().to_torch()) for s in shards]
    all_cnt = torch.stack([r.cpu() for r in rows])
    n_max = int(all_cnt.sum(1).max())
    rb = shards[0].rollout_record_bytes()
    assert rb == (96 if fix_depth else 64)
    bufs = []
    for s in shards:
        pad = torch.full((n_max, rb), 0xAB, dtype=torch.uint8, device="cuda")
        s.pack_rollout(pad)
        bufs.append(pad)
    got = mb.unpack_rollout(gather.reassemble(bufs, all_cnt))
    want = {"obs": full.construct_obs(False), "reward": full.reward_tensor(False).to_torch(),
            "stats": full.stats_tensor(False).to_torch()}
    for k in want:
        assert torch.equal(got[k].view(torch.int32), want[k].contiguous().view(torch.int32)), k
    # the records hold what the learner needs at 64 B/agent against 280 B of f32 rows + reward
    assert full.pack_rollout().numel() == full.num_agents() * rb


@pytest.mark.gpu
def test_schedules_agree_16384_worlds(monkeypatch):
    """The step's two schedules at large world counts -- K1 / K2 on the
    caller's stream with the sensor forked off (the default), and K1 / K2 /
    the sensor on the internal stream with the caller joining after K2
    (MBOTS_SWAP=1) -- give the same tables, and the oracle's, over 60 steps of
    16384 worlds."""
    import madrona_bots as mb
    W, T = 16384, 60
    mgrs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MBOTS_SWAP", mode)   # read when the manager is created
        mgrs[mode] = mb.SimManager(0, W, 69, 32)
    monkeypatch.delenv("MBOTS_SWAP", raising=False)
    orc = pyoracle.OracleSim(W, 69, 32, num_threads=16)
    for t in range(T):
        wh = t % 3 == 0
        for m in mgrs.values():
            m.write_synthetic_actions(1234, t, wh)
            m.step()
            m.shift_observations()
        orc.write_synthetic_actions(1234, t, wh)
        orc.step()
        orc.shift_observations()
        if t % 20 == 19:
            ref = mgrs["0"]
            for mode in ("1",):
                for name, _ in COLUMNS:
                    for prev in (False, True):
                        a = getattr(ref, name)(prev).to_torch()
                        b = getattr(mgrs[mode], name)(prev).to_torch()
                        assert a.shape == b.shape and torch.equal(a.view(torch.uint8), b.view(torch.uint8)), \
                            (t, mode, name, prev)
    errs = compare(mgrs["0"], orc, "end")
    assert not errs, errs[:5]

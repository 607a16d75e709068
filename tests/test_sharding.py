"""CPU, world_size 2 over gloo: world sharding is exact.

Each rank holds worlds [r*W/2, (r+1)*W/2) with world_offset = r*W/2 (the layout
bench.py uses on GPUs, no collective on the step); every world's RNG key is
split from its *global* index (sim.cpp:1238-1239), so the concatenated shard
states must equal a single instance holding all W worlds, bit for bit.  The
only cross-world read in the reference -- rewards[speciesID] for species 4
reading the next world's SpeciesInfo row (sim.cpp:943) -- reads 0
past a shard's last world; tests/test_parity_gpu.py covers the fixed mode."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as po

W, STEPS = 16, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _world_states(sim, offset):
    out = {}
    for w in range(sim.num_worlds):
        st = sim.world_state(w)
        out[offset + w] = {k: v.copy() for k, v in st.items()}
    return out


def _rewards_by_world(sim, offset):
    """reward column regrouped per (global world, species) in slot order."""
    sc = sim.species_count()
    rew = sim.column(po.COL_REWARD).ravel()
    out, row = {}, 0
    for s in range(4):
        for w in range(sim.num_worlds):
            out[(offset + w, s)] = rew[row:row + sc[w, s]].copy()
            row += sc[w, s]
    return out


def _run(sim):
    for t in range(STEPS):
        sim.write_synthetic_actions(1234, t, True)
        sim.step()
        sim.shift_observations()


def _worker(rank, port, q, reward_fixed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    half = W // 2
    sim = po.OracleSim(half, 69, 32, world_offset=rank * half, reward_fixed=reward_fixed)
    _run(sim)
    # bench.py's reductions: max time over ranks, sum of agent-steps
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([float(sim.num_agents())])
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    states = [None, None]
    dist.all_gather_object(states, (_world_states(sim, rank * half),
                                    _rewards_by_world(sim, rank * half)))
    if rank == 0:
        q.put((float(t.item()), float(n.item()), states))
    dist.destroy_process_group()


@pytest.mark.parametrize("reward_fixed", [True, False])
def test_two_shards_equal_one(reward_fixed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, reward_fixed)) for r in range(2)]
    for p in procs:
        p.start()
    tmax, nsum, states = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    ref = po.OracleSim(W, 69, 32, reward_fixed=reward_fixed)
    _run(ref)
    assert nsum == ref.num_agents()
    full_states = _world_states(ref, 0)
    full_rew = _rewards_by_world(ref, 0)
    for shard_states, shard_rew in states:
        for w, st in shard_states.items():
            for k in st:
                assert np.array_equal(st[k], full_states[w][k]), (w, k)
        for (w, s), r in shard_rew.items():
            boundary = (not reward_fixed) and s == 3 and w == W // 2 - 1
            if boundary:
                # species 4 of the shard's last world: next SpeciesInfo row is
                # past this shard's table (0 here, world 8's rewards[0] unsharded)
                assert r.shape == full_rew[(w, s)].shape
            else:
                assert np.array_equal(r, full_rew[(w, s)]), (w, s)

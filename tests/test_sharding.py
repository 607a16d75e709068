"""CPU, world_size 2 over gloo: world sharding is exact.

Each rank holds worlds [r*W/2, (r+1)*W/2) with world_offset = r*W/2 (the layout
bench.py uses on GPUs, no collective on the step), here through the product's
CPU execution mode; every world's RNG key is split from its *global* index
(sim.cpp:1238-1239), so the concatenated shard states must equal one oracle
instance holding all W worlds, bit for bit.  The one cross-world read in the
reference -- rewards[speciesID] for species 4 reading the next world's
SpeciesInfo row (sim.cpp:943) -- is served by the shard ghost
(shard_ghost=True: each shard also steps the next shard's first world, never
exported), so faithful rewards match too; without the ghost a shard's last
world reads 0 there."""
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


def _world_states(sim, offset, n_worlds, product):
    out = {}
    for w in range(n_worlds):
        st = sim.world_state(w)
        if product:   # madrona_bots key names -> the oracle's
            st = {"xy": st["position"], "rot": st["rotation_wz"], "species": st["species"],
                  "health": st["health"], "finder": st["finder"], "food": st["food"]}
        out[offset + w] = {k: np.asarray(v).copy() for k, v in st.items()}
    return out


def _rewards_by_world(sc, rew, offset):
    """reward column regrouped per (global world, species) in slot order."""
    out, row = {}, 0
    for s in range(4):
        for w in range(sc.shape[0]):
            out[(offset + w, s)] = rew[row:row + sc[w, s]].copy()
            row += sc[w, s]
    return out


def _run(sim):
    for t in range(STEPS):
        sim.write_synthetic_actions(1234, t, True)
        sim.step()
        sim.shift_observations()


def _worker(rank, port, q, reward_fixed, ghost):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MBOTS_CPU_THREADS="2")
    import madrona_bots as mb
    dist.init_process_group("gloo", rank=rank, world_size=2)
    half = W // 2
    # the last shard has no next shard: its last world reads past the table, as
    # one device's last world does
    sim = mb.SimManager(0, half, 69, 32, exec_mode="cpu", world_offset=rank * half,
                        reward_fixed=reward_fixed, shard_ghost=ghost and rank == 0)
    _run(sim)
    # bench.py's reductions: max time over ranks, sum of agent-steps
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([float(sim.num_agents())])
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    sc = sim.species_count_tensor().to_torch().numpy()
    rew = sim.reward_tensor(False).to_torch().numpy().ravel()
    states = [None, None]
    dist.all_gather_object(states, (_world_states(sim, rank * half, half, True),
                                    _rewards_by_world(sc, rew, rank * half)))
    if rank == 0:
        q.put((float(t.item()), float(n.item()), states))
    dist.destroy_process_group()


@pytest.mark.parametrize("reward_fixed,ghost", [(True, False), (False, True), (False, False)])
def test_two_shards_equal_one(reward_fixed, ghost):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, reward_fixed, ghost)) for r in range(2)]
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
    full_states = _world_states(ref, 0, W, False)
    full_rew = _rewards_by_world(ref.species_count(), ref.column(po.COL_REWARD).ravel(), 0)
    for shard_states, shard_rew in states:
        for w, st in shard_states.items():
            for k in st:
                assert np.array_equal(st[k], full_states[w][k]), (w, k)
        for (w, s), r in shard_rew.items():
            if not reward_fixed and not ghost and s == 3 and w == W // 2 - 1:
                # no ghost: species 4 of the shard's last world reads past its
                # table (0 here, world 8's rewards[0] unsharded)
                assert r.shape == full_rew[(w, s)].shape
            else:
                assert np.array_equal(r.view(np.uint32), full_rew[(w, s)].view(np.uint32)), (w, s)

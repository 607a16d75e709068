"""CPU, world_size 2 and 8 over gloo: world sharding is exact.

Each rank holds worlds [r*W/N, (r+1)*W/N) with world_offset = r*W/N (the layout
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


def _worker(rank, port, q, reward_fixed, ghost, ws):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      MBOTS_CPU_THREADS="2" if ws <= 2 else "1")
    import madrona_bots as mb
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    per = W // ws
    # the last shard has no next shard: its last world reads past the table, as
    # one device's last world does (bench.py: shard_ghost=rank < world_size - 1)
    sim = mb.SimManager(0, per, 69, 32, exec_mode="cpu", world_offset=rank * per,
                        reward_fixed=reward_fixed, shard_ghost=ghost and rank < ws - 1)
    _run(sim)
    # bench.py's reductions: max time over ranks, sum of agent-steps
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([float(sim.num_agents())])
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    sc = sim.species_count_tensor().to_torch().numpy()
    rew = sim.reward_tensor(False).to_torch().numpy().ravel()
    states = [None] * ws
    dist.all_gather_object(states, (_world_states(sim, rank * per, per, True),
                                    _rewards_by_world(sc, rew, rank * per)))
    if rank == 0:
        q.put((float(t.item()), float(n.item()), states))
    dist.destroy_process_group()


@pytest.mark.parametrize("reward_fixed,ghost,ws", [(True, False, 2), (False, True, 2), (False, False, 2),
                                                   (False, True, 8)])
def test_shards_equal_one(reward_fixed, ghost, ws):
    """N shards (N = 2; and 8, the node the driver scales to: ranks of two
    worlds each, every shard but the last with its ghost) equal one oracle
    holding every world, and bench.py's max / sum reductions see every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, reward_fixed, ghost, ws)) for r in range(ws)]
    for p in procs:
        p.start()
    tmax, nsum, states = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(ws)
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
            if not reward_fixed and not ghost and s == 3 and (w + 1) % (W // ws) == 0 and w != W - 1:
                # no ghost: species 4 of the shard's last world reads past its
                # table (0 here, world 8's rewards[0] unsharded)
                assert r.shape == full_rew[(w, s)].shape
            else:
                assert np.array_equal(r.view(np.uint32), full_rew[(w, s)].view(np.uint32)), (w, s)

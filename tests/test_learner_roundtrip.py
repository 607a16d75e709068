"""The config-5 learner round trip (BASELINE config 5; SURVEY 8e steps 1-3;
learn/training_loop.py:36-137): after every step the learner's reads travel to
rank 0 as learner records (harness/gather.py gather_learner: current and
previous observation columns, reward, stats, Action, HiddenState,
PrevHiddenState), rank 0 chooses actions and memory from them, and
scatter_actions writes them back into the rows of the ranks that own them --
the shard ghosts' rows included, so the faithful B.3 reward (sim.cpp:943) of a
shard's last world stays one device's.

Checked bitwise every step against one manager holding every world that
receives the same actions through write_actions (the whole-table form of
training_loop.py:136-137's view writes): the gathered tensors == that
manager's own views (construct_obs, reward, stats, action, hidden state and
their previous forms), and therefore its next steps.
"""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "madrona-bots_amd", "harness")
SEED = 69


def _learner(got, t):
    """A deterministic stand-in for the PPO step (learn/models.py, out of
    scope): one-hot actions and new memory computed from what was gathered."""
    bits = got["obs"].view(torch.int32).to(torch.int64).sum(dim=1) + got["action"].to(torch.int64).sum(dim=1) * 7
    k = (bits + t) % 6
    actions = torch.nn.functional.one_hot(k, 6).to(torch.int32)
    memory = got["obs"][:, :16] * 0.25 + got["hidden"] * 0.5 - got["prev_hidden"] * 0.125
    return actions, memory


def _own_views(m):
    """What training_loop.py reads, straight from one manager's views."""
    return {"obs": m.construct_obs(False), "prev_obs": m.construct_obs(True),
            "reward": m.reward_tensor(False).to_torch().clone(),
            "stats": m.stats_tensor(False).to_torch().clone(),
            "action": m.action_tensor(False).to_torch().clone(),
            "hidden": m.hidden_state_tensor(False).to_torch().clone(),
            "prev_hidden": m.hidden_state_tensor(True).to_torch().clone()}


def _bitwise(a, b):
    if a.device != b.device:
        a, b = a.cpu(), b.cpu()
    return a.shape == b.shape and torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))


def _roundtrip_in_process(shards, full, steps, full_records=False, slim=False):
    """Shards and the full manager in one process: the gather / scatter data
    movement of harness/gather.py without the collectives (the reassembly and
    its inverse are the same functions).  full_records: the gathered tensors
    are also compared with the full manager's own learner records
    (pack_learner -> unpack_learner).  slim: from the second step on the shards
    ship slim records and Action / HiddenState / PrevHiddenState are rebuilt
    from the learner's own writes (gather.LearnerState)."""
    sys.path.insert(0, HARNESS)
    import gather
    import madrona_bots as mb
    bad = []
    state = gather.LearnerState() if slim else None
    for m in shards + [full]:
        m.write_synthetic_actions(1234, 0, True)
    for t in range(steps):
        for m in shards + [full]:
            m.step()
        counts = [m.species_count_tensor().to_torch() for m in shards]
        plan = {"counts": torch.stack([c.sum(dim=0).to(torch.int64).cpu() for c in counts]),
                "first": torch.stack([c[0].to(torch.int64).cpu() for c in counts])}
        use_slim = state is not None and state.ready
        recs = gather.reassemble([m.pack_learner(slim=use_slim) for m in shards], plan["counts"])
        if use_slim:
            assert recs.shape[1] == shards[0].learner_record_bytes(slim=True) in (128, 192)
            got = gather.rebuild(mb.unpack_learner(recs), plan["counts"], state)
            del got["src"]
        else:
            got = mb.unpack_learner(recs)
        if state is not None:
            state.note_gathered(got)
        ref = _own_views(full)
        bad += [f"step {t}: {k}" for k in ref if not _bitwise(got[k], ref[k])]
        if full_records:
            own = mb.unpack_learner(full.pack_learner())
            bad += [f"step {t}: {k} (records)" for k in own if not _bitwise(got[k], own[k])]
            del own
        del ref
        actions, memory = _learner(got, t)
        del got
        for m in shards + [full]:
            m.shift_observations()
        full.write_actions(actions, memory)
        both = torch.cat([actions, memory.view(torch.int32)], dim=1)
        for r, m in enumerate(shards):
            part = gather.split_rows(both, plan, r)
            assert part.shape[0] == m.num_rows()
            m.write_actions(part[:, :6].contiguous(), part[:, 6:].contiguous().view(torch.float32))
        if state is not None:
            state.commit(plan, actions, memory)
    if slim:
        assert state.ready
    return bad


@pytest.mark.parametrize("slim", [False, True])
@pytest.mark.parametrize("fix_depth", [False, True])
def test_learner_roundtrip_cpu_shards_equal_one(fix_depth, slim):
    """CPU mode: 2 shards x 6 worlds (faithful rewards through the ghost) ==
    one 12-world manager under learner-chosen actions and memory (slim: from
    provenance records from the second step on)."""
    import madrona_bots as mb
    W = 6
    kw = dict(exec_mode="cpu", fix_depth_alias=fix_depth)
    shards = [mb.SimManager(0, W, SEED, 32, world_offset=r * W, shard_ghost=r == 0, **kw) for r in range(2)]
    full = mb.SimManager(0, 2 * W, SEED, 32, **kw)
    assert _roundtrip_in_process(shards, full, 6, slim=slim) == []


def test_provenance_rows_map_old_rows_into_the_last_global_table():
    """gather.provenance_rows against a brute-force map: a rank's local old
    row -> its row in the last global (species, world, slot) table."""
    sys.path.insert(0, HARNESS)
    import gather
    g = torch.Generator().manual_seed(3)
    for R in (1, 2, 5):
        last = torch.randint(0, 6, (R, 4), generator=g)
        last[0, 1] = 0   # an empty species segment
        glob = {}
        for s in range(4):
            for r in range(R):
                a = int(last[r, :s].sum())
                for k in range(int(last[r, s])):
                    glob[(r, a + k)] = len(glob)
        cur = torch.randint(0, 6, (R, 4), generator=g)
        owner = gather.row_ranks(cur)
        src = []
        for i in range(owner.shape[0]):
            n = int(last[int(owner[i])].sum())
            new = n == 0 or int(torch.randint(0, 5, (1,), generator=g)) == 0
            src.append(-1 if new else int(torch.randint(0, n, (1,), generator=g)))
        src = torch.tensor(src, dtype=torch.int32)
        got = gather.provenance_rows(src, owner, last).tolist()
        assert got == [-1 if o < 0 else glob[(int(owner[i]), o)] for i, o in enumerate(src.tolist())]
        # the native rebuild (host path of mbots_rebuild_learner) takes the same rows
        import madrona_bots as mb
        m = int(last.sum())
        la = torch.randint(0, 9, (m, 6), generator=g, dtype=torch.int32)
        lm, lh = torch.randn((m, 16), generator=g), torch.randn((m, 16), generator=g)
        out = mb.rebuild_learner(src, cur, last, la, lm, lh)
        for key, t in (("action", la), ("hidden", lm), ("prev_hidden", lh)):
            want = torch.stack([t[x] if x >= 0 else torch.zeros_like(t[0]) for x in got]) if got else t[:0]
            assert torch.equal(out[key], want), key


def test_split_rows_inverts_reassemble():
    sys.path.insert(0, HARNESS)
    import gather
    cnt = torch.tensor([[3, 1, 0, 2], [2, 2, 1, 0], [1, 0, 4, 1]])
    first = torch.tensor([[1, 0, 0, 1], [1, 1, 0, 0], [0, 0, 2, 1]])
    n = int(cnt.sum())
    glob = torch.arange(n)
    plan = {"counts": cnt, "first": first}
    own = [gather.split_rows(glob, plan, r)[:int(cnt[r].sum())] for r in range(3)]
    assert torch.equal(gather.reassemble(own, cnt), glob)
    # rank 0's ghost rows are rank 1's first world: the first rows of each of
    # rank 1's species segments
    ghost = gather.split_rows(glob, plan, 0)[int(cnt[0].sum()):]
    tot = cnt.sum(dim=0)
    exp = [int(tot[:s].sum()) + int(cnt[0, s]) + k for s in range(4) for k in range(int(first[1, s]))]
    assert ghost.tolist() == exp
    assert gather.split_rows(glob, plan, 2).shape[0] == int(cnt[2].sum())


def _worker(rank, world, port, q, steps, slim=False):
    sys.path[:0] = [HARNESS, os.path.join(ROOT, "madrona-bots_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gather
        import madrona_bots as mb
        W = 5
        sim = mb.SimManager(0, W, SEED, 32, world_offset=rank * W, shard_ghost=rank < world - 1, exec_mode="cpu")
        full = mb.SimManager(0, world * W, SEED, 32, exec_mode="cpu") if rank == 0 else None
        for m in (sim, full):
            if m is not None:
                m.write_synthetic_actions(1234, 0, True)
        bad = []
        state = gather.LearnerState() if slim else None
        for t in range(steps):
            sim.step()
            got, plan = gather.gather_learner(sim, dst=0, state=state)
            if got is not None:
                got.pop("src", None)
            actions = memory = None
            if rank == 0:
                full.step()
                ref = _own_views(full)
                bad += [f"step {t}: {k}" for k in ref if not _bitwise(got[k], ref[k])]
                actions, memory = _learner(got, t)
                full.shift_observations()
                full.write_actions(actions, memory)
            sim.shift_observations()
            gather.scatter_actions(sim, actions, memory, plan, src=0, state=state)
        if rank == 0:
            q.put(bad)
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    return q.get(timeout=5)


@pytest.mark.parametrize("world,slim", [(2, False), (2, True), (3, False), (3, True), (8, True)])
def test_learner_roundtrip_gloo(world, slim):
    """gather_learner / scatter_actions over gloo with 2, 3 and 8 CPU-mode ranks:
    rank 0's gathered tensors equal one manager of every world, step after
    step, while the learner's actions drive both (slim: provenance records
    and the learner's rebuild from the second step on)."""
    assert _spawn(_worker, world, 5, slim) == []


@pytest.mark.gpu
@pytest.mark.parametrize("slim", [False, True])
@pytest.mark.parametrize("fix_depth", [False, True])
def test_learner_roundtrip_hip_shards_equal_one(fix_depth, slim):
    """HIP: 2 shards x 1024 worlds on the device (faithful rewards through the
    ghost) == one 2048-world manager under learner-chosen actions and memory,
    every gathered tensor bitwise, 8 steps."""
    import madrona_bots as mb
    W = 1024
    kw = dict(fix_depth_alias=fix_depth)
    shards = [mb.SimManager(0, W, SEED, 32, world_offset=r * W, shard_ghost=r == 0, **kw) for r in range(2)]
    full = mb.SimManager(0, 2 * W, SEED, 32, **kw)
    assert _roundtrip_in_process(shards, full, 8, slim=slim) == []


def _rccl_worker(rank, world, port, q):
    sys.path[:0] = [HARNESS, os.path.join(ROOT, "madrona-bots_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import gather
        import madrona_bots as mb
        sim = mb.SimManager(0, 512, SEED, 32)
        ref_m = mb.SimManager(0, 512, SEED, 32)
        for m in (sim, ref_m):
            m.write_synthetic_actions(1234, 0, True)
        bad = []
        for t in range(4):
            sim.step()
            ref_m.step()
            got, plan = gather.gather_learner(sim, dst=0)
            ref = _own_views(ref_m)
            bad += [f"step {t}: {k}" for k in ref if not _bitwise(got[k], ref[k])]
            actions, memory = _learner(got, t)
            sim.shift_observations()
            ref_m.shift_observations()
            gather.scatter_actions(sim, actions, memory, plan, src=0)
            ref_m.write_actions(actions, memory)
        torch.cuda.synchronize()
        q.put(bad)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_learner_roundtrip_over_rccl_one_rank():
    """The round trip's collectives (all_gather of the plan, gather of the
    learner records, scatter of actions + memory) executed by RCCL on the
    device at one rank: equal to a manager driven through write_actions."""
    assert _spawn(_rccl_worker, 1) == []


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("fix_depth,slim", [(False, False), (True, False), (False, True), (True, True)])
def test_config5_eight_shards_at_full_size(fix_depth, slim):
    """BASELINE config 5 at its own size: 262144 worlds as
    8 x 32768-world shards on one device (ranks 0..6 with their shard ghosts),
    against one 262144-world manager, 3 steps of the learner round trip of
    learn/training_loop.py:43-93, :136-137: every shard's pack_learner ->
    reassemble -> unpack_learner == the full manager's views and its own
    pack_learner -> unpack_learner, bitwise on every key; split_rows +
    write_actions drive the 8 shards with the learner's actions and memory
    exactly as write_actions drives the full manager.  (The RCCL transport
    between 8 GPUs is the driver's multi-GPU run.)"""
    import madrona_bots as mb
    R, WS = 8, 32768
    kw = dict(fix_depth_alias=fix_depth)
    shards = [mb.SimManager(0, WS, SEED, 32, world_offset=r * WS, shard_ghost=r < R - 1, **kw) for r in range(R)]
    full = mb.SimManager(0, R * WS, SEED, 32, **kw)
    assert _roundtrip_in_process(shards, full, 4 if slim else 3, full_records=True, slim=slim) == []
    assert sum(m.num_agents() for m in shards) == full.num_agents() > 8 * WS * 30

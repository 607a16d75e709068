"""Rollout gather to the learner rank and the learner's writes back
(BASELINE config 5).

Each rank steps its own world shard ([r*W, (r+1)*W), no collective on the
step) and exports species-major rows.  The learner (PPO, learn/train.py --
out of scope) runs on one rank; this moves the per-species row tensors it
consumes there:

  1. all_gather of the per-rank species row counts (4 x int64),
  2. one gather per tensor of the rows padded to the largest rank
     (torch.distributed.gather: RCCL send/recv over xGMI with the nccl
     backend -- each peer has a direct link to the learner -- gloo on CPU),
  3. on the learner rank, per species s the concatenation over ranks of
     rank r's species-s rows: the global (species, world, slot) order, i.e.
     exactly the table one device holding every world would export.

    out = gather_rollout({"obs": obs, "reward": rew}, species_rows, dst=0)

The full round trip the reference training loop makes after every step
(learn/training_loop.py:36-137):

    got, plan = gather_learner(mgr, dst=0)          # what :43-93 read
    if rank == 0: actions, memory = learner(got)    # [sum N_r, 6] / [sum N_r, 16]
    mgr.shift_observations()                        # :135
    scatter_actions(mgr, actions, memory, plan)     # :136-137, to the owning ranks

scatter_actions also sends every rank but the last the rows of its shard
ghost (the next rank's first world, SimManager(shard_ghost=True)), so the
ghost acts as that world does on its own rank and the faithful B.3 reward
(sim.cpp:943) of the shard's last world equals one device's under a learner.
"""
import torch
import torch.distributed as dist


def species_rows(counts):
    """Per-species row counts of this rank from species_count_tensor() [W, 4]."""
    return counts.sum(dim=0).to(torch.int64)


def reassemble(bufs, all_cnt):
    """Learner-side reassembly: bufs[r] holds rank r's species-major rows
    (padded), all_cnt [world, 4] the per-rank species row counts.  Returns the
    rows in global (species, world, slot) order: per species s, rank 0's
    species-s rows, then rank 1's, ... -- the table one device holding every
    world would export."""
    all_cnt = torch.as_tensor(all_cnt).cpu()
    parts = []
    for s in range(4):
        for r, b in enumerate(bufs):
            a = int(all_cnt[r, :s].sum())
            parts.append(b[a:a + int(all_cnt[r, s])])
    return torch.cat(parts)


def gather_records(mgr, dst=0, group=None):
    """Config 5 as SURVEY 8e sizes it: every rank packs its export rows'
    raw columns into fixed rollout records (SimManager.pack_rollout: 64 B per
    agent, 96 with real depth -- not the 276-B f32 learner rows), one padded
    gather ships them to the learner rank, which reassembles the global
    (species, world, slot) order and rebuilds the learner rows there with the
    construct_obs-equivalent kernel (madrona_bots.unpack_rollout).  Returns
    {"obs" [N, 69] f32, "reward" [N, 1] f32, "stats" [N, 4] i32} on `dst`,
    None elsewhere; N = the rows of every rank.
    (learn/training_loop.py:43-57, :87 -- the learner's reads after step())"""
    import madrona_bots as mb
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dst_global = dst if group is None else dist.get_global_rank(group, dst)
    dev = mgr.device
    # counts travel on the collective's device (RCCL: the GPU; gloo: host)
    cdev = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
    cnt = species_rows(mgr.species_count_tensor().to_torch()).to(cdev)
    all_cnt = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(all_cnt, cnt, group=group)
    all_cnt = torch.stack(all_cnt).cpu()
    n_max = int(all_cnt.sum(dim=1).max())
    rb = mgr.rollout_record_bytes()
    pad = torch.empty((max(n_max, 1), rb), dtype=torch.uint8, device=dev)   # rows past N: padding
    mgr.pack_rollout(pad)
    send = pad if cdev.type == dev.type else pad.to(cdev)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, bufs, dst=dst_global, group=group)
    if rank != dst:
        return None
    recs = reassemble([b[:n_max] for b in bufs], all_cnt)
    return mb.unpack_rollout(recs.to(dev))


def _counts_device(mgr, group):
    return mgr.device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def exchange_plan(mgr, group=None):
    """all_gather of every rank's per-species row counts and its first world's
    species counts (the rows of the previous rank's shard ghost): the plan the
    reassembly (gather) and its inverse (scatter_actions) follow."""
    world = dist.get_world_size(group)
    counts = mgr.species_count_tensor().to_torch()
    cdev = _counts_device(mgr, group)
    mine = torch.cat([counts.sum(dim=0).to(torch.int64), counts[0].to(torch.int64)]).to(cdev)
    allc = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allc, mine, group=group)
    allc = torch.stack(allc).cpu()
    return {"counts": allc[:, :4], "first": allc[:, 4:]}


def gather_learner(mgr, dst=0, group=None, keys=None, state=None):
    """Config 5, learner side of the step: every rank packs its export rows'
    learner records (SimManager.pack_learner: current and previous observation
    columns, reward, stats, Action, HiddenState, PrevHiddenState -- what
    learn/training_loop.py:43-93 reads), one padded gather ships them to `dst`,
    which reassembles the global (species, world, slot) order and unpacks them
    (madrona_bots.unpack_learner).  Returns (tensors on `dst` / None elsewhere,
    plan) -- the plan is scatter_actions' argument.  With a ready
    LearnerState the ranks ship slim records (128 B instead of 272) and `dst`
    rebuilds Action / HiddenState / PrevHiddenState from its own last writes."""
    import madrona_bots as mb
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dst_global = dst if group is None else dist.get_global_rank(group, dst)
    dev = mgr.device
    cdev = _counts_device(mgr, group)
    plan = exchange_plan(mgr, group)
    all_cnt = plan["counts"]
    n_max = int(all_cnt.sum(dim=1).max())
    slim = state is not None and state.ready
    rb = mgr.learner_record_bytes(slim)
    pad = torch.empty((max(n_max, 1), rb), dtype=torch.uint8, device=dev)   # rows past N: padding
    mgr.pack_learner(pad, slim=slim)
    send = pad if cdev.type == dev.type else pad.to(cdev)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, bufs, dst=dst_global, group=group)
    if rank != dst:
        return None, plan
    recs = reassemble([b[:n_max] for b in bufs], all_cnt)
    if slim:
        got = rebuild(mb.unpack_learner(recs.to(dev)), all_cnt, state)
    else:   # (the state keeps this step's HiddenState: every key then)
        kw = {} if keys is None or state is not None else {"keys": keys}
        got = mb.unpack_learner(recs.to(dev), **kw)
    if state is not None:
        state.note_gathered(got)
    if keys is not None:
        got = {k: got[k] for k in keys}
    return got, plan


class LearnerState:
    """What the learner rank remembers of its own writes, so the ranks can
    ship slim learner records (include/mbots.h MBOTS_LEARNER_SLIM_BYTES: no
    Action, HiddenState, PrevHiddenState -- 152 of the 272 B per agent -- but
    each row's provenance src, its index in the table before the step).  After
    step t the manager's columns are the learner's own values moved by the
    species sort (learn/training_loop.py:136-137 wrote them after step t-1;
    the shift copied HiddenState into PrevHiddenState first):

        Action(t)[r]          = A_{t-1}[src[r]]
        HiddenState(t)[r]     = M_{t-1}[src[r]]
        PrevHiddenState(t)[r] = HiddenState(t-1)[src[r]]     (0 for src = -1)

    with A_{t-1} / M_{t-1} the actions and memory scattered after step t-1 and
    src mapped from the owning rank's old rows into the last global table
    (that step's plan).  Valid while every row's action and memory are written
    after every step, after its shift(s) (scatter_actions does; a shift
    between per-species writes, SURVEY B.9, breaks it) -- after any other write, a
    checkpoint load or a new manager, call reset() on every rank: the next
    gather then ships full records again.  Every rank holds one (they agree on
    the record width); only the learner rank holds tensors.  The learner must
    not modify the actions / memory it passed to scatter_actions in place."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.ready = False
        self.counts = None            # [ranks, 4] per-rank species rows of the last table
        self.action = self.memory = self.hidden = None   # its rows, global order
        self._hidden_now = None       # HiddenState of the table being learned on

    def note_gathered(self, got):
        if got is not None:
            self._hidden_now = got["hidden"]

    def commit(self, plan, actions, memory):
        """After the learner's writes went out (every rank)."""
        if actions is not None:
            self.counts = plan["counts"].clone()
            self.action, self.memory, self.hidden = actions, memory, self._hidden_now
        self._hidden_now = None
        self.ready = True


def row_ranks(counts):
    """The owning rank of every row of the global (species, world, slot) order
    reassemble() builds from per-rank species counts [ranks, 4]."""
    ranks = counts.shape[0]
    ids = torch.arange(ranks).repeat(4)
    return torch.repeat_interleave(ids, counts.t().reshape(-1).to(torch.int64))


def provenance_rows(src, owner, last_counts):
    """Global row of each row's old row in the last table: src [N] int32 (the
    owning rank's local old row, -1 new), owner [N] its rank, last_counts
    [ranks, 4] the last table's per-rank species rows.  Returns int64 [N]
    (-1 for new rows)."""
    dev = src.device
    lc = last_counts.to(device=dev, dtype=torch.int64)
    lstart = torch.cumsum(lc, dim=1) - lc                       # [R, 4] local species starts
    tot = lc.sum(dim=0)
    gstart = (torch.cumsum(tot, 0) - tot)[None, :] + (torch.cumsum(lc, dim=0) - lc)   # [R, 4]
    o = src.to(torch.int64)
    valid = o >= 0
    oc = o.clamp(min=0)
    ls = lstart[owner.to(dev)]                                  # [N, 4]
    sp = ((oc[:, None] >= ls).sum(dim=1) - 1).clamp(min=0)      # the old row's species segment
    g = gstart[owner.to(dev), sp] + oc - ls.gather(1, sp[:, None]).squeeze(1)
    return torch.where(valid, g, torch.full_like(g, -1))


def rebuild(got, cur_counts, state):
    """Slim records: Action / HiddenState / PrevHiddenState of every gathered
    row from the learner's own last writes (LearnerState), bit-identical to
    the manager's columns -- one native pass (madrona_bots.rebuild_learner:
    the provenance_rows map and the three gathers)."""
    import madrona_bots as mb
    got.update(mb.rebuild_learner(got["src"], cur_counts, state.counts, state.action, state.memory, state.hidden))
    return got


def gather_learner_local(mgr, state=None):
    """gather_learner for one rank without torch.distributed: the same records
    packed and unpacked locally (slim ones once `state` is ready)."""
    import madrona_bots as mb
    counts = mgr.species_count_tensor().to_torch()
    plan = {"counts": counts.sum(dim=0).to(torch.int64).cpu()[None], "first": counts[0].to(torch.int64).cpu()[None]}
    slim = state is not None and state.ready
    got = mb.unpack_learner(mgr.pack_learner(slim=slim))
    if slim:
        got = rebuild(got, plan["counts"], state)
    if state is not None:
        state.note_gathered(got)
    return got, plan


def split_rows(glob, plan, r):
    """Inverse of reassemble for rank r: its own rows (species-major) and then
    its shard ghost's (r < ranks - 1: the next rank's first world, species by
    species) out of the global (species, world, slot) order."""
    cnt, first = plan["counts"], plan["first"]
    ranks = cnt.shape[0]
    tot = cnt.sum(dim=0)
    parts = []

    def seg(s, q, n):
        off = int(tot[:s].sum()) + int(cnt[:q, s].sum())
        parts.append(glob[off:off + n])
    for s in range(4):
        seg(s, r, int(cnt[r, s]))
    if r < ranks - 1:
        for s in range(4):
            seg(s, r + 1, int(first[r + 1, s]))
    return torch.cat(parts)


def scatter_actions(mgr, actions, memory, plan, src=0, group=None, state=None):
    """The learner's writes (training_loop.py:136-137) sent to the ranks that
    own the rows: on `src`, int32 [sum N_r, 6] actions and
    float32 [sum N_r, 16] memory in the global order gather_learner produced;
    every rank receives its rows (plus its shard ghost's) in one padded
    scatter and writes them with SimManager.write_actions.  `state`: the
    LearnerState the next gather_learner rebuilds from (every rank)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    src_global = src if group is None else dist.get_global_rank(group, src)
    dev = mgr.device
    cdev = _counts_device(mgr, group)
    cnt, first = plan["counts"], plan["first"]
    rows = [int(cnt[r].sum()) + (int(first[r + 1].sum()) if r < world - 1 else 0) for r in range(world)]
    r_max = max(max(rows), 1)
    recv = torch.empty((r_max, 22), dtype=torch.int32, device=cdev)
    chunks = None
    if rank == src:
        both = torch.cat([actions.to(torch.int32), memory.to(torch.float32).view(torch.int32)], dim=1).to(cdev)
        chunks = []
        for r in range(world):
            part = split_rows(both, plan, r)
            buf = torch.zeros((r_max, 22), dtype=torch.int32, device=cdev)
            buf[:part.shape[0]] = part
            chunks.append(buf)
    dist.scatter(recv, chunks, src=src_global, group=group)
    mine = recv[:rows[rank]].to(dev)
    if mine.shape[0] != mgr.num_rows():
        raise RuntimeError(f"rank {rank}: {mine.shape[0]} rows received, the table holds {mgr.num_rows()} "
                           "(is shard_ghost set on every rank but the last?)")
    mgr.write_actions(mine[:, :6].contiguous(), mine[:, 6:].contiguous().view(torch.float32))
    if state is not None:
        state.commit(plan, actions if rank == src else None, memory if rank == src else None)


def gather_rollout(tensors, rows_per_species, dst=0, group=None):
    """tensors: name -> [N_r, ...] species-major rows of this rank (same N_r);
    rows_per_species: int64 [4] summing to N_r.  Returns name -> [sum N_r, ...]
    in global species-major order on rank dst, None elsewhere.  `dst` is a
    rank within `group` (the default group: the global rank)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    # torch.distributed.gather takes a global rank
    dst_global = dst if group is None else dist.get_global_rank(group, dst)
    dev = next(iter(tensors.values())).device
    cnt = rows_per_species.to(device=dev, dtype=torch.int64).reshape(4)
    all_cnt = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(all_cnt, cnt, group=group)
    all_cnt = torch.stack(all_cnt).cpu()              # [world, 4]
    totals = all_cnt.sum(dim=1)
    n_max = int(totals.max())
    out = {} if rank == dst else None
    for name, t in tensors.items():
        n = int(totals[rank])
        if t.shape[0] != n:
            raise ValueError(f"{name}: {t.shape[0]} rows, species counts sum to {n}")
        pad = torch.zeros((n_max,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        pad[:n] = t
        bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
        dist.gather(pad, bufs, dst=dst_global, group=group)
        if rank == dst:
            out[name] = reassemble(bufs, all_cnt)
    return out

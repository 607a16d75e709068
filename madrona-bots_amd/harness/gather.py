"""Rollout gather to the learner rank (BASELINE config 5).

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

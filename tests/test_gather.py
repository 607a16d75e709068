"""Rollout gather to the learner rank (harness/gather.py, BASELINE config 5)
over gloo with 2 CPU ranks: rank r steps worlds [r*W, (r+1)*W) through the
oracle adapter; the gathered observation / action / health rows on rank 0 must
equal the single-process table of all 2W worlds (global species-major order).
Rewards are excluded: the faithful B.3 reward of species 4 in a shard's last
world reads 0 per shard."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "madrona-bots_amd", "harness")
W, STEPS, SEED = 6, 4, 69


def _rows(sim):
    import rollout
    obs = torch.cat([rollout.construct_obs(sim, s, e) for s, e in rollout.species_offsets(sim)])
    return {"obs": obs, "action": sim.action_tensor(False).to_torch().clone(),
            "health": sim.health_tensor(False).to_torch().clone()}


def _run(sim, steps):
    for t in range(steps):
        sim._s.write_synthetic_actions(1234, t)
        sim.step()
        sim.shift_observations()


def _worker(rank, world, port, q):
    sys.path[:0] = [HARNESS, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle_adapter import OracleSimManager
        import gather
        sim = OracleSimManager(0, W, SEED, 32, world_offset=rank * W)
        _run(sim, STEPS)
        rows = _rows(sim)
        cnt = gather.species_rows(sim.species_count_tensor().to_torch())
        out = gather.gather_rollout(rows, cnt, dst=0)
        if rank == 0:
            full = OracleSimManager(0, world * W, SEED, 32)
            _run(full, STEPS)
            ref = _rows(full)
            ok = {k: torch.equal(out[k].view(torch.int32), ref[k].contiguous().view(torch.int32))
                  for k in ref}
            q.put(ok)
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


def test_gather_two_shards_equals_one():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    ok = q.get(timeout=5)
    assert all(ok.values()), ok


def _records_worker(rank, world, port, q, fix_depth):
    sys.path[:0] = [HARNESS, os.path.join(ROOT, "madrona-bots_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gather
        import madrona_bots as mb
        kw = dict(exec_mode="cpu", fix_depth_alias=fix_depth)

        def run(m):
            for t in range(STEPS):
                m.write_synthetic_actions(1234, t, True)
                m.step()
                if t < STEPS - 1:
                    m.shift_observations()

        # faithful B.3 rewards: every shard but the last steps the shard ghost
        sim = mb.SimManager(0, W, SEED, 32, world_offset=rank * W, shard_ghost=rank < world - 1, **kw)
        run(sim)
        out = gather.gather_records(sim, dst=0)
        if rank == 0:
            full = mb.SimManager(0, world * W, SEED, 32, **kw)
            run(full)
            ref = {"obs": full.construct_obs(False), "reward": full.reward_tensor(False).to_torch(),
                   "stats": full.stats_tensor(False).to_torch()}
            q.put({k: torch.equal(out[k].view(torch.int32), ref[k].contiguous().view(torch.int32))
                   for k in ref})
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fix_depth", [False, True])
def test_gather_records_two_cpu_shards_equal_one(fix_depth):
    """Config 5 as SURVEY 8e sizes it: 64-B (96-B with real depth) rollout
    records from two CPU-mode shards gathered over gloo, the [N, 69] learner
    rows rebuilt on rank 0 == one manager's construct_obs bitwise, with its
    rewards (faithful B.3 through the shard ghost) and stats."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_records_worker, args=(r, 2, port, q, fix_depth)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    ok = q.get(timeout=5)
    assert all(ok.values()), ok


def _rccl_worker(port, q):
    sys.path[:0] = [HARNESS, os.path.join(ROOT, "madrona-bots_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import gather
        import madrona_bots as mb
        sim = mb.SimManager(0, 512, SEED, 32)
        for t in range(STEPS):
            sim.write_synthetic_actions(1234, t, True)
            sim.step()
            if t < STEPS - 1:
                sim.shift_observations()
        out = gather.gather_records(sim, dst=0)
        ref = {"obs": sim.construct_obs(False), "reward": sim.reward_tensor(False).to_torch(),
               "stats": sim.stats_tensor(False).to_torch()}
        torch.cuda.synchronize()
        q.put({k: bool(torch.equal(out[k].view(torch.int32).cpu(), ref[k].contiguous().view(torch.int32).cpu()))
               for k in ref})
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gather_records_over_rccl_one_rank():
    """The config-5 gather's collectives (all_gather of the species counts,
    gather of the packed records) executed by RCCL (the nccl backend) on the
    device, one rank: the rows rebuilt from the gathered records equal the
    manager's own construct_obs / reward / stats bitwise.  (Several ranks need
    several GPUs: the driver's multi-GPU bench runs that; tests/test_gather's
    gloo cases cover the reassembly across shards.)"""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0
    ok = q.get(timeout=5)
    assert all(ok.values()), ok

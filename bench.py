#!/usr/bin/env python3
"""bench.py -- agent-steps/s of the MI355X madrona-bots world step.

One "step" = Manager::step() (Step + Sensor graphs, sim.cpp:1061-1188) +
shift_observations() (sim.cpp:1190-1220) + writing the next one-hot actions
for every live agent (the learner's write, learn/env.py:94-98), on synthetic
identity-keyed actions.  Worlds are sharded across ranks with
no collective on the step (weak scaling: `--worlds` per GPU, default 65536 =
BASELINE config 3).  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--worlds WPG]
    torchrun --nproc-per-node N bench.py --gpus N ...

With several ranks (or --gather) a second timed loop measures BASELINE config
5: after every step each rank's learner records (what the reference training
loop reads, 272 B/agent) are gathered to rank 0 over RCCL and unpacked there,
rank 0 picks actions and memory, and they are scattered back to the ranks that
own the rows (madrona-bots_amd/harness/gather.py); reported as "config5".
`python bench.py --gpus N` without a launcher starts the N ranks itself.

After the main line (unless --no-secondary): "steady_state", the same loop
from step 250 on, once the worlds' food has reached its cap (the per-step cost
rises with the food count over the first ~250 steps, so the early window of a
short run is not the long-run rate: profiles/r05_drivergap.json); "config2",
the same loop at 4096 worlds/GPU; "config4", BASELINE config 4's 262144 worlds
sharded over the N ranks (strong scaling); and the reference training loop's
call sequence (learn/training_loop.py:36-137 without the learner math: step,
the action / memory views, reward and health clones, construct_obs of the
current and previous rows, PrevHiddenState, shift, the learner's one-hot
actions and memory written back) at 4096 worlds/GPU -- BASELINE config 2,
"random-action rollout, obs/reward tensors on-device", reported as
"secondary" -- and at the main line's size ("reference_loop"), each with its
own HBM roofline.
"""
import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd", "harness"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles
# per SIMD (32 lanes/cycle, MI355X_MICROARCH.md), 2.4 GHz
VALU_PEAK_INSTR_S = 1024 * 2.4e9 / 2
SEED = 69                   # learn/env.py:15
ACTION_SEED = 1234
AGENTS_PER_WORLD = 32       # learn/env.py:15
CONFIG4_WORLDS = 262144     # BASELINE config 4 (sharded across 8 GPUs)
CONFIG5_WORLDS = 262144     # BASELINE config 5 (the learner round trip over 8 GPUs)
STEADY_FROM, STEADY_STEPS = 250, 100   # the steady-state line: food at its cap


def algorithmic_bytes(n_agents, n_worlds):
    """B_step = 552 N + 1952 W bytes per step (step + shift)."""
    return 552.0 * n_agents + 1952.0 * n_worlds


# B_step counts 88 B per agent the lazy shift never moves when nothing reads
# the table between step() and shift_observations() (the 44 B of previous-obs
# reads and the 44 B of Prev{Species,Position,Health,Surrounding,Reward,Stats}
# writes, DESIGN.md "Lazy shift"), and the 64 B of the prev-sensor move (32
# read + 32 written), which a step owes until a reader needs it and which
# dies at the next step (DESIGN.md "Lazy prev sensor", round 6): the bytes
# the bench loop must move
LAZY_BYTES_PER_AGENT = 552.0 - 88.0 - 64.0
# the reference loop on top of B_step: construct_obs of the current and the
# previous rows (84 B read + 276 B written each), the reward / health clones
# (4 + 4 B each way), the learner's one-hot action + memory write (24 + 64 B)
LOOP_EXTRA_PER_AGENT = 2 * (84.0 + 276.0) + 16.0 + 88.0


def cgroup_cpu_quota():
    """CPUs of CPU time the process's cgroup grants per second (cgroup v2
    cpu.max, or v1 cfs quota / period), or None when unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def cpu_share():
    """(effective CPUs, affinity CPUs, cgroup quota, machine CPUs): the
    effective count is the affinity set capped by the cgroup's CPU quota --
    what the process can actually run on at once (the affinity
    mask alone overstated it)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    eff = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return eff, aff, quota, os.cpu_count()


def load_traffic(worlds):
    """HBM bytes per step from the committed rocprofv3 PMC summary
    (profiles/*_traffic.json, scripts/traffic.py: 2 x FETCH_SIZE + WRITE_SIZE per
    MI355X_MICROARCH.md 'HBM'), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("worlds") == worlds:
            best = (os.path.relpath(f, ROOT), d)
    return best


def load_kernel_stats():
    """Average duration (ms) per kernel from the committed rocprofv3 --stats
    summary (profiles/*_kernel_stats.csv, the latest), or {}."""
    import csv
    import glob
    import re
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats.csv"))
                   if re.fullmatch(r"r\d+_kernel_stats\.csv", os.path.basename(f)))
    if not files:
        return {}, None
    out = {}
    with open(files[-1]) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"<.*>", "", r["Name"].split("(")[0]).split()[-1].replace("mbots::", "")
            out[name] = float(r["AverageNs"]) * 1e-6
    return out, os.path.relpath(files[-1], ROOT)


def measured_valu_peak():
    """The VALU issue rate measured on MI355X by scripts/ubench/valu_rate.hip
    (profiles/*_valu_rate.json, the latest), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu_rate.json")))
    if not files:
        return None
    try:
        return os.path.relpath(files[-1], ROOT), json.load(open(files[-1]))["measured_peak_wave_instr_per_s"]
    except (OSError, ValueError, KeyError):
        return None


def load_profile(suffix, worlds):
    """profiles/*_<suffix>.json recorded at `worlds` (the latest), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{suffix}.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("worlds") == worlds:
            best = (os.path.relpath(f, ROOT), d)
    return best


def cpu_baseline(worlds_sample, target_s, threads=None):
    """The build's C++ CPU restatement (SURVEY 8d "CPU baseline"): the
    product's own CPU execution mode (madrona_bots exec_mode="cpu",
    mbots_cpu.cpp: the same systems, bit-identical to the HIP path), worlds
    split over `threads` host threads (default: every CPU in this process's
    affinity set), on a bounded sample of the same workload (same seed,
    agents, action stream, step+shift+write)."""
    import madrona_bots as mb
    eff, aff, quota, nproc = cpu_share()
    if threads is None:
        threads = eff
    os.environ["MBOTS_CPU_THREADS"] = str(threads)
    sim = mb.SimManager(0, worlds_sample, SEED, AGENTS_PER_WORLD, exec_mode="cpu")
    sim.write_synthetic_actions(ACTION_SEED, 0)
    sim.step()
    sim.shift_observations()
    s0, steps = sim.agent_steps(), 0
    t0 = time.perf_counter()
    while True:
        sim.write_synthetic_actions(ACTION_SEED, steps + 1)
        sim.step()
        sim.shift_observations()
        steps += 1
        dt = time.perf_counter() - t0
        if dt >= target_s or steps >= 5000:
            break
    return {"value": (sim.agent_steps() - s0) / dt, "unit": "agent-steps/s", "cores": threads,
            "nproc": nproc, "affinity_cpus": aff, "cgroup_cpu_quota": quota, "kind": "port",
            "impl": "madrona_bots exec_mode='cpu' (madrona-bots_amd/csrc/mbots_cpu.cpp), "
                    "std::thread per world range",
            "sample": f"{worlds_sample} worlds x {AGENTS_PER_WORLD} agents, {steps} steps "
                      f"(step+shift+actions), {threads} threads, {dt:.1f} s"}


def reference_loop(W, args, rank, world_size, dev, distributed, label):
    """learn/training_loop.py:36-137 without the learner math (out of scope),
    one rank's shard of W worlds; returns the line's dict."""
    import madrona_bots as mb
    m = mb.SimManager(dev.index, W, SEED, AGENTS_PER_WORLD, world_offset=rank * W,
                      shard_ghost=rank < world_size - 1)

    def one(t):
        m.step()                                             # :36
        ends = m.species_count_tensor().to_torch().sum(dim=0).cumsum(dim=0)   # :42-44
        m.action_tensor(False).to_torch()                    # :47-48, views before the shift
        m.hidden_state_tensor(False).to_torch()
        rew = m.reward_tensor(False).to_torch().clone()      # :49-50
        hp = m.health_tensor(False).to_torch().clone()
        # util.construct_obs of the previous rows (:86) issued before the current
        # rows' (:58-70): it needs no sensor rows, so it runs beside the sensor
        # instead of queueing behind the current rows' wait for it
        prev = m.construct_obs(True)
        obs = m.construct_obs(False)                         # every species at once
        ph = m.hidden_state_tensor(True).to_torch()          # :88
        m.shift_observations()                               # :135
        m.write_synthetic_actions(ACTION_SEED, t + 1, True)  # :136-137 actions + memory
        return ends, rew, hp, obs, prev, ph

    # a small-world step is ~0.14 ms and host-latency-bound: time at least
    # 400 steps so a host hiccup does not move the line (100 steps: +-40 %)
    steps = args.steps if W > 8192 else max(args.steps, 400)
    m.write_synthetic_actions(ACTION_SEED, 0, True)
    for t in range(args.warmup):
        one(t)
    torch.cuda.synchronize()
    s0 = m.agent_steps()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + steps):
        one(t)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n_local = m.agent_steps() - s0
    st = torch.tensor([el, float(n_local)], dtype=torch.float64,
                      device=dev if args.backend == "nccl" else "cpu")
    if distributed:
        dist.barrier()
        tm = st[0:1].clone(); dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        tot = st[1:2].clone(); dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        el, total = float(tm.item()), float(tot.item())
    else:
        total = float(st[1].item())
    ktimes = {}
    if not args.no_kernel_timing:
        m.enable_kernel_timing(True)
        t = args.warmup + steps
        for k in range(min(steps, 30)):
            one(t + k)
        torch.cuda.synchronize()
        ktimes = {k: round(ms / n, 5) for k, (ms, n) in m.kernel_times().items() if n}
        m.enable_kernel_timing(False)
    del m
    n_mean = n_local / steps
    ms = el / steps * 1e3
    nb = algorithmic_bytes(n_mean, W) + LOOP_EXTRA_PER_AGENT * n_mean
    gbs = nb / (ms * 1e-3) / 1e9
    return {"worlds_per_gpu": W, "value": total / el, "unit": "agent-steps/s",
            "ms_per_step": ms, "steps": steps, "n_gpus": world_size, "what": label,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_step": nb,
                         "bytes": "552 N + 1952 W (SURVEY 8d) + 824 N: construct_obs cur/prev "
                                  "(84 B read + 276 B written each), reward/health clones, "
                                  "the learner's action + memory write",
                         "timing": "wall clock of the timed steps (host-synchronising accessors "
                                   "included, as in the reference loop)"},
            "kernel_ms": ktimes}


def bare_loop(W, args, rank, world_size, dev, distributed, label):
    """The headline's loop -- step(), shift_observations(), the next one-hot
    actions -- on a shard of W worlds per rank (BASELINE config 2 at W = 4096:
    the metric's other half measured on the headline's workload); wall clock of
    the timed steps, max over ranks; its own HBM roofline (B_step / step time)."""
    import madrona_bots as mb
    m = mb.SimManager(dev.index, W, SEED, AGENTS_PER_WORLD, world_offset=rank * W,
                      shard_ghost=rank < world_size - 1)
    # short steps: time at least 400 so a host hiccup does not move the line
    steps = max(args.steps, 400)
    m.write_synthetic_actions(ACTION_SEED, 0)
    for t in range(args.warmup):
        m.step(); m.shift_observations(); m.write_synthetic_actions(ACTION_SEED, t + 1)
    torch.cuda.synchronize()
    s0 = m.agent_steps()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + steps):
        m.step(); m.shift_observations(); m.write_synthetic_actions(ACTION_SEED, t + 1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n_local = m.agent_steps() - s0
    st = torch.tensor([el, float(n_local)], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    if distributed:
        dist.barrier()
        tm = st[0:1].clone(); dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        tot = st[1:2].clone(); dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        el, total = float(tm.item()), float(tot.item())
    else:
        total = float(st[1].item())
    del m
    n_mean = n_local / steps
    ms = el / steps * 1e3
    nb = algorithmic_bytes(n_mean, W)
    gbs = nb / (ms * 1e-3) / 1e9
    return {"worlds_per_gpu": W, "value": total / el, "unit": "agent-steps/s", "ms_per_step": ms,
            "steps": steps, "n_gpus": world_size, "what": label, "mean_agents_per_world": n_mean / W,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_step": nb,
                         "bytes": "552 N + 1952 W (SURVEY 8d)",
                         "timing": "wall clock of the timed steps (step + shift + action write)"}}


def spawn_ranks(args):
    """One rank per GPU for `--gpus N` when no launcher set WORLD_SIZE: this
    GPU-free parent runs torch.distributed.run as a child process (never an
    exec: the children initialise the GPUs) on 127.0.0.1 and returns its exit
    code.  Each rank then takes cuda:LOCAL_RANK (distinct devices unless
    --same-device)."""
    import socket
    import subprocess
    # no GPU call here (not even a device count, which can fall back to
    # hipGetDeviceCount): each rank checks that it has a device of its own
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL over dmabuf IPC on this host
    return subprocess.run(cmd, env=env).returncode


def config5_loop(main_mgr, args, rank, world_size, dev, distributed):
    """BASELINE config 5: every rank steps its shard; after each step what the
    learner reads (learn/training_loop.py:43-93: current and previous
    observation columns, reward, stats, Action, HiddenState, PrevHiddenState)
    travels to rank 0 as learner records (harness/gather.py gather_learner:
    RCCL gather over xGMI with the nccl backend) and is unpacked there; rank 0
    picks actions and memory (a stand-in for the PPO step, learn/models.py,
    out of scope: random one-hot actions, memory from the gathered hidden
    state); shift; the actions and memory go back to the ranks that own the
    rows (scatter_actions, :136-137).  Wall clock of the timed steps, max over
    ranks; returns the line's dict on rank 0.  Its own shards: BASELINE config
    5's 262144 worlds in all, 262144 / N per rank (the main line's manager when
    N does not divide it)."""
    import gather
    import madrona_bots as mb
    if CONFIG5_WORLDS % world_size == 0:
        W5 = CONFIG5_WORLDS // world_size
        mgr = mb.SimManager(dev.index, W5, SEED, AGENTS_PER_WORLD, world_offset=rank * W5,
                            shard_ghost=rank < world_size - 1)
    else:
        mgr, W5 = main_mgr, main_mgr.num_worlds
    steps = max(10, args.steps // 2)
    gsec = [0.0, 0.0]
    nrows = [0]
    gen = torch.Generator(device=dev).manual_seed(ACTION_SEED)
    # slim learner records (128 B/agent instead of 272) from the second step
    # on: rank 0 rebuilds Action / HiddenState / PrevHiddenState from its own
    # last writes and the rows' provenance (harness/gather.py LearnerState)
    state = None if args.full_records else gather.LearnerState()

    def one(t, timed):
        mgr.step()
        g0 = time.perf_counter()
        if distributed:
            got, plan = gather.gather_learner(mgr, dst=0, state=state)
        else:   # one rank: the same records, packed and unpacked locally
            got, plan = gather.gather_learner_local(mgr, state)
        actions = memory = None
        if got is not None:
            n = got["obs"].shape[0]
            nrows[0] += n if timed else 0
            k = torch.randint(0, 6, (n,), device=dev, generator=gen)
            actions = torch.nn.functional.one_hot(k, 6).to(torch.int32)
            memory = got["hidden"] * 0.5 + got["obs"][:, :16] * (1.0 / 256.0)
        g1 = time.perf_counter()
        mgr.shift_observations()
        if distributed:
            gather.scatter_actions(mgr, actions, memory, plan, src=0, state=state)
        else:
            mgr.write_actions(actions, memory)
            if state is not None:
                state.commit(plan, actions, memory)
        if timed:
            gsec[0] += g1 - g0
            gsec[1] += time.perf_counter() - g1

    t0s = args.warmup + args.steps + 100
    mgr.write_synthetic_actions(ACTION_SEED, t0s, True)
    for k in range(3):
        one(t0s + k, False)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        one(t0s + 3 + k, True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = torch.tensor([el, gsec[0], gsec[1]], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    if distributed:
        dist.barrier()
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
    el, gs, ss = (float(x) for x in st.tolist())
    slim = state is not None and state.ready
    rb = mgr.learner_record_bytes(slim)
    # the learner rank's record work alone (untimed above: it overlaps the
    # step there): pack + unpack (+ the rebuild from provenance) of one step's
    # records on an idle device, priced at the bytes it must move per agent --
    # pack reads the columns and writes the record (2 rb), unpack reads it (rb)
    # and writes obs + prev_obs (2 x 276) + reward 4 + stats 16 (+ src 4); the
    # rebuild gathers Action / HiddenState / PrevHiddenState (152 B read +
    # written) -- and the xGMI payload per peer (every rank ships its records
    # to rank 0 and receives 88 B of actions + memory per row)
    rt = None
    if not distributed:
        mgr.step()
        torch.cuda.synchronize()
        r0 = time.perf_counter()
        for _ in range(3):
            got, _ = gather.gather_learner_local(mgr, state)
            del got
        torch.cuda.synchronize()
        rt_ms = (time.perf_counter() - r0) / 3 * 1e3
        n_rt = mgr.num_agents()
        per = 3 * rb + 2 * 276 + 20 + (4 + 2 * 152 if slim else 0)
        rt = {"ms": rt_ms, "rows": n_rt, "bytes_per_agent": per,
              "achieved": n_rt * per / (rt_ms * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
              "frac": n_rt * per / (rt_ms * 1e-3) / 8e12,
              "note": "pack + unpack (+ provenance rebuild) of one step's records on an idle device, host "
                      "launch time included; bytes: 2 rb pack, rb + 572 (+ 4 src) unpack, 2 x 152 rebuild"}
    rows_rank = mgr.num_agents()
    del mgr
    if rank != 0:
        return None
    rows = nrows[0] / steps
    return {"what": "step + what the learner reads (current and previous observation columns, reward, stats, "
                    f"Action, HiddenState, PrevHiddenState; records of {rb} B/agent) gathered to rank 0 and "
                    "unpacked there + actions / memory chosen there + shift + actions / memory scattered back to "
                    "the owning ranks (harness/gather.py gather_learner / scatter_actions)",
            "backend": args.backend if distributed else "none (one rank: pack + unpack + write locally)",
            "n_gpus": world_size, "worlds_per_gpu": W5, "total_worlds": W5 * world_size,
            "steps": steps, "ms_per_step": el / steps * 1e3,
            "value": rows / (el / steps), "unit": "agent-steps/s (every rank's agents through the learner round trip)",
            "gather_ms_per_step": gs / steps * 1e3, "scatter_ms_per_step": ss / steps * 1e3,
            "rows_per_step_at_learner": rows,
            "gathered_bytes_per_step": rows * rb, "scattered_bytes_per_step": rows * 88, "bytes_per_agent": rb,
            "records": "slim: provenance, Action / HiddenState / PrevHiddenState rebuilt on rank 0" if slim
                       else "full learner records",
            "xgmi_bytes_per_step_per_peer": (rows_rank * rb + rows_rank * 88) if world_size > 1 else 0,
            "roundtrip_roofline": rt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--worlds", type=int, default=65536, help="worlds per GPU")
    ap.add_argument("--cpu-worlds", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the untimed per-kernel event pass after the timed region")
    ap.add_argument("--full-records", action="store_true",
                    help="config 5: ship the full 272-B learner records every step (no provenance rebuild)")
    ap.add_argument("--gather", action="store_true",
                    help="config 5 also at one rank (always run with several ranks): learner records "
                         "gathered to rank 0, actions / memory scattered back")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for the bench's barrier/max/sum (nccl = RCCL); "
                         "gloo allows a rehearsal with several ranks on one GPU")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank uses cuda:0 (with --backend gloo)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary lines (config 2 at 4096 worlds/GPU, config 4 at 262144 worlds "
                         "in all, the reference loop at 4096 worlds/GPU and at --worlds)")
    ap.add_argument("--stream-priority", choices=("high", "normal"), default="high",
                    help="priority of the torch stream the step is launched on (the sensor's internal "
                         "stream is always high): both chains at high priority run the step 1.6 %% "
                         "faster than the caller's chain at normal (DESIGN.md 'Schedule')")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks
        # ourselves (this parent makes no GPU call at all: spawn_ranks)
        sys.exit(spawn_ranks(args))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world_size} but --gpus {args.gpus}: launch one rank per GPU "
                 f"(torchrun --nproc-per-node {args.gpus}) or drop the launcher")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world_size > 1
    if distributed and not args.same_device:
        ndev = torch.cuda.device_count()
        if ndev < world_size:
            sys.exit(f"bench.py: --gpus {world_size} needs {world_size} devices, {ndev} visible "
                     "(--same-device with --backend gloo rehearses several ranks on one GPU)")
    if distributed and args.same_device and args.backend == "nccl":
        sys.exit("bench.py: --same-device needs --backend gloo (RCCL takes one rank per GPU)")
    dev_index = 0 if (args.same_device or not distributed) else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if args.stream_priority == "high":
        # the caller's chain (K1, K2, K3a, shift, action write) on a
        # high-priority stream like the library's sensor stream
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    if distributed:
        if args.backend == "nccl":
            # (a bounded timeout: a collective that cannot complete ends the run
            # with an error instead of holding the node)
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=300))
        else:
            dist.init_process_group(args.backend, timeout=datetime.timedelta(seconds=300))

    import madrona_bots as mb
    W = args.worlds
    # every rank but the last steps a ghost of the next rank's first world, so the
    # faithful B.3 reward of its last world equals one device's (sim.cpp:943)
    ghost = rank < world_size - 1
    mgr = mb.SimManager(dev_index, W, SEED, AGENTS_PER_WORLD, world_offset=rank * W, shard_ghost=ghost)

    def one_step(t):
        mgr.step()
        mgr.shift_observations()
        mgr.write_synthetic_actions(ACTION_SEED, t + 1)

    mgr.write_synthetic_actions(ACTION_SEED, 0)
    for t in range(args.warmup):
        one_step(t)
    torch.cuda.synchronize()
    steps_before = mgr.agent_steps()
    # device time of the timed steps: an event on the launch stream (torch's
    # current stream, the one libmbots launches on) before the first step, and
    # the later of an event there after the last action write and one the
    # library records after the last sensor on its own stream -- both chains
    # of every step, no event inside the region (round 6: per-step sampled
    # spans started at the previous action write, and so also counted the
    # next K1's wait for the previous sensor whenever the sensor's chain was
    # the longer one)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for t in range(args.warmup, args.warmup + args.steps):
        one_step(t)
    ev[1].record()
    mgr.record_sensor_done(ev[2])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if distributed:
        dist.barrier()
    elapsed = t1 - t0
    span_ms = max(ev[0].elapsed_time(ev[1]), ev[0].elapsed_time(ev[2])) / args.steps
    agent_steps = mgr.agent_steps() - steps_before

    # per-kernel event spans: a separate pass after the timed region (the
    # events between kernels would idle the GPU inside the timed steps)
    ktimes = {}
    if not args.no_kernel_timing:
        mgr.enable_kernel_timing(True)
        t = args.warmup + args.steps
        for _ in range(min(args.steps, 50)):
            one_step(t)
            t += 1
        torch.cuda.synchronize()
        ktimes = mgr.kernel_times()
        mgr.enable_kernel_timing(False)
        t = args.warmup + args.steps + min(args.steps, 50)
    else:
        t = args.warmup + args.steps
    # the same loop once the worlds' food has reached its cap (30 per world,
    # from about step 200 on; the first steps run with little food, so the
    # sensor has fewer objects to test: profiles/r05_drivergap.json)
    steady = None
    if not args.no_secondary:
        while t < STEADY_FROM:
            one_step(t)
            t += 1
        torch.cuda.synchronize()
        s0 = mgr.agent_steps()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        ts0 = time.perf_counter()
        for k in range(STEADY_STEPS):
            one_step(t + k)
        torch.cuda.synchronize()
        el_s = time.perf_counter() - ts0
        n_s = mgr.agent_steps() - s0
        st_s = torch.tensor([el_s, float(n_s)], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        tot_s = float(n_s)
        if distributed:
            dist.barrier()
            tm_s = st_s[0:1].clone(); dist.all_reduce(tm_s, op=dist.ReduceOp.MAX)
            tt_s = st_s[1:2].clone(); dist.all_reduce(tt_s, op=dist.ReduceOp.SUM)
            el_s, tot_s = float(tm_s.item()), float(tt_s.item())
        nb_s = algorithmic_bytes(n_s / STEADY_STEPS, W)
        ms_s = el_s / STEADY_STEPS * 1e3
        steady = {"what": f"the headline loop at steps {t}-{t + STEADY_STEPS - 1} (food at its cap of 30 per world)",
                  "value": tot_s / el_s, "unit": "agent-steps/s", "ms_per_step": ms_s, "steps": STEADY_STEPS,
                  "mean_agents_per_world": n_s / STEADY_STEPS / W,
                  "roofline": {"bound": "hbm", "achieved": nb_s / (ms_s * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": nb_s / (ms_s * 1e-3) / 1e9 / HBM_PEAK_GBS,
                               "algorithmic_bytes_per_step": nb_s,
                               "timing": "wall clock of the timed steps (step + shift + action write)"}}
    # config 5 (BASELINE: sim + learner on rank 0, RCCL gather of the rollout
    # tensors): its own timed loop after the main line, by default whenever the
    # bench runs several ranks (so the driver's 1..8-GPU run covers it)
    cfg5 = None
    if distributed or args.gather:
        try:
            cfg5 = config5_loop(mgr, args, rank, world_size, dev, distributed)
        except Exception as e:   # reported in the line; the main measurement stands
            cfg5 = {"error": f"{type(e).__name__}: {e}"[:400]}
    secondary = ref_main = config2 = config4 = None
    if not args.no_secondary:
        config2 = bare_loop(4096, args, rank, world_size, dev, distributed,
                            "BASELINE config 2 on the headline's workload: step + shift + action write at "
                            "4096 worlds/GPU")
        # BASELINE config 4: 262144 worlds in all, sharded over the ranks
        # (strong scaling: 262144 / N worlds per GPU; at N = 8 the config itself)
        if CONFIG4_WORLDS % world_size == 0:
            config4 = bare_loop(CONFIG4_WORLDS // world_size, args, rank, world_size, dev, distributed,
                                f"BASELINE config 4: {CONFIG4_WORLDS} worlds sharded over {world_size} GPU(s) "
                                "(strong scaling), step + shift + action write")
            config4["scaling"] = "strong"
            config4["total_worlds"] = CONFIG4_WORLDS
        secondary = reference_loop(4096, args, rank, world_size, dev, distributed,
                                   "BASELINE config 2: random-action rollout, obs/reward tensors "
                                   "on device (learn/training_loop.py call sequence)")
        ref_main = reference_loop(W, args, rank, world_size, dev, distributed,
                                  "the reference training loop's call sequence at the main line's size")
    stats = torch.tensor([elapsed, float(agent_steps)], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
    if distributed:
        tmax = stats[0:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tot = stats[1:2].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, total_agent_steps = float(tmax.item()), float(tot.item())
    else:
        total_agent_steps = float(agent_steps)

    if rank == 0:
        mean_agents = agent_steps / args.steps          # this rank's mean population
        value = total_agent_steps / elapsed
        out = {
            "metric": "agent-steps/sec at 4096 & 65536 worlds; 1/2/4/8 MI355X scaling",
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (identity-keyed one-hot action stream, seed 69)",
            "stream_priority": args.stream_priority,
            "config": {"workload": f"{W} worlds/GPU x {AGENTS_PER_WORLD} initial agents "
                                   f"(BASELINE config {'3' if W == 65536 else 'custom'}), "
                                   "step+shift+action write",
                       "worlds_per_gpu": W, "total_worlds": W * world_size,
                       "mean_agents_per_world": mean_agents / W,
                       "world_steps_per_s": W * world_size * args.steps / elapsed,
                       "parallelism": f"world-shard x{world_size}, no collective"
                                      + (" (+1 ghost world on ranks 0..N-2: faithful B.3)"
                                         if world_size > 1 else "")},
        }
        nb = algorithmic_bytes(mean_agents, W)
        achieved = nb / (span_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": "world step: step()+shift_observations()+action write "
                "(K1 world_step, K2 scan, K3a export_rows, K5 shift (fused gather), actions || K3b sensor)",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "algorithmic_bytes_per_launch": nb, "avg_launch_ms": span_ms,
                "timing": "HIP events over the whole timed region / steps: one on the launch stream before "
                          "the first step, the later of one there after the last action write and one the "
                          "library records after the last sensor on its own stream (both chains, no event "
                          "inside the region)"}
        # the same span priced at the bytes this design must move in this loop
        nb_lazy = LAZY_BYTES_PER_AGENT * mean_agents + 1952.0 * W
        lazy_gbs = nb_lazy / (span_ms * 1e-3) / 1e9
        roof["lazy_bytes"] = {"bytes_per_agent": LAZY_BYTES_PER_AGENT, "bytes_per_step": nb_lazy,
                              "achieved": lazy_gbs, "frac": lazy_gbs / HBM_PEAK_GBS,
                              "note": "B_step minus the 88 B/agent of Prev* traffic the lazy shift "
                                      "skips when nothing reads the table between step and shift and "
                                      "the 64 B/agent prev-sensor move nothing reads before the next step"}
        wall_gbs = nb / (elapsed / args.steps) / 1e9
        roof["wall_clock"] = {"achieved": wall_gbs, "frac": wall_gbs / HBM_PEAK_GBS,
                              "frac_lazy_bytes": nb_lazy / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS,
                              "note": "B_step / ms_per_step (includes the action write)"}
        tr = load_traffic(W)
        if tr:
            roof["traffic"] = tr[1]["bytes_per_step"]
            roof["traffic_source"] = tr[0]
        out["roofline"] = roof
        if ktimes:
            per = {k: (ms / n if n else 0.0) for k, (ms, n) in ktimes.items()}
            out["kernel_ms"] = {k: round(v, 5) for k, v in per.items() if v}
            out["kernel_ms_note"] = ("HIP events around each kernel in an untimed pass after "
                                     "the timed region (overlapped schedule)")
            # per-kernel HBM rate: PMC bytes per launch / event span in the
            # overlapped schedule, beside rocprofv3's average for the same kernel
            kmap = {"world_step": "world_step_kernel", "scan": "scan_kernel",
                    "export": "export_rows_kernel", "move": "move_kernel",
                    "sensor": "sensor_kernel", "shift": "shift_kernel",
                    "actions": "synthetic_actions_kernel"}
            if tr:
                kst, kst_src = load_kernel_stats()
                kh = {}
                # a shift that follows a step is the fused gather (shift_move_kernel)
                if "shift_move_kernel" in tr[1]["kernels"]:
                    kmap["shift"] = "shift_move_kernel"
                for k, kn in kmap.items():
                    b = tr[1]["kernels"].get(kn, {}).get("hbm_bytes_per_launch")
                    if b and per.get(k):
                        gbs = b / (per[k] * 1e-3) / 1e9
                        kh[k] = {"hbm_bytes": b, "event_ms": round(per[k], 5),
                                 "rocprof_avg_ms": round(kst[kn], 5) if kn in kst else None,
                                 "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
                out["kernel_hbm"] = kh
                out["kernel_hbm_sources"] = {"bytes": tr[0], "rocprof": kst_src}
            vp = load_profile("valu", W)
            sens = vp[1]["kernels"].get("sensor_kernel") if vp else None
            if sens and per.get("sensor"):
                rate = sens["SQ_INSTS_VALU"] / (per["sensor"] * 1e-3)
                out["sensor_valu"] = {
                    "bound": "valu-issue", "kernel": "K3b sensor (the step's critical path)",
                    "valu_instr_per_launch": sens["SQ_INSTS_VALU"],
                    "salu_instr_per_launch": sens.get("SQ_INSTS_SALU"),
                    "launch_ms": per["sensor"], "achieved": rate, "peak": VALU_PEAK_INSTR_S,
                    "unit": "wave64 VALU instr/s", "frac": rate / VALU_PEAK_INSTR_S,
                    "source": vp[0],
                    "note": "launch_ms is the sensor's event span inside the overlapped schedule; "
                            "peak: the guide's nominal 2 cycles per wave64 instruction"}
                # issue cost per wave64 VALU instruction per SIMD at 2.4 GHz: the
                # nominal peak is 2 cycles; the microbenchmark's independent fp32
                # FMA / add streams take ~4.9, its compare/select mix ~3.5
                out["sensor_valu"]["cycles_per_instr_per_simd"] = 1024 * 2.4e9 / rate
                mp = measured_valu_peak()
                if mp:
                    out["sensor_valu"]["microbench_rate"] = mp[1]
                    out["sensor_valu"]["microbench_source"] = mp[0]
        if cfg5:
            out["config5"] = cfg5
        if config2:
            out["config2"] = config2
        if config4:
            out["config4"] = config4
        if steady:
            out["steady_state"] = steady
        if secondary:
            out["secondary"] = secondary
            out["reference_loop"] = ref_main
        if not args.no_cpu_baseline:
            # every CPU the process can actually use ("all host
            # cores"): its affinity set capped by the cgroup's CPU quota, one
            # thread each, on a sample of >= 64 worlds per thread
            eff = cpu_share()[0]
            out["cpu_baseline"] = cpu_baseline(max(args.cpu_worlds, 64 * eff), args.cpu_seconds, threads=eff)
        print(json.dumps(out), flush=True)

    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

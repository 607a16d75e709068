#!/usr/bin/env python3
"""A few steps of the reference training loop's call sequence (bench.py
reference_loop) at a given size, for a rocprofv3 kernel trace; or, with
--summarise DIR, the per-step timeline (us from each step's world_step start)
of the last steps in that trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rt -o run -- \
        python scripts/reftrace.py --worlds 4096
    python scripts/reftrace.py --summarise gpurun_out/rt
"""
import argparse
import csv
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(worlds, steps, main_loop):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
    import torch
    import bench
    import madrona_bots as mb
    m = mb.SimManager(0, worlds, bench.SEED, bench.AGENTS_PER_WORLD)
    m.write_synthetic_actions(bench.ACTION_SEED, 0, True)
    for t in range(steps):
        m.step()
        if not main_loop:
            m.species_count_tensor().to_torch().sum(dim=0).cumsum(dim=0)
            m.action_tensor(False).to_torch()
            m.hidden_state_tensor(False).to_torch()
            m.reward_tensor(False).to_torch().clone()
            m.health_tensor(False).to_torch().clone()
            m.construct_obs(False)
            m.construct_obs(True)
            m.hidden_state_tensor(True).to_torch()
        m.shift_observations()
        m.write_synthetic_actions(bench.ACTION_SEED, t + 1, not main_loop)
    torch.cuda.synchronize()


def summarise(d, last):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] == "world_step_kernel"]
    for a, b in zip(starts[-last - 1:-1], starts[-last:]):
        t0 = rows[a][0]
        print(f"step ({(rows[b][0] - t0) / 1e3:.1f} us)")
        for s, e, n in rows[a:b]:
            print(f"   {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--main-loop", action="store_true", help="bench.py's main loop instead")
    ap.add_argument("--summarise", default=None)
    ap.add_argument("--last", type=int, default=2)
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise, a.last)
    else:
        run(a.worlds, a.steps, a.main_loop)

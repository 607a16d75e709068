#!/usr/bin/env python3
"""Per-step device spans of the bench loop from the first step on (VERDICT r4
item 2: where the driver's 20-step / 5-warmup line loses against a 100-step
one).  Every step of `--steps` is bracketed like bench.py's sampled steps (an
event before step(), the later of one after shift() and one after the
sensor), and the host wall time of each step is recorded too.  Prints one JSON
line: per-step span (ms), host ms, and live agents per world."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--every", type=int, default=1, help="bracket every k-th step with events")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    import madrona_bots as mb
    t_create = time.perf_counter()
    m = mb.SimManager(0, args.worlds, 69, 32)
    torch.cuda.synchronize()
    t_create = time.perf_counter() - t_create
    m.write_synthetic_actions(1234, 0)
    ev = []
    host = []
    agents = []
    for t in range(args.steps):
        rec = t % args.every == 0
        if rec:
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                 torch.cuda.Event(enable_timing=True))
            e[0].record()
        h0 = time.perf_counter()
        m.step()
        m.shift_observations()
        if rec:
            e[1].record()
            m.record_sensor_done(e[2])
            ev.append((t, e))
        m.write_synthetic_actions(1234, t + 1)
        host.append((time.perf_counter() - h0) * 1e3)
        if t % 10 == 9:
            agents.append(m.num_agents() / args.worlds)
    torch.cuda.synchronize()
    spans = [(t, max(a.elapsed_time(b), a.elapsed_time(c))) for t, (a, b, c) in ev]
    print(json.dumps({"worlds": args.worlds, "create_s": t_create,
                      "span_ms": [[t, round(s, 5)] for t, s in spans],
                      "host_ms": [round(h, 4) for h in host],
                      "agents_per_world_every10": [round(a, 3) for a in agents]}), flush=True)


if __name__ == "__main__":
    main()

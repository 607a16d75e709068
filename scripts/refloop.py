#!/usr/bin/env python3
"""The bench's reference-loop line alone (A/B of library builds):
    MBOTS_LIB=build_var/libmbots_x.so python scripts/refloop.py [--worlds 4096]"""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import _variant  # noqa: E402,F401  (MBOTS_LIB: A/B builds)
import torch
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=4096)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--warmup", type=int, default=20)
a = ap.parse_args()
args = argparse.Namespace(steps=a.steps, warmup=a.warmup, no_kernel_timing=True, backend="nccl")
torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
r = bench.reference_loop(a.worlds, args, 0, 1, torch.device("cuda", 0), False, "ab")
print(json.dumps({"lib": os.path.basename(os.environ.get("MBOTS_LIB", "default")), "worlds": a.worlds,
                  "ms_per_step": r["ms_per_step"]}), flush=True)

#!/usr/bin/env python3
"""Unprofiled kernel timeline of the last step of a bench-like loop, from the
tlprobe variant (scripts/tlprobe_variant.py): per kernel, first wave start and
last wave end (us, relative to K1's first wave), and the gaps between them."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
import torch
import madrona_bots as mb
KINDS = ["world_step", "scan", "export", "sensor", "shift", "actions"]
NW = 1 << 17
W = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
lib = ctypes.CDLL(os.environ["MBOTS_LIB"])
m = mb.SimManager(0, W, 69, 32)
m.write_synthetic_actions(1234, 0)
res = []
for rep in range(5):
    for t in range(60):
        s = rep * 60 + t
        m.step(); m.shift_observations(); m.write_synthetic_actions(1234, s + 1)
    torch.cuda.synchronize()
    t0 = (ctypes.c_ulonglong * (6 * NW))()
    t1 = (ctypes.c_ulonglong * (6 * NW))()
    assert lib.mbots_dbg_probe_read(t0, t1) == 0
    row = {}
    for k, name in enumerate(KINDS):
        a = [t0[k * NW + i] for i in range(NW) if t1[k * NW + i]]
        b = [t1[k * NW + i] for i in range(NW) if t1[k * NW + i]]
        row[name] = (min(a), max(b), len(a))
    base = row["world_step"][0]
    out = {name: [round((v[0] - base) / 100.0, 2), round((v[1] - base) / 100.0, 2), v[2]] for name, v in row.items()}
    res.append(out)
    print(json.dumps(out), flush=True)

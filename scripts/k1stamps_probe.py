#!/usr/bin/env python3
"""K1 phase shares from an s_memtime-instrumented build (scratch; see
scripts/k1stamps_variant.py): per-wave cycles of each phase summed over a few
steps at 65536 worlds, and K1's event time with and without the stamps."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
import torch
import madrona_bots as mb
lib = ctypes.CDLL(os.environ["MBOTS_LIB"])
W = int(os.environ.get("WORLDS", "65536"))
m = mb.SimManager(0, W, 69, 32)
m.write_synthetic_actions(1234, 0)
for t in range(150):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
lib.mbots_dbg_clear_stamps()
for t in range(150, 160):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
a = (ctypes.c_ulonglong * 16)()
lib.mbots_dbg_read_stamps(a)
names = ["staging", "addfood", "action", "health", "surround", "species_respawn", "compaction", "block_tail"]
tot = a[8]
waves = max(1, a[9])
print(json.dumps({"worlds": W, "waves": a[9], "cycles_per_wave": tot / waves,
                  "share": {n: round(a[i] / tot, 4) for i, n in enumerate(names)},
                  "cycles": {n: round(a[i] / waves, 1) for i, n in enumerate(names)}}))

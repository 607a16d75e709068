#!/usr/bin/env python3
"""Sensor phase shares from an s_memtime-instrumented build (scratch; the
build's .so exports mbots_dbg_read_stamps): staging, P1 (cull), P2 (survivors
+ wide), output, per wave summed over a few steps."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madrona-bots_amd"))
import torch
import madrona_bots as mb
lib = ctypes.CDLL(os.environ["MBOTS_LIB"])
m = mb.SimManager(0, 65536, 69, 32)
m.write_synthetic_actions(1234, 0)
for t in range(150):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
lib.mbots_dbg_clear_stamps()
for t in range(150, 160):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
a = (ctypes.c_ulonglong * 8)()
lib.mbots_dbg_read_stamps(a)
tot = a[4]
print({"staging": a[0] / tot, "p1": a[1] / tot, "p2": a[2] / tot, "output": a[3] / tot,
       "waves": a[5], "cycles_per_wave": tot / max(1, a[5])})

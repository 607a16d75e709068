#!/usr/bin/env python3
"""Per-kernel shader clock of the last launch of each probed kernel
(scripts/clockprobe_variant.py): median over waves of (d s_memtime /
d s_memrealtime) x 100 MHz, after --steps of the bench's loop at --worlds.
    MBOTS_LIB=build_var/libmbots_clockprobe.so python scripts/clockprobe.py [--worlds W] [--steps K] [--alone]
--alone: one step then each kernel run serialised (AMD_SERIALIZE_KERNEL must
be set by the caller for that), for the clock of a kernel without neighbours."""
import argparse, ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "madrona-bots_amd"), os.path.join(ROOT, "scripts")]
import _variant  # noqa: E402,F401
import torch  # noqa: E402
import madrona_bots as mb  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--worlds", type=int, default=65536)
ap.add_argument("--steps", type=int, default=60)
a = ap.parse_args()
m = mb.SimManager(0, a.worlds, 69, 32)
m.write_synthetic_actions(1234, 0)
for t in range(a.steps):
    m.step(); m.shift_observations(); m.write_synthetic_actions(1234, t + 1)
torch.cuda.synchronize()
NW = 1 << 17
buf = np.zeros((5, 4, NW), np.uint64)
rc = mb._lib.mbots_dbg_clock_read(ctypes.c_void_p(buf.ctypes.data))
assert rc == 0, rc
out = {}
for k, name in enumerate(["world_step", "export_rows", "sensor", "shift_move", "synthetic_actions"]):
    r0, r1, c0, c1 = (buf[k, i].astype(np.float64) for i in range(4))
    ok = (r1 > r0) & (c1 > c0)
    if not ok.any():
        continue
    ghz = (c1[ok] - c0[ok]) / (r1[ok] - r0[ok]) * 0.1
    out[name] = {"waves": int(ok.sum()), "clock_ghz_median": round(float(np.median(ghz)), 3),
                 "p10": round(float(np.percentile(ghz, 10)), 3), "p90": round(float(np.percentile(ghz, 90)), 3)}
print(json.dumps({"worlds": a.worlds, "steps": a.steps, "clocks": out}))

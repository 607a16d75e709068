#!/usr/bin/env python3
"""HBM traffic per kernel launch / per step from rocprofv3 --pmc passes.

FETCH_SIZE and WRITE_SIZE (KB) come from separate passes (they do not fit one
pass on gfx950).  Correction per MI355X_MICROARCH.md 'HBM': FETCH_SIZE reports
1/2 of the bytes of a wide coalesced streaming read on gfx950, so reads are
counted as 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B stores.

    python scripts/traffic.py gpurun_out/<tag> <worlds> <out.json>
"""
import collections
import re
import csv
import glob
import json
import sys

root, worlds, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in sorted(glob.glob(f"{root}_p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
        if not k.endswith("_kernel"):
            continue
        d = int(r["Dispatch_Id"])
        vals[(r["Counter_Name"], k)][d] += float(r["Counter_Value"])
per = {}
for (cn, k), byd in vals.items():
    ds = sorted(byd)[-5:]                      # last launches (steady state)
    per.setdefault(k, {})[cn] = sum(byd[d] for d in ds) / len(ds)
step_kernels = ("world_step_kernel", "scan_kernel", "export_rows_kernel", "move_kernel",
                "sensor_kernel", "shift_kernel", "shift_move_kernel")
res = {"worlds": worlds, "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024",
       "kernels": {}}
tot = 0.0
# launches per step: a kernel a step does not launch every time (move_kernel
# runs at init and on deferred-move materialisation only) counts by its share
launches = {k: len(byd) for (cn, k), byd in vals.items() if cn == "FETCH_SIZE"}
n_steps = max(launches.get("world_step_kernel", 1), 1)
for k, c in sorted(per.items()):
    b = (2.0 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
    share = min(launches.get(k, n_steps) / n_steps, 1.0)
    res["kernels"][k] = {"FETCH_SIZE_KB": c.get("FETCH_SIZE"), "WRITE_SIZE_KB": c.get("WRITE_SIZE"),
                         "hbm_bytes_per_launch": b, "launches_per_step": share}
    if k in step_kernels:
        tot += b * share
res["bytes_per_step"] = tot
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))

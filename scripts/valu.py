#!/usr/bin/env python3
"""VALU / SALU wave-instructions per kernel launch from a rocprofv3 --pmc run
(SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_WAVES summed over XCDs, mean of the last 5
launches): the sensor's secondary (VALU-issue) roofline in bench.py.

    python scripts/valu.py gpurun_out/<dir> <worlds> <out.json>
"""
import collections
import re
import csv
import json
import sys

d, worlds, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
    k = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
    if k.endswith("_kernel"):
        vals[(r["Counter_Name"], k)][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
per = {}
for (cn, k), byd in vals.items():
    ds = sorted(byd)[-5:]
    per.setdefault(k, {})[cn] = sum(byd[x] for x in ds) / len(ds)
json.dump({"worlds": worlds, "counters": "SQ_INSTS_VALU/SALU: wave-instructions per launch",
           "kernels": per}, open(out, "w"), indent=1)
print(json.dumps(per.get("sensor_kernel", {})))

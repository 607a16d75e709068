#!/usr/bin/env python3
"""Per-launch kernel durations in launch order from a rocprofv3 kernel trace
(the cost of each step along the trajectory, kernel by kernel):
    python scripts/perstep.py run_kernel_trace.csv [first] [count]"""
import collections
import csv
import sys

KERNELS = ("world_step_kernel", "scan_kernel", "sensor_kernel", "export_rows_kernel", "shift_move_kernel",
           "synthetic_actions_kernel")
rows = collections.defaultdict(list)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        for k in KERNELS:
            if k in name:
                rows[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 60
for k in rows:
    rows[k].sort()
print("step " + " ".join(f"{k.replace('_kernel', ''):>18s}" for k in KERNELS))
for i in range(first, first + count):
    vals = []
    for k in KERNELS:
        v = rows[k]
        vals.append(f"{(v[i][1] - v[i][0]) / 1e3:18.1f}" if i < len(v) else f"{'-':>18s}")
    print(f"{i:4d} " + " ".join(vals))

#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (last N dispatches)."""
import csv, glob, sys, collections
import re
root = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}_p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
        rows[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
for k, cs in rows.items():
    print(k)
    for c, vals in sorted(cs.items()):
        # sum over XCD/instances with the same dispatch id, then average the last 5 dispatches
        per = collections.defaultdict(float)
        for d, v in vals:
            per[d] += v
        ds = sorted(per)[-5:]
        print(f"   {c:28s} {sum(per[d] for d in ds)/len(ds):16.1f}")

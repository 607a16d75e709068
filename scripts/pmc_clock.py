#!/usr/bin/env python3
"""Effective shader clock and issue-state split per kernel from one rocprofv3
--pmc pass that holds GRBM_GUI_ACTIVE (+ SQ_* wave-state counters), joined
with the same pass's kernel trace (MI355X_MICROARCH.md "DVFS give-back":
clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; SQ_WAVE_CYCLES =
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, quad-cycles).

    python scripts/pmc_clock.py <rocprofv3 output dir> [skip_dispatches]
"""
import collections, csv, json, re, statistics, sys

d = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 20
name = lambda s: re.sub(r"<.*>", "", s.split("(")[0]).split()[-1].replace("mbots::", "")   # noqa: E731
dur = {}
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    dur[int(r["Dispatch_Id"])] = (name(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
    vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
per = collections.defaultdict(list)
for did in sorted(vals)[skip:]:
    k, t = dur[did]
    c = dict(vals[did])
    c["_s"] = t
    per[k].append(c)
out = {}
for k, lst in per.items():
    m = {c: statistics.mean(x[c] for x in lst) for c in lst[0]}
    o = {"dispatches": len(lst), "mean_us": m["_s"] * 1e6}
    if "GRBM_GUI_ACTIVE" in m and m["_s"] > 0:
        o["clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / m["_s"] / 1e9
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_SALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if c in m:
                o[c + "_frac"] = m[c] / wc
    out[k] = o
print(json.dumps(out, indent=1))

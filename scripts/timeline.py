#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV: mean step
period (K1 start to K1 start), mean kernel durations, and the median step's
kernels (queue, start, end in us from its K1 start).

    python scripts/timeline.py <run_kernel_trace.csv> [skip_steps]
"""
import csv, re, statistics, sys
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r["Queue_Id"]))
rows.sort()
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 10
k1 = [r[0] for r in rows if r[2] == "world_step_kernel"][skip:]
per = [(b - a) / 1e3 for a, b in zip(k1, k1[1:])]
print(f"steps {len(per)}: mean step {statistics.mean(per):.1f} us, median {statistics.median(per):.1f}")
dur = {}
for s, e, k, q in rows:
    if k1 and k1[0] <= s < k1[-1]:
        dur.setdefault(k, []).append((e - s) / 1e3)
for k, v in sorted(dur.items(), key=lambda kv: -statistics.mean(kv[1])):
    print(f"  {k:32s} {statistics.mean(v):8.1f} us  x{len(v) / max(1, len(per)):.2f}/step")
i = sorted(range(len(per)), key=lambda j: per[j])[len(per) // 2]
t0, t1 = k1[i], k1[i + 1]
print("median step (us from its K1 start): name queue start end")
for s, e, k, q in rows:
    if t0 <= s < t1 or (s < t0 < e):
        print(f"  {k:32s} q{q:3s} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}")

#!/usr/bin/env python3
"""Per-step timeline from a rocprofv3 kernel trace: where the step's wall time
goes (kernel spans per stream, idle gaps on the critical path).

    python scripts/timeline.py gpurun_out/prof_r01/run_kernel_trace.csv [last_steps]
"""
import csv, sys
import re
from collections import defaultdict

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        name = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r["Queue_Id"]))
rows.sort()
steps, cur = [], None
for s, e, n, q in rows:
    if n == "world_step_kernel":
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append((s, e, n, q))
steps = steps[-last - 1:-1]          # drop the tail step (may be incomplete)
span = defaultdict(float); gap_k1 = []; total = []
for st in steps:
    t0 = st[0][0]
    for s, e, n, q in st:
        span[n] += (e - s) / 1e3
    total.append(None)
for a, b in zip(steps, steps[1:]):
    total[steps.index(a)] = (b[0][0] - a[0][0]) / 1e3
    ends = {n: e for s, e, n, q in a}
    k1 = b[0][0]
    gap_k1.append({n: (k1 - ends[n]) / 1e3 for n in ("sensor_kernel", "synthetic_actions_kernel") if n in ends})
n = len(steps)
tot = [t for t in total if t is not None]
print(f"steps {n}: mean step {sum(tot)/len(tot):.1f} us")
for k, v in sorted(span.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v/n:8.1f} us")
# one representative step, offsets from K1 start
st = steps[len(steps) // 2]
t0 = st[0][0]
print("representative step (us from K1 start): name queue start end")
for s, e, nme, q in st:
    print(f"  {nme:28s} q{q} {(s-t0)/1e3:8.1f} {(e-t0)/1e3:8.1f}")
g = defaultdict(float)
for d in gap_k1:
    for k, v in d.items():
        g[k] += v
print("next K1 start minus end of:", {k: round(v / len(gap_k1), 1) for k, v in g.items()})

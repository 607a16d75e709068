#!/usr/bin/env python3
"""Which chain ends each step (rocprofv3 --kernel-trace CSV of the bench's
loop): per step, the sensor's end and the caller chain's last kernel's end
(the action write), in us from that step's K1 start, and the step period.

    python scripts/chain_ends.py <run_kernel_trace.csv> [first_step] [last_step]
"""
import csv, re, sys
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).split()[-1].replace("mbots::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
k1 = [r[0] for r in rows if r[2] == "world_step_kernel"]
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else len(k1) - 2
print("step  period  k1_end  sensor_start  sensor_end  export_end  shift_end  write_end  last")
for i in range(lo, min(hi + 1, len(k1) - 1)):
    t0, t1 = k1[i], k1[i + 1]
    ends = {}
    for s, e, k in rows:
        if t0 <= s < t1:
            ends.setdefault(k, (s, e))
    g = lambda k, j: (ends[k][j] - t0) / 1e3 if k in ends else float("nan")   # noqa: E731
    se, we = g("sensor_kernel", 1), g("synthetic_actions_kernel", 1)
    print(f"{i:4d} {(t1 - t0) / 1e3:7.1f} {g('world_step_kernel', 1):7.1f} {g('sensor_kernel', 0):12.1f} "
          f"{se:10.1f} {g('export_rows_kernel', 1):10.1f} {g('shift_move_kernel', 1):9.1f} {we:9.1f}  "
          f"{'sensor' if se > we else 'caller'}")

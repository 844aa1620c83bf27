#!/usr/bin/env python3
"""Print one bench step's kernel timeline (start offset, gap before, duration) from a rocprofv3 trace.

usage: step_timeline.py gpurun_out/prof_TAG/trace/run_kernel_trace.csv [step_from_end=2]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
starts = [i for i, r in enumerate(rows) if "k_mlp_fwd" in r["Kernel_Name"]]
a, b = starts[-k - 1], starts[-k]
t0 = int(rows[a]["Start_Timestamp"])
pe = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - pe) / 1e3 if pe else 0.0
    print(f"{(s - t0) / 1e3:8.1f} {gap:7.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
    pe = e
print(f"step wall {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")

#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel time inside the bench's timed steps and idle gaps."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# step boundaries: each step launches exactly one MLP forward (split-bf16 k_fwd or exact k_mlp_fwd)
starts = [int(r["Start_Timestamp"]) for r in rows
          if "k_mlp_fwd<true>" in r["Kernel_Name"] or "mlps::k_fwd<true" in r["Kernel_Name"]  # <SAVE[, FOLD]>
          or "mlps::k_fwd8(" in r["Kernel_Name"]]
if len(starts) < 3:
    sys.exit("not enough steps")
# last 5 complete timed steps: the final k_fwd is bench.py's pair-count render after the timed loop,
# so the window ends at the one before it (the post-loop host work is not step idle)
if len(starts) < 8:
    sys.exit("not enough steps")
lo, hi = starts[-7], starts[-2]
steps = 5
busy = 0
per = defaultdict(float)
prev_end = None
gaps = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < lo or s >= hi:
        continue
    busy += e - s
    per[r["Kernel_Name"][:90]] += (e - s)
    if prev_end is not None and s > prev_end:
        gaps.append((s - prev_end, r["Kernel_Name"][:60]))
    prev_end = max(prev_end or 0, e)
wall = hi - lo
print(f"wall/step {wall/steps/1e6:.3f} ms  busy/step {busy/steps/1e6:.3f} ms  idle {100*(1-busy/wall):.1f}%")
for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v/steps/1e3:9.1f} us  {k}")
gaps.sort(reverse=True)
print("largest gaps (us) before:")
for g, k in gaps[:12]:
    print(f"{g/1e3:9.1f}  {k}")

#!/usr/bin/env python3
"""Per-kernel averages of the tools/stall_pmc.sh counter passes (default: the split-bf16 MLP kernels;
KERNELS="name=substring,..." picks others, e.g. KERNELS="fwd=k_blend_fwd,bwd2=k_blend_bwd2<,bwd2s=k_blend_bwd2s")."""
import csv
import glob
import os
import sys
from collections import defaultdict

KERNELS = {"k_fwd": "mlps::k_fwd<true", "k_bwd": "mlps::k_bwd<", "k_dws": "mlps::k_dws("}
if os.environ.get("KERNELS"):
    KERNELS = dict(kv.split("=", 1) for kv in os.environ["KERNELS"].split(","))


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = next((k for k, s in KERNELS.items() if s in r.get("Kernel_Name", "")), None)
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c in sorted(avg):
            print(f"   {c:28s} {avg[c]:.4g}")
        w = avg.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                if c in avg:
                    print(f"   {c:28s} / wave cycles = {avg[c] / w:.3f}")


if __name__ == "__main__":
    main()

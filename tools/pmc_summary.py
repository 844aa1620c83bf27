#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc CSV outputs under a directory:
python3 tools/pmc_summary.py gpurun_out/mlp_pmc_<tag> [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    keys = sys.argv[2:] or ["k_fwd", "k_bwd", "k_dw", "k_mlp"]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v) / len(v):.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()

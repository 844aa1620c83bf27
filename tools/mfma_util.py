#!/usr/bin/env python3
"""MFMA utilisation per kernel class from one rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES and
GRBM_GUI_ACTIVE (tools/mfma_util.sh): util = MFMA busy cycles (summed over the SIMDs) / (kernel
cycles x 1024 SIMDs), kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs;
MI355X_MICROARCH.md, DVFS note). The effective clock GRBM_GUI_ACTIVE / 8 / duration is printed too.
usage: mfma_util.py gpurun_out/mfma_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict

CLASSES = {"mlp_fwd": ("mlps::k_fwd",), "mlp_bwd": ("mlps::k_bwd",), "mlp_dw": ("mlps::k_dws(", "mlp::k_dw("),
           "blend_fwd": ("k_blend_fwd",), "blend_bwd": ("k_blend_bwd",)}


def main():
    root = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            cls = next((c for c, subs in CLASSES.items() if any(s in name for s in subs)), None)
            if cls is None:
                continue
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id") or "", name)
            vals[cls][r["Counter_Name"]].append((key, float(r["Counter_Value"]),
                                                 int(r.get("End_Timestamp", 0) or 0) - int(r.get("Start_Timestamp", 0) or 0)))
    print(f"{'kernel':10s} {'launches':>8s} {'MFMA busy':>12s} {'util':>7s} {'eff. clock':>10s}")
    for cls, cs in vals.items():
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", [])
        gui = cs.get("GRBM_GUI_ACTIVE", [])
        if not busy or not gui:
            continue
        b = sum(v for _, v, _ in busy) / len(busy)
        g = sum(v for _, v, _ in gui) / len(gui)
        cyc = g / 8.0
        util = b / (cyc * 1024.0) if cyc else 0.0
        durs = [d for _, _, d in gui if d > 0]
        clk = (cyc / (sum(durs) / len(durs)) if durs else 0.0)  # cycles per ns = GHz
        print(f"{cls:10s} {len(busy):8d} {b:12.4g} {util:7.3f} {clk:9.2f}G")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_prof.sh).

FETCH_SIZE / WRITE_SIZE are reported in KiB. On gfx950 FETCH_SIZE counts half the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section), so it is doubled here; WRITE_SIZE is exact for
16-B-per-lane stores and float atomics. Output: JSON {kernel_class: {fetch_bytes, write_bytes,
traffic_bytes, launches}} for the bench.py kernel classes.

usage: pmc_traffic.py gpurun_out/prof_TAG > profiles/<round>_pmc_traffic.json
"""
import csv
import json
import os
import sys
from collections import defaultdict

CLASSES = {  # bench.py kernel class -> substring(s) of the device symbol (split-bf16 | exact-fp32 MLP)
    # mlp_fwd: the training forward (saved activations) only, the launches bench.py times
    "mlp_fwd": ("mlps::k_fwd8(", "mlps::k_fwd<true", "k_mlp_fwd<true"), "mlp_bwd": ("mlps::k_bwd", "k_mlp_bwd"),
    "mlp_dw": ("mlp::k_dw(", "mlps::k_dw(", "mlps::k_dws(", "mlps::k_dwg(", "mlp4k_dw"), "mlp_dw_reduce": "k_dw_reduce",
    "preprocess_fwd": ("k_preprocess(", "k_preprocess<"), "duplicate": "k_duplicate", "ranges": "k_ranges",
    "blend_fwd": "k_blend_fwd", "blend_bwd": "k_blend_bwd", "preprocess_bwd": "k_preprocess_bwd",
    "ssim_fwd": "k_ssim_fwd", "ssim_bwd": "k_ssim_bwd", "adam": "k_adam", "inputs_fwd": "k_inputs_fwd",
    "inputs_bwd": "k_inputs_bwd", "count": "k_rect_count", "scan": "k_rect_colscan", "place": "k_rect_place",
    "tile_sort": "k_tile_sort", "depth_sort": ("radix::k_hist", "radix::k_scatter"), "blend_gather": "k_rect_gather",
}


def load(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    root = sys.argv[1]
    fetch = load(os.path.join(root, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(root, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for cls, sub in CLASSES.items():
        subs = sub if isinstance(sub, tuple) else (sub,)

        def match(k):  # the readable part of the symbol rocprofv3 prints
            return any(x in k for x in subs) and ("k_dw_reduce" not in k or cls == "mlp_dw_reduce")
        fk = [k for k in fetch if match(k)]
        wk = [k for k in write if match(k)]
        if not fk or not wk:
            continue
        fv = [v for k in fk for v in fetch[k]]
        wv = [v for k in wk for v in write[k]]
        f = 2.0 * sum(fv) / len(fv)
        w = sum(wv) / len(wv)
        out[cls] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w, "launches": len(fv),
                    "source": os.path.basename(root.rstrip("/"))}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()

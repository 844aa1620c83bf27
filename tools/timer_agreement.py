#!/usr/bin/env python3
"""Agreement of bench.py's HIP-event roofline timing with rocprofv3 in the SAME traced run
(tools/gpu_prof.sh): the rocprofv3 durations of the roofline kernel's launches that bench.py timed
(the last --steps launches, every 4th one sampled) vs the bench line's roofline.avg_launch_ms.
usage: timer_agreement.py gpurun_out/prof_TAG [steps]"""
import csv
import glob
import json
import os
import sys

SYMBOL = {"mlp_fwd": ("mlps::k_fwd8(", "mlps::k_fwd<true"), "mlp_bwd": ("mlps::k_bwd<", "mlps::k_bwd8("),
          "mlp_dw": ("mlps::k_dws(",)}


def main():
    root = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    line = [ln for ln in open(os.path.join(root, "bench_trace.log")) if ln.startswith("{")][-1]
    b = json.loads(line)
    r = b["roofline"]
    # the bench times the roofline candidates on every `period`-th step (bench.py: 8 when steps >= 16,
    # 4 when >= 8); read it from the bench line so both sides average the same launches
    period = int(b.get("kernel_timing", {}).get("period", 4))
    f = glob.glob(os.path.join(root, "trace", "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
    d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in rows
         if any(k in x["Kernel_Name"] for k in SYMBOL[r["kernel"]])]
    timed = d[-steps:]
    sampled = timed[0::period] if r["launches"] < steps else timed
    rp = sum(sampled) / len(sampled)
    print(json.dumps({"kernel": r["kernel"], "bench_hip_events_ms": r["avg_launch_ms"], "bench_launches": r["launches"],
                      "rocprof_same_launches_ms": rp, "rocprof_all_timed_ms": sum(timed) / len(timed),
                      "period": period, "ratio": r["avg_launch_ms"] / rp}))


if __name__ == "__main__":
    main()

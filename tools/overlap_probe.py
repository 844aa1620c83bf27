#!/usr/bin/env python3
"""Does a gradient collective overlap the network backward on MI355X?

The data-parallel step (NativeStep.step_data_parallel) issues the Gaussian-gradient all-reduce on
RCCL's stream right after phase 1 and queues phase 2 — the network's dX (k_bwd, a persistent grid of
one 147-KB workgroup per CU) and dW (k_dws, 256 workgroups that each fill a CU's register file) —
behind it on the compute stream. A one-GPU box cannot run RCCL with two ranks, so this probe runs
the same step on one GPU with a STAND-IN for the collective (dgs_debug_collective_standin: `nwg`
workgroups of 256 threads streaming read-modify-write sweeps over the 23.6 MB Gaussian gradient
buffer, the shape of an RCCL ring all-reduce) enqueued exactly where the all-reduce goes, and with
the MLP kernels optionally leaving `reserve` CUs free (dgs_mlp_set_reserved_cus).

  python tools/overlap_probe.py --mode standin --reserve 0 [--nwg 16 --passes 2]   # one config
  python tools/overlap_probe.py --sweep [--wide]                                    # A/B table
  python tools/overlap_probe.py --analyze <rocprofv3 kernel_trace.csv>              # overlap from a trace

Each config prints one JSON line: ms per step over --steps timed steps, and (from HIP events on the
side stream) the stand-in's own duration in the step vs alone.
"""
import argparse
import csv
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)


def setup(N=100_000, R=800):
    import torch
    from deformgs import native_step
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.renderer import render
    from deformgs.synthetic import synth_camera, synth_gaussians
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g = synth_gaussians(N, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    opt = OptimizationParams()
    gs.training_setup(opt)
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    with torch.no_grad():  # bench.py's steady-state head scale
        for h in (deform.deform.gaussian_warp, deform.deform.gaussian_rotation, deform.deform.gaussian_scaling):
            h.weight.mul_(0.01)
            h.bias.mul_(0.01)
    deform.train_setting(opt)
    pipe, bg = PipelineParams(), torch.zeros(3, device=dev)
    cams = [synth_camera(R, R, index=k, fid=k / 30.0, device=dev) for k in range(8)]
    gts = []
    gen = torch.Generator(device=dev).manual_seed(100)
    with torch.no_grad():
        for cam in cams:
            d = deform.step(gs.get_xyz.detach(), cam.fid.unsqueeze(0).expand(N, -1))
            img = render(cam, gs, pipe, bg, d[0], d[1], d[2], False)["render"]
            gts.append((img + 0.02 * torch.randn(img.shape, device=dev, generator=gen)).clamp_(0.0, 1.0))
    ns = native_step.NativeStep(gs, deform)
    return gs, deform, cams, gts, bg, ns


def run(mode, reserve, steps, warmup, nwg, passes, state=None):
    import torch
    from deformgs import _lib
    from deformgs.train_step import optimizer_step
    lib = _lib.load()
    lib.dgs_mlp_set_reserved_cus(reserve)
    gs, deform, cams, gts, bg, ns = state or setup()
    comp = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    ev_a = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    ev_b = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    it = [3000]

    def step(k, timed):
        cam, gt = cams[k % 8], gts[k % 8]
        _, _, over = ns(cam, gt, bg, True, 0.0, 0.2, True, phase=1)
        if over:
            ns(cam, gt, bg, True, 0.0, 0.2, False, phase=1)
        if mode == "standin":
            side.wait_stream(comp)  # the Gaussian gradients are final: the collective may start
            with torch.cuda.stream(side):
                if timed:
                    ev_a[k].record(side)
                _lib.check(lib.dgs_debug_collective_standin(ctypes.c_void_p(ns.gflat.data_ptr()), ns.gflat.numel(),
                                                            nwg, passes, ctypes.c_void_p(side.cuda_stream)),
                           "collective_standin")
                if timed:
                    ev_b[k].record(side)
        ns.network_backward()
        if mode == "standin":
            comp.wait_stream(side)  # Adam after the collective (as RCCL's wait())
        elif mode == "serial":  # no overlap: the collective queued after the network backward
            _lib.check(lib.dgs_debug_collective_standin(ctypes.c_void_p(ns.gflat.data_ptr()), ns.gflat.numel(),
                                                        nwg, passes, ctypes.c_void_p(comp.cuda_stream)),
                       "collective_standin")
        optimizer_step(gs, deform, it[0])
        it[0] += 1

    for k in range(warmup):
        step(k, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k, True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    res = {"mode": mode, "reserve": reserve, "nwg": nwg, "passes": passes, "ms_per_step": ms,
           "gflat_mb": ns.gflat.numel() * 4 / 1e6}
    if mode == "standin":
        inside = sorted(a.elapsed_time(b) for a, b in zip(ev_a, ev_b))
        # the stand-in alone (nothing else on the GPU), same launch shape
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        alone = []
        for _ in range(5):
            a.record(side)
            lib.dgs_debug_collective_standin(ctypes.c_void_p(ns.gflat.data_ptr()), ns.gflat.numel(), nwg, passes,
                                             ctypes.c_void_p(side.cuda_stream))
            b.record(side)
            side.synchronize()
            alone.append(a.elapsed_time(b))
        res["standin_ms_in_step_median"] = inside[len(inside) // 2]
        res["standin_ms_alone_median"] = sorted(alone)[2]
    lib.dgs_mlp_set_reserved_cus(0)
    return res


def analyze(path):
    """Per stand-in launch in a rocprofv3 kernel trace: its start / end relative to the phase-2 MLP
    kernels it should overlap (k_bwd, k_dws) and the fraction of its lifetime spent under them."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    mlp = [(s, e, n) for s, e, n in iv if "mlps::k_bwd" in n or "mlps::k_dws" in n]
    out = []
    for s, e, n in iv:
        if "k_collective_standin" not in n:
            continue
        under = 0
        for ms, me, _ in mlp:
            under += max(0, min(e, me) - max(s, ms))
        nxt = [x for x in mlp if x[0] >= s - 2_000_000]
        bwd = next((x for x in nxt if "k_bwd" in x[2]), None)
        out.append({"standin_us": (e - s) / 1e3, "under_mlp_frac": under / max(1, e - s),
                    "start_minus_k_bwd_start_us": (s - bwd[0]) / 1e3 if bwd else None,
                    "end_minus_k_bwd_end_us": (e - bwd[1]) / 1e3 if bwd else None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["plain", "standin", "serial"], default="standin")
    ap.add_argument("--reserve", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nwg", type=int, default=16)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--wide", action="store_true", help="with --sweep: stand-in widths 16 / 32, reserves 16 / 32, serial")
    ap.add_argument("--analyze")
    a = ap.parse_args()
    if a.analyze:
        rows = analyze(a.analyze)
        for r in rows:
            print(json.dumps(r))
        if rows:
            fr = sorted(r["under_mlp_frac"] for r in rows)
            print(json.dumps({"launches": len(rows), "under_mlp_frac_median": fr[len(fr) // 2],
                              "standin_us_median": sorted(r["standin_us"] for r in rows)[len(rows) // 2]}))
        return
    if not a.sweep:
        print(json.dumps(run(a.mode, a.reserve, a.steps, a.warmup, a.nwg, a.passes)), flush=True)
        return
    state = setup()
    # alternating order, twice, so box drift does not pose as an effect
    configs = [("plain", 0, a.nwg), ("standin", 0, a.nwg), ("plain", 4, a.nwg), ("standin", 4, a.nwg),
               ("plain", 8, a.nwg), ("standin", 8, a.nwg)]
    if a.wide:  # the stand-in's workgroup count against the reserve, and the serial (no-overlap) form
        configs = [("plain", 0, 16), ("serial", 0, 16), ("serial", 0, 32), ("standin", 0, 16), ("standin", 0, 32),
                   ("plain", 16, 16), ("standin", 16, 16), ("standin", 16, 32),
                   ("plain", 32, 32), ("standin", 32, 32), ("standin", 32, 16)]
    for rep in range(2):
        for mode, reserve, nwg in configs:
            r = run(mode, reserve, a.steps, a.warmup, nwg, a.passes, state)
            r["rep"] = rep
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

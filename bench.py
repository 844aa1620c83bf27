#!/usr/bin/env python3
"""Training-step throughput of the MI355X deformable-Gaussian path (BASELINE.json metric).

One step = one camera/timestep of train_baseline.py:104-182: fused deformation MLP forward ->
HIP rasterizer forward -> 0.8*L1 + 0.2*(1-SSIM) -> backward (raster + MLP) -> [RCCL grad
all-reduce when N>1] -> Adam on the Gaussians and the MLP. Workload: synth-100k:
100k Gaussians, 800x800, blender deformation network (timenet on), SH degree 3, synthetic
(random-init weights, random target image). Inputs are resident in HBM before timing starts.

Run: python bench.py [--gpus N --steps K --warmup W]. N>1: one rank per GPU over RCCL. Under
torch.distributed.run (WORLD_SIZE set) each process is one rank; invoked directly with --gpus N > 1 the
parent makes no GPU call and starts `python -m torch.distributed.run --nproc-per-node N bench.py ...` as
a child process, waits for it and exits with its return code (launcher_cmd). Rank 0 prints ONE JSON line
(value = whole-job iters/s = world * K / max-rank time).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense FP32 matrix peak (spec)
# split-f16 GEMMs (csrc/mlp_split.hip, round 6): an fp32 product costs three f16 MFMA products (hh + hl +
# lh of a scaled two-piece split), so their fp32 roofline is the dense f16 MFMA peak (~2.5 PF, the bf16
# rate: MI355X_MICROARCH.md) / 3 (rounds 1-5: the bf16x6 split, / 6)
SPLIT_MFMA_PEAK_TFLOPS = 2500.0 / 3
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")  # tools/pmc_traffic.py output
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak (spec)

# multiply-accumulates per point of the blender network with one frame time per step
# (train_baseline.py:107-110): the timenet (13*256 + 256*30 = 11,008 MACs) is evaluated
# once per launch, and its gradients come from the layer-0/5 bias gradients (DGS_MLP_UNIFORM_T). The
# reference network has 508,928 trunk + head weights; with one frame time t_emb is a constant whose
# 2 x 256 x 30 linear.0 / linear.5 columns fold into the biases (once per launch), so the per-point
# work the kernels do, and are credited with, is 508,928 - 15,360 = 493,568 MACs forward and for dW
MLP_FWD_MAC = 493568            # every trunk + head weight once, t_emb columns folded
MLP_DX_MAC = 461312             # W^T products whose input gradient is needed (heads, L7..L1 hidden rows)
MLP_DW_MAC = 493568             # every trunk + head weight once, t_emb columns from gb (x) te
# Algorithmic HBM bytes per point of the MLP kernels (blender network, one frame time):
#   k_fwd8: the saved activations it writes for dW (x_emb 64 + H0..H7 2048 rows, fp32) + the relu' bits
#           of the 2048 trunk rows + xyz in + the 10 outputs
#   k_bwd:  the dZ rows it writes (8 x 256 + the 32 dOut rows, fp32) + the relu' bits + dOut in
#   k_dws:  every row the dW jobs read once (X: 2 x 64 x_emb + H0..H6 + H4 again + H7 = 2432 rows; dZ:
#           8 x 256 + dZ5 again + 32 = 2336 rows), plus the per-workgroup slabs (constant per launch)
MLP_FWD_BYTES = 4 * 2112 + 2048 / 8 + 12 + 40
MLP_BWD_BYTES = 4 * 2080 + 2048 / 8 + 40
MLP_DW_BYTES = 4 * (2432 + 2336)
MLP_DW_SLAB_BYTES = 256 * (256 * 256 + 256) * 4


ARGV_ENV = "DGS_BENCH_ARGV"  # the parent's arguments for the launched ranks (JSON list)


def launcher_cmd(argv, nproc, port):
    """(command, extra environment) that run this bench as `nproc` ranks on one node (no GPU call in the
    parent): torch.distributed.run on 127.0.0.1. The bench arguments travel in DGS_BENCH_ARGV, not on the
    command line: torch.distributed.run's parser matches option prefixes even after the script name
    (`--n` is ambiguous with its --nnodes / --nproc-per-node / --node-rank)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    return cmd, {ARGV_ENV: json.dumps(list(argv))}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def maybe_launch(args, argv):
    """--gpus N > 1 without WORLD_SIZE: run the ranks as a child torch.distributed.run (subprocess, not
    exec: the parent has touched no GPU and simply waits) and return its exit code; else None."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    cmd, extra = launcher_cmd(argv, args.gpus, _free_port())
    print("[bench] launching " + " ".join(cmd) + " with " + str(extra), file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ, **extra))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--cpu-steps", type=int, default=20, help="timed CPU steps (median; SURVEY.md 8d: 3 + 20)")
    ap.add_argument("--no-adam", action="store_true", help="time only the reference's span (fwd+bwd)")
    ap.add_argument("--kernel-timing", choices=["roofline", "major", "all", "none"], default="roofline",
                    help="kernel classes timed with HIP events inside the timed region. Each event record costs "
                         "~6 us of GPU idle on the launch stream (profiles/r2c trace), so the default times only the "
                         "three MLP classes, the candidates for the longest launch of the step, on every 4th step; "
                         "'major' adds the blend classes, 'all' every class, 'none' nothing (every step)")
    ap.add_argument("--6dof", dest="six_dof", action="store_true",
                    help="6-DoF screw deformation head (config 4, trex --is_6dof) instead of d_xyz")
    ap.add_argument("--raw-init", action="store_true",
                    help="keep nn.Linear's default init on the deformation heads (the iteration-3000 transient: "
                         "deltas O(0.3) make every Gaussian hundreds of pixels wide)")
    return ap.parse_args(argv)


SYNC_COUNT = os.environ.get("DGS_BENCH_SYNC_COUNT", "0") == "1"  # A/B: the synchronous pair count


def mfma_peak(name):
    """Dense MFMA peak (fp32-equivalent TFLOP/s) of the arithmetic kernel class `name` runs on."""
    exact = os.environ.get("DGS_MLP_EXACT_FP32", "0") not in ("", "0")
    if name == "mlp_dw" and os.environ.get("DGS_MLP_SPLIT_DW", "3") == "0":
        return FP32_MFMA_PEAK_TFLOPS, "fp32 MFMA (v_mfma_f32_32x32x2_f32)"
    if exact:
        return FP32_MFMA_PEAK_TFLOPS, "fp32 MFMA (v_mfma_f32_32x32x2_f32)"
    return SPLIT_MFMA_PEAK_TFLOPS, "f16 MFMA peak / 3 (scaled hi/lo f16 split, three products per fp32 product)"


def mlp_bytes(name, N):
    """Algorithmic HBM bytes per launch of an MLP kernel class (padded points: 64-point blocks)."""
    Ns = -(-N // 64) * 64
    if name == "mlp_fwd":
        return MLP_FWD_BYTES * Ns
    if name == "mlp_bwd":
        return MLP_BWD_BYTES * Ns
    if name == "mlp_dw":
        return MLP_DW_BYTES * Ns + MLP_DW_SLAB_BYTES
    return None


def kernel_algorithmic(name, N, P, HW, cap=None, T=None):
    """(amount, unit, bound) per launch for the roofline of a kernel class. P = pairs,
    cap = the launched pair capacity of the sort-path kernels (>= P; their loops cover cap items),
    T = tiles."""
    cap = max(cap or P, P)
    T = T or 1
    NB = -(-N // 256)
    if name == "mlp_fwd":
        return 2.0 * MLP_FWD_MAC * N, "flop", "mfma"
    if name == "mlp_bwd":
        return 2.0 * MLP_DX_MAC * N, "flop", "mfma"
    if name == "mlp_dw":
        return 2.0 * MLP_DW_MAC * N, "flop", "mfma"
    if name == "preprocess_fwd":
        return 327.0 * N, "byte", "hbm"
    if name == "preprocess_bwd":
        return 600.0 * N, "byte", "hbm"
    if name == "blend_fwd":
        return 44.0 * P + 24.0 * HW, "byte", "hbm"
    if name == "blend_bwd":
        return 44.0 * P + 24.0 * HW + 48.0 * N, "byte", "hbm"
    if name == "depth_sort":
        return 64.0 * N, "byte", "hbm"       # 4 passes x (read + write) x (4-B key + 4-B id)
    # rect binning (default): count matrix NB x T u32, no keys
    if name == "count":
        return 16.0 * N + 4.0 * NB * T, "byte", "hbm"      # order, xy, radii in; count matrix out
    if name == "scan":
        return 8.0 * NB * T + 24.0 * T, "byte", "hbm"      # count matrix in + offsets out; totals, starts, ranges
    if name == "place":
        return 16.0 * N + 4.0 * NB * T + 4.0 * T + 4.0 * P, "byte", "hbm"  # + pair ids out
    # sort binning (DGS_BINNING=sort): loops cover the launched capacity
    if name == "sort":
        return 24.0 * cap, "byte", "hbm"     # 2 passes x (read + write) x (2-B key + 4-B id)
    if name == "duplicate":
        return 20.0 * N + 12.0 * cap, "byte", "hbm"  # + all-ones key fill of the tail
    if name == "ranges":
        return 8.0 * cap, "byte", "hbm"
    if name == "ssim_fwd":
        return 3 * HW * (4 + 4 + 12), "byte", "hbm"
    if name == "ssim_bwd":
        return 3 * HW * (4 + 4 + 12 + 4), "byte", "hbm"
    return None


KERNEL_CLASSES = ["mlp_fwd", "mlp_bwd", "mlp_dw", "mlp_dw_reduce", "mlp_tgrad", "preprocess_fwd", "depth_sort", "count", "scan",
                  "place", "tile_sort", "duplicate", "sort", "ranges",
                  "blend_fwd", "blend_bwd", "blend_gather", "preprocess_bwd", "ssim_fwd", "ssim_bwd", "inputs_fwd", "inputs_bwd", "adam"]


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_baseline(N, res, steps, warmup=3):
    """SURVEY.md 8d's CPU column: the build's CPU restatement of the same step on the host — the
    reference's own torch forward of DeformNetworkBaseline (deform_network.glue_forward: PE by cat of
    sin / cos bands, timenet, 8 x Linear + ReLU with the skip, heads; fp32, autograd backward) + the C
    raster oracle (oracle/raster_ref.c: OpenMP forward and OpenMP backward over fixed tile chunks) + the
    reference's torch-CPU L1 / SSIM; `warmup` untimed then `steps` timed full steps (median)."""
    from deformgs.deform_network import DeformNetworkBaseline
    from deformgs.loss import l1_loss, ssim
    from deformgs.synthetic import synth_camera, synth_gaussians
    threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    from oracle.raster import OracleRaster, make_settings
    torch.set_num_threads(threads)
    g = synth_gaussians(N, seed=0, device="cpu")
    cam = synth_camera(res, res, index=0, fid=0.5, device="cpu")
    torch.manual_seed(0)
    net = DeformNetworkBaseline(is_blender=True)
    with torch.no_grad():  # same steady-state head scale as the GPU run
        for head in (net.gaussian_warp, net.gaussian_rotation, net.gaussian_scaling):
            head.weight.mul_(0.01)
            head.bias.mul_(0.01)
    gt = torch.rand((3, res, res), generator=torch.Generator().manual_seed(7))
    s = make_settings(res, res, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), [0, 0, 0], 1.0,
                      cam.world_view_transform.numpy(), cam.full_proj_transform.numpy(), 3, cam.camera_center.numpy())
    xyz = g["xyz"]
    shs = torch.cat([g["features_dc"], g["features_rest"]], 1).numpy()
    sc = torch.exp(g["scaling"])
    rq = torch.nn.functional.normalize(g["rotation"])
    op = torch.sigmoid(g["opacity"]).numpy()
    t = torch.full((N, 1), 0.5)
    times = []
    for it in range(warmup + steps):
        t0 = time.perf_counter()
        net.zero_grad(set_to_none=True)
        d_xyz, d_rot, d_scale = net.glue_forward(xyz, t)
        means = (xyz + d_xyz).detach().numpy()
        scales = (sc + d_scale).detach().numpy()
        rots = (rq + d_rot).detach().numpy()
        o = OracleRaster(s, means, shs=shs, opacities=op, scales=scales, rotations=rots)
        img = torch.from_numpy(o.color).requires_grad_(True)
        loss = 0.8 * l1_loss(img, gt) + 0.2 * (1.0 - ssim(img, gt))
        loss.backward()
        gr = o.backward(img.grad.numpy())
        torch.autograd.backward([d_xyz, d_rot, d_scale], [torch.from_numpy(gr[k]) for k in
                                                          ("means3D", "rotations", "scales")])
        if it >= warmup:
            times.append(time.perf_counter() - t0)
    return dict(value=1.0 / float(np.median(times)), unit="iters/s", cores=threads, kind="port",
                cpu=_cpu_model(),
                sample=f"median of {steps} timed full steps after {warmup} warm-up (SURVEY 8d protocol) of "
                       f"synth-{N // 1000}k at {res}x{res} on {threads} threads of {_cpu_model()}: fp32 torch-CPU "
                       f"DeformNetworkBaseline (the reference's forward, autograd backward) + C raster oracle "
                       f"(OpenMP forward and backward) + torch-CPU L1/SSIM; no Adam",
                median_s=float(np.median(times)), min_s=float(np.min(times)))


def main():
    # a launched rank takes the parent's arguments from DGS_BENCH_ARGV (launcher_cmd)
    args = parse(json.loads(os.environ[ARGV_ENV]) if "WORLD_SIZE" in os.environ and ARGV_ENV in os.environ else None)
    rc = maybe_launch(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    from deformgs import _lib
    from deformgs.dist import OverflowAgreement, OverlappedGradAllReduce, init_from_env
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import optimizer_step, train_step
    import torch.distributed as dist

    rank, world, local = init_from_env()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    N, R = args.n, args.res
    torch.manual_seed(0)
    g = synth_gaussians(N, seed=0, device=dev)
    gaussians = GaussianModel(3)
    gaussians.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    opt = OptimizationParams()
    gaussians.training_setup(opt)
    torch.manual_seed(0)
    six = args.six_dof
    deform = DeformModelBaseline(is_blender=True, is_6dof=six, device=dev)
    if not args.raw_init:
        # steady-state training: the learned deltas are small (O(1e-3)); scale the random heads so the
        # rasterizer sees the Gaussians' own footprint, as in every iteration after the first few
        net = deform.deform
        heads = (net.branch_w, net.branch_v) if six else (net.gaussian_warp,)
        with torch.no_grad():
            for head in heads + (net.gaussian_rotation, net.gaussian_scaling):
                head.weight.mul_(0.01)
                head.bias.mul_(0.01)
    deform.train_setting(opt)
    pipe = PipelineParams()
    bg = torch.zeros(3, device=dev)
    cams = [synth_camera(R, R, index=rank * 97 + k, fid=((rank * 97 + k) % 30) / 30.0, device=dev) for k in range(8)]
    # targets: each camera's initial render plus noise (sigma 0.02), i.e. a model near convergence as
    # in steady-state training; a random target would drag the Gaussians (and the pair count) along
    # during the run and make the workload depend on --steps
    from deformgs.renderer import render
    gts = []
    gen = torch.Generator(device=dev).manual_seed(100 + rank)
    with torch.no_grad():
        for cam in cams:
            d = deform.step(gaussians.get_xyz.detach(), cam.fid.unsqueeze(0).expand(N, -1))
            img = render(cam, gaussians, pipe, bg, d[0], d[1], d[2], six)["render"]
            gts.append((img + 0.02 * torch.randn(img.shape, device=dev, generator=gen)).clamp_(0.0, 1.0))
    # Gaussian gradients are all-reduced during the MLP backward (their hooks fire first), the MLP's after
    allreduce = OverlappedGradAllReduce(
        lambda: [gaussians._xyz, gaussians._features_dc, gaussians._features_rest, gaussians._scaling,
                 gaussians._rotation, gaussians._opacity],
        lambda: list(deform.deform.parameters()))
    agreement = OverflowAgreement()

    state = {"it": 3000, "P": 0, "redos": 0, "host_fb": 0.0, "host_opt": 0.0}

    def step(k):
        cam = cams[k % len(cams)]
        h0 = time.perf_counter()
        # the rasterizer does not wait for the pair count (the host keeps issuing); a step whose
        # speculative pair capacity overflowed on any rank is redone synchronously on every rank
        # (OverflowAgreement: a 1-int host all-reduce), before the gradients are used
        loss, pkg, redone = train_step(gaussians, deform, cam, gts[k % len(cams)], pipe, bg, six,
                                       deferred_count=not SYNC_COUNT, allreduce=allreduce, agreement=agreement)
        state["redos"] += int(redone)
        h1 = time.perf_counter()
        if not args.no_adam:
            optimizer_step(gaussians, deform, state["it"])
        state["host_fb"] += h1 - h0
        state["host_opt"] += time.perf_counter() - h1
        state["it"] += 1

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    lib.dgs_timing_reset()
    lib.dgs_timing_select({"roofline": b"mlp_fwd,mlp_bwd,mlp_dw", "major": b"mlp_fwd,mlp_bwd,mlp_dw,blend_fwd,blend_bwd",
                           "all": b"", "none": b""}[args.kernel_timing])
    # the roofline candidates are timed on every 8th step (each timed launch adds two stream markers, ~6 us
    # of GPU idle each, inside the timed region: 28 us per timed step, profiles/r5y2 trace), every 4th on
    # shorter runs; the other classes, when asked for, on every step. The roofline reports the timed class
    # with the longest average launch (the dominant kernel)
    period = (8 if args.steps >= 16 else 4 if args.steps >= 8 else 1) if args.kernel_timing == "roofline" else 1
    lib.dgs_timing_sample(period)
    lib.dgs_timing_enable(0 if args.kernel_timing == "none" else 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    state["host_fb"] = state["host_opt"] = 0.0
    waits = ctypes.c_longlong(0)
    wait0 = lib.dgs_debug_count_wait_ns(waits)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0  # this rank's own steps, before waiting for the others
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    wait_ms = (lib.dgs_debug_count_wait_ns(waits) - wait0) / 1e6
    lib.dgs_timing_enable(0)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    # per rank: its own timed span, the wait for the slowest rank at the closing barrier (imbalance
    # plus collective waits the stream dependencies pushed to the end), the host's pair-count wait and
    # forward / backward issue time, and the world size it saw
    mine = torch.tensor([rank, world, t_local * 1e3 / args.steps, (elapsed - t_local) * 1e3 / args.steps,
                         wait_ms / args.steps, state["host_fb"] * 1e3 / args.steps, state["redos"]],
                        dtype=torch.float64, device=dev)
    per_rank = [mine]
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        per_rank = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
    elapsed = float(el.item())
    ranks_info = [{"rank": int(v[0]), "world_seen": int(v[1]), "own_ms_per_step": float(v[2]),
                   "barrier_wait_ms_per_step": float(v[3]), "count_wait_ms_per_step": float(v[4]),
                   "host_fwd_bwd_ms_per_step": float(v[5]), "redone_steps": int(v[6])}
                  for v in (t.cpu() for t in per_rank)]

    # pair count of one render (for the raster rooflines), measured once outside the timed region
    with torch.no_grad():
        d = deform.step(gaussians.get_xyz.detach(), cams[0].fid.unsqueeze(0).expand(N, -1))
    import diff_gaussian_rasterization as dgr
    # count pairs: rerun one forward through the autograd function to read ctx.num_rendered
    pk = render(cams[0], gaussians, pipe, bg, d[0], d[1], d[2], six)
    P_pairs = int(pk["render"].grad_fn.num_rendered) if hasattr(pk["render"].grad_fn, "num_rendered") else 0
    del pk
    pair_cap = int(lib.dgs_debug_pair_cap(local))  # the speculative capacity the sort-path loops cover
    n_tiles = -(-R // 16) * -(-R // 16)

    # per class: accumulated ms over the timed launches, how many were timed, how many ran (the
    # roofline candidates are timed on every `period`-th launch)
    kernels = {}
    for name in KERNEL_CLASSES:
        n_l = _lib.I(0)
        ms = lib.dgs_timing_query(name.encode(), n_l)
        if n_l.value:
            kernels[name] = (ms, n_l.value, int(lib.dgs_timing_launches(name.encode())))
    HW = R * R
    best = None
    for name, (ms, n, _) in kernels.items():
        info = kernel_algorithmic(name, N, P_pairs, HW, cap=pair_cap, T=n_tiles)
        if info is None:
            continue
        if best is None or ms / n > best[1] / best[2]:  # the longest AVERAGE launch: the dominant kernel
            best = (name, ms, n, info)
    roofline = None
    if best:
        name, ms, n, (amount, unit, bound) = best
        avg_s = ms / 1000.0 / n
        if bound == "mfma":
            # the MLP kernels move ~1-2 GB per launch beside their FLOPs: their roofline is the larger of
            # the MFMA time and the HBM time of their algorithmic bytes (attainable = min(peak, AI x BW));
            # frac = that ideal time / the measured launch
            peak, arith = mfma_peak(name)
            nbytes = mlp_bytes(name, N)
            t_flop = amount / (peak * 1e12)
            t_hbm = nbytes / (HBM_PEAK_GBS * 1e9) if nbytes else 0.0
            if t_hbm > t_flop:
                roofline = {"bound": "hbm", "kernel": name, "achieved": nbytes / avg_s / 1e9, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": t_hbm / avg_s, "traffic": None, "algorithmic_bytes": nbytes,
                            "mfma": {"achieved_tflops": amount / avg_s / 1e12, "peak_tflops": peak,
                                     "peak_basis": arith, "frac": t_flop / avg_s},
                            "avg_launch_ms": avg_s * 1e3, "launches": n}
            else:
                roofline = {"bound": "mfma", "kernel": name, "achieved": amount / avg_s / 1e12, "peak": peak,
                            "peak_basis": arith, "unit": "TFLOP/s", "frac": t_flop / avg_s, "traffic": None,
                            "hbm": {"algorithmic_bytes": nbytes, "achieved_gbs": (nbytes or 0) / avg_s / 1e9,
                                    "frac": t_hbm / avg_s},
                            "avg_launch_ms": avg_s * 1e3, "launches": n}
        else:
            achieved = amount / avg_s / 1e9
            roofline = {"bound": "hbm", "kernel": name, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None, "avg_launch_ms": avg_s * 1e3,
                        "launches": n}
    if roofline is not None and os.path.exists(PMC_TRAFFIC):
        # HBM bytes per launch of the same kernel from the committed rocprofv3 --pmc passes
        # (FETCH_SIZE doubled for gfx950 + WRITE_SIZE; tools/gpu_prof.sh, tools/pmc_traffic.py)
        try:
            t = json.load(open(PMC_TRAFFIC)).get(roofline["kernel"])
            if t:
                roofline["traffic"] = t["traffic_bytes"]
                roofline["traffic_source"] = "profiles/pmc_traffic.json (" + t.get("source", "?") + ")"
        except (OSError, ValueError, KeyError):
            pass
    value = world * args.steps / elapsed
    step_s = elapsed / args.steps
    if roofline is not None:
        # SURVEY.md 8d's step-level figure: (MLP FLOPs / MFMA peak + raster bytes / HBM peak) / step time,
        # on both MFMA bases (the split-f16 GEMMs' ceiling and the native fp32 MFMA peak)
        mlp_flop = 2.0 * (MLP_FWD_MAC + MLP_DX_MAC + MLP_DW_MAC) * N
        raster_bytes = 1000.0 * N + 132.0 * P_pairs + 48.0 * HW
        roofline["step"] = {
            "mlp_flop": mlp_flop, "raster_bytes": raster_bytes, "step_ms": step_s * 1e3,
            "frac_split_basis": (mlp_flop / (SPLIT_MFMA_PEAK_TFLOPS * 1e12) + raster_bytes / (HBM_PEAK_GBS * 1e9)) / step_s,
            "frac_fp32_basis": (mlp_flop / (FP32_MFMA_PEAK_TFLOPS * 1e12) + raster_bytes / (HBM_PEAK_GBS * 1e9)) / step_s,
            "note": "kernel frac is vs the split-f16 ceiling (2.5 PF f16 / 3); vs the 157.3 TF fp32 MFMA peak the "
                    "split kernels can exceed 1 (three f16 products per fp32 product at 16x the fp32 rate)"}
    scene = "synth-100k" if N == 100_000 else f"synth-{N // 1000}k (the synth-100k protocol at {N} Gaussians)"
    result = {
        "metric": f"train iters/s (deform+raster fwd+bwd), {N // 1000}k Gaussians @ {R}x{R}",
        "value": value, "unit": "iters/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": f"synthetic ({scene}, random-init weights, targets = initial renders + noise)",
        "config": {"workload": f"{scene}: {N} Gaussians, {R}x{R}, blender DeformNetworkBaseline"
                   + (" (6-DoF screw head)" if six else "") + ", SH3"
                   + (" (raw-init heads)" if args.raw_init else " (heads at 1/100 init: steady-state deltas)"),
                   "global_batch": world, "includes_adam": not args.no_adam, "pairs_per_render": P_pairs,
                   "pair_capacity": pair_cap, "redone_steps": state["redos"],
                   "parallelism": "dp1 (one rank, no collective)" if world == 1 else
                   f"dp{world} (frame-parallel, "
                   + ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend()) + " grad all-reduce)"},
        "roofline": roofline,
        # average timed launch x launches per step (every launch ran, every `period`-th was timed)
        "kernels_ms_per_step": {k: v[0] / v[1] * v[2] / args.steps for k, v in kernels.items()},
        "kernel_timing": {"period": period, "timed_launches": {k: v[1] for k, v in kernels.items()},
                          "launches": {k: v[2] for k, v in kernels.items()}},
        # host time per step: issuing forward + backward (including the wait for the pair count
        # inside it) and the optimizer step; a count wait near 0 means the host, not the GPU, paced it
        "host_ms_per_step": {"fwd_bwd": state["host_fb"] / args.steps * 1e3, "count_wait": wait_ms / args.steps,
                             "optimizer": state["host_opt"] / args.steps * 1e3},
        "cpu_baseline": None,
        "dist": {"world_size": world, "backend": dist.get_backend() if world > 1 else None,
                 "ranks": ranks_info},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(N, R, args.cpu_steps, args.cpu_warmup)
        except Exception as e:  # report, never hide
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

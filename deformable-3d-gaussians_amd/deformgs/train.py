"""Training loop — train_baseline.py:34-184 on the MI355X path (SURVEY.md §8a H1 + H2, §8e).

`training()` keeps the reference's per-iteration order (file:line in train_baseline.py):
  :76-77   oneupSHdegree every 1000 iterations
  :80-100  viewpoint stack: the train cameras sorted by fid, `sequence_length` uniformly spaced
           frames (int(round(i * step))), random pops (random.randint), refilled when empty;
           time_interval = 1 / len(stack) taken before the pop
  :106-115 warm-up (iteration < warm_up): deltas 0.0 (no deformation); after it deform.step on the
           detached xyz with fid + ast_noise (non-blender: randn(1,1) * time_interval * smooth_term)
  :119-128 render -> (1 - l) L1 + l (1 - SSIM) -> backward
  :145-146 max_radii2D = max(max_radii2D, radii) over the visible Gaussians
  :162-173 densification statistics from viewspace_points_densify; densify_and_prune every
           densification_interval in (densify_from_iter, densify_until_iter) with size threshold 20
           after the first opacity reset; reset_opacity every opacity_reset_interval (and at
           densify_from_iter on a white background)
  :175-182 Adam on the Gaussians, xyz LR, Adam on the deformation network, zero_grad, deform LR —
           for iteration < iterations (on a densify iteration the replaced Gaussian tensors carry no
           gradient and keep their values, as upstream)
  :210-267 training_report: L1 / PSNR over the test cameras at testing_iterations
  :157-160 saving: point_cloud/iteration_k/point_cloud.ply and deform/iteration_k/deform.pth

fused=True (the product): fused MLP, fused render inputs, split-SH HIP rasterizer, fused L1+SSIM,
one-launch Adam over both optimizers, one-launch densification compaction, deferred pair count.
fused=False: the same loop through the reference's torch glue (the network's torch forward, render()'s
generic glue, torch L1/SSIM, torch.optim.Adam, boolean indexing) around the same HIP rasterizer — the
comparison path of tests/test_gpu_train.py.

Frame parallelism (world > 1): every rank keeps the same (seeded) stack and pops
`world` cameras per iteration, rank r rendering the r-th; gradients are averaged by
OverlappedGradAllReduce, an overflowing deferred count is redone on every rank (OverflowAgreement),
densification statistics are summed / maxed right before densify_and_prune, and the split noise comes
from a rank-identical generator, so replicas stay identical.
"""
import os
import random
import time

import numpy as np
import torch

from .arguments import ModelParams, OptimizationParams, PipelineParams
from .deform_model import DeformModelBaseline
from .dist import OverflowAgreement, OverlappedGradAllReduce, rank_identical_generator, sync_densification_stats
from .general import get_linear_noise_func
from .loss import l1_loss, psnr, ssim
from .renderer import render, set_fused
from .train_step import optimizer_step, reset_agreement, train_step


def build_viewpoint_stack(cameras, sequence_length):
    """train_baseline.py:80-89: cameras sorted by fid, `sequence_length` uniformly spaced indices."""
    stack = sorted(cameras, key=lambda c: float(c.fid))
    total = len(stack)
    step = (total - 1) / (sequence_length - 1)
    return [stack[int(round(i * step))] for i in range(sequence_length)]


def training_report(iteration, testing_iterations, test_cameras, train_cameras, gaussians, deform, pipe, background,
                    is_6dof, log=None):
    """train_baseline.py:210-267 without TensorBoard: test and train-sample L1 / PSNR."""
    if iteration not in testing_iterations:
        return None
    out = {}
    configs = (("test", test_cameras), ("train", [train_cameras[i % len(train_cameras)] for i in range(5, 30, 5)]))
    with torch.no_grad():
        for name, cams in configs:
            if not cams:
                continue
            images, gts = [], []
            for cam in cams:
                xyz = gaussians.get_xyz
                d_xyz, d_rot, d_scale = deform.step(xyz.detach(), cam.fid.unsqueeze(0).expand(xyz.shape[0], -1))
                img = render(cam, gaussians, pipe, background, d_xyz, d_rot, d_scale, is_6dof)["render"]
                images.append(torch.clamp(img, 0.0, 1.0))
                gts.append(torch.clamp(cam.original_image, 0.0, 1.0))
            images, gts = torch.stack(images), torch.stack(gts)
            out[name] = (float(l1_loss(images, gts)), float(psnr(images, gts).mean()))
            if log:
                log(f"[ITER {iteration}] Evaluating {name}: L1 {out[name][0]} PSNR {out[name][1]}")
    return out


def _glue_step(gaussians, deform, cam, gt, pipe, bg, is_6dof, lambda_dssim, warm, ast_noise):
    """train_baseline.py:104-128 through the reference's torch glue (comparison path)."""
    if not warm:
        d_xyz, d_rot, d_scale = 0.0, 0.0, 0.0
    else:
        N = gaussians.get_xyz.shape[0]
        t = cam.fid.unsqueeze(0).expand(N, -1) + ast_noise
        d_xyz, d_rot, d_scale = deform.deform.glue_forward(gaussians.get_xyz.detach(), t)
    pkg = render(cam, gaussians, pipe, bg, d_xyz, d_rot, d_scale, is_6dof)
    image = pkg["render"]
    Ll1 = l1_loss(image, gt)
    loss = (1.0 - lambda_dssim) * Ll1 + lambda_dssim * (1.0 - ssim(image, gt))
    loss.backward()
    return loss, pkg


def training(dataset, opt, pipe, testing_iterations, saving_iterations, scene, gaussians, deform=None, fused=True,
             deferred_count=True, seed=0, model_path=None, log=None, on_iteration=None):
    """Runs opt.iterations iterations on `scene` (scene.getTrainCameras() / getTestCameras() /
    cameras_extent, cameras carrying fid and original_image) and the GaussianModel `gaussians`
    (already initialised). Returns a history dict: per-iteration loss, Gaussian count and redo flag,
    training_report results, fwd+bwd milliseconds (iter_start..iter_end events, train_baseline.py:
    46-47,73,130) and the loop's wall time."""
    dev = gaussians.get_xyz.device
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    set_fused(fused)
    reset_agreement()  # this run agrees on its own native-vs-autograd path (train_step)
    try:
        torch_adam = None if fused else torch.optim.Adam
        gaussians.row_select = None if fused else (lambda mask, ts: [t[mask] for t in ts])
        if deform is None:
            deform = DeformModelBaseline(dataset.is_blender, dataset.is_6dof, device=dev)
        deform.train_setting(opt, optimizer_cls=torch_adam)
        gaussians.training_setup(opt, optimizer_cls=torch_adam)
        bg = torch.tensor([1, 1, 1] if dataset.white_background else [0, 0, 0], dtype=torch.float32, device=dev)
        rng = random.Random(seed)  # the reference's random.randint camera pops (rank-identical)
        noise_gen = torch.Generator(device=dev).manual_seed(seed + 1 + rank)
        split_gen = rank_identical_generator(dev, seed + 2)
        smooth_term = get_linear_noise_func(lr_init=0.1, lr_final=1e-15, lr_delay_mult=0.01, max_steps=20000)
        allreduce = agreement = None
        if world > 1:
            allreduce = OverlappedGradAllReduce(
                lambda: [gaussians._xyz, gaussians._features_dc, gaussians._features_rest, gaussians._scaling,
                         gaussians._rotation, gaussians._opacity],
                lambda: list(deform.deform.parameters()))
            agreement = OverflowAgreement()
        hist = dict(loss=[], n=[], redone=[], report={}, iter_ms=[])
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stack = None
        t_start = time.perf_counter()
        for iteration in range(1, opt.iterations + 1):
            if iteration % 1000 == 0:
                gaussians.oneupSHdegree()
            picked = []
            for _ in range(world):  # the global batch: one camera per rank
                if not stack:
                    stack = build_viewpoint_stack(scene.getTrainCameras(), opt.sequence_length)
                total_frame = len(stack)
                picked.append((stack.pop(rng.randint(0, len(stack) - 1)), 1.0 / total_frame))
            cam, time_interval = picked[rank]
            warm = iteration >= opt.warm_up
            ast_noise = 0.0
            if warm and not dataset.is_blender:
                ast_noise = (torch.randn(1, 1, device=dev, generator=noise_gen) * time_interval
                             * float(smooth_term(iteration)))
            gt = cam.original_image
            ev0.record()
            if fused:
                loss, pkg, redone = train_step(gaussians, deform, cam, gt, pipe, bg, dataset.is_6dof, opt.lambda_dssim,
                                               warm, ast_noise, deferred_count=deferred_count, allreduce=allreduce,
                                               agreement=agreement)
            else:
                if allreduce is not None:
                    allreduce.arm()
                loss, pkg = _glue_step(gaussians, deform, cam, gt, pipe, bg, dataset.is_6dof, opt.lambda_dssim, warm,
                                       ast_noise)
                if allreduce is not None:
                    allreduce()
                redone = False
            ev1.record()
            with torch.no_grad():
                vis, radii = pkg["visibility_filter"], pkg["radii"]
                # train_baseline.py:145-146 (max over the visible Gaussians; one select, no index kernels)
                gaussians.max_radii2D = torch.where(vis, torch.maximum(gaussians.max_radii2D, radii.float()),
                                                    gaussians.max_radii2D)
                rep = training_report(iteration, testing_iterations, scene.getTestCameras(), scene.getTrainCameras(),
                                      gaussians, deform, pipe, bg, dataset.is_6dof, log)
                if rep is not None:
                    hist["report"][iteration] = rep
                if iteration in saving_iterations and model_path and rank == 0:
                    gaussians.save_ply(os.path.join(model_path, "point_cloud", f"iteration_{iteration}",
                                                    "point_cloud.ply"))
                    deform.save_weights(model_path, iteration)
                if iteration < opt.densify_until_iter:
                    gaussians.add_densification_stats(pkg["viewspace_points_densify"], vis)
                    if iteration > opt.densify_from_iter and iteration % opt.densification_interval == 0:
                        size_threshold = 20 if iteration > opt.opacity_reset_interval else None
                        if world > 1:
                            sync_densification_stats(gaussians)
                        gaussians.densify_and_prune(opt.densify_grad_threshold, 0.005, scene.cameras_extent,
                                                    size_threshold, generator=split_gen)
                    if iteration % opt.opacity_reset_interval == 0 or (
                            dataset.white_background and iteration == opt.densify_from_iter):
                        gaussians.reset_opacity()
                if iteration < opt.iterations:
                    if fused:
                        optimizer_step(gaussians, deform, iteration)
                    else:
                        gaussians.optimizer.step()
                        gaussians.update_learning_rate(iteration)
                        deform.optimizer.step()
                        gaussians.optimizer.zero_grad(set_to_none=True)
                        deform.optimizer.zero_grad()
                        deform.update_learning_rate(iteration)
            hist["loss"].append(loss.detach())
            hist["n"].append(gaussians.get_xyz.shape[0])
            hist["redone"].append(redone)
            hist["iter_ms"].append((ev0, ev1))
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if on_iteration is not None:
                on_iteration(iteration, gaussians, deform)
        torch.cuda.synchronize(dev)
        hist["wall_s"] = time.perf_counter() - t_start
        hist["loss"] = [float(v) for v in torch.stack(hist["loss"]).cpu()] if hist["loss"] else []
        hist["iter_ms"] = [a.elapsed_time(b) for a, b in hist["iter_ms"]]
        hist["deform"] = deform
        return hist
    finally:
        set_fused(True)
        gaussians.row_select = None
        # the one-launch Adam's cached tables refer to the optimizers' groups: drop them with the loop
        from .adam import clear_fast_cache
        clear_fast_cache(getattr(gaussians, "optimizer", None), getattr(deform, "optimizer", None))


class SyntheticScene:
    """Stand-in for scene.Scene (scene/__init__.py:23-112) on synthetic data (the D-NeRF / NeRF-DS
    datasets are not available here): `n_train` train and `n_test` test cameras around the object, each
    holding `original_image` = a render of a ground-truth deformable model, so the loop has a real
    target to converge to. cameras_extent = 1.1 x the largest camera distance from the mean camera
    centre (dataset_readers.py:77-98 getNerfppNorm). init_gaussians(model) seeds the trained model from
    a perturbed copy of the ground truth's positions (the reader's random point cloud,
    dataset_readers.py:286-290, stands behind the same role).

    motion="smooth" (default): the ground truth deforms by a displacement FIELD that is smooth in
    position and time, d(x, t) = a (sin(2 pi t + w x_y + p0), sin(2 pi t + w x_z + p1), sin(2 pi t + w
    x_x + p2)) — a D-NeRF-like scene that a deformation network can learn and interpolate; "random":
    every Gaussian follows its own random sinusoid (round-3 behaviour: memorisable per frame only).
    interleave=True (default): train frames take fids k/n_train on the camera ring and every test
    camera sits between two train cameras, at the midpoint of their azimuths and of their frame times,
    so the test views measure interpolation in view and time (the D-NeRF split's held-out role);
    False: test cameras continue the train ring (round-3 behaviour)."""

    def __init__(self, n_gaussians, width, height, n_train=30, n_test=5, seed=0, device="cuda", motion="smooth",
                 amplitude=0.08, white_background=False, interleave=True):
        from .arguments import PipelineParams as _PP
        from .gaussian_model import GaussianModel
        from .synthetic import synth_camera, synth_gaussians
        self.device = torch.device(device)
        g = synth_gaussians(n_gaussians, seed=seed, device=device)
        self.gt_tensors = g
        gt = GaussianModel(3)
        gt.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
        rng = np.random.default_rng(seed + 100)
        self.kind = motion
        if motion == "random":
            self.dirs = torch.tensor(rng.standard_normal((n_gaussians, 3)), dtype=torch.float32,
                                     device=device) * amplitude
            self.phase = torch.tensor(rng.uniform(0, 2 * np.pi, (n_gaussians, 1)), dtype=torch.float32, device=device)
        elif motion == "smooth":
            self.amp = float(amplitude)
            self.freq = 2.0
            self.phases = [float(v) for v in rng.uniform(0, 2 * np.pi, 3)]
        else:
            raise ValueError(motion)
        bg = torch.tensor([1.0, 1.0, 1.0] if white_background else [0.0, 0.0, 0.0], device=device)
        self.train, self.test = [], []
        specs = []
        if interleave:
            az = [2 * np.pi * k / n_train for k in range(n_train)]
            el = [0.25 * np.sin(0.7 * k) for k in range(n_train)]
            fids = [k / n_train for k in range(n_train)]
            specs += [(az[k], el[k], fids[k]) for k in range(n_train)]
            for j in range(n_test):
                k = (j * n_train) // max(n_test, 1) + n_train // (2 * max(n_test, 1))
                k1 = (k + 1) % n_train
                specs.append((az[k] + np.pi / n_train, 0.5 * (el[k] + el[k1]), (k + 0.5) / n_train))
        else:
            for k in range(n_train + n_test):
                specs.append((None, None, (k * 0.618033988749895) % 1.0, k))
        for k, sp in enumerate(specs):
            if interleave:
                cam = synth_camera(width, height, fid=float(sp[2]), device=device, az=float(sp[0]), el=float(sp[1]))
            else:
                cam = synth_camera(width, height, index=sp[3], fid=sp[2], device=device)
            with torch.no_grad():
                d_xyz = self.motion(float(cam.fid))
                img = render(cam, gt, _PP(), bg, d_xyz, 0.0, 0.0)["render"]
            cam.original_image = img.clamp(0.0, 1.0)
            (self.train if k < n_train else self.test).append(cam)
        centers = np.stack([c.camera_center.cpu().numpy() for c in self.train])
        self.cameras_extent = float(np.max(np.linalg.norm(centers - centers.mean(0), axis=1)) * 1.1)

    def motion(self, fid):
        if self.kind == "random":
            return self.dirs * torch.sin(2 * np.pi * fid + self.phase)
        x = self.gt_tensors["xyz"]
        w, p = self.freq, self.phases
        ph = 2 * np.pi * fid
        return self.amp * torch.stack([torch.sin(ph + w * x[:, 1] + p[0]), torch.sin(ph + w * x[:, 2] + p[1]),
                                       torch.sin(ph + w * x[:, 0] + p[2])], 1)

    def getTrainCameras(self):
        return self.train

    def getTestCameras(self):
        return self.test

    def init_gaussians(self, gaussians, seed=1, jitter=0.02):
        g = self.gt_tensors
        gen = torch.Generator(device=self.device).manual_seed(seed)
        xyz = g["xyz"] + jitter * torch.randn(g["xyz"].shape, device=self.device, generator=gen)
        fdc = g["features_dc"] + 0.1 * torch.randn(g["features_dc"].shape, device=self.device, generator=gen)
        gaussians.from_tensors(xyz, fdc, torch.zeros_like(g["features_rest"]), g["scaling"] + 0.2, g["rotation"],
                               torch.zeros_like(g["opacity"]) - 2.0, active_sh_degree=0)
        return gaussians


def main(argv=None):
    """Synthetic-scene training run with the reference's defaults (config 3: a full train loop);
    prints one JSON line: iters/s over the whole loop (densification, reports and Adam included), the
    reference's fwd+bwd span per iteration, the final Gaussian count and the test PSNR."""
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=55_000)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--iterations", type=int, default=3000)
    ap.add_argument("--warm-up", type=int, default=None)
    ap.add_argument("--densify-from", type=int, default=None)
    ap.add_argument("--densify-interval", type=int, default=None)
    ap.add_argument("--opacity-reset", type=int, default=None)
    ap.add_argument("--sequence-length", type=int, default=30)
    ap.add_argument("--non-blender", action="store_true")
    ap.add_argument("--6dof", dest="six_dof", action="store_true")
    ap.add_argument("--test-every", type=int, default=0)
    ap.add_argument("--no-deferred", action="store_true")
    args = ap.parse_args(argv)
    from .dist import init_from_env
    from .gaussian_model import GaussianModel
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    kw = dict(iterations=args.iterations, sequence_length=args.sequence_length)
    for k, v in (("warm_up", args.warm_up), ("densify_from_iter", args.densify_from),
                 ("densification_interval", args.densify_interval), ("opacity_reset_interval", args.opacity_reset)):
        if v is not None:
            kw[k] = v
    opt = OptimizationParams(**kw)
    dataset = ModelParams(is_blender=not args.non_blender, is_6dof=args.six_dof)
    scene = SyntheticScene(args.n, args.res, args.res, device=dev)
    g = scene.init_gaussians(GaussianModel(3))
    tests = list(range(args.test_every, args.iterations + 1, args.test_every)) if args.test_every else [args.iterations]
    torch.manual_seed(0)
    hist = training(dataset, opt, PipelineParams(), tests, [], scene, g, deferred_count=not args.no_deferred,
                    log=(lambda s: print(s, flush=True)) if rank == 0 else None)
    fb = float(np.median(hist["iter_ms"])) if hist["iter_ms"] else 0.0
    out = {"metric": f"train iters/s (full loop: densify + Adam + reports), {args.n} Gaussians init @ "
                     f"{args.res}x{args.res}", "value": args.iterations * world / hist["wall_s"], "unit": "iters/s",
           "n_gpus": world, "iterations": args.iterations, "fwd_bwd_ms_median": fb,
           "final_gaussians": hist["n"][-1], "redone_iterations": int(sum(hist["redone"])),
           "report": {str(k): v for k, v in hist["report"].items()}, "final_loss": hist["loss"][-1]}
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""One training iteration of train_baseline.py:104-182 on the HIP path (shared by bench.py and the
harness): deform -> render -> 0.8*L1 + 0.2*(1-SSIM) -> backward [-> grad all-reduce] -> Adam.
"""
import torch
import torch.distributed as dist

import diff_gaussian_rasterization as dgr

from . import _lib, native_step
from .adam import step_all
from .loss import l1_ssim_loss
from .renderer import render


_DEFER = {"before": 0}


def forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof=False, lambda_dssim=0.2,
                     warm=True, ast_noise=0.0, deferred_count=False, rank_agreed=False):
    """train_baseline.py:104-128 (timed span of the reference's iter_start/iter_end events).

    deferred_count: the rasterizer does not wait for num_rendered in the forward nor in the backward
    (the host keeps issuing the loss and the whole backward; the count is read once that is queued);
    if the speculative pair capacity overflowed, `deferred_overflowed()`
    is True afterwards and the caller must redo the step with deferred_count=False after dropping
    the gradients (`drop_grads`). With several ranks the redo must be agreed on by every rank before
    the gradients are used (`train_step` does it with dist.OverflowAgreement): a multi-rank caller
    must pass rank_agreed=True to promise that, else this raises."""
    if deferred_count and not rank_agreed and dist.is_initialized() and dist.get_world_size() > 1:
        raise RuntimeError("forward_backward(deferred_count=True) with several ranks needs a rank agreement on "
                           "overflow redos (use train_step(), or pass rank_agreed=True after arranging one)")
    if not deferred_count:
        return _forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof, lambda_dssim, warm,
                                 ast_noise)
    lib = _lib.load()
    _DEFER["before"] = lib.dgs_raster_deferred_overflows()
    lib.dgs_raster_set_deferred_count(1)
    # the raster backward neither waits for the pair count nor frees its context: the host issues the
    # whole backward (render inputs, MLP dX, dW) first and resolves the count here, at the end
    dgr._KEEP_CTX["on"] = True
    pkg = None
    try:
        loss, pkg = _forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof, lambda_dssim,
                                      warm, ast_noise)
        return loss, pkg
    finally:
        dgr._KEEP_CTX["on"] = False
        if pkg is not None:
            dgr.release_context(pkg["render"])
        lib.dgs_raster_set_deferred_count(0)


def train_step(gaussians, deform, cam, gt_image, pipe, background, is_6dof=False, lambda_dssim=0.2, warm=True,
               ast_noise=0.0, deferred_count=True, allreduce=None, agreement=None):
    """One iteration's compute up to the optimizer. On render()'s fused training path it runs as one C
    call (native_step.NativeStep: dgs_train_step, the same kernels in the same order as
    forward_backward, without the autograd engine; DGS_NATIVE_STEP=0 keeps forward_backward), or, with
    several ranks, two calls around the overlapped Gaussian gradient all-reduce (step_data_parallel: an
    overflowed pair count is redone by its rank alone, no agreement);
    otherwise forward_backward (deferred pair count unless deferred_count=False), the synchronous redo of a step whose speculative pair capacity overflowed
    (agreed across ranks by `agreement`, a dist.OverflowAgreement, when world > 1), and the gradient
    all-reduce (`allreduce`, an armed dist.OverlappedGradAllReduce, when world > 1).
    Returns (loss, render package, redone)."""
    multi = allreduce is not None and allreduce.world() > 1
    single = not dist.is_initialized() or dist.get_world_size() == 1
    if multi and gt_image.is_cuda and not gt_image.is_contiguous():
        gt_image = gt_image.contiguous()  # a per-step input: never a reason for ranks to take different paths
    local = (multi or single) and getattr(deform.deform, "is_6dof", False) == bool(is_6dof) and \
        native_step.usable(gaussians, deform, pipe, gt_image)
    if multi:
        local = agreed_native_path(local, gaussians, deform, pipe, gt_image, is_6dof, allreduce.group)
    if local:
        # one C call per step (dgs_train_step): no autograd engine, no per-step allocations but the
        # image and the loss (deformgs/native_step.py); several ranks: two calls around the
        # Gaussian gradient all-reduce
        ns = getattr(gaussians, "_dgs_native", None)
        if ns is None or ns.deform is not deform:
            ns = gaussians._dgs_native = native_step.NativeStep(gaussians, deform)
        if multi:
            return ns.step_data_parallel(cam, gt_image, background, warm, ast_noise, lambda_dssim, deferred_count,
                                         agreement, allreduce.group)
        loss, pkg, over = ns(cam, gt_image, background, warm, ast_noise, lambda_dssim, deferred_count)
        if deferred_count and over:
            loss, pkg, _ = ns(cam, gt_image, background, warm, ast_noise, lambda_dssim, False)
        return loss, pkg, bool(deferred_count and over)
    if multi and deferred_count and agreement is None:
        raise RuntimeError("train_step: several ranks with the deferred pair count need an OverflowAgreement")
    if multi:
        allreduce.arm()
    loss, pkg = forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof, lambda_dssim, warm,
                                 ast_noise, deferred_count=deferred_count, rank_agreed=multi)
    redone = False
    if deferred_count:
        over = deferred_overflowed()
        if multi:
            over = agreement(over)
        if over:
            redone = True
            if multi:
                allreduce.discard()
            drop_grads(gaussians, deform)
            if multi:
                allreduce.arm()
            loss, pkg = forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof, lambda_dssim,
                                         warm, ast_noise, deferred_count=False)
    if multi:
        allreduce()
    return loss, pkg, redone


_AGREED = {"key": None, "native": None}


def reset_agreement():
    """Forget the agreed native-vs-autograd choice: called when a process group or a training run
    starts (dist.init_from_env, train.training), so a later run never reuses a decision taken under
    another group or model."""
    _AGREED["key"] = _AGREED["native"] = None


def agreed_native_path(local, gaussians, deform, pipe, gt_image, is_6dof, group=None):
    """The native-vs-autograd choice of a data-parallel step, the same on every rank (the two paths
    issue different collectives: ranks split between them would hang in RCCL or fail in gloo).

    The ranks MIN-reduce their local `native_step.usable` flag whenever a RANK-INVARIANT key changes —
    the process group, the Gaussian count, the network's configuration, the pipe / renderer switches,
    the SH layout — so every rank issues that 1-int collective at the same step; between such changes
    the agreed choice is reused with no collective. The image size is NOT part of the key: each rank
    renders its own camera, and the reference's readers allow a different width / height per camera
    (scene/dataset_readers.py:113-114), so it can change on one rank and not on the others; usable()
    does not depend on it. A rank that cannot take an agreed native path without a key change (a
    condition only it sees, e.g. a misaligned parameter) raises; the other ranks then block in their next
    collective until the backend's timeout (no process-group abort is attempted). A rank that could but
    the others cannot simply takes the autograd path."""
    from .renderer import _FUSED, _HONOR_OVERRIDE, _SPLIT_SH
    net = deform.deform
    key = (id(group), int(gaussians._xyz.shape[0]), bool(is_6dof), getattr(net, "flags", None),
           bool(getattr(net, "exact_fp32", False)), native_step.enabled(), bool(_FUSED["on"]), bool(_SPLIT_SH),
           bool(_HONOR_OVERRIDE["on"]), bool(getattr(pipe, "compute_cov3D_python", False)),
           bool(getattr(pipe, "convert_SHs_python", False)), bool(getattr(pipe, "debug", False)),
           int(gaussians._features_rest.shape[1]))
    if key != _AGREED["key"]:
        dev = gt_image.device if (gt_image.is_cuda and dist.get_backend(group) == "nccl") else "cpu"
        flag = torch.tensor([1 if local else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        _AGREED["key"], _AGREED["native"] = key, bool(flag.item())
    if _AGREED["native"] and not local:
        raise RuntimeError(f"rank {dist.get_rank()}: the native training step is not usable on this rank while the "
                           "ranks agreed on it (a rank-local condition changed without a change of the Gaussian "
                           "count / configuration): the ranks' collectives would not match; the other ranks "
                           "block in their next collective until the backend's timeout")
    return _AGREED["native"]


def deferred_overflowed():
    """The last deferred_count step overflowed its speculative pair capacity (redo it)."""
    return _lib.load().dgs_raster_deferred_overflows() != _DEFER["before"]


def drop_grads(gaussians, deform):
    """Gradients of a step that is being redone."""
    gaussians.optimizer.zero_grad(set_to_none=True)
    deform.optimizer.zero_grad(set_to_none=True)


def _forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof, lambda_dssim, warm, ast_noise):
    if not warm:
        d_xyz, d_rotation, d_scaling = 0.0, 0.0, 0.0
    else:
        N = gaussians.get_xyz.shape[0]
        # time_input = fid.unsqueeze(0).expand(N, -1) + ast_noise (train_baseline.py:107-110); the noise
        # is one value per iteration (randn(1, 1).expand), so it is added before the expand and the
        # network sees a stride-0 time column (one frame time: DGS_MLP_UNIFORM_T)
        t = cam.fid.unsqueeze(0)
        if torch.is_tensor(ast_noise) or ast_noise != 0.0:
            t = t + (ast_noise.reshape(-1)[:1].reshape(1, 1) if torch.is_tensor(ast_noise) else ast_noise)
        time_input = t.expand(N, -1)
        d_xyz, d_rotation, d_scaling = deform.step(gaussians.get_xyz.detach(), time_input)
    pkg = render(cam, gaussians, pipe, background, d_xyz, d_rotation, d_scaling, is_6dof)
    image = pkg["render"]
    # (1-l)*l1_loss(image, gt) + l*(1-ssim(image, gt)) (train_baseline.py:126-127), fused HIP kernels
    loss, Ll1, _ = l1_ssim_loss(image, gt_image, lambda_dssim)
    loss.backward(_unit(loss))
    return loss, pkg


_UNITS = {}


def _unit(loss):
    """d loss / d loss = 1, cached per device (loss.backward() would fill a new ones tensor)."""
    u = _UNITS.get(loss.device)
    if u is None or u.dtype != loss.dtype:
        u = _UNITS[loss.device] = torch.ones((), dtype=loss.dtype, device=loss.device)
    return u


def optimizer_step(gaussians, deform, iteration):
    """train_baseline.py:176-182 (both optimizers' Adam updates in one HIP launch)."""
    step_all(gaussians.optimizer, deform.optimizer)
    gaussians.update_learning_rate(iteration)
    gaussians.optimizer.zero_grad(set_to_none=True)
    deform.optimizer.zero_grad()
    deform.update_learning_rate(iteration)

"""One training iteration of train_baseline.py:104-182 on the HIP path (shared by bench.py and the
harness): deform -> render -> 0.8*L1 + 0.2*(1-SSIM) -> backward [-> grad all-reduce] -> Adam.
"""
import torch

from .adam import step_all
from .loss import l1_ssim_loss
from .renderer import render


def forward_backward(gaussians, deform, cam, gt_image, pipe, background, is_6dof=False, lambda_dssim=0.2,
                     warm=True, ast_noise=0.0):
    """train_baseline.py:104-128 (timed span of the reference's iter_start/iter_end events)."""
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

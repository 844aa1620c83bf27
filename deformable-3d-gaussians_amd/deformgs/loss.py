"""Photometric loss — mirror of utils/loss_utils.py:18-73 (L1, SSIM 11x11 sigma 1.5) and
utils/image_utils.py:19-21 (psnr). Pinned by tests/golden/loss.npz."""
from math import exp

import torch
import torch.nn.functional as F


def l1_loss(network_output, gt):
    return torch.abs(network_output - gt).mean()


def l2_loss(network_output, gt):
    return ((network_output - gt) ** 2).mean()


def gaussian(window_size, sigma):
    g = torch.Tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)])
    return g / g.sum()


_WIN = {}


def create_window(window_size, channel, device, dtype):
    key = (window_size, channel, str(device), dtype)
    w = _WIN.get(key)
    if w is None:
        g1 = gaussian(window_size, 1.5).unsqueeze(1)
        w2 = g1.mm(g1.t()).float().unsqueeze(0).unsqueeze(0)
        w = w2.expand(channel, 1, window_size, window_size).contiguous().to(device=device, dtype=dtype)
        _WIN[key] = w
    return w


def ssim(img1, img2, window_size=11, size_average=True):
    channel = img1.size(-3)
    window = create_window(window_size, channel, img1.device, img1.dtype)
    return _ssim(img1, img2, window, window_size, channel, size_average)


def _ssim(img1, img2, window, window_size, channel, size_average=True):
    pad = window_size // 2
    mu1 = F.conv2d(img1, window, padding=pad, groups=channel)
    mu2 = F.conv2d(img2, window, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = F.conv2d(img1 * img1, window, padding=pad, groups=channel) - mu1_sq
    sigma2_sq = F.conv2d(img2 * img2, window, padding=pad, groups=channel) - mu2_sq
    sigma12 = F.conv2d(img1 * img2, window, padding=pad, groups=channel) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    if size_average:
        return ssim_map.mean()
    return ssim_map.mean(1).mean(1).mean(1)


def psnr(img1, img2):
    mse = ((img1 - img2) ** 2).view(img1.shape[0], -1).mean(1, keepdim=True)
    return 20 * torch.log10(1.0 / torch.sqrt(mse))


# ---- fused HIP path (libdgs_hip: dgs_l1_ssim_*) used by the training step ----
class _FusedL1SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, gt, lambda_dssim):
        from . import _lib
        lib = _lib.load()
        img = img.float().contiguous()
        gt = gt.float().contiguous()
        _lib.require_cuda(img, gt)
        C, H, W = img.shape[-3:]
        scratch = torch.empty(lib.dgs_l1_ssim_scratch_floats(C, H, W), dtype=torch.float32, device=img.device)
        out = torch.empty(3, dtype=torch.float32, device=img.device)
        _lib.check(lib.dgs_l1_ssim_forward(C, H, W, _lib.ptr(img), _lib.ptr(gt), float(lambda_dssim), _lib.ptr(out),
                                           _lib.ptr(scratch), _lib.stream_ptr(img.device)), "l1_ssim_forward")
        ctx.save_for_backward(img, gt, scratch)
        ctx.lam = float(lambda_dssim)
        ctx.set_materialize_grads(False)  # l1 / ssim are not differentiable: no zero-fill kernels
        loss, l1, s = out[0], out[1], out[2]
        ctx.mark_non_differentiable(l1, s)
        return loss, l1, s

    @staticmethod
    def backward(ctx, dloss, dl1, dssim):
        from . import _lib
        img, gt, scratch = ctx.saved_tensors
        if dloss is None:
            return None, None, None
        C, H, W = img.shape[-3:]
        grad = torch.empty_like(img)
        dl = dloss.float().contiguous()
        _lib.check(_lib.load().dgs_l1_ssim_backward(C, H, W, _lib.ptr(img), _lib.ptr(gt), ctx.lam, _lib.ptr(scratch),
                                                    _lib.ptr(dl), _lib.ptr(grad), _lib.stream_ptr(img.device)),
                   "l1_ssim_backward")
        return grad, None, None


def l1_ssim_loss(image, gt, lambda_dssim=0.2):
    """(1-l)*l1_loss + l*(1-ssim) of train_baseline.py:126-127 in one fused HIP kernel pair.
    Returns (loss, Ll1, ssim_value); only `loss` carries a gradient (w.r.t. image)."""
    if gt.requires_grad and torch.is_grad_enabled():
        raise NotImplementedError("fused L1+SSIM differentiates w.r.t. the rendered image only")
    loss, l1, s = _FusedL1SSIM.apply(image, gt.detach(), lambda_dssim)
    return loss, l1, s

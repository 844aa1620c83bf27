"""6-DoF rigid-body helpers — mirror of utils/rigid_utils.py:4-107 (torch, autograd-friendly).

Used by the 6-DoF deformation head (utils/time_utils.py:114-121) on the raw (w, v) the fused MLP
kernel emits, and by render() (gaussian_renderer/__init__.py:71-76). Pinned by tests/golden/rigid.npz.
"""
import torch


def skew(w):
    zeros = torch.zeros(w.shape[0], device=w.device, dtype=w.dtype)
    return torch.stack([zeros, -w[:, 2], w[:, 1], w[:, 2], zeros, -w[:, 0], -w[:, 1], w[:, 0], zeros],
                       dim=-1).reshape(-1, 3, 3)


def rp_to_se3(R, p):
    bottom = torch.tensor([[0.0, 0.0, 0.0, 1.0]], device=R.device, dtype=R.dtype).repeat(R.shape[0], 1, 1)
    return torch.cat([torch.cat([R, p], dim=-1), bottom], dim=1)


def exp_so3(w, theta):
    W = skew(w)
    I = torch.eye(3, device=W.device, dtype=W.dtype).unsqueeze(0).repeat(W.shape[0], 1, 1)
    W2 = torch.bmm(W, W)
    return I + torch.sin(theta.unsqueeze(-1)) * W + (1.0 - torch.cos(theta.unsqueeze(-1))) * W2


def exp_se3(S, theta):
    w, v = torch.split(S, 3, dim=-1)
    W = skew(w)
    R = exp_so3(w, theta)
    I = torch.eye(3, device=W.device, dtype=W.dtype).unsqueeze(0).repeat(W.shape[0], 1, 1)
    W2 = torch.bmm(W, W)
    theta = theta.view(-1, 1, 1)
    p = torch.bmm(theta * I + (1.0 - torch.cos(theta)) * W + (theta - torch.sin(theta)) * W2, v.unsqueeze(-1))
    return rp_to_se3(R, p)


def to_homogenous(v):
    return torch.cat([v, torch.ones_like(v[..., :1])], dim=-1)


def from_homogenous(v):
    return v[..., :3] / v[..., -1:]


def screw_from_raw(w, v):
    """time_utils.py:117-121: theta = |w|; w = w/theta + 1e-5; v = v/theta + 1e-5 -> exp_se3."""
    theta = torch.norm(w, dim=-1, keepdim=True)
    w = w / theta + 1e-5
    v = v / theta + 1e-5
    return exp_se3(torch.cat([w, v], dim=-1), theta)

"""ORACLE (test infrastructure only) — float64 numpy restatement of the reference deformation MLP.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, and only
as the checker / CPU baseline. The product path never imports it.

Restates (file:line in preacherwhite/Deformable-3D-Gaussians):
  utils/time_utils.py:7-54     get_embedder / Embedder.embed: [x, sin(2^0 x), cos(2^0 x), ...,
                               sin(2^(L-1) x), cos(2^(L-1) x)], sin for all dims then cos per band
  utils/time_utils.py:56-127   DeformNetworkBaseline.forward: optional timenet (blender), 8 x
                               (Linear + ReLU) with skip cat(x_emb, t_emb, h) after layer 4, heads
  utils/time_utils.py:114-121  6-DoF head: theta=|w|, w=w/theta+1e-5, v=v/theta+1e-5, exp_se3
  utils/time_utils.py:129-201  DeformNetwork: same trunk, rot/scale returned as 0
  utils/rigid_utils.py:4-83    skew, exp_so3, exp_se3
Backward is written by hand (chain rule), so this file is independent of torch autograd.
Pinned against tests/golden/mlp_*.npz (outputs of the reference itself).
"""
import numpy as np

D = 8
W = 256
SKIP = 4


def embed(x, L):
    """utils/time_utils.py:42-54 (log_sampling=True, include_input=True)."""
    x = np.asarray(x, np.float64)
    outs = [x]
    for i in range(L):
        f = 2.0 ** i
        outs.append(np.sin(x * f))
        outs.append(np.cos(x * f))
    return np.concatenate(outs, -1)


def _lin(p, name, h):
    return h @ p[name + ".weight"].astype(np.float64).T + p[name + ".bias"].astype(np.float64)


def forward(p, x, t, is_blender, is_6dof, fork=False):
    """Returns (outputs dict, cache). Outputs: d_xyz (N,3) or (N,4,4) for 6-DoF, d_rot, d_scale."""
    c = {}
    te_in = embed(t, 6 if is_blender else 10)
    c["te_in"] = te_in
    if is_blender:
        z = _lin(p, "timenet.0", te_in)
        c["tz0"] = z
        th = np.maximum(z, 0.0)
        c["th"] = th
        te = _lin(p, "timenet.2", th)
    else:
        te = te_in
    xe = embed(x, 10)
    c["xe"], c["te"] = xe, te
    h = np.concatenate([xe, te], -1)
    c["hin"] = []
    c["z"] = []
    for i in range(D):
        c["hin"].append(h)
        z = _lin(p, f"linear.{i}", h)
        c["z"].append(z)
        h = np.maximum(z, 0.0)
        if i == SKIP:
            h = np.concatenate([xe, te, h], -1)
    c["hlast"] = h
    out = {}
    if is_6dof:
        w = _lin(p, "branch_w", h)
        v = _lin(p, "branch_v", h)
        out["w_raw"], out["v_raw"] = w, v
        out["d_xyz"] = se3_from_raw(w, v)
    else:
        out["d_xyz"] = _lin(p, "gaussian_warp", h)
    if fork:
        out["d_rot"] = 0.0
        out["d_scale"] = 0.0
    else:
        out["d_rot"] = _lin(p, "gaussian_rotation", h)
        out["d_scale"] = _lin(p, "gaussian_scaling", h)
    return out, c


def skew(w):
    z = np.zeros(w.shape[0])
    return np.stack([z, -w[:, 2], w[:, 1], w[:, 2], z, -w[:, 0], -w[:, 1], w[:, 0], z], -1).reshape(-1, 3, 3)


def se3_from_raw(w_raw, v_raw):
    """time_utils.py:117-121 then rigid_utils.exp_se3 (Modern Robotics 3.51 / 3.88)."""
    theta = np.linalg.norm(w_raw, axis=-1, keepdims=True)
    w = w_raw / theta + 1e-5
    v = v_raw / theta + 1e-5
    Wm = skew(w)
    W2 = Wm @ Wm
    th = theta[:, :, None]
    I = np.eye(3)[None]
    R = I + np.sin(th) * Wm + (1.0 - np.cos(th)) * W2
    G = th * I + (1.0 - np.cos(th)) * Wm + (th - np.sin(th)) * W2
    pvec = G @ v[:, :, None]
    M = np.zeros((w.shape[0], 4, 4))
    M[:, :3, :3] = R
    M[:, :3, 3:] = pvec
    M[:, 3, 3] = 1.0
    return M


def _se3_vjp(w_raw, v_raw, gM, eps=1e-6):
    """d<se3(w,v), gM>/d(w,v) by central differences in float64 (per point, 6 inputs)."""
    gw = np.zeros_like(w_raw)
    gv = np.zeros_like(v_raw)
    for j in range(3):
        for arr, g in ((w_raw, gw), (v_raw, gv)):
            a = arr.copy()
            a[:, j] += eps
            fp = se3_from_raw(a if arr is w_raw else w_raw, a if arr is v_raw else v_raw)
            a[:, j] -= 2 * eps
            fm = se3_from_raw(a if arr is w_raw else w_raw, a if arr is v_raw else v_raw)
            g[:, j] = ((fp - fm) * gM).sum((1, 2)) / (2 * eps)
    return gw, gv


def backward(p, c, out, g, is_blender, is_6dof, fork=False, relu_masks=None, abs_sums=None):
    """g: dict of upstream grads for d_xyz / d_rot / d_scale. Returns dict param-name -> grad.

    relu_masks (optional): {layer i: bool (N, 256), "th": bool (N, 256)} overriding relu'(z) = z > 0.
    A pre-activation within a few fp32 ulps of 0 can take either sign in an fp32 forward, which flips
    a whole row of dZ; the GPU parity tests pass the kernel's own masks so they check the arithmetic
    and not that tie (tests/test_gpu_mlp.py).
    abs_sums (optional dict): filled with, per parameter, the sum over points of the absolute values
    of the terms its gradient sums (|dZ|^T |X|, sum |dZ|): the scale of an fp32 summation's rounding
    error, which a nearly cancelling gradient sum does not show."""
    relu_masks = relu_masks or {}
    gr = {}
    h = c["hlast"]
    dh = np.zeros_like(h)

    def record(name, dz, x):
        gr[name + ".weight"] = dz.T @ x
        gr[name + ".bias"] = dz.sum(0)
        if abs_sums is not None:
            abs_sums[name + ".weight"] = np.abs(dz).T @ np.abs(x)
            abs_sums[name + ".bias"] = np.abs(dz).sum(0)

    def head(name, gout):
        nonlocal dh
        gout = np.asarray(gout, np.float64)
        record(name, gout, h)
        dh = dh + gout @ p[name + ".weight"].astype(np.float64)

    if is_6dof:
        if "w_raw" in g:  # upstream gradient given on the raw head outputs (kernel-level checks)
            gw, gv = np.asarray(g["w_raw"], np.float64), np.asarray(g["v_raw"], np.float64)
        else:
            gw, gv = _se3_vjp(out["w_raw"], out["v_raw"], np.asarray(g["d_xyz"], np.float64))
        head("branch_w", gw)
        head("branch_v", gv)
    else:
        head("gaussian_warp", g["d_xyz"])
    if not fork:
        head("gaussian_rotation", g["d_rot"])
        head("gaussian_scaling", g["d_scale"])
    nx = c["xe"].shape[1]
    nt = c["te"].shape[1]
    dte = np.zeros_like(c["te"])
    for i in reversed(range(D)):
        if i == SKIP:
            dte += dh[:, nx:nx + nt]
            dh = dh[:, nx + nt:]
        dz = dh * relu_masks.get(i, c["z"][i] > 0)
        record(f"linear.{i}", dz, c["hin"][i])
        dh = dz @ p[f"linear.{i}.weight"].astype(np.float64)
    dte += dh[:, nx:nx + nt]
    if is_blender:
        record("timenet.2", dte, c["th"])
        dth = dte @ p["timenet.2.weight"].astype(np.float64)
        dz = dth * relu_masks.get("th", c["tz0"] > 0)
        record("timenet.0", dz, c["te_in"])
    return gr


def param_shapes(is_blender, is_6dof, D_=8, W_=256, multires=10):
    """state_dict key order and shapes of DeformNetworkBaseline (time_utils.py:56-100)."""
    xin = 3 + 3 * 2 * multires
    tin = 1 + 2 * (6 if is_blender else 10)
    shapes = {}
    if is_blender:
        shapes["timenet.0.weight"] = (256, tin)
        shapes["timenet.0.bias"] = (256,)
        shapes["timenet.2.weight"] = (30, 256)
        shapes["timenet.2.bias"] = (30,)
        tout = 30
    else:
        tout = tin
    for i in range(D_):
        if i == 0:
            k = xin + tout
        elif i == D_ // 2 + 1:
            k = W_ + xin + tout
        else:
            k = W_
        shapes[f"linear.{i}.weight"] = (W_, k)
        shapes[f"linear.{i}.bias"] = (W_,)
    if is_6dof:
        for n in ("branch_w", "branch_v"):
            shapes[n + ".weight"] = (3, W_)
            shapes[n + ".bias"] = (3,)
    else:
        shapes["gaussian_warp.weight"] = (3, W_)
        shapes["gaussian_warp.bias"] = (3,)
    shapes["gaussian_rotation.weight"] = (4, W_)
    shapes["gaussian_rotation.bias"] = (4,)
    shapes["gaussian_scaling.weight"] = (3, W_)
    shapes["gaussian_scaling.bias"] = (3,)
    return shapes

"""CPU: pin the oracle. MLP oracle vs the reference's own outputs (golden fixtures); rasterizer oracle
vs a dense float64 autograd restatement and closed-form known answers (rasterizer parity is
unpinned by the reference — see oracle/raster_ref.c)."""
import math

import numpy as np
import pytest
import torch

from dense_raster import dense_render
from helpers import scene
from oracle import mlp_ref
from oracle.raster import OracleRaster, make_settings
from weights import mlp_weights, proj_mats

VARIANTS = {"blender": (True, False, False), "nonblender": (False, False, False), "6dof": (True, True, False),
            "fork": (True, False, True)}


@pytest.mark.parametrize("name", list(VARIANTS))
def test_mlp_oracle_matches_reference(name, golden_dir):
    bl, d6, fork = VARIANTS[name]
    f = np.load(f"{golden_dir}/mlp_{name}.npz")
    p = mlp_weights(mlp_ref.param_shapes(bl, d6), int(f["seed_w"]))
    out, c = mlp_ref.forward(p, f["x"], f["t"], bl, d6, fork)
    assert np.abs(out["d_xyz"] - f["d_xyz"]).max() < 1e-6
    g = {"d_xyz": f["g_xyz"]}
    if not fork:
        assert np.abs(out["d_rot"] - f["d_rot"]).max() < 1e-6
        assert np.abs(out["d_scale"] - f["d_scale"]).max() < 1e-6
        g["d_rot"], g["d_scale"] = f["g_rot"], f["g_scale"]
    gr = mlp_ref.backward(p, c, out, g, bl, d6, fork)
    for k, v in gr.items():
        if "grad." + k in f:
            ref = f["grad." + k]
            assert np.abs(v - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1e-6), k
        else:
            r1, r2 = proj_mats(v.shape, 3000)
            assert (np.abs(r1 @ v @ r2.T - f["gproj." + k]) <= 1e-5 * f["gabs." + k] + 1e-9).all(), k


def _dense_vs_oracle(N, H, W, ci, boost, bg, deg=3):
    inputs, rs, cam = scene(N, H, W, cam_index=ci, scale_boost=boost, bg=bg, sh_degree=deg)
    s = make_settings(H, W, rs["tanfovx"], rs["tanfovy"], rs["bg"].numpy(), 1.0, rs["viewmatrix"].numpy(),
                      rs["projmatrix"].numpy(), deg, rs["campos"].numpy())
    rot = inputs["rotations"] * 1.1  # un-normalised quaternion, as render() produces after + d_rot
    o = OracleRaster(s, inputs["means3D"].numpy(), shs=inputs["shs"].numpy(), opacities=inputs["opacities"].numpy(),
                     scales=inputs["scales"].numpy(), rotations=rot.numpy())
    d = lambda a: a.detach().double().clone().requires_grad_(True)  # noqa: E731
    m3, sh, op, sc, ro = d(inputs["means3D"]), d(inputs["shs"]), d(inputs["opacities"]), d(inputs["scales"]), d(rot)
    m2 = torch.zeros(N, 3, dtype=torch.float64, requires_grad=True)
    img, dep, rad = dense_render(H, W, rs["tanfovx"], rs["tanfovy"], rs["bg"].double(), 1.0,
                                 rs["viewmatrix"].double(), rs["projmatrix"].double(), deg, rs["campos"].double(),
                                 m3, m2, op, shs=sh, scales=sc, rotations=ro)
    assert (rad.numpy() == o.radii).all()
    assert np.abs(img.detach().numpy() - o.color).max() < 1e-5
    assert np.abs(dep.detach().numpy() - o.depth).max() < 1e-4
    rng = np.random.default_rng(0)
    gc = rng.standard_normal(o.color.shape).astype(np.float32)
    gd = rng.standard_normal(o.depth.shape).astype(np.float32)
    ((img * torch.from_numpy(gc).double()).sum() + (dep * torch.from_numpy(gd).double()).sum()).backward()
    gr = o.backward(gc, gd)
    for name, t, key in [("means3D", m3, "means3D"), ("shs", sh, "shs"), ("opacities", op, "opacities"),
                         ("scales", sc, "scales"), ("rotations", ro, "rotations"), ("means2D", m2, "means2D")]:
        ref = t.grad.numpy().reshape(gr[key].shape)
        rel = np.abs(ref - gr[key]).max() / max(np.abs(ref).max(), 1e-12)
        assert rel < 2e-5, (name, rel)
    return o


def test_raster_oracle_vs_dense_autograd():
    _dense_vs_oracle(300, 48, 64, 3, 1.0, (0.2, 0.5, 0.9))
    _dense_vs_oracle(150, 33, 40, 6, 1.6, (0.0, 0.0, 0.0), deg=1)


def _single(opac, sigma_px, H=33, W=33, center=None, depth=2.0):
    """One isotropic Gaussian straight ahead: closed form is o*exp(-d^2/(2 s^2)) (no EWA clamp)."""
    fov = 2 * math.atan(0.5)
    tan = math.tan(fov / 2)
    fx = W / (2 * tan)
    view = np.eye(4, dtype=np.float32)
    from deformgs.cameras import getProjectionMatrix
    proj = (torch.from_numpy(view) @ getProjectionMatrix(0.01, 100.0, fov, fov).T).numpy()
    # world sigma so that the 2D variance (+0.3 low-pass) is sigma_px^2
    s_world = math.sqrt(max(sigma_px ** 2 - 0.3, 1e-6)) * depth / fx
    s = make_settings(H, W, tan, tan, [0, 0, 0], 1.0, view, proj, 0, [0, 0, 0])
    mean = np.array([[0.0, 0.0, depth]], np.float32) if center is None else np.array([center], np.float32)
    sh = np.zeros((1, 1, 3), np.float32)
    sh[0, 0, :] = (1.0 - 0.5) / 0.28209479177387814  # colour 1.0
    o = OracleRaster(s, mean, shs=sh, opacities=np.array([opac], np.float32),
                     scales=np.full((1, 3), s_world, np.float32), rotations=np.array([[1, 0, 0, 0]], np.float32))
    return o


def test_known_answer_isotropic():
    o = _single(0.8, 3.0)
    H = W = 33
    cx = (W - 1) / 2
    yy, xx = np.mgrid[0:H, 0:W]
    a = 0.8 * np.exp(-((xx - cx) ** 2 + (yy - cx) ** 2) / (2 * 9.0))
    expect = np.where(a >= 1 / 255, a, 0.0)
    assert np.abs(o.color[0] - expect).max() < 1e-4
    lam = 9.0 + math.sqrt(0.1)  # mid + sqrt(max(0.1, mid^2 - det)) with mid^2 == det
    assert o.radii[0] == math.ceil(3 * math.sqrt(lam))


def test_known_answer_alpha_clamp_and_termination():
    o = _single(1.0, 3.0)
    assert abs(o.color[0, 16, 16] - 0.99) < 1e-6  # alpha clamped at 0.99
    # two opaque Gaussians at the same pixel: front one wins, T stops before 1e-4
    from oracle.raster import OracleRaster as OR
    s = o.s
    means = np.array([[0, 0, 2.0], [0, 0, 3.0]], np.float32)
    sh = np.zeros((2, 1, 3), np.float32)
    sh[0, 0, 0] = (1.0 - 0.5) / 0.28209479177387814   # red in front
    sh[1, 0, 1] = (1.0 - 0.5) / 0.28209479177387814   # green behind
    sh[:, 0, :] += -0.5 / 0.28209479177387814 * (sh[:, 0, :] == 0)
    two = OR(s, means, shs=sh, opacities=np.array([0.99, 0.99], np.float32),
             scales=np.full((2, 3), 0.2, np.float32), rotations=np.tile(np.array([[1, 0, 0, 0]], np.float32), (2, 1)))
    c = two.color[:, 16, 16]
    assert c[0] > 0.98 and c[1] < 0.02, c
    T, n = two.pixel_state()
    # the second Gaussian would take T to 0.01*0.01 < 1e-4: it is refused (stop BEFORE adding)
    assert abs(T[16, 16] - 0.01) < 1e-6 and n[16, 16] == 1


def test_known_answer_skip_threshold():
    # opacity below 1/255 everywhere -> nothing rendered, T stays 1
    o = _single(1.0 / 256.0, 3.0)
    assert o.color.max() == 0.0
    T, n = o.pixel_state()
    assert (T == 1.0).all() and (n == 0).all()


def test_trace_flags_known_answers():
    """The oracle's near-threshold reporting used by the parity tests (tests/helpers.py tail_flags):
    or_flip_flags flags a pixel whose o G sits exactly on the 0.99 clamp; or_preprocess_flags flags a
    Gaussian whose SH colour + 0.5 is exactly 0 (the colour clamp) and not one far from it;
    or_pixel_gaussians flags the Gaussians blended in a masked pixel and nothing for a pixel they miss."""
    o = _single(0.99, 3.0)  # o G = 0.99 exactly at the centre pixel (G = 1 there)
    g, px = o.flip_flags(1e-4)
    assert px[16, 16] and g[0]
    far = _single(0.8, 3.0)
    g2, px2 = far.flip_flags(1e-4)
    assert px2[16, 16]  # power == 0 exactly at the mean's pixel: the power > 0 skip is on its threshold
    assert not px2[16, 19] and not px2[5, 16]  # o G well inside (0, 0.99), power well below 0
    assert not far.preprocess_flags(1e-4)[0]  # colour 1.0, straight ahead: no clamp near
    m = np.zeros((33, 33), bool)
    m[16, 16] = True
    assert far.pixel_gaussians(m).tolist() == [True]
    m[:] = False
    m[0, 0] = True  # alpha 0.8 exp(-(16^2 + 16^2) / 18) < 1/255: not blended there
    assert far.pixel_gaussians(m).tolist() == [False]
    # colour channels exactly at the clamp (SH colour + 0.5 == 0)
    s = far.s
    sh = np.full((1, 1, 3), -0.5 / 0.28209479177387814, np.float32)
    sh[0, 0, 0] = (1.0 - 0.5) / 0.28209479177387814
    from oracle.raster import OracleRaster as OR
    z = OR(s, np.array([[0, 0, 2.0]], np.float32), shs=sh, opacities=np.array([0.8], np.float32),
           scales=np.full((1, 3), 0.2, np.float32), rotations=np.array([[1, 0, 0, 0]], np.float32))
    assert z.preprocess_flags(1e-4)[0]

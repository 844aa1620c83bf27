"""Generate golden vectors by running the REFERENCE's own Python code (CPU, this container only).

This script imports modules from /root/reference (read-only) and records their outputs for
seeded inputs as small .npz fixtures under tests/golden/. The reference never travels to the
GPU box: only the .npz files do. Re-run with:  python tests/golden/make_golden.py

Sources exercised (file:line in /root/reference):
  utils/time_utils.py:56-127   DeformNetworkBaseline fwd + bwd (blender / non-blender / 6-DoF)
  utils/time_utils.py:129-201  DeformNetwork (fork variant, rot/scale = 0)
  utils/rigid_utils.py:60-107  exp_se3, to/from_homogenous
  utils/loss_utils.py:18-73    l1_loss, ssim (+ grads of 0.8*L1 + 0.2*(1-SSIM))
  utils/sh_utils.py:57-112     eval_sh, deg 0..3
  utils/general_utils.py:42-163 get_expon_lr_func, build_rotation, build_scaling_rotation, strip_symmetric
  utils/graphics_utils.py:42-84 getWorld2View2, getProjectionMatrix, fov2focal
  scene/cameras.py:18-61       Camera matrices (loaded by file path; scene/__init__ pulls missing deps)

Weights are NOT stored: they are drawn from numpy's PCG64 (`mlp_weights` below), which is
bit-stable across numpy versions, and loaded into the reference module with load_state_dict.
The tests regenerate the same weights with the same function (tests/golden/weights.py).
"""
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, REF)

from weights import mlp_weights, proj_mats  # noqa: E402


def _load_by_path(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def gen_mlp():
    import utils.time_utils as tu

    variants = {
        "blender": dict(is_blender=True, is_6dof=False, cls=tu.DeformNetworkBaseline),
        "nonblender": dict(is_blender=False, is_6dof=False, cls=tu.DeformNetworkBaseline),
        "6dof": dict(is_blender=True, is_6dof=True, cls=tu.DeformNetworkBaseline),
        "fork": dict(is_blender=True, is_6dof=False, cls=tu.DeformNetwork),
    }
    N = 64
    for vi, (name, v) in enumerate(variants.items()):
        net = v["cls"](is_blender=v["is_blender"], is_6dof=v["is_6dof"])
        sd = net.state_dict()
        shapes = {k: tuple(t.shape) for k, t in sd.items()}
        w = mlp_weights(shapes, seed=1000 + vi)
        net.load_state_dict({k: torch.from_numpy(a) for k, a in w.items()})
        rng = np.random.default_rng(2000 + vi)
        x = rng.uniform(-1.3, 1.3, size=(N, 3)).astype(np.float32)
        if name == "nonblender":
            # per-row times (ast_noise-like), exercises non-uniform t
            t = rng.uniform(0.0, 1.0, size=(N, 1)).astype(np.float32)
        else:
            t = np.full((N, 1), rng.uniform(0.0, 1.0), dtype=np.float32)
        xt = torch.from_numpy(x)
        tt = torch.from_numpy(t)
        d_xyz, d_rot, d_scale = net(xt, tt)
        out = {"x": x, "t": t}
        loss = 0.0
        if torch.is_tensor(d_xyz):
            g = rng.standard_normal(tuple(d_xyz.shape)).astype(np.float32)
            out["d_xyz"] = d_xyz.detach().numpy()
            out["g_xyz"] = g
            loss = loss + (d_xyz * torch.from_numpy(g)).sum()
        for key, val in (("d_rot", d_rot), ("d_scale", d_scale)):
            if torch.is_tensor(val):
                g = rng.standard_normal(tuple(val.shape)).astype(np.float32)
                out[key] = val.detach().numpy()
                out["g" + key[1:]] = g
                loss = loss + (val * torch.from_numpy(g)).sum()
        loss.backward()
        for k, p in net.named_parameters():
            if p.grad is None:  # DeformNetwork's rot/scale heads are unused (time_utils.py:198-199)
                continue
            gr = p.grad.numpy().astype(np.float32)
            if p.dim() == 1 or name == "blender":
                out["grad." + k] = gr
            else:
                r1, r2 = proj_mats(gr.shape, seed=3000)
                out["gproj." + k] = (r1 @ gr.astype(np.float64) @ r2.T).astype(np.float64)
                out["gabs." + k] = (np.abs(r1) @ np.abs(gr.astype(np.float64)) @ np.abs(r2).T)
        out["seed_w"] = np.int64(1000 + vi)
        np.savez(os.path.join(HERE, f"mlp_{name}.npz"), **out)
        print("mlp", name, {k: v.shape for k, v in out.items() if hasattr(v, "shape")}.__len__(), "arrays")


def gen_rigid():
    import utils.rigid_utils as ru
    rng = np.random.default_rng(4000)
    N = 128
    w = rng.standard_normal((N, 3)).astype(np.float32)
    v = rng.standard_normal((N, 3)).astype(np.float32)
    theta = np.linalg.norm(w, axis=-1, keepdims=True).astype(np.float32)
    S = torch.from_numpy(np.concatenate([w / theta + 1e-5, v / theta + 1e-5], -1).astype(np.float32))
    M = ru.exp_se3(S, torch.from_numpy(theta))
    xyz = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
    moved = ru.from_homogenous(torch.bmm(M, ru.to_homogenous(torch.from_numpy(xyz)).unsqueeze(-1)).squeeze(-1))
    np.savez(os.path.join(HERE, "rigid.npz"), w=w, v=v, theta=theta, screw=S.numpy(), M=M.numpy(),
             xyz=xyz, moved=moved.numpy())


def gen_loss():
    import utils.loss_utils as lu
    rng = np.random.default_rng(5000)
    img1 = rng.uniform(0, 1, (3, 40, 56)).astype(np.float32)
    img2 = np.clip(img1 + 0.1 * rng.standard_normal(img1.shape), 0, 1).astype(np.float32)
    a = torch.from_numpy(img1).requires_grad_(True)
    b = torch.from_numpy(img2)
    l1 = lu.l1_loss(a, b)
    s = lu.ssim(a, b)
    loss = 0.8 * l1 + 0.2 * (1.0 - s)
    loss.backward()
    np.savez(os.path.join(HERE, "loss.npz"), img1=img1, img2=img2, l1=l1.item(), ssim=s.item(),
             loss=loss.item(), grad=a.grad.numpy())


def gen_sh():
    import utils.sh_utils as su
    rng = np.random.default_rng(6000)
    N = 256
    sh = (0.3 * rng.standard_normal((N, 3, 16))).astype(np.float32)
    d = rng.standard_normal((N, 3))
    d = (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(np.float32)
    out = {"sh": sh, "dirs": d}
    for deg in range(4):
        out[f"rgb{deg}"] = su.eval_sh(deg, torch.from_numpy(sh), torch.from_numpy(d)).numpy()
    out["rgb2sh"] = su.RGB2SH(torch.tensor([0.0, 0.5, 1.0])).numpy()
    np.savez(os.path.join(HERE, "sh.npz"), **out)


def gen_cov_and_lr():
    import utils.general_utils as gu
    # build_rotation / strip_lowerdiag allocate with device="cuda" (general_utils.py:115,135,155);
    # for CPU capture drop that kwarg while the reference functions run.
    real_zeros = torch.zeros

    def cpu_zeros(*a, **k):
        k.pop("device", None)
        return real_zeros(*a, **k)

    rng = np.random.default_rng(7000)
    N = 256
    s = np.exp(rng.uniform(-4, -1, (N, 3))).astype(np.float32)
    q = rng.standard_normal((N, 4)).astype(np.float32)
    torch.zeros = cpu_zeros
    try:
        R = gu.build_rotation(torch.from_numpy(q))
        L = gu.build_scaling_rotation(torch.from_numpy(1.3 * s), torch.from_numpy(q))
        cov = gu.strip_symmetric(L @ L.transpose(1, 2))
    finally:
        torch.zeros = real_zeros
    f = gu.get_expon_lr_func(lr_init=1.6e-4 * 5, lr_final=1.6e-6, lr_delay_mult=0.01, max_steps=40000)
    steps = np.array([0, 1, 100, 3000, 20000, 39999, 40000, 50000])
    lrs = np.array([f(int(k)) for k in steps])
    g = gu.get_linear_noise_func(lr_init=0.1, lr_final=1e-15, lr_delay_mult=0.01, max_steps=20000)
    noise = np.array([g(int(k)) for k in steps])
    np.savez(os.path.join(HERE, "cov_lr.npz"), scales=s, quats=q, mod=np.float32(1.3), R=R.numpy(),
             cov6=cov.numpy(), steps=steps, lrs=lrs, noise=noise,
             inv_sig=gu.inverse_sigmoid(torch.tensor([0.1, 0.5, 0.9])).numpy())


def gen_camera():
    gr = _load_by_path("ref_graphics_utils", os.path.join(REF, "utils/graphics_utils.py"))
    sys.modules["utils.graphics_utils"] = gr
    cams = _load_by_path("ref_cameras", os.path.join(REF, "scene/cameras.py"))
    # D-NeRF-style camera: look at origin from (0,0,4.0311); transforms_*.json c2w -> R,T exactly as
    # scene/dataset_readers.py:223-266 does (flip y/z columns, w2c, R = w2c[:3,:3].T)
    out = {}
    rng = np.random.default_rng(8000)
    for ci in range(3):
        az = rng.uniform(-np.pi, np.pi)
        el = rng.uniform(-0.6, 0.6)
        r = 4.0311
        cpos = np.array([r * np.cos(el) * np.sin(az), -r * np.cos(el) * np.cos(az), r * np.sin(el)])
        fwd = -cpos / np.linalg.norm(cpos)
        up = np.array([0.0, 0.0, 1.0])
        right = np.cross(fwd, up); right /= np.linalg.norm(right)
        upv = np.cross(right, fwd)
        c2w = np.eye(4)
        c2w[:3, 0] = right; c2w[:3, 1] = upv; c2w[:3, 2] = -fwd; c2w[:3, 3] = cpos  # Blender/OpenGL
        # scene/dataset_readers.py:235-238 (readCamerasFromTransforms)
        matrix = np.linalg.inv(c2w)
        R = -np.transpose(matrix[:3, :3])
        R[:, 0] = -R[:, 0]
        T = -matrix[:3, 3]
        fov = 0.6911112070083618
        img = torch.zeros(3, 64, 80)
        cam = cams.Camera(colmap_id=ci, R=R, T=T, FoVx=fov, FoVy=fov * 64 / 80, image=img,
                          gt_alpha_mask=None, image_name="x", uid=ci, data_device="cpu", fid=0.5)
        out[f"R{ci}"] = R
        out[f"T{ci}"] = T
        out[f"fovx{ci}"] = np.float64(cam.FoVx)
        out[f"fovy{ci}"] = np.float64(cam.FoVy)
        out[f"view{ci}"] = cam.world_view_transform.numpy()
        out[f"proj{ci}"] = cam.projection_matrix.numpy()
        out[f"full{ci}"] = cam.full_proj_transform.numpy()
        out[f"center{ci}"] = cam.camera_center.numpy()
    np.savez(os.path.join(HERE, "camera.npz"), **out)


if __name__ == "__main__":
    torch.set_num_threads(4)
    gen_mlp()
    gen_rigid()
    gen_loss()
    gen_sh()
    gen_cov_and_lr()
    gen_camera()
    print("golden vectors written to", HERE)

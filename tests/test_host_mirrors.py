"""CPU: the host-side mirrors of the reference's Python helpers against its own outputs (golden)."""
import numpy as np
import pytest
import torch

from deformgs import cameras, general, loss, rigid, sh


def test_eval_sh(golden_dir):
    f = np.load(f"{golden_dir}/sh.npz")
    for deg in range(4):
        got = sh.eval_sh(deg, torch.from_numpy(f["sh"]), torch.from_numpy(f["dirs"])).numpy()
        assert np.abs(got - f[f"rgb{deg}"]).max() < 1e-6
    assert np.allclose(sh.RGB2SH(torch.tensor([0.0, 0.5, 1.0])).numpy(), f["rgb2sh"])


def test_rotation_cov_lr(golden_dir):
    f = np.load(f"{golden_dir}/cov_lr.npz")
    q = torch.from_numpy(f["quats"])
    assert np.abs(general.build_rotation(q).numpy() - f["R"]).max() < 1e-6
    L = general.build_scaling_rotation(torch.from_numpy(f["mod"] * f["scales"]), q)
    cov = general.strip_symmetric(L @ L.transpose(1, 2)).numpy()
    assert np.abs(cov - f["cov6"]).max() < 1e-7
    fn = general.get_expon_lr_func(lr_init=1.6e-4 * 5, lr_final=1.6e-6, lr_delay_mult=0.01, max_steps=40000)
    assert np.allclose([fn(int(s)) for s in f["steps"]], f["lrs"], rtol=1e-12)
    gn = general.get_linear_noise_func(lr_init=0.1, lr_final=1e-15, lr_delay_mult=0.01, max_steps=20000)
    assert np.allclose([gn(int(s)) for s in f["steps"]], f["noise"], rtol=1e-12)
    assert np.allclose(general.inverse_sigmoid(torch.tensor([0.1, 0.5, 0.9])).numpy(), f["inv_sig"])


def test_cov3d_kernel_math_matches_reference(golden_dir):
    """The rasterizer's Sigma (oracle / kernel math: L = R diag(s), raw q) equals the reference's
    compute_cov3D_python path (general_utils.py:154-163) for unit quaternions."""
    from helpers import oracle_run
    f = np.load(f"{golden_dir}/cov_lr.npz")
    q = f["quats"] / np.linalg.norm(f["quats"], axis=1, keepdims=True)
    L = general.build_scaling_rotation(torch.from_numpy(f["mod"] * f["scales"]), torch.from_numpy(q))
    ref = general.strip_symmetric(L @ L.transpose(1, 2)).numpy()
    # run the oracle on Gaussians placed in front of a camera and read back its Sigma
    import math
    from oracle.raster import OracleRaster, make_settings
    N = q.shape[0]
    view = np.eye(4, dtype=np.float32)
    proj = (torch.eye(4) @ cameras.getProjectionMatrix(0.01, 100, 1.0, 1.0).T).numpy()
    s = make_settings(64, 64, math.tan(0.5), math.tan(0.5), [0, 0, 0], float(f["mod"]), view, proj, 0, [0, 0, 0])
    means = np.tile(np.array([[0.0, 0.0, 3.0]], np.float32), (N, 1))
    o = OracleRaster(s, means, shs=np.zeros((N, 1, 3), np.float32), opacities=np.full((N,), 0.5, np.float32),
                     scales=f["scales"], rotations=q.astype(np.float32))
    assert np.abs(o.geometry()["cov3D"] - ref).max() < 1e-6


def test_camera_matrices(golden_dir):
    f = np.load(f"{golden_dir}/camera.npz")
    for ci in range(3):
        cam = cameras.Camera(f[f"R{ci}"], f[f"T{ci}"], float(f[f"fovx{ci}"]), float(f[f"fovy{ci}"]), 80, 64,
                             fid=0.5, data_device="cpu")
        assert np.abs(cam.world_view_transform.numpy() - f[f"view{ci}"]).max() < 1e-6
        assert np.abs(cam.projection_matrix.numpy() - f[f"proj{ci}"]).max() < 1e-6
        assert np.abs(cam.full_proj_transform.numpy() - f[f"full{ci}"]).max() < 1e-5
        assert np.abs(cam.camera_center.numpy() - f[f"center{ci}"]).max() < 1e-5


def test_rigid(golden_dir):
    f = np.load(f"{golden_dir}/rigid.npz")
    M = rigid.exp_se3(torch.from_numpy(f["screw"]), torch.from_numpy(f["theta"]))
    assert np.abs(M.numpy() - f["M"]).max() < 1e-5
    M2 = rigid.screw_from_raw(torch.from_numpy(f["w"]), torch.from_numpy(f["v"]))
    assert np.abs(M2.numpy() - f["M"]).max() < 1e-5
    moved = rigid.from_homogenous(torch.bmm(M, rigid.to_homogenous(torch.from_numpy(f["xyz"])).unsqueeze(-1)).squeeze(-1))
    assert np.abs(moved.numpy() - f["moved"]).max() < 1e-5


def test_loss(golden_dir):
    f = np.load(f"{golden_dir}/loss.npz")
    a = torch.from_numpy(f["img1"]).requires_grad_(True)
    b = torch.from_numpy(f["img2"])
    l1 = loss.l1_loss(a, b)
    s = loss.ssim(a, b)
    total = 0.8 * l1 + 0.2 * (1.0 - s)
    total.backward()
    assert abs(l1.item() - float(f["l1"])) < 1e-7
    assert abs(s.item() - float(f["ssim"])) < 1e-6
    assert np.abs(a.grad.numpy() - f["grad"]).max() < 1e-8


def test_ply_roundtrip(tmp_path):
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_gaussians
    g = synth_gaussians(100, device="cpu")
    m = GaussianModel(3)
    m.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    path = str(tmp_path / "point_cloud.ply")
    m.save_ply(path)
    m2 = GaussianModel(3)
    m2.load_ply(path, device="cpu")
    for a in ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity"):
        assert torch.equal(getattr(m, a).detach(), getattr(m2, a).detach()), a
    names = m.construct_list_of_attributes()
    assert names[:6] == ['x', 'y', 'z', 'nx', 'ny', 'nz'] and names[-4:] == ['rot_0', 'rot_1', 'rot_2', 'rot_3']
    assert len(names) == 6 + 3 + 45 + 1 + 3 + 4


def test_deform_network_state_dict_keys():
    """state_dict keys/shapes identical to DeformNetworkBaseline (time_utils.py:56-100) so deform.pth
    checkpoints interchange; construction needs no GPU."""
    from deformgs.deform_network import DeformNetworkBaseline
    from oracle import mlp_ref
    for bl, d6 in ((True, False), (False, False), (True, True)):
        net = DeformNetworkBaseline(is_blender=bl, is_6dof=d6)
        got = [(k, tuple(v.shape)) for k, v in net.state_dict().items()]
        exp = list(mlp_ref.param_shapes(bl, d6).items())
        assert sorted(got) == sorted(exp)
        assert len(net.kernel_params()) == len(exp)
    with pytest.raises(NotImplementedError):
        DeformNetworkBaseline(W=128)


def test_loss_kernel_window_matches_reference_window_total():
    """The fused loss filters separably (csrc/ssim.hip make_window): its taps must stay within a few
    fp32 ulps of the reference's 1-D Gaussian (loss_utils.py:30-39 via deformgs.loss, which mirrors it)
    and the total of their exact outer product must equal the total of the reference's fp32-rounded
    2-D window (the SSIM normalisation a near-render target is sensitive to) to 1e-10."""
    import ctypes

    import numpy as np
    import torch

    from deformgs import _lib
    from deformgs.loss import create_window, gaussian
    out = (ctypes.c_float * 11)()
    _lib.load().dgs_l1_ssim_window(out)
    w = np.array(out[:], np.float32)
    ref1 = gaussian(11, 1.5).numpy().astype(np.float32)
    ulps = np.abs(w.view(np.int32).astype(np.int64) - ref1.view(np.int32).astype(np.int64))
    assert ulps.max() <= 4, ulps
    assert np.array_equal(w, w[::-1])  # symmetric: the backward applies the same taps
    S2 = create_window(11, 1, torch.device("cpu"), torch.float32).double().sum().item()
    assert abs(w.astype(np.float64).sum() ** 2 - S2) < 1e-10, (w.astype(np.float64).sum() ** 2, S2)

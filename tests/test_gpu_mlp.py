"""Fused HIP deformation MLP vs the reference's own outputs (tests/golden/mlp_*.npz) and the
float64 numpy oracle (oracle/mlp_ref.py) at larger, ragged N.

Tolerance (fp32 MFMA, exact fma chains, vs a float64 oracle / the reference's fp32 CPU run):
outputs |err| <= 2e-5 + 1e-4 |ref|; parameter gradients within 1e-4 relative to each tensor's
max (or to its sketch scale for the projected fixtures).
"""
import numpy as np
import pytest
import torch

from oracle import mlp_ref
from weights import mlp_weights, proj_mats

pytestmark = pytest.mark.gpu

VARIANTS = {"blender": (True, False, False), "nonblender": (False, False, False), "6dof": (True, True, False),
            "fork": (True, False, True)}


def _net(name, seed):
    from deformgs.deform_network import DeformNetwork, DeformNetworkBaseline
    bl, d6, fork = VARIANTS[name]
    cls = DeformNetwork if fork else DeformNetworkBaseline
    net = cls(is_blender=bl, is_6dof=d6).cuda()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    w = mlp_weights(shapes, seed)
    net.load_state_dict({k: torch.from_numpy(a) for k, a in w.items()})
    return net, w


@pytest.mark.parametrize("name", list(VARIANTS))
def test_mlp_golden(name, golden_dir):
    f = np.load(f"{golden_dir}/mlp_{name}.npz")
    net, _ = _net(name, int(f["seed_w"]))
    x = torch.from_numpy(f["x"]).cuda()
    t = torch.from_numpy(f["t"]).cuda()
    d_xyz, d_rot, d_scale = net(x, t)
    loss = (d_xyz * torch.from_numpy(f["g_xyz"]).cuda()).sum()
    assert np.allclose(d_xyz.detach().cpu().numpy(), f["d_xyz"], atol=2e-5, rtol=1e-4)
    if torch.is_tensor(d_rot):
        assert np.allclose(d_rot.detach().cpu().numpy(), f["d_rot"], atol=2e-5, rtol=1e-4)
        assert np.allclose(d_scale.detach().cpu().numpy(), f["d_scale"], atol=2e-5, rtol=1e-4)
        loss = loss + (d_rot * torch.from_numpy(f["g_rot"]).cuda()).sum() + (
            d_scale * torch.from_numpy(f["g_scale"]).cuda()).sum()
    loss.backward()
    for k, p in net.named_parameters():
        g = p.grad.cpu().numpy().astype(np.float64)
        if "grad." + k in f:
            ref = f["grad." + k]
            assert np.abs(g - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-6) + 1e-7, k
        elif "gproj." + k in f:
            r1, r2 = proj_mats(g.shape, 3000)
            pr = r1 @ g @ r2.T
            assert (np.abs(pr - f["gproj." + k]) <= 1e-4 * f["gabs." + k] + 1e-7).all(), k
        else:
            assert np.abs(g).max() == 0.0, k  # unused heads of the fork variant


def _times(rng, N, mode):
    if mode == "random":
        return rng.uniform(0, 1, (N, 1)).astype(np.float32)
    t = np.full((N, 1), 0.37, np.float32)  # one frame time (train_baseline.py:107-110)
    if mode == "mixed":  # a few 32-point blocks carry other times: per-point timenet there
        t[min(37, N - 1)] = 0.81
        t[N // 2:N // 2 + 40] = rng.uniform(0, 1, (min(40, N - N // 2), 1)).astype(np.float32)
    return t


@pytest.mark.parametrize("name,tmode", [("blender", "random"), ("nonblender", "random"), ("blender", "uniform"),
                                        ("blender", "mixed"), ("nonblender", "uniform")])
@pytest.mark.parametrize("N", [1, 63, 1000, 4099])
def test_mlp_vs_oracle_ragged(name, tmode, N):
    bl, d6, fork = VARIANTS[name]
    net, w = _net(name, 77)
    rng = np.random.default_rng(N)
    x = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
    t = _times(rng, N, tmode)
    out, c = mlp_ref.forward(w, x, t, bl, d6)
    d_xyz, d_rot, d_scale = net(torch.from_numpy(x).cuda(), torch.from_numpy(t).cuda())
    for a, b in ((d_xyz, out["d_xyz"]), (d_rot, out["d_rot"]), (d_scale, out["d_scale"])):
        assert np.allclose(a.detach().cpu().numpy(), b, atol=2e-5, rtol=1e-4)
    g = {k: rng.standard_normal(out[k].shape) for k in ("d_xyz", "d_rot", "d_scale")}
    loss = sum((v * torch.from_numpy(g[k]).float().cuda()).sum() for k, v in
               (("d_xyz", d_xyz), ("d_rot", d_rot), ("d_scale", d_scale)))
    loss.backward()
    gr = mlp_ref.backward(w, c, out, g, bl, d6)
    for k, p in net.named_parameters():
        ref = gr[k]
        got = p.grad.cpu().numpy()
        assert np.abs(got - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-6) + 1e-6, (k, N)


def test_mlp_deterministic_and_empty():
    net, _ = _net("blender", 5)
    x = torch.rand(3000, 3, device="cuda") * 2.6 - 1.3
    t = torch.full((3000, 1), 0.3, device="cuda")
    outs = []
    for _ in range(2):
        net.zero_grad()
        a, b, c = net(x, t)
        (a.sum() + b.square().sum() + c.sum()).backward()
        outs.append([p.grad.clone() for p in net.parameters()] + [a.detach().clone()])
    for u, v in zip(*outs):
        assert torch.equal(u, v), "fused MLP fwd+bwd must be bitwise reproducible"
    a, b, c = net(torch.zeros(0, 3, device="cuda"), torch.zeros(0, 1, device="cuda"))
    assert a.shape == (0, 3)
    with pytest.raises(NotImplementedError):
        net(x.requires_grad_(True), t)


def test_expanded_time_input():
    # train_baseline.py:110 passes fid.unsqueeze(0).expand(N, -1) (stride 0)
    net, w = _net("blender", 9)
    x = torch.rand(500, 3, device="cuda")
    fid = torch.tensor([0.42], device="cuda")
    a = net(x, fid.unsqueeze(0).expand(500, -1))[0]
    b = net(x, torch.full((500, 1), 0.42, device="cuda"))[0]
    assert torch.equal(a, b)

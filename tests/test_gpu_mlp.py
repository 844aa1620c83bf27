"""Fused HIP deformation MLP vs the reference's own outputs (tests/golden/mlp_*.npz) and the
float64 numpy oracle (oracle/mlp_ref.py) at larger, ragged N, for both GEMM arithmetics: the default
split-f16 path (fp32 operands scaled by a power of two and split into hi / lo f16, three MFMA
products per fp32 product; round 6, rounds 1-5 ran a six-product bf16 split) and the exact
fp32-input MFMA path (DGS_MLP_EXACT_FP32).

Tolerance (either path, vs a float64 oracle / the reference's fp32 CPU run): outputs
|err| <= 2e-5 + 1e-4 |ref|; parameter gradients within 1e-4 relative to each tensor's max (or to
its sketch scale for the projected fixtures). test_split_accuracy_matches_fp32 additionally holds
the split path's error to within 2x the exact-fp32 path's error (plus 1e-6 absolute).

Oracle gradients at N >= 1000 use the kernel's own relu' masks (helpers.mlp_relu_masks): among
~10^7 pre-activations a few sit within an fp32 ulp of 0 and take either sign in any fp32 forward
(tests/diag/mlp_diag.py found one such flip at N = 4099), which swaps a whole dZ row; the forward outputs
are still compared with the oracle's own masks, and the golden tests use the reference's.
"""
import numpy as np
import pytest
import torch

from helpers import mlp_relu_masks
from oracle import mlp_ref
from weights import mlp_weights, proj_mats

pytestmark = pytest.mark.gpu

VARIANTS = {"blender": (True, False, False), "nonblender": (False, False, False), "6dof": (True, True, False),
            "fork": (True, False, True)}


ARITH = {"split": False, "exact": True}


def _net(name, seed, exact=False):
    from deformgs.deform_network import DeformNetwork, DeformNetworkBaseline
    bl, d6, fork = VARIANTS[name]
    cls = DeformNetwork if fork else DeformNetworkBaseline
    net = cls(is_blender=bl, is_6dof=d6, exact_fp32=exact).cuda()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    w = mlp_weights(shapes, seed)
    net.load_state_dict({k: torch.from_numpy(a) for k, a in w.items()})
    return net, w


@pytest.mark.parametrize("arith", list(ARITH))
@pytest.mark.parametrize("name", list(VARIANTS))
def test_mlp_golden(name, arith, golden_dir):
    f = np.load(f"{golden_dir}/mlp_{name}.npz")
    net, _ = _net(name, int(f["seed_w"]), ARITH[arith])
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
@pytest.mark.parametrize("arith", list(ARITH))
def test_mlp_vs_oracle_ragged(name, tmode, N, arith):
    bl, d6, fork = VARIANTS[name]
    net, w = _net(name, 77, ARITH[arith])
    rng = np.random.default_rng(N)
    x = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
    t = _times(rng, N, tmode)
    out, c = mlp_ref.forward(w, x, t, bl, d6)
    d_xyz, d_rot, d_scale = net(torch.from_numpy(x).cuda(), torch.from_numpy(t).cuda())
    # read before backward frees the saved activations; a one-element t (N = 1) runs DGS_MLP_UNIFORM_T
    masks = mlp_relu_masks(d_xyz, N, bl, ARITH[arith], th_saved=N > 1 or ARITH[arith])
    for a, b in ((d_xyz, out["d_xyz"]), (d_rot, out["d_rot"]), (d_scale, out["d_scale"])):
        assert np.allclose(a.detach().cpu().numpy(), b, atol=2e-5, rtol=1e-4)
    g = {k: rng.standard_normal(out[k].shape) for k in ("d_xyz", "d_rot", "d_scale")}
    loss = sum((v * torch.from_numpy(g[k]).float().cuda()).sum() for k, v in
               (("d_xyz", d_xyz), ("d_rot", d_rot), ("d_scale", d_scale)))
    loss.backward()
    gr = mlp_ref.backward(w, c, out, g, bl, d6, relu_masks=masks)
    for k, p in net.named_parameters():
        ref = gr[k]
        got = p.grad.cpu().numpy()
        assert np.abs(got - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-6) + 1e-6, (k, N)


@pytest.mark.parametrize("arith", list(ARITH))
def test_mlp_deterministic_and_empty(arith):
    net, _ = _net("blender", 5, ARITH[arith])
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
    # the stride-0 column runs DGS_MLP_UNIFORM_T (t_emb folded into the biases): fp32 rounding apart
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()))


@pytest.mark.parametrize("name,N", [("blender", 20000), ("nonblender", 20000), ("6dof", 20000), ("fork", 20000),
                                    ("blender", 100000)])
def test_split_accuracy_matches_fp32(name, N):
    """The split-f16 GEMMs are as accurate as fp32 MFMA: max error vs the float64 oracle within 2x
    the exact path's (every kernel output and every parameter gradient), at N = 20000 (ragged: 312.5
    blocks) and N = 100000. The upstream gradient is given on the kernel's raw outputs (for 6-DoF: w, v before
    exp_se3, whose 1/|w| amplifies any fp32 difference; that chain is checked by test_mlp_golden).
    N = 100000 is the bench size: each dW workgroup then sums ~3000-point ranges of fresh 32-point
    accumulators (k_dws)."""
    bl, d6, fork = VARIANTS[name]
    rng = np.random.default_rng(11)
    x = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
    t = np.full((N, 1), 0.61, np.float32)
    nout = 13 if d6 else 10
    G = rng.standard_normal((N, nout))
    if fork:
        G[:, 3:] = 0.0  # rotation / scaling heads are unused by the fork variant
    errs = {}
    for arith in ARITH:
        net, w = _net(name, 123, ARITH[arith])
        out, c = mlp_ref.forward(w, x, t, bl, d6)
        ref_raw = np.concatenate([out["w_raw"], out["v_raw"]] if d6 else [out["d_xyz"]], 1)
        if not fork:
            ref_raw = np.concatenate([ref_raw, out["d_rot"], out["d_scale"]], 1)
        raw = net.raw(torch.from_numpy(x).cuda(), torch.from_numpy(t).cuda())
        masks = mlp_relu_masks(raw, N, bl, ARITH[arith])
        e = {"out": np.abs(raw.detach().cpu().numpy()[:, :ref_raw.shape[1]] - ref_raw).max()}
        (raw * torch.from_numpy(G).float().cuda()).sum().backward()
        if d6:
            g = {"w_raw": G[:, 0:3], "v_raw": G[:, 3:6], "d_rot": G[:, 6:10], "d_scale": G[:, 10:13]}
        else:
            g = {"d_xyz": G[:, 0:3], "d_rot": G[:, 3:7], "d_scale": G[:, 7:10]}
        ref_g = mlp_ref.backward(w, c, out, g, bl, d6, fork, relu_masks=masks)
        for k, p in net.named_parameters():
            if k in ref_g:
                e[k] = np.abs(p.grad.cpu().numpy() - ref_g[k]).max()
        errs[arith] = e
    for k in errs["exact"]:
        assert errs["split"][k] <= 2.0 * errs["exact"][k] + 1e-6, (k, errs["split"][k], errs["exact"][k])


def _bench_regime():
    """Inputs of bench.py's step at its own configuration (tests/test_gpu_step_parity.py bench-100k):
    synth-100k (seed 0) at 800^2, blender network (mlp_weights seed 4, heads at 1/100), camera 1 (fid
    1/30), target = that camera's initial render + N(0, 0.02), clamped. Returns (weights, xyz, t0, G)
    with G = dL/d(raw network output), the upstream gradient the fused L1 + SSIM loss and the rasterizer
    backward hand the network there: against a near-render target its per-point terms nearly cancel in
    every dW sum, which is the regime the step-parity bar at bench size exercises."""
    from deformgs.arguments import PipelineParams
    from deformgs.deform_network import DeformNetworkBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.loss import l1_ssim_loss
    from deformgs.renderer import render
    from deformgs.synthetic import synth_camera, synth_gaussians
    from weights import mlp_weights
    dev = torch.device("cuda", 0)
    N = 100_000
    g = synth_gaussians(N, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    net = DeformNetworkBaseline(is_blender=True).cuda()
    w = mlp_weights(mlp_ref.param_shapes(True, False), seed=4)
    for k in w:
        if k.startswith(("gaussian_warp", "gaussian_rotation", "gaussian_scaling")):
            w[k] = (w[k] * 0.01).astype(np.float32)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    cam = synth_camera(800, 800, index=1, fid=1.0 / 30.0, device=dev)
    pipe, bg = PipelineParams(), torch.zeros(3, device=dev)
    x = gs.get_xyz.detach()
    t = cam.fid.unsqueeze(0).expand(N, -1)
    with torch.no_grad():
        r0 = net.raw(x, t)
        img0 = render(cam, gs, pipe, bg, r0[:, 0:3], r0[:, 3:7], r0[:, 7:10])["render"]
        noise = torch.randn(img0.shape, generator=torch.Generator().manual_seed(101)).to(dev)
        gt = (img0 + 0.02 * noise).clamp_(0.0, 1.0).contiguous()
        del r0, img0
    raw = net.raw(x, t)
    raw.retain_grad()
    img = render(cam, gs, pipe, bg, raw[:, 0:3], raw[:, 3:7], raw[:, 7:10])["render"]
    loss, _, _ = l1_ssim_loss(img, gt)
    loss.backward()
    G = raw.grad.detach().double().cpu().numpy()
    t0 = float(cam.fid.item())
    del net, gs, raw, img
    torch.cuda.empty_cache()
    return w, x.cpu().numpy(), t0, G


def test_split_accuracy_bench_regime():
    """the default GEMM arithmetic against the fp32-MFMA path at the benchmarked
    configuration. The network-output gradient of bench.py's own step (_bench_regime: a near-render
    target, so every dW sum over the 100k points nearly cancels) is fed to both arithmetics on the
    kernels the bench runs (stride-0 frame time: the folded-t_emb forward, the dX chain, k_dws / k_dw,
    k_tgrad); every kernel output and every parameter gradient must be within 2x the fp32-MFMA path's
    max error against the float64 oracle (plus 1e-12 absolute). Both errors are recorded
    (gpurun_out/parity_stats.jsonl -> profiles/)."""
    from helpers import write_stats
    w, x, t0, G = _bench_regime()
    N = x.shape[0]
    out, c = mlp_ref.forward(w, x, np.full((N, 1), t0, np.float32), True, False)
    ref_raw = np.concatenate([out["d_xyz"], out["d_rot"], out["d_scale"]], 1)
    errs, scale = {}, {}
    for arith in ARITH:
        net = _net_from(w, ARITH[arith])
        tt = torch.full((1, 1), t0, device="cuda").expand(N, -1)
        raw = net.raw(torch.from_numpy(x).cuda(), tt)
        masks = mlp_relu_masks(raw, N, True, ARITH[arith], th_saved=ARITH[arith])
        e = {"out": float(np.abs(raw.detach().cpu().numpy() - ref_raw).max())}
        (raw * torch.from_numpy(G).float().cuda()).sum().backward()
        ref_g = mlp_ref.backward(w, c, out, _raw_grads(G, False, False), True, False, relu_masks=masks)
        for k, p in net.named_parameters():
            if k in ref_g:
                e[k] = float(np.abs(p.grad.cpu().numpy() - ref_g[k]).max())
                scale[k] = float(np.abs(ref_g[k]).max())
        errs[arith] = e
        del net, raw
    write_stats("mlp_split_accuracy_bench_regime", {"split": errs["split"], "exact": errs["exact"],
                                                     "ref_max": scale})
    for k in errs["exact"]:
        assert errs["split"][k] <= 2.0 * errs["exact"][k] + 1e-12, (k, errs["split"][k], errs["exact"][k])


def _net_from(w, exact):
    from deformgs.deform_network import DeformNetworkBaseline
    net = DeformNetworkBaseline(is_blender=True, exact_fp32=exact).cuda()
    net.load_state_dict({k: torch.from_numpy(a) for k, a in w.items()})
    return net


def _raw_grads(G, d6, fork):
    if d6:
        return {"w_raw": G[:, 0:3], "v_raw": G[:, 3:6], "d_rot": G[:, 6:10], "d_scale": G[:, 10:13]}
    return {"d_xyz": G[:, 0:3], "d_rot": G[:, 3:7], "d_scale": G[:, 7:10]}


@pytest.mark.parametrize("name", ["blender", "6dof", "nonblender", "fork"])
@pytest.mark.parametrize("N", [63, 4099])
def test_uniform_t_flag(name, N):
    """A stride-0 time column (train_baseline.py:107-110) sets DGS_MLP_UNIFORM_T: the backward skips
    the per-point t_emb GEMMs and k_tgrad forms the timenet gradients from the layer-0/5 bias
    gradients. On a blender network the uniform path also folds t_emb into the linear.0 / linear.5
    biases (k_timenet's C0 / C5; the forward GEMMs and dW then cover x_emb | h only and k_tgrad writes
    the t_emb weight columns), so its outputs equal the per-point path's to fp32 rounding (1e-5
    relative + 1e-6 of the largest output), bit for bit otherwise; gradients match the oracle (1e-4
    of each tensor's max) and the per-point path."""
    bl, d6, fork = VARIANTS[name]
    rng = np.random.default_rng(N + 1)
    x = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
    t0 = 0.43
    xt = torch.from_numpy(x).cuda()
    G = rng.standard_normal((N, 13 if d6 else 10))
    if fork:
        G[:, 3:] = 0.0
    res = {}
    for mode in ("expanded", "full"):
        net, w = _net(name, 31)
        tt = torch.full((1, 1), t0, device="cuda").expand(N, -1) if mode == "expanded" else \
            torch.full((N, 1), t0, device="cuda")
        raw = net.raw(xt, tt)
        masks = mlp_relu_masks(raw, N, bl, False, th_saved=mode == "full")
        (raw * torch.from_numpy(G).float().cuda()).sum().backward()
        res[mode] = (raw.detach().clone(), {k: p.grad.clone() for k, p in net.named_parameters()}, masks)
    if bl:  # folded t_emb: a different fp32 summation order for linear.0 / linear.5
        a, b = res["expanded"][0], res["full"][0]
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max())), float((a - b).abs().max())
    else:
        assert torch.equal(res["expanded"][0], res["full"][0])
    out, c = mlp_ref.forward(w, x, np.full((N, 1), t0, np.float32), bl, d6)
    ref = mlp_ref.backward(w, c, out, _raw_grads(G, d6, fork), bl, d6, fork, relu_masks=res["expanded"][2])
    for k, g in res["expanded"][1].items():
        got = g.cpu().numpy()
        if k not in ref:
            assert np.abs(got).max() == 0.0, k
            continue
        tol = 1e-4 * max(np.abs(ref[k]).max(), 1e-6) + 1e-6
        assert np.abs(got - ref[k]).max() <= tol, (k, np.abs(got - ref[k]).max(), tol)
        assert np.abs(got - res["full"][1][k].cpu().numpy()).max() <= 2 * tol, k


def test_tail_blocks_bitwise_equal_64_point_blocks(tmp_path):
    """The fused forward / dX kernels run the sparse last round of 64-point blocks as 16-point
    blocks (mlp_split.hip block_split); every output and parameter gradient must equal the all-64-
    point decomposition (DGS_MLP_NO_TAIL=1, read once per process) bit for bit. (Round 6: every
    operand scale of the split-f16 GEMMs is per 16-point column tile, so this still holds.)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(root, "tools", "tail_check.py")
    outs = []
    for env_val in ("0", "1"):
        out = str(tmp_path / f"tail_{env_val}.npz")
        env = dict(os.environ, DGS_MLP_NO_TAIL=env_val)
        subprocess.run([sys.executable, script, out], check=True, env=env, timeout=300)
        outs.append(np.load(out))
    a, b = outs
    assert set(a.files) == set(b.files) and len(a.files) > 0
    for k in a.files:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_dw_linearity_past_32bit_operand_offsets():
    """Maximum size: at N = 2,150,016 points one 256-row dW operand spans more than 2^31 bytes, so the
    split k_dws (32-bit buffer offsets) hands the dW to the fp32 fallback (mlp_split.hip dw_split_once ->
    mlp::dw_fp32). Size-independent check of that path: the forward is per point (per 16-point column
    tile scales: a half split on a tile boundary computes bitwise the same rows), and every parameter
    gradient is a sum over points, so the full launch must equal the two halves' (each below the limit,
    on k_dws) to fp32 summation error: 1e-4 of each tensor's max."""
    net, _ = _net("blender", 11)
    N = 2_150_016
    gen = torch.Generator(device="cpu").manual_seed(21)
    x = (torch.rand((N, 3), generator=gen) * 2 - 1).cuda()
    G = torch.randn((N, 10), generator=gen).cuda()
    t = torch.full((1, 1), 0.37, device="cuda")

    def run(xs, gs):
        net.zero_grad(set_to_none=True)
        raw = net.raw(xs, t.expand(xs.shape[0], -1))
        (raw * gs).sum().backward()
        torch.cuda.synchronize()
        return raw.detach(), {k: p.grad.detach().clone() for k, p in net.named_parameters()}

    from deformgs import _lib
    lib = _lib.load()
    f0 = lib.dgs_debug_dw_fallbacks()
    raw_full, g_full = run(x, G)
    assert lib.dgs_debug_dw_fallbacks() == f0 + 1, "the full launch must take the fp32 dW fallback"
    h = N // 2
    raw_a, g_a = run(x[:h].contiguous(), G[:h].contiguous())
    raw_b, g_b = run(x[h:].contiguous(), G[h:].contiguous())
    assert lib.dgs_debug_dw_fallbacks() == f0 + 1, "the halves run k_dws"
    assert torch.equal(raw_full, torch.cat([raw_a, raw_b]))
    for k, gf in g_full.items():
        want = g_a[k] + g_b[k]
        tol = 1e-4 * float(want.abs().max())
        assert float((gf - want).abs().max()) <= tol, (k, float((gf - want).abs().max()), tol)

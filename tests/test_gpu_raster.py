"""HIP rasterizer (libdgs_hip.so through the drop-in diff_gaussian_rasterization) vs the C oracle.

Tolerances (floating point, stated per test): the forward image must match the oracle to a mean
absolute error <= 1e-5 (the north star's bar is 1e-4 L1) with >= 99.9 % of pixels within 1e-4;
gradients are compared with a per-tensor relative tolerance because float atomics sum in arrival
order and a Gaussian whose alpha sits exactly on the 1/255 or T<1e-4 thresholds can flip between
fp32 implementations (exp differs by an ulp). Parity of the rasterizer is UNPINNED by the reference
(no CUDA op, no fixture); the oracle is the spec (oracle/raster_ref.c header).
"""
import numpy as np
import pytest
import torch

from helpers import (check_gaussian_grad, check_image, check_integer_outputs, frac_close, oracle_run, rel_err, scene,
                     settings_for_gpu, tail_sets, write_stats)

pytestmark = pytest.mark.gpu

CONFIGS = [
    # N, H, W, cam, scale_boost, bg
    (5000, 256, 256, 0, 0.0, (0.0, 0.0, 0.0)),      # config 1: 5k @ 256^2
    (2000, 61, 83, 3, 1.0, (0.2, 0.5, 0.9)),        # ragged image, big Gaussians, coloured bg
    (3000, 128, 96, 5, 0.5, (1.0, 1.0, 1.0)),
]


@pytest.fixture(params=["rect", "sort"])
def binning(request):
    """Both tile binnings: rect (count -> column scan -> place, the default) and sort (duplicate +
    tile-key radix sort + ranges, the upstream scheme). Restores the default afterwards."""
    from deformgs import _lib
    lib = _lib.load()
    lib.dgs_debug_set_binning(0 if request.param == "rect" else 1)
    yield request.param
    lib.dgs_debug_set_binning(0)


def _run_gpu(inputs, rs, dcolor, ddepth, use_cov=False, use_colors=False, requires=True):
    from diff_gaussian_rasterization import GaussianRasterizer
    dev = "cuda"
    t = {k: v.to(dev).clone().requires_grad_(requires) for k, v in inputs.items()}
    N = t["means3D"].shape[0]
    m2 = torch.zeros((N, 3), device=dev, requires_grad=True)
    m2d = torch.zeros((N, 3), device=dev, requires_grad=True)
    r = GaussianRasterizer(settings_for_gpu(rs))
    kw = dict(means3D=t["means3D"], means2D=m2, means2D_densify=m2d, opacities=t["opacities"])
    if use_colors:
        kw["colors_precomp"] = t["colors"]
    else:
        kw["shs"] = t["shs"]
    if use_cov:
        kw["cov3D_precomp"] = t["cov3D"]
    else:
        kw["scales"] = t["scales"]
        kw["rotations"] = t["rotations"]
    color, radii, depth = r(**kw)
    _run_gpu.num_rendered = int(color.grad_fn.num_rendered)
    loss = (color * torch.tensor(dcolor, device=dev)).sum()
    if ddepth is not None:
        loss = loss + (depth * torch.tensor(ddepth, device=dev)).sum()
    loss.backward()
    grads = {k: v.grad.cpu().numpy() for k, v in t.items()}
    grads["means2D"] = m2.grad.cpu().numpy()
    grads["means2D_densify"] = m2d.grad.cpu().numpy()
    return color.detach().cpu().numpy(), radii.cpu().numpy(), depth.detach().cpu().numpy(), grads


def _check(o, g, color, radii, depth, grads, keys, nr=None, tag=None):
    """radii exact and num_rendered equal to the oracle's (up to fp32-ambiguous ceil / rect / cull
    decisions, helpers.check_integer_outputs); image mean |err| <= 1e-5 and >= 99.9 % within 1e-4,
    every larger error at a pixel with a near-threshold blend decision; gradients: tolerance 2e-3 of
    the max + 1e-3 relative, at most 1e-4 of the elements outside it, every such element on a Gaussian
    with a decision within 1e-5 of its threshold (helpers.tail_sets), none beyond 10x the tolerance
    (helpers.check_gaussian_grad)."""
    stats = {}
    try:
        amb = check_integer_outputs(o, radii, nr, stats)
        sets = tail_sets(o, amb)
        check_image(color, o, sets, stats)
        derr = np.abs(depth - o.depth)
        assert (derr <= 1e-4 * max(1.0, np.abs(o.depth).max())).mean() >= 0.999
        for k, ok in keys:
            check_gaussian_grad(grads[k], g[ok], sets, k, stats)
    finally:
        if tag:
            write_stats(tag, stats)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_raster_sh_scale_rot(cfg, binning):
    N, H, W, ci, boost, bg = cfg
    inputs, rs, _ = scene(N, H, W, cam_index=ci, scale_boost=boost, bg=bg)
    rng = np.random.default_rng(1)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    ddepth = rng.standard_normal((1, H, W)).astype(np.float32) * 0.1
    o, g = oracle_run(inputs, rs, dcolor, ddepth)
    color, radii, depth, grads = _run_gpu(inputs, rs, dcolor, ddepth)
    _check(o, g, color, radii, depth, grads,
           [("means3D", "means3D"), ("shs", "shs"), ("opacities", "opacities"), ("scales", "scales"),
            ("rotations", "rotations"), ("means2D", "means2D"), ("means2D_densify", "means2D_densify")],
           nr=_run_gpu.num_rendered, tag=f"raster_sh_scale_rot[{N}x{H}x{W},{binning}]")


def test_raster_precomputed_colors_and_cov():
    N, H, W = 1500, 80, 112
    inputs, rs, _ = scene(N, H, W, cam_index=2, scale_boost=0.7)
    from deformgs.general import build_scaling_rotation, strip_symmetric
    L = build_scaling_rotation(inputs["scales"], inputs["rotations"])
    inputs["cov3D"] = strip_symmetric(L @ L.transpose(1, 2))
    inputs["colors"] = torch.rand((N, 3), generator=torch.Generator().manual_seed(3))
    rng = np.random.default_rng(2)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    sub = {k: inputs[k] for k in ("means3D", "opacities", "cov3D", "colors")}
    o, g = oracle_run(inputs, rs, dcolor, None, use_cov=True, use_colors=True)
    color, radii, depth, grads = _run_gpu(sub, rs, dcolor, None, use_cov=True, use_colors=True)
    _check(o, g, color, radii, depth, grads,
           [("means3D", "means3D"), ("opacities", "opacities"), ("cov3D", "cov3D"), ("colors", "colors")],
           nr=_run_gpu.num_rendered, tag="raster_precomputed")


def test_raster_sh_degrees():
    for deg in range(4):
        inputs, rs, _ = scene(800, 64, 64, cam_index=1, scale_boost=0.8, sh_degree=deg)
        rng = np.random.default_rng(deg)
        dcolor = rng.standard_normal((3, 64, 64)).astype(np.float32)
        o, g = oracle_run(inputs, rs, dcolor, None)
        color, radii, depth, grads = _run_gpu(inputs, rs, dcolor, None)
        _check(o, g, color, radii, depth, grads, [("shs", "shs"), ("means3D", "means3D")], nr=_run_gpu.num_rendered,
               tag=f"raster_sh_degree{deg}")


def test_raster_edge_cases():
    from diff_gaussian_rasterization import GaussianRasterizer
    # everything behind the camera (culled): image = background, radii 0, zero grads
    inputs, rs, _ = scene(300, 40, 40, cam_index=0, bg=(0.3, 0.2, 0.1))
    view = rs["viewmatrix"]
    cam_center = rs["campos"]
    behind = cam_center[None] * 1.5 + 0.01 * inputs["means3D"]
    inputs["means3D"] = behind
    dcolor = np.ones((3, 40, 40), np.float32)
    color, radii, depth, grads = _run_gpu(inputs, rs, dcolor, None)
    o, g = oracle_run(inputs, rs, dcolor, None)
    assert (radii == 0).all() and (o.radii == 0).all()
    assert np.allclose(color, o.color) and np.allclose(color[0], 0.3)
    assert np.abs(grads["means3D"]).max() == 0.0
    # empty input
    r = GaussianRasterizer(settings_for_gpu(rs))
    z = torch.zeros((0, 3), device="cuda", requires_grad=True)
    c, rad, d = r(means3D=z, means2D=torch.zeros((0, 3), device="cuda"), opacities=torch.zeros((0, 1), device="cuda"),
                  shs=torch.zeros((0, 16, 3), device="cuda"), scales=torch.zeros((0, 3), device="cuda"),
                  rotations=torch.zeros((0, 4), device="cuda"))
    assert rad.numel() == 0 and torch.allclose(c[1], torch.full_like(c[1], 0.2))
    # argument validation matches upstream (Exception on bad combination)
    with pytest.raises(Exception):
        r(means3D=z, means2D=z, opacities=z)


def test_mark_visible():
    from diff_gaussian_rasterization import GaussianRasterizer
    inputs, rs, _ = scene(1000, 32, 32, cam_index=4)
    r = GaussianRasterizer(settings_for_gpu(rs))
    vis = r.markVisible(inputs["means3D"].cuda()).cpu().numpy()
    p = torch.cat([inputs["means3D"], torch.ones(1000, 1)], 1) @ rs["viewmatrix"]
    assert (vis == (p[:, 2] > 0.2).numpy()).all()


def _forward_only(inputs, rs, debug):
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    st = settings_for_gpu(rs)._replace(debug=debug)
    t = {k: v.cuda() for k, v in inputs.items()}
    N = t["means3D"].shape[0]
    with torch.no_grad():
        color, radii, depth = GaussianRasterizer(st)(
            means3D=t["means3D"], means2D=torch.zeros((N, 3), device="cuda"),
            means2D_densify=torch.zeros((N, 3), device="cuda"), shs=t["shs"], opacities=t["opacities"],
            scales=t["scales"], rotations=t["rotations"])
    return color.cpu().numpy(), radii.cpu().numpy(), depth.cpu().numpy()


def test_speculative_binning_matches_exact():
    """Binning runs for a speculative pair capacity learned from earlier frames; a frame with far
    more pairs overflows it and is re-binned. Both must equal the exact (debug: synchronous,
    num_rendered-sized) path bit for bit, since the sort is stable and the padding sorts last."""
    small, rs_s, _ = scene(500, 64, 64, seed=3, cam_index=1)
    big, rs_b, _ = scene(4000, 200, 160, seed=4, cam_index=2, scale_boost=1.5)
    for inputs, rs in [(small, rs_s), (small, rs_s), (big, rs_b), (big, rs_b), (small, rs_s)]:
        a = _forward_only(inputs, rs, debug=False)
        b = _forward_only(inputs, rs, debug=True)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    o, _ = oracle_run(big, rs_b)
    c, r, d = _forward_only(big, rs_b, debug=False)
    assert np.abs(c - o.color).mean() <= 1e-5


def test_speculative_overflow_redo_is_exact(binning):
    """Force the overflow path: the per-device pair capacity is overridden with a small value that
    is not a multiple of 256 (so the ranges/sort grids overhang it), and with a capacity left over
    from a much larger frame (stale keys past the new pairs). Every forced overflow must be redone
    (debug counter) and equal the synchronous exact path bit for bit."""
    from deformgs import _lib
    lib = _lib.load()
    dev = torch.cuda.current_device()
    big, rs_b, _ = scene(4000, 200, 160, seed=4, cam_index=2, scale_boost=1.5)  # ~45k pairs
    small, rs_s, _ = scene(1500, 96, 80, seed=3, cam_index=1, scale_boost=0.8)  # ~3.7k pairs
    ref_big = _forward_only(big, rs_b, debug=True)
    ref_small = _forward_only(small, rs_s, debug=True)
    nr_small = _num_rendered(small, rs_s)
    assert nr_small > 2000, "the small scene must have enough pairs to overflow the capacities below"
    for cap in (1, 255, 1000 + 37, 5 * 256 + 129):
        for inputs, ref in ((big, ref_big), (small, ref_small)):
            lib.dgs_debug_set_pair_cap(dev, cap)
            before = lib.dgs_debug_binning_redos()
            out = _forward_only(inputs, rs_b if inputs is big else rs_s, debug=False)
            redone = lib.dgs_debug_binning_redos() - before
            torch.cuda.synchronize()
            for x, y in zip(out, ref):
                np.testing.assert_array_equal(x, y)
            assert redone == 1, f"cap={cap}: expected one overflow redo, saw {redone}"
    # a capacity far above the count (tail padded with all-ones keys), after the big frame
    lib.dgs_debug_set_pair_cap(dev, 3_000_000 + 77)
    out = _forward_only(small, rs_s, debug=False)
    for x, y in zip(out, ref_small):
        np.testing.assert_array_equal(x, y)
    # and the backward after an overflowing forward matches the exact path's backward
    lib.dgs_debug_set_pair_cap(dev, 999)
    g1 = _grads_of(big, rs_b, debug=False)
    g2 = _grads_of(big, rs_b, debug=True)
    for k in g1:
        np.testing.assert_allclose(g1[k], g2[k], rtol=1e-4, atol=1e-6 * max(1.0, np.abs(g2[k]).max()))


def _num_rendered(inputs, rs):
    from diff_gaussian_rasterization import GaussianRasterizer
    t = {k: v.cuda().requires_grad_(True) for k, v in inputs.items()}
    N = t["means3D"].shape[0]
    color, _, _ = GaussianRasterizer(settings_for_gpu(rs))(
        means3D=t["means3D"], means2D=torch.zeros((N, 3), device="cuda"), shs=t["shs"],
        opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
    return int(color.grad_fn.num_rendered)


def _grads_of(inputs, rs, debug):
    from diff_gaussian_rasterization import GaussianRasterizer
    st = settings_for_gpu(rs)._replace(debug=debug)
    t = {k: v.cuda().requires_grad_(True) for k, v in inputs.items()}
    N = t["means3D"].shape[0]
    color, radii, depth = GaussianRasterizer(st)(
        means3D=t["means3D"], means2D=torch.zeros((N, 3), device="cuda"),
        means2D_densify=torch.zeros((N, 3), device="cuda"), shs=t["shs"], opacities=t["opacities"],
        scales=t["scales"], rotations=t["rotations"])
    w = torch.linspace(-1, 1, color.numel(), device="cuda").reshape(color.shape)
    (color * w).sum().backward()
    return {k: v.grad.cpu().numpy() for k, v in t.items()}


@pytest.mark.parametrize("case", [
    # N, H, W, cam, scale_boost: small Gaussians, ragged tiles, big Gaussians (rects of many tiles),
    # a wide image (2772 tiles), more Gaussians than one count block column (> 256 blocks)
    (3000, 128, 96, 5, 0.0), (2000, 61, 83, 3, 1.0), (1500, 100, 120, 2, 3.0), (5000, 700, 1000, 0, 0.5),
    (150000, 160, 160, 1, 0.0)])
def test_rect_binning_equals_sort_binning(case):
    """The rect binning places every (tile, Gaussian) pair where the stable tile sort of the depth-
    ordered pairs puts it, so images, depth, radii, the pair count and every gradient must equal the
    sort binning's bit for bit (same pair lists -> same blend order -> same float sums; gradient
    atomics can differ in arrival order, so gradients are compared to 1e-5 relative)."""
    from deformgs import _lib
    lib = _lib.load()
    N, H, W, ci, boost = case
    inputs, rs, _ = scene(N, H, W, cam_index=ci, scale_boost=boost, seed=11)
    out = {}
    try:
        for mode in (1, 0):
            lib.dgs_debug_set_binning(mode)
            out[mode] = (_forward_only(inputs, rs, debug=False), _forward_only(inputs, rs, debug=True),
                         _num_rendered(inputs, rs), _grads_of(inputs, rs, debug=False))
    finally:
        lib.dgs_debug_set_binning(0)
    (fs, fsd, ns, gs), (fr, frd, nr, gr) = out[1], out[0]
    assert ns == nr and nr > 0
    for a, b in zip(fs + fsd, fr + frd):
        np.testing.assert_array_equal(a, b)
    for k in gs:
        np.testing.assert_allclose(gr[k], gs[k], rtol=1e-5, atol=1e-6 * max(1.0, np.abs(gs[k]).max()))


def test_deferred_count_redo_matches_sync(binning):
    """Deferred pair count: a forced overflow (tiny speculative capacity) is detected at the
    backward, counted, stays in bounds, and the redone step equals a synchronous step; without
    overflow the deferred step equals the synchronous one outright."""
    from deformgs import _lib
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import deferred_overflowed, drop_grads, forward_backward
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g = synth_gaussians(6000, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    gs.training_setup(OptimizationParams())
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    deform.train_setting(OptimizationParams())
    cam = synth_camera(160, 128, index=2, fid=0.3, device=dev)
    gt = torch.rand((3, 128, 160), device=dev)
    params = [gs._xyz, gs._features_dc, gs._features_rest, gs._scaling, gs._rotation, gs._opacity] + \
        list(deform.deform.parameters())

    def run(deferred):
        drop_grads(gs, deform)
        loss, pkg = forward_backward(gs, deform, cam, gt, PipelineParams(), torch.zeros(3, device=dev),
                                     deferred_count=deferred)
        torch.cuda.synchronize()
        return loss.item(), pkg["render"].detach().clone(), [p.grad.clone() for p in params]

    ref = run(False)
    # no overflow (capacity learned from the synchronous frame)
    got = run(True)
    assert not deferred_overflowed()
    assert got[0] == ref[0] and torch.equal(got[1], ref[1])
    for a, b in zip(got[2], ref[2]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6 * max(1.0, b.abs().max().item()))
    # forced overflow: detected, then the synchronous redo equals the reference
    lib.dgs_debug_set_pair_cap(dev.index, 777)
    run(True)
    assert deferred_overflowed()
    redo = run(False)
    assert redo[0] == ref[0] and torch.equal(redo[1], ref[1])
    for a, b in zip(redo[2], ref[2]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6 * max(1.0, b.abs().max().item()))


def test_two_streams_at_once_match_sequential():
    """Two renders in flight on two HIP streams (two rasterizer contexts, both sorting at once) equal
    the same renders run one after the other: the radix / compaction scratch is per stream."""
    a_in, rs_a, _ = scene(20000, 320, 240, seed=21, cam_index=1)
    b_in, rs_b, _ = scene(15000, 200, 280, seed=22, cam_index=4, scale_boost=0.5)
    for binning_mode in (0, 1):
        from deformgs import _lib
        lib = _lib.load()
        lib.dgs_debug_set_binning(binning_mode)
        try:
            ref_a = _forward_only(a_in, rs_a, debug=False)
            ref_b = _forward_only(b_in, rs_b, debug=False)
            s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
            torch.cuda.synchronize()
            for _ in range(3):
                with torch.cuda.stream(s1):
                    got_a = _forward_only(a_in, rs_a, debug=False)
                with torch.cuda.stream(s2):
                    got_b = _forward_only(b_in, rs_b, debug=False)
                torch.cuda.synchronize()
                for x, y in zip(got_a + got_b, ref_a + ref_b):
                    np.testing.assert_array_equal(x, y)
        finally:
            lib.dgs_debug_set_binning(0)


def test_shrinking_point_sets_reuse_contexts_exactly():
    """Frames whose Gaussian count shrinks (prune) and grows again reuse pooled contexts with
    smaller / larger count matrices; every frame equals the synchronous exact (debug) path, which
    runs no speculative binning. (The rect binning's tagged tile totals live in their own zeroed
    buffer: a stale count-matrix word can never carry the current generation tag.)"""
    sizes = [150000, 40000, 3000, 90000, 500, 150000]
    for n in sizes:
        inp, rs, _ = scene(n, 256, 256, seed=n % 97, cam_index=n % 5)
        a = _forward_only(inp, rs, debug=False)
        b = _forward_only(inp, rs, debug=True)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def test_second_backward_recomputes_not_doubles():
    """A kept context (retain_graph + _KEEP_CTX) backpropagated twice gives the same gradients twice
    (the accumulators are re-zeroed, not added onto); without the kept context the second backward
    raises instead of reading a released context."""
    import diff_gaussian_rasterization as dgr
    inputs, rs, _ = scene(3000, 96, 96, seed=5, cam_index=2)
    t = {k: v.cuda().requires_grad_(True) for k, v in inputs.items()}
    N = t["means3D"].shape[0]
    from diff_gaussian_rasterization import GaussianRasterizer
    dgr._KEEP_CTX["on"] = True
    try:
        color, _, _ = GaussianRasterizer(settings_for_gpu(rs))(
            means3D=t["means3D"], means2D=torch.zeros((N, 3), device="cuda"), shs=t["shs"],
            opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
        w = torch.linspace(-1, 1, color.numel(), device="cuda").reshape(color.shape)
        (color * w).sum().backward(retain_graph=True)
        g1 = t["means3D"].grad.clone()
        t["means3D"].grad = None
        (color * w).sum().backward(retain_graph=True)
        torch.testing.assert_close(t["means3D"].grad, g1, rtol=1e-5, atol=1e-7 * float(g1.abs().max()))
        dgr.release_context(color)
    finally:
        dgr._KEEP_CTX["on"] = False
    color, _, _ = GaussianRasterizer(settings_for_gpu(rs))(
        means3D=t["means3D"], means2D=torch.zeros((N, 3), device="cuda"), shs=t["shs"],
        opacities=t["opacities"], scales=t["scales"], rotations=t["rotations"])
    color.sum().backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="second backward"):
        color.sum().backward()


def test_scale_gradient_conventions():
    """dL/dscales with scale_modifier != 1: the upstream convention (default; the oracle's) is the
    gradient w.r.t. the modified scale; dgs_raster_set_exact_scale_grad(1) multiplies it by the
    modifier (the chain rule). scale_modifier = 1.3 here."""
    from deformgs import _lib
    lib = _lib.load()
    inputs, rs, _ = scene(2000, 80, 96, seed=8, cam_index=3)
    rs = dict(rs, scale_modifier=1.3)
    rng = np.random.default_rng(4)
    dcolor = rng.standard_normal((3, 80, 96)).astype(np.float32)
    o, g = oracle_run(inputs, rs, dcolor, None)
    _, _, _, up = _run_gpu(inputs, rs, dcolor, None)
    assert frac_close(up["scales"], g["scales"], atol=2e-3 * np.abs(g["scales"]).max(), rtol=1e-3) >= 0.995
    lib.dgs_raster_set_exact_scale_grad(1)
    try:
        _, _, _, ex = _run_gpu(inputs, rs, dcolor, None)
    finally:
        lib.dgs_raster_set_exact_scale_grad(0)
    np.testing.assert_allclose(ex["scales"], up["scales"] * np.float32(1.3), rtol=1e-4,
                               atol=1e-6 * np.abs(up["scales"]).max())


@pytest.mark.parametrize("case", [
    # N, H, W, cam, scale_boost: config 1, ragged tiles with big Gaussians (long lists: many segments),
    # the bench workload
    (5000, 256, 256, 0, 0.0), (2000, 61, 83, 3, 1.0), (3000, 128, 96, 5, 2.0), (100_000, 800, 800, 0, 0.0)])
def test_segmented_blend_backward(case):
    """k_blend_bwd2s (dgs_debug_set_blend_seg(1)): every 128 list positions of every tile replayed as an
    independent work item from the forward's per-pixel (T, C) checkpoints. Same checks vs the oracle as
    every raster test (image, radii, pair count, gradients with their tails accounted for), and the
    gradients equal the serial replay's (k_blend_bwd2) to 1e-4 relative + 1e-6 of each tensor's max
    (float atomics in arrival order; T and the colour behind restart from the checkpoints)."""
    from deformgs import _lib
    lib = _lib.load()
    N, H, W, ci, boost = case
    inputs, rs, _ = scene(N, H, W, cam_index=ci, scale_boost=boost, seed=12)
    rng = np.random.default_rng(7)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    o, g = oracle_run(inputs, rs, dcolor, None)
    res = {}
    before = lib.dgs_debug_get_blend_seg()  # restored after (a session may run with DGS_BLEND_SEG=1)
    try:
        for seg in (0, 1):
            lib.dgs_debug_set_blend_seg(seg)
            res[seg] = _run_gpu(inputs, rs, dcolor, None) + (_run_gpu.num_rendered,)
    finally:
        lib.dgs_debug_set_blend_seg(before)
    color, radii, depth, grads, nr = res[1]
    for a, b in zip(res[1][:3], res[0][:3]):
        np.testing.assert_array_equal(a, b)  # the forward is the same with or without checkpoints
    _check(o, g, color, radii, depth, grads,
           [("means3D", "means3D"), ("shs", "shs"), ("opacities", "opacities"), ("scales", "scales"),
            ("rotations", "rotations"), ("means2D", "means2D"), ("means2D_densify", "means2D_densify")],
           nr=nr, tag=f"raster_segmented[{N}x{H}x{W}]")
    for k in grads:
        ref = res[0][3][k]
        np.testing.assert_allclose(grads[k], ref, rtol=1e-4, atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=k)


@pytest.mark.parametrize("case", [
    # N, H, W, cam, scale_boost, depth gradient: config 1, ragged tiles with big Gaussians, the bench workload
    (5000, 256, 256, 0, 0.0, False), (2000, 61, 83, 3, 1.0, True), (100_000, 800, 800, 0, 0.0, False)])
def test_deterministic_blend_backward(case):
    """dgs_raster_set_deterministic(1): k_blend_bwd2<DET> writes per-pair slots, k_rect_gather sums them
    per Gaussian in tile row-major order. Two forward + backward runs on the same inputs give
    bitwise-identical gradients; the oracle checks of every raster test hold; and the gradients equal the atomic path's to
    1e-4 relative + 1e-6 of each tensor's max (the same sums in another order)."""
    from deformgs.renderer import set_deterministic
    N, H, W, ci, boost, with_depth = case
    inputs, rs, _ = scene(N, H, W, cam_index=ci, scale_boost=boost, seed=13)
    rng = np.random.default_rng(9)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    ddepth = rng.standard_normal((1, H, W)).astype(np.float32) * 0.1 if with_depth else None
    o, g = oracle_run(inputs, rs, dcolor, ddepth)
    before = set_deterministic(True)
    try:
        r1 = _run_gpu(inputs, rs, dcolor, ddepth) + (_run_gpu.num_rendered,)
        r2 = _run_gpu(inputs, rs, dcolor, ddepth)
        set_deterministic(False)
        ra = _run_gpu(inputs, rs, dcolor, ddepth)
    finally:
        set_deterministic(before)
    color, radii, depth, grads, nr = r1
    for k in grads:
        np.testing.assert_array_equal(grads[k], r2[3][k], err_msg=k)  # bitwise reproducible
    pairs = [("means3D", "means3D"), ("shs", "shs"), ("opacities", "opacities"), ("scales", "scales"),
             ("rotations", "rotations"), ("means2D", "means2D"), ("means2D_densify", "means2D_densify")]
    _check(o, g, color, radii, depth, grads, pairs, nr=nr, tag=f"raster_deterministic[{N}x{H}x{W}]")
    for k in grads:
        ref = ra[3][k]
        np.testing.assert_allclose(grads[k], ref, rtol=1e-4, atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=k)


@pytest.mark.parametrize("case", [
    # N, H, W, cam, scale_boost: config 1; ragged tiles with big Gaussians; lists far beyond k_tile_sort's
    # 2048-entry LDS sort (sorted runs merged by rank: up to ~10 runs per tile); the bench workload
    (5000, 256, 256, 0, 0.0), (2000, 61, 83, 3, 1.0), (20000, 64, 80, 1, 3.0), (100_000, 800, 800, 0, 0.0)])
def test_tile_sort_matches_global_depth_sort(case):
    """Rect binning in index order + k_tile_sort (the default) vs the global stable depth sort
    (dgs_debug_set_tile_sort(0)): the tile lists are the same, so the image, depth and radii are bitwise
    equal and the gradients equal up to the float atomics' arrival order (1e-4 relative + 1e-6 of each
    tensor's max); the tile-sorted result also passes every oracle check."""
    from deformgs import _lib
    lib = _lib.load()
    N, H, W, ci, boost = case
    inputs, rs, _ = scene(N, H, W, cam_index=ci, scale_boost=boost, seed=21)
    rng = np.random.default_rng(11)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    res = {}
    before = lib.dgs_debug_get_tile_sort()
    try:
        for ts in (0, 1):
            lib.dgs_debug_set_tile_sort(ts)
            res[ts] = _run_gpu(inputs, rs, dcolor, None) + (_run_gpu.num_rendered,)
    finally:
        lib.dgs_debug_set_tile_sort(before)
    for a, b in zip(res[1][:3], res[0][:3]):
        np.testing.assert_array_equal(a, b)
    assert res[1][4] == res[0][4]
    for k in res[1][3]:
        ref = res[0][3][k]
        np.testing.assert_allclose(res[1][3][k], ref, rtol=1e-4, atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=k)
    if N <= 20000:
        o, g = oracle_run(inputs, rs, dcolor, None)
        color, radii, depth, grads, nr = res[1]
        _check(o, g, color, radii, depth, grads,
               [("means3D", "means3D"), ("opacities", "opacities"), ("means2D", "means2D")],
               nr=nr, tag=f"raster_tile_sort[{N}x{H}x{W}]")


@pytest.mark.parametrize("case", [
    (5000, 256, 256, 0, 0.0), (2000, 61, 83, 3, 1.0), (100_000, 800, 800, 0, 0.0)])
def test_two_pixel_forward_blend_is_bitwise_equal(case):
    """k_blend_fwd2 (two pixels per lane, dgs_debug_set_blend_fwd2(1)) vs k_blend_fwd: image, depth and
    radii bitwise equal, and — with the deterministic backward, so the gradients are fixed-order sums —
    every gradient bitwise equal (the backward replays from the forward's transmittance and contributor
    counts, so this pins those too)."""
    from deformgs import _lib
    from deformgs.renderer import set_deterministic
    lib = _lib.load()
    N, H, W, ci, boost = case
    inputs, rs, _ = scene(N, H, W, cam_index=ci, scale_boost=boost, seed=23)
    rng = np.random.default_rng(13)
    dcolor = rng.standard_normal((3, H, W)).astype(np.float32)
    res = {}
    before, det0 = lib.dgs_debug_get_blend_fwd2(), set_deterministic(True)
    try:
        for f2 in (0, 1):
            lib.dgs_debug_set_blend_fwd2(f2)
            res[f2] = _run_gpu(inputs, rs, dcolor, None)
    finally:
        lib.dgs_debug_set_blend_fwd2(before)
        set_deterministic(det0)
    for a, b in zip(res[1][:3], res[0][:3]):
        np.testing.assert_array_equal(a, b)
    for k in res[0][3]:
        np.testing.assert_array_equal(res[1][3][k], res[0][3][k], err_msg=k)


def test_deterministic_mode_under_overflow_and_both_binnings(binning):
    """The deterministic backward through the training step's deferred pair count: without overflow the
    deferred step's gradients equal the synchronous step's BITWISE (rect binning; the sort binning keeps
    the float atomics and is held to the atomics' tolerance); a forced overflow (speculative capacity
    777) runs its clipped backward in bounds and is detected; the synchronous redo equals the reference
    (bitwise with rect binning)."""
    from deformgs import _lib
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.renderer import set_deterministic
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import deferred_overflowed, drop_grads, forward_backward
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g = synth_gaussians(6000, seed=1, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    gs.training_setup(OptimizationParams())
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    deform.train_setting(OptimizationParams())
    cam = synth_camera(160, 128, index=3, fid=0.6, device=dev)
    gt = torch.rand((3, 128, 160), device=dev)
    params = [gs._xyz, gs._features_dc, gs._features_rest, gs._scaling, gs._rotation, gs._opacity] + \
        list(deform.deform.parameters())

    def run(deferred):
        drop_grads(gs, deform)
        loss, pkg = forward_backward(gs, deform, cam, gt, PipelineParams(), torch.zeros(3, device=dev),
                                     deferred_count=deferred)
        torch.cuda.synchronize()
        return loss.item(), pkg["render"].detach().clone(), [p.grad.clone() for p in params]

    def same(a, b):
        assert a[0] == b[0] and torch.equal(a[1], b[1])
        for x, y in zip(a[2], b[2]):
            if binning == "rect":
                assert torch.equal(x, y)
            else:
                torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-6 * max(1.0, y.abs().max().item()))

    before = set_deterministic(True)
    try:
        ref = run(False)
        same(run(True), ref)
        assert not deferred_overflowed()
        lib.dgs_debug_set_pair_cap(dev.index, 777)
        run(True)
        assert deferred_overflowed()
        same(run(False), ref)
    finally:
        set_deterministic(before)

"""The training loop (deformgs/train.py, train_baseline.py:56-182) on the HIP path vs the same loop
driven through the reference's torch glue (the network's torch forward, render()'s generic glue, torch
L1/SSIM, torch.optim.Adam, boolean-index densification) around the same HIP rasterizer.

25 iterations on a small synthetic scene, crossing the warm-up boundary (deformation on from
iteration 10), two densify_and_prune calls (iterations 10 and 20, the second with the size threshold
after the opacity reset at 15) and the viewpoint-stack refill. Tolerances: the Gaussian count must be
identical after the first densify; later counts within 0.1 % (the blend backward sums float atomics
in arrival order, so the accumulated densification statistic of a Gaussian sitting on the 0.0007
threshold can fall either side between ANY two runs, fused or not: 1 of ~20k flipped in the first GPU
run); per-iteration losses within 2e-4 relative while the counts agree, 2e-3 after (the primary
check). Parameters are compared as wholes, not element-wise: Adam from fresh moments moves an element
whose gradient is near zero by lr-sized steps of either sign, so fp32-level gradient differences show
up element-wise at full learning rate (seen on the GPU: 2 % of the opacity range after the reset, 1.5 %
of a weight tensor's largest entry). Final Gaussian tensors: ||a - b|| <= 1e-3 ||b|| when the counts
agree; deformation-network UPDATES over the run: ||dW_a - dW_b|| <= 10 % of ||dW_b|| per tensor.
"""
import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _opt(**kw):
    from deformgs.arguments import OptimizationParams
    base = dict(iterations=25, warm_up=10, densify_from_iter=5, densification_interval=10, opacity_reset_interval=15,
                sequence_length=8)
    base.update(kw)
    return OptimizationParams(**base)


def _run(scene, fused, is_blender=True, seed=0, opt=None):
    from deformgs.arguments import ModelParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.train import training
    dev = torch.device("cuda", 0)
    g = scene.init_gaussians(GaussianModel(3))
    torch.manual_seed(seed)
    deform = DeformModelBaseline(is_blender=is_blender, is_6dof=False, device=dev)
    with torch.no_grad():  # a trained network's small deltas
        for h in (deform.deform.gaussian_warp, deform.deform.gaussian_rotation, deform.deform.gaussian_scaling):
            h.weight.mul_(0.01)
            h.bias.mul_(0.01)
    init = {k: v.detach().clone() for k, v in deform.deform.state_dict().items()}
    opt = opt or _opt()
    hist = training(ModelParams(is_blender=is_blender), opt, PipelineParams(), [opt.iterations], [], scene, g, deform,
                    fused=fused, seed=seed)
    params = {k: getattr(g, k).detach().clone() for k in
              ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity")}
    params.update({k: v.detach().clone() - init[k] for k, v in deform.deform.state_dict().items()})  # updates
    return hist, params


@pytest.fixture(scope="module")
def scene():
    from deformgs.train import SyntheticScene
    return SyntheticScene(3000, 96, 80, n_train=10, n_test=2, seed=3, device="cuda")


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("is_blender", [True, False])
def test_loop_matches_torch_glue(scene, is_blender):
    from deformgs import _lib
    ha, pa = _run(scene, True, is_blender)
    hb, pb = _run(scene, False, is_blender)
    _same_run(ha, hb, pa, pb)
    assert ha["n"][9] != ha["n"][8], "the first densify_and_prune must change the count"
    # the test report ran and is finite
    assert np.isfinite(ha["report"][25]["test"][1]) and abs(ha["report"][25]["test"][1] - hb["report"][25]["test"][1]) < 1e-2
    assert _lib.load().dgs_debug_guard_expiries() == 0


def _same_run(ha, hb, pa=None, pb=None, first_densify=9, tight_until=None, sorted_rows=False, net_bar=0.1,
              loose=2e-3):
    """tight_until: the 2e-4 loss bar holds for the first tight_until iterations only (then 2e-3): the
    two paths' last-bit differences (glue exp / SSIM convolution vs the fused kernels) grow once the
    deformation network trains, as between two runs of the reference (float atomics)."""
    na, nb = np.array(ha["n"]), np.array(hb["n"])
    assert na[first_densify] == nb[first_densify], (na, nb)
    assert np.all(np.abs(na - nb) <= np.maximum(2, 1e-3 * nb)), (na, nb)
    agree = np.cumprod(na == nb).astype(bool)
    if tight_until is not None:
        agree[tight_until:] = False
    la, lb = np.array(ha["loss"]), np.array(hb["loss"])
    rel = np.abs(la - lb) / np.abs(lb)
    assert np.all(rel[agree] <= 2e-4) and np.all(rel <= loose), rel
    if pa is None:
        return
    for k in pa:
        if pa[k].shape != pb[k].shape:
            assert na[-1] != nb[-1], k
            continue
        x, y = pa[k], pb[k]
        if k.startswith("_") and sorted_rows:
            # one different densify decision near its threshold reorders every row after it (clone /
            # split append in index order, prune compacts): compare the per-column value distributions
            x, y = x.reshape(x.shape[0], -1).sort(0).values, y.reshape(y.shape[0], -1).sort(0).values
        err = float((x - y).norm()) / max(float(y.norm()), 1e-12)
        if not k.startswith("_") and net_bar is None:
            continue
        assert err < (1e-3 if k.startswith("_") else net_bar), (k, err)  # Gaussians / network updates


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_loop_converges_and_redoes_overflows(scene):
    """Loss falls over 120 iterations (warm-up 40, densification, an opacity reset); a forced
    overflow of the deferred pair count at iteration 50 is redone synchronously. Two runs of the same
    loop are not bitwise equal (float atomics in the blend backward; Adam and densification amplify
    the last-bit differences: ~1 % loss spread after 120 iterations on the first GPU run), so the runs
    with and without the redo are compared until the deformation network starts (iteration 40, losses
    2e-4) and by their final loss (5 %); the redone step itself is pinned bitwise by
    tests/test_gpu_raster.py::test_deferred_count_redo_matches_sync."""
    from deformgs import _lib
    lib = _lib.load()
    opt = _opt(iterations=120, warm_up=40, densify_from_iter=20, densification_interval=25,
               opacity_reset_interval=60)
    ha, _ = _run(scene, True, opt=opt)
    assert not any(ha["redone"][5:])
    first, last = np.mean(ha["loss"][:5]), np.mean(ha["loss"][-5:])
    assert last < 0.7 * first, (first, last)

    def force(it, g, d):
        if it == 49:
            lib.dgs_debug_set_pair_cap(0, 100)

    from deformgs.arguments import ModelParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.train import training
    g = scene.init_gaussians(GaussianModel(3))
    torch.manual_seed(0)
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device="cuda")
    with torch.no_grad():
        for h in (deform.deform.gaussian_warp, deform.deform.gaussian_rotation, deform.deform.gaussian_scaling):
            h.weight.mul_(0.01)
            h.bias.mul_(0.01)
    hb = training(ModelParams(is_blender=True), opt, PipelineParams(), [120], [], scene, g, deform, on_iteration=force)
    assert hb["redone"][49], "the forced overflow must be redone"
    assert sum(hb["redone"]) == 1
    la, lb = np.array(ha["loss"]), np.array(hb["loss"])
    assert np.all(np.abs(la[:39] - lb[:39]) <= 2e-4 * la[:39])
    assert ha["n"][24] == hb["n"][24]
    assert abs(np.mean(lb[-5:]) - np.mean(la[-5:])) <= 0.05 * np.mean(la[-5:])


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_deterministic_loop_is_bitwise_reproducible(scene):
    """With the deterministic blend backward (deformgs.renderer.set_deterministic) the fused loop has no
    order-dependent sum left (the MLP's split GEMMs, the loss reduction, Adam and densification are
    deterministic already): two 60-iteration runs (warm-up 20, densify at 20 and 40, an opacity reset at
    30) give bitwise-identical losses, Gaussian counts, Gaussian tensors and network updates. Without it
    two runs differ in the last bits from the first backward on (test_loop_converges_and_redoes_overflows)."""
    from deformgs.renderer import set_deterministic
    opt = _opt(iterations=60, warm_up=20, densify_from_iter=10, densification_interval=20, opacity_reset_interval=30)
    before = set_deterministic(True)
    try:
        ha, pa = _run(scene, True, opt=opt)
        hb, pb = _run(scene, True, opt=opt)
    finally:
        set_deterministic(before)
    assert ha["n"] == hb["n"] and ha["n"][19] != ha["n"][18]
    np.testing.assert_array_equal(np.array(ha["loss"]), np.array(hb["loss"]))
    for k in pa:
        assert torch.equal(pa[k], pb[k]), k


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_config3_loop_at_size_matches_torch_glue():
    """Config 3's loop at its size (55k Gaussians @ 800x800, bouncingballs-like; synthetic scene):
    200 iterations across the warm-up boundary (deformation on from iteration 100) and densify_and_prune
    at iterations 100 and 200, fused HIP path vs the reference's torch glue around the same rasterizer
    (the count after the first densify identical; losses within 2e-4 through the static warm-up, then
    4e-3: first measured run, 1.9-4e-5 in the warm-up and up to 1.6e-3 once the network trains;
    Gaussian parameters compared as sorted columns: row order after a densify differs as soon as one
    decision near its threshold does — 11 % row-wise norm difference on the first run. The network's
    updates are not compared at this size: over 100 trained iterations Adam's normalised steps follow
    the last-bit noise of near-cancelling gradient sums over 55k points, and the per-tensor update
    difference measured 12.8 % (timenet.0.weight) and 30.6 % (linear.4.weight) on two runs; the losses
    above are the check that the network learns the same)."""
    from deformgs.train import SyntheticScene
    scene = SyntheticScene(55_000, 800, 800, n_train=30, n_test=2, seed=7, device="cuda")
    opt = _opt(iterations=200, warm_up=100, densify_from_iter=50, densification_interval=100,
               opacity_reset_interval=3000, sequence_length=30)
    ha, pa = _run(scene, True, opt=opt)
    hb, pb = _run(scene, False, opt=opt)
    _same_run(ha, hb, pa, pb, first_densify=99, tight_until=100, sorted_rows=True, net_bar=None, loose=4e-3)
    assert ha["n"][99] != ha["n"][98], "the densify at iteration 100 must change the count"
    assert not any(ha["redone"][1:])


@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
@pytest.mark.parametrize("is_blender", [True, False], ids=["blender", "nonblender-ast-noise"])
def test_loop_generalises_to_held_out_views(is_blender):
    """Held-out signal for the loop (the stand-in for config 5's test PSNR, train_baseline.py:210-267):
    3000 iterations on a 20k-Gaussian scene at 400x400 whose ground truth deforms smoothly in position
    and time, with test cameras interleaved between the train views and frame times
    (deformgs/train.py SyntheticScene). Reference defaults otherwise (densify every 100 from 500, reset
    at 3000), warm-up 500. The test PSNR must rise: by 1 dB from the end of the static warm-up to the
    end of the run (the deformation network is what it learns after the warm-up) and above the first
    iteration's. Both networks: the blender one (timenet) and config 5's NeRF-DS one (is_blender=False:
    no timenet, 21-channel t PE, and the ast_noise of train_baseline.py:107-112 on the frame time after
    the warm-up), with densification on."""
    from deformgs.arguments import ModelParams, OptimizationParams, PipelineParams
    from deformgs.gaussian_model import GaussianModel
    from deformgs.train import SyntheticScene, training
    from helpers import write_stats
    scene = SyntheticScene(20_000, 400, 400, n_train=30, n_test=5, seed=5, device="cuda")
    g = scene.init_gaussians(GaussianModel(3))
    torch.manual_seed(0)
    opt = OptimizationParams(iterations=3000, warm_up=500)
    hist = training(ModelParams(is_blender=is_blender), opt, PipelineParams(), [1, 500, 3000], [], scene, g, seed=0)
    rep = hist["report"]
    p1, p500, p3000 = (rep[k]["test"][1] for k in (1, 500, 3000))
    train = [rep[k]["train"][1] for k in (1, 500, 3000)]
    print("test PSNR", p1, p500, p3000, "train", train)
    write_stats(f"heldout_loop[{'blender' if is_blender else 'nonblender'}]",
                dict(test_psnr=[p1, p500, p3000], train_psnr=train, n_final=hist["n"][-1],
                     n_after_first_densify=hist["n"][600], redone=int(sum(hist["redone"]))))
    assert hist["n"][600] != hist["n"][400], "densification must change the Gaussian count"
    assert p3000 > p500 + 1.0 and p3000 > p1, (p1, p500, p3000)

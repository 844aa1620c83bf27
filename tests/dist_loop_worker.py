"""One rank of the 2-rank training-LOOP test (tests/test_gpu_dist_step.py::test_two_rank_loop_*); not
collected by pytest.

Env: torchrun-style RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, DGS_DEVICE=0 (both ranks on the one
GPU) and DGS_DIST_BACKEND=gloo. argv: out_dir [nonblender]. Runs deformgs.train.training() — the
train_baseline.py:56-182 loop with frame parallelism — for 34 iterations across the
warm-up boundary (deformation on from iteration 10), three densify_and_prune calls (iterations 10, 20,
30; the last two with the size threshold after the opacity reset at 15) and the viewpoint-stack
refill; every iteration that densifies or resets opacity and the end are snapshotted (Gaussian count and
every Gaussian / network parameter) to out_dir/rank{r}.pt.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "deformable-3d-gaussians_amd"), HERE]

import torch  # noqa: E402

SNAP_AT = (10, 11, 15, 20, 30)


def main():
    out_dir = sys.argv[1]
    non_blender = len(sys.argv) > 2 and sys.argv[2] == "nonblender"
    import torch.distributed as dist
    from deformgs import _lib
    from deformgs.arguments import ModelParams, OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.dist import init_from_env
    from deformgs.gaussian_model import GaussianModel
    from deformgs.train import SyntheticScene, training
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    scene = SyntheticScene(3000, 96, 80, n_train=10, n_test=2, seed=3, device=dev)
    g = scene.init_gaussians(GaussianModel(3))
    torch.manual_seed(0)
    deform = DeformModelBaseline(is_blender=not non_blender, is_6dof=False, device=dev)
    with torch.no_grad():
        for h in (deform.deform.gaussian_warp, deform.deform.gaussian_rotation, deform.deform.gaussian_scaling):
            h.weight.mul_(0.01)
            h.bias.mul_(0.01)
    opt = OptimizationParams(iterations=34, warm_up=10, densify_from_iter=5, densification_interval=10,
                             opacity_reset_interval=15, sequence_length=8)
    snaps = {}

    def snap(it, gs, d):
        if it in SNAP_AT:
            ps = [gs._xyz, gs._features_dc, gs._features_rest, gs._scaling, gs._rotation, gs._opacity]
            snaps[it] = {"n": int(gs._xyz.shape[0]),
                         "params": [p.detach().clone().cpu() for p in ps + list(d.deform.parameters())],
                         "accum": gs.xyz_gradient_accum.detach().clone().cpu(),
                         "max_radii2D": gs.max_radii2D.detach().clone().cpu()}

    hist = training(ModelParams(is_blender=not non_blender), opt, PipelineParams(), [opt.iterations], [], scene, g,
                    deform, seed=0, on_iteration=snap)
    snap_end = {"n": int(g._xyz.shape[0]),
                "params": [p.detach().clone().cpu() for p in [g._xyz, g._features_dc, g._features_rest, g._scaling,
                                                                g._rotation, g._opacity]
                           + list(deform.deform.parameters())]}
    torch.save({"snaps": snaps, "end": snap_end, "n": hist["n"], "loss": hist["loss"], "redone": hist["redone"],
                "expiries": int(_lib.load().dgs_debug_guard_expiries())},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

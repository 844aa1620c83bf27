"""One rank of the 2-rank training-step test (tests/test_gpu_dist_step.py); not collected by pytest.

Env: torchrun-style RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, DGS_DEVICE=0 (both ranks on the
one GPU) and DGS_DIST_BACKEND=gloo (RCCL refuses two ranks on one device). argv: out_dir mode [6dof], mode
"plain" or "overflow" (rank 1 forces its deferred pair count to overflow: every rank must redo);
"6dof": the screw deformation head of config 4 (trex --is_6dof) instead of d_xyz.
Writes out_dir/rank{r}.pt = {"grads", "params", "redone"}.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "deformable-3d-gaussians_amd"), HERE]

import torch  # noqa: E402


def build(dev, n=4000, res=128, six=False):
    """The test's model / cameras / targets (identical on every rank and in the parent)."""
    from deformgs.arguments import OptimizationParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_camera, synth_gaussians
    torch.manual_seed(0)
    g = synth_gaussians(n, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    gs.training_setup(OptimizationParams())
    deform = DeformModelBaseline(is_blender=True, is_6dof=six, device=dev)
    net = deform.deform
    heads = (net.branch_w, net.branch_v) if six else (net.gaussian_warp,)
    with torch.no_grad():
        for h in heads + (net.gaussian_rotation, net.gaussian_scaling):
            h.weight.mul_(0.01)
            h.bias.mul_(0.01)
    deform.train_setting(OptimizationParams())
    cams = [synth_camera(res, res, index=3 + 5 * k, fid=0.1 + 0.3 * k, device=dev) for k in range(2)]
    gen = torch.Generator(device="cpu").manual_seed(7)
    gts = [torch.rand((3, res, res), generator=gen).to(dev) for _ in range(2)]
    return gs, deform, cams, gts


def params_of(gs, deform):
    ps = [gs._xyz, gs._features_dc, gs._features_rest, gs._scaling, gs._rotation, gs._opacity]
    return ps + list(deform.deform.parameters())


def main():
    out_dir, mode = sys.argv[1], sys.argv[2]
    six = len(sys.argv) > 3 and sys.argv[3] == "6dof"
    from deformgs import _lib
    from deformgs.arguments import PipelineParams
    from deformgs.dist import OverflowAgreement, OverlappedGradAllReduce, init_from_env
    from deformgs.train_step import optimizer_step, train_step
    import torch.distributed as dist
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    gs, deform, cams, gts = build(dev, six=six)
    bg = torch.zeros(3, device=dev)
    allreduce = OverlappedGradAllReduce(lambda: params_of(gs, deform)[:6], lambda: list(deform.deform.parameters()))
    agreement = OverflowAgreement()
    lib = _lib.load()
    # learn the pair capacity on a synchronous render of this rank's frame, then (overflow mode)
    # shrink rank 1's so its deferred count overflows
    train_step(gs, deform, cams[rank], gts[rank], PipelineParams(), bg, six, deferred_count=False, allreduce=allreduce,
               agreement=agreement)
    gs.optimizer.zero_grad(set_to_none=True)
    deform.optimizer.zero_grad(set_to_none=True)
    if mode == "overflow" and rank == 1:
        lib.dgs_debug_set_pair_cap(local, 100)
    loss, pkg, redone = train_step(gs, deform, cams[rank], gts[rank], PipelineParams(), bg, six, deferred_count=True,
                                   allreduce=allreduce, agreement=agreement)
    grads = [p.grad.detach().clone().cpu() for p in params_of(gs, deform)]
    optimizer_step(gs, deform, 3000)
    torch.cuda.synchronize()
    params = [p.detach().clone().cpu() for p in params_of(gs, deform)]
    torch.save({"grads": grads, "params": params, "redone": redone, "loss": float(loss),
                "native": getattr(gs, "_dgs_native", None) is not None},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

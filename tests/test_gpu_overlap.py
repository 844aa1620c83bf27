"""The overlapped gradient all-reduce (deformgs/dist.py OverlappedGradAllReduce) relies on the
autograd engine accumulating the Gaussian gradients (and running their post-accumulate hooks) before
it runs the deformation MLP's backward: then the early collective is issued ahead of ~1 ms of MLP
backward + dW kernels. Checked on the real training step (single process; the collective itself is
covered by tests/test_dist.py on gloo)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_gaussian_grads_complete_before_mlp_backward():
    from deformgs import deform_network
    from deformgs.arguments import OptimizationParams, PipelineParams
    from deformgs.deform_model import DeformModelBaseline
    from deformgs.gaussian_model import GaussianModel
    from deformgs.synthetic import synth_camera, synth_gaussians
    from deformgs.train_step import forward_backward

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g = synth_gaussians(4000, seed=0, device=dev)
    gs = GaussianModel(3)
    gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
    gs.training_setup(OptimizationParams())
    deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev)
    deform.train_setting(OptimizationParams())
    cam = synth_camera(128, 128, index=3, fid=0.4, device=dev)
    gt = torch.rand((3, 128, 128), device=dev)
    events = []
    early = [gs._xyz, gs._features_dc, gs._features_rest, gs._scaling, gs._rotation, gs._opacity]
    handles = [p.register_post_accumulate_grad_hook(lambda p, i=i: events.append(("gaussian", i)))
               for i, p in enumerate(early)]
    orig = deform_network._FusedDeformMLP.backward

    def wrapped(ctx, *grads):
        events.append(("mlp_backward", None))
        return orig(ctx, *grads)

    deform_network._FusedDeformMLP.backward = staticmethod(wrapped)
    try:
        forward_backward(gs, deform, cam, gt, PipelineParams(), torch.zeros(3, device=dev))
    finally:
        deform_network._FusedDeformMLP.backward = staticmethod(orig)
        for h in handles:
            h.remove()
    names = [e[0] for e in events]
    assert names.count("gaussian") == 6 and "mlp_backward" in names, events
    assert max(i for i, n in enumerate(names) if n == "gaussian") < names.index("mlp_backward"), events

import os, sys
ROOT='/root/repo'
sys.path.insert(0, os.path.join(ROOT, "deformable-3d-gaussians_amd")); sys.path.insert(0, ROOT)
import torch
from torch.utils._python_dispatch import TorchDispatchMode
from deformgs.arguments import OptimizationParams, PipelineParams
from deformgs.deform_model import DeformModelBaseline
from deformgs.gaussian_model import GaussianModel
from deformgs.synthetic import synth_camera, synth_gaussians
from deformgs.train_step import forward_backward, optimizer_step
dev = torch.device("cuda", 0)
N, R = 100_000, 800
g = synth_gaussians(N, seed=0, device=dev)
gs = GaussianModel(3)
gs.from_tensors(g["xyz"], g["features_dc"], g["features_rest"], g["scaling"], g["rotation"], g["opacity"])
opt = OptimizationParams(); gs.training_setup(opt)
deform = DeformModelBaseline(is_blender=True, is_6dof=False, device=dev); deform.train_setting(opt)
pipe = PipelineParams(); bg = torch.zeros(3, device=dev)
cam = synth_camera(R, R, index=0, fid=0.5, device=dev); gt = torch.rand((3, R, R), device=dev)
for it in range(3):
    forward_backward(gs, deform, cam, gt, pipe, bg, deferred_count=True); optimizer_step(gs, deform, 3000 + it)
class Log(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        import traceback
        if "clone" in str(func) or "fill" in str(func) or "zero" in str(func) or "copy" in str(func):
            shapes = [tuple(a.shape) if torch.is_tensor(a) else a for a in args]
            print("OP", func, shapes, "".join(traceback.format_stack(limit=8)[:-1]))
        else:
            print("OP", func)
        return func(*args, **(kwargs or {}))
with Log():
    forward_backward(gs, deform, cam, gt, pipe, bg, deferred_count=True)
    optimizer_step(gs, deform, 3010)
torch.cuda.synchronize()

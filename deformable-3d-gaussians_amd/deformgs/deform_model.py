"""DeformModel wrappers — mirror of scene/deform_model.py:253-357 on the fused HIP network.

step(xyz, t) -> (d_xyz, d_rotation, d_scaling); Adam(eps=1e-15) on all network parameters with the
exponential LR schedule; weights saved/loaded as deform/iteration_k/deform.pth (same state_dict keys
as the reference, loaded with weights_only=True).
"""
import os

import torch

from .deform_network import DeformNetwork, DeformNetworkBaseline
from .adam import Adam
from .general import get_expon_lr_func


def searchForMaxIteration(folder):
    saved = [int(f.split("_")[-1]) for f in os.listdir(folder)]
    return max(saved)


class DeformModelBaseline:
    """scene/deform_model.py:317-357."""
    net_cls = DeformNetworkBaseline

    def __init__(self, is_blender=False, is_6dof=False, D=8, W=256, input_ch=3, output_ch=59, multires=10,
                 device="cuda"):
        self.deform = self.net_cls(is_blender=is_blender, is_6dof=is_6dof, D=D, W=W, input_ch=input_ch,
                                   output_ch=output_ch, multires=multires).to(device)
        self.optimizer = None
        self.spatial_lr_scale = 5

    def step(self, xyz, time_emb):
        return self.deform(xyz, time_emb)

    def train_setting(self, training_args, optimizer_cls=None):
        l = [{'params': list(self.deform.parameters()),
              'lr': training_args.position_lr_init * self.spatial_lr_scale, "name": "deform"}]
        self.optimizer = (optimizer_cls or Adam)(l, lr=0.0, eps=1e-15)
        self.deform_scheduler_args = get_expon_lr_func(lr_init=training_args.position_lr_init * self.spatial_lr_scale,
                                                       lr_final=training_args.position_lr_final,
                                                       lr_delay_mult=training_args.position_lr_delay_mult,
                                                       max_steps=training_args.deform_lr_max_steps)

    def save_weights(self, model_path, iteration):
        out = os.path.join(model_path, "deform/iteration_{}".format(iteration))
        os.makedirs(out, exist_ok=True)
        torch.save(self.deform.state_dict(), os.path.join(out, 'deform.pth'))

    def load_weights(self, model_path, iteration=-1):
        it = searchForMaxIteration(os.path.join(model_path, "deform")) if iteration == -1 else iteration
        path = os.path.join(model_path, "deform/iteration_{}/deform.pth".format(it))
        self.deform.load_state_dict(torch.load(path, weights_only=True))

    def update_learning_rate(self, iteration):
        for group in self.optimizer.param_groups:
            if group["name"] == "deform":
                lr = self.deform_scheduler_args(iteration)
                group['lr'] = lr
                return lr


class DeformModel(DeformModelBaseline):
    """scene/deform_model.py:253-315 (fork variant): per time column, stacked d_xyz, rot/scale 0."""
    net_cls = DeformNetwork

    def step(self, xyz, time_emb):
        d_xyz_list, d_rot_list, d_scale_list = [], [], []
        for i in range(time_emb.shape[1]):
            d_xyz, d_rot, d_scale = self.deform(xyz, time_emb[:, i].unsqueeze(1))
            d_xyz_list.append(d_xyz)
            d_rot_list.append(d_rot)
            d_scale_list.append(d_scale)
        return torch.stack(d_xyz_list, dim=0), d_rot_list, d_scale_list

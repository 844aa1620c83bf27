"""GaussianModel — parameter store with the reference's tensor layout (scene/gaussian_model.py).

Same attribute names, shapes, activations and optimizer groups as scene/gaussian_model.py:25-401:
  _xyz (N,3) _features_dc (N,1,3) _features_rest (N,15,3) _scaling (N,3) _rotation (N,4) (w,x,y,z)
  _opacity (N,1); get_* apply exp / F.normalize / sigmoid / cat (:58-81).
create_from_pcd uses libdgs_hip's dgs_knn_dist2 in place of simple_knn.distCUDA2 (:105-106).
PLY I/O (:154-240) is implemented with numpy (plyfile is not a dependency here); attribute order
x y z nx ny nz f_dc_* f_rest_* opacity scale_* rot_* is kept so files interchange with the reference.
"""
import os

import numpy as np
import torch
from torch import nn

from .compact import select_rows
from . import _lib
from .general import build_rotation, get_expon_lr_func, inverse_sigmoid, strip_symmetric, build_scaling_rotation
from .adam import Adam
from .sh import RGB2SH


def distCUDA2(points):
    """simple_knn._C.distCUDA2 equivalent: mean squared distance to the 3 nearest neighbours."""
    pts = points.float().contiguous()
    _lib.require_cuda(pts)
    out = torch.empty((pts.shape[0],), dtype=torch.float32, device=pts.device)
    _lib.check(_lib.load().dgs_knn_dist2(pts.shape[0], _lib.ptr(pts), _lib.ptr(out), _lib.stream_ptr(pts.device)),
               "distCUDA2")
    return out


class GaussianModel:
    def __init__(self, sh_degree: int):
        def build_covariance_from_scaling_rotation(scaling, scaling_modifier, rotation):
            L = build_scaling_rotation(scaling_modifier * scaling, rotation)
            return strip_symmetric(L @ L.transpose(1, 2))

        self.active_sh_degree = 0
        self.max_sh_degree = sh_degree
        self._xyz = torch.empty(0)
        self._features_dc = torch.empty(0)
        self._features_rest = torch.empty(0)
        self._scaling = torch.empty(0)
        self._rotation = torch.empty(0)
        self._opacity = torch.empty(0)
        self.max_radii2D = torch.empty(0)
        self.xyz_gradient_accum = torch.empty(0)
        self.denom = torch.empty(0)
        self.optimizer = None
        self.percent_dense = 0.01
        self.spatial_lr_scale = 5
        self.scaling_activation = torch.exp
        self.scaling_inverse_activation = torch.log
        self.covariance_activation = build_covariance_from_scaling_rotation
        self.opacity_activation = torch.sigmoid
        self.inverse_opacity_activation = inverse_sigmoid
        self.rotation_activation = torch.nn.functional.normalize

    # ---- getters (gaussian_model.py:58-81) ----
    @property
    def get_scaling(self):
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation(self):
        return self.rotation_activation(self._rotation)

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_opacity(self):
        return self.opacity_activation(self._opacity)

    def get_covariance(self, scaling_modifier=1):
        return self.covariance_activation(self.get_scaling, scaling_modifier, self._rotation)

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # ---- construction ----
    def create_from_pcd(self, pcd, spatial_lr_scale=5, max_gaussians=None, device="cuda"):
        self.spatial_lr_scale = 5
        pts = torch.tensor(np.asarray(pcd.points)).float().to(device)
        col = RGB2SH(torch.tensor(np.asarray(pcd.colors)).float().to(device))
        if max_gaussians and pts.shape[0] > max_gaussians:
            idx = torch.randperm(pts.shape[0])[:max_gaussians]
            pts, col = pts[idx], col[idx]
        feats = torch.zeros((col.shape[0], 3, (self.max_sh_degree + 1) ** 2), device=device)
        feats[:, :3, 0] = col
        dist2 = torch.clamp_min(distCUDA2(pts), 0.0000001)
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        rots = torch.zeros((pts.shape[0], 4), device=device)
        rots[:, 0] = 1
        opac = inverse_sigmoid(0.1 * torch.ones((pts.shape[0], 1), dtype=torch.float, device=device))
        self._set(pts, feats[:, :, 0:1].transpose(1, 2).contiguous(), feats[:, :, 1:].transpose(1, 2).contiguous(),
                  scales, rots, opac)

    def from_tensors(self, xyz, features_dc, features_rest, scaling, rotation, opacity, active_sh_degree=None):
        self._set(xyz, features_dc, features_rest, scaling, rotation, opacity)
        self.active_sh_degree = self.max_sh_degree if active_sh_degree is None else active_sh_degree

    def _set(self, xyz, fdc, frest, scaling, rotation, opacity):
        self._xyz = nn.Parameter(xyz.detach().clone().requires_grad_(True))
        self._features_dc = nn.Parameter(fdc.detach().clone().requires_grad_(True))
        self._features_rest = nn.Parameter(frest.detach().clone().requires_grad_(True))
        self._scaling = nn.Parameter(scaling.detach().clone().requires_grad_(True))
        self._rotation = nn.Parameter(rotation.detach().clone().requires_grad_(True))
        self._opacity = nn.Parameter(opacity.detach().clone().requires_grad_(True))
        self.max_radii2D = torch.zeros((xyz.shape[0]), device=xyz.device)

    # ---- optimisation (gaussian_model.py:120-152) ----
    # row selection of densification: the one-launch HIP compaction; the torch-glue training loop
    # (deformgs/train.py, fused=False) sets torch indexing here, as the reference does it
    row_select = None

    def _select(self, mask, tensors):
        return (self.row_select or select_rows)(mask, tensors)

    def training_setup(self, training_args, optimizer_cls=None):
        self.percent_dense = training_args.percent_dense
        dev = self._xyz.device
        self.xyz_gradient_accum = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.denom = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.spatial_lr_scale = 5
        l = [
            {'params': [self._xyz], 'lr': training_args.position_lr_init * self.spatial_lr_scale, "name": "xyz"},
            {'params': [self._features_dc], 'lr': training_args.feature_lr, "name": "f_dc"},
            {'params': [self._features_rest], 'lr': training_args.feature_lr / 20.0, "name": "f_rest"},
            {'params': [self._opacity], 'lr': training_args.opacity_lr, "name": "opacity"},
            {'params': [self._scaling], 'lr': training_args.scaling_lr * self.spatial_lr_scale, "name": "scaling"},
            {'params': [self._rotation], 'lr': training_args.rotation_lr, "name": "rotation"},
        ]
        self.optimizer = (optimizer_cls or Adam)(l, lr=0.0, eps=1e-15)
        self.xyz_scheduler_args = get_expon_lr_func(lr_init=training_args.position_lr_init * self.spatial_lr_scale,
                                                    lr_final=training_args.position_lr_final * self.spatial_lr_scale,
                                                    lr_delay_mult=training_args.position_lr_delay_mult,
                                                    max_steps=training_args.position_lr_max_steps)

    def update_learning_rate(self, iteration):
        for group in self.optimizer.param_groups:
            if group["name"] == "xyz":
                lr = self.xyz_scheduler_args(iteration)
                group['lr'] = lr
                return lr

    # ---- PLY I/O (gaussian_model.py:154-240) ----
    def construct_list_of_attributes(self):
        l = ['x', 'y', 'z', 'nx', 'ny', 'nz']
        for i in range(self._features_dc.shape[1] * self._features_dc.shape[2]):
            l.append('f_dc_{}'.format(i))
        for i in range(self._features_rest.shape[1] * self._features_rest.shape[2]):
            l.append('f_rest_{}'.format(i))
        l.append('opacity')
        for i in range(self._scaling.shape[1]):
            l.append('scale_{}'.format(i))
        for i in range(self._rotation.shape[1]):
            l.append('rot_{}'.format(i))
        return l

    def save_ply(self, path):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        xyz = self._xyz.detach().cpu().numpy()
        normals = np.zeros_like(xyz)
        f_dc = self._features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
        f_rest = self._features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
        opac = self._opacity.detach().cpu().numpy()
        scale = self._scaling.detach().cpu().numpy()
        rot = self._rotation.detach().cpu().numpy()
        attrs = np.concatenate((xyz, normals, f_dc, f_rest, opac, scale, rot), axis=1).astype('<f4')
        names = self.construct_list_of_attributes()
        write_ply(path, names, attrs)

    def load_ply(self, path, device="cuda"):
        names, data = read_ply(path)
        col = {n: data[:, i] for i, n in enumerate(names)}
        xyz = np.stack([col['x'], col['y'], col['z']], 1)
        opac = col['opacity'][:, None]
        fdc = np.stack([col['f_dc_0'], col['f_dc_1'], col['f_dc_2']], 1)[:, :, None]
        extra = sorted([n for n in names if n.startswith('f_rest_')], key=lambda s: int(s.split('_')[-1]))
        assert len(extra) == 3 * (self.max_sh_degree + 1) ** 2 - 3
        fr = np.stack([col[n] for n in extra], 1).reshape(xyz.shape[0], 3, (self.max_sh_degree + 1) ** 2 - 1)
        sc = np.stack([col[n] for n in sorted([n for n in names if n.startswith('scale_')], key=lambda s: int(s.split('_')[-1]))], 1)
        ro = np.stack([col[n] for n in sorted([n for n in names if n.startswith('rot')], key=lambda s: int(s.split('_')[-1]))], 1)
        t = lambda a: torch.tensor(a, dtype=torch.float, device=device)  # noqa: E731
        self._set(t(xyz), t(fdc).transpose(1, 2).contiguous(), t(fr).transpose(1, 2).contiguous(), t(sc), t(ro), t(opac))
        self.active_sh_degree = self.max_sh_degree

    # ---- densification (gaussian_model.py:242-401) ----
    def replace_tensor_to_optimizer(self, tensor, name):
        out = {}
        for group in self.optimizer.param_groups:
            if group["name"] == name:
                st = self.optimizer.state.get(group['params'][0], None)
                st["exp_avg"] = torch.zeros_like(tensor)
                st["exp_avg_sq"] = torch.zeros_like(tensor)
                del self.optimizer.state[group['params'][0]]
                group["params"][0] = nn.Parameter(tensor.requires_grad_(True))
                self.optimizer.state[group['params'][0]] = st
                out[group["name"]] = group["params"][0]
        return out

    def reset_opacity(self):
        new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        self._opacity = self.replace_tensor_to_optimizer(new, "opacity")["opacity"]

    def _prune_optimizer(self, mask, extra=()):
        """Keeps the rows of `mask` in every parameter and its Adam moments (and in the tensors of
        `extra`, returned second) with ONE row-selection launch (deformgs/compact.py)."""
        groups, srcs = [], []
        for group in self.optimizer.param_groups:
            st = self.optimizer.state.get(group['params'][0], None)
            groups.append((group, st))
            srcs.append(group["params"][0].detach())
            if st is not None:
                srcs += [st["exp_avg"], st["exp_avg_sq"]]
        sel = self._select(mask, srcs + list(extra))
        out, k = {}, 0
        for group, st in groups:
            new_p = sel[k]
            k += 1
            if st is not None:
                st["exp_avg"], st["exp_avg_sq"] = sel[k], sel[k + 1]
                k += 2
                del self.optimizer.state[group['params'][0]]
            group["params"][0] = nn.Parameter(new_p.requires_grad_(True))
            if st is not None:
                self.optimizer.state[group['params'][0]] = st
            out[group["name"]] = group["params"][0]
        return out, sel[k:]

    def _assign(self, t):
        self._xyz, self._features_dc, self._features_rest = t["xyz"], t["f_dc"], t["f_rest"]
        self._opacity, self._scaling, self._rotation = t["opacity"], t["scaling"], t["rotation"]

    def prune_points(self, mask):
        valid = ~mask
        params, (self.xyz_gradient_accum, self.denom, self.max_radii2D) = self._prune_optimizer(
            valid, (self.xyz_gradient_accum, self.denom, self.max_radii2D))
        self._assign(params)

    def cat_tensors_to_optimizer(self, d):
        out = {}
        for group in self.optimizer.param_groups:
            ext = d[group["name"]]
            st = self.optimizer.state.get(group['params'][0], None)
            if st is not None:
                st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(ext)), dim=0)
                st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
                del self.optimizer.state[group['params'][0]]
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
                self.optimizer.state[group['params'][0]] = st
            else:
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def densification_postfix(self, new_xyz, new_fdc, new_frest, new_opac, new_scaling, new_rot):
        d = {"xyz": new_xyz, "f_dc": new_fdc, "f_rest": new_frest, "opacity": new_opac, "scaling": new_scaling,
             "rotation": new_rot}
        self._assign(self.cat_tensors_to_optimizer(d))
        dev = self._xyz.device
        self.xyz_gradient_accum = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.denom = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.max_radii2D = torch.zeros((self.get_xyz.shape[0]), device=dev)

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2, generator=None):
        n0 = self.get_xyz.shape[0]
        dev = self._xyz.device
        padded = torch.zeros((n0), device=dev)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values > self.percent_dense * scene_extent)
        xyz, fdc, frest, opac, scaling, rot = self._select(sel, [
            self._xyz.detach(), self._features_dc.detach(), self._features_rest.detach(), self._opacity.detach(),
            self._scaling.detach(), self._rotation.detach()])
        sel_scaling = self.scaling_activation(scaling)
        stds = sel_scaling.repeat(N, 1)
        means = torch.zeros((stds.size(0), 3), device=dev)
        samples = torch.normal(mean=means, std=stds, generator=generator)
        rots = build_rotation(rot).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + xyz.repeat(N, 1)
        new_scaling = self.scaling_inverse_activation(sel_scaling.repeat(N, 1) / (0.8 * N))
        self.densification_postfix(new_xyz, fdc.repeat(N, 1, 1), frest.repeat(N, 1, 1), opac.repeat(N, 1),
                                   new_scaling, rot.repeat(N, 1))
        prune = torch.cat((sel, torch.zeros(N * sel.sum(), device=dev, dtype=bool)))
        self.prune_points(prune)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        sel = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values <= self.percent_dense * scene_extent)
        self.densification_postfix(*self._select(sel, [
            self._xyz.detach(), self._features_dc.detach(), self._features_rest.detach(), self._opacity.detach(),
            self._scaling.detach(), self._rotation.detach()]))

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, generator=None):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent, generator=generator)
        prune = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_vs = self.max_radii2D > max_screen_size
            big_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune = torch.logical_or(torch.logical_or(prune, big_vs), big_ws)
        self.prune_points(prune)

    def add_densification_stats(self, viewspace_point_tensor, update_filter):
        self.xyz_gradient_accum[update_filter] += torch.norm(viewspace_point_tensor.grad[update_filter, :2], dim=-1,
                                                             keepdim=True)
        self.denom[update_filter] += 1


def write_ply(path, names, attrs):
    attrs = np.ascontiguousarray(attrs, dtype='<f4')
    header = "ply\nformat binary_little_endian 1.0\nelement vertex {}\n".format(attrs.shape[0])
    header += "".join("property float {}\n".format(n) for n in names) + "end_header\n"
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(attrs.tobytes())


def read_ply(path):
    """Binary little-endian PLY with one float vertex element (the layout save_ply writes)."""
    with open(path, "rb") as f:
        names, n = [], None
        line = f.readline().decode("ascii").strip()
        if line != "ply":
            raise ValueError("not a PLY file")
        while True:
            line = f.readline().decode("ascii").strip()
            if line.startswith("format") and "binary_little_endian" not in line:
                raise ValueError("only binary_little_endian PLY is supported")
            if line.startswith("element vertex"):
                n = int(line.split()[-1])
            elif line.startswith("property"):
                parts = line.split()
                if parts[1] not in ("float", "float32"):
                    raise ValueError("only float vertex properties are supported")
                names.append(parts[-1])
            elif line == "end_header":
                break
        data = np.frombuffer(f.read(4 * n * len(names)), dtype='<f4').reshape(n, len(names))
    return names, data.copy()

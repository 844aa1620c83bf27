"""Camera matrices — host-side mirror of the reference's camera conventions.

Mirrors (file:line in preacherwhite/Deformable-3D-Gaussians):
  utils/graphics_utils.py:42-53  getWorld2View2
  utils/graphics_utils.py:56-76  getProjectionMatrix (znear 0.01, zfar 100, z_sign 1)
  utils/graphics_utils.py:79-84  fov2focal / focal2fov
  scene/cameras.py:18-75         Camera: world_view_transform = W2C^T, projection_matrix = P^T,
                                 full_proj_transform = view @ proj, camera_center = inv(view)[3,:3]
  scene/cameras.py:78-89         MiniCam
  scene/dataset_readers.py:235-238  Blender transforms -> (R, T)
Pinned by tests/golden/camera.npz.
"""
import math

import numpy as np
import torch


def getWorld2View2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = (C2W[:3, 3] + translate) * scale
    C2W[:3, 3] = cam_center
    return np.float32(np.linalg.inv(C2W))


def getProjectionMatrix(znear, zfar, fovX, fovY):
    tanHalfFovY = math.tan(fovY / 2)
    tanHalfFovX = math.tan(fovX / 2)
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


def blender_c2w_to_RT(c2w):
    """scene/dataset_readers.py:235-238 (readCamerasFromTransforms)."""
    matrix = np.linalg.inv(np.asarray(c2w, np.float64))
    R = -np.transpose(matrix[:3, :3])
    R[:, 0] = -R[:, 0]
    T = -matrix[:3, 3]
    return R, T


class Camera:
    """Same fields and matrix conventions as scene/cameras.py:18-61 (no nn.Module / image I/O)."""

    def __init__(self, R, T, FoVx, FoVy, width, height, fid=0.0, image=None, uid=0,
                 trans=np.array([0.0, 0.0, 0.0]), scale=1.0, data_device="cuda"):
        self.uid = uid
        self.R, self.T = R, T
        self.FoVx, self.FoVy = FoVx, FoVy
        self.image_width, self.image_height = int(width), int(height)
        self.zfar, self.znear = 100.0, 0.01
        self.trans, self.scale = trans, scale
        dev = torch.device(data_device)
        self.data_device = dev
        self.fid = torch.tensor([fid], dtype=torch.float32, device=dev)
        self.original_image = None if image is None else image.clamp(0.0, 1.0).to(dev)
        # stored contiguous (same values as the reference's transposed view): the rasterizer takes it as
        # a raw 4x4 row-major pointer, so a strided view would cost a copy kernel per render
        self.world_view_transform = torch.tensor(getWorld2View2(R, T, trans, scale)).transpose(0, 1).contiguous().to(dev)
        self.projection_matrix = getProjectionMatrix(self.znear, self.zfar, FoVx, FoVy).transpose(0, 1).to(dev)
        self.full_proj_transform = self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0)).squeeze(0)
        # (the inverse comes back column-major: its row is a strided view; stored contiguous for the
        # same reason as above)
        self.camera_center = self.world_view_transform.inverse()[3, :3].contiguous()


class MiniCam:
    def __init__(self, width, height, fovy, fovx, znear, zfar, world_view_transform, full_proj_transform):
        self.image_width, self.image_height = width, height
        self.FoVy, self.FoVx = fovy, fovx
        self.znear, self.zfar = znear, zfar
        self.world_view_transform = world_view_transform
        self.full_proj_transform = full_proj_transform
        self.camera_center = torch.inverse(world_view_transform)[3][:3].contiguous()


def orbit_camera(azimuth, elevation, radius, fov, width, height, fid=0.0, data_device="cuda"):
    """A D-NeRF-style camera looking at the origin (Blender c2w, then the reader's conversion)."""
    cpos = np.array([radius * np.cos(elevation) * np.sin(azimuth),
                     -radius * np.cos(elevation) * np.cos(azimuth),
                     radius * np.sin(elevation)])
    fwd = -cpos / np.linalg.norm(cpos)
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    upv = np.cross(right, fwd)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, upv, -fwd, cpos
    R, T = blender_c2w_to_RT(c2w)
    fovy = focal2fov(fov2focal(fov, width), height)
    # dataset_readers.py:260-262 swaps the names: FovY = fovx, FovX = fovy
    return Camera(R, T, FoVx=fovy, FoVy=fov, width=width, height=height, fid=fid, data_device=data_device)

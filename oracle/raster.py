"""ORACLE (test infrastructure only) — ctypes front-end for oracle/liboracle_raster.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
PARITY UNPINNED: see the header of oracle/raster_ref.c (the CUDA rasterizer is an un-vendored
submodule, .gitmodules:4-7). Argument meaning follows gaussian_renderer/__init__.py:53-124.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_raster.so")


class ORSettings(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int), ("image_width", ctypes.c_int),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
        ("bg", ctypes.c_float * 3), ("scale_modifier", ctypes.c_float),
        ("viewmatrix", ctypes.c_float * 16), ("projmatrix", ctypes.c_float * 16),
        ("sh_degree", ctypes.c_int), ("campos", ctypes.c_float * 3), ("prefiltered", ctypes.c_int),
    ]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        _lib.or_forward.argtypes = [ctypes.POINTER(ORSettings), ctypes.c_int, ctypes.c_int] + [P] * 10 + [ctypes.POINTER(P)]
        _lib.or_forward.restype = ctypes.c_int
        _lib.or_backward.argtypes = [P] * 12
        _lib.or_backward.restype = ctypes.c_int
        _lib.or_free.argtypes = [P]
        _lib.or_num_rendered.argtypes = [P]
        _lib.or_num_rendered.restype = ctypes.c_int
        _lib.or_geometry.argtypes = [P] * 6
        _lib.or_pixel_state.argtypes = [P] * 3
        _lib.or_preprocess_raw.argtypes = [P] * 4
        _lib.or_flip_flags.argtypes = [P, ctypes.c_float, P, P]
        _lib.or_flip_flags.restype = ctypes.c_int
        _lib.or_preprocess_flags.argtypes = [P, ctypes.c_float, P]
        _lib.or_preprocess_flags.restype = ctypes.c_int
        _lib.or_pixel_gaussians.argtypes = [P, P, P]
        _lib.or_pixel_gaussians.restype = ctypes.c_int
    return _lib


def make_settings(H, W, tanfovx, tanfovy, bg, scale_modifier, viewmatrix, projmatrix, sh_degree,
                  campos, prefiltered=False):
    s = ORSettings()
    s.image_height, s.image_width = int(H), int(W)
    s.tanfovx, s.tanfovy = float(tanfovx), float(tanfovy)
    s.bg[:] = [float(v) for v in np.asarray(bg, np.float32).reshape(3)]
    s.scale_modifier = float(scale_modifier)
    s.viewmatrix[:] = [float(v) for v in np.asarray(viewmatrix, np.float32).reshape(16)]
    s.projmatrix[:] = [float(v) for v in np.asarray(projmatrix, np.float32).reshape(16)]
    s.sh_degree = int(sh_degree)
    s.campos[:] = [float(v) for v in np.asarray(campos, np.float32).reshape(3)]
    s.prefiltered = int(bool(prefiltered))
    return s


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a, shape=None):
    if a is None:
        return None
    a = np.ascontiguousarray(np.asarray(a, np.float32))
    return a if shape is None else a.reshape(shape)


class OracleRaster:
    """One forward (and optionally backward) of the CPU restatement."""

    def __init__(self, settings, means3D, shs=None, colors_precomp=None, opacities=None, scales=None,
                 rotations=None, cov3D_precomp=None):
        L = lib()
        self.s = settings
        self.N = int(np.asarray(means3D).shape[0])
        self.means3D = _f32(means3D, (self.N, 3))
        self.shs = _f32(shs)
        self.M = 0 if shs is None else int(np.asarray(shs).size // (self.N * 3))
        if self.shs is not None:
            self.shs = self.shs.reshape(self.N, self.M, 3)
        self.colors = _f32(colors_precomp)
        self.opac = _f32(opacities, (self.N,))
        self.scales = _f32(scales)
        self.rots = _f32(rotations)
        self.cov = _f32(cov3D_precomp)
        H, W = settings.image_height, settings.image_width
        self.color = np.zeros((3, H, W), np.float32)
        self.depth = np.zeros((1, H, W), np.float32)
        self.radii = np.zeros((self.N,), np.int32)
        self._st = ctypes.c_void_p()
        rc = L.or_forward(ctypes.byref(settings), self.N, self.M, _ptr(self.means3D), _ptr(self.shs),
                          _ptr(self.colors), _ptr(self.opac), _ptr(self.scales), _ptr(self.rots),
                          _ptr(self.cov), _ptr(self.color), _ptr(self.depth), _ptr(self.radii),
                          ctypes.byref(self._st))
        if rc != 0:
            raise ValueError(f"oracle forward rejected the argument combination (code {rc})")
        self.num_rendered = L.or_num_rendered(self._st)

    def geometry(self):
        N = self.N
        xy = np.zeros((N, 2), np.float32)
        co = np.zeros((N, 4), np.float32)
        rgb = np.zeros((N, 3), np.float32)
        dep = np.zeros((N,), np.float32)
        cov = np.zeros((N, 6), np.float32)
        lib().or_geometry(self._st, _ptr(xy), _ptr(co), _ptr(rgb), _ptr(dep), _ptr(cov))
        return dict(xy=xy, conic_opacity=co, rgb=rgb, depth=dep, cov3D=cov)

    def pixel_state(self):
        H, W = self.s.image_height, self.s.image_width
        T = np.zeros((H, W), np.float32)
        n = np.zeros((H, W), np.int32)
        lib().or_pixel_state(self._st, _ptr(T), _ptr(n))
        return T, n

    def preprocess_raw(self):
        """radf = 3 sqrt(lambda_max) (radius = ceil(radf)), vz = view-space z, pxy = pixel centre."""
        N = self.N
        radf = np.zeros((N,), np.float32)
        vz = np.zeros((N,), np.float32)
        pxy = np.zeros((N, 2), np.float32)
        lib().or_preprocess_raw(self._st, _ptr(radf), _ptr(vz), _ptr(pxy))
        return dict(radf=radf, vz=vz, pxy=pxy)

    def flip_flags(self, eps):
        """(per-Gaussian flags, per-pixel flags) of blend decisions within relative eps of their
        threshold (raster_ref.c or_flip_flags)."""
        H, W = self.s.image_height, self.s.image_width
        g = np.zeros((self.N,), np.uint8)
        px = np.zeros((H, W), np.uint8)
        lib().or_flip_flags(self._st, float(eps), _ptr(g), _ptr(px))
        return g.astype(bool), px.astype(bool)

    def preprocess_flags(self, eps):
        """Per-Gaussian flags of gradient-only preprocess decisions within eps of their threshold: the
        EWA Jacobian's frustum clamp and the SH colour clamp (raster_ref.c or_preprocess_flags)."""
        g = np.zeros((self.N,), np.uint8)
        lib().or_preprocess_flags(self._st, float(eps), _ptr(g))
        return g.astype(bool)

    def pixel_gaussians(self, pmask):
        """Per-Gaussian flags of the Gaussians blended in the pixels of pmask (H, W) (raster_ref.c
        or_pixel_gaussians)."""
        m = np.ascontiguousarray(pmask, np.uint8)
        g = np.zeros((self.N,), np.uint8)
        lib().or_pixel_gaussians(self._st, _ptr(m), _ptr(g))
        return g.astype(bool)

    def backward(self, dL_dcolor, dL_ddepth=None):
        N, M = self.N, self.M
        g = dict(
            means3D=np.zeros((N, 3), np.float32), means2D=np.zeros((N, 3), np.float32),
            means2D_densify=np.zeros((N, 3), np.float32), colors=np.zeros((N, 3), np.float32),
            opacities=np.zeros((N, 1), np.float32), cov3D=np.zeros((N, 6), np.float32),
            shs=np.zeros((N, max(M, 1), 3), np.float32), scales=np.zeros((N, 3), np.float32),
            rotations=np.zeros((N, 4), np.float32))
        dc = _f32(dL_dcolor)
        dd = _f32(dL_ddepth)
        rc = lib().or_backward(self._st, _ptr(dc), _ptr(dd), _ptr(g["means3D"]), _ptr(g["means2D"]),
                               _ptr(g["means2D_densify"]), _ptr(g["colors"]), _ptr(g["opacities"]),
                               _ptr(g["cov3D"]), _ptr(g["shs"]), _ptr(g["scales"]), _ptr(g["rotations"]))
        if rc != 0:
            raise MemoryError("oracle raster backward: host allocation failed")
        return g

    def __del__(self):
        try:
            if self._st:
                lib().or_free(self._st)
        except Exception:
            pass

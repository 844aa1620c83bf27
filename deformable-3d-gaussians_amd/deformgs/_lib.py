"""ctypes binding of libdgs_hip.so (C ABI: include/dgs.h).

The library is the product path: if it is missing or fails to load, every op raises — there is no
CPU or PyTorch fallback. torch is imported first so libdgs_hip.so binds to the HIP runtime torch
already loaded (one runtime per process; both have SONAME libamdhip64.so.7).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load)

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DGS_LIB: diagnostic builds only (tools/build_diag.sh); the product path is lib/libdgs_hip.so
LIB_PATH = os.environ.get("DGS_LIB") or os.path.join(_PKG, "lib", "libdgs_hip.so")

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
SZ = ctypes.c_size_t


class RasterSettings(ctypes.Structure):
    """dgs_raster_settings (include/dgs.h)."""
    _fields_ = [
        ("image_height", I), ("image_width", I), ("tanfovx", F), ("tanfovy", F),
        ("bg", P), ("scale_modifier", F), ("viewmatrix", P), ("projmatrix", P),
        ("sh_degree", I), ("campos", P), ("prefiltered", I), ("debug", I),
    ]


class AdamTensor(ctypes.Structure):
    """dgs_adam_tensor (include/dgs.h)."""
    _fields_ = [
        ("param", P), ("grad", P), ("exp_avg", P), ("exp_avg_sq", P), ("numel", ctypes.c_int64),
        ("step_size", F), ("bc2_sqrt", F),
    ]


class RowJob(ctypes.Structure):
    """dgs_row_job (include/dgs.h)."""
    _fields_ = [("src", P), ("dst", P), ("width", I)]


_SIGS = {
    "dgs_last_error": ([], ctypes.c_char_p),
    "dgs_version": ([], ctypes.c_char_p),
    "dgs_raster_forward": ([ctypes.POINTER(RasterSettings), I, I] + [P] * 10 + [ctypes.POINTER(P), ctypes.POINTER(I), P], I),
    "dgs_raster_backward": ([P] * 12 + [P], I),
    "dgs_raster_forward_split_sh": ([ctypes.POINTER(RasterSettings), I] + [P] * 10 + [ctypes.POINTER(P), ctypes.POINTER(I), P], I),
    "dgs_raster_backward_split_sh": ([P] * 11 + [P], I),
    "dgs_raster_ctx_free": ([P], None),
    "dgs_raster_ctx_num_rendered": ([P], I),
    "dgs_mark_visible": ([I, P, P, P, P, P], I),
    "dgs_debug_set_pair_cap": ([I, I], None),
    "dgs_debug_binning_redos": ([], ctypes.c_longlong),
    "dgs_debug_count_wait_ns": ([ctypes.POINTER(ctypes.c_longlong)], ctypes.c_longlong),
    "dgs_debug_pair_cap": ([I], I),
    "dgs_raster_set_deferred_count": ([I], None),
    "dgs_raster_set_exact_scale_grad": ([I], None),
    "dgs_debug_guard_expiries": ([], ctypes.c_longlong),
    "dgs_debug_dw_fallbacks": ([], ctypes.c_longlong),
    "dgs_debug_sort_pairs": ([P, P, P, P, I, I, I, P], I),
    "dgs_raster_deferred_overflows": ([], ctypes.c_longlong),
    "dgs_debug_set_binning": ([I], None),
    "dgs_debug_set_blend_seg": ([I], None),
    "dgs_raster_set_deterministic": ([I], None),
    "dgs_raster_get_deterministic": ([], I),
    "dgs_debug_set_tile_sort": ([I], None),
    "dgs_debug_get_tile_sort": ([], I),
    "dgs_debug_set_blend_fwd2": ([I], None),
    "dgs_debug_get_blend_fwd2": ([], I),
    "dgs_debug_get_blend_seg": ([], I),
    "dgs_mlp_set_reserved_cus": ([I], None),
    "dgs_mlp_reserved_cus": ([], I),
    "dgs_debug_collective_standin": ([P, ctypes.c_longlong, I, I, P], I),
    "dgs_timing_enable": ([I], None),
    "dgs_timing_query": ([ctypes.c_char_p, ctypes.POINTER(I)], ctypes.c_double),
    "dgs_timing_reset": ([], None),
    "dgs_timing_select": ([ctypes.c_char_p], None),
    "dgs_timing_sample": ([I], None),
    "dgs_timing_launches": ([ctypes.c_char_p], ctypes.c_longlong),
    "dgs_deform_num_params": ([I], I),
    "dgs_deform_packed_floats": ([I], SZ),
    "dgs_deform_saved_floats": ([I, I], SZ),
    "dgs_deform_scratch_floats": ([I, I], SZ),
    "dgs_deform_pack": ([I, P, P, P], I),
    "dgs_deform_forward": ([I, I, P, P, P, P, P, P], I),
    "dgs_deform_pack_forward": ([I, P, I, P, P, P, P, P, P], I),
    "dgs_deform_backward": ([I, I, P, P, P, P, P, P], I),
    "dgs_deform_outputs": ([I], I),
    "dgs_knn_dist2": ([I, P, P, P], I),
    "dgs_l1_ssim_scratch_floats": ([I, I, I], SZ),
    "dgs_l1_ssim_window": ([P], None),
    "dgs_l1_ssim_forward": ([I, I, I, P, P, F, P, P, P], I),
    "dgs_l1_ssim_backward": ([I, I, I, P, P, F, P, P, P, P], I),
    "dgs_adam_step": ([I, ctypes.POINTER(AdamTensor), ctypes.c_double, ctypes.c_double, ctypes.c_double, P], I),
    "dgs_select_rows": ([I, P, I, ctypes.POINTER(RowJob), P], I),
    "dgs_gaussian_inputs_forward": ([I, I] + [P] * 7 + [I] + [P] * 5 + [P], I),
    "dgs_gaussian_inputs_backward": ([I, I] + [P] * 15 + [I, P], I),
    "dgs_gaussian_inputs_se3_forward": ([I, I] + [P] * 7 + [I] + [P] * 5 + [P], I),
    "dgs_gaussian_inputs_se3_backward": ([I, I, P, P, I] + [P] * 15 + [P], I),
    "dgs_se3_forward": ([I, P, I, P, P], I),
    "dgs_se3_backward": ([I, P, I, P, P, I, P], I),
    # (dgs_train_step_args*, int* overflowed, int* num_rendered, stream): deformgs/native_step.py
    "dgs_train_step": ([P, ctypes.POINTER(I), ctypes.POINTER(I), P], I),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load():
    """Load libdgs_hip.so (raises if absent: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libdgs_hip.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or make -C deformable-3d-gaussians_amd/csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib


def check(rc, what):
    if rc != 0:
        msg = load().dgs_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr_array(tensors):
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ValueError("libdgs_hip ops take device (HIP) tensors; got a CPU tensor")

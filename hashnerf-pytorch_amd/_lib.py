"""ctypes binding of the C ABI in ``include/hashnerf_amd.h``.

This is the drop-in boundary the reference's Python would bind: plain
``extern "C"`` entry points taking device pointers, sizes and a hipStream_t.
There is deliberately NO CPU fallback: if the HIP library is missing or the
tensors are not on a ROCm device, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HN_LIB_PATH") or os.path.join(HERE, "lib", "libhashnerf_amd.so")
MAX_LEVELS = 32
ABI_VERSION = 14                # HN_ABI_VERSION
RENDER_FEAT_PER_RAY = 9728      # HN_RENDER_FEAT_PER_RAY
MLP_PARAMS = 9344
MLP_PACKED_FLOATS = 30208

_lib = None


class HnGrid(C.Structure):
    _fields_ = [("n_levels", C.c_int32), ("n_features", C.c_int32),
                ("log2_hashmap_size", C.c_int32), ("reserved", C.c_int32),
                ("box_min", C.c_float * 3), ("box_max", C.c_float * 3),
                ("grid_size", (C.c_float * 3) * MAX_LEVELS)]


class HnMlp(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("sigma0", "sigma1", "color0", "color1", "color2")]


class HnMlpGrad(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("sigma0", "sigma1", "color0", "color1", "color2")]


class HnRenderCfg(C.Structure):
    _fields_ = [("grid", HnGrid), ("n_samples", C.c_int32), ("n_importance", C.c_int32),
                ("white_bkgd", C.c_int32), ("lindisp", C.c_int32), ("perturb", C.c_int32),
                ("scatter", C.c_int32), ("bin_cap", C.c_int32), ("dense_bwd", C.c_int32)]


_P = C.c_void_p


class HnRenderLoss(C.Structure):
    _fields_ = [("target", _P), ("rgb", _P), ("rgb0", _P), ("sparsity", _P), ("sparsity0", _P), ("tv", _P),
                ("n_tv", C.c_int32), ("world", C.c_float), ("sparse_w", C.c_float), ("tv_w", C.c_float),
                ("out", _P)]


class HnRenderFwdArgs(C.Structure):
    _fields_ = [("n_rays", C.c_int64), ("rays", _P), ("t_vals", _P), ("t_rand", _P), ("u", _P),
                ("noise_c", _P), ("noise_f", _P), ("table", _P), ("coarse", HnMlp), ("fine", HnMlp),
                ("rgb", _P), ("depth", _P), ("acc", _P), ("sparsity", _P),
                ("rgb0", _P), ("depth0", _P), ("acc0", _P), ("sparsity0", _P),
                ("z_std", _P), ("z_coarse", _P), ("z_fine", _P), ("raw_c", _P), ("raw_f", _P),
                ("fine_src", _P), ("feat", _P), ("weights_packed", C.c_int32), ("skip_dead_color", C.c_int32)]


class HnRadamTensor(C.Structure):
    _fields_ = [("p", _P), ("g", _P), ("m", _P), ("v", _P), ("n", C.c_int64),
                ("beta1", C.c_float), ("beta2", C.c_float), ("one_minus_beta1", C.c_float),
                ("one_minus_beta2", C.c_float), ("eps", C.c_float), ("neg_wd_lr", C.c_float),
                ("neg_step_lr", C.c_float), ("mode", C.c_int32), ("has_wd", C.c_int32),
                ("reserved", C.c_int32)]


class HnRenderBwdArgs(C.Structure):
    _fields_ = [("n_rays", C.c_int64), ("rays", _P), ("noise_c", _P), ("noise_f", _P), ("table", _P),
                ("coarse", HnMlp), ("fine", HnMlp), ("z_coarse", _P), ("z_fine", _P), ("raw_c", _P),
                ("raw_f", _P), ("fine_src", _P), ("feat", _P), ("weights_packed", C.c_int32),
                ("d_table_mode", C.c_int32), ("g_rgb", _P), ("g_depth", _P), ("g_acc", _P), ("g_sparsity", _P),
                ("g_rgb0", _P), ("g_depth0", _P), ("g_acc0", _P), ("g_sparsity0", _P),
                ("g_raw_f", _P), ("d_table", _P), ("d_coarse", HnMlpGrad), ("d_fine", HnMlpGrad),
                ("table_step", C.POINTER(HnRadamTensor)), ("tv", C.c_void_p), ("g_tv", _P),
                ("table_live", _P), ("table_live_levels", C.c_int32), ("owner_defer", C.c_int32),
                ("loss", C.POINTER(HnRenderLoss)), ("mlp_step", C.POINTER(HnRadamTensor)),
                ("repack", C.c_int32)]


class HnTvArgs(C.Structure):
    _fields_ = [("n_levels", C.c_int32), ("log2_hashmap_size", C.c_int32),
                ("cube", C.c_int32 * MAX_LEVELS), ("min_vertex", _P), ("table", _P)]


RADAM_MAX_TENSORS = 16


class HnRaySampler(C.Structure):
    _fields_ = [("H", C.c_int32), ("W", C.c_int32), ("crop_y0", C.c_int32), ("crop_x0", C.c_int32),
                ("crop_h", C.c_int32), ("crop_w", C.c_int32), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("near", C.c_float), ("far", C.c_float),
                ("seed", C.c_uint64)]


class HnUniformDraw(C.Structure):
    _fields_ = [("out", _P), ("numel", C.c_int64), ("threads", C.c_int64), ("offset", C.c_uint64)]


UNIFORM_MAX_DRAWS = 4


class HnRayPool(C.Structure):
    _fields_ = [("n_images", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("pose_stride", C.c_int32),
                ("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("near", C.c_float), ("far", C.c_float), ("seed", C.c_uint64)]


# name -> (restype, argtypes); must match include/hashnerf_amd.h exactly.
SIGNATURES = {
    "hn_abi_version": (C.c_int32, []),
    "hn_status_string": (C.c_char_p, [C.c_int32]),
    "hn_device_faults": (C.c_int32, [C.POINTER(C.c_int32), C.c_int32]),
    "hn_encode_fwd": (C.c_int32, [C.POINTER(HnGrid), _P, C.c_int64, _P, _P, _P, _P]),
    "hn_encode_bwd": (C.c_int32, [C.POINTER(HnGrid), _P, C.c_int64, _P, _P, _P]),
    "hn_sh_fwd": (C.c_int32, [_P, C.c_int64, _P, _P]),
    "hn_mlp_workspace_bytes": (C.c_size_t, []),
    "hn_mlp_fwd": (C.c_int32, [C.POINTER(HnMlp), _P, C.c_int64, _P, _P, C.c_size_t, _P]),
    "hn_mlp_bwd": (C.c_int32, [C.POINTER(HnMlp), _P, _P, C.c_int64, _P, C.POINTER(HnMlpGrad), _P,
                               C.c_size_t, _P]),
    "hn_composite_fwd": (C.c_int32, [_P, _P, _P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P,
                                     _P, _P, _P, _P]),
    "hn_composite_bwd": (C.c_int32, [_P, _P, _P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P,
                                     _P, _P, _P, _P]),
    "hn_sample_pdf": (C.c_int32, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P]),
    "hn_tv_fwd": (C.c_int32, [C.POINTER(HnTvArgs), _P, _P]),
    "hn_tv_bwd": (C.c_int32, [C.POINTER(HnTvArgs), _P, _P, _P]),
    "hn_radam_step": (C.c_int32, [C.POINTER(HnRadamTensor), C.c_int32, _P]),
    "hn_sample_rays": (C.c_int32, [C.POINTER(HnRaySampler), _P, _P, C.c_int64, _P, _P, _P]),
    "hn_sample_rays_morton_workspace_bytes": (C.c_size_t, [C.POINTER(HnRaySampler)]),
    "hn_uniform_philox": (C.c_int32, [C.c_uint64, C.POINTER(HnUniformDraw), C.c_int32, _P]),
    "hn_sample_batch_morton": (C.c_int32, [C.POINTER(HnRaySampler), _P, _P, C.c_int64, _P, _P, _P, C.c_size_t,
                                           C.c_uint64, C.POINTER(HnUniformDraw), C.c_int32, _P]),
    "hn_sample_rays_morton": (C.c_int32, [C.POINTER(HnRaySampler), _P, _P, C.c_int64, _P, _P, _P, C.c_size_t,
                                          _P]),
    "hn_sample_pool": (C.c_int32, [C.POINTER(HnRayPool), _P, _P, _P, C.c_int64, C.c_int64, _P, _P, _P]),
    "hn_blender_images": (C.c_int32, [_P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P]),
    "hn_loss_fwd": (C.c_int32, [_P, _P, _P, _P, _P, C.c_int64, _P, C.c_int32, C.c_float, C.c_float,
                                C.c_float, _P, _P]),
    "hn_loss_bwd": (C.c_int32, [_P, _P, _P, C.c_int64, C.c_int32, C.c_float, C.c_float, C.c_float, _P,
                                _P, _P, _P, _P, _P, _P]),
    "hn_loss_fwd_bwd": (C.c_int32, [_P, _P, _P, _P, _P, C.c_int64, _P, C.c_int32, C.c_float, C.c_float,
                                    C.c_float, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hn_render_workspace_bytes": (C.c_size_t, [C.POINTER(HnRenderCfg), C.c_int64]),
    "hn_render_scatter_mode": (C.c_int32, [C.POINTER(HnRenderCfg), C.c_int64]),
    "hn_render_fwd": (C.c_int32, [C.POINTER(HnRenderCfg), C.POINTER(HnRenderFwdArgs), _P,
                                  C.c_size_t, _P]),
    "hn_render_bwd": (C.c_int32, [C.POINTER(HnRenderCfg), C.POINTER(HnRenderBwdArgs), _P,
                                  C.c_size_t, _P]),
    "hn_render_bins": (C.c_int32, [C.POINTER(HnRenderCfg), C.c_int64, C.POINTER(C.c_int32)]),
    "hn_render_bwd_owner": (C.c_int32, [C.POINTER(HnRenderCfg), C.POINTER(HnRenderBwdArgs), _P,
                                        C.c_size_t, C.c_int32, C.c_int32, _P]),
}


def lib():
    """Load (once) the HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"hashnerf_amd: HIP library not built ({LIB_PATH}); run "
                "`python -c 'import __graft_entry__ as g; g.build()'` -- there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status: int, what: str):
    if status != 0:
        msg = lib().hn_status_string(status).decode()
        raise RuntimeError(f"hashnerf_amd.{what} failed: {msg} (status {status})")


FAULT_BITS = {1: "ring slot wait", 2: "ring drain (tiles left unscattered)", 4: "coarse-grad flag wait",
              8: "dW buffer wait", 16: "binned-scatter overflow records exhausted",
              32: "non-finite (NaN / Inf) feature gradient or sample point in the binned scatter",
              64: "gradient on a table row pair the live mask marks dead (fused table step)"}


def check_device_faults(clear: bool = True):
    """Raise if a kernel reported a failed bounded wait since the last clear
    (hn_device_faults; synchronises the device)."""
    w = C.c_int32(0)
    check(lib().hn_device_faults(C.byref(w), int(clear)), "device_faults")
    if w.value:
        what = ", ".join(v for k, v in FAULT_BITS.items() if w.value & k) or str(w.value)
        raise RuntimeError(f"hashnerf_amd: the render backward reported a fault ({what}); "
                           "the gradients of the launches since the last check are invalid")


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(*tensors: torch.Tensor):
    """The product path runs only on a ROCm device: fail loudly otherwise."""
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("hashnerf_amd: tensors must live on a ROCm (HIP) device; "
                               "the reference CPU path is not part of this package")
        if t.dtype != torch.float32:
            raise TypeError(f"hashnerf_amd: expected float32, got {t.dtype}")


def contig(t: Optional[torch.Tensor]):
    return None if t is None else t.contiguous()


def make_grid(n_levels, n_features, log2T, box_min, box_max, grid_sizes) -> HnGrid:
    g = HnGrid()
    g.n_levels, g.n_features, g.log2_hashmap_size = int(n_levels), int(n_features), int(log2T)
    bmin = [float(v) for v in box_min]
    bmax = [float(v) for v in box_max]
    for a in range(3):
        g.box_min[a] = bmin[a]
        g.box_max[a] = bmax[a]
    for l, row in enumerate(grid_sizes):
        for a in range(3):
            g.grid_size[l][a] = float(row[a])
    return g


def make_mlp(ws) -> HnMlp:
    m = HnMlp()
    for k, t in zip(("sigma0", "sigma1", "color0", "color1", "color2"), ws):
        setattr(m, k, t.data_ptr())
    return m


def make_mlp_grad(gs) -> HnMlpGrad:
    m = HnMlpGrad()
    for k, t in zip(("sigma0", "sigma1", "color0", "color1", "color2"), gs):
        setattr(m, k, t.data_ptr())
    return m

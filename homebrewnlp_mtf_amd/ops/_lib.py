"""Loader for the in-tree gfx950 kernel library (``homebrewnlp_mtf_amd/_kernels.so``, built by ``make`` /
``__graft_entry__.build``) through a plain C ABI.

Why ctypes and not a torch C++ extension: the kernels only need raw device pointers and a stream, the C ABI is
independent of the torch/HIP C++ ABI (torch ships its own ROCm 7.0 runtime while hipcc is 7.2), and a launch
costs ~2 us of host time. Every launch is also captured correctly by ``torch.cuda.graphs`` because it is issued
on the current torch stream.

On a GPU box the library MUST load: ops on CUDA tensors raise ``KernelLibraryMissing`` instead of silently falling
back to PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("OBST_KERNELS", os.path.join(_HERE, "_kernels.so"))

_lib = None
_lock = threading.Lock()


class KernelLibraryMissing(RuntimeError):
    pass


class KernelError(RuntimeError):
    pass


c_p = ctypes.c_void_p
c_ll = ctypes.c_longlong
c_i = ctypes.c_int
c_f = ctypes.c_float


class GemmDesc(ctypes.Structure):
    _fields_ = [("A", c_p), ("B", c_p), ("C", c_p), ("R", c_p), ("Zout", c_p), ("Zin", c_p),
                ("lda", c_ll), ("ldb", c_ll), ("ldc", c_ll),
                ("a_s1", c_ll), ("a_s2", c_ll), ("b_s1", c_ll), ("b_s2", c_ll), ("c_s1", c_ll), ("c_s2", c_ll),
                ("M", c_i), ("N", c_i), ("K", c_i), ("batch1", c_i), ("batch2", c_i),
                ("a_t", c_i), ("b_t", c_i), ("out_f32", c_i), ("act", c_i), ("mode", c_i),
                ("alpha", c_f), ("beta", c_f), ("tri", c_i), ("kin", c_i), ("a_sk", c_ll), ("b_sk", c_ll)]


class AttnDesc(ctypes.Structure):
    _fields_ = [("Q", c_p), ("K", c_p), ("V", c_p), ("O", c_p), ("dO", c_p),
                ("Oout", c_p), ("dQ", c_p), ("dK", c_p), ("dV", c_p), ("LSE", c_p), ("delta", c_p),
                ("B", c_i), ("S", c_i), ("H", c_i), ("D", c_i), ("ld", c_ll), ("scale", c_f), ("causal", c_i),
                ("ld_o", c_ll), ("Res", c_p), ("Sum", c_p)]


class MapDesc(ctypes.Structure):
    _fields_ = [("Q", c_p), ("K", c_p), ("V", c_p), ("O", c_p), ("dO", c_p),
                ("Out", c_p), ("dQ", c_p), ("dK", c_p), ("dV", c_p), ("bias", c_p), ("cmap", c_p),
                ("dbias", c_p), ("dcmap", c_p), ("dbias_out", c_p), ("dcmap_out", c_p), ("LSE", c_p), ("delta", c_p),
                ("B", c_i), ("S", c_i), ("H", c_i), ("D", c_i), ("bsplit", c_i), ("scale", c_f), ("causal", c_i)]


class NormDesc(ctypes.Structure):
    _fields_ = [("X", c_p), ("scale", c_p), ("shift", c_p), ("Y", c_p), ("stats", c_p),
                ("DY", c_p), ("DX", c_p), ("dscale", c_p), ("dshift", c_p), ("partial", c_p), ("ext", c_p),
                ("rows", c_ll), ("F", c_i), ("groups", c_i), ("Ffull", c_i), ("eps", c_f), ("R", c_p), ("ws", c_p),
                ("R32", c_p), ("DX32", c_p), ("act", c_i), ("in_relu", c_i)]


class EwDesc(ctypes.Structure):
    _fields_ = [("X", c_p), ("Z", c_p), ("Y", c_p), ("sptr", c_p), ("n", c_ll), ("op", c_i), ("act", c_i),
                ("alpha", c_f), ("beta", c_f), ("seed", ctypes.c_ulonglong), ("keep", c_f)]


class OptDesc(ctypes.Structure):
    _fields_ = [("tensors", c_p), ("chunks", c_p), ("ntensors", c_i), ("nchunks", c_i),
                ("grad", c_p), ("uin", c_p), ("uout", c_p), ("master", c_p), ("compute", c_p),
                ("stats", c_p), ("fac", c_p), ("sstate", c_p), ("mom", c_p), ("adam_m", c_p), ("adam_v", c_p),
                ("sm3_old", c_p), ("sm3_new", c_p), ("af_state", c_p), ("af_rows_sum", c_p), ("af_cols_sum", c_p),
                ("stages", c_i * 32), ("nst", c_i), ("final_seg", c_i), ("emit_stats", c_i), ("emit_factored", c_i),
                ("lr", c_f), ("wd", c_f), ("rezero_mult", c_f), ("grad_scale", c_f), ("beta1", c_f), ("beta2", c_f),
                ("step_count", c_f), ("tp_size", c_i), ("dyn", c_p), ("part", c_p), ("part_base", c_i)]


_SIGS = {
    "obst_gemm": [ctypes.POINTER(GemmDesc), c_p],
    "obst_attn_fwd": [ctypes.POINTER(AttnDesc), c_p],
    "obst_attn_bwd": [ctypes.POINTER(AttnDesc), c_p],
    "obst_attn_fwd_bias": [ctypes.POINTER(AttnDesc), c_p, c_p],
    "obst_attn_bwd_bias": [ctypes.POINTER(AttnDesc), c_p, c_p, c_p, c_p],
    "obst_attn_map_fwd": [ctypes.POINTER(MapDesc), c_p],
    "obst_attn_map_bwd": [ctypes.POINTER(MapDesc), c_p],
    "obst_attn_map_bsplit": [c_i, c_i, c_i],
    "obst_norm_fwd": [ctypes.POINTER(NormDesc), c_p],
    "obst_norm_bwd": [ctypes.POINTER(NormDesc), c_p],
    "obst_norm_partial": [ctypes.POINTER(NormDesc), c_p],
    "obst_norm_bwd_ws": [ctypes.POINTER(NormDesc)],
    "obst_elementwise": [ctypes.POINTER(EwDesc), c_p],
    "obst_dot": [c_p, c_p, c_p, c_p, c_ll, c_p],
    "obst_dot_parts": [c_ll],
    "obst_scatter_add_sorted": [c_p, c_p, c_p, c_p, c_ll, c_i, c_p],
    "obst_gather": [c_p, c_p, c_p, c_ll, c_i, c_i, c_p],
    "obst_scatter_add": [c_p, c_p, c_p, c_ll, c_i, c_i, c_p],
    "obst_scatter_add_chunked": [c_p, c_p, c_p, c_p, c_p, c_ll, c_i, c_p, c_p],
    "obst_scatter_ws": [c_ll, c_i],
    "obst_cumsum": [c_p, c_p, c_ll, c_i, c_ll, c_i, c_i, c_i, c_p],
    "obst_cast_f32_bf16": [c_p, c_p, c_ll, c_p],
    "obst_add2_f32_bf16": [c_p, c_p, c_p, c_ll, c_p],
    "obst_cast_bf16_f32": [c_p, c_p, c_ll, c_p],
    "obst_tril": [c_p, c_p, c_ll, c_ll, c_p],
    "obst_zero": [c_p, c_ll, c_p],
    "obst_copy2d": [c_p, c_p, c_ll, c_ll, c_ll, c_ll, c_i, c_ll, c_ll, c_p],
    "obst_transpose": [c_p, c_p, c_ll, c_ll, c_ll, c_ll, c_i, c_ll, c_ll, c_p],
    "obst_mix_f32": [c_p, c_p, c_p, c_p, c_ll, c_f, c_f, c_p],
    "obst_xent_fwd": [c_p, c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_f, c_p],
    "obst_xent_bwd": [c_p, c_p, c_p, c_p, c_p, c_f, c_ll, c_i, c_i, c_f, c_p],
    "obst_opt_stats": [ctypes.POINTER(OptDesc), c_p],
    "obst_opt_scalar": [ctypes.POINTER(OptDesc), c_p],
    "obst_opt_apply": [ctypes.POINTER(OptDesc), c_p],
    "obst_opt_fold": [ctypes.POINTER(OptDesc), c_p, c_i, c_p],
    "obst_opt_apply_rows": [ctypes.POINTER(OptDesc), c_p, c_i, c_p],
    "obst_opt_factored": [ctypes.POINTER(OptDesc), c_p, c_p, c_i, c_p, c_i, c_p, c_p, c_p],

    "obst_glu": [c_p, c_p, c_p, c_p, c_p, c_ll, c_p],
    "obst_pkm_top1": [c_p, c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_p],
    "obst_pkm_top1_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_p],
    "obst_pkm_gather": [c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_i, c_p],
    "obst_pkm_gather_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_i, c_p],
    "obst_moe_fwd": [c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_p],
    "obst_moe_bwd": [c_p, c_p, c_p, c_p, c_p, c_ll, c_i, c_i, c_p],
    "obst_sum_axis": [c_p, c_p, c_ll, c_i, c_ll, c_p],
    "obst_axial_fwd": [c_p, c_p, c_i, c_i, c_p, c_p],
    "obst_axial_bwd": [c_p, c_p, c_i, c_i, c_p, c_p, c_p],
    "obst_sample": [c_p, c_ll, c_i, c_i, c_p, c_p, c_p, c_p, c_i, c_p, ctypes.c_ulonglong, c_p, c_p],
    "obst_sample_parts": [c_ll, c_i],
    "obst_frames": [c_p, c_i, c_p, c_ll, c_i, c_i, c_i, c_p],
    "obst_l1": [c_p, c_p, c_p, c_ll, c_ll, c_p, c_p, c_p, c_f, c_p],
    "obst_skinny_gemm": [c_p, c_i, c_p, c_i, c_p, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_f, c_i, c_p],
    "obst_skinny_ws": [c_i, c_i, c_i],
    "obst_calib_mfma": [c_p, c_i, c_p],
    "obst_calib_mfma_flops": [c_i],
    "obst_decode_attn": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_f, c_i, c_p, c_p],
}
_RESTYPES = {"obst_calib_mfma_flops": ctypes.c_double, "obst_norm_bwd_ws": c_ll, "obst_skinny_ws": c_ll, "obst_scatter_ws": c_ll}


def lib():
    """The loaded kernel library; raises ``KernelLibraryMissing`` if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise KernelLibraryMissing(f"{LIB_PATH} not found: run `make` (or __graft_entry__.build()) first; "
                                           "GPU ops never fall back to PyTorch")
            torch.cuda.init()  # the HIP runtime torch bundles must be loaded before our library binds to it
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, args in _SIGS.items():
                fn = getattr(handle, name)
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, c_i)
            _lib = handle
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except (KernelLibraryMissing, OSError, RuntimeError):
        return False


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def check(rc: int, what: str):
    if rc != 0:
        raise KernelError(f"{what} failed with code {rc} (negative: host-side shape/alignment check; positive: "
                          f"hipError_t)")


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()

"""ctypes binding of libcsm_hip.so (include/csm_hip.h).

The shared library is the only compute path: if it is missing or no GPU is
visible, every compute call raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CSM_HIP_LIB: A/B-test another in-tree build of the same ABI (profiling only)
LIB_PATH = os.environ.get("CSM_HIP_LIB") or os.path.join(_HERE, "libcsm_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "csm_hip.h")
PROF_HEADER_PATH = os.path.join(os.path.dirname(HEADER_PATH), "csm_hip_prof.h")  # tuning / profiling hooks

CSM_OK, CSM_ERR_ARG, CSM_ERR_HIP, CSM_ERR_STATE, CSM_ERR_TOO_LONG = 0, -1, -2, -3, -4
CSM_F32, CSM_BF16, CSM_Q4, CSM_U32 = 0, 1, 2, 3


class CsmLlamaDims(ctypes.Structure):
    _fields_ = [("n_layers", ctypes.c_int), ("hidden", ctypes.c_int), ("n_heads", ctypes.c_int),
                ("n_kv_heads", ctypes.c_int), ("head_dim", ctypes.c_int), ("intermediate", ctypes.c_int),
                ("eps", ctypes.c_float)]


class CsmDims(ctypes.Structure):
    _fields_ = [("backbone", CsmLlamaDims), ("decoder", CsmLlamaDims), ("n_text_vocab", ctypes.c_int),
                ("n_audio_vocab", ctypes.c_int), ("n_audio_codebooks", ctypes.c_int),
                ("max_seq_len", ctypes.c_int)]


class MimiDims(ctypes.Structure):
    _fields_ = [("channels", ctypes.c_int), ("dimension", ctypes.c_int), ("n_filters", ctypes.c_int),
                ("n_ratios", ctypes.c_int), ("ratios", ctypes.c_int * 8), ("kernel_size", ctypes.c_int),
                ("residual_kernel_size", ctypes.c_int), ("last_kernel_size", ctypes.c_int),
                ("compress", ctypes.c_int), ("num_heads", ctypes.c_int), ("num_layers", ctypes.c_int),
                ("dim_feedforward", ctypes.c_int), ("context", ctypes.c_int), ("n_q", ctypes.c_int),
                ("bins", ctypes.c_int), ("codebook_dim", ctypes.c_int), ("downsample_stride", ctypes.c_int),
                ("norm_eps", ctypes.c_float), ("gelu_erf", ctypes.c_int), ("attn_mode", ctypes.c_int)]


class CsmHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


_lib = None


def declared_symbols(headers=(HEADER_PATH, PROF_HEADER_PATH)):
    """Function names declared in include/csm_hip.h (the reference-facing ABI) and
    include/csm_hip_prof.h (profiling hooks)."""
    out = set()
    for h in headers:
        out |= set(re.findall(r"^\s*(?:int|const char\*)\s+((?:csm|mimi)_\w+)\s*\(", open(h).read(), re.M))
    return sorted(out)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        P, I, F, U64, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, ctypes.c_int64
        sig = {
            "csm_last_error": ([], ctypes.c_char_p),
            "csm_device_count": ([ctypes.POINTER(I)], I),
            "csm_engine_create": ([ctypes.POINTER(CsmDims), I, I, I, I, ctypes.POINTER(P)], I),
            "csm_engine_destroy": ([P], I),
            "csm_load_tensor": ([P, ctypes.c_char_p, P, I, ctypes.POINTER(I64), I], I),
            "csm_set_rope_table": ([P, I, P, I, I], I),
            "csm_weights_ready": ([P], I),
            "csm_quantize": ([P, I, I], I),
            "csm_begin": ([P, I, P, F, I], I),
            "csm_set_sampler_filters": ([P, ctypes.c_double, ctypes.c_double, I], I),
            "csm_prefill": ([P, I, I, P, P], I),
            "csm_prefill_batch": ([P, I, P, P, P, P], I),
            "csm_run_frames": ([P, I, ctypes.POINTER(I)], I),
            "csm_run_frames_ahead": ([P, I, ctypes.POINTER(I)], I),
            "csm_frame_step": ([P, P, P], I),
            "csm_frame_c0_logits": ([P, P], I),
            "csm_frame_finish": ([P, P, ctypes.POINTER(I)], I),
            "csm_frame_forced": ([P, P, P, P, P], I),
            "csm_frame_host_step": ([P, P, P, ctypes.POINTER(I)], I),
            "csm_read_codes": ([P, P, P, P, ctypes.POINTER(I)], I),
            "csm_debug_read": ([P, ctypes.c_char_p, P, I64, ctypes.POINTER(I64)], I),
            "csm_codes_device_ptr": ([P, ctypes.POINTER(P)], I),
            "csm_read_rows": ([P, ctypes.c_char_p, I, P, P], I),
            "csm_linear": ([P, ctypes.c_char_p, I, P, P], I),
            "csm_synchronize": ([P], I),
            "csm_set_option": ([P, ctypes.c_char_p, I], I),
            "csm_xs_shape": ([I, I, I, I, I, ctypes.POINTER(I)], I),
            "csm_q4_gemv_shape": ([I, I, ctypes.POINTER(I)], I),
            "csm_q4_expand": ([P, I, P], I),
            "csm_bench_gemv": ([P, I, I, I, ctypes.POINTER(F), ctypes.POINTER(ctypes.c_double)], I),
            "csm_bench_dec_frame": ([P, I, ctypes.POINTER(F), ctypes.POINTER(ctypes.c_double)], I),
            "csm_bench_bb_step": ([P, I, ctypes.POINTER(F), ctypes.POINTER(ctypes.c_double)], I),
            "csm_bench_dec_xsd": ([P, I, ctypes.POINTER(F), ctypes.POINTER(ctypes.c_double)], I),
            "csm_weight_buffers": ([P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), I,
                                    ctypes.POINTER(I)], I),
            "csm_weights_received": ([P], I),
            "mimi_create": ([ctypes.POINTER(MimiDims), I, I, I, ctypes.POINTER(P)], I),
            "mimi_destroy": ([P], I),
            "mimi_load_tensor": ([P, ctypes.c_char_p, P, I, ctypes.POINTER(I64), I], I),
            "mimi_set_rope_table": ([P, P, I, I], I),
            "mimi_weights_ready": ([P], I),
            "mimi_encode": ([P, I, I, P, P, ctypes.POINTER(I)], I),
            "mimi_encode_rows": ([P, I, I, P, P, P, ctypes.POINTER(I)], I),
            "mimi_decode": ([P, I, I, P, I, I, P, I], I),
            "mimi_reset_state": ([P, I], I),
            "mimi_decode_step": ([P, I, P, P], I),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc: int):
    if rc == CSM_OK:
        return
    msg = lib().csm_last_error().decode(errors="replace")
    if rc == CSM_ERR_ARG:
        raise ValueError(msg)
    if rc == CSM_ERR_TOO_LONG:
        raise ValueError(msg)
    raise CsmHipError(rc, msg)


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().csm_device_count(ctypes.byref(n)))
    return n.value


def ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def shape_arr(shape):
    return (ctypes.c_int64 * len(shape))(*shape)


def host_tensor(a):
    """(contiguous array, csm dtype) for float32 / bf16-bits (uint16) / packed-int4 (uint32) host data."""
    a = np.asarray(a)
    if a.dtype == np.uint32:  # MLX-packed int4 (QuantizedLinear / QuantizedEmbedding .weight)
        return np.ascontiguousarray(a), CSM_U32
    if a.dtype == np.uint16:
        return np.ascontiguousarray(a), CSM_BF16
    if str(a.dtype) == "bfloat16":  # ml_dtypes-style arrays
        return np.ascontiguousarray(a.view(np.uint16)), CSM_BF16
    return np.ascontiguousarray(a, dtype=np.float32), CSM_F32

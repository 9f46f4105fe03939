"""ctypes binding of libquantizations.so (declarations: include/quantizations.h).

The library is the product: there is no CPU or PyTorch fallback.  If the
shared object is missing or does not export a declared symbol, importing this
module raises immediately.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so the library binds to the same one

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QZ_LIB_PATH", os.path.join(HERE, "libquantizations.so"))

DT_F16, DT_BF16, DT_F32 = 0, 1, 2
FP4, NF4 = 0, 1
QUANT_TYPES = {"fp4": FP4, "nf4": NF4}
EXACT_CODES = 0x100  # QZ_EXACT_CODES: GEMV quant_type flag, decode with the fp32 codes

_STATUS = {
    -1: "invalid argument (null pointer or negative size)",
    -2: "unsupported blocksize",
    -3: "unsupported shape",
    -4: "unsupported dtype or quant type",
}

_p = ctypes.c_void_p
_i = ctypes.c_int
_ll = ctypes.c_longlong
_f = ctypes.c_float

GEMV_MAX_SEGMENTS = 4  # QZ_GEMV_MAX_SEGMENTS
QZ_ERR_SHAPE = -3


class GemvSegment(ctypes.Structure):
    """struct qz_gemv_segment (include/quantizations.h)."""
    _fields_ = [("M", ctypes.c_int), ("B", ctypes.c_void_p), ("absmax", ctypes.c_void_p),
                ("qabsmax", ctypes.c_void_p), ("absmax2", ctypes.c_void_p), ("code2", ctypes.c_void_p),
                ("offset", ctypes.c_void_p), ("block_base", ctypes.c_longlong), ("bias", ctypes.c_void_p),
                ("y", ctypes.c_void_p)]


# name -> argtypes (restype int unless noted); mirrors include/quantizations.h
SIGNATURES = {
    "cgemm_4bit_inference_naive_fp32": [_i, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i],
    "cquantize_blockwise_fp16_fp4": [_p, _p, _p, _p, _i, _i],
    "cdequantize_blockwise_fp16_fp4": [_p, _p, _p, _p, _i, _i],
    "cquantize_blockwise_fp32": [_p, _p, _p, _p, _i, _i],
    "cdequantize_blockwise_fp32": [_p, _p, _p, _p, _i, _i],
    "cgemm_4bit_inference_naive_fp32_stream": [_i, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p],
    "cquantize_blockwise_fp16_fp4_stream": [_p, _p, _p, _p, _i, _i, _p],
    "cdequantize_blockwise_fp16_fp4_stream": [_p, _p, _p, _p, _i, _i, _p],
    "cquantize_blockwise_fp32_stream": [_p, _p, _p, _p, _i, _i, _p],
    "cdequantize_blockwise_fp32_stream": [_p, _p, _p, _p, _i, _i, _p],
    "qz_gemv_4bit": [_i, _i, _p, _i, _p, _i, _i, _p, _p, _p, _p, _p, _i, _ll, _p, _p, _p, _p],
    "qz_gemv_4bit_residual": [_i, _i, _p, _i, _p, _i, _i, _p, _p, _p, _p, _p, _i, _ll, _p, _p, _p, _p, _p],
    "qz_gemv_4bit_grouped": [_i, _p, _i, _p, _i, _i, _i, _i, _p, _p],
    "qz_gemv_4bit_grouped_rmsnorm": [_i, _p, _i, _p, _i, _i, _i, _i, _p, _p, _f, _p],
    "qz_gemv_4bit_pair_silu": [_p, _i, _p, _i, _i, _i, _i, _p, _p, _f, _p, _p],
    "qz_decode_attention": [_i, _i, _i, _i, _i, _i, _p, _ll, _p, _ll, _p, _ll, _p, _p, _ll, _p, _p, _p, _ll, _ll,
                            _p, _p, _p, _ll, _p, _f, _p],
    "qz_gemm_4bit": [_i, _i, _i, _p, _i, _i, _p, _i, _i, _p, _p, _p, _p, _p, _i, _p, _p, _i, _p, _ll, _p],
    "qz_gemm_4bit_workspace_size": [_i, _i, _i],
    "qz_gemm_16bit": [_i, _i, _i, _p, _i, _i, _p, _p, _p, _i, _p],
    "qz_gemm_16bit_ok": [_i, _i, _i, _p, _i, _p, _p, _i],
    "qz_gemm_4bit_grouped": [_i, _p, _i, _i, _p, _i, _i, _i, _i, _i, _p],
    "qz_quantize_4bit": [_p, _i, _ll, _i, _i, _p, _p, _p],
    "qz_absmax_mean_workspace": [_ll],
    "qz_absmax_mean": [_p, _ll, _p, _p, _p],
    "qz_quantize_blockwise_8bit": [_p, _p, _ll, _i, _p, _p, _p, _p],
    "qz_dequantize_blockwise_8bit": [_p, _p, _p, _ll, _i, _p, _p, _p],
    "qz_dequantize_4bit": [_p, _ll, _i, _i, _p, _p, _p, _p, _p, _i, _p, _i, _p],
    "qz_rmsnorm": [_p, _i, _ll, _i, _ll, _p, _f, _p, _ll, _p],
    "qz_rope_qk": [_i, _i, _i, _i, _p, _i, _p, _p, _p, _p, _i, _p, _p, _p, _p, _p, _p, _p],
    "qz_silu_mul": [_p, _p, _i, _ll, _p, _p],
    "qz_decode_mask": [_p, _i, _i, _p, _p],
    "qz_gemv_dense": [_i, _i, _p, _i, _p, _p, _p],
    "qz_greedy_step": [_p, _i, _i, _ll, _ll, _p, _ll, _ll, _p, _p, _p, _p],
    "qz_greedy_step_work_bytes": [_i, _ll],
    "qz_rope_table": [_i, _i, _i, _i, _p, _ll, _ll, _p, _p, _ll, _p, _f, _p, _p, _p],
    "qz_add_rmsnorm": [_p, _p, _i, _ll, _i, _ll, _p, _f, _p, _p, _ll, _p],
    "qz_bench_read_floor": [_p, _ll, _p, _p],
    "qz_bench_empty": [_p, _p],
    "qz_ipc_handle_size": [],
    "qz_exchange_bytes": [_i, _ll],
    "qz_exchange_alloc": [_ll, _p],
    "qz_exchange_free": [_p],
    "qz_ipc_get_handle": [_p, _p],
    "qz_ipc_open_handle": [_p, _p],
    "qz_ipc_close_handle": [_p],
    "qz_enable_peer_access": [_i],
    "qz_allgather_oneshot": [_p, _i, _p, _i, _i, _p, _p, _ll, _p, _p, _p],
    "qz_allgather_oneshot_mode": [_p, _i, _p, _i, _i, _p, _p, _ll, _p, _p, _i, _p],
    "qz_gemv_knobs": [_p, _i],
    "qz_gemv_set_knob": [ctypes.c_char_p, _i],
    "qz_version": [],
}
RESTYPES = {"qz_absmax_mean_workspace": _ll, "qz_gemm_4bit_workspace_size": _ll, "qz_exchange_bytes": _ll,
            "qz_greedy_step_work_bytes": _ll}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libquantizations.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the export is missing -> loud
        fn.argtypes = args
        fn.restype = RESTYPES.get(name, _i)
    return lib


lib = _load()


class QuantizationsError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _STATUS.get(rc, f"HIP error {rc}")
        raise QuantizationsError(f"{what} failed: {msg}")


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float16:
        return DT_F16
    if dt == torch.bfloat16:
        return DT_BF16
    if dt == torch.float32:
        return DT_F32
    raise NotImplementedError(f"dtype {dt} is not supported by the 4-bit kernels")


def stream_of(t: torch.Tensor) -> int:
    """HIP stream handle of torch's current stream on t's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def gemv_knobs() -> dict:
    """The decode launchers' measurement knobs as the library read them at load (qz_gemv_knobs)."""
    import json
    buf = ctypes.create_string_buffer(512)
    n = lib.qz_gemv_knobs(buf, len(buf))
    return json.loads(buf.value.decode()) if 0 < n < len(buf) else {}


def set_gemv_knob(name: str, value: int) -> None:
    """Set one decode-launcher knob explicitly (qz_gemv_set_knob); the environment is read only once,
    at library load."""
    check(lib.qz_gemv_set_knob(name.encode(), int(value)), f"qz_gemv_set_knob({name})")

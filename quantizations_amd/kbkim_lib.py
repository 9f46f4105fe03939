"""Drop-in replacement for the reference's native module ``kbkim_lib``.

The reference builds ``kbkim_lib.so`` from pythonInterface.cpp:154-178: five
functions taking device pointers as Python ints (``"iiiKKKKKiiii"`` /
``"KKKKii"``, pythonInterface.cpp:56,77,97,117,137).  This module exposes the
same five callables with the same argument order, backed by the ``extern "C"``
symbols of libquantizations.so through ctypes.  Differences (documented in
INTEGRATION.md): launches go to torch's current HIP stream instead of the
legacy default stream, and a failing launch raises ``RuntimeError`` instead of
being silently ignored.  Argument-type errors raise ``TypeError`` like
``PyArg_ParseTuple`` does.
"""
from __future__ import annotations

import torch

from . import _lib


def _ints(name, vals, n):
    if len(vals) != n:
        raise TypeError(f"{name}() takes exactly {n} arguments ({len(vals)} given)")
    for v in vals:
        if not isinstance(v, int) or isinstance(v, bool):
            raise TypeError(f"{name}(): an integer is required (got {type(v).__name__})")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def cgemm_4bit_inference_naive_fp32(*args):
    """(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize) -- pythonInterface.cpp:52-69."""
    _ints("cgemm_4bit_inference_naive_fp32", args, 12)
    _lib.check(_lib.lib.cgemm_4bit_inference_naive_fp32_stream(*args, _stream()), "cgemm_4bit_inference_naive_fp32")


def cquantize_blockwise_fp16_fp4(*args):
    """(code, A, absmax, out, blocksize, n) -- pythonInterface.cpp:73-89."""
    _ints("cquantize_blockwise_fp16_fp4", args, 6)
    _lib.check(_lib.lib.cquantize_blockwise_fp16_fp4_stream(*args, _stream()), "cquantize_blockwise_fp16_fp4")


def cdequantize_blockwise_fp16_fp4(*args):
    """(code, A, absmax, out, blocksize, n) -- pythonInterface.cpp:93-109."""
    _ints("cdequantize_blockwise_fp16_fp4", args, 6)
    _lib.check(_lib.lib.cdequantize_blockwise_fp16_fp4_stream(*args, _stream()), "cdequantize_blockwise_fp16_fp4")


def cquantize_blockwise_fp32(*args):
    """(code, A, absmax, out, blocksize, n) -- pythonInterface.cpp:113-129."""
    _ints("cquantize_blockwise_fp32", args, 6)
    _lib.check(_lib.lib.cquantize_blockwise_fp32_stream(*args, _stream()), "cquantize_blockwise_fp32")


def cdequantize_blockwise_fp32(*args):
    """(code, A, absmax, out, blocksize, n) -- pythonInterface.cpp:133-149."""
    _ints("cdequantize_blockwise_fp32", args, 6)
    _lib.check(_lib.lib.cdequantize_blockwise_fp32_stream(*args, _stream()), "cdequantize_blockwise_fp32")

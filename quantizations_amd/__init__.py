"""quantizations_amd -- MI355X (gfx950) native 4-bit Linear4bit.

Drop-in for the reference kkbwilldo/quantizations (``core``, ``modules``,
``kbkim_lib``): same classes/functions, backed by hand-written HIP kernels in
``libquantizations.so`` (C-ABI: include/quantizations.h).
"""
from ._lib import LIB_PATH, QuantizationsError  # noqa: F401  (loads the native library; fails loudly)
from .core import (  # noqa: F401
    Params4bit,
    QuantState,
    create_dynamic_map,
    dequantize_4bit,
    dequantize_blockwise,
    gemm_4bit,
    gemv_4bit,
    get_4bit_type,
    get_ptr,
    quantize_4bit,
    quantize_blockwise,
)
from .modules import Linear4bit, matmul_4bit  # noqa: F401

__version__ = "0.1.0"

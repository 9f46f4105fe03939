"""Functional 4-bit API -- same names, arguments and errors as the reference
``core.py``, running on the MI355X-native kernels of libquantizations.so.

Reference map (kkbwilldo/quantizations, core.py):
  QuantState            :23-88     Params4bit           :91-190
  get_4bit_type         :193-229   get_ptr              :232-248
  create_dynamic_map    :251-314   quantize_blockwise   :317-366
  dequantize_blockwise  :369-423   gemv_4bit            :426-504
  quantize_4bit         :507-578   dequantize_4bit      :581-634

What differs, on purpose (DESIGN.md "Host layer"):
  * ``quant_type="nf4"`` is supported (the reference only knows "fp4").
  * ``compress_statistics`` (bnb's name for double quant) is honoured; the
    reference always double-quantises.
  * ``gemv_4bit`` is ONE fused launch (scale rebuild, LUT decode, dot, cast,
    bias) instead of dequantize_blockwise + ``+= offset`` + GEMV; no
    per-call allocation besides the output.
  * the absmax mean is a fixed-order fp64 reduction (deterministic), not
    torch's fp32 ``mean()``.
  * every launch goes to torch's current stream; failures raise.
"""
from __future__ import annotations

import copy
import ctypes
import json
import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._lib import check, dtype_code, lib, ptr

name2qmap: dict = {}

dtype2bytes = {torch.uint8: 1}

_VALID_BLOCKSIZES = (4096, 2048, 1024, 512, 256, 128, 64)

# NF4 codebook: reference csrc/kernels.cu:851 (q_data)
NF4_CODE = [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453, -0.28444138169288635,
            -0.18477343022823334, -0.09105003625154495, 0.0, 0.07958029955625534, 0.16093020141124725,
            0.24611230194568634, 0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
            0.7229568362236023, 1.0]


class QuantState:
    """Container of the 4-bit quantisation statistics (reference core.py:23-88)."""

    valid_quant_types = ("fp4", "nf4")
    valid_qs_keys = [
        "absmax", "quant_map", "nested_absmax", "nested_quant_map", "quant_state", "quant_type",
        "blocksize", "dtype", "shape", "nested_blocksize", "nested_dtype", "nested_offset",
    ]

    def __init__(self, absmax, shape=None, code=None, blocksize=None, quant_type=None, dtype=None, offset=None,
                 state2=None):
        self.absmax = absmax
        self.shape = shape
        self.code = code
        self.dtype = dtype
        self.blocksize = blocksize
        self.quant_type = quant_type
        self.offset = offset
        self.state2 = state2
        self.nested = state2 is not None

    def to(self, device):
        """Move the statistics to `device` (reference core.py:78-88; also valid without double quant)."""
        self.absmax = self.absmax.to(device)
        if self.code is not None:
            self.code = self.code.to(device)
        if self.nested:
            self.offset = self.offset.to(device)
            self.state2.absmax = self.state2.absmax.to(device)
            self.state2.code = self.state2.code.to(device)

    # -- scale-source view used by every 4-bit consumer --------------------
    def scale_args(self):
        """(absmax, qabsmax, absmax2, code2, offset, blocksize2) pointers for the C-ABI."""
        if self.nested:
            return (0, ptr(self.absmax), ptr(self.state2.absmax), ptr(self.state2.code), ptr(self.offset),
                    int(self.state2.blocksize))
        return (ptr(self.absmax), 0, 0, 0, 0, 0)

    # -- serialisation ------------------------------------------------------
    # Key names are the reference's valid_qs_keys (core.py:29-42), which it
    # declares but never serialises; the layout is the bitsandbytes one those
    # names come from, so checkpoints interoperate: tensors under their own
    # keys, every non-tensor field JSON-encoded into ONE uint8 tensor under
    # "quant_state.bitsandbytes__<quant_type>" (safetensors holds tensors only).
    PACKED_PREFIX = "quant_state.bitsandbytes__"

    def as_dict(self, packed: bool = False) -> dict:
        d = {
            "quant_type": self.quant_type,
            "absmax": self.absmax,
            "blocksize": self.blocksize,
            "quant_map": self.code,
            "dtype": str(self.dtype).replace("torch.", ""),
            "shape": tuple(self.shape),
        }
        if self.nested:
            d.update({
                "nested_absmax": self.state2.absmax,
                "nested_blocksize": self.state2.blocksize,
                "nested_quant_map": self.state2.code,
                "nested_dtype": str(self.state2.dtype).replace("torch.", ""),
                "nested_offset": float(self.offset.item()),
            })
        if not packed:
            return d
        out = {k: v for k, v in d.items() if isinstance(v, Tensor)}
        meta = {k: (list(v) if isinstance(v, tuple) else v) for k, v in d.items() if not isinstance(v, Tensor)}
        out[self.PACKED_PREFIX + self.quant_type] = _pack_json(meta)
        return out

    @classmethod
    def from_dict(cls, qs_dict: dict, device) -> "QuantState":
        """Rebuild from as_dict() output, packed or not.  Keys may carry a
        module prefix (e.g. "layers.0.q_proj.weight.absmax")."""
        d = {}
        for k, v in qs_dict.items():
            short = k[k.index(cls.PACKED_PREFIX):] if cls.PACKED_PREFIX in k else k.split(".")[-1]
            d[short] = v
        packed_keys = [k for k in d if k.startswith(cls.PACKED_PREFIX)]
        if len(packed_keys) > 1:
            raise ValueError(f"more than one packed quant_state entry: {packed_keys}")
        if packed_keys:
            d.update(_unpack_json(d.pop(packed_keys[0])))
        missing = [k for k in ("absmax", "quant_map", "quant_type", "blocksize", "dtype", "shape") if k not in d]
        if missing:
            raise ValueError(f"quant_state is missing {missing}")
        if d["quant_type"] not in cls.valid_quant_types:
            raise ValueError(f"unknown quant_type {d['quant_type']!r}")
        state2 = None
        offset = None
        if "nested_absmax" in d:
            state2 = cls(absmax=d["nested_absmax"].to(device), blocksize=int(d["nested_blocksize"]),
                         code=d["nested_quant_map"].to(device), dtype=getattr(torch, d["nested_dtype"]))
            off = d["nested_offset"]
            offset = (off if isinstance(off, Tensor) else torch.tensor(float(off))).to(device=device,
                                                                                       dtype=torch.float32)
        return cls(quant_type=d["quant_type"], absmax=d["absmax"].to(device), blocksize=int(d["blocksize"]),
                   code=d["quant_map"].to(device), dtype=getattr(torch, d["dtype"]), shape=torch.Size(d["shape"]),
                   offset=offset, state2=state2)


def _pack_json(obj: dict) -> Tensor:
    return torch.tensor(list(json.dumps(obj, sort_keys=True).encode("utf-8")), dtype=torch.uint8)


def _unpack_json(t: Tensor) -> dict:
    return json.loads(bytes(t.detach().cpu().to(torch.uint8).tolist()).decode("utf-8"))


class Params4bit(torch.nn.Parameter):
    """4-bit weight parameter (reference core.py:91-190); ``.to(cuda)`` quantises once."""

    def __new__(cls, data: Optional[Tensor] = None, requires_grad=False, quant_state: Optional[QuantState] = None,
                blocksize: int = 64, quant_type: str = "fp4", quant_storage: torch.dtype = torch.uint8,
                module=None, bnb_quantized: bool = False, compress_statistics: bool = True, **_ignored):
        if data is None:
            data = torch.empty(0)
        self = Tensor._make_subclass(cls, data, requires_grad)
        self.blocksize = blocksize
        self.quant_type = quant_type
        self.quant_state = quant_state
        self.quant_storage = quant_storage
        self.bnb_quantized = bnb_quantized
        self.compress_statistics = compress_statistics
        self.data = data
        self.module = module
        return self

    @classmethod
    def from_prequantized(cls, data: Tensor, quantized_stats: dict, requires_grad: bool = False, device="cuda",
                          module=None, **kwargs) -> "Params4bit":
        """A Params4bit around already-packed bytes and their statistics (the
        QuantState.as_dict keys, packed or not): loading a pre-quantised
        checkpoint never re-quantises."""
        qs = QuantState.from_dict(quantized_stats, device=device)
        self = cls(data.to(device), requires_grad=requires_grad, quant_state=qs, blocksize=qs.blocksize,
                   quant_type=qs.quant_type, quant_storage=data.dtype, module=module, bnb_quantized=True,
                   compress_statistics=qs.nested)
        if module is not None:
            module.quant_state = qs
        return self

    def __deepcopy__(self, memo):
        """A copy that keeps the 4-bit state (torch's Parameter.__deepcopy__ would rebuild an
        un-quantised Params4bit from the packed bytes, as bnb's own Params4bit avoids too): the
        packed bytes and the QuantState are copied, and the module back-reference follows the
        module when the whole module is being copied."""
        if id(self) in memo:
            return memo[id(self)]
        new = type(self)(self.data.clone(memory_format=torch.preserve_format), requires_grad=self.requires_grad,
                         quant_state=copy.deepcopy(self.quant_state, memo), blocksize=self.blocksize,
                         quant_type=self.quant_type, quant_storage=self.quant_storage,
                         module=memo.get(id(self.module), self.module), bnb_quantized=self.bnb_quantized,
                         compress_statistics=self.compress_statistics)
        memo[id(self)] = new
        return new

    def _quantize(self, device):
        w = self.data.contiguous().to(device)
        w_4bit, quant_state = quantize_4bit(w, blocksize=self.blocksize, quant_type=self.quant_type,
                                            quant_storage=self.quant_storage,
                                            compress_statistics=self.compress_statistics)
        self.data = w_4bit
        self.quant_state = quant_state
        if self.module is not None:
            self.module.quant_state = quant_state
        self.bnb_quantized = True
        return self

    def cuda(self, device=None, non_blocking: bool = False):
        return self.to(device="cuda" if device is None else device, non_blocking=non_blocking)

    def to(self, *args, **kwargs):
        device, dtype, non_blocking, _ = torch._C._nn._parse_to(*args, **kwargs)
        if device is not None and device.type == "cuda" and not self.bnb_quantized:
            return self._quantize(device)
        if self.quant_state is not None and device is not None:
            self.quant_state.to(device)
        new = Params4bit(super().to(device=device, dtype=dtype, non_blocking=non_blocking),
                         requires_grad=self.requires_grad, quant_state=self.quant_state, blocksize=self.blocksize,
                         quant_type=self.quant_type, quant_storage=self.quant_storage, module=self.module,
                         bnb_quantized=self.bnb_quantized, compress_statistics=self.compress_statistics)
        return new


def get_4bit_type(typename, device=None, blocksize=64):
    """16-entry codebook of `typename` (reference core.py:193-229; "nf4" = kernels.cu:851)."""
    if device is None:
        device = "cuda"
    if typename == "fp4":
        data = torch.tensor([0, 0.0625, 8.0, 12.0, 4.0, 6.0, 2.0, 3.0, -0, -0.0625, -8.0, -12.0, -4.0, -6.0, -2.0,
                             -3.0], device=device)
        data.div_(data.abs().max())
        return data
    if typename == "nf4":
        return torch.tensor(NF4_CODE, dtype=torch.float32, device=device)
    raise NotImplementedError(f"Typename {typename} not supported")


def get_ptr(A: Optional[Tensor]) -> int:
    """Device address of A, 0 for None (reference core.py:232-248)."""
    return 0 if A is None else A.data.data_ptr()


def create_dynamic_map(signed=True, max_exponent_bits=7, total_bits=8) -> Tensor:
    """Signed dynamic 8-bit code (reference core.py:251-314): for exponent i, the
    midpoints of linspace(0.1, 1, 2^i + 1) scaled by 10^(i-6), both signs, plus 0 and 1."""
    values = []
    non_sign_bits = total_bits - 1
    for i in range(max_exponent_bits):
        n = 2 ** (i + non_sign_bits - max_exponent_bits) + 1 if signed else \
            2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1
        grid = torch.linspace(0.1, 1, int(n))
        mids = (grid[:-1] + grid[1:]) / 2.0
        scale = 10 ** (-(max_exponent_bits - 1) + i)
        values.extend((scale * mids).tolist())
        if signed:
            values.extend((-scale * mids).tolist())
    extra = 2 ** (non_sign_bits - max_exponent_bits) - 1
    if extra > 0:
        grid = torch.linspace(0.1, 1, extra + 1)
        mids = (grid[:-1] + grid[1:]) / 2.0
        scale = 10 ** (-(max_exponent_bits - 1) + max_exponent_bits - 1)
        values.extend((scale * mids).tolist())
        if signed:
            values.extend((-scale * mids).tolist())
    values.extend([0, 1.0])
    assert len(values) == 2 ** total_bits
    values.extend([0] * (256 - len(values)))
    values.sort()
    return Tensor(values)


def _dynamic_code(device) -> Tensor:
    key = ("dynamic", str(device))
    if key not in name2qmap:
        name2qmap[key] = create_dynamic_map().to(device)
    return name2qmap[key]


def _require_cuda(t: Tensor, what: str):
    if t.device.type != "cuda":
        raise NotImplementedError(f"Device type not supported for {what}: {t.device.type}")


def quantize_blockwise(A: Tensor, blocksize=4096, offset: Optional[Tensor] = None) -> Tuple[Tensor, QuantState]:
    """8-bit blockwise quantisation with the dynamic code (reference core.py:317-366).
    `offset` (device scalar) fuses the reference's preceding ``A -= offset``."""
    _require_cuda(A, "blockwise quantization")
    assert blocksize in _VALID_BLOCKSIZES
    code = _dynamic_code(A.device)
    n = A.numel()
    blocks = (n + blocksize - 1) // blocksize
    absmax = torch.zeros((blocks,), device=A.device, dtype=torch.float32)
    out = torch.zeros_like(A, dtype=torch.uint8)
    A = A.contiguous().float()
    check(lib.qz_quantize_blockwise_8bit(ptr(code), ptr(A), n, blocksize, ptr(offset), ptr(absmax), ptr(out),
                                         _lib.stream_of(A)), "quantize_blockwise")
    return out, QuantState(absmax=absmax, code=code, blocksize=blocksize, dtype=torch.float32)


def dequantize_blockwise(A: Tensor, quant_state: Optional[QuantState] = None, absmax: Optional[Tensor] = None,
                         code: Optional[Tensor] = None, out: Optional[Tensor] = None, blocksize: int = 4096,
                         nested=False, offset: Optional[Tensor] = None) -> Tensor:
    """Inverse of quantize_blockwise (reference core.py:369-423); `offset` fuses ``+= offset``."""
    assert quant_state is not None or absmax is not None
    if quant_state is None:
        quant_state = QuantState(absmax=absmax, code=code if code is not None else _dynamic_code(A.device),
                                 blocksize=blocksize, dtype=torch.float32)
    if quant_state.blocksize not in _VALID_BLOCKSIZES:
        raise ValueError(f"The blockwise of {quant_state.blocksize} is not supported. "
                         f"Supported values: [2048, 4096, 1024, 512, 256, 128, 64]")
    if out is None:
        out = torch.empty(A.shape, dtype=torch.float32, device=A.device)
    check(lib.qz_dequantize_blockwise_8bit(ptr(quant_state.code), ptr(A), ptr(quant_state.absmax), A.numel(),
                                           quant_state.blocksize, ptr(offset), ptr(out), _lib.stream_of(A)),
          "dequantize_blockwise")
    return out


def quantize_4bit(A: Tensor, blocksize=64, quant_type="fp4", quant_storage=torch.uint8,
                  compress_statistics: bool = True) -> Tuple[Tensor, QuantState]:
    """Blockwise 4-bit quantisation (reference core.py:507-578): pack two codes per
    byte (high nibble first), then -- with double quant -- offset = mean(absmax)
    and an 8-bit blockwise code of absmax - offset with blocksize 256."""
    _require_cuda(A, "FP4 quantization")
    if quant_type not in QuantState.valid_quant_types:
        raise NotImplementedError(f"4-bit quantization data type {quant_type} is not implemented.")
    assert blocksize in _VALID_BLOCKSIZES
    if quant_storage != torch.uint8:
        raise NotImplementedError(f"quant_storage {quant_storage} is not supported (uint8 only)")
    n = A.numel()
    input_shape = A.shape
    A = A.contiguous()
    s = _lib.stream_of(A)
    blocks = (n + blocksize - 1) // blocksize
    absmax = torch.zeros((blocks,), device=A.device, dtype=torch.float32)
    out = torch.zeros(((n + 1) // 2, 1), dtype=torch.uint8, device=A.device)
    check(lib.qz_quantize_4bit(ptr(A), dtype_code(A.dtype), n, blocksize, _lib.QUANT_TYPES[quant_type], ptr(absmax),
                               ptr(out), s), "quantize_4bit")
    code = get_4bit_type(quant_type, device=A.device)
    if not compress_statistics:
        return out, QuantState(absmax=absmax, shape=input_shape, dtype=A.dtype, blocksize=blocksize, code=code,
                               quant_type=quant_type)
    offset = torch.empty((), device=A.device, dtype=torch.float32)
    ws = torch.empty(int(lib.qz_absmax_mean_workspace(blocks)), device=A.device, dtype=torch.float64)
    check(lib.qz_absmax_mean(ptr(absmax), blocks, ptr(ws), ptr(offset), s), "absmax mean")
    qabsmax, state2 = quantize_blockwise(absmax, blocksize=256, offset=offset)
    del absmax
    return out, QuantState(absmax=qabsmax, shape=input_shape, dtype=A.dtype, blocksize=blocksize, code=code,
                           quant_type=quant_type, offset=offset, state2=state2)


def dequantize_4bit(A: Tensor, quant_state: Optional[QuantState] = None, blocksize: int = 64, quant_type="fp4",
                    out_dtype: Optional[torch.dtype] = None) -> Tensor:
    """Full-weight dequantisation (reference core.py:581-634); returns ``out.t()``
    like the reference.  FP4 follows the dDequantizeFP4Tree semantics."""
    if blocksize not in _VALID_BLOCKSIZES:
        raise ValueError(f"The blockwise of {blocksize} is not supported. "
                         f"Supported values: [2048, 4096, 1024, 512, 256, 128, 64]")
    qt = quant_state.quant_type or quant_type
    if qt not in QuantState.valid_quant_types:
        raise NotImplementedError(f"4-bit quantization data type {qt} is not implemented.")
    dt = out_dtype or quant_state.dtype
    out = torch.empty(quant_state.shape, dtype=dt, device=A.device)
    check(lib.qz_dequantize_4bit(ptr(A), out.numel(), _lib.QUANT_TYPES[qt], quant_state.blocksize,
                                 *quant_state.scale_args(), ptr(out), dtype_code(dt), _lib.stream_of(A)),
          "dequantize_4bit")
    return out.t()


# Decode GEMV code table, chosen by activation dtype (the kernel picks the table; see
# _gemv_quant_type and gemv.hip's qz_gemv_4bit):
#  * fp32 x: the fp32 codebook values multiplied into the raw x (v_fma_f32) -- the
#    reference's own numerics (kernels.cu:1115-1120,1169-1170); the flag is ignored.
#  * bf16 x: each code as bf16 hi + lo (~2^-16) dotted against the raw bf16 x pairs;
#    the flag is ignored.
#  * fp16 x: `exact_codes` picks the exact codes (c * 2^14 = hi + lo fp16 parts, fp32-class)
#    over the fp16-rounded codes (<= 2.4e-4 relative per NF4 code).  Linear4bit passes
#    exact_codes=True when its compute_dtype is fp32 (the reference default: the layer's
#    products are then the reference's), otherwise None = this default: "auto"/"0" =
#    fp16-rounded codes, "1" = exact codes.  FP4 codes are exact in either table.
GEMV_EXACT_CODES = os.environ.get("QZ_GEMV_EXACT_CODES", "auto")   # "auto" | "1" | "0"


def _gemv_quant_type(quant_type: str, exact_codes: Optional[bool], dtype: torch.dtype) -> int:
    if exact_codes is None:
        exact_codes = dtype == torch.float32 if GEMV_EXACT_CODES == "auto" else GEMV_EXACT_CODES == "1"
    return _lib.QUANT_TYPES[quant_type] | (_lib.EXACT_CODES if exact_codes else 0)


def exact_codes_for(compute_dtype):
    """Decode code table for a layer's compute_dtype.  The reference casts x to
    compute_dtype (modules.py:141-142); with fp32 -- its config default -- the GEMV
    multiplies x by the fp32 codebook values (kernels.cu:1115-1120,1169-1170).  An
    fp16 x is exact in fp32, so skipping the cast and dotting the fp16 x against the
    exact (hi + lo) codes gives the reference's products; other compute dtypes keep
    the default table (GEMV_EXACT_CODES)."""
    return True if compute_dtype == torch.float32 else None


def gemv_4bit(A: Tensor, B: Tensor, out: Optional[Tensor] = None, transposed_A=False, transposed_B=False,
              state=None, bias: Optional[Tensor] = None, block_base: int = 0,
              exact_codes: Optional[bool] = None, residual: Optional[Tensor] = None) -> Tensor:
    """Batch-1 4-bit GEMV (reference core.py:426-504) as ONE fused kernel:
    y = x . W^T (+ bias), W from `state`; out dtype = A.dtype.  fp32 activations are
    multiplied by the fp32 codebook values and bf16 ones by bf16 hi + lo codes; for fp16
    activations `exact_codes` (default GEMV_EXACT_CODES) picks the exact hi + lo fp16 codes
    over the fp16-rounded ones.  `residual` (a contiguous A.dtype tensor of M elements;
    not in the reference): returns residual + y with the add in the kernel's epilogue
    (qz_gemv_4bit_residual, bit-identical to the torch add)."""
    if state is None:
        raise ValueError("state cannot None. gem_4bit( ) requires the state from quantize_4bit( )")
    if A.numel() != A.shape[-1]:
        raise ValueError('Dimensions of A are invalid. Must be a vector with the leading dimensions of "1", '
                         'e.g. [1, 1, 2048]')
    M, K = state.shape[0], state.shape[1]
    if A.shape[-1] != K:
        raise ValueError(f"A has {A.shape[-1]} features, the 4-bit weight expects {K}")
    if out is None:
        shape = (A.shape[0], A.shape[1], M) if A.dim() == 3 else (A.shape[0], M) if A.dim() == 2 else (M,)
        out = torch.empty(shape, dtype=A.dtype, device=A.device)
    A = A.contiguous()
    if bias is not None and bias.dtype != A.dtype:
        bias = bias.to(A.dtype)
    if residual is not None:
        if residual.dtype != A.dtype or residual.numel() != M or not residual.is_contiguous() \
                or residual.device != A.device:
            raise ValueError(f"gemv_4bit: residual must be a contiguous {A.dtype} tensor of {M} elements")
        check(lib.qz_gemv_4bit_residual(M, K, ptr(A), dtype_code(A.dtype), ptr(B),
                                        _gemv_quant_type(state.quant_type, exact_codes, A.dtype), state.blocksize,
                                        *state.scale_args(), block_base, 0, ptr(bias), ptr(residual), ptr(out),
                                        _lib.stream_of(A)), "gemv_4bit(residual)")
        return out
    check(lib.qz_gemv_4bit(M, K, ptr(A), dtype_code(A.dtype), ptr(B), _gemv_quant_type(state.quant_type, exact_codes, A.dtype),
                           state.blocksize, *state.scale_args(), block_base, 0, ptr(bias), ptr(out),
                           _lib.stream_of(A)), "gemv_4bit")
    return out


# how the last gemv_4bit_pair_silu / gemv_4bit_grouped call ran (launch forms, for bench.py's
# chain_roofline line): "pair" / "pair (norm fused)" / "norm launch + pair", "grouped" / ...
LAST_FORM = {}


def gemv_4bit_pair_silu(A: Tensor, items, exact_codes: Optional[bool] = None, norm=None) -> Optional[Tensor]:
    """F.silu(gate) * up for items = [(B, state, bias[, block_base])] of gate_proj and up_proj
    (equal shapes; block_base for row shards, parallel.sharded_silu_pair) and a single-token A,
    in ONE launch (qz_gemv_4bit_pair_silu): bit-identical to gemv_4bit_grouped +
    layer_ops.silu_mul.  norm=(weight, eps) as in gemv_4bit_grouped.  Returns None for what
    the kernel does not take (the caller runs the two launches)."""
    items = [tuple(it) + (0,) * (4 - len(it)) for it in items]
    if len(items) != 2 or A.numel() != A.shape[-1] or A.dtype not in (torch.float16, torch.bfloat16):
        return None
    s0, s1 = items[0][1], items[1][1]
    K = s0.shape[1]
    if (A.shape[-1] != K or s1.shape != s0.shape or s1.quant_type != s0.quant_type or s1.blocksize != s0.blocksize
            or s1.nested != s0.nested or (s0.nested and s1.state2.blocksize != s0.state2.blocksize)):
        return None
    A = A.contiguous()
    M = s0.shape[0]
    segs = (_lib.GemvSegment * 2)()
    for i, (B, st, bias, block_base) in enumerate(items):
        if bias is not None and bias.dtype != A.dtype:
            bias = bias.to(A.dtype)
        am, qam, am2, code2, off, _ = st.scale_args()
        segs[i] = _lib.GemvSegment(M, ptr(B), am, qam, am2, code2, off, int(block_base), ptr(bias), None)
    shape = (A.shape[0], A.shape[1], M) if A.dim() == 3 else (A.shape[0], M) if A.dim() == 2 else (M,)
    h = torch.empty(shape, dtype=A.dtype, device=A.device)
    nw, eps = (None, 0.0) if norm is None else norm
    if nw is not None and not (nw.dtype == A.dtype and nw.is_cuda and nw.is_contiguous() and nw.numel() == K):
        return None
    bs2 = int(s0.state2.blocksize) if s0.nested else 0
    qt = _gemv_quant_type(s0.quant_type, exact_codes, A.dtype)
    rc = lib.qz_gemv_4bit_pair_silu(ctypes.cast(segs, ctypes.c_void_p), K, ptr(A), dtype_code(A.dtype), qt,
                                    s0.blocksize, bs2, 0, ptr(nw), float(eps), ptr(h), _lib.stream_of(A))
    form = "pair" if nw is None else "pair (norm fused)"
    if rc == _lib.QZ_ERR_SHAPE and nw is not None:
        # the fused norm is not taken here (the split pair at K = 8192, or too many workgroups to
        # repeat the norm prologue in): the norm launch, then the pair on its output -- the same
        # bits as norm -> grouped -> silu_mul.  (Where the pair declines both, that norm launch is
        # wasted and the caller runs its own.)
        from .layer_ops import rms_norm
        A = rms_norm(A, nw, eps).contiguous()
        rc = lib.qz_gemv_4bit_pair_silu(ctypes.cast(segs, ctypes.c_void_p), K, ptr(A), dtype_code(A.dtype), qt,
                                        s0.blocksize, bs2, 0, None, 0.0, ptr(h), _lib.stream_of(A))
        form = "norm launch + pair"
    if rc == _lib.QZ_ERR_SHAPE:
        return None
    check(rc, "gemv_4bit_pair_silu")
    LAST_FORM["pair"] = form
    return h


def gemv_4bit_grouped(A: Tensor, items, exact_codes: Optional[bool] = None, norm=None) -> list:
    """Several batch-1 4-bit GEMVs that share the input vector A, in ONE launch
    (qz_gemv_4bit_grouped).  items: sequence of
    (B, state, bias[, block_base[, out]]) with equal K, quant_type, blocksize
    and scale format; returns [y_i] as gemv_4bit(A, B_i, state=state_i,
    bias=bias_i, block_base=...) would (`out`, if given, is written in place:
    a contiguous tensor of M_i elements).

    norm=(weight, eps): A is the INPUT of a Llama RMSNorm and every GEMV takes
    layer_ops.rms_norm(A, weight, eps) -- computed inside the same launch
    (qz_gemv_4bit_grouped_rmsnorm, bit-identical to the separate norm) where the
    kernel takes the shape, else as two launches."""
    items = list(items)
    if not 1 <= len(items) <= _lib.GEMV_MAX_SEGMENTS:
        raise ValueError(f"gemv_4bit_grouped takes 1..{_lib.GEMV_MAX_SEGMENTS} weights, got {len(items)}")
    if A.numel() != A.shape[-1]:
        raise ValueError("gemv_4bit_grouped needs a single input vector")
    s0 = items[0][1]
    K = s0.shape[1]
    if A.shape[-1] != K:
        raise ValueError(f"A has {A.shape[-1]} features, the 4-bit weights expect {K}")
    A = A.contiguous()
    segs = (_lib.GemvSegment * len(items))()
    outs = []
    for i, item in enumerate(items):
        B, st, bias = item[0], item[1], item[2]
        block_base = int(item[3]) if len(item) > 3 else 0
        y = item[4] if len(item) > 4 else None
        if (st.shape[1] != K or st.quant_type != s0.quant_type or st.blocksize != s0.blocksize
                or st.nested != s0.nested or (st.nested and st.state2.blocksize != s0.state2.blocksize)):
            raise ValueError("gemv_4bit_grouped: weights must share K, quant_type, blocksize and scale format")
        M = st.shape[0]
        if y is None:
            shape = (A.shape[0], A.shape[1], M) if A.dim() == 3 else (A.shape[0], M) if A.dim() == 2 else (M,)
            y = torch.empty(shape, dtype=A.dtype, device=A.device)
        elif y.numel() != M or not y.is_contiguous() or y.dtype != A.dtype:
            raise ValueError(f"gemv_4bit_grouped: out {i} must be a contiguous {A.dtype} tensor of {M} elements")
        if bias is not None and bias.dtype != A.dtype:
            bias = bias.to(A.dtype)
        am, qam, am2, code2, off, _ = st.scale_args()
        segs[i] = _lib.GemvSegment(M, ptr(B), am, qam, am2, code2, off, block_base, ptr(bias), ptr(y))
        outs.append(y)
    bs2 = int(s0.state2.blocksize) if s0.nested else 0
    qt = _gemv_quant_type(s0.quant_type, exact_codes, A.dtype)
    segp = ctypes.cast(segs, ctypes.c_void_p)
    if norm is not None:
        nw, eps = norm
        if nw.dtype == A.dtype and nw.is_cuda and nw.is_contiguous() and nw.numel() == K:
            rc = lib.qz_gemv_4bit_grouped_rmsnorm(len(items), segp, K, ptr(A), dtype_code(A.dtype), qt, s0.blocksize,
                                                  bs2, 0, ptr(nw), float(eps), _lib.stream_of(A))
            if rc != _lib.QZ_ERR_SHAPE:
                check(rc, "gemv_4bit_grouped(norm)")
                LAST_FORM["grouped"] = "grouped (norm fused)"
                return outs
        from .layer_ops import rms_norm
        A = rms_norm(A, nw, eps).contiguous()   # shapes the fused launch does not take: two launches
    LAST_FORM["grouped"] = "grouped" if norm is None else "norm launch + grouped"
    check(lib.qz_gemv_4bit_grouped(len(items), segp, K, ptr(A), dtype_code(A.dtype), qt, s0.blocksize, bs2, 0,
                                   _lib.stream_of(A)),
          "gemv_4bit_grouped")
    return outs


# Prefill route (matmul_4bit with more than one token).  "fused": the MFMA
# kernel qz_gemm_4bit (dequant in LDS, never in HBM); "dequant": the
# reference's own route (modules.py:62-64) -- full-weight dequantize_4bit (our
# bit-exact HIP kernel) then the library GEMM (hipBLASLt), or, with
# PREFILL_GEMM16 (env QZ_PREFILL_GEMM16=1) and >= GEMM16_MIN_TILES 256 x 256
# output tiles, our 4-wave LDS-DMA MFMA GEMM (qz_gemm_16bit); "gemm16"
# forces the latter where it applies.  "auto" takes the fused kernel up to
# fused_max_tokens(M) tokens and the dequant route above it (DESIGN.md
# section 4.2 has the measured crossovers: hipBLASLt is 4-7 % faster than
# qz_gemm_16bit at T = 16384 today, so it stays the default).
_FUSED_MAX_T_ENV = os.environ.get("QZ_PREFILL_FUSED_MAX_T")
PREFILL_FUSED_MAX_TOKENS = int(_FUSED_MAX_T_ENV) if _FUSED_MAX_T_ENV else None   # None = the measured table
PREFILL_GEMM16 = os.environ.get("QZ_PREFILL_GEMM16", "0") == "1"
GEMM16_MIN_TILES = int(os.environ.get("QZ_GEMM16_MIN_TILES", "256"))


def fused_max_tokens(M: int, K: int = 4096) -> int:
    """Largest token count the auto route sends to the fused kernels for an M x K
    weight.  An explicit QZ_PREFILL_FUSED_MAX_T (PREFILL_FUSED_MAX_TOKENS) replaces the
    table.  The table is the measured crossover against dequantize_4bit + hipBLASLt,
    whole routes (scripts/prefill_lowT_sweep.py [8b|70b]): the Llama-3-8B shapes
    (profiles/r2_prefill_lowT_sweep.txt) give 256 tokens for 2048..8192 rows, 128
    otherwise; the Llama-3-70B shapes (profiles/r6_prefill_lowT_sweep_70b.txt) keep that
    rule (8192 x 8192 and 8192 x 28672: fused ahead through 256, behind at 384; 28672 x 8192:
    through 128, behind at 192) except the narrow k/v projections at K = 8192, where the
    fused kernel stays ahead at every measured T up to 512 (1024 x 8192: 33.7 vs 35.9 us)."""
    if PREFILL_FUSED_MAX_TOKENS is not None:
        return PREFILL_FUSED_MAX_TOKENS
    if M <= 1024 and K >= 8192:
        return 512
    return 256 if 2048 <= M <= 8192 else 128


def gemm_16bit(A: Tensor, W: Tensor, bias: Optional[Tensor] = None) -> Optional[Tensor]:
    """Y = A . W^T (+ bias) on qz_gemm_16bit for fp16/bf16 A [..., K] and a contiguous
    W [M, K] of the same dtype; None if the kernel does not take the shapes (the
    caller then uses the library GEMM)."""
    M, K = W.shape
    lead = A.shape[:-1]
    A2 = A.reshape(-1, K)
    if A2.stride(-1) != 1 or A2.data_ptr() % 16 != 0:
        A2 = A2.contiguous()
    T = A2.shape[0]
    if (A.dtype not in (torch.float16, torch.bfloat16) or W.dtype != A.dtype or not W.is_contiguous()
            or (bias is not None and (bias.numel() != M or not bias.is_contiguous()))):
        return None
    out = torch.empty((T, M), dtype=A.dtype, device=A.device)
    if not lib.qz_gemm_16bit_ok(T, M, K, ptr(A2), A2.stride(0), ptr(W), ptr(out), M):
        return None
    if bias is not None and bias.dtype != A.dtype:
        bias = bias.to(A.dtype)
    check(lib.qz_gemm_16bit(T, M, K, ptr(A2), A2.stride(0), dtype_code(A.dtype), ptr(W), ptr(bias), ptr(out), M,
                            _lib.stream_of(A)), "gemm_16bit")
    return out.reshape(*lead, M)


def _gemm_fused_ok(A2: Tensor, state: QuantState, M: int, K: int) -> bool:
    return (A2.dtype in (torch.float16, torch.bfloat16) and K % 64 == 0 and M % 4 == 0
            and state.blocksize >= 64 and A2.stride(0) % 8 == 0 and A2.data_ptr() % 16 == 0)


def gemm_4bit(A: Tensor, B: Tensor, state: QuantState, bias: Optional[Tensor] = None, route: str = "auto") -> Tensor:
    """Batched (prefill) 4-bit GEMM: A[..., K] . W^T (+ bias) -> [..., M].

    The fused MFMA kernel decodes W to exactly the values dequantize_4bit(B,
    state, out_dtype=A.dtype) stores, so every route multiplies the same operand
    and differs only in fp32 summation order (fp16/bf16 activations; other
    dtypes take the dequant route).  route: "auto", "fused", "dequant" (dequant +
    the library GEMM, or qz_gemm_16bit with PREFILL_GEMM16), "blas" (dequant +
    the library GEMM, the reference's F.linear) or "gemm16" (dequant +
    qz_gemm_16bit where it applies)."""
    if route not in ("auto", "fused", "dequant", "blas", "gemm16"):
        raise ValueError(f"route must be 'auto', 'fused', 'dequant', 'blas' or 'gemm16', got {route!r}")
    M, K = state.shape[0], state.shape[1]
    lead = A.shape[:-1]
    A2 = A.reshape(-1, K)
    if A2.stride(-1) != 1 or A2.data_ptr() % 16 != 0:
        A2 = A2.contiguous()
    T = A2.shape[0]
    if T == 0 or M == 0:  # an empty batch (F.linear's result; the C-ABI rejects null buffers)
        return torch.empty((*lead, M), dtype=A.dtype, device=A.device)
    fused_ok = _gemm_fused_ok(A2, state, M, K)
    if route == "fused" and not fused_ok:
        raise ValueError("gemm_4bit: the fused kernel needs fp16/bf16 activations, K % 64 == 0, M % 4 == 0 "
                         "and blocksize >= 64")
    if fused_ok and (route == "fused" or (route == "auto" and T <= fused_max_tokens(M, K))):
        out = torch.empty((T, M), dtype=A.dtype, device=A.device)
        if bias is not None and bias.dtype != A.dtype:
            bias = bias.to(A.dtype)
        ws_bytes = int(lib.qz_gemm_4bit_workspace_size(T, M, K))
        ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=A.device) if ws_bytes > 0 else None
        check(lib.qz_gemm_4bit(T, M, K, ptr(A2), A2.stride(0), dtype_code(A.dtype), ptr(B),
                               _lib.QUANT_TYPES[state.quant_type], state.blocksize, *state.scale_args(), ptr(bias),
                               ptr(out), M, ptr(ws), ws_bytes, _lib.stream_of(A)), "gemm_4bit")
        return out.reshape(*lead, M)
    cd = A.dtype if A.dtype in (torch.float16, torch.bfloat16) else None
    W = dequantize_4bit(B, state, out_dtype=cd).t()          # [M, K], contiguous
    tiles = ((T + 255) // 256) * ((M + 255) // 256)
    if cd is not None and (route == "gemm16" or (route != "blas" and PREFILL_GEMM16 and tiles >= GEMM16_MIN_TILES)):
        Y = gemm_16bit(A, W, bias)
        if Y is not None:
            return Y
    if route == "gemm16":  # asked for our GEMM explicitly: never a silent library fallback
        raise ValueError("gemm_4bit: route 'gemm16' needs fp16/bf16 activations, K % 64 == 0, M % 8 == 0 and "
                         "16-byte aligned operands")
    return torch.nn.functional.linear(A, W.to(A.dtype), None if bias is None else bias.to(A.dtype))


# Token counts the multi-token kernel (and so the grouped batched-decode launch) takes
MT_MIN_TOKENS, MT_MAX_TOKENS, MT_K_MULTIPLE = 2, 16, 256


def grouped_tokens_ok(A: Tensor, items) -> bool:
    """Whether gemm_4bit_grouped can run `items` on A in one launch."""
    K = A.shape[-1]
    T = A.numel() // K if K else 0
    if not (MT_MIN_TOKENS <= T <= MT_MAX_TOKENS and K % MT_K_MULTIPLE == 0
            and 1 <= len(items) <= _lib.GEMV_MAX_SEGMENTS and A.dtype in (torch.float16, torch.bfloat16)):
        return False
    s0 = items[0][1]
    return all(it[1].shape[1] == K and it[1].quant_type == s0.quant_type and it[1].blocksize == s0.blocksize
               and it[1].blocksize >= 64 and it[1].nested == s0.nested and it[1].shape[0] % 4 == 0
               and (not it[1].nested or it[1].state2.blocksize == s0.state2.blocksize) for it in items)


def gemm_4bit_grouped(A: Tensor, items) -> list:
    """Batched decode over a few tokens (2..16) for several 4-bit weights that
    share A (q/k/v, gate/up of one layer), in ONE launch (qz_gemm_4bit_grouped).
    items: (B, state, bias[, block_base]) as for gemv_4bit_grouped; returns
    [y_i] of shape [..., M_i], each bit-identical to gemm_4bit(A, B_i, state_i,
    bias_i) on the multi-token kernel.  grouped_tokens_ok() says when it applies."""
    items = list(items)
    if not grouped_tokens_ok(A, items):
        raise ValueError("gemm_4bit_grouped needs 2..16 fp16/bf16 tokens, K % 256 == 0, 1..4 weights that share "
                         "K, quant_type, blocksize (>= 64) and scale format, and out_features % 4 == 0")
    K = A.shape[-1]
    lead = A.shape[:-1]
    A2 = A.reshape(-1, K)
    if A2.stride(-1) != 1 or A2.stride(0) % 8 != 0 or A2.data_ptr() % 16 != 0:
        A2 = A2.contiguous()
    T = A2.shape[0]
    segs = (_lib.GemvSegment * len(items))()
    outs = []
    for i, item in enumerate(items):
        B, st, bias = item[0], item[1], item[2]
        block_base = int(item[3]) if len(item) > 3 else 0
        M = st.shape[0]
        y = torch.empty((T, M), dtype=A.dtype, device=A.device)
        if bias is not None and bias.dtype != A.dtype:
            bias = bias.to(A.dtype)
        am, qam, am2, code2, off, _ = st.scale_args()
        segs[i] = _lib.GemvSegment(M, ptr(B), am, qam, am2, code2, off, block_base, ptr(bias), ptr(y))
        outs.append(y)
    s0 = items[0][1]
    bs2 = int(s0.state2.blocksize) if s0.nested else 0
    check(lib.qz_gemm_4bit_grouped(len(items), ctypes.cast(segs, ctypes.c_void_p), T, K, ptr(A2), A2.stride(0),
                                   dtype_code(A.dtype), _lib.QUANT_TYPES[s0.quant_type], s0.blocksize, bs2,
                                   _lib.stream_of(A)), "gemm_4bit_grouped")
    return [y.reshape(*lead, y.shape[-1]) for y in outs]

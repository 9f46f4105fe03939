"""One-launch HIP forms of the small ops around a Llama layer's 4-bit
projections (csrc/layer_ops.hip, C-ABI include/quantizations.h):

* ``rms_norm``  -- LlamaRMSNorm.forward (transformers modeling_llama.py:62-67),
  which produces the input of q/k/v and gate/up;
* ``rope_qk``   -- apply_rotary_pos_emb (modeling_llama.py:138-160), applied to
  the outputs of q_proj/k_proj;
* ``silu_mul``  -- LlamaMLP's act_fn(gate_proj(x)) * up_proj(x)
  (modeling_llama.py:175), the input of down_proj;
* ``add_rms_norm`` -- LlamaDecoderLayer's ``residual + h`` followed by the
  post-attention RMSNorm (modeling_llama.py:317-321).

None of them is in the reference (it leaves them to transformers).  They exist
because at batch-1 decode the eager torch forms cost ~8, ~10 and 2 dependent
launches per call, which dominate the step once the Linear4bit GEMVs are
fused.  ``integration.fuse_layer_ops`` installs them.
No CPU or torch fallback lives here: the callers decide what is supported.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_SUPPORTED = (torch.float16, torch.bfloat16, torch.float32)


def rms_norm_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype in _SUPPORTED and weight.dtype == x.dtype and weight.device == x.device
            and weight.dim() == 1 and x.dim() >= 1 and x.shape[-1] == weight.shape[0] and weight.is_contiguous()
            and x.stride(-1) == 1)


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """weight * (x.float() * rsqrt(mean(x.float()**2, -1) + eps)).to(x.dtype), one launch."""
    if not rms_norm_supported(x, weight):
        raise ValueError(f"rms_norm: unsupported input ({x.dtype} on {x.device}, weight {weight.dtype})")
    K = x.shape[-1]
    x2 = x.reshape(-1, K)  # a view for every layout HF produces (row stride may exceed K)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    y = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib.qz_rmsnorm(x2.data_ptr(), _lib.dtype_code(x.dtype), x2.shape[0], K, x2.stride(0),
                                   weight.data_ptr(), float(eps), y.data_ptr(), K, _lib.stream_of(x)),
               "qz_rmsnorm")
    return y


def add_rms_norm_supported(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor) -> bool:
    return (rms_norm_supported(x, weight) and residual.dtype == x.dtype and residual.device == x.device
            and residual.shape == x.shape and x.is_contiguous() and residual.is_contiguous())


def add_rms_norm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor, eps: float):
    """(s, rms_norm(s)) with s = residual + x (rounded to x.dtype, bit-exact to the
    torch add), one launch."""
    if not add_rms_norm_supported(x, residual, weight):
        raise ValueError("add_rms_norm: unsupported input")
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    s = torch.empty_like(x)
    y = torch.empty_like(x)
    _lib.check(_lib.lib.qz_add_rmsnorm(x.data_ptr(), residual.data_ptr(), _lib.dtype_code(x.dtype), rows, K, K,
                                       weight.data_ptr(), float(eps), s.data_ptr(), y.data_ptr(), K,
                                       _lib.stream_of(x)), "qz_add_rmsnorm")
    return s, y


def _strides3(t: torch.Tensor):
    return (ctypes.c_longlong * 3)(t.stride(0), t.stride(1), t.stride(2))


def rope_supported(q: torch.Tensor, k: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                   unsqueeze_dim: int = 1) -> bool:
    if unsqueeze_dim != 1 or q.dim() != 4 or k.dim() != 4 or cos.dim() != 3 or sin.shape != cos.shape:
        return False
    if not (q.is_cuda and q.dtype in _SUPPORTED and k.dtype == q.dtype and cos.dtype == q.dtype
            and sin.dtype == q.dtype and k.device == q.device and cos.device == q.device and sin.device == q.device):
        return False
    B, _, S, D = q.shape
    if k.shape[0] != B or k.shape[2] != S or k.shape[3] != D or D % 2 or cos.shape[1] != S or cos.shape[2] != D:
        return False
    if cos.shape[0] not in (1, B) or cos.stride() != sin.stride():
        return False
    return q.stride(-1) == 1 and k.stride(-1) == 1 and cos.stride(-1) == 1


def rope_qk(q: torch.Tensor, k: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor):
    """(q*cos + rotate_half(q)*sin, k*cos + rotate_half(k)*sin) for q/k [B, H, S, D]
    and cos/sin [B or 1, S, D]; one launch, bit-identical to the torch expression."""
    if not rope_supported(q, k, cos, sin):
        raise ValueError("rope_qk: unsupported shapes/dtypes/layout")
    B, Hq, S, D = q.shape
    Hk = k.shape[1]
    qo = torch.empty_like(q)  # keeps q's (transposed) layout, as torch's elementwise ops do
    ko = torch.empty_like(k)
    if qo.stride(-1) != 1 or ko.stride(-1) != 1:
        qo = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        ko = torch.empty(k.shape, dtype=k.dtype, device=k.device)
    q3, qo3, k3, ko3 = (t[:, :, :, 0] for t in (q, qo, k, ko))
    cs = (ctypes.c_longlong * 2)(cos.stride(0) if cos.shape[0] == B else 0, cos.stride(1))
    _lib.check(_lib.lib.qz_rope_qk(_lib.dtype_code(q.dtype), B, S, D,
                                   q.data_ptr(), Hq, _strides3(q3), qo.data_ptr(), _strides3(qo3),
                                   k.data_ptr(), Hk, _strides3(k3), ko.data_ptr(), _strides3(ko3),
                                   cos.data_ptr(), sin.data_ptr(), cs, _lib.stream_of(q)),
               "qz_rope_qk")
    return qo, ko


def silu_mul_supported(g: torch.Tensor, u: torch.Tensor) -> bool:
    return (g.is_cuda and g.dtype in _SUPPORTED and u.dtype == g.dtype and u.device == g.device
            and g.shape == u.shape and g.is_contiguous() and u.is_contiguous())


def silu_mul(g: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """F.silu(g) * u with torch's per-op rounding, one launch."""
    if not silu_mul_supported(g, u):
        raise ValueError("silu_mul: unsupported shapes/dtypes/layout")
    y = torch.empty_like(g)
    _lib.check(_lib.lib.qz_silu_mul(g.data_ptr(), u.data_ptr(), _lib.dtype_code(g.dtype), g.numel(), y.data_ptr(),
                                    _lib.stream_of(g)), "qz_silu_mul")
    return y

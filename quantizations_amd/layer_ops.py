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


ATTN_CHUNK = 128  # key positions per workgroup of qz_decode_attention (csrc/layer_ops.hip)


def decode_attention_supported(q: torch.Tensor, cos: torch.Tensor, key_cache: torch.Tensor,
                               value_cache: torch.Tensor, mask, pos, num_heads: int) -> bool:
    """What qz_decode_attention takes: one new token per sequence (q, or the layer input:
    [B, 1, *]), 16-bit activations, a contiguous static cache [B, Hkv, L, D] with D in {64, 128}
    and Hq/Hkv <= 8, a bool mask [B or 1, 1, 1, L], cos/sin [B or 1, 1, D] and an int64 position
    on the GPU.  Metadata only: nothing is launched or allocated."""
    if not (q.is_cuda and q.dtype in (torch.float16, torch.bfloat16) and q.dim() == 3 and q.shape[1] == 1):
        return False
    if key_cache.dim() != 4 or value_cache.shape != key_cache.shape:
        return False
    B, Hkv, L, D = key_cache.shape
    if D not in (64, 128) or num_heads % Hkv or num_heads // Hkv > 8 or q.shape[0] != B or L == 0:
        return False
    for t in (key_cache, value_cache):
        if t.dtype != q.dtype or t.device != q.device or not t.is_contiguous() or t.data_ptr() % 16:
            return False
    if not (isinstance(mask, torch.Tensor) and mask.dtype == torch.bool and mask.device == q.device
            and mask.dim() == 4 and mask.shape[0] in (1, B) and mask.shape[1] == 1 and mask.shape[2] == 1
            and mask.shape[3] == L):
        return False
    if not (cos.dim() == 3 and cos.shape[0] in (1, B) and cos.shape[1] == 1 and cos.shape[2] == D
            and cos.dtype == q.dtype and cos.device == q.device and cos.stride(-1) == 1):
        return False
    return (isinstance(pos, torch.Tensor) and pos.dtype == torch.int64 and pos.numel() == 1 and pos.device == q.device)


def decode_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                     key_cache: torch.Tensor, value_cache: torch.Tensor, mask: torch.Tensor, pos: torch.Tensor,
                     arrive: torch.Tensor, num_heads: int, scale: float) -> torch.Tensor:
    """LlamaAttention.forward for one new token per sequence against a static cache, up to the
    o_proj input: rotary of q/k, key_cache/value_cache[:, :, pos] = k, v, pos += 1 (all on the
    GPU, graph-capturable), masked GQA softmax(q k^T * scale) v.  q [B, 1, Hq*D], k/v
    [B, 1, Hkv*D] (the projection outputs), cos/sin [B or 1, 1, D], caches [B, Hkv, L, D],
    mask bool [B or 1, 1, 1, L], pos int64 (StaticLayer.cumulative_length), arrive a zeroed
    int32 scratch word.  Returns [B, 1, Hq*D]."""
    if not decode_attention_supported(q, cos, key_cache, value_cache, mask, pos, num_heads):
        raise ValueError("decode_attention: unsupported shapes/dtypes/layout")
    B, Hkv, L, D = key_cache.shape
    G = num_heads // Hkv
    if q.shape[2] != num_heads * D:
        raise ValueError("decode_attention: q width differs from num_heads * head_dim")
    if sin.shape != cos.shape or sin.stride() != cos.stride() or sin.dtype != cos.dtype:
        raise ValueError("decode_attention: sin must match cos")
    q2, k2, v2 = (t.reshape(B, -1) for t in (q, k, v))
    k2 = k2 if k2.stride(-1) == 1 else k2.contiguous()
    q2 = q2 if q2.stride(-1) == 1 else q2.contiguous()
    if v2.stride(-1) != 1 or v2.stride(0) % 2 or v2.data_ptr() % 4:
        v2 = v2.contiguous()
    if k2.shape[1] != Hkv * D or v2.shape[1] != Hkv * D:
        raise ValueError("decode_attention: k/v width differs from the cache's heads")
    out = torch.empty((B, 1, num_heads * D), dtype=q.dtype, device=q.device)
    nsplit = -(-L // ATTN_CHUNK)
    work = torch.empty(B * Hkv * nsplit * G * (D + 2), dtype=torch.float32, device=q.device) if nsplit > 1 else None
    cs_row = cos.stride(0) if cos.shape[0] == B and B > 1 else 0
    mb = mask.stride(0) if mask.shape[0] == B and B > 1 else 0
    _lib.check(_lib.lib.qz_decode_attention(
        _lib.dtype_code(q.dtype), B, num_heads, Hkv, D, L, q2.data_ptr(), q2.stride(0), k2.data_ptr(), k2.stride(0),
        v2.data_ptr(), v2.stride(0), cos.data_ptr(), sin.data_ptr(), cs_row, key_cache.data_ptr(),
        value_cache.data_ptr(), mask.data_ptr(), mb, mask.stride(3), pos.data_ptr(), arrive.data_ptr(),
        out.data_ptr(), num_heads * D, work.data_ptr() if work is not None else None, float(scale),
        _lib.stream_of(q)), "qz_decode_attention")
    return out


def decode_mask(q_offset: torch.Tensor, batch: int, kv_length: int) -> torch.Tensor:
    """masking_utils.create_causal_mask's sdpa mask for one new token per sequence against a static
    cache (no padding mask, kv_offset 0): bool [batch, 1, 1, kv_length], True where kv position
    j <= q_offset (StaticLayer.cumulative_length, a device int64 read in-kernel)."""
    if not (q_offset.is_cuda and q_offset.dtype == torch.int64 and q_offset.numel() == 1):
        raise ValueError("decode_mask: q_offset must be one int64 on the GPU")
    mask = torch.empty((batch, 1, 1, kv_length), dtype=torch.bool, device=q_offset.device)
    _lib.check(_lib.lib.qz_decode_mask(q_offset.data_ptr(), batch, kv_length, mask.data_ptr(),
                                       _lib.stream_of(q_offset)), "qz_decode_mask")
    return mask


def rope_table(position_ids: torch.Tensor, cos_t: torch.Tensor, sin_t: torch.Tensor, inv_freq: torch.Tensor,
               scale: float):
    """LlamaRotaryEmbedding.forward from tables: cos/sin [B, S, D] of position_ids [B, S] (int64)
    copied from cos_t/sin_t [T, D] (what the module computed for positions 0..T-1); positions
    outside the table computed in-kernel from inv_freq (fp32) and scale."""
    if not (position_ids.is_cuda and position_ids.dtype == torch.int64 and position_ids.dim() == 2):
        raise ValueError("rope_table: position_ids must be int64 [B, S] on the GPU")
    T, D = cos_t.shape
    if sin_t.shape != cos_t.shape or sin_t.dtype != cos_t.dtype or not (cos_t.is_contiguous() and sin_t.is_contiguous()):
        raise ValueError("rope_table: cos/sin tables must be contiguous [T, D] of one dtype")
    if inv_freq.dtype != torch.float32 or inv_freq.numel() * 2 != D or not inv_freq.is_contiguous():
        raise ValueError("rope_table: inv_freq must be contiguous fp32 [D / 2]")
    B, S = position_ids.shape
    cos = torch.empty((B, S, D), dtype=cos_t.dtype, device=position_ids.device)
    sin = torch.empty_like(cos)
    _lib.check(_lib.lib.qz_rope_table(_lib.dtype_code(cos_t.dtype), B, S, D, position_ids.data_ptr(),
                                      position_ids.stride(0), position_ids.stride(1), cos_t.data_ptr(),
                                      sin_t.data_ptr(), T, inv_freq.data_ptr(), float(scale), cos.data_ptr(),
                                      sin.data_ptr(), _lib.stream_of(position_ids)), "qz_rope_table")
    return cos, sin


def greedy_step(logits: torch.Tensor, hist: torch.Tensor, pos: torch.Tensor, tok: torch.Tensor) -> None:
    """A decode loop's greedy pick and feedback in two launches (qz_greedy_step): next = logits.argmax(-1) (torch's
    order: NaN first, then the largest, the first index among equals) for logits [B, V] (rows of
    any stride, unit element stride); hist[b, pos] = next[b]; tok[b] = next[b]; pos += 1.  hist
    [B, H] contiguous int64, pos one int64, tok B contiguous int64, all on the logits' GPU."""
    if logits.dim() != 2 or logits.stride(-1) != 1 or not logits.is_cuda:
        raise ValueError("greedy_step: logits must be [B, V] on the GPU with unit element stride")
    B, V = logits.shape
    for t in (hist, pos, tok):
        if t.dtype != torch.int64 or t.device != logits.device or not t.is_contiguous():
            raise ValueError("greedy_step: hist/pos/tok must be contiguous int64 on the logits' device")
    if hist.dim() != 2 or hist.shape[0] != B or pos.numel() != 1 or tok.numel() != B:
        raise ValueError("greedy_step: hist [B, H], pos [1], tok [B]")
    work = torch.empty(_lib.lib.qz_greedy_step_work_bytes(B, V), dtype=torch.uint8, device=logits.device)
    _lib.check(_lib.lib.qz_greedy_step(logits.data_ptr(), _lib.dtype_code(logits.dtype), B, V, logits.stride(0),
                                       hist.data_ptr(), hist.shape[1], hist.shape[1], pos.data_ptr(), tok.data_ptr(),
                                       work.data_ptr(), _lib.stream_of(logits)), "qz_greedy_step")


DENSE_K = (4096, 8192)   # the widths qz_gemv_dense takes (Llama-3 8B / 70B)


def gemv_dense_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """One token through an unquantised fp16/bf16 [M, K] weight (the lm_head) with qz_gemv_dense."""
    if not (x.is_cuda and weight.is_cuda and x.device == weight.device and x.dtype == weight.dtype
            and x.dtype in (torch.float16, torch.bfloat16) and weight.dim() == 2 and weight.is_contiguous()):
        return False
    K = weight.shape[1]
    return (K in DENSE_K and x.shape[-1] == K and x.numel() == K and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0 and weight.shape[0] < 2 ** 31)


def gemv_dense(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """F.linear(x, weight) for one token ([..., K] with one row) -- fp32 accumulation, rounded once
    (the library's numerics class; the summation order differs)."""
    if not gemv_dense_supported(x, weight):
        raise ValueError("gemv_dense: unsupported shapes/dtypes/layout")
    M, K = weight.shape
    y = torch.empty((*x.shape[:-1], M), dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib.qz_gemv_dense(M, K, x.data_ptr(), _lib.dtype_code(x.dtype), weight.data_ptr(), y.data_ptr(),
                                      _lib.stream_of(x)), "qz_gemv_dense")
    return y

"""transformers integration -- the equivalent of the reference README recipe that
patches ``transformers/integrations/bitsandbytes.py::_replace_with_bnb_linear``
(README.md:52-86) to build ``Linear4bit`` instead of ``bnb.nn.Linear4bit``.

Installed transformers (5.x) only routes ``load_in_4bit`` through bitsandbytes,
which does not exist on ROCm here, so the replacement is done explicitly on an
already-built model: every ``nn.Linear`` (except ``modules_to_not_convert``,
``lm_head`` by default as in transformers) becomes a ``Linear4bit`` and its
weight is quantised on the GPU.
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch
import torch.nn as nn

from .core import Params4bit, QuantState
from .modules import DecodeGroup, Linear4bit, _linear4bit_group_compute


def _cfg(quantization_config, name, default):
    return getattr(quantization_config, name, default) if quantization_config is not None else default


def replace_with_bnb_linear(model: nn.Module, modules_to_not_convert: Optional[Iterable[str]] = None,
                            quantization_config=None, quant_type: Optional[str] = None,
                            compress_statistics: Optional[bool] = None, compute_dtype=None,
                            device=None) -> nn.Module:
    """Replace nn.Linear modules with Linear4bit (same kwargs the README recipe passes:
    compute dtype, compress_statistics=bnb_4bit_use_double_quant, quant_type,
    quant_storage) and quantise their weights on `device` (default: the weight's
    device, which must be a GPU)."""
    skip = set(modules_to_not_convert or ["lm_head"])
    qt = quant_type or _cfg(quantization_config, "bnb_4bit_quant_type", "nf4")
    cs = compress_statistics if compress_statistics is not None else \
        _cfg(quantization_config, "bnb_4bit_use_double_quant", True)
    cd = compute_dtype if compute_dtype is not None else _cfg(quantization_config, "bnb_4bit_compute_dtype", None)
    qstorage = _cfg(quantization_config, "bnb_4bit_quant_storage", torch.uint8)

    def visit(parent: nn.Module, prefix: str):
        for name, child in list(parent.named_children()):
            full = f"{prefix}.{name}" if prefix else name
            if isinstance(child, nn.Linear) and not isinstance(child, Linear4bit) and \
                    name not in skip and full not in skip:
                dev = torch.device(device) if device is not None else child.weight.device
                new = Linear4bit(child.in_features, child.out_features, child.bias is not None, cd,
                                 compress_statistics=cs, quant_type=qt, quant_storage=qstorage, device="meta")
                new.weight = Params4bit(child.weight.data, requires_grad=False, quant_type=qt,
                                        quant_storage=qstorage, module=new, compress_statistics=cs).to(dev)
                if child.bias is not None:
                    new.bias = nn.Parameter(child.bias.data.to(dev), requires_grad=False)
                parent._modules[name] = new
                del child
            else:
                visit(child, full)

    visit(model, "")
    return model


# the name used by transformers (README.md:67)
_replace_with_bnb_linear = replace_with_bnb_linear


# projections of one block that read the same input (Llama/Mistral/Qwen naming,
# plus the Mixtral-style w1/w3 expert pair)
DEFAULT_PROJECTION_GROUPS = (("q_proj", "k_proj", "v_proj"), ("gate_proj", "up_proj"), ("w1", "w3"))


def _group_compatible(members) -> bool:
    from .parallel import RowShardedLinear4bit

    cls = type(members[0])
    if any(type(m) is not cls for m in members):
        return False
    if cls is Linear4bit:
        states = [m.weight.quant_state for m in members]
        if any(s is None for s in states):
            return False
        if len({m.compute_dtype for m in members}) != 1:
            return False
    elif cls is RowShardedLinear4bit:
        states = [m.state for m in members]
        if len({(m.world_size, id(m.group), m.gather) for m in members}) != 1 or \
                any(m._local_matmul is not members[0]._local_matmul for m in members):
            return False
    else:
        return False
    s0 = states[0]
    return all(s.shape[1] == s0.shape[1] and s.quant_type == s0.quant_type and s.blocksize == s0.blocksize
               and s.nested == s0.nested and (not s.nested or s.state2.blocksize == s0.state2.blocksize)
               for s in states)


def fuse_projection_groups(model: nn.Module, groups=DEFAULT_PROJECTION_GROUPS) -> int:
    """Attach a DecodeGroup to every set of sibling 4-bit projections named in
    `groups` (e.g. q/k/v and gate/up of each decoder layer) so that batch-1
    decode issues ONE grouped GEMV per set (and, for row-sharded layers, one
    all-gather per set).  Works on Linear4bit and on RowShardedLinear4bit (call
    it after ``parallel.shard_model_linear4bit``).  Prefill is unchanged.
    Returns the number of groups formed."""
    from .parallel import RowShardedLinear4bit, sharded_group_compute

    n = 0
    for parent in model.modules():
        for names in groups:
            members = [parent._modules.get(nm) for nm in names]
            if any(m is None for m in members) or not _group_compatible(members):
                continue
            compute = _linear4bit_group_compute if isinstance(members[0], Linear4bit) else sharded_group_compute
            assert isinstance(members[0], (Linear4bit, RowShardedLinear4bit))
            g = DecodeGroup(members, compute)
            for m in members:
                m.__dict__["_qz_group"] = g
            n += 1
    return n


def unfuse_projection_groups(model: nn.Module) -> None:
    """Remove every DecodeGroup attached by fuse_projection_groups (and with them any RMSNorm
    fuse_prenorm absorbed into one)."""
    unfuse_prenorm(model)
    for m in model.modules():
        m.__dict__.pop("_qz_group", None)


def _identity(x):
    return x


def fuse_prenorm(model: nn.Module) -> int:
    """Absorb each decoder layer's input_layernorm into its q/k/v decode group and its
    post_attention_layernorm into its gate/up group (DecodeGroup.prenorm).  The norm module
    then returns its input unchanged, and the group's single-token launch normalises x in its
    prologue (qz_gemv_4bit_grouped_rmsnorm, bit-identical to the separate qz_rmsnorm launch):
    one launch fewer per norm.  Other inputs (prefill, small batches) run the norm as the model
    did before, then the group.  In a LlamaDecoderLayer these norms feed nothing else
    (modeling_llama.py:306-321).  Call after fuse_projection_groups (and fuse_layer_ops);
    layers whose norm, groups or decoder forward do not match are left alone.  Returns the
    number of norms absorbed."""
    from .parallel import RowShardedLinear4bit, sharded_group_compute

    n = 0
    for layer in model.modules():
        if type(layer).__name__ not in DECODER_CLASSES or "_qz_fused_decoder" in layer.__dict__:
            continue
        attn, mlp = getattr(layer, "self_attn", None), getattr(layer, "mlp", None)
        pairs = (("input_layernorm", attn, ("q_proj", "k_proj", "v_proj")),
                 ("post_attention_layernorm", mlp, ("gate_proj", "up_proj")))
        for ln_name, parent, names in pairs:
            ln = getattr(layer, ln_name, None)
            if ln is None or parent is None or type(ln).__name__ not in RMSNORM_CLASSES or \
                    "_qz_absorbed_norm" in ln.__dict__ or not hasattr(ln, "variance_epsilon"):
                continue
            w = getattr(ln, "weight", None)
            members = [getattr(parent, nm, None) for nm in names]
            g = members[0].__dict__.get("_qz_group") if isinstance(members[0], (Linear4bit, RowShardedLinear4bit)) \
                else None
            # Linear4bit groups, and groups of row shards (x is replicated: every rank normalises
            # it in its own launch's prologue, the bits of the unsharded launch)
            if w is None or g is None or g.prenorm is not None or \
                    (g._compute is _linear4bit_group_compute and not w.is_cuda) or \
                    g._compute not in (_linear4bit_group_compute, sharded_group_compute) or \
                    [id(m) for m in g.members] != [id(m) for m in members]:
                continue
            g.prenorm = (w, float(ln.variance_epsilon), ln.forward)   # the norm as the model runs it now
            ln.__dict__["_qz_absorbed_norm"] = ln.__dict__.get("forward")
            ln.__dict__["forward"] = _identity
            n += 1
    return n


def unfuse_prenorm(model: nn.Module) -> None:
    """Undo fuse_prenorm: every absorbed norm computes again, no group applies one."""
    for m in model.modules():
        if "_qz_absorbed_norm" in m.__dict__:
            prev = m.__dict__.pop("_qz_absorbed_norm")
            if prev is None:
                m.__dict__.pop("forward", None)
            else:
                m.__dict__["forward"] = prev
        g = m.__dict__.get("_qz_group")
        if g is not None:
            g.prenorm = None


# ---------------------------------------------------------------------------
# the Linear4bit's neighbours in a decoder layer: RMSNorm and rotary embedding
# ---------------------------------------------------------------------------

# norms whose forward is exactly LlamaRMSNorm's (modeling_llama.py:62-67)
RMSNORM_CLASSES = ("LlamaRMSNorm", "MistralRMSNorm", "Qwen2RMSNorm")
# MLPs whose forward is down_proj(act_fn(gate_proj(x)) * up_proj(x)) (modeling_llama.py:174-176)
MLP_CLASSES = ("LlamaMLP", "MistralMLP", "Qwen2MLP")
# decoder layers whose forward is exactly LlamaDecoderLayer's (modeling_llama.py:295-324)
DECODER_CLASSES = ("LlamaDecoderLayer",)
# attention modules whose modeling module's apply_rotary_pos_emb is Llama's half-split
# rotation (modeling_llama.py:138-160); others (e.g. Cohere's interleaved
# rotate_half) keep their own code
ATTENTION_CLASSES = ("LlamaAttention", "MistralAttention", "Qwen2Attention")
_ROPE_PATCHED = {}  # module name -> original apply_rotary_pos_emb


def _fused_rmsnorm_forward(mod: nn.Module, orig):
    from .layer_ops import rms_norm, rms_norm_supported

    def forward(hidden_states: torch.Tensor) -> torch.Tensor:
        if rms_norm_supported(hidden_states, mod.weight):
            return rms_norm(hidden_states, mod.weight, mod.variance_epsilon)
        return orig(hidden_states)  # transformers' own eager code (e.g. CPU tensors, mixed dtypes)
    return forward


def _half_split_rotate(mod) -> bool:
    """True iff the modeling module's rotate_half is the half-split form
    cat(-x[..., D/2:], x[..., :D/2]) that k_rope_qk implements."""
    fn = getattr(mod, "rotate_half", None)
    if fn is None:
        return False
    try:
        r = fn(torch.arange(1.0, 5.0))
    except Exception:
        return False
    return isinstance(r, torch.Tensor) and r.tolist() == [-3.0, -4.0, 1.0, 2.0]


def _fused_rope(orig):
    from .layer_ops import rope_qk, rope_supported

    def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1, **kw):
        if not kw and rope_supported(q, k, cos, sin, unsqueeze_dim):
            return rope_qk(q, k, cos, sin)
        return orig(q, k, cos, sin, unsqueeze_dim, **kw)
    apply_rotary_pos_emb._qz_orig = orig
    return apply_rotary_pos_emb


def _fused_mlp_forward(mod: nn.Module, pair: bool = True):
    from .layer_ops import silu_mul, silu_mul_supported

    from . import parallel
    from .modules import linear4bit_silu_pair

    def forward(x: torch.Tensor, _qz_residual=None) -> torch.Tensor:
        h = None
        grp = mod.gate_proj.__dict__.get("_qz_group")
        if pair and grp is not None and len(grp.members) == 2 and grp.members[0] is mod.gate_proj and \
                grp.members[1] is mod.up_proj:
            # gate, up and their product: one launch (row shards: on this rank's rows, then one
            # exchange of the product)
            h = linear4bit_silu_pair(grp, x) if grp._compute is not parallel.sharded_group_compute \
                else parallel.sharded_silu_pair(grp, x)
        if h is None:
            g = mod.gate_proj(x)  # same call order as LlamaMLP.forward (a DecodeGroup launches gate+up here)
            u = mod.up_proj(x)
            h = silu_mul(g, u) if silu_mul_supported(g, u) else mod.act_fn(g) * u
        return _project(mod.down_proj, h, _qz_residual)
    return forward


def _residual_decoder_forward(mod: nn.Module):
    """LlamaDecoderLayer.forward (modeling_llama.py:295-324) with both `residual + h` adds
    moved into the epilogues of the o_proj and down_proj GEMVs (their modules were patched by
    fuse_layer_ops and take `_qz_residual`); the norms are called as the model has them (an
    identity once fuse_prenorm absorbed them).  Bit-identical to the original."""
    def forward(hidden_states, attention_mask=None, position_ids=None, past_key_values=None, use_cache=False,
                position_embeddings=None, **kwargs):
        h = mod.input_layernorm(hidden_states)
        hidden_states, _ = mod.self_attn(hidden_states=h, attention_mask=attention_mask, position_ids=position_ids,
                                         past_key_values=past_key_values, use_cache=use_cache,
                                         position_embeddings=position_embeddings, _qz_residual=hidden_states, **kwargs)
        h = mod.post_attention_layernorm(hidden_states)
        return mod.mlp(h, _qz_residual=hidden_states)
    return forward


def _static_layer(cache, idx):
    """The StaticLayer (cache_utils.py:400-487) holding layer `idx` of a StaticCache, or None."""
    layers = getattr(cache, "layers", None)
    if layers is None or idx is None or idx >= len(layers):
        return None
    layer = layers[idx]
    if type(layer).__name__ != "StaticLayer" or not getattr(layer, "is_initialized", False):
        return None
    return layer


def _fused_attention_forward(mod: nn.Module, orig):
    """LlamaAttention.forward (modeling_llama.py:243-281) with everything between the q/k/v
    projections and o_proj as ONE launch (layer_ops.decode_attention) when a single new token
    meets a StaticCache layer and the bool mask sdpa would get; any other call (prefill, other
    caches, eager/flash attention, float masks) runs the original forward."""
    from .layer_ops import decode_attention, decode_attention_supported

    def forward(hidden_states, position_embeddings=None, attention_mask=None, past_key_values=None,
                _qz_residual=None, **kwargs):
        # _qz_residual (the residual-fused decoder layer): return residual + attention output
        layer = None
        if (hidden_states.dim() == 3 and hidden_states.shape[1] == 1 and position_embeddings is not None
                and not kwargs.get("output_attentions", False) and not mod.training
                and getattr(mod.config, "_attn_implementation", None) == "sdpa"):
            layer = _static_layer(past_key_values, getattr(mod, "layer_idx", None))
        if layer is not None:
            cos, sin = position_embeddings
            # query heads of THIS module: the cache holds its kv heads (a tensor-parallel rank
            # keeps a share of them), the GQA ratio is the model's
            nq = layer.keys.shape[1] * (mod.config.num_attention_heads // mod.config.num_key_value_heads) \
                if layer.keys.dim() == 4 else 0
            if layer.keys.shape[-1] == mod.head_dim and decode_attention_supported(
                    hidden_states, cos, layer.keys, layer.values, attention_mask, layer.cumulative_length, nq):
                arrive = mod.__dict__.get("_qz_attn_arrive")
                if arrive is None or arrive.device != hidden_states.device:
                    arrive = torch.zeros(1, dtype=torch.int32, device=hidden_states.device)
                    mod.__dict__["_qz_attn_arrive"] = arrive
                q = mod.q_proj(hidden_states)
                k = mod.k_proj(hidden_states)
                v = mod.v_proj(hidden_states)
                if q.shape[-1] != nq * mod.head_dim or k.shape[-1] != layer.keys.shape[1] * mod.head_dim:
                    h, w = orig(hidden_states, position_embeddings, attention_mask, past_key_values, **kwargs)
                    return (h if _qz_residual is None else _qz_residual + h), w
                out = decode_attention(q, k, v, cos, sin, layer.keys, layer.values, attention_mask,
                                       layer.cumulative_length, arrive, nq, mod.scaling)
                return _project(mod.o_proj, out, _qz_residual), None
        h, w = orig(hidden_states, position_embeddings, attention_mask, past_key_values, **kwargs)
        return (h if _qz_residual is None else _qz_residual + h), w
    return forward


def _project(proj: nn.Module, x: torch.Tensor, residual):
    """proj(x), or residual + proj(x) with the add in the GEMV epilogue where proj is a
    Linear4bit that decodes x on its own (Linear4bit.forward_residual)."""
    if residual is None:
        return proj(x)
    fr = getattr(proj, "forward_residual", None)
    return fr(x, residual) if fr is not None else residual + proj(x)


def _fused_decoder_forward(mod: nn.Module):
    """LlamaDecoderLayer.forward (modeling_llama.py:295-324) with lines 317-321
    (`residual + h`, then post_attention_layernorm) as one add_rms_norm launch."""
    from .layer_ops import add_rms_norm, add_rms_norm_supported

    def forward(hidden_states, attention_mask=None, position_ids=None, past_key_values=None, use_cache=False,
                position_embeddings=None, **kwargs):
        residual = hidden_states
        h = mod.input_layernorm(hidden_states)
        h, _ = mod.self_attn(hidden_states=h, attention_mask=attention_mask, position_ids=position_ids,
                             past_key_values=past_key_values, use_cache=use_cache,
                             position_embeddings=position_embeddings, **kwargs)
        ln = mod.post_attention_layernorm
        if add_rms_norm_supported(h, residual, ln.weight):
            residual, h = add_rms_norm(h, residual, ln.weight, ln.variance_epsilon)
        else:
            h = residual + h
            residual = h
            h = ln(h)
        h = mod.mlp(h)
        return residual + h
    return forward


def fuse_layer_ops(model: nn.Module, norm: bool = True, rope: bool = True, mlp: bool = True,
                   decoder: bool = False, attention: bool = True, residual: bool = True,
                   mlp_pair: bool = True) -> int:
    """Route every Llama-style RMSNorm of `model`, the rotary embedding of its
    attention modules, the SiLU-gate product of its MLPs and each decoder
    layer's residual add + post-attention norm through one HIP launch each
    (layer_ops.rms_norm / rope_qk / silu_mul / add_rms_norm) instead of
    transformers' 8-, 10-, 2- and 9-launch eager forms.  Inputs the kernels do not
    take keep the original code.  Returns the number of modules patched (norms,
    MLPs, decoder layers, and modeling modules whose apply_rotary_pos_emb was
    replaced).  `decoder` (opt-in) replaces LlamaDecoderLayer.forward itself with
    a restatement; it measured no gain on the bs=1 graph step.
    `attention` routes a decode step's rotary + StaticCache update + sdpa attention of
    each Llama/Mistral/Qwen2 attention module through layer_ops.decode_attention (counted
    once per module).  `residual` (with `attention` and `mlp`) moves each decoder layer's two
    residual adds into the o_proj / down_proj GEMV epilogues (counted once per layer).
    `mlp_pair` lets a fused MLP compute gate/up and act_fn(gate) * up in one launch
    (modules.linear4bit_silu_pair) where its projections form a decode group."""
    import sys

    n = 0
    for m in model.modules():
        name = type(m).__name__
        if norm and name in RMSNORM_CLASSES and "forward" not in m.__dict__ and hasattr(m, "variance_epsilon"):
            m.__dict__["forward"] = _fused_rmsnorm_forward(m, m.forward)
            m.__dict__["_qz_fused_norm"] = True
            n += 1
        elif decoder and name in DECODER_CLASSES and "forward" not in m.__dict__ and \
                type(getattr(m, "post_attention_layernorm", None)).__name__ in RMSNORM_CLASSES and \
                all(hasattr(m, a) for a in ("input_layernorm", "self_attn", "mlp")):
            m.__dict__["forward"] = _fused_decoder_forward(m)
            m.__dict__["_qz_fused_decoder"] = True
            n += 1
        elif mlp and name in MLP_CLASSES and "forward" not in m.__dict__ and \
                "silu" in type(getattr(m, "act_fn", None)).__name__.lower() and \
                all(hasattr(m, p) for p in ("gate_proj", "up_proj", "down_proj")):
            m.__dict__["forward"] = _fused_mlp_forward(m, pair=mlp_pair)
            m.__dict__["_qz_fused_mlp"] = True
            n += 1
        elif (rope or attention) and name in ATTENTION_CLASSES:
            if attention and "forward" not in m.__dict__ and all(
                    hasattr(m, a) for a in ("q_proj", "k_proj", "v_proj", "o_proj", "scaling", "head_dim")):
                m.__dict__["forward"] = _fused_attention_forward(m, m.forward)
                m.__dict__["_qz_fused_attn"] = True
                n += 1
            if not rope:
                continue
            modname = type(m).__module__
            mod = sys.modules.get(modname)
            fn = getattr(mod, "apply_rotary_pos_emb", None)
            if fn is not None and modname not in _ROPE_PATCHED and _half_split_rotate(mod):
                _ROPE_PATCHED[modname] = fn
                mod.apply_rotary_pos_emb = _fused_rope(fn)
                n += 1
    if residual and attention and mlp and not decoder:
        for m in model.modules():
            if type(m).__name__ in DECODER_CLASSES and "forward" not in m.__dict__ and \
                    "_qz_fused_attn" in getattr(m, "self_attn", nn.Module()).__dict__ and \
                    "_qz_fused_mlp" in getattr(m, "mlp", nn.Module()).__dict__:
                m.__dict__["forward"] = _residual_decoder_forward(m)
                m.__dict__["_qz_residual_decoder"] = True
                n += 1
    return n


def unfuse_layer_ops(model: nn.Module) -> None:
    """Undo fuse_layer_ops (norm forwards and every patched apply_rotary_pos_emb) and any
    fuse_prenorm on top of it."""
    import sys

    unfuse_prenorm(model)
    for m in model.modules():
        if m.__dict__.pop("_qz_fused_norm", None) or m.__dict__.pop("_qz_fused_mlp", None) or \
                m.__dict__.pop("_qz_fused_decoder", None) or m.__dict__.pop("_qz_fused_attn", None) or \
                m.__dict__.pop("_qz_residual_decoder", None):
            m.__dict__.pop("forward", None)
            m.__dict__.pop("_qz_attn_arrive", None)
    for modname, fn in list(_ROPE_PATCHED.items()):
        setattr(sys.modules[modname], "apply_rotary_pos_emb", fn)
        del _ROPE_PATCHED[modname]


# ---------------------------------------------------------------------------
# the host model's per-step glue around the decoder layers (not the Linear4bit path): the causal
# mask and the rotary cos/sin, one launch each in place of the 7-9 small torch kernels each of them
# costs a decode step (profiles/r5_decode_anatomy_8b.txt), with the same values
# ---------------------------------------------------------------------------

ROTARY_CLASSES = ("LlamaRotaryEmbedding", "MistralRotaryEmbedding", "Qwen2RotaryEmbedding")
MODEL_CLASSES = ("LlamaModel", "MistralModel", "Qwen2Model")
_MASK_PATCHED = {}  # modeling module name -> original create_causal_mask
_ROPE_TABLE_MAX = 1 << 17


def _table_rope_forward(mod: nn.Module, orig):
    from .layer_ops import rope_table

    def forward(x, position_ids, *args, **kw):
        t = mod.__dict__.get("_qz_rope_tables", {}).get((x.dtype, x.device))
        if t is None or args or kw or not (isinstance(position_ids, torch.Tensor) and position_ids.dim() == 2 and
                                           position_ids.dtype == torch.int64 and position_ids.device == x.device):
            return orig(x, position_ids, *args, **kw)
        return rope_table(position_ids, t[0], t[1], mod.__dict__["_qz_inv_f32"], mod.attention_scaling)
    return forward


def _fast_causal_mask(orig):
    from .layer_ops import decode_mask

    def create_causal_mask(*args, **kw):
        # one new token per sequence, keywords as LlamaModel.forward passes them, no padding mask,
        # sdpa's bool mask, a static (compileable, non-sliding) cache: the mask is kv j <= q_offset
        emb, pkv, cfg = kw.get("inputs_embeds"), kw.get("past_key_values"), kw.get("config")
        if (not args and set(kw) <= {"config", "inputs_embeds", "attention_mask", "past_key_values", "position_ids"}
                and kw.get("attention_mask") is None and cfg is not None and isinstance(emb, torch.Tensor)
                and emb.is_cuda and emb.dim() == 3 and emb.shape[1] == 1 and pkv is not None
                and getattr(cfg, "is_causal", True) and getattr(cfg, "_attn_implementation", None) == "sdpa"
                and getattr(cfg, "sliding_window", None) is None and getattr(pkv, "is_compileable", False)
                and not any(getattr(pkv, "is_sliding", ()))):
            try:
                q_off = pkv.get_query_offset(0)
                kv_length, kv_offset = pkv.get_mask_sizes(1, 0)
            except Exception:
                q_off = kv_offset = None
            if (isinstance(q_off, torch.Tensor) and q_off.dtype == torch.int64 and q_off.numel() == 1
                    and q_off.device == emb.device and kv_offset == 0 and isinstance(kv_length, int)):
                return decode_mask(q_off, emb.shape[0], kv_length)
        return orig(*args, **kw)
    create_causal_mask._qz_orig = orig
    return create_causal_mask


def fuse_decode_glue(model: nn.Module) -> int:
    """Route a GPU model's rotary embedding through cos/sin tables its own forward computes once
    here (positions 0..max_position_embeddings-1, the model's dtype; looked up by
    layer_ops.rope_table) and its modeling module's create_causal_mask, for one new token against
    a static cache, through layer_ops.decode_mask.  Everything else (CPU models, dynamic rope
    types, padding masks, other caches) keeps transformers' own code.  Returns the number of
    patches."""
    import sys

    n = 0
    emb = model.get_input_embeddings() if hasattr(model, "get_input_embeddings") else None
    dtype = emb.weight.dtype if emb is not None and hasattr(emb, "weight") else None
    for m in model.modules():
        if type(m).__name__ not in ROTARY_CLASSES or "_qz_rope_orig" in m.__dict__:
            continue
        inv = getattr(m, "inv_freq", None)
        rt = str(getattr(m, "rope_type", "default"))
        T = min(int(getattr(m, "max_seq_len_cached", 0) or 0), _ROPE_TABLE_MAX)
        if (not isinstance(inv, torch.Tensor) or not inv.is_cuda or not inv.is_floating_point() or "dynamic" in rt
                or rt == "longrope" or T <= 0 or dtype not in (torch.float16, torch.bfloat16, torch.float32)):
            continue
        orig = m.forward
        with torch.no_grad():
            cos, sin = orig(torch.empty(0, dtype=dtype, device=inv.device),
                            torch.arange(T, device=inv.device).unsqueeze(0))
        m.__dict__["_qz_rope_orig"] = orig
        m.__dict__["_qz_inv_f32"] = inv.float().contiguous()   # what forward's .float() makes of it
        m.__dict__["_qz_rope_tables"] = {(dtype, inv.device): (cos[0].contiguous(), sin[0].contiguous())}
        m.__dict__["forward"] = _table_rope_forward(m, orig)
        n += 1
    for m in model.modules():
        modname = type(m).__module__
        if type(m).__name__ in MODEL_CLASSES and modname not in _MASK_PATCHED and n:
            mod = sys.modules.get(modname)
            fn = getattr(mod, "create_causal_mask", None) if mod is not None else None
            if fn is not None:
                _MASK_PATCHED[modname] = fn
                setattr(mod, "create_causal_mask", _fast_causal_mask(fn))
                n += 1
    return n


def fuse_lm_head(model: nn.Module) -> int:
    """Route the model's unquantised fp16/bf16 output projection (get_output_embeddings(), no bias)
    through layer_ops.gemv_dense for a single decode token (6.8 vs 5.7 TB/s for hipBLASLt at
    128256 x 4096, profiles/r5_lm_head_times.txt); every other input keeps F.linear.  Returns 1 if
    patched."""
    head = model.get_output_embeddings() if hasattr(model, "get_output_embeddings") else None
    if not isinstance(head, nn.Linear) or head.bias is not None or "_qz_dense_head" in head.__dict__:
        return 0
    from .layer_ops import gemv_dense, gemv_dense_supported

    orig = head.forward

    def forward(x):
        if gemv_dense_supported(x, head.weight):
            return gemv_dense(x, head.weight)
        return orig(x)
    head.__dict__["forward"] = forward
    head.__dict__["_qz_dense_head"] = True
    return 1


def unfuse_lm_head(model: nn.Module) -> None:
    head = model.get_output_embeddings() if hasattr(model, "get_output_embeddings") else None
    if head is not None and head.__dict__.pop("_qz_dense_head", None):
        head.__dict__.pop("forward", None)


def unfuse_decode_glue(model: nn.Module) -> None:
    """Undo fuse_decode_glue."""
    import sys

    for m in model.modules():
        if m.__dict__.pop("_qz_rope_orig", None) is not None:
            m.__dict__.pop("forward", None)
            m.__dict__.pop("_qz_rope_tables", None)
            m.__dict__.pop("_qz_inv_f32", None)
    for modname, fn in list(_MASK_PATCHED.items()):
        setattr(sys.modules[modname], "create_causal_mask", fn)
        del _MASK_PATCHED[modname]


# ---------------------------------------------------------------------------
# pre-quantised checkpoints
# ---------------------------------------------------------------------------

def save_quantized(model: nn.Module, path: str) -> None:
    """Write `model`'s state dict (Linear4bit weights as packed bytes + their
    quant_state in the bnb key layout) to a safetensors file."""
    from safetensors.torch import save_file

    sd = {}
    seen = {}
    for k, v in model.state_dict().items():
        t = v.detach().to("cpu").contiguous()
        key = (t.data_ptr(), t.dtype, tuple(t.shape)) if t.numel() else None
        if key is not None and key in seen:  # tied tensors: safetensors stores each once
            t = t.clone()
        seen[key] = k
        sd[k] = t
    save_file(sd, path, metadata={"format": "pt", "quantization": "bitsandbytes-4bit-compatible (quantizations_amd)"})


def load_quantized(model: nn.Module, path: str, device=None, modules_to_not_convert: Optional[Iterable[str]] = None,
                   compute_dtype=None) -> nn.Module:
    """Load a save_quantized() checkpoint into `model` without re-quantising.

    `model` may be built on the meta device (``with torch.device("meta"):``).
    Every nn.Linear whose checkpoint entry carries a packed quant_state becomes
    a Linear4bit around the stored bytes; everything else is assigned as is.
    The model is then moved to `device` (default "cuda")."""
    from safetensors.torch import load_file

    sd = load_file(path, device="cpu")
    marker = "." + QuantState.PACKED_PREFIX
    quantised = {k[:k.index(marker)] for k in sd if marker in k}   # e.g. "model.layers.0.self_attn.q_proj.weight"
    skip = set(modules_to_not_convert or [])

    def visit(parent: nn.Module, prefix: str):
        for name, child in list(parent.named_children()):
            full = f"{prefix}.{name}" if prefix else name
            if isinstance(child, nn.Linear) and not isinstance(child, Linear4bit) and \
                    full + ".weight" in quantised and name not in skip:
                parent._modules[name] = Linear4bit(child.in_features, child.out_features, child.bias is not None,
                                                   compute_dtype, device="meta")
            else:
                visit(child, full)

    visit(model, "")
    missing, unexpected = model.load_state_dict(sd, strict=False, assign=True)
    missing = [k for k in missing if not k.endswith("rotary_emb.inv_freq")]
    if missing or unexpected:
        raise RuntimeError(f"load_quantized: missing {missing[:5]}..., unexpected {unexpected[:5]}...")
    return model.to(device or "cuda")

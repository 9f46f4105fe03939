"""Row-sharded Linear4bit across GPUs (one process per GPU, RCCL all-gather).

The 4-bit layer is independent per output row, so rank p of P keeps rows
[p*M/P, (p+1)*M/P).  In the flat row-major layout that is a contiguous slice
of the packed bytes, of the per-block scales and (with double quant) of the
256-block second-level scales -- the GLOBAL quant state is sliced, never
re-quantised, so every rank multiplies exactly the single-GPU layer's weights
(outputs equal up to fp32 summation order where the shard's launch geometry
differs).
x is replicated; after the local fused GEMV/GEMM the fp16 row shards are
exchanged with ``all_gather_into_tensor`` (RCCL over xGMI on MI355X, gloo in
the CPU tests), or -- with a ``gatherer`` (exchange.OneShotAllGather) -- by one
launch that stores every shard straight into the peers' IPC-mapped buffers.  The reference has no multi-GPU path; this is the build's
(SURVEY.md section 8e).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .core import QuantState, exact_codes_for
from .exchange import all_gather_into


@dataclass
class RowShard:
    """Tensors and indices of one rank's rows of a 4-bit weight."""
    packed: torch.Tensor          # u8 bytes of rows [r0, r1)
    state: QuantState             # sliced statistics (shape = (r1 - r0, K))
    r0: int
    r1: int
    block_base: int               # first block index inside the sliced scale arrays


def shard_rows(packed: torch.Tensor, qs: QuantState, rank: int, world: int) -> RowShard:
    """Slice rows [rank*M/world, (rank+1)*M/world) of a quantised weight (device agnostic)."""
    M, K = int(qs.shape[0]), int(qs.shape[1])
    if M % world != 0:
        raise ValueError(f"out_features {M} is not divisible by world size {world}")
    if K % 2 != 0:
        raise ValueError("row sharding needs an even in_features (rows start on a byte)")
    rows = M // world
    r0, r1 = rank * rows, (rank + 1) * rows
    bs = qs.blocksize
    e0, e1 = r0 * K, r1 * K
    if e0 % bs != 0:
        raise ValueError("row shard must start on a scale-block boundary (rows*K % blocksize == 0)")
    flat = packed.reshape(-1)
    sub_packed = flat[e0 // 2:e1 // 2]
    b0, b1 = e0 // bs, (e1 + bs - 1) // bs
    block_base = 0
    if qs.nested:
        # the kernel reads qabsmax[block_base + b] and absmax2[(block_base + b) / bs2] (b local):
        # slice both from the second-level block that contains b0
        bs2 = qs.state2.blocksize
        c0 = b0 // bs2
        block_base = b0 - c0 * bs2
        state2 = QuantState(absmax=qs.state2.absmax[c0:(b1 + bs2 - 1) // bs2], code=qs.state2.code,
                            blocksize=bs2, dtype=qs.state2.dtype)
        absmax = qs.absmax[c0 * bs2:b1]
    else:
        state2 = None
        absmax = qs.absmax[b0:b1]
    st = QuantState(absmax=absmax, shape=torch.Size([rows, K]), code=qs.code, blocksize=bs,
                    quant_type=qs.quant_type, dtype=qs.dtype, offset=qs.offset, state2=state2)
    return RowShard(sub_packed, st, r0, r1, block_base)


def gather_rows(y: torch.Tensor, world: int, group=None, gatherer=None) -> torch.Tensor:
    """Every rank's output rows [..., M/P] -> the full [..., M] on every rank, rank-major."""
    lead = y.shape[:-1]
    rows = y.shape[-1]
    y2 = y.reshape(-1, rows).contiguous()
    T = y2.shape[0]
    gathered = torch.empty((world * T, rows), dtype=y.dtype, device=y.device)
    all_gather_into(gathered, y2, group, gatherer)
    if T == 1:
        return gathered.reshape(*lead, world * rows)
    full = gathered.view(world, T, rows).permute(1, 0, 2).reshape(T, world * rows)
    return full.reshape(*lead, world * rows)


class RowShardedLinear4bit(nn.Module):
    """This rank's rows of a (quantised) ``Linear4bit``; forward returns the FULL
    output on every rank: local fused 4-bit matmul, then an all-gather."""

    def __init__(self, full: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None,
                 group=None, local_matmul: Optional[Callable] = None, gather: bool = True, gatherer=None):
        super().__init__()
        self.gather = gather  # False: column-parallel (Megatron), the output stays this rank's shard
        self.gatherer = gatherer  # None: dist.all_gather_into_tensor; else e.g. exchange.OneShotAllGather
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world_size = dist.get_world_size(group) if world_size is None else world_size
        self.group = group
        qs = full.weight.quant_state
        shard = shard_rows(full.weight.data, qs, self.rank, self.world_size)
        # own the shard's memory so the full weight can be freed
        self.register_buffer("packed", shard.packed.clone(), persistent=False)
        st = shard.state
        st.absmax = st.absmax.clone()
        if st.nested:
            st.state2.absmax = st.state2.absmax.clone()
        self.state = st
        self.block_base = shard.block_base
        self.r0, self.r1 = shard.r0, shard.r1
        self.in_features = full.in_features
        self.out_features = full.out_features
        bias = None if full.bias is None else full.bias.data[shard.r0:shard.r1].clone()
        self.register_buffer("bias", bias, persistent=False)
        self._local_matmul = local_matmul  # test hook; None = the fused HIP kernels
        self.exact_codes = exact_codes_for(getattr(full, "compute_dtype", None))
        # True (shard_attention_heads, on o_proj): the input is this rank's slice of the features
        # (its attention heads' output), gathered to the full width before the local rows
        self.gather_input = False

    def gathered_input(self, x: torch.Tensor) -> torch.Tensor:
        """x itself, or (gather_input) every rank's slice of it gathered to the full in_features."""
        if not self.gather_input or self.world_size == 1:
            return x
        if x.shape[-1] * self.world_size != self.in_features:
            raise ValueError(f"head-gathered input: expected {self.in_features // self.world_size} features, "
                             f"got {x.shape[-1]}")
        return gather_rows(x, self.world_size, self.group, self.gatherer)

    def local_forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._local_matmul is not None:
            return self._local_matmul(x, self)
        from .core import gemm_4bit, gemv_4bit
        if x.numel() == x.shape[-1]:
            return gemv_4bit(x, self.packed, state=self.state, bias=self.bias, block_base=self.block_base,
                             exact_codes=self.exact_codes)
        if self.block_base != 0:
            raise ValueError("prefill on a shard needs block-aligned second-level scales")
        return gemm_4bit(x, self.packed, self.state, bias=self.bias)

    def gather_rows(self, y: torch.Tensor) -> torch.Tensor:
        """This rank's output rows [..., M/P] -> the full [..., M] on every rank (the
        all-gather); column-parallel layers (gather=False) and world size 1 return y."""
        if not self.gather or self.world_size == 1:
            return y
        return gather_rows(y, self.world_size, self.group, self.gatherer)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        group = self.__dict__.get("_qz_group")
        if group is not None and group.accepts(x):
            return group.take(self, x)
        if group is not None and group.prenorm is not None:
            x = group.prenorm[2](x)      # prefill through a group that absorbed its RMSNorm
        return self.gather_rows(self.local_forward(self.gathered_input(x)))   # [..., M/P] -> [..., M]

    def forward_residual(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """residual + self(x), for LlamaDecoderLayer's residual adds (integration._project):
        a single token's add rides in the local GEMV's epilogue on this rank's rows
        (qz_gemv_4bit_residual: the same bits as the unsharded layer's fused epilogue), and the
        rows are gathered afterwards.  Anything else: the two-op form."""
        x_in, x = x, self.gathered_input(x)
        if (self._local_matmul is None and self.gather and x.is_cuda and x.numel() == x.shape[-1]
                and residual.dtype == x.dtype and residual.device == x.device and residual.is_contiguous()
                and residual.numel() == self.out_features and residual.shape[:-1] == x.shape[:-1]
                and self.__dict__.get("_qz_group") is None):
            from .core import gemv_4bit
            rows = residual.reshape(-1)[self.r0:self.r1]
            y = gemv_4bit(x, self.packed, state=self.state, bias=self.bias, block_base=self.block_base,
                          exact_codes=self.exact_codes, residual=rows)
            return self.gather_rows(y).reshape(residual.shape)
        return residual + self(x_in)


def _group_input(group, x: torch.Tensor, fused_ok: bool):
    """The input the members multiply and the norm for the launch: a DecodeGroup's absorbed
    RMSNorm (integration.fuse_prenorm) rides inside a single-token launch where the kernel
    takes it (fused_ok), else it runs first as the model ran it."""
    norm = group.prenorm
    if norm is None:
        return x, None
    if (fused_ok and x.is_cuda and x.numel() == x.shape[-1] and norm[0].dtype == x.dtype
            and norm[0].is_contiguous() and norm[0].numel() == x.shape[-1]):
        return x, norm[:2]
    return norm[2](x), None


def _sharded_group_tokens(group, x: torch.Tensor):
    """T = 2..16 decode tokens (a small batch of streams): ONE grouped
    multi-token launch for the members' row shards, then (gather mode) ONE
    all-gather of the [T, sum(rows)] concatenation."""
    from .core import gemm_4bit_grouped, grouped_tokens_ok

    ms = group.members
    x, _ = _group_input(group, x, fused_ok=False)
    K = x.shape[-1]
    T = x.numel() // K
    lead = x.shape[:-1]
    items = [(m.packed, m.state, m.bias, m.block_base) for m in ms]
    if ms[0]._local_matmul is not None:  # test hook (CPU)
        outs = [m._local_matmul(x, m) for m in ms]
    elif grouped_tokens_ok(x, items):
        outs = gemm_4bit_grouped(x, items)
    else:
        outs = [m.local_forward(x) for m in ms]
    if not ms[0].gather or ms[0].world_size == 1:  # column-parallel / one rank: nothing to exchange
        return [o.reshape(*lead, o.shape[-1]) for o in outs]
    rows = [m.r1 - m.r0 for m in ms]
    S = sum(rows)
    P = ms[0].world_size
    buf = torch.cat([o.reshape(T, r) for o, r in zip(outs, rows)], dim=1).contiguous()   # [T, S]
    gathered = torch.empty((P * T, S), dtype=buf.dtype, device=buf.device)
    all_gather_into(gathered, buf, ms[0].group, ms[0].gatherer)
    gathered = gathered.view(P, T, S)
    res, o = [], 0
    for r in rows:
        res.append(gathered[:, :, o:o + r].permute(1, 0, 2).reshape(*lead, P * r))
        o += r
    return res


def sharded_group_compute(group, x: torch.Tensor):
    """Decode step of a DecodeGroup of RowShardedLinear4bit layers: ONE grouped
    local GEMV writes every member's row shard into one buffer, ONE all-gather
    exchanges it (instead of one all-gather per layer: bs=1 decode collectives
    are latency-bound), then each member's full output is cut out of the
    [world, sum(rows)] result.  2..16 tokens: _sharded_group_tokens."""
    from .core import gemv_4bit_grouped

    if x.numel() != x.shape[-1]:
        return _sharded_group_tokens(group, x)
    ms = group.members
    x, norm = _group_input(group, x, fused_ok=ms[0]._local_matmul is None)
    rows = [m.r1 - m.r0 for m in ms]
    S = sum(rows)
    buf = torch.empty(S, dtype=x.dtype, device=x.device)
    views, o = [], 0
    for r in rows:
        views.append(buf[o:o + r])
        o += r
    if ms[0]._local_matmul is not None:  # test hook (CPU): per-member local matmul
        for m, v in zip(ms, views):
            v.copy_(m._local_matmul(x, m).reshape(-1))
    else:
        gemv_4bit_grouped(x, [(m.packed, m.state, m.bias, m.block_base, v) for m, v in zip(ms, views)],
                          exact_codes=ms[0].exact_codes, norm=norm)
    lead = x.shape[:-1]
    if not ms[0].gather or ms[0].world_size == 1:  # column-parallel / one rank: nothing to exchange
        return [v.view(*lead, r) for v, r in zip(views, rows)]
    P = ms[0].world_size
    gathered = torch.empty(P * S, dtype=x.dtype, device=x.device)
    all_gather_into(gathered, buf, ms[0].group, ms[0].gatherer)
    g2 = gathered.view(P, S)
    outs, o = [], 0
    for r in rows:
        outs.append(g2[:, o:o + r].reshape(*lead, P * r))
        o += r
    return outs


def sharded_silu_pair(group, x: torch.Tensor) -> Optional[torch.Tensor]:
    """act_fn(gate_proj(x)) * up_proj(x) for a decode group of exactly the row shards of
    (gate_proj, up_proj) and a single token: ONE launch on this rank's rows
    (core.gemv_4bit_pair_silu with the shards' block_base, an absorbed RMSNorm inside), then
    ONE all-gather of the [M/P] product h -- instead of the grouped launch, the exchange of
    gate AND up, and a separate SiLU-product launch.  Column-parallel shards (the Megatron
    pairing) keep their h rows: they are exactly what the row-parallel down_proj takes.  None
    when the launch does not take the case (the caller then calls the members)."""
    ms = group.members
    if group._compute is not sharded_group_compute or len(ms) != 2 or x.numel() != x.shape[-1]:
        return None
    g, u = ms
    if (g.r0, g.r1) != (u.r0, u.r1) or g.exact_codes != u.exact_codes or \
            (g._local_matmul is None and not (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16))):
        return None
    xin, norm = _group_input(group, x, fused_ok=g._local_matmul is None)
    if g._local_matmul is not None:  # test hook (CPU): the two local products and torch's SiLU
        h = torch.nn.functional.silu(g._local_matmul(xin, g)) * u._local_matmul(xin, u)
    else:
        from .core import gemv_4bit_pair_silu
        h = gemv_4bit_pair_silu(xin, [(g.packed, g.state, g.bias, g.block_base), (u.packed, u.state, u.bias, u.block_base)],
                                exact_codes=g.exact_codes, norm=norm)
        if h is None:
            return None
    return g.gather_rows(h.reshape(*x.shape[:-1], g.r1 - g.r0))


def consumer_absmax(qs: QuantState) -> torch.Tensor:
    """Per-block fp32 absmax exactly as the kernels rebuild it (core.py:467-468:
    code2[q] * absmax2[b / bs2], then + offset, two fp32 roundings)."""
    if not qs.nested:
        return qs.absmax
    nb = qs.absmax.numel()
    idx = torch.arange(nb, device=qs.absmax.device) // qs.state2.blocksize
    prod = qs.state2.code[qs.absmax.long()].float() * qs.state2.absmax[idx].float()
    return prod + qs.offset.float()


@dataclass
class ColShard:
    """One rank's input columns [k0, k1) of every row of a 4-bit weight."""
    packed: torch.Tensor          # u8, re-packed [M, (k1-k0)/2] row-major
    state: QuantState             # shape (M, k1-k0), fp32 per-block absmax (double quant resolved)
    k0: int
    k1: int


def shard_cols(packed: torch.Tensor, qs: QuantState, rank: int, world: int) -> ColShard:
    """Slice input columns [rank*K/world, (rank+1)*K/world) of every row (row-parallel
    layers).  Blocks stay whole (K/world must be a multiple of blocksize); the
    rows' bytes are re-packed contiguously and the per-block scales become the
    fp32 values the kernel would have rebuilt, so every local product is
    bit-identical to the full layer's."""
    M, K = int(qs.shape[0]), int(qs.shape[1])
    if K % world != 0:
        raise ValueError(f"in_features {K} is not divisible by world size {world}")
    Kp = K // world
    bs = qs.blocksize
    if Kp % bs != 0 or K % bs != 0:
        raise ValueError(f"column shard width {Kp} must be a multiple of blocksize {bs}")
    k0, k1 = rank * Kp, (rank + 1) * Kp
    loc = packed.reshape(M, K // 2)[:, k0 // 2:k1 // 2].contiguous().reshape(-1, 1)
    am = consumer_absmax(qs).reshape(M, K // bs)[:, k0 // bs:k1 // bs].contiguous().reshape(-1)
    st = QuantState(absmax=am, shape=torch.Size([M, Kp]), code=qs.code, blocksize=bs, quant_type=qs.quant_type,
                    dtype=qs.dtype)
    return ColShard(loc, st, k0, k1)


class RowParallelLinear4bit(nn.Module):
    """Megatron row-parallel 4-bit layer: this rank's input columns; takes the
    LOCAL slice of the activation (the output of a column-parallel layer) and
    all-reduces the partial products.  The bias is added once (rank 0).  The
    partials are summed in fp32 and rounded to the activation dtype once, so the
    result differs from the single-GPU layer only by the one rounding of each
    rank's partial (not by P extra fp16 roundings inside the collective)."""

    def __init__(self, full: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None,
                 group=None, local_matmul: Optional[Callable] = None, gatherer=None):
        super().__init__()
        self.gatherer = gatherer  # None: dist.all_reduce; else the partials are all-gathered and summed
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world_size = dist.get_world_size(group) if world_size is None else world_size
        self.group = group
        sh = shard_cols(full.weight.data, full.weight.quant_state, self.rank, self.world_size)
        self.register_buffer("packed", sh.packed, persistent=False)
        self.state = sh.state
        self.block_base = 0
        self.k0, self.k1 = sh.k0, sh.k1
        self.in_features = full.in_features
        self.out_features = full.out_features
        bias = None if (full.bias is None or self.rank != 0) else full.bias.data.clone()
        self.register_buffer("bias", bias, persistent=False)
        self._local_matmul = local_matmul  # test hook; None = the fused HIP kernels
        self.exact_codes = exact_codes_for(getattr(full, "compute_dtype", None))

    def forward(self, x_local: torch.Tensor) -> torch.Tensor:
        if x_local.shape[-1] != self.k1 - self.k0:
            raise ValueError(f"row-parallel layer expects its {self.k1 - self.k0}-wide input slice, "
                             f"got {x_local.shape[-1]}")
        if self._local_matmul is not None:
            y = self._local_matmul(x_local, self)
        else:
            from .core import gemm_4bit, gemv_4bit
            if x_local.numel() == x_local.shape[-1]:
                y = gemv_4bit(x_local, self.packed, state=self.state, bias=self.bias, exact_codes=self.exact_codes)
            else:
                y = gemm_4bit(x_local, self.packed, self.state, bias=self.bias)
        y32 = y.float().contiguous()   # [..., M] fp32: 16 KiB at bs=1 for M = 4096
        if self.gatherer is not None and self.gatherer.accepts(y32):
            # one-shot: every rank's fp32 partial lands here, summed in rank order (the same
            # order on every rank, so all ranks hold identical sums)
            parts = torch.empty((self.world_size,) + tuple(y32.shape), dtype=torch.float32, device=y32.device)
            self.gatherer(parts, y32)
            y32 = parts.sum(0)
        else:
            dist.all_reduce(y32, group=self.group)
        return y32.to(y.dtype)


# (column-parallel, row-parallel) projection names per block kind
TP_BLOCKS = ((("q_proj", "k_proj", "v_proj"), "o_proj"), (("gate_proj", "up_proj"), "down_proj"))


def apply_tensor_parallel(model: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None,
                          group=None, local_matmul: Optional[Callable] = None, gatherer=None) -> int:
    """Megatron-style TP pairing over the Linear4bit layers of a decoder
    (SURVEY.md 8f row 3): q/k/v and gate/up become column-parallel (each rank
    keeps its attention heads / MLP columns, no collective), o_proj and
    down_proj row-parallel (one all-reduce each) -- two collectives per layer
    instead of one per Linear.  Attention then runs on the rank's local heads
    (transformers infers the head count from the projection width and sizes the
    KV cache lazily).  Returns the number of blocks converted."""
    from .modules import Linear4bit

    rank = dist.get_rank(group) if rank is None else rank
    world = dist.get_world_size(group) if world_size is None else world_size
    n = 0
    for parent in list(model.modules()):
        for cols, row in TP_BLOCKS:
            mods = [parent._modules.get(nm) for nm in cols + (row,)]
            if any(not isinstance(m, Linear4bit) for m in mods):
                continue
            if hasattr(parent, "head_dim") and cols[0] == "q_proj":
                hd = parent.head_dim
                for m in mods[:3]:
                    if (m.out_features // hd) % world != 0:
                        raise ValueError(f"{m.out_features // hd} heads do not split over {world} ranks")
            for nm in cols:
                parent._modules[nm] = RowShardedLinear4bit(parent._modules[nm], rank, world, group, local_matmul,
                                                           gather=False)
            parent._modules[row] = RowParallelLinear4bit(parent._modules[row], rank, world, group, local_matmul,
                                                         gatherer=gatherer)
            n += 1
    return n


def shard_model_linear4bit(model: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None,
                           group=None, local_matmul: Optional[Callable] = None, gatherer=None) -> nn.Module:
    """Replace every Linear4bit of `model` by its RowShardedLinear4bit (row split +
    all-gather: the north-star multi-GPU layout).  `gatherer`: the
    exchange every layer uses (None = dist.all_gather_into_tensor)."""
    from .modules import Linear4bit

    for name, child in list(model.named_children()):
        if isinstance(child, Linear4bit):
            model._modules[name] = RowShardedLinear4bit(child, rank, world_size, group, local_matmul,
                                                        gatherer=gatherer)
        else:
            shard_model_linear4bit(child, rank, world_size, group, local_matmul, gatherer)
    return model


def shard_attention_heads(model: nn.Module) -> int:
    """Head-sharded attention for the row-split layout (after shard_model_linear4bit): each attention
    module's q/k/v row shards ARE whole heads (rank p's rows [p*M/P, (p+1)*M/P) of q_proj are query
    heads [p*Hq/P, (p+1)*Hq/P), likewise for k/v and the kv heads), so they stay local (gather=False,
    no exchange) and the rank runs the attention of its own heads against a KV cache of only its kv
    heads (transformers takes the head count from the projection width; the StaticCache sizes its
    layers at the first update).  o_proj then gathers the heads' outputs (gather_input, rank-major =
    head order) before its row split and its usual exchange.  Per decoder layer: the q/k/v exchange
    becomes the attention-output exchange, and the replicated attention and KV cache shrink by P.
    Modules whose heads do not split evenly are left replicated.  Returns the number converted."""
    n = 0
    for mod in model.modules():
        projs = [mod._modules.get(nm) for nm in ("q_proj", "k_proj", "v_proj", "o_proj")]
        if any(not isinstance(m, RowShardedLinear4bit) for m in projs) or not hasattr(mod, "head_dim"):
            continue
        q, k, v, o = projs
        P, hd = q.world_size, int(mod.head_dim)
        if P == 1 or any(m.out_features % (hd * P) != 0 for m in (q, k, v)) or \
                not (q.gather and k.gather and v.gather) or o.in_features != q.out_features:
            continue
        for m in (q, k, v):
            m.gather = False
        o.gather_input = True
        n += 1
    return n


class RowShardedDenseLinear(nn.Module):
    """This rank's rows of an unquantised ``nn.Linear`` -- the lm_head, which transformers keeps in
    the model dtype (128256 rows: 1.05 GB for Llama-3-8B, 2.1 GB for 70B, replicated on every rank
    otherwise).  forward returns the FULL output on every rank: the local rows (one decode token on
    the GPU: layer_ops.gemv_dense; anything else F.linear), then the all-gather of the row-split
    layers.  Each output element is the same dot product as the unsharded layer's.  `dense_kernel`
    False keeps F.linear for the local rows too (the bench's --lm-head-library)."""

    def __init__(self, full: nn.Linear, rank: Optional[int] = None, world_size: Optional[int] = None,
                 group=None, gatherer=None, dense_kernel: bool = True):
        super().__init__()
        self.dense_kernel = dense_kernel
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world_size = dist.get_world_size(group) if world_size is None else world_size
        self.group, self.gatherer = group, gatherer
        M = full.out_features
        if M % self.world_size != 0:
            raise ValueError(f"out_features {M} is not divisible by world size {self.world_size}")
        rows = M // self.world_size
        self.r0, self.r1 = self.rank * rows, (self.rank + 1) * rows
        self.in_features, self.out_features = full.in_features, M
        self.register_buffer("weight", full.weight.data[self.r0:self.r1].contiguous().clone(), persistent=False)
        bias = None if full.bias is None else full.bias.data[self.r0:self.r1].clone()
        self.register_buffer("bias", bias, persistent=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .layer_ops import gemv_dense, gemv_dense_supported
        if self.dense_kernel and self.bias is None and gemv_dense_supported(x, self.weight):
            y = gemv_dense(x, self.weight)
        else:
            y = nn.functional.linear(x, self.weight, self.bias)
        return y if self.world_size == 1 else gather_rows(y, self.world_size, self.group, self.gatherer)


def shard_lm_head(model: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None, group=None,
                  gatherer=None, dense_kernel: bool = True) -> bool:
    """Replace the model's unquantised output projection with this rank's rows of it
    (RowShardedDenseLinear); False (nothing changed) where it is not an nn.Linear, its rows do
    not split evenly, or it is tied to the input embedding (tie_word_embeddings: the embedding
    stays whole, so nothing would be saved, and a later model.tie_weights() would put the full
    embedding Parameter back in place of the rank's rows)."""
    head = model.get_output_embeddings() if hasattr(model, "get_output_embeddings") else None
    world = dist.get_world_size(group) if world_size is None else world_size
    if not isinstance(head, nn.Linear) or world <= 1 or head.out_features % world != 0:
        return False
    emb = model.get_input_embeddings() if hasattr(model, "get_input_embeddings") else None
    if getattr(getattr(model, "config", None), "tie_word_embeddings", False) or \
            (emb is not None and getattr(emb, "weight", None) is head.weight):
        return False
    model.set_output_embeddings(RowShardedDenseLinear(head, rank, world, group, gatherer, dense_kernel))
    return True

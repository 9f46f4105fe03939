"""Row-sharded Linear4bit across GPUs (one process per GPU, RCCL all-gather).

The 4-bit layer is independent per output row, so rank p of P keeps rows
[p*M/P, (p+1)*M/P).  In the flat row-major layout that is a contiguous slice
of the packed bytes, of the per-block scales and (with double quant) of the
256-block second-level scales -- the GLOBAL quant state is sliced, never
re-quantised, so every rank's rows are bit-identical to the single-GPU layer.
x is replicated; after the local fused GEMV/GEMM the fp16 row shards are
exchanged with ``all_gather_into_tensor`` (RCCL over xGMI on MI355X, gloo in
the CPU tests).  The reference has no multi-GPU path; this is the build's
(SURVEY.md section 8e).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .core import QuantState


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


class RowShardedLinear4bit(nn.Module):
    """This rank's rows of a (quantised) ``Linear4bit``; forward returns the FULL
    output on every rank: local fused 4-bit matmul, then an all-gather."""

    def __init__(self, full: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None,
                 group=None, local_matmul: Optional[Callable] = None):
        super().__init__()
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

    def local_forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._local_matmul is not None:
            return self._local_matmul(x, self)
        from .core import gemm_4bit, gemv_4bit
        if x.numel() == x.shape[-1]:
            return gemv_4bit(x, self.packed, state=self.state, bias=self.bias, block_base=self.block_base)
        if self.block_base != 0:
            raise ValueError("prefill on a shard needs block-aligned second-level scales")
        return gemm_4bit(x, self.packed, self.state, bias=self.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        group = self.__dict__.get("_qz_group")
        if group is not None and x.numel() == x.shape[-1]:
            return group.take(self, x)
        y = self.local_forward(x)                       # [..., M/P]
        lead = y.shape[:-1]
        rows = y.shape[-1]
        y2 = y.reshape(-1, rows).contiguous()
        T = y2.shape[0]
        gathered = torch.empty((self.world_size * T, rows), dtype=y.dtype, device=y.device)
        dist.all_gather_into_tensor(gathered, y2, group=self.group)
        if T == 1:
            return gathered.reshape(*lead, self.world_size * rows)
        full = gathered.view(self.world_size, T, rows).permute(1, 0, 2).reshape(T, self.world_size * rows)
        return full.reshape(*lead, self.world_size * rows)


def sharded_group_compute(group, x: torch.Tensor):
    """Decode step of a DecodeGroup of RowShardedLinear4bit layers: ONE grouped
    local GEMV writes every member's row shard into one buffer, ONE all-gather
    exchanges it (instead of one all-gather per layer: bs=1 decode collectives
    are latency-bound), then each member's full output is cut out of the
    [world, sum(rows)] result."""
    from .core import gemv_4bit_grouped

    ms = group.members
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
        gemv_4bit_grouped(x, [(m.packed, m.state, m.bias, m.block_base, v) for m, v in zip(ms, views)])
    P = ms[0].world_size
    gathered = torch.empty(P * S, dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(gathered, buf, group=ms[0].group)
    g2 = gathered.view(P, S)
    lead = x.shape[:-1]
    outs, o = [], 0
    for r in rows:
        outs.append(g2[:, o:o + r].reshape(*lead, P * r))
        o += r
    return outs


def shard_model_linear4bit(model: nn.Module, rank: Optional[int] = None, world_size: Optional[int] = None,
                           group=None) -> nn.Module:
    """Replace every Linear4bit of `model` by its RowShardedLinear4bit."""
    from .modules import Linear4bit

    for name, child in list(model.named_children()):
        if isinstance(child, Linear4bit):
            model._modules[name] = RowShardedLinear4bit(child, rank, world_size, group)
        else:
            shard_model_linear4bit(child, rank, world_size, group)
    return model

"""``Linear4bit`` -- drop-in for ``bnb.nn.Linear4bit`` / the reference
``modules.Linear4bit`` (reference modules.py:67-151), inference only.

Dispatch (reference modules.py:28-64): a single-token input
(``A.numel() == A.shape[-1]``) runs the fused decode GEMV; anything else runs
the fused prefill GEMM (MFMA).  Both consume the 4-bit weight directly -- no
dequantised copy of W is ever materialised in HBM on the supported shapes.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from . import _lib
from .core import (MT_MAX_TOKENS, Params4bit, QuantState, dequantize_4bit, exact_codes_for, gemm_4bit,
                   gemm_4bit_grouped, gemv_4bit, gemv_4bit_grouped, gemv_4bit_pair_silu, grouped_tokens_ok)


def matmul_4bit(A: torch.Tensor, B: torch.Tensor, quant_state: QuantState, out: torch.Tensor = None, bias=None,
                exact_codes=None):
    """x . W^T (+ bias) for a 4-bit W (reference modules.py:28-64).  `B` is the packed
    weight (the reference passes ``weight.t()``; only its storage is used).
    `exact_codes` (decode only): see gemv_4bit; Linear4bit sets it from compute_dtype."""
    assert quant_state is not None
    if A.numel() == A.shape[-1]:
        return gemv_4bit(A, B, out, state=quant_state, bias=bias, exact_codes=exact_codes)
    return gemm_4bit(A, B, quant_state, bias=bias)


class DecodeGroup:
    """Linear4bit layers that read the same input (q/k/v or gate/up of one
    decoder layer), fused for decode into one grouped launch (SURVEY.md 8f
    row 2): one grouped GEMV for a single token, one grouped multi-token GEMM
    for a small batch of decode streams (2..16 tokens).  The first member
    called with a decode-shaped x computes every member's output; the others
    pick theirs up if they are called with the SAME tensor object (identity +
    version check, so a new or modified input always recomputes).  Prefill
    inputs (more tokens) bypass the group.  Built by
    ``integration.fuse_projection_groups``."""

    def __init__(self, members, compute):
        self.members = list(members)
        self._compute = compute          # (group, x) -> list of outputs, one per member
        self._x = None                   # weakref to the input the cached outputs belong to
        self._ver = -1
        self._outs = {}
        # (weight, eps, fn): the members' input is the input of this RMSNorm, absorbed into the
        # group by integration.fuse_prenorm (fn(x) = the norm as the model computed it)
        self.prenorm = None

    @staticmethod
    def accepts(x: torch.Tensor) -> bool:
        """Decode-shaped input: 1..MT_MAX_TOKENS tokens."""
        k = x.shape[-1]
        return k > 0 and 1 <= x.numel() // k <= MT_MAX_TOKENS

    @staticmethod
    def _version(x: torch.Tensor) -> int:
        # inference-mode tensors carry no version counter: identity alone keys them
        return -2 if x.is_inference() else x._version

    def take(self, member, x: torch.Tensor) -> torch.Tensor:
        key = id(member)
        ver = self._version(x)
        if self._x is None or self._x() is not x or self._ver != ver or key not in self._outs:
            outs = self._compute(self, x)
            self._outs = {id(m): o for m, o in zip(self.members, outs)}
            self._x = weakref.ref(x)
            self._ver = ver
        out = self._outs.pop(key)
        if not self._outs:
            self._x = None
        return out


def _linear4bit_group_compute(group: DecodeGroup, x: torch.Tensor):
    m0 = group.members[0]
    inp_dtype = x.dtype
    norm = group.prenorm
    fused_norm = (norm is not None and x.numel() == x.shape[-1] and m0._input(x) is x and x.is_cuda
                  and norm[0].dtype == x.dtype and norm[0].is_contiguous() and norm[0].numel() == x.shape[-1])
    if norm is not None and not fused_norm:
        x = norm[2](x)                   # the absorbed RMSNorm as its own launch
    xin = m0._input(x)
    items = []
    for m in group.members:
        bias = None if m.bias is None else m.bias.to(xin.dtype)
        items.append((m.weight, m.weight.quant_state, bias))
    if xin.numel() == xin.shape[-1]:
        outs = gemv_4bit_grouped(xin, items, exact_codes=exact_codes_for(m0.compute_dtype),
                                 norm=norm[:2] if fused_norm else None)
    elif grouped_tokens_ok(xin, items):
        outs = gemm_4bit_grouped(xin, items)
    else:  # shapes the multi-token kernel does not take: each member as it would run alone
        outs = [matmul_4bit(xin, w, bias=b, quant_state=st, exact_codes=exact_codes_for(m0.compute_dtype))
                for w, st, b in items]
    return [o if o.dtype == inp_dtype else o.to(inp_dtype) for o in outs]


def linear4bit_silu_pair(group: DecodeGroup, x: torch.Tensor):
    """act_fn(gate_proj(x)) * up_proj(x) for a decode group of exactly (gate_proj, up_proj) and a
    single token, in one launch (core.gemv_4bit_pair_silu; an RMSNorm absorbed by fuse_prenorm
    is applied inside too).  None when that launch does not take the case: the caller then calls
    the members (the grouped launch) and multiplies."""
    if group._compute is not _linear4bit_group_compute or len(group.members) != 2:
        return None
    if not (x.is_cuda and x.numel() == x.shape[-1] and x.dtype in (torch.float16, torch.bfloat16)):
        return None
    for m in group.members:
        if m.weight.quant_state is None:
            return None
        if not m.compute_type_is_set:
            m.set_compute_type(x)
            m.compute_type_is_set = True
    m0, m1 = group.members
    if m0._input(x) is not x or m1._input(x) is not x or \
            exact_codes_for(m0.compute_dtype) != exact_codes_for(m1.compute_dtype):
        return None
    norm = group.prenorm
    items = [(m.weight, m.weight.quant_state, None if m.bias is None else m.bias.to(x.dtype)) for m in group.members]
    return gemv_4bit_pair_silu(x, items, exact_codes=exact_codes_for(m0.compute_dtype),
                               norm=None if norm is None else norm[:2])


class Linear4bit(nn.Linear):
    """4-bit linear layer with the bnb / reference constructor signature
    (reference modules.py:86-96).  ``quant_type`` is "fp4" or "nf4";
    ``compress_statistics`` toggles double quantisation of the absmax."""

    def __init__(self, input_features, output_features, bias=False, compute_dtype=None, compress_statistics=True,
                 quant_type="fp4", quant_storage=torch.uint8, device=None):
        super().__init__(input_features, output_features, bias, device)
        self.weight = Params4bit(self.weight.data, requires_grad=False, quant_type=quant_type,
                                 quant_storage=quant_storage, module=self, compress_statistics=compress_statistics)
        self.compute_dtype = compute_dtype
        self.compute_type_is_set = False
        self.quant_state = None
        self.quant_storage = quant_storage

    def set_compute_type(self, x):
        """Reference modules.py:112-122: fp32/bf16 inputs select their own dtype."""
        if x.dtype in [torch.float32, torch.bfloat16]:
            self.compute_dtype = x.dtype

    def _input(self, x: torch.Tensor) -> torch.Tensor:
        # The reference casts x to compute_dtype before the matmul (modules.py:141-142).
        # Our kernels always accumulate in fp32, so an up-cast (e.g. fp16 -> fp32) is
        # exact and skipped; a narrowing cast (e.g. fp16 -> bf16) changes values and
        # is applied to keep the reference's numerics.
        cd = self.compute_dtype
        if cd is None or cd == x.dtype or cd == torch.float32:
            return x
        return x.to(cd)

    def forward(self, x: torch.Tensor):
        if not self.compute_type_is_set:
            self.set_compute_type(x)
            self.compute_type_is_set = True
        qs = self.weight.quant_state
        if qs is None:
            raise RuntimeError("Linear4bit weight is not quantised yet: move the module to a GPU first")
        group = self.__dict__.get("_qz_group")
        if group is not None and group.accepts(x):
            return group.take(self, x)
        if group is not None and group.prenorm is not None:
            x = group.prenorm[2](x)      # prefill through a group that absorbed its RMSNorm
        inp_dtype = x.dtype
        xin = self._input(x)
        bias = None if self.bias is None else self.bias.to(xin.dtype)
        out = matmul_4bit(xin, self.weight, bias=bias, quant_state=qs,
                          exact_codes=exact_codes_for(self.compute_dtype))
        return out if out.dtype == inp_dtype else out.to(inp_dtype)

    def forward_residual(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """residual + self(x) -- LlamaDecoderLayer's `residual + h` after o_proj / down_proj --
        with the add in the decode GEMV's epilogue (one launch, bit-identical to the torch
        add) when x is a single token this layer decodes on its own; otherwise the two ops."""
        qs = self.weight.quant_state
        if (qs is not None and x.is_cuda and x.numel() == x.shape[-1] and self.__dict__.get("_qz_group") is None
                and residual.dtype == x.dtype and residual.device == x.device and residual.is_contiguous()
                and residual.numel() == qs.shape[0] and residual.shape[:-1] == x.shape[:-1]):
            if not self.compute_type_is_set:
                self.set_compute_type(x)
                self.compute_type_is_set = True
            if self._input(x) is x:
                bias = None if self.bias is None else self.bias.to(x.dtype)
                return gemv_4bit(x, self.weight, state=qs, bias=bias, exact_codes=exact_codes_for(self.compute_dtype),
                                 residual=residual)
        return residual + self(x)

    # -- checkpoints: bnb-compatible keys (QuantState.as_dict(packed=True)) --
    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        qs = self.weight.quant_state
        if qs is None:
            return  # not quantised yet: the plain float weight is saved
        w = self.weight
        destination[prefix + "weight"] = w if keep_vars else w.data.detach()
        for k, v in qs.as_dict(packed=True).items():
            destination[prefix + "weight." + k] = v if keep_vars else v.detach()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        wkey = prefix + "weight"
        stats = {k[len(wkey) + 1:]: v for k, v in state_dict.items() if k.startswith(wkey + ".")}
        if not stats or wkey not in state_dict:  # float checkpoint: quantised on .to(cuda)
            super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                          unexpected_keys, error_msgs)
            return
        data = state_dict[wkey]
        dev = self.weight.device if self.weight.device.type != "meta" else data.device
        self.weight = Params4bit.from_prequantized(data, stats, requires_grad=False, device=dev, module=self)
        rest = {k: v for k, v in state_dict.items() if k != wkey and not k.startswith(wkey + ".")}
        n_missing = len(missing_keys)
        super()._load_from_state_dict(rest, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)
        missing_keys[n_missing:] = [k for k in missing_keys[n_missing:] if k != wkey]

    def dequantize(self) -> torch.Tensor:
        """Dense weight [out, in] in the original dtype (for checks and export)."""
        return dequantize_4bit(self.weight, self.weight.quant_state).t()

    @property
    def native_lib(self) -> str:
        return _lib.LIB_PATH

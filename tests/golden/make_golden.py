"""Generate the committed golden fixtures under tests/golden/.

Two kinds of vectors:

1. ``reference_*`` -- produced by importing the reference Python
   (/root/reference/core.py) with a stand-in ``kbkim_lib`` module:
   * ``reference_tables.npz``: ``create_dynamic_map()`` (core.py:251-314) and
     ``get_4bit_type("fp4")`` (core.py:193-229) exactly as the reference builds
     them.
   * ``reference_calls.json``: the native-call sequence and integer arguments
     the reference host code issues for decode (``gemv_4bit``), prefill
     (``dequantize_4bit``) and double quant (``quantize_blockwise``), recorded
     by a stub that logs every ``kbkim_lib.*`` call (pointers are replaced by
     the name of the tensor they point into).
   * ``reference_pipeline.npz``: the reference's own host orchestration
     (core.py:426-504, 581-634, 317-366, 369-423 and the steps of 507-578)
     executed on CPU tensors with ``kbkim_lib`` backed by the C oracle -- this
     pins the composition (offset = mean, ``absmax -= offset``, DQ blocksize
     256, ``absmax += offset``, GEMV argument marshalling, transposes).

2. ``oracle_*`` -- seeded weights quantised by the C oracle (FP4 and NF4,
   with and without double quant) used by the GPU parity tests as committed
   data.  NF4 decision boundaries are build-defined ("parity unpinned").

The reference never travels to the GPU box: only these data files do.
Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

import oracle  # noqa: E402

# ----------------------------------------------------------------------------
# stand-in kbkim_lib: records calls and (optionally) forwards to the oracle
# ----------------------------------------------------------------------------
_tensors: dict[int, str] = {}
_calls: list = []
_forward = False


def _label(ptr: int) -> str:
    if ptr == 0:
        return "NULL"
    for base, name in _tensors.items():
        if base == ptr:
            return name
    return "?"


def _arr(ptr, n, ct):
    return np.ctypeslib.as_array((ct * n).from_address(ptr))


def _rec(name, args, kinds):
    _calls.append([name] + [(_label(a) if k == "p" else a) for a, k in zip(args, kinds)])


def cgemm_4bit_inference_naive_fp32(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize):
    _rec("cgemm_4bit_inference_naive_fp32", (m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize),
         "iiipppppiiii")
    if _forward:
        x = _arr(A, k, ctypes.c_float)
        packed = _arr(B, (m * k + 1) // 2, ctypes.c_uint8)
        am = _arr(absmax, (m * k + blocksize - 1) // blocksize, ctypes.c_float)
        lut = _arr(datatype, 16, ctypes.c_float)
        _arr(out, m, ctypes.c_float)[:] = oracle.gemv_4bit(x, packed, am, lut, m, k, blocksize).astype(np.float32)


def cquantize_blockwise_fp32(code, A, absmax, out, blocksize, n):
    _rec("cquantize_blockwise_fp32", (code, A, absmax, out, blocksize, n), "ppppii")
    if _forward:
        q, am = oracle.quantize_blockwise_8bit(_arr(code, 256, ctypes.c_float), _arr(A, n, ctypes.c_float), blocksize)
        _arr(out, n, ctypes.c_uint8)[:] = q
        _arr(absmax, am.size, ctypes.c_float)[:] = am


def cdequantize_blockwise_fp32(code, A, absmax, out, blocksize, n):
    _rec("cdequantize_blockwise_fp32", (code, A, absmax, out, blocksize, n), "ppppii")
    if _forward:
        nb = (n + blocksize - 1) // blocksize
        _arr(out, n, ctypes.c_float)[:] = oracle.dequantize_blockwise_8bit(
            _arr(code, 256, ctypes.c_float), _arr(A, n, ctypes.c_uint8), _arr(absmax, nb, ctypes.c_float), blocksize)


def cquantize_blockwise_fp16_fp4(code, A, absmax, out, blocksize, n):
    _rec("cquantize_blockwise_fp16_fp4", (code, A, absmax, out, blocksize, n), "ppppii")
    if _forward:
        w = _arr(A, n, ctypes.c_uint16).view(np.float16).astype(np.float32)
        packed, am = oracle.quantize_4bit_raw(w, blocksize, "fp4")
        _arr(out, packed.size, ctypes.c_uint8)[:] = packed
        _arr(absmax, am.size, ctypes.c_float)[:] = am


def cdequantize_blockwise_fp16_fp4(code, A, absmax, out, blocksize, n):
    _rec("cdequantize_blockwise_fp16_fp4", (code, A, absmax, out, blocksize, n), "ppppii")
    if _forward:
        nb = (n + blocksize - 1) // blocksize
        w = oracle.dequantize_4bit(_arr(A, (n + 1) // 2, ctypes.c_uint8), _arr(absmax, nb, ctypes.c_float), n,
                                   blocksize, "fp4")
        _arr(out, n, ctypes.c_uint16)[:] = w.astype(np.float16).view(np.uint16)


def _install_stub():
    m = types.ModuleType("kbkim_lib")
    for f in (cgemm_4bit_inference_naive_fp32, cquantize_blockwise_fp32, cdequantize_blockwise_fp32,
              cquantize_blockwise_fp16_fp4, cdequantize_blockwise_fp16_fp4):
        setattr(m, f.__name__, f)
    sys.modules["kbkim_lib"] = m
    sys.path.insert(0, REF)
    import core as ref_core  # noqa: E402  (reference, read-only, no bytecode written)
    return ref_core


def _track(**named):
    for name, t in named.items():
        _tensors[t.data_ptr()] = name


def main():
    assert os.environ.get("PYTHONDONTWRITEBYTECODE") == "1", "run with PYTHONDONTWRITEBYTECODE=1"
    global _forward
    ref = _install_stub()
    oracle.build()

    # ---- 1. tables ---------------------------------------------------------
    dyn = ref.create_dynamic_map().numpy().astype(np.float32)
    fp4 = ref.get_4bit_type("fp4", device="cpu").numpy().astype(np.float32)
    np.savez(os.path.join(HERE, "reference_tables.npz"), dynamic_map=dyn, fp4_lut=fp4)

    # ---- 2. call marshalling for the headline shape (4096x4096) --------------
    calls = {}
    M, K = 4096, 4096
    n = M * K
    nb = n // 64
    qs2 = ref.QuantState(absmax=torch.zeros((nb + 255) // 256), code=torch.tensor(dyn), blocksize=256,
                         dtype=torch.float32)
    qs = ref.QuantState(absmax=torch.zeros(nb, dtype=torch.uint8), shape=torch.Size([M, K]), code=torch.tensor(fp4),
                        blocksize=64, quant_type="fp4", dtype=torch.float16, offset=torch.tensor(0.0), state2=qs2)
    B = torch.zeros(((n + 1) // 2, 1), dtype=torch.uint8)
    x = torch.zeros((1, 1, K), dtype=torch.float32)
    _track(B=B, x=x, qabsmax=qs.absmax, absmax2=qs2.absmax, code2=qs2.code, code=qs.code)
    _calls.clear()
    ref.gemv_4bit(x, B.t(), state=qs)
    calls["decode_gemv_4096x4096"] = list(_calls)
    _calls.clear()
    ref.dequantize_4bit(B, qs)
    calls["prefill_dequant_4096x4096"] = list(_calls)
    _calls.clear()
    a = torch.zeros(nb, dtype=torch.float32)
    _track(absmax_minus_offset=a)
    ref.quantize_blockwise(a, blocksize=256)
    calls["double_quant_4096x4096"] = list(_calls)
    with open(os.path.join(HERE, "reference_calls.json"), "w") as f:
        json.dump(calls, f, indent=1)

    # ---- 3. reference orchestration on the oracle ----------------------------
    _forward = True
    pipe = {}
    for tag, (M, K, seed) in {"a": (64, 512, 0), "b": (24, 320, 1)}.items():
        g = torch.Generator().manual_seed(seed)
        W = (torch.randn(M, K, generator=g) * 0.02).to(torch.float16)
        xh = torch.randn(1, 1, K, generator=g).to(torch.float16)
        n = M * K
        nb = (n + 63) // 64
        absmax = torch.zeros(nb, dtype=torch.float32)
        packed = torch.zeros(((n + 1) // 2, 1), dtype=torch.uint8)
        # core.py:552-559 (the kernel), then 563-565 (torch mean, subtract, DQ) -- the reference's own steps
        cquantize_blockwise_fp16_fp4(0, W.data_ptr(), absmax.data_ptr(), packed.data_ptr(), 64, n)
        absmax_raw = absmax.clone()
        offset = absmax.mean()
        absmax -= offset
        qabsmax, state2 = ref.quantize_blockwise(absmax, blocksize=256)
        st = ref.QuantState(absmax=qabsmax, shape=W.shape, dtype=W.dtype, blocksize=64,
                            code=ref.get_4bit_type("fp4", device="cpu"), quant_type="fp4", offset=offset,
                            state2=state2)
        y = ref.gemv_4bit(xh.to(torch.float32), packed.t(), state=st)          # modules.py:58 path
        wdeq_t = ref.dequantize_4bit(packed, st)                                # modules.py:64 path
        pipe.update({
            f"{tag}_W": W.view(torch.int16).numpy(), f"{tag}_x": xh.view(torch.int16).numpy(),
            f"{tag}_packed": packed.numpy().ravel(), f"{tag}_absmax_raw": absmax_raw.numpy(),
            f"{tag}_offset_torch_mean": np.float32(offset.item()), f"{tag}_qabsmax": qabsmax.numpy(),
            f"{tag}_absmax2": state2.absmax.numpy(), f"{tag}_y": y.numpy().ravel(),
            f"{tag}_wdeq": wdeq_t.t().contiguous().view(torch.int16).numpy(),
            f"{tag}_shape": np.array([M, K]),
        })
    np.savez(os.path.join(HERE, "reference_pipeline.npz"), **pipe)
    _forward = False

    # ---- 4. oracle vectors for GPU parity (FP4/NF4 x DQ) ----------------------
    ov = {}
    for qt in ("fp4", "nf4"):
        for (M, K, seed) in ((128, 1024, 11), (40, 2112, 12)):
            g = torch.Generator().manual_seed(seed)
            W = (torch.randn(M, K, generator=g) * 0.02).to(torch.float16)
            x = torch.randn(K, generator=g).to(torch.float16)
            st = oracle.quantize_4bit(W.float().numpy(), 64, qt, double_quant=True)
            key = f"{qt}_{M}x{K}"
            ov.update({
                f"{key}_W": W.view(torch.int16).numpy(), f"{key}_x": x.view(torch.int16).numpy(),
                f"{key}_packed": st.packed, f"{key}_absmax_raw": st.absmax_raw, f"{key}_offset": st.offset,
                f"{key}_qabsmax": st.qabsmax, f"{key}_absmax2": st.absmax2,
                f"{key}_y": oracle.gemv(x.float().numpy(), st),
                f"{key}_wdeq16": oracle.dequantize(st).astype(np.float16).view(np.int16),
            })
    np.savez_compressed(os.path.join(HERE, "oracle_vectors.npz"), **ov)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()

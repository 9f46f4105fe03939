"""GPU: edge cases of the Linear4bit path against the oracle, and the opt-in
dequant + qz_gemm_16bit prefill route.

* Ragged shapes: in_features not a multiple of the blocksize (scale blocks run
  across rows, as in the reference's flat blockwise quantiser, kernels.cu:431),
  odd out_features, and token counts on every route boundary (1 = GEMV,
  2..16 = multi-token kernel, 17..512 = fused tile kernel, > 512 = dequant +
  library GEMM); checked against the oracle's dequantised weight (oracle.c,
  pinned in test_oracle.py) in fp64.
* Empty batches: zero tokens in, an empty [..., out_features] tensor out.
* gemm_4bit(route="gemm16"): our dense 16-bit GEMM after the bit-exact dequant,
  ragged T and M tiles, bias, fp16 and bf16, vs fp64.
Bars are the file-wide ones: 1e-3 relative (north_star) via assert_close.
"""
import numpy as np
import pytest
import torch

from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _layer(orc, in_f, out_f, quant_type, dq, seed, dtype=torch.float16):
    import quantizations_amd as qa

    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(out_f, in_f, generator=g) * 0.02).to(dtype)
    m = qa.Linear4bit(in_f, out_f, bias=True, quant_type=quant_type, compress_statistics=dq, compute_dtype=dtype)
    m.weight = qa.Params4bit(W, requires_grad=False, quant_type=quant_type, module=m, compress_statistics=dq)
    b = (torch.randn(out_f, generator=g) * 0.1).to(dtype)
    m.bias = torch.nn.Parameter(b, requires_grad=False)
    m = m.to(DEV)
    o = orc.quantize_4bit(W.float().numpy(), 64, quant_type, double_quant=dq)
    wref = torch.from_numpy(orc.dequantize(o)).double().reshape(out_f, in_f)
    return m, wref, b.double()


@pytest.mark.parametrize("in_f,out_f", [(100, 3), (72, 130), (4100, 24), (320, 1000)])
@pytest.mark.parametrize("T", [1, 5, 40, 600])
def test_linear4bit_ragged_shapes_all_routes(orc, in_f, out_f, T):
    m, wref, b = _layer(orc, in_f, out_f, "nf4", True, seed=in_f + out_f + T)
    X = torch.randn(1, T, in_f, generator=torch.Generator().manual_seed(T)).half()
    y = m(X.to(DEV))
    assert y.shape == (1, T, out_f) and y.dtype == torch.float16
    ref = X.double().reshape(T, in_f) @ wref.t() + b
    assert_close(y.float().cpu().reshape(T, out_f), ref.numpy(), torch.float16, f"{in_f}x{out_f} T={T}")


@pytest.mark.parametrize("quant_type,dq", [("fp4", False), ("nf4", False), ("fp4", True)])
def test_linear4bit_ragged_codebooks(orc, quant_type, dq):
    m, wref, b = _layer(orc, 200, 36, quant_type, dq, seed=7)
    for T in (1, 3, 33):
        X = torch.randn(T, 200, generator=torch.Generator().manual_seed(T)).half()
        ref = X.double() @ wref.t() + b
        assert_close(m(X.to(DEV)).float().cpu(), ref.numpy(), torch.float16, f"{quant_type} dq={dq} T={T}")


@pytest.mark.parametrize("shape", [(0, 256), (2, 0, 256), (0, 0, 256)])
def test_linear4bit_empty_batch(orc, shape):
    m, _, _ = _layer(orc, 256, 64, "nf4", True, seed=3)
    y = m(torch.empty(*shape, dtype=torch.float16, device=DEV))
    assert y.shape == (*shape[:-1], 64) and y.dtype == torch.float16


def test_gemv_and_gemm_empty_and_single_row(orc):
    from quantizations_amd.core import gemm_4bit, gemv_4bit, quantize_4bit

    W = (torch.randn(8, 256, generator=torch.Generator().manual_seed(5)) * 0.02).half()
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    assert gemm_4bit(torch.empty(0, 256, dtype=torch.float16, device=DEV), packed, st).shape == (0, 8)
    o = orc.quantize_4bit(W.float().numpy(), 64, "nf4")
    wref = torch.from_numpy(orc.dequantize(o)).double().reshape(8, 256)
    x = torch.randn(1, 256, generator=torch.Generator().manual_seed(6)).half()
    y = gemv_4bit(x.to(DEV), packed, state=st)
    assert_close(y.float().cpu().reshape(-1), (wref @ x.double().reshape(-1)).numpy(), torch.float16, "M=8 GEMV")


def _gemm16_case(T, M, K, dtype, bias, seed):
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, quantize_4bit

    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(M, K, generator=g) * 0.02).to(dtype).to(DEV)
    packed, st = quantize_4bit(W, quant_type="nf4")
    wd = dequantize_4bit(packed, st, out_dtype=dtype).t().double()       # [M, K], bit-exact to the oracle
    X = torch.randn(T, K, device=DEV, generator=torch.Generator(device="cuda").manual_seed(seed)).to(dtype)
    bv = (torch.randn(M, device=DEV) * 0.1).to(dtype) if bias else None
    y = gemm_4bit(X, packed, st, bias=bv, route="gemm16")
    ref = X.double() @ wd.t() + (bv.double() if bias else 0.0)
    return y, ref


@pytest.mark.parametrize("T,M", [(4096, 1024), (4100, 1032), (300, 264)])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gemm16_route_vs_fp64(T, M, dtype):
    """dequantize_4bit (bit-exact) + qz_gemm_16bit: 256 x 256 tiles with ragged T and M edges."""
    y, ref = _gemm16_case(T, M, 4096, dtype, bias=True, seed=T + M)
    assert y.shape == (T, M) and y.dtype == dtype
    rel = ((y.double() - ref).norm() / ref.norm()).item()
    assert rel <= (1e-3 if dtype == torch.float16 else 4e-3), f"rel err {rel:.3e}"
    ulp = 2.0 ** (-10 if dtype == torch.float16 else -7)
    worst = ((y.double() - ref).abs() - (1e-3 * ref.abs().max() + ulp * ref.abs())).max().item()
    assert worst <= 0, f"elementwise bound exceeded by {worst:.3e}"


@pytest.mark.parametrize("T,M,K", [(37, 264, 64), (300, 520, 128), (257, 1032, 192), (1, 8, 64)])
def test_gemm16_short_k_loops(T, M, K):
    """qz_gemm_16bit with 1-, 2- and 3-step K loops (K = 64 / 128 / 192; the prologue and the
    last steps of the 8-phase schedule) and ragged T / M."""
    y, ref = _gemm16_case(T, M, K, torch.float16, bias=True, seed=T * M + K)
    assert y.shape == (T, M)
    worst = ((y.double() - ref).abs() - (1e-3 * ref.abs().max() + 2.0 ** -10 * ref.abs())).max().item()
    assert worst <= 0, f"elementwise bound exceeded by {worst:.3e}"


def test_gemm16_route_rejects_unsupported_shape():
    """route='gemm16' raises where qz_gemm_16bit does not apply (M % 8 != 0) instead of
    silently running the library GEMM; route='auto' takes the library GEMM there."""
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    W = (torch.randn(1028, 256, device=DEV) * 0.02).half()
    packed, st = quantize_4bit(W, quant_type="nf4")
    X = torch.randn(300, 256, device=DEV).half()
    with pytest.raises(ValueError):
        gemm_4bit(X, packed, st, route="gemm16")
    y = gemm_4bit(X, packed, st, route="auto")
    assert y.shape == (300, 1028) and torch.isfinite(y).all()


def test_gemm16_matches_library_route():
    """The two dequant routes multiply the same operand: gemm16 vs the library GEMM."""
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    W = (torch.randn(2048, 4096, device=DEV) * 0.02).half()
    packed, st = quantize_4bit(W, quant_type="nf4")
    X = torch.randn(4096, 4096, device=DEV).half()
    a = gemm_4bit(X, packed, st, route="gemm16").double()
    b = gemm_4bit(X, packed, st, route="blas").double()
    assert ((a - b).norm() / b.norm()).item() < 1e-3
    assert torch.isfinite(a).all()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,K", [(100, 3 * 64), (37, 100), (256, 2112), (1024, 4160), (64, 8192), (4096, 1024),
                                 (8192, 8192), (28672, 8192)])
@pytest.mark.parametrize("qt,dq", [("nf4", True), ("fp4", False)])
def test_gemv_bf16_fp32_tables_on_every_geometry(orc, dt, M, K, qt, dq):
    """The bf16 / fp32 code tables on every GEMV geometry: K not a multiple of 2048 (the
    generic step loads), small M (K split over 2-4 waves), ragged K (the scalar kernel), the
    Llama-3-70B rows of 8192 (R = 4, WK = 2), FP4 without and NF4 with double quant, single
    and grouped launches -- against the oracle's fp32 weight products."""
    from quantizations_amd.core import gemv_4bit, gemv_4bit_grouped, quantize_4bit

    g = torch.Generator().manual_seed(M + K)
    W = (torch.randn(M, K, generator=g) * 0.02).half()
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=dq)
    o = orc.quantize_4bit(W.float().numpy(), 64, qt, double_quant=dq)
    x = torch.randn(K, generator=g).to(dt)
    yref = orc.gemv(x.float().numpy(), o)
    y = gemv_4bit(x.to(DEV).reshape(1, K), packed, state=st).double().cpu().numpy().ravel()
    # the grouped launch (the R = 4, WK = 2 K-split geometry at K = 8192) returns the same outputs
    (yg,) = gemv_4bit_grouped(x.to(DEV).reshape(1, K), [(packed, st, None)])
    assert np.array_equal(yg.double().cpu().numpy().ravel(), y)
    tol = 2.0 ** -8 if dt == torch.bfloat16 else 1e-5
    rel = float(np.linalg.norm(y - yref) / np.linalg.norm(yref))
    assert rel <= tol, (rel, dt, M, K, qt)

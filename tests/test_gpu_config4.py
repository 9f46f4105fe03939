"""GPU: BASELINE config #4 at its real size -- Llama-3-8B NF4 (double quant)
prefill of 8 x 2048 tokens (T = 16384) through the three distinct Linear4bit
shapes -- and the prefill route boundary (T = 513, 2048).

Both prefill routes are checked against an on-device fp64 product of the
bit-exact dequantised fp16 weight (dequantize_4bit is pinned to the oracle bit
for bit in test_gpu_parity; the oracle itself is too slow for 2e14 FLOP):
  * Linear4bit.forward in its default (auto) mode, i.e. modules.py:62-64's
    `F.linear(A, dequantize_4bit(W).t())` as the product routes it;
  * gemm_4bit(route="fused"): the hand-written MFMA kernel (256 x 256 tile at
    T >= 4096, 128-row tile below);
  * gemm_4bit(route="gemm16"): the bit-exact dequant, then qz_gemm_16bit (its default
    schedule, the persistent k_gemm16_4q) -- the hand-written replacement for the library GEMM.
Bar: ||y - y_ref|| / ||y_ref|| <= 1e-3 and |y - y_ref| <= 1e-3 max|y_ref| + 1 ulp
(fp16), as everywhere else.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _assert_close_dev(y: torch.Tensor, ref: torch.Tensor, what: str):
    y = y.reshape(ref.shape).double()
    rel = ((y - ref).norm() / ref.norm()).item()
    assert rel <= 1e-3, f"{what}: rel err {rel:.3e}"
    bound = 1e-3 * ref.abs().max() + (2.0 ** -10) * ref.abs()
    worst = ((y - ref).abs() - bound).max().item()
    assert worst <= 0, f"{what}: elementwise bound exceeded by {worst:.3e}"
    assert torch.isfinite(y).all()


def _layer(M, K, seed):
    import quantizations_amd as qa

    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(M, K, generator=g) * 0.02).half()
    m = qa.Linear4bit(K, M, bias=False, quant_type="nf4", compress_statistics=True)
    m.weight = qa.Params4bit(W, requires_grad=False, quant_type="nf4", module=m, compress_statistics=True)
    m = m.to(DEV)
    wd = qa.dequantize_4bit(m.weight, m.weight.quant_state).t()   # [M, K] fp16, bit-exact to the oracle
    return m, wd


@pytest.mark.parametrize("M,K", [(4096, 4096), (14336, 4096), (4096, 14336)])
def test_config4_prefill_T16384_both_routes(M, K):
    from quantizations_amd.core import fused_max_tokens, gemm_4bit

    m, wd = _layer(M, K, seed=M + K)
    g = torch.Generator(device="cuda").manual_seed(2)
    X = torch.randn(8, 2048, K, device=DEV, generator=g).half()     # seq 2048 x batch 8
    ref = X.reshape(-1, K).double() @ wd.double().t()               # [16384, M] fp64
    y_auto = m(X)                                                   # product route (modules.py:62-64)
    assert y_auto.shape == (8, 2048, M) and y_auto.dtype == torch.float16
    assert 16384 > fused_max_tokens(M)                              # auto = dequant + library GEMM here
    _assert_close_dev(y_auto.reshape(-1, M), ref, f"Linear4bit auto {M}x{K}")
    del y_auto
    y_fused = gemm_4bit(X, m.weight, m.weight.quant_state, route="fused")   # 256 x 256 MFMA tile kernel
    assert y_fused.shape == (8, 2048, M)
    _assert_close_dev(y_fused.reshape(-1, M), ref, f"fused {M}x{K}")
    del y_fused
    y16 = gemm_4bit(X, m.weight, m.weight.quant_state, route="gemm16")   # dequant + k_gemm16_4q
    assert y16.shape == (8, 2048, M)
    _assert_close_dev(y16.reshape(-1, M), ref, f"gemm16 {M}x{K}")


@pytest.mark.parametrize("T", [513, 2048])
@pytest.mark.parametrize("M,K", [(4096, 4096), (1024, 4096)])
def test_linear4bit_prefill_above_fused_threshold(T, M, K):
    """Linear4bit's auto route above the fused crossover (fused_max_tokens: 256 / 128) and at
    one sequence of config #4 (2048), and the fused kernel at the same T."""
    from quantizations_amd.core import gemm_4bit

    m, wd = _layer(M, K, seed=T + M)
    X = torch.randn(1, T, K, device=DEV, generator=torch.Generator(device="cuda").manual_seed(T)).half()
    ref = X.reshape(T, K).double() @ wd.double().t()
    _assert_close_dev(m(X).reshape(T, M), ref, f"Linear4bit auto T={T}")
    _assert_close_dev(gemm_4bit(X, m.weight, m.weight.quant_state, route="fused").reshape(T, M), ref,
                      f"fused T={T}")

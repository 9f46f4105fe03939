"""GPU parity: the HIP kernels (through the C-ABI) against the CPU oracle and the
committed golden vectors.

Bars (DESIGN.md "Parity"):
  * 4-bit codes, 8-bit double-quant codes, absmax, absmax2, offset: bit-exact.
  * dequantised weights (fp16/bf16/fp32 stores of fp32 products): bit-exact.
  * GEMV / GEMM outputs: ||y - y_ref||_2 / ||y_ref||_2 <= 1e-3 and
    |y - y_ref| <= 1e-3 * max|y_ref| + 1 ulp(out dtype), y_ref = fp64 sum of the
    reference's fp32 weight products (oracle.gemv) -- SURVEY.md appendix A.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")
REL_TOL = 1e-3


def _w(M, K, seed=0, dtype=torch.float16, scale=0.02):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(M, K, generator=g) * scale).to(dtype)


def _x(K, seed=1, dtype=torch.float16):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(K, generator=g).to(dtype)


def _ulp(dtype):
    return {torch.float16: 2.0 ** -10, torch.bfloat16: 2.0 ** -7, torch.float32: 2.0 ** -23}[dtype]


def assert_close(y, yref, dtype, what=""):
    """1e-3 relative (north_star) on the fp32-accumulated result.  A bf16 output
    cannot carry 1e-3 (its own rounding is up to 2^-9, and an fp32 result a
    hair away from the reference's may round to the other bf16 neighbour), so
    for bf16 the norm bar applies after removing the output format's own
    1-ulp rounding from each element."""
    y = np.asarray(y, np.float64).ravel()
    yref = np.asarray(yref, np.float64).ravel()
    if dtype == torch.bfloat16:
        d = y - yref
        ulp = np.exp2(np.floor(np.log2(np.maximum(np.abs(yref), 1e-30))) - 7)
        rel = np.linalg.norm(np.sign(d) * np.maximum(np.abs(d) - ulp, 0)) / max(np.linalg.norm(yref), 1e-30)
        yref = torch.from_numpy(yref).to(torch.bfloat16).double().numpy()
    else:
        rel = np.linalg.norm(y - yref) / max(np.linalg.norm(yref), 1e-30)
    assert rel <= REL_TOL, f"{what}: rel err {rel:.3e}"
    bound = 1e-3 * np.max(np.abs(yref)) + _ulp(dtype) * np.abs(yref) + 1e-30
    worst = np.max(np.abs(y - yref) - bound)
    assert worst <= 0, f"{what}: elementwise bound exceeded by {worst:.3e}"


# ---------------------------------------------------------------------------
# quantisation: bit-exact
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("qt", ["fp4", "nf4"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,bs", [((128, 1024), 64), ((40, 2112), 64), ((3, 37), 64), ((257, 33), 128),
                                      ((64, 1024), 256), ((16, 4096), 1024), ((8, 8192), 4096)])
def test_quantize_4bit_bit_exact(orc, qt, dtype, shape, bs):
    from quantizations_amd.core import quantize_4bit

    W = _w(*shape, seed=shape[0] + 7 * shape[1] + bs + (qt == "nf4"), dtype=dtype)
    packed, st = quantize_4bit(W.to(DEV), blocksize=bs, quant_type=qt, compress_statistics=True)
    o = orc.quantize_4bit(W.float().numpy(), bs, qt, double_quant=True)
    assert np.array_equal(packed.cpu().numpy().ravel(), o.packed)
    assert float(st.offset) == float(o.offset) and st.offset.dtype == torch.float32
    assert np.array_equal(st.absmax.cpu().numpy(), o.qabsmax)
    assert np.array_equal(st.state2.absmax.cpu().numpy().view(np.uint32), o.absmax2.view(np.uint32))
    p2, st_nodq = quantize_4bit(W.to(DEV), blocksize=bs, quant_type=qt, compress_statistics=False)
    assert np.array_equal(p2.cpu().numpy().ravel(), o.packed)
    assert np.array_equal(st_nodq.absmax.cpu().numpy().view(np.uint32), o.absmax_raw.view(np.uint32))


def test_quantize_edge_values(orc):
    from quantizations_amd.core import quantize_4bit

    W = _w(4, 256, seed=5)
    W[0, :64] = 0                   # all-zero block
    W[1, 5] = float("nan")          # NaN ignored by absmax
    W[2, 0] = 65504.0               # fp16 max
    W[3, 64:] = -W[3, 64:].abs()    # negative-only blocks
    for qt in ("fp4", "nf4"):
        packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=False)
        o = orc.quantize_4bit(W.float().numpy(), 64, qt, double_quant=False)
        assert np.array_equal(packed.cpu().numpy().ravel(), o.packed)
        assert np.array_equal(st.absmax.cpu().numpy().view(np.uint32), o.absmax_raw.view(np.uint32))


def test_golden_vectors(oracle_vectors):
    """Committed oracle vectors (tests/golden/oracle_vectors.npz)."""
    from quantizations_amd.core import dequantize_4bit, gemv_4bit, quantize_4bit

    V = oracle_vectors
    for key in sorted({k.rsplit("_", 1)[0] for k in V if k.endswith("_packed")}):
        qt = key.split("_")[0]
        W = torch.from_numpy(V[f"{key}_W"].view(np.float16))
        x = torch.from_numpy(V[f"{key}_x"].view(np.float16))
        packed, st = quantize_4bit(W.to(DEV), quant_type=qt)
        assert np.array_equal(packed.cpu().numpy().ravel(), V[f"{key}_packed"]), key
        assert np.array_equal(st.absmax.cpu().numpy(), V[f"{key}_qabsmax"]), key
        assert float(st.offset) == float(V[f"{key}_offset"]), key
        y = gemv_4bit(x.to(DEV).reshape(1, 1, -1), packed.t(), state=st)
        assert_close(y.float().cpu(), V[f"{key}_y"], torch.float16, key)
        assert np.array_equal(st.state2.absmax.cpu().numpy(), V[f"{key}_absmax2"]), key
        wd = dequantize_4bit(packed, st).t().contiguous().cpu().numpy().view(np.int16)
        bad = np.argwhere(wd != V[f"{key}_wdeq16"])
        assert bad.size == 0, (key, len(bad), bad[:5].tolist(), wd[tuple(bad[0])], V[f"{key}_wdeq16"][tuple(bad[0])])


def test_absmax_mean_bit_exact(orc):
    from quantizations_amd import _lib

    for n in (1, 7, 1024, 1025, 262144, 917504, 3670016):
        a = torch.rand(n, generator=torch.Generator().manual_seed(n)) * 0.05
        ad = a.to(DEV)
        off = torch.empty((), device=DEV)
        ws = torch.empty(int(_lib.lib.qz_absmax_mean_workspace(n)), device=DEV, dtype=torch.float64)
        _lib.check(_lib.lib.qz_absmax_mean(ad.data_ptr(), n, ws.data_ptr(), off.data_ptr(), 0), "mean")
        assert float(off) == float(orc.absmax_mean(a.numpy())), n


# ---------------------------------------------------------------------------
# dequantisation: bit-exact
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("qt", ["fp4", "nf4"])
@pytest.mark.parametrize("out_dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(128, 1024), (3, 37), (40, 2112)])
def test_dequantize_4bit_bit_exact(orc, qt, out_dtype, shape):
    from quantizations_amd.core import dequantize_4bit, quantize_4bit

    W = _w(*shape, seed=11)
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt)
    wd = dequantize_4bit(packed, st, out_dtype=out_dtype)
    assert wd.shape == (shape[1], shape[0])  # reference returns out.t() (core.py:634)
    o = orc.quantize_4bit(W.float().numpy(), 64, qt)
    ref = torch.from_numpy(orc.dequantize(o)).to(out_dtype)
    got = wd.t().contiguous().cpu()
    assert torch.equal(got.view(torch.int16 if out_dtype != torch.float32 else torch.int32),
                       ref.view(torch.int16 if out_dtype != torch.float32 else torch.int32))


def test_fp4_dequant_negative_zero():
    from quantizations_amd import kbkim_lib

    packed = torch.tensor([0x88, 0x80, 0x08, 0x00] * 16, dtype=torch.uint8, device=DEV)
    absmax = torch.ones(2, device=DEV)
    out = torch.empty(128, dtype=torch.float16, device=DEV)
    kbkim_lib.cdequantize_blockwise_fp16_fp4(0, packed.data_ptr(), absmax.data_ptr(), out.data_ptr(), 64, 128)
    o = out.cpu()
    assert torch.equal(o.view(torch.int16)[:8], torch.tensor([-32768, -32768, -32768, 0, 0, -32768, 0, 0],
                                                             dtype=torch.int16))


# ---------------------------------------------------------------------------
# the five reference entry points (kbkim_lib), called as core.py calls them
# ---------------------------------------------------------------------------


def test_kbkim_lib_reference_call_sequence(orc):
    from quantizations_amd import kbkim_lib

    M, K = 512, 4096
    W = _w(M, K, seed=21)
    x = _x(K, seed=22).float()
    n = M * K
    Wd, xd = W.to(DEV), x.to(DEV)
    absmax = torch.zeros(n // 64, device=DEV)
    packed = torch.zeros((n // 2, 1), dtype=torch.uint8, device=DEV)
    kbkim_lib.cquantize_blockwise_fp16_fp4(0, Wd.data_ptr(), absmax.data_ptr(), packed.data_ptr(), 64, n)  # core.py:552
    o = orc.quantize_4bit(W.float().numpy(), 64, "fp4")
    assert np.array_equal(packed.cpu().numpy().ravel(), o.packed)
    # double quant exactly as core.py:563-565 (torch mean, subtract, quantize_blockwise)
    offset = absmax.mean()
    a = absmax - offset
    code = torch.from_numpy(orc.create_dynamic_map()).to(DEV)
    q = torch.zeros_like(a, dtype=torch.uint8)
    a2 = torch.zeros(n // 64 // 256, device=DEV)
    kbkim_lib.cquantize_blockwise_fp32(code.data_ptr(), a.data_ptr(), a2.data_ptr(), q.data_ptr(), 256, a.numel())
    oq, oa2 = orc.quantize_blockwise_8bit(code.cpu().numpy(), a.cpu().numpy(), 256)
    assert np.array_equal(q.cpu().numpy(), oq) and np.array_equal(a2.cpu().numpy(), oa2)
    # decode: dequantize_blockwise + offset + GEMV (core.py:467-499)
    am = torch.empty_like(a)
    kbkim_lib.cdequantize_blockwise_fp32(code.data_ptr(), q.data_ptr(), a2.data_ptr(), am.data_ptr(), 256, q.numel())
    am += offset
    oam = orc.dequantize_blockwise_8bit(code.cpu().numpy(), oq, oa2, 256, float(offset))
    assert np.array_equal(am.cpu().numpy(), oam)
    lut = torch.from_numpy(orc.codebook("fp4")).to(DEV)
    out = torch.empty(1, 1, M, device=DEV)
    kbkim_lib.cgemm_4bit_inference_naive_fp32(M, 1, K, xd.data_ptr(), packed.data_ptr(), am.data_ptr(),
                                              lut.data_ptr(), out.data_ptr(), M, (K + 1) // 2, M, 64)
    yref = orc.gemv_4bit(x.numpy(), o.packed, oam, orc.codebook("fp4"), M, K, 64)
    assert_close(out.cpu(), yref, torch.float32, "cgemm_4bit_inference_naive_fp32")
    # prefill dequant (core.py:624)
    wout = torch.empty(n, dtype=torch.float16, device=DEV)
    kbkim_lib.cdequantize_blockwise_fp16_fp4(0, packed.data_ptr(), am.data_ptr(), wout.data_ptr(), 64, n)
    ow = orc.dequantize_4bit(o.packed, oam, n, 64, "fp4").astype(np.float16)
    assert np.array_equal(wout.cpu().numpy().view(np.int16), ow.view(np.int16))
    with pytest.raises(TypeError):
        kbkim_lib.cquantize_blockwise_fp32(1.5, 0, 0, 0, 256, 1)


# ---------------------------------------------------------------------------
# fused GEMV
# ---------------------------------------------------------------------------

GEMV_SHAPES = [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336), (1000, 2048), (37, 2112), (7, 96),
               (130, 1024), (8, 8192), (3, 100), (5, 62)]


@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("dq", [True, False])
@pytest.mark.parametrize("shape", GEMV_SHAPES)
def test_gemv_f16(orc, qt, dq, shape):
    from quantizations_amd.core import gemv_4bit, quantize_4bit

    M, K = shape
    W = _w(M, K, seed=M + K)
    x = _x(K, seed=K)
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=dq)
    y = gemv_4bit(x.to(DEV).reshape(1, 1, K), packed.t(), state=st)
    assert y.shape == (1, 1, M) and y.dtype == torch.float16
    o = orc.quantize_4bit(W.float().numpy(), 64, qt, double_quant=dq)
    assert_close(y.float().cpu(), orc.gemv(x.float().numpy(), o), torch.float16, f"{qt} dq={dq} {shape}")


@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(4096, 4096), (1024, 4096), (333, 2048), (7, 96), (5, 62)])
def test_gemv_bf16_f32_activations(orc, qt, dtype, shape):
    from quantizations_amd.core import gemv_4bit, quantize_4bit

    M, K = shape
    W = _w(M, K, seed=3 * M + K)
    x = _x(K, seed=2 * K, dtype=dtype)
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt)
    y = gemv_4bit(x.to(DEV).reshape(1, K), packed.t(), state=st)
    assert y.shape == (1, M) and y.dtype == dtype
    o = orc.quantize_4bit(W.float().numpy(), 64, qt)
    assert_close(y.float().cpu(), orc.gemv(x.float().numpy(), o), dtype, f"{qt} {dtype} {shape}")


def test_gemv_bias_and_large_activations(orc):
    from quantizations_amd.core import gemv_4bit, quantize_4bit

    M, K = 2048, 4096
    W = _w(M, K, seed=77)
    x = _x(K, seed=78) * 300  # large activations (fp16 range), fp32 path split hi/lo
    bias = torch.randn(M, generator=torch.Generator().manual_seed(79))
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    o = orc.quantize_4bit(W.float().numpy(), 64, "nf4")
    yref = orc.gemv(x.float().numpy(), o) + bias.numpy().astype(np.float64)
    for dt in (torch.float16, torch.float32):
        y = gemv_4bit(x.to(dt).to(DEV).reshape(1, 1, K), packed, state=st, bias=bias.to(dt).to(DEV))
        yr = orc.gemv(x.to(dt).float().numpy(), o) + bias.to(dt).float().numpy()
        assert_close(y.float().cpu(), yr, dt, f"bias {dt}")
    del yref


def test_gemv_deterministic_and_full_size_properties(orc):
    """4096x4096 (the headline shape): repeat launches are bitwise identical and
    y is linear in x (y(2x) == 2 y(x) exactly for fp32 accumulation of fp16 inputs)."""
    from quantizations_amd.core import gemv_4bit, quantize_4bit

    W = _w(4096, 4096, seed=99)
    x = _x(4096, seed=98).to(DEV).reshape(1, 1, -1)
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    y1 = gemv_4bit(x, packed, state=st)
    y2 = gemv_4bit(x, packed, state=st)
    assert torch.equal(y1, y2)
    y3 = gemv_4bit(x.float() * 2, packed, state=st)
    y4 = gemv_4bit(x.float(), packed, state=st)
    assert torch.allclose(y3, 2 * y4, rtol=1e-5, atol=1e-6)
    o = orc.quantize_4bit(W.float().numpy(), 64, "nf4")
    assert_close(y4.cpu(), orc.gemv(x.float().cpu().numpy().ravel(), o), torch.float32, "4096 fp32")


def test_gemv_row_shard_block_base(orc):
    """A row shard addressed with block_base gives the same rows as the full layer."""
    from quantizations_amd.core import gemv_4bit, quantize_4bit
    from quantizations_amd.parallel import shard_rows

    M, K = 96, 640
    W = _w(M, K, seed=41)
    x = _x(K, seed=42).to(DEV).reshape(1, K)
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    full = gemv_4bit(x, packed, state=st)
    for world in (2, 4):
        for r in range(world):
            sh = shard_rows(packed, st, r, world)
            y = gemv_4bit(x, sh.packed, state=sh.state, block_base=sh.block_base)
            assert torch.equal(y, full[:, sh.r0:sh.r1]), (world, r)


@pytest.mark.parametrize("bs", [128, 256, 1024, 4096])
@pytest.mark.parametrize("qt,dq", [("nf4", True), ("fp4", False)])
def test_gemv_grouped_gemm_dequant_other_blocksizes(orc, bs, qt, dq):
    """blocksize != 64 through every consumer: GEMV, grouped GEMV (vs the oracle),
    GEMM (vs fp64 of the dequantised weight) and the dequant kernel (bit-exact)."""
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, gemv_4bit, gemv_4bit_grouped, quantize_4bit

    M, K = 256, 4096
    W = _w(M, K, seed=bs)
    x = _x(K, seed=bs + 1).to(DEV).reshape(1, K)
    packed, st = quantize_4bit(W.to(DEV), blocksize=bs, quant_type=qt, compress_statistics=dq)
    o = orc.quantize_4bit(W.float().numpy(), bs, qt, double_quant=dq)
    yref = orc.gemv(x.float().cpu().numpy().ravel(), o)
    assert_close(gemv_4bit(x, packed, state=st).float().cpu(), yref, torch.float16, f"gemv bs={bs}")
    (yg,) = gemv_4bit_grouped(x, [(packed, st, None)])
    assert_close(yg.float().cpu(), yref, torch.float16, f"grouped bs={bs}")
    wd = dequantize_4bit(packed, st).t()
    ow = orc.dequantize(o).astype(np.float16).reshape(M, K)
    assert np.array_equal(wd.cpu().numpy().view(np.int16), ow.view(np.int16)), f"dequant bs={bs}"
    X = torch.randn(40, K, generator=torch.Generator().manual_seed(bs)).half().to(DEV)
    Y = gemm_4bit(X, packed, st, route="fused")
    assert_close(Y.float().cpu(), (X.double() @ wd.double().t()).cpu().numpy(), torch.float16, f"gemm bs={bs}")


@pytest.mark.parametrize("M,K", [(8192, 28672), (28672, 8192), (10240, 8192)])
def test_gemv_llama70b_shapes_vs_fp64_of_dequant(M, K):
    """Full Llama-3-70B shapes (down, gate/up, fused q/k/v): GEMV vs an fp64 product
    of the bit-exact dequantised weight (the oracle is too slow at 235 M weights; the
    dequant kernel is pinned to it bit for bit at smaller sizes)."""
    from quantizations_amd.core import dequantize_4bit, gemv_4bit, quantize_4bit

    torch.manual_seed(M + K)
    W = (torch.randn(M, K, device=DEV) * 0.02).half()
    packed, st = quantize_4bit(W, quant_type="nf4")
    del W
    x = torch.randn(1, K, device=DEV).half()
    y = gemv_4bit(x, packed, state=st)
    wd = dequantize_4bit(packed, st, out_dtype=torch.float32).t()   # [M, K] fp32 = the reference's weight products
    ref = (wd.double() @ x.double().reshape(K, 1)).reshape(1, M)
    del wd
    assert_close(y.float().cpu(), ref.cpu().numpy(), torch.float16, f"gemv {M}x{K}")


@pytest.mark.parametrize("act", [torch.bfloat16, torch.float32])
def test_linear4bit_bf16_fp32_activations_and_compute_dtype(orc, act):
    """Linear4bit with bf16/fp32 inputs (compute_dtype follows the input, reference
    modules.py:112-122): decode and prefill outputs keep the input dtype.  Decode is
    checked against the reference's fp32 weight products (kernels.cu:1169: the fp32
    dequantised weight, bit-exact to the oracle); prefill against the weight in the
    activation dtype that the kernels
    multiply: dequantize_4bit(out_dtype=act), i.e. bf16(code*absmax) rounded once.
    (The reference's bf16 path multiplies W.to(bf16) of the fp16 dequant, modules.py:64,
    a double rounding that differs by one bf16 ulp on ~1/16 of the weights -- the
    output difference that makes is ~2^-9 relative)"""
    import quantizations_amd as qa

    torch.manual_seed(5)
    lin = torch.nn.Linear(1024, 768, bias=True)
    m = qa.Linear4bit(1024, 768, bias=True, quant_type="nf4")
    m.weight = qa.Params4bit(lin.weight.data.half(), requires_grad=False, quant_type="nf4", module=m)
    m.bias = torch.nn.Parameter(lin.bias.data.clone(), requires_grad=False)
    m = m.to(DEV)
    Wd = qa.dequantize_4bit(m.weight, m.weight.quant_state, out_dtype=torch.float32).t().double()
    for shape in ((1, 1, 1024), (3, 5, 1024)):
        x = torch.randn(*shape, generator=torch.Generator().manual_seed(sum(shape))).to(act)
        y = m(x.to(DEV))
        assert y.dtype == act and y.shape == (*shape[:-1], 768)
        Wop = Wd if shape[1] == 1 else \
            qa.dequantize_4bit(m.weight, m.weight.quant_state, out_dtype=act if act != torch.float32 else None).t().double()
        ref = x.double().reshape(-1, 1024) @ Wop.t().cpu() + lin.bias.detach().double()
        assert_close(y.float().cpu().reshape(-1, 768), ref.numpy(), act, f"{act} {shape}")


GROUPED_SETS = [  # (segment rows, K): Llama-3-8B q/k/v and gate/up, plus odd and tiny cases
    ((4096, 1024, 1024), 4096), ((14336, 14336), 4096), ((512, 128, 128), 1024), ((37, 5, 64, 3), 2112),
    ((7, 9), 96), ((3, 4), 62)]


@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("dq", [True, False])
@pytest.mark.parametrize("rows,K", GROUPED_SETS)
def test_gemv_grouped_matches_oracle(orc, qt, dq, rows, K):
    """One grouped launch (q/k/v-style segments sharing x) == each layer's oracle GEMV."""
    from quantizations_amd.core import gemv_4bit, gemv_4bit_grouped, quantize_4bit

    x = _x(K, seed=K + 5).to(DEV).reshape(1, 1, K)
    items, refs = [], []
    for i, M in enumerate(rows):
        W = _w(M, K, seed=100 + 7 * i + M)
        packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=dq)
        bias = torch.randn(M, generator=torch.Generator().manual_seed(i)).half().to(DEV) if i == 1 else None
        items.append((packed, st, bias))
        o = orc.quantize_4bit(W.float().numpy(), 64, qt, double_quant=dq)
        r = orc.gemv(x.float().cpu().numpy().ravel(), o).astype(np.float32)
        refs.append(r + (bias.float().cpu().numpy() if bias is not None else 0))
    ys = gemv_4bit_grouped(x, items)
    for i, (y, r) in enumerate(zip(ys, refs)):
        assert y.shape == (1, 1, rows[i]) and y.dtype == torch.float16
        assert_close(y.float().cpu(), r, torch.float16, f"segment {i} {qt} dq={dq} rows={rows} K={K}")
        single = gemv_4bit(x, items[i][0], state=items[i][1], bias=items[i][2])
        assert_close(y.float().cpu(), single.float().cpu().numpy(), torch.float16, f"vs single {i}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemv_grouped_activation_dtypes_and_out(orc, dtype):
    from quantizations_amd.core import gemv_4bit_grouped, quantize_4bit

    K = 2048
    x = _x(K, seed=3, dtype=dtype).to(DEV).reshape(1, K)
    rows = (1000, 24)
    buf = torch.full((sum(rows),), float("nan"), dtype=dtype, device=DEV)
    items, refs, o0 = [], [], 0
    for i, M in enumerate(rows):
        W = _w(M, K, seed=50 + i)
        packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
        items.append((packed, st, None, 0, buf[o0:o0 + M]))
        o0 += M
        refs.append(orc.gemv(x.float().cpu().numpy().ravel(), orc.quantize_4bit(W.float().numpy(), 64, "nf4")))
    ys = gemv_4bit_grouped(x, items)
    assert ys[0].data_ptr() == buf.data_ptr()  # written in place
    for y, r in zip(ys, refs):
        assert_close(y.float().cpu(), r, dtype, f"grouped {dtype}")


def test_gemv_grouped_rejects_mismatched_weights():
    from quantizations_amd.core import gemv_4bit_grouped, quantize_4bit

    x = torch.randn(1, 256, device=DEV, dtype=torch.float16)
    a = quantize_4bit(_w(64, 256).to(DEV), quant_type="nf4")
    b = quantize_4bit(_w(64, 512).to(DEV), quant_type="nf4")
    c = quantize_4bit(_w(64, 256).to(DEV), quant_type="nf4", compress_statistics=False)
    with pytest.raises(ValueError):
        gemv_4bit_grouped(x, [(a[0], a[1], None), (b[0], b[1], None)])       # different K
    with pytest.raises(ValueError):
        gemv_4bit_grouped(x, [(a[0], a[1], None), (c[0], c[1], None)])       # DQ vs fp32 absmax
    with pytest.raises(ValueError):
        gemv_4bit_grouped(x, [(a[0], a[1], None)] * 5)                       # > QZ_GEMV_MAX_SEGMENTS


def test_gemv_grouped_row_shards(orc):
    """Row shards (block_base != 0) of three layers in one grouped launch."""
    from quantizations_amd.core import gemv_4bit, gemv_4bit_grouped, quantize_4bit
    from quantizations_amd.parallel import shard_rows

    K = 640
    x = _x(K, seed=61).to(DEV).reshape(1, K)
    fulls, shards = [], []
    for i, M in enumerate((96, 32, 64)):
        packed, st = quantize_4bit(_w(M, K, seed=70 + i).to(DEV), quant_type="nf4")
        fulls.append(gemv_4bit(x, packed, state=st))
        shards.append(shard_rows(packed, st, 1, 2))
    ys = gemv_4bit_grouped(x, [(sh.packed, sh.state, None, sh.block_base) for sh in shards])
    for y, f, sh in zip(ys, fulls, shards):
        assert_close(y.float().cpu(), f[:, sh.r0:sh.r1].float().cpu().numpy(), torch.float16, "grouped shard")


@pytest.mark.parametrize("T", [2, 5, 16])
@pytest.mark.parametrize("qt,dq,dtype", [("nf4", True, torch.float16), ("fp4", False, torch.float16),
                                         ("nf4", True, torch.bfloat16)])
def test_gemm_grouped_multitoken_bit_identical(T, qt, dq, dtype):
    """Grouped multi-token launch (q/k/v-style segments over a small batch of
    decode tokens) == each segment's own gemm_4bit (the multi-token kernel),
    bit for bit; row shards with block_base != 0 == the full weight's rows."""
    from quantizations_amd.core import gemm_4bit, gemm_4bit_grouped, grouped_tokens_ok, quantize_4bit
    from quantizations_amd.parallel import shard_rows

    K = 1024
    x = torch.randn(T, K, generator=torch.Generator().manual_seed(T), dtype=torch.float32).to(dtype).to(DEV)
    items, singles = [], []
    for i, M in enumerate((512, 128, 96)):
        packed, st = quantize_4bit(_w(M, K, seed=200 + i).to(DEV), quant_type=qt, compress_statistics=dq)
        bias = torch.randn(M, generator=torch.Generator().manual_seed(i)).to(dtype).to(DEV) if i == 2 else None
        items.append((packed, st, bias))
        singles.append(gemm_4bit(x, packed, st, bias=bias, route="fused"))
    assert grouped_tokens_ok(x, items)
    ys = gemm_4bit_grouped(x, items)
    for y, r in zip(ys, singles):
        assert y.shape == r.shape and y.dtype == dtype
        assert torch.equal(y, r)
    # row shards of a double-quant weight whose second shard starts inside a 256-block group
    packed, st = quantize_4bit(_w(72, K, seed=300).to(DEV), quant_type=qt, compress_statistics=dq)  # 36-row shards
    full = gemm_4bit(x, packed, st, route="fused")
    shards = [shard_rows(packed, st, r, 2) for r in range(2)]
    ys = gemm_4bit_grouped(x, [(sh.packed, sh.state, None, sh.block_base) for sh in shards])
    if dq:
        assert shards[1].block_base != 0
    for y, sh in zip(ys, shards):
        assert torch.equal(y, full[:, sh.r0:sh.r1])


def test_gemm_grouped_rejects_unsupported():
    from quantizations_amd.core import gemm_4bit_grouped, grouped_tokens_ok, quantize_4bit

    a = quantize_4bit(_w(64, 512).to(DEV), quant_type="nf4")
    x1 = torch.randn(1, 512, device=DEV, dtype=torch.float16)
    x20 = torch.randn(20, 512, device=DEV, dtype=torch.float16)
    x_k = torch.randn(3, 320, device=DEV, dtype=torch.float16)
    b = quantize_4bit(_w(64, 320).to(DEV), quant_type="nf4")
    assert not grouped_tokens_ok(x1, [(a[0], a[1], None)])      # one token: the grouped GEMV's job
    assert not grouped_tokens_ok(x20, [(a[0], a[1], None)])     # > 16 tokens: prefill
    assert not grouped_tokens_ok(x_k, [(b[0], b[1], None)])     # K % 256 != 0
    with pytest.raises(ValueError):
        gemm_4bit_grouped(x20, [(a[0], a[1], None)])


def test_tiny_llama_batched_decode_groups():
    """Three bs=1 decode streams in one batch (the bench's weak-scaling layout
    per GPU): with fuse_projection_groups the q/k/v and gate/up members run as
    one grouped multi-token launch each and the logits equal the unfused
    model's bit for bit; a 20-token prefill bypasses the groups."""
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import fuse_projection_groups, replace_with_bnb_linear

    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(4)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4")
    ids = torch.randint(0, 512, (3, 20), device=DEV)
    with torch.no_grad():
        ref = model(input_ids=ids, use_cache=True)
        tok = ref.logits[:, -1:].argmax(-1)
        ref_step = model(input_ids=tok, past_key_values=ref.past_key_values, use_cache=True).logits
        assert fuse_projection_groups(model) == 2 * cfg.num_hidden_layers
        out = model(input_ids=ids, use_cache=True)
        assert torch.equal(out.logits, ref.logits)
        step = model(input_ids=tok, past_key_values=out.past_key_values, use_cache=True).logits
    assert torch.equal(step, ref_step)


# ---------------------------------------------------------------------------
# fused prefill GEMM (MFMA)
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("dq", [True, False])
@pytest.mark.parametrize("T,M,K", [(128, 128, 64), (200, 384, 1024), (17, 4096, 4096), (1024, 1024, 4096),
                                   (64, 14336, 4096), (33, 4096, 14336)])
def test_gemm_prefill(orc, qt, dq, T, M, K):
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    W = _w(M, K, seed=T + M)
    g = torch.Generator().manual_seed(T)
    X = torch.randn(T, K, generator=g).to(torch.float16)
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=dq)
    Y = gemm_4bit(X.to(DEV), packed, st)
    assert Y.shape == (T, M) and Y.dtype == torch.float16
    o = orc.quantize_4bit(W.float().numpy(), 64, qt, double_quant=dq)
    Wd = torch.from_numpy(orc.dequantize(o)).double()
    Yref = (X.double() @ Wd.t()).numpy()
    assert_close(Y.float().cpu(), Yref, torch.float16, f"gemm {qt} dq={dq} {T}x{M}x{K}")


def test_gemm_large_t_tile_bias_and_fp4(orc):
    """T >= 4096 (the 256 x 256 tile kernel): bias, FP4 without double quant, a
    partial last token tile, vs the oracle's dequantised weight in fp64."""
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    T, M, K = 4097, 768, 1024
    W = _w(M, K, seed=41)
    X = torch.randn(T, K, generator=torch.Generator().manual_seed(42)).to(torch.float16)
    bias = torch.randn(M, generator=torch.Generator().manual_seed(43)).to(torch.float16)
    packed, st = quantize_4bit(W.to(DEV), quant_type="fp4", compress_statistics=False)
    Y = gemm_4bit(X.to(DEV), packed, st, bias=bias.to(DEV), route="fused")
    o = orc.quantize_4bit(W.float().numpy(), 64, "fp4", double_quant=False)
    Wd = torch.from_numpy(orc.dequantize(o)).double()
    Yref = (X.double() @ Wd.t() + bias.double()).numpy()
    assert_close(Y.float().cpu(), Yref, torch.float16, "gemm 256-tile fp4 + bias")


def test_gemm_bias_and_batch_dims(orc):
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    T, M, K = 2 * 77, 640, 512
    W = _w(M, K, seed=5)
    X = torch.randn(2, 77, K, generator=torch.Generator().manual_seed(6)).to(torch.float16)
    bias = torch.randn(M, generator=torch.Generator().manual_seed(7)).to(torch.float16)
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    Y = gemm_4bit(X.to(DEV), packed, st, bias=bias.to(DEV))
    o = orc.quantize_4bit(W.float().numpy(), 64, "nf4")
    Wd = torch.from_numpy(orc.dequantize(o)).double()
    Yref = (X.reshape(T, K).double() @ Wd.t() + bias.double()).numpy()
    assert Y.shape == (2, 77, M)
    assert_close(Y.reshape(T, M).float().cpu(), Yref, torch.float16, "gemm bias")


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("dq", [True, False])
@pytest.mark.parametrize("T,M,K", [(1, 256, 4096), (37, 512, 1024), (64, 4096, 4096), (200, 1024, 2048),
                                   (4100, 520, 1024), (4096, 264, 64), (4352, 256, 128)])
def test_gemm_w_operand_is_the_dequantised_weight(qt, dq, dt, T, M, K):
    """One-hot activations read single weights back through the MFMA path: row t
    of Y must equal column k_t of dequantize_4bit(W, out_dtype=dt) BIT FOR BIT
    (values; -0.0 reads back as +0.0).  Pins the in-LDS decode (per-block
    fp16/bf16 table of code*absmax, double-quant rebuild, pair order shared by
    X and W) to the dequant kernel; covers both token tiles, split-K and (T >= 4096)
    the 256 x 256 tile kernel with partial token and row tiles, and its one- and two-step
    K loops (K = 64, 128: no DMA two steps ahead, stale-ring decode of the last step)."""
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, quantize_4bit

    W = _w(M, K, seed=3 * T + M)
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=dq)
    ks = (torch.arange(T) * 997 + 13) % K          # probe positions across blocks and nibble slots
    X = torch.zeros(T, K, dtype=dt)
    X[torch.arange(T), ks] = 1.0
    Y = gemm_4bit(X.to(DEV), packed, st, route="fused")
    assert Y.shape == (T, M) and Y.dtype == dt
    Wd = dequantize_4bit(packed, st, out_dtype=dt).t()   # [M, K]
    assert torch.equal(Y, Wd[:, ks.to(DEV)].t()), f"{qt} dq={dq} {dt} {T}x{M}x{K}"


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("T,M,K", [(5, 512, 1024), (64, 4096, 4096), (300, 768, 4096), (4096, 1024, 4096),
                                   (4352, 264, 512)])
def test_gemm_random_activations_vs_fp64(dt, T, M, K):
    """Random activations: fused result vs an fp64 matmul of the dequantised
    weight -- only fp32 summation order and the output rounding differ."""
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, quantize_4bit

    W = _w(M, K, seed=T + 7 * M)
    X = torch.randn(T, K, generator=torch.Generator().manual_seed(T + K)).to(dt).to(DEV)
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    Y = gemm_4bit(X, packed, st, route="fused")
    ref = X.double() @ dequantize_4bit(packed, st, out_dtype=dt).double()
    assert_close(Y.float().cpu(), ref.cpu().numpy(), dt, f"gemm vs fp64 {dt} {T}x{M}x{K}")


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("qt,dq", [("nf4", True), ("fp4", True), ("nf4", False)])
@pytest.mark.parametrize("T,M,K", [(2, 4096, 4096), (3, 1028, 1280), (8, 14336, 4096), (16, 4096, 14336),
                                   (16, 132, 256)])
def test_multi_token_gemv_exact_operand_and_oracle(orc, qt, dq, dt, T, M, K):
    """2..16 tokens take the multi-token MFMA GEMV: one-hot tokens read back
    dequantize_4bit's weights bit for bit; random tokens match the oracle."""
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, quantize_4bit

    W = _w(M, K, seed=M + 3 * K + T)
    packed, st = quantize_4bit(W.to(DEV), quant_type=qt, compress_statistics=dq)
    ks = (torch.arange(T) * 389 + 7) % K
    X1 = torch.zeros(T, K, dtype=dt)
    X1[torch.arange(T), ks] = 1.0
    Y1 = gemm_4bit(X1.to(DEV), packed, st, route="fused")
    Wd = dequantize_4bit(packed, st, out_dtype=dt).t()
    assert torch.equal(Y1, Wd[:, ks.to(DEV)].t()), f"one-hot {qt} dq={dq} {dt} {T}x{M}x{K}"
    X = torch.randn(T, K, generator=torch.Generator().manual_seed(T * K)).to(dt)
    bias = torch.randn(M, generator=torch.Generator().manual_seed(M)).to(dt)
    Y = gemm_4bit(X.to(DEV), packed, st, bias=bias.to(DEV), route="fused")
    ref = X.double() @ Wd.double().cpu().t() + bias.double()
    assert_close(Y.float().cpu(), ref.numpy(), dt, f"mt {qt} dq={dq} {dt} {T}x{M}x{K}")


def test_multi_token_gemv_without_workspace():
    """Direct C-ABI call with no workspace: the multi-token kernel runs unsplit when
    the K slice fits LDS, else the tiled kernel takes it -- same results."""
    from quantizations_amd import _lib
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    for K in (1024, 4096):
        T, M = 5, 512
        W = _w(M, K, seed=K)
        packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
        X = torch.randn(T, K, generator=torch.Generator().manual_seed(1)).half().to(DEV)
        Y = torch.empty(T, M, dtype=torch.float16, device=DEV)
        _lib.check(_lib.lib.qz_gemm_4bit(T, M, K, X.data_ptr(), K, _lib.DT_F16, packed.data_ptr(), _lib.NF4, 64,
                                         *st.scale_args(), 0, Y.data_ptr(), M, 0, 0,
                                         torch.cuda.current_stream().cuda_stream), "gemm")
        ref = gemm_4bit(X, packed, st, route="fused")
        assert ((Y.double() - ref.double()).norm() / ref.double().norm()) < 1e-3


def test_gemm_routes_agree_and_fallbacks():
    """route='fused' and route='dequant' multiply the same operand; shapes the
    fused kernel does not take (M % 4 != 0, fp32 input) fall back in 'auto'."""
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    W = _w(512, 1024, seed=1)
    X = torch.randn(100, 1024, generator=torch.Generator().manual_seed(2)).half().to(DEV)
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    a = gemm_4bit(X, packed, st, route="fused").double()
    b = gemm_4bit(X, packed, st, route="dequant").double()
    assert ((a - b).norm() / b.norm()) < 2e-3
    W2 = _w(510, 1024, seed=3)
    p2, s2 = quantize_4bit(W2.to(DEV), quant_type="nf4")
    with pytest.raises(ValueError):
        gemm_4bit(X, p2, s2, route="fused")
    y2 = gemm_4bit(X, p2, s2)  # auto -> dequant route
    assert y2.shape == (100, 510)
    y3 = gemm_4bit(X.float(), packed, st)  # fp32 activations -> dequant route, fp32 out
    assert y3.dtype == torch.float32 and ((y3.double() - b).norm() / b.norm()) < 2e-3


def test_gemm_split_k_with_bias_matches_unsplit(orc):
    """Small T splits K over workgroups (fp32 partials + reduce kernel): same
    result as the oracle, bias added once."""
    from quantizations_amd import _lib
    from quantizations_amd.core import gemm_4bit, quantize_4bit

    T, M, K = 20, 1024, 8192   # > 16 tokens: the tiled kernel, K split over workgroups
    assert _lib.lib.qz_gemm_4bit_workspace_size(T, M, K) > 0  # this shape does split
    assert _lib.lib.qz_gemm_4bit_workspace_size(8, M, K) == 0  # 2..16 tokens reduce in LDS
    W = _w(M, K, seed=11)
    X = torch.randn(T, K, generator=torch.Generator().manual_seed(12)).half()
    bias = torch.randn(M, generator=torch.Generator().manual_seed(13)).half()
    packed, st = quantize_4bit(W.to(DEV), quant_type="nf4")
    Y = gemm_4bit(X.to(DEV), packed, st, bias=bias.to(DEV), route="fused")
    o = orc.quantize_4bit(W.float().numpy(), 64, "nf4")
    Yref = (X.double() @ torch.from_numpy(orc.dequantize(o)).double().t() + bias.double()).numpy()
    assert_close(Y.float().cpu(), Yref, torch.float16, "split-K + bias")


# ---------------------------------------------------------------------------
# module level: Linear4bit drop-in
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("qt", ["fp4", "nf4"])
def test_linear4bit_decode_and_prefill(orc, qt):
    import quantizations_amd as qa

    torch.manual_seed(0)
    lin = torch.nn.Linear(1024, 768, bias=True).half().requires_grad_(False)
    m = qa.Linear4bit(1024, 768, bias=True, compute_dtype=torch.float32, quant_type=qt)
    m.weight = qa.Params4bit(lin.weight.data.clone(), requires_grad=False, quant_type=qt, module=m)
    m.bias = torch.nn.Parameter(lin.bias.data.clone(), requires_grad=False)
    m = m.to(DEV)
    assert m.weight.bnb_quantized and m.quant_state is m.weight.quant_state
    o = orc.quantize_4bit(lin.weight.data.float().numpy(), 64, qt)
    Wd = torch.from_numpy(orc.dequantize(o)).double()
    x1 = torch.randn(1, 1, 1024).half()
    y1 = m(x1.to(DEV))
    assert y1.dtype == torch.float16 and y1.shape == (1, 1, 768)
    assert_close(y1.float().cpu(), (x1.double().reshape(1, -1) @ Wd.t() + lin.bias.detach().double()).numpy(),
                 torch.float16, "decode")
    x2 = torch.randn(2, 9, 1024).half()
    y2 = m(x2.to(DEV))
    assert y2.shape == (2, 9, 768)
    assert_close(y2.float().cpu().reshape(18, -1),
                 (x2.double().reshape(18, -1) @ Wd.t() + lin.bias.detach().double()).numpy(), torch.float16, "prefill")


def test_linear4bit_hip_graph_capture(orc):
    """The decode path launches on torch's current stream and is capturable."""
    import quantizations_amd as qa

    m = qa.Linear4bit(4096, 4096, quant_type="nf4").half()
    m = m.to(DEV)
    x = torch.randn(1, 1, 4096, device=DEV, dtype=torch.float16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            m(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = m(x)
    x.copy_(torch.randn_like(x))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, m(x))


def test_tiny_llama_with_linear4bit(orc):
    """replace_with_bnb_linear on a small LlamaForCausalLM: logits match the same
    model with the dequantised weights in a plain fp32 nn.Linear."""
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import replace_with_bnb_linear
    import quantizations_amd as qa

    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4")
    ids = torch.randint(0, 512, (1, 12), device=DEV)
    with torch.no_grad():
        out = model(input_ids=ids).logits.float()
        # reference: same model, each Linear4bit replaced by fp32 linear on its dequantised weight
        ref = LlamaForCausalLM(cfg).to(DEV).eval()
        ref.load_state_dict({k: v for k, v in model.state_dict().items() if "weight" in k and v.dtype != torch.uint8},
                            strict=False)
        for name, mod in model.named_modules():
            if isinstance(mod, qa.Linear4bit):
                tgt = ref.get_submodule(name)
                tgt.weight.data.copy_(mod.dequantize().float())
        out_ref = ref(input_ids=ids).logits.float()
    rel = (out - out_ref).norm() / out_ref.norm()
    assert rel < 5e-3, rel


def test_tiny_llama_fused_projection_groups(orc):
    """fuse_projection_groups (q/k/v and gate/up in one launch each): greedy
    decode tokens and logits match the unfused model; also under HIP-graph
    capture of the decode step."""
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import (fuse_projection_groups, replace_with_bnb_linear,
                                               unfuse_projection_groups)

    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(1)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    ids = torch.randint(0, 512, (1, 8), device=DEV)
    with torch.no_grad():
        ref = model(input_ids=ids, use_cache=True)
        tok = ref.logits[:, -1:].argmax(-1)
        ref_step = model(input_ids=tok, past_key_values=ref.past_key_values, use_cache=True).logits.float()
        tok2 = ref_step[:, -1:].argmax(-1)
        ref_step2 = model(input_ids=tok2, past_key_values=ref.past_key_values, use_cache=True).logits.float()
        assert fuse_projection_groups(model) == 2 * cfg.num_hidden_layers
        out = model(input_ids=ids, use_cache=True)     # prefill bypasses the groups
        assert torch.equal(out.logits, ref.logits)
        # two decode steps: each step's new input must recompute the groups
        for t, r in ((tok, ref_step), (tok2, ref_step2)):
            step = model(input_ids=t, past_key_values=out.past_key_values, use_cache=True).logits.float()
            rel = (step - r).norm() / r.norm()
            assert rel < 2e-3, rel
        unfuse_projection_groups(model)
        assert all("_qz_group" not in m.__dict__ for m in model.modules())


def test_fused_groups_hip_graph_capture():
    """Grouped q/k/v inside a captured graph: replays follow new inputs."""
    import quantizations_amd as qa
    from quantizations_amd.integration import fuse_projection_groups

    parent = torch.nn.Module()
    for name, M in (("q_proj", 2048), ("k_proj", 512), ("v_proj", 512)):
        parent.add_module(name, qa.Linear4bit(2048, M, quant_type="nf4").half().to(DEV))
    assert fuse_projection_groups(parent) == 1
    x = torch.randn(1, 1, 2048, device=DEV, dtype=torch.float16)

    def run():
        return parent.q_proj(x), parent.k_proj(x), parent.v_proj(x)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            run()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = run()
    x.copy_(torch.randn_like(x))
    g.replay()
    torch.cuda.synchronize()
    for o, name in zip(outs, ("q_proj", "k_proj", "v_proj")):
        m = getattr(parent, name)
        ref = torch.nn.functional.linear(x.float(), m.dequantize().float())
        rel = (o.float() - ref).norm() / ref.norm()
        assert rel < 2e-3, (name, rel)


def test_tensor_parallel_pair_world1_rccl():
    """apply_tensor_parallel through the real kernels and RCCL (world size 1):
    column-parallel q/k/v/gate/up, row-parallel o/down (re-packed column slice,
    fp32 per-block absmax resolved from the double quant) + all-reduce; logits
    equal the unsharded quantised model's."""
    import socket

    import torch.distributed as dist
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import fuse_projection_groups, replace_with_bnb_linear
    from quantizations_amd.parallel import RowParallelLinear4bit, apply_tensor_parallel

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                          num_key_value_heads=2, vocab_size=512)
        torch.manual_seed(3)
        model = LlamaForCausalLM(cfg).half().to(DEV).eval()
        replace_with_bnb_linear(model, quant_type="nf4")
        ids = torch.randint(0, 512, (1, 7), device=DEV)
        with torch.no_grad():
            ref = model(input_ids=ids).logits.float()
            assert apply_tensor_parallel(model, 0, 1) == 2 * cfg.num_hidden_layers
            assert isinstance(model.model.layers[1].mlp.down_proj, RowParallelLinear4bit)
            fuse_projection_groups(model)
            out = model(input_ids=ids, use_cache=True)
            nxt = out.logits[:, -1:].argmax(-1)
            step = model(input_ids=nxt, past_key_values=out.past_key_values, use_cache=True).logits.float()
        assert ((out.logits.float() - ref).norm() / ref.norm()) < 2e-3
        assert torch.isfinite(step).all()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("M,K", [(8192, 8192), (1024, 8192), (28672, 8192), (8192, 28672)])
def test_config5_70b_rowsplit_shards_on_one_gpu(M, K):
    """Config #5's layout at its workload, rank by rank on one GPU: every
    Llama-3-70B Linear4bit shape row-split 8 ways exactly as parallel.shard_rows
    gives each rank (slices of the global quant state + block_base).  The
    all-gather order (rank-major concatenation) of the ranks' fused GEMVs matches
    an fp64 product of the bit-exact dequantised weight, as the unsharded launch
    does; a shard differs from the unsharded rows only by fp32 summation order
    (the shard's and the full launch's geometries split K differently): one fp16
    ulp of the output plus fp32 rounding relative to the terms' magnitude sum."""
    from quantizations_amd.core import dequantize_4bit, gemv_4bit, quantize_4bit
    from quantizations_amd.parallel import shard_rows

    torch.manual_seed(M ^ K)
    W = (torch.randn(M, K, device=DEV) * 0.02).half()
    packed, st = quantize_4bit(W, quant_type="nf4")
    del W
    x = torch.randn(1, 1, K, device=DEV).half()
    full = gemv_4bit(x, packed, state=st)
    world = 8
    parts = []
    for r in range(world):
        sh = shard_rows(packed, st, r, world)
        y = gemv_4bit(x, sh.packed, state=sh.state, block_base=sh.block_base)
        parts.append(y.reshape(-1))
    gathered = torch.cat(parts)
    wd = dequantize_4bit(packed, st, out_dtype=torch.float32).t()
    ref = (wd.double() @ x.double().reshape(K, 1)).reshape(1, M)
    absdot = (wd.double().abs() @ x.double().abs().reshape(K, 1)).reshape(-1)   # sum of |terms| per row
    del wd
    # two fp32 summation orders of the same products: one fp16 rounding of the output apart, plus
    # the fp32 rounding of partial sums (relative to the terms' magnitude, not to the result)
    d = (gathered.double() - full.reshape(-1).double()).abs()
    bound = torch.finfo(torch.float16).eps * full.reshape(-1).double().abs().clamp_min(2.0 ** -14) + 2.0 ** -20 * absdot
    assert bool((d <= bound).all()), float((d / bound).max())
    assert_close(full.float().cpu().reshape(1, M), ref.cpu().numpy(), torch.float16, f"70B {M}x{K}")
    assert_close(gathered.float().cpu().reshape(1, M), ref.cpu().numpy(), torch.float16, f"70B 8-way {M}x{K}")

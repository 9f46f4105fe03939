"""GPU: LlamaMLP's gate/up projections and act_fn(gate) * up in ONE launch
(qz_gemv_4bit_pair_silu, core.gemv_4bit_pair_silu, modules.linear4bit_silu_pair).

The bar is bit-identity with the grouped launch followed by the separate product -- and with
torch's own F.silu(g) * u on those outputs -- for fp16 (exact and fp16-rounded NF4 codes) and
bf16, FP4 without double quant, with and without a bias and with the absorbed RMSNorm; and a
Llama model whose MLPs run the pair launch decodes bit-identical logits to transformers' MLP.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


@pytest.fixture
def knobs():
    """qz_gemv_set_knob (the library reads its environment once, at load); the defaults come back after."""
    from quantizations_amd import _lib

    yield _lib.set_gemv_knob
    for name, v in (("QZ_PAIR_PS", -1), ("QZ_PAIR_WT", 1), ("QZ_PAIR_R", 0), ("QZ_PAIR_WK1", 2)):
        _lib.set_gemv_knob(name, v)


def _items(M, K, dtype, seed, quant="nf4", dq=True, bias=False):
    from quantizations_amd.core import quantize_4bit

    g = torch.Generator(device="cuda").manual_seed(seed)
    items = []
    for _ in range(2):
        W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(dtype)
        packed, st = quantize_4bit(W, quant_type=quant, compress_statistics=dq)
        b = (torch.randn(M, device=DEV, generator=g) * 0.1).to(dtype) if bias else None
        items.append((packed, st, b))
    return items


@pytest.mark.parametrize("dtype,exact", [(torch.float16, True), (torch.float16, None), (torch.bfloat16, None)])
@pytest.mark.parametrize("M,K,norm,bias", [(14336, 4096, True, False), (14336, 4096, False, False),
                                           (3000, 2048, True, True), (4096, 6144, False, True)])
def test_pair_silu_bit_identical_to_grouped_plus_product(dtype, exact, M, K, norm, bias):
    from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu
    from quantizations_amd.layer_ops import silu_mul

    items = _items(M, K, dtype, seed=M + K, bias=bias)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 2).to(dtype)
    nw = (1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).to(dtype) if norm else None
    nrm = (nw, 1e-5) if norm else None
    gate, up = gemv_4bit_grouped(x, items, exact_codes=exact, norm=nrm)
    h = gemv_4bit_pair_silu(x, items, exact_codes=exact, norm=nrm)
    torch.cuda.synchronize()
    assert h is not None and h.shape == gate.shape and h.dtype == dtype
    assert torch.equal(h, silu_mul(gate, up))
    assert torch.equal(h, F.silu(gate) * up)


@pytest.mark.parametrize("ps", [2, 3, 448])
@pytest.mark.filterwarnings("ignore")
@pytest.mark.parametrize("M,norm,bias,dtype", [(14336, True, False, torch.float16), (14336, False, True, torch.float16),
                                               (3002, True, True, torch.float16), (7168, True, False, torch.bfloat16)])
def test_pair_silu_persistent_workgroups_bit_identical(knobs, ps, M, norm, bias, dtype):
    """QZ_PAIR_PS: persistent pair workgroups (ps per CU, or a grid of ps; each taking blocks b, b + grid, ...) give
    the one-workgroup-per-block launch's bits, ragged last block included (K = 4096: two-step waves)."""
    from quantizations_amd.core import gemv_4bit_pair_silu

    K = 4096
    items = _items(M, K, dtype, seed=M + ps, bias=bias)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 2).to(dtype)
    nrm = ((1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).to(dtype), 1e-5) if norm else None
    knobs("QZ_PAIR_PS", 0)
    ref = gemv_4bit_pair_silu(x, items, exact_codes=True if dtype == torch.float16 else None, norm=nrm)
    knobs("QZ_PAIR_PS", ps)
    for wt in (0, 1):   # the 16-copy and the 256-B-entry exact-code tables
        knobs("QZ_PAIR_WT", wt)
        h = gemv_4bit_pair_silu(x, items, exact_codes=True if dtype == torch.float16 else None, norm=nrm)
        torch.cuda.synchronize()
        assert ref is not None and h is not None
        assert torch.equal(h, ref), wt
    knobs("QZ_PAIR_PS", -1)
    knobs("QZ_PAIR_WT", 1)   # the product default
    h = gemv_4bit_pair_silu(x, items, exact_codes=True if dtype == torch.float16 else None, norm=nrm)
    assert torch.equal(h, ref)


def test_pair_silu_persistent_fp4_without_double_quant(knobs):
    """The persistent pair (the default with the fused norm) on the FP4 codebook without double quant."""
    from quantizations_amd.core import gemv_4bit_pair_silu

    items = _items(14336, 4096, torch.float16, seed=21, quant="fp4", dq=False)
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.randn(1, 1, 4096, device=DEV, generator=g).half()
    nrm = ((1.0 + 0.1 * torch.randn(4096, device=DEV, generator=g)).half(), 1e-5)
    knobs("QZ_PAIR_PS", 0)
    ref = gemv_4bit_pair_silu(x, items, norm=nrm)
    knobs("QZ_PAIR_PS", -1)
    assert torch.equal(gemv_4bit_pair_silu(x, items, norm=nrm), ref)


def test_pair_silu_fp4_without_double_quant():
    from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu

    items = _items(4096, 4096, torch.float16, seed=9, quant="fp4", dq=False)
    x = torch.randn(1, 1, 4096, device=DEV).half()
    gate, up = gemv_4bit_grouped(x, items)
    assert torch.equal(gemv_4bit_pair_silu(x, items), F.silu(gate) * up)


@pytest.mark.parametrize("world,rank", [(8, 3), (2, 1), (4, 0)])
def test_pair_silu_on_row_shards(world, rank):
    """The pair launch on row shards of gate/up (parallel.sharded_silu_pair's local launch:
    block_base addressing; at 8 ranks the geometry is one row per wave, R = 1): bit-identical
    to the grouped launch + product on the same shards AND to the unsharded pair's rows."""
    from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu
    from quantizations_amd.parallel import shard_rows

    M, K = 14336, 4096
    items = _items(M, K, torch.float16, seed=21)
    g = torch.Generator(device="cuda").manual_seed(4)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 2).half()
    nw = (1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).half()
    full = gemv_4bit_pair_silu(x, items, exact_codes=True, norm=(nw, 1e-5))
    shards = [shard_rows(p, st, rank, world) for p, st, _ in items]
    sh_items = [(sh.packed, sh.state, None, sh.block_base) for sh in shards]
    h = gemv_4bit_pair_silu(x, sh_items, exact_codes=True, norm=(nw, 1e-5))
    gate, up = gemv_4bit_grouped(x, sh_items, exact_codes=True, norm=(nw, 1e-5))
    torch.cuda.synchronize()
    r0, r1 = shards[0].r0, shards[0].r1
    assert h is not None and h.shape[-1] == r1 - r0
    assert torch.equal(h, F.silu(gate) * up)
    assert torch.equal(h.reshape(-1), full.reshape(-1)[r0:r1])


def _rel_to_grouped(h, gate, up):
    ref = F.silu(gate.float()) * up.float()
    return ((h.float() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("M,norm,bias,quant,dq", [
    (5000, False, False, "nf4", True), (4098, True, True, "nf4", True),    # ragged last block, bias
    (28672, True, False, "nf4", True),                                     # Llama-3-70B gate/up as decoded
    (4100, False, False, "fp4", False), (4100, True, False, "nf4", False), (4100, False, True, "fp4", True)])
def test_pair_silu_whole_rows_at_k8192(knobs, M, norm, bias, quant, dq):
    """K = 8192, where the grouped launch splits K over two waves: the pair keeps whole rows per wave
    -- the same products in another fp32 summation order, so within fp16 rounding of the grouped
    launch + product.  With a norm it is fused (persistent workgroups): bit-identical to norm launch ->
    pair without norm, which is what QZ_PAIR_WK1=1 runs (the C entry declines, core launches the
    norm first); 0 declines (None, nothing launched)."""
    from quantizations_amd.core import LAST_FORM, gemv_4bit_grouped, gemv_4bit_pair_silu
    from quantizations_amd.layer_ops import rms_norm

    K = 8192
    items = _items(M, K, torch.float16, seed=M, quant=quant, dq=dq, bias=bias)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 2).half()
    nw = (1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).half() if norm else None
    nrm = (nw, 1e-5) if norm else None
    h = gemv_4bit_pair_silu(x, items, exact_codes=True, norm=nrm)
    assert h is not None
    assert LAST_FORM["pair"] == ("pair (norm fused)" if norm else "pair")
    xn = rms_norm(x, nw, 1e-5) if norm else x
    gate, up = gemv_4bit_grouped(xn, items, exact_codes=True)
    assert _rel_to_grouped(h, gate, up) < 2e-3
    if norm:
        assert torch.equal(h, gemv_4bit_pair_silu(xn, items, exact_codes=True))
        knobs("QZ_PAIR_WK1", 1)
        h2 = gemv_4bit_pair_silu(x, items, exact_codes=True, norm=nrm)
        assert LAST_FORM["pair"] == "norm launch + pair" and torch.equal(h2, h)
    knobs("QZ_PAIR_WK1", 0)
    assert gemv_4bit_pair_silu(xn, items, exact_codes=True) is None


def test_pair_silu_whole_rows_for_small_k_split_pairs(knobs):
    """(1000, 6144): R = 1 with K over two waves in the grouped geometry -- whole rows in the pair."""
    from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu

    items = _items(1000, 6144, torch.float16, seed=1000)
    x = torch.randn(1, 1, 6144, device=DEV).half()
    h = gemv_4bit_pair_silu(x, items, exact_codes=True)
    gate, up = gemv_4bit_grouped(x, items, exact_codes=True)
    assert h is not None and _rel_to_grouped(h, gate, up) < 2e-3
    knobs("QZ_PAIR_WK1", 0)
    assert gemv_4bit_pair_silu(x, items, exact_codes=True) is None


def test_pair_silu_declines_what_it_cannot_take():
    """Odd K, fp32 x, unequal shapes: None, nothing launched (the grouped launch + product then run)."""
    from quantizations_amd.core import gemv_4bit_pair_silu

    items = _items(512, 1000, torch.float16, seed=2)
    assert gemv_4bit_pair_silu(torch.randn(1, 1, 1000, device=DEV).half(), items) is None
    items = _items(512, 2048, torch.float32, seed=3)
    assert gemv_4bit_pair_silu(torch.randn(1, 1, 2048, device=DEV), items) is None
    a = _items(512, 2048, torch.float16, seed=4)
    b = _items(256, 2048, torch.float16, seed=5)
    assert gemv_4bit_pair_silu(torch.randn(1, 1, 2048, device=DEV).half(), [a[0], b[0]]) is None


def test_llama_mlp_pair_logits_bit_identical_to_transformers_mlp():
    from transformers import LlamaConfig, LlamaForCausalLM
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import (fuse_layer_ops, fuse_prenorm, fuse_projection_groups,
                                               replace_with_bnb_linear, unfuse_layer_ops)

    cfg = LlamaConfig(hidden_size=2048, intermediate_size=4096, num_hidden_layers=2, num_attention_heads=16,
                      num_key_value_heads=4, vocab_size=512)
    torch.manual_seed(8)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    fuse_projection_groups(model)
    ids = torch.randint(0, 512, (1, 7), device=DEV, generator=torch.Generator(device="cuda").manual_seed(6))

    def decode():
        cache = StaticCache(config=cfg, max_cache_len=24)
        out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(7, device=DEV))
        logits = [out.logits[:, -1].clone()]
        tok = out.logits[:, -1:].argmax(-1)
        for i in range(5):
            pos = torch.tensor([7 + i], device=DEV)
            lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits
            logits.append(lo[:, -1].clone())
            tok = lo[:, -1:].argmax(-1)
        return logits

    try:
        with torch.no_grad():
            fuse_layer_ops(model, mlp=False)     # transformers' LlamaMLP: act_fn(gate) * up in torch
            fuse_prenorm(model)
            ref = decode()
            unfuse_layer_ops(model)
            fuse_layer_ops(model)                # the pair launch (+ residual epilogue)
            fuse_prenorm(model)
            got = decode()
            assert all(torch.equal(a, b) for a, b in zip(got, ref))
    finally:
        unfuse_layer_ops(model)


@pytest.mark.parametrize("M,norm", [(28672, True), (3584, True), (28672, False)])
def test_pair_silu_k8192_against_fp64(M, norm):
    """K = 8192 (Llama-3-70B gate/up, whole and its 8-way row shard): the pair launch keeps whole rows
    per wave (the grouped launch splits K over two waves there, so the two differ in fp32 summation
    order) -- held to the fp64 product of the bit-exact dequantised weights through the norm and SiLU,
    within fp16 rounding; persistent workgroups and the step loop where the norm rides in it."""
    from quantizations_amd.core import dequantize_4bit, gemv_4bit_pair_silu

    K = 8192
    items = _items(M, K, torch.float16, seed=M + 1)
    g = torch.Generator(device="cuda").manual_seed(11)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 2).half()
    nw = (1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).half()
    h = gemv_4bit_pair_silu(x, items, exact_codes=True, norm=(nw, 1e-5) if norm else None)
    torch.cuda.synchronize()
    assert h is not None
    xd = x.double().view(-1)
    if norm:
        xd = (nw.double() * (xd * torch.rsqrt((xd * xd).mean() + 1e-5)).half().double()).half().double()
    gv, uv = [(dequantize_4bit(p, s, out_dtype=torch.float32).t().double() @ xd).half().double() for p, s, _ in items]
    ref = (gv / (1 + torch.exp(-gv))).half().double() * uv
    rel = ((h.double().view(-1) - ref).norm() / ref.norm()).item()
    assert rel < 2e-3, rel

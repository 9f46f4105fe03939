"""GPU parity of the layer ops around the 4-bit projections (csrc/layer_ops.hip)
against transformers' own torch code for the same op.

Bars:
  * rope_qk: bit-exact vs modeling_llama.apply_rotary_pos_emb (torch rounds
    every elementwise op to the storage dtype; the kernel does the same).
  * rms_norm: the fp32 sum of squares is taken in a different order than
    torch's reduction tree, so outputs may differ in the last place: every
    element within 2 ulp of the output dtype (at the output's magnitude) of
    LlamaRMSNorm.forward -- a 1-ulp change of the rounded normalised value,
    times the weight, rounded again -- and >= 99 % of elements bit-identical
    (fp16/bf16); fp32 outputs within 4 ulp.
  * add_rms_norm: the residual sum bit-exact, the norm as rms_norm.
  * silu_mul: vs F.silu(g) * u, >= 99 % bit-identical, all within 2 ulp
    (torch's and the kernel's expf may differ in the last place).
  * tiny Llama with fuse_layer_ops: greedy tokens identical to the unfused
    model, logits rel. err. <= 2e-3, also under HIP-graph capture.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")
DTYPES = (torch.float16, torch.bfloat16, torch.float32)


def _hf_norm(K, dtype, eps=1e-5, seed=0):
    from transformers.models.llama.modeling_llama import LlamaRMSNorm

    torch.manual_seed(seed)
    m = LlamaRMSNorm(K, eps=eps).to(DEV)
    with torch.no_grad():
        m.weight.copy_(1.0 + 0.1 * torch.randn(K))
    return m.to(dtype)


def _ulp_at(y, dtype):
    eps = {torch.float16: 2.0 ** -10, torch.bfloat16: 2.0 ** -7, torch.float32: 2.0 ** -23}[dtype]
    tiny = {torch.float16: 2.0 ** -24, torch.bfloat16: 2.0 ** -133, torch.float32: 2.0 ** -149}[dtype]
    return torch.clamp(y.abs().double() * eps, min=tiny)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(1, 1, 4096), (2, 7, 4096), (3, 5, 1000), (1, 1, 8192), (4096, 256),
                                   (1, 1, 16384), (2, 1, 16392)])   # the register-held kernel's limit, past it
def test_rms_norm_vs_llama_rmsnorm(dtype, shape):
    from quantizations_amd.layer_ops import rms_norm

    K = shape[-1]
    m = _hf_norm(K, dtype)
    x = (torch.randn(shape, device=DEV) * 3).to(dtype)
    with torch.no_grad():
        ref = m(x)
        y = rms_norm(x, m.weight, m.variance_epsilon)
    assert y.dtype == ref.dtype and y.shape == ref.shape
    d = (y.double() - ref.double()).abs()
    # fp16/bf16: a 1-ulp change of the rounded h is scaled by weight and rounded again -> <= 2 ulp of y;
    # fp32: no storage rounding absorbs the rsqrt / sum-order ulps
    ulps = 4 if dtype == torch.float32 else 2
    assert bool((d <= ulps * _ulp_at(ref, dtype)).all()), float(d.max())
    if dtype != torch.float32:
        assert (y == ref).float().mean().item() >= 0.99


def test_rms_norm_strided_rows_and_zero_rows():
    from quantizations_amd.layer_ops import rms_norm

    m = _hf_norm(512, torch.float16)
    base = torch.randn(6, 1024, device=DEV, dtype=torch.float16)
    x = base[:, 256:768]  # row stride 1024 > K, and not 16-B aligned relative to K
    with torch.no_grad():
        ref = m(x)
        y = rms_norm(x, m.weight, m.variance_epsilon)
    assert bool(((y.double() - ref.double()).abs() <= 2 * _ulp_at(ref, torch.float16)).all())
    z = torch.zeros(2, 512, device=DEV, dtype=torch.float16)
    with torch.no_grad():
        assert torch.equal(rms_norm(z, m.weight, m.variance_epsilon), m(z))  # rsqrt(eps) * 0
    e = torch.empty(0, 512, device=DEV, dtype=torch.float16)
    assert rms_norm(e, m.weight, 1e-5).shape == (0, 512)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("B,Hq,Hk,S,D,bcast", [(1, 32, 8, 1, 128, False), (2, 4, 2, 9, 64, False),
                                               (3, 8, 8, 5, 32, True), (1, 6, 2, 300, 128, False)])
def test_rope_qk_bit_exact_vs_apply_rotary_pos_emb(dtype, B, Hq, Hk, S, D, bcast):
    from transformers.models.llama.modeling_llama import apply_rotary_pos_emb

    from quantizations_amd.layer_ops import rope_qk

    g = torch.Generator(device="cpu").manual_seed(B * 100 + S)
    # the layouts HF produces: proj(h).view(B, S, H, D).transpose(1, 2)
    q = (torch.randn(B, S, Hq, D, generator=g) * 4).to(dtype).to(DEV).transpose(1, 2)
    k = (torch.randn(B, S, Hk, D, generator=g) * 4).to(dtype).to(DEV).transpose(1, 2)
    ang = torch.rand(1 if bcast else B, S, D // 2, generator=g) * 50
    emb = torch.cat((ang, ang), dim=-1)
    cos, sin = emb.cos().to(dtype).to(DEV), emb.sin().to(dtype).to(DEV)
    fn = getattr(apply_rotary_pos_emb, "_qz_orig", apply_rotary_pos_emb)
    qr, kr = fn(q, k, cos, sin)
    qo, ko = rope_qk(q, k, cos, sin)
    assert torch.equal(qo, qr) and torch.equal(ko, kr)
    assert qo.stride() == q.stride()  # torch's elementwise ops keep the transposed layout too


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(1, 1, 14336), (4, 1, 14336), (2, 9, 1000), (3, 333), (1, 1, 28672), (1, 1, 36)])
def test_silu_mul_vs_torch(dtype, shape):
    from quantizations_amd.layer_ops import silu_mul

    g = (torch.randn(shape, device=DEV) * 4).to(dtype)
    u = (torch.randn(shape, device=DEV) * 4).to(dtype)
    ref = torch.nn.functional.silu(g) * u
    y = silu_mul(g, u)
    # bit-exact where the device expf agrees with torch's; at most 1 ulp of silu(g) (times u) otherwise
    d = (y.double() - ref.double()).abs()
    assert bool((d <= 2 * _ulp_at(ref, dtype) + 1e-30).all()), float(d.max())
    assert (y == ref).float().mean().item() >= 0.99


@pytest.mark.parametrize("dtype", DTYPES)
def test_silu_mul_vector_and_scalar_kernels_agree(dtype):
    """16-B aligned operands take the vector kernel, an offset view the per-element one: same bits."""
    from quantizations_amd.layer_ops import silu_mul

    n = 28672
    g = (torch.randn(n + 1, device=DEV) * 4).to(dtype)
    u = (torch.randn(n + 1, device=DEV) * 4).to(dtype)
    a = silu_mul(g[1:], u[1:])              # 2- or 4-byte offset: scalar kernel
    b = silu_mul(g[1:].clone(), u[1:].clone())
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(1, 1, 4096), (4, 1, 4096), (2, 9, 1000)])
def test_add_rms_norm_vs_residual_add_and_llama_rmsnorm(dtype, shape):
    from quantizations_amd.layer_ops import add_rms_norm

    K = shape[-1]
    m = _hf_norm(K, dtype)
    x = (torch.randn(shape, device=DEV) * 3).to(dtype)
    r = (torch.randn(shape, device=DEV) * 3).to(dtype)
    with torch.no_grad():
        s_ref = r + x
        y_ref = m(s_ref)
        s, y = add_rms_norm(x, r, m.weight, m.variance_epsilon)
    assert torch.equal(s, s_ref)  # the residual stream is bit-exact
    d = (y.double() - y_ref.double()).abs()
    ulps = 4 if dtype == torch.float32 else 2
    assert bool((d <= ulps * _ulp_at(y_ref, dtype)).all()), float(d.max())


def _tiny_llama(seed=3):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import fuse_projection_groups, replace_with_bnb_linear

    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(seed)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    fuse_projection_groups(model)
    return model, cfg


def test_tiny_llama_fuse_layer_ops_decode_and_graph():
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import fuse_layer_ops, unfuse_layer_ops

    model, cfg = _tiny_llama()
    ids = torch.randint(0, 512, (1, 10), device=DEV)

    def greedy(n):
        cache = StaticCache(config=cfg, max_cache_len=32)
        out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(10, device=DEV))
        toks, logits = [], [out.logits[:, -1].float()]
        tok = out.logits[:, -1:].argmax(-1)
        for i in range(n):
            pos = torch.tensor([10 + i], device=DEV)
            lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits
            logits.append(lo[:, -1].float())
            tok = lo[:, -1:].argmax(-1)
            toks.append(tok)
        return torch.cat(toks, 1), logits

    def graph_logits(tok0):
        # one decode step captured into a HIP graph (the bench layout), replayed once
        cache = StaticCache(config=cfg, max_cache_len=32)
        model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(10, device=DEV))
        tok = tok0.clone()
        pos = torch.tensor([10], device=DEV)

        def step():
            return model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            out = step()
        gph.replay()
        torch.cuda.synchronize()
        return out[:, -1].float().clone()

    with torch.no_grad():
        ref_toks, ref_logits = greedy(6)
        ref_graph = graph_logits(ref_toks[:, :1])
        n = fuse_layer_ops(model, decoder=True)
        # 2 norms + MLP + decoder layer + attention module each, final norm, rope
        assert n == 5 * cfg.num_hidden_layers + 1 + 1
        toks, logits = greedy(6)
        assert torch.equal(toks, ref_toks)
        for a, b in zip(logits, ref_logits):
            assert ((a - b).norm() / b.norm()).item() <= 2e-3
        got_graph = graph_logits(ref_toks[:, :1])
        assert ((got_graph - ref_graph).norm() / ref_graph.norm()).item() <= 2e-3
        unfuse_layer_ops(model)
        toks2, _ = greedy(6)
        assert torch.equal(toks2, ref_toks)

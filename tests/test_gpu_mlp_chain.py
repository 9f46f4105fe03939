"""GPU: a Llama decoder layer's MLP half -- o_proj + residual, the post-attention RMSNorm,
gate/up + SiLU, down_proj + residual -- as ONE persistent launch (csrc/chain.hip,
core.gemv_4bit_mlp_chain, integration._mlp_chain).

The bar is bit-identity with the three launches it replaces (qz_gemv_4bit_residual ->
qz_gemv_4bit_pair_silu with the fused norm -> qz_gemv_4bit_residual), which are themselves checked
against the CPU oracle (test_gpu_parity.py, test_gpu_mlp_pair.py, test_gpu_residual.py): fp16 with
the exact and the fp16-rounded NF4 codes, bf16, FP4 without double quant, K-step counts 1..7 (every
tail of the step loop), repeated calls (the epoch of the grid barriers) and HIP-graph replays; at
K = 8192, where the three-launch form splits K over two waves, the chain is checked against an fp64
product of the bit-exact dequantised weights.  A Llama model decodes the same tokens and logits
with the chain as without it."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _layer(H, I, dtype, seed, quant="nf4", dq=True):
    from quantizations_amd.core import quantize_4bit

    g = torch.Generator(device="cuda").manual_seed(seed)
    items = {}
    for name, (M, K) in (("o", (H, H)), ("gate", (I, H)), ("up", (I, H)), ("down", (H, I))):
        W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(dtype)
        packed, st = quantize_4bit(W, quant_type=quant, compress_statistics=dq)
        items[name] = (packed, st, None)
    x = (torch.randn(1, 1, H, device=DEV, generator=g) * 2).to(dtype)
    res = torch.randn(1, 1, H, device=DEV, generator=g).to(dtype)
    nw = (1.0 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(dtype)
    return items, x, res, nw


def _three_launches(items, x, res, nw, exact):
    from quantizations_amd.core import gemv_4bit, gemv_4bit_pair_silu

    o, g, u, d = items["o"], items["gate"], items["up"], items["down"]
    h1 = gemv_4bit(x, o[0], state=o[1], exact_codes=exact, residual=res.view(-1))
    act = gemv_4bit_pair_silu(h1, [g, u], exact_codes=exact, norm=(nw, 1e-5))
    assert act is not None
    return gemv_4bit(act, d[0], state=d[1], exact_codes=exact, residual=h1.view(-1))


def _chain(items, x, res, nw, exact, state):
    from quantizations_amd.core import gemv_4bit_mlp_chain

    return gemv_4bit_mlp_chain(x, res, items["o"], items["gate"], items["up"], items["down"], (nw, 1e-5), state,
                               exact_codes=exact)


@pytest.mark.parametrize("H,I,dtype,exact,quant,dq", [
    (4096, 14336, torch.float16, True, "nf4", True),     # Llama-3-8B, the bench's exact codes
    (4096, 14336, torch.float16, None, "nf4", True),     # fp16-rounded codes
    (4096, 14336, torch.bfloat16, None, "nf4", True),
    (4096, 14336, torch.float16, None, "fp4", False),    # config #3's codebook, fp32 absmax
    (2048, 6144, torch.float16, True, "nf4", True),      # 1-step o / gate / up, 3-step down
    (4096, 2048, torch.float16, True, "nf4", True),      # 1-step down
    (2048, 10240, torch.bfloat16, None, "nf4", True),    # 5-step down
])
def test_mlp_chain_bit_identical_to_three_launches(H, I, dtype, exact, quant, dq):
    from quantizations_amd.core import mlp_chain_failed, mlp_chain_state

    items, x, res, nw = _layer(H, I, dtype, seed=H + I, quant=quant, dq=dq)
    ref = _three_launches(items, x, res, nw, exact)
    st = mlp_chain_state(DEV)
    for _ in range(3):   # epochs 0, 1, 2 of the grid barriers
        out = _chain(items, x, res, nw, exact, st)
        torch.cuda.synchronize()
        assert out is not None and out.shape == res.shape and out.dtype == dtype
        assert torch.equal(out, ref)
    assert not mlp_chain_failed(st)
    assert int(st[0].item()) == 3   # the epoch word counts completed launches


def test_mlp_chain_graph_replays_and_changing_inputs():
    """Captured once, replayed with new inputs each time: every replay equals the three launches."""
    from quantizations_amd.core import mlp_chain_failed, mlp_chain_state

    H, I = 4096, 14336
    items, x, res, nw = _layer(H, I, torch.float16, seed=77)
    st = mlp_chain_state(DEV)
    xs, rs = x.clone(), res.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _chain(items, xs, rs, nw, True, st)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = _chain(items, xs, rs, nw, True, st)
    gen = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(4):
        xs.copy_(torch.randn(xs.shape, device=DEV, generator=gen).half())
        rs.copy_(torch.randn(rs.shape, device=DEV, generator=gen).half())
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, _three_launches(items, xs, rs, nw, True))
    assert not mlp_chain_failed(st)


def test_mlp_chain_70b_width_against_fp64():
    """K = 8192 (Llama-3-70B's width, the normed stage at its 8192 maximum): the three-launch form
    splits K over two waves there, so the chain (whole rows per wave) is held to the fp64 product
    of the bit-exact dequantised weights, through the norm and the SiLU, within fp16 rounding."""
    from quantizations_amd.core import dequantize_4bit, mlp_chain_failed, mlp_chain_state

    H, I = 8192, 4096
    items, x, res, nw = _layer(H, I, torch.float16, seed=8192)
    st = mlp_chain_state(DEV)
    out = _chain(items, x, res, nw, True, st)
    torch.cuda.synchronize()
    assert out is not None and not mlp_chain_failed(st)

    def W(name):
        p, s, _ = items[name]
        return dequantize_4bit(p, s, out_dtype=torch.float32).t().double()   # [M, K]
    h1 = (res.double().view(-1) + (W("o") @ x.double().view(-1)).half().double()).half()
    h1d = h1.double()
    var = (h1d * h1d).mean()
    xn = (nw.double() * (h1d * torch.rsqrt(var + 1e-5)).half().double()).half().double()
    gv, uv = (W("gate") @ xn).half().double(), (W("up") @ xn).half().double()
    act = ((gv / (1 + torch.exp(-gv))).half().double() * uv).half().double()
    ref = (h1d + (W("down") @ act).half().double())
    got = out.double().view(-1)
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 2e-3, rel


def _model(dtype, layers=2):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import replace_with_bnb_linear

    cfg = LlamaConfig(hidden_size=2048, intermediate_size=6144, num_hidden_layers=layers, num_attention_heads=16,
                      num_key_value_heads=4, vocab_size=2048, max_position_embeddings=256)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).to(dtype).to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    return cfg, model


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_llama_decode_with_the_chain_equals_three_launches(dtype):
    """bench.py's decode loop (HIP graph) on a Llama whose decoder layers run the chain, against the
    same model with the chain switched off: identical greedy tokens; the chain ran in every layer."""
    import bench
    import quantizations_amd.integration as integ

    cfg, model = _model(dtype)
    bench.prepare_decode_model(model, 0, 1, False, mlp_chain=True)
    calls = {"n": 0}
    orig = integ._mlp_chain

    def spy(layer, x, r):
        out = orig(layer, x, r)
        calls["n"] += out is not None
        return out
    integ._mlp_chain = spy
    try:
        _, hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    finally:
        integ._mlp_chain = orig
    assert calls["n"] >= cfg.num_hidden_layers, calls
    for lay in model.model.layers:
        lay.__dict__["_qz_mlp_chain"] = False
    _, ref_hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    assert torch.equal(hist, ref_hist)
    for lay in model.model.layers:
        st = lay.__dict__.get("_qz_chain_state")
        assert st is not None and not bool(st[-32].item())


def test_llama_single_token_logits_identical():
    """One cached decode step, eager: the chained layers give the three-launch logits bit for bit."""
    import bench

    cfg, model = _model(torch.float16, layers=3)
    bench.prepare_decode_model(model, 0, 1, False, mlp_chain=True)
    ids = torch.randint(0, cfg.vocab_size, (1, 10), generator=torch.Generator().manual_seed(3)).to(DEV)
    from transformers.cache_utils import StaticCache

    def step(chain):
        for lay in model.model.layers:
            lay.__dict__["_qz_mlp_chain"] = chain
        cache = StaticCache(config=cfg, max_cache_len=16)
        with torch.inference_mode():
            model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(10, device=DEV), use_cache=True)
            pos = torch.tensor([10], device=DEV)
            return model(input_ids=ids[:, -1:], past_key_values=cache, cache_position=pos,
                         position_ids=pos.view(1, 1), use_cache=True).logits
    a, b = step(True), step(False)
    assert torch.equal(a, b)

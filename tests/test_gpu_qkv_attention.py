"""GPU: a decode token's q/k/v projections and its attention as ONE launch (csrc/qkv_attn.hip,
core.gemv_4bit_qkv_attention, integration._qkv_attention): every query head's attention runs in the
q/k/v GEMV launch, by the last workgroup that stored the head's rows.

The bar is bit-identity with the two launches it replaces -- gemv_4bit_grouped (with the absorbed
input RMSNorm) then layer_ops.decode_attention, each checked against the CPU oracle / torch
elsewhere (test_gpu_prenorm.py, test_gpu_decode_attention.py): the attention output, the cache rows
written and the advanced position, over consecutive decode steps (the counters re-arm themselves),
fp16 with exact and fp16-rounded NF4 codes, bf16, FP4 without double quant, D = 128 and 64, with and
without the norm, inside HIP-graph replays, and a Llama decode with identical tokens."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _setup(H, Hq, Hkv, D, L, dtype, seed, quant="nf4", dq=True):
    from quantizations_amd.core import quantize_4bit

    g = torch.Generator(device="cuda").manual_seed(seed)
    items = []
    for M in (Hq * D, Hkv * D, Hkv * D):
        W = (torch.randn(M, H, device=DEV, generator=g) * 0.02).to(dtype)
        packed, st = quantize_4bit(W, quant_type=quant, compress_statistics=dq)
        items.append((packed, st, None))
    kc = torch.randn(1, Hkv, L, D, device=DEV, generator=g).to(dtype)
    vc = torch.randn(1, Hkv, L, D, device=DEV, generator=g).to(dtype)
    cos = torch.rand(1, 1, D, device=DEV, generator=g).to(dtype)
    sin = torch.rand(1, 1, D, device=DEV, generator=g).to(dtype)
    nw = (1.0 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(dtype)
    return items, kc, vc, cos, sin, nw


def _two_launches(x, items, norm, cos, sin, kc, vc, mask, pos, Hq, exact):
    from quantizations_amd.core import gemv_4bit_grouped
    from quantizations_amd.layer_ops import decode_attention

    q, k, v = gemv_4bit_grouped(x, items, exact_codes=exact, norm=norm)
    arrive = torch.zeros(1, dtype=torch.int32, device=DEV)
    D = kc.shape[-1]
    return decode_attention(q.view(1, 1, -1), k.view(1, 1, -1), v.view(1, 1, -1), cos, sin, kc, vc, mask, pos, arrive,
                            Hq, D ** -0.5)


@pytest.mark.parametrize("H,Hq,Hkv,D,L,dtype,exact,quant,dq,norm", [
    (4096, 32, 8, 128, 112, torch.float16, True, "nf4", True, True),     # Llama-3-8B, the bench's codes
    (4096, 32, 8, 128, 128, torch.float16, None, "nf4", True, True),     # fp16-rounded codes, L at the limit
    (4096, 32, 8, 128, 64, torch.bfloat16, None, "nf4", True, True),
    (4096, 32, 8, 128, 100, torch.float16, None, "fp4", False, False),   # config #3's codebook, no norm
    (4096, 32, 4, 128, 40, torch.float16, True, "nf4", True, False),     # 8 query heads per kv head
    (4096, 64, 8, 64, 96, torch.float16, True, "nf4", True, True),       # D = 64
])
def test_qkv_attention_bit_identical_to_two_launches(H, Hq, Hkv, D, L, dtype, exact, quant, dq, norm):
    from quantizations_amd.core import gemv_4bit_qkv_attention, qkv_attention_failed, qkv_attention_state

    items, kc, vc, cos, sin, nw = _setup(H, Hq, Hkv, D, L, dtype, seed=H + L, quant=quant, dq=dq)
    nrm = (nw, 1e-5) if norm else None
    kc2, vc2 = kc.clone(), vc.clone()
    p0 = L - 5
    pos, pos2 = (torch.tensor([p0], dtype=torch.int64, device=DEV) for _ in range(2))
    st = qkv_attention_state(Hq, Hkv, DEV)
    g = torch.Generator(device="cuda").manual_seed(7)
    for step in range(6):     # the last step writes past the cache end: NaN output, position kept
        mask = torch.zeros(1, 1, 1, L, dtype=torch.bool, device=DEV)
        mask[..., : min(p0 + step + 1, L)] = True
        x = (torch.randn(1, 1, H, device=DEV, generator=g) * 2).to(dtype)
        ref = _two_launches(x, items, nrm, cos, sin, kc, vc, mask, pos, Hq, exact)
        out = gemv_4bit_qkv_attention(x, items, nrm, cos, sin, kc2, vc2, mask, pos2, st, Hq, D ** -0.5,
                                      exact_codes=exact)
        torch.cuda.synchronize()
        assert out is not None and out.shape == ref.shape and out.dtype == dtype
        assert torch.equal(out, ref) or (torch.isnan(ref).all() and torch.isnan(out).all())
        assert torch.equal(kc2, kc) and torch.equal(vc2, vc)
        assert int(pos2.item()) == int(pos.item())
        assert int(st.sum().item()) == 0          # every counter re-armed
    assert not qkv_attention_failed(st, Hq, Hkv)


def test_qkv_attention_graph_replays():
    """Captured once, replayed over consecutive positions with new inputs: every replay equals the
    two launches (run eagerly on copies)."""
    from quantizations_amd.core import gemv_4bit_qkv_attention, qkv_attention_state

    H, Hq, Hkv, D, L = 4096, 32, 8, 128, 112
    items, kc, vc, cos, sin, nw = _setup(H, Hq, Hkv, D, L, torch.float16, seed=3)
    kc2, vc2 = kc.clone(), vc.clone()
    pos = torch.tensor([20], dtype=torch.int64, device=DEV)
    pos2 = pos.clone()
    mask = torch.ones(1, 1, 1, L, dtype=torch.bool, device=DEV)
    st = qkv_attention_state(Hq, Hkv, DEV)
    xs = torch.randn(1, 1, H, device=DEV).half()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up call (advances pos2 by one; the reference follows)
        gemv_4bit_qkv_attention(xs, items, (nw, 1e-5), cos, sin, kc2, vc2, mask, pos2, st, Hq, D ** -0.5,
                                exact_codes=True)
    torch.cuda.current_stream().wait_stream(s)
    _two_launches(xs, items, (nw, 1e-5), cos, sin, kc, vc, mask, pos, Hq, True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = gemv_4bit_qkv_attention(xs, items, (nw, 1e-5), cos, sin, kc2, vc2, mask, pos2, st, Hq, D ** -0.5,
                                      exact_codes=True)
    gen = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(4):
        xs.copy_(torch.randn(xs.shape, device=DEV, generator=gen).half())
        graph.replay()
        ref = _two_launches(xs, items, (nw, 1e-5), cos, sin, kc, vc, mask, pos, Hq, True)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        assert torch.equal(kc2, kc) and torch.equal(vc2, vc) and int(pos2.item()) == int(pos.item())


def test_qkv_attention_declines_what_it_cannot_take():
    """A cache longer than one key chunk (L > 128) or two sequences: None, nothing launched."""
    from quantizations_amd.core import gemv_4bit_qkv_attention, qkv_attention_state

    H, Hq, Hkv, D = 2048, 16, 4, 128
    items, kc, vc, cos, sin, _ = _setup(H, Hq, Hkv, D, 200, torch.float16, seed=5)
    pos = torch.tensor([10], dtype=torch.int64, device=DEV)
    st = qkv_attention_state(Hq, Hkv, DEV)
    mask = torch.ones(1, 1, 1, 200, dtype=torch.bool, device=DEV)
    x = torch.randn(1, 1, H, device=DEV).half()
    assert gemv_4bit_qkv_attention(x, items, None, cos, sin, kc, vc, mask, pos, st, Hq, D ** -0.5) is None
    assert int(pos.item()) == 10


def _model(dtype, layers=2):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import replace_with_bnb_linear

    # 4096 wide (32 / 8 heads of 128): the q/k/v geometry keeps row pairs per wave, which the fused
    # launch needs (a narrower model's 1-row waves take the two launches)
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=4096, num_hidden_layers=layers, num_attention_heads=32,
                      num_key_value_heads=8, vocab_size=2048, max_position_embeddings=256)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).to(dtype).to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    return cfg, model


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_llama_decode_with_qkv_attention_equals_two_launches(dtype):
    """bench.py's decode loop (HIP graph) with the fused q/k/v + attention launch in every layer (opt-in),
    against the same model with it switched off: identical greedy tokens; the fused launch ran."""
    import bench
    import quantizations_amd.integration as integ

    cfg, model = _model(dtype)
    bench.prepare_decode_model(model, 0, 1, False, qkv_attention=True)
    calls = {"n": 0}
    orig = integ._qkv_attention

    def spy(*a, **k):
        out = orig(*a, **k)
        calls["n"] += out is not None
        return out
    integ._qkv_attention = spy
    try:
        _, hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    finally:
        integ._qkv_attention = orig
    assert calls["n"] >= cfg.num_hidden_layers, calls
    for m in model.modules():
        if "_qz_qkv_attn" in m.__dict__:
            m.__dict__["_qz_qkv_attn"] = False
    _, ref_hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    assert torch.equal(hist, ref_hist)

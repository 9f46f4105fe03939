"""GPU: one-launch decode attention against a static KV cache (qz_decode_attention,
layer_ops.decode_attention, integration.fuse_layer_ops(attention=True)).

What it replaces -- transformers' apply_rotary_pos_emb, StaticLayer.update and
sdpa_attention_forward for one new token -- is restated here in torch:
  * the cache row written at position p must be bit-identical to the rotated k of the
    torch rotary expression, the new v copied, every other row untouched, p advanced by 1;
  * the attention output must match an fp64 softmax(q k^T * scale) v over the masked
    positions within 2 ulp-ish of the 16-bit output (atol/rtol 2e-3 fp16, 1e-2 bf16) --
    the kernel keeps scores and probabilities in fp32 where SDPA's flash kernel rounds the
    probabilities to 16 bits, so the two agree to that bound, not bitwise;
  * a Llama model decodes the same greedy tokens with and without the fused attention and
    its HIP-graph replay equals its eager step bitwise.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _rotate_half(x):
    x1, x2 = x[..., : x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def _case(B, Hq, Hkv, D, L, p, dtype, holes=False, seed=0, batch_mask=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    q = torch.randn(B, 1, Hq * D, device=DEV, generator=g).to(dtype)
    k = torch.randn(B, 1, Hkv * D, device=DEV, generator=g).to(dtype)
    v = torch.randn(B, 1, Hkv * D, device=DEV, generator=g).to(dtype)
    ang = torch.rand(B if batch_mask else 1, 1, D // 2, device=DEV, generator=g) * 6.0
    cos = torch.cat((ang.cos(), ang.cos()), -1).to(dtype)
    sin = torch.cat((ang.sin(), ang.sin()), -1).to(dtype)
    kc = torch.randn(B, Hkv, L, D, device=DEV, generator=g).to(dtype)
    vc = torch.randn(B, Hkv, L, D, device=DEV, generator=g).to(dtype)
    mask = torch.zeros(B if batch_mask else 1, 1, 1, L, dtype=torch.bool, device=DEV)
    mask[..., : p + 1] = True
    if holes:
        mask &= torch.rand(mask.shape, device=DEV, generator=g) > 0.3
        mask[..., p] = True
    pos = torch.tensor(p, dtype=torch.int64, device=DEV)
    return q, k, v, cos, sin, kc, vc, mask, pos


def _reference(q, k, v, cos, sin, kc, vc, mask, p, Hq):
    B, Hkv, L, D = kc.shape
    qh = q.view(B, 1, Hq, D).transpose(1, 2)
    kh = k.view(B, 1, Hkv, D).transpose(1, 2)
    c, s = cos.unsqueeze(1), sin.unsqueeze(1)
    qr = (qh * c) + (_rotate_half(qh) * s)        # apply_rotary_pos_emb, torch's own rounding
    kr = (kh * c) + (_rotate_half(kh) * s)
    kc2, vc2 = kc.clone(), vc.clone()
    kc2[:, :, p] = kr[:, :, 0]
    vc2[:, :, p] = v.view(B, Hkv, D)
    G = Hq // Hkv
    kk = kc2.double().repeat_interleave(G, dim=1)
    vv = vc2.double().repeat_interleave(G, dim=1)
    sc = (qr.double() @ kk.transpose(-1, -2)) * (1.0 / math.sqrt(D))
    sc = sc.masked_fill(~mask.expand(B, 1, 1, L), float("-inf"))
    o = torch.softmax(sc, dim=-1) @ vv                     # [B, Hq, 1, D]
    return o.transpose(1, 2).reshape(B, 1, Hq * D), kc2, vc2


CASES = [  # B, Hq, Hkv, D, L, p, holes
    (1, 32, 8, 128, 112, 40, False),      # the bench's Llama-3-8B cache: one chunk
    (1, 32, 8, 128, 128, 127, False),     # the last position of a full chunk
    (1, 32, 8, 128, 129, 128, False),     # two chunks, p alone in the second
    (1, 32, 8, 128, 1000, 517, True),     # eight chunks, masked holes, chunks past p
    (2, 8, 8, 64, 300, 257, True),        # MHA, D = 64, per-sequence masks
    (1, 64, 8, 128, 400, 399, False),     # G = 8 (Llama-3-70B)
    (3, 28, 4, 128, 50, 0, False),        # G = 7, the first token
]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,Hq,Hkv,D,L,p,holes", CASES)
def test_decode_attention_matches_rope_cache_update_and_softmax(dtype, B, Hq, Hkv, D, L, p, holes):
    from quantizations_amd.layer_ops import decode_attention

    q, k, v, cos, sin, kc, vc, mask, pos = _case(B, Hq, Hkv, D, L, p, dtype, holes=holes, seed=L + p,
                                                 batch_mask=B > 1)
    ref, kc_ref, vc_ref = _reference(q, k, v, cos, sin, kc, vc, mask, p, Hq)
    arrive = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = decode_attention(q, k, v, cos, sin, kc, vc, mask, pos, arrive, Hq, 1.0 / math.sqrt(D))
    torch.cuda.synchronize()
    assert torch.equal(kc, kc_ref), "cache keys: row p must be the rotated k bit-exactly, other rows untouched"
    assert torch.equal(vc, vc_ref)
    assert int(pos) == p + 1 and int(arrive) == 0
    tol = 2e-3 if dtype == torch.float16 else 1e-2
    torch.testing.assert_close(out.double(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize("L", [112, 300])   # one chunk / three chunks (the combine launch)
def test_decode_attention_full_cache_is_loud(L):
    """One token past max_cache_len: HF's StaticLayer.update fails on the out-of-range
    index_copy_; the fused launch has no slot either, so its output is NaN, the cache is
    untouched and the position stays at L (never a silently stale output)."""
    from quantizations_amd.layer_ops import decode_attention

    q, k, v, cos, sin, kc, vc, mask, pos = _case(1, 32, 8, 128, L, L - 1, torch.float16, seed=11)
    pos.fill_(L)
    kc0, vc0 = kc.clone(), vc.clone()
    arrive = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = decode_attention(q, k, v, cos, sin, kc, vc, mask, pos, arrive, 32, 1.0 / math.sqrt(128))
    torch.cuda.synchronize()
    assert torch.isnan(out).all()
    assert torch.equal(kc, kc0) and torch.equal(vc, vc0)
    assert int(pos) == L and int(arrive) == 0


def test_decode_attention_consecutive_steps_and_sdpa():
    """Two steps in a row (the arrival counter and the position carry over) and the same
    output as torch's own SDPA on the updated cache within fp16 flash-attention tolerance."""
    from quantizations_amd.layer_ops import decode_attention

    B, Hq, Hkv, D, L = 1, 32, 8, 128, 300
    q, k, v, cos, sin, kc, vc, mask, pos = _case(B, Hq, Hkv, D, L, 130, torch.float16, seed=5)
    arrive = torch.zeros(1, dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(D)
    decode_attention(q, k, v, cos, sin, kc, vc, mask, pos, arrive, Hq, scale)
    q2, k2, v2 = (t.roll(7, -1) for t in (q, k, v))
    mask2 = mask.clone()
    mask2[..., 131] = True
    ref, kc_ref, vc_ref = _reference(q2, k2, v2, cos, sin, kc, vc, mask2, 131, Hq)
    out = decode_attention(q2, k2, v2, cos, sin, kc, vc, mask2, pos, arrive, Hq, scale)
    torch.cuda.synchronize()
    assert int(pos) == 132 and int(arrive) == 0
    assert torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref)
    torch.testing.assert_close(out.double(), ref, atol=2e-3, rtol=2e-3)
    qh = q2.view(B, 1, Hq, D).transpose(1, 2)
    qr = qh * cos.unsqueeze(1) + _rotate_half(qh) * sin.unsqueeze(1)
    sd = torch.nn.functional.scaled_dot_product_attention(
        qr, kc.repeat_interleave(Hq // Hkv, 1), vc.repeat_interleave(Hq // Hkv, 1), attn_mask=mask2, scale=scale)
    torch.testing.assert_close(out.float(), sd.transpose(1, 2).reshape(B, 1, Hq * D).float(), atol=4e-3, rtol=4e-3)


def test_decode_attention_rejects_what_it_cannot_take():
    from quantizations_amd import _lib
    from quantizations_amd.layer_ops import decode_attention, decode_attention_supported

    q, k, v, cos, sin, kc, vc, mask, pos = _case(1, 32, 8, 128, 64, 10, torch.float16)
    assert decode_attention_supported(q, cos, kc, vc, mask, pos, 32)
    assert not decode_attention_supported(q.float(), cos, kc, vc, mask, pos, 32)     # fp32 activations
    assert not decode_attention_supported(q, cos, kc, vc, mask.half(), pos, 32)       # additive float mask
    assert not decode_attention_supported(q, cos, kc, vc, mask, pos, 96)              # G = 12 > 8
    kc96 = torch.zeros(1, 8, 64, 96, device=DEV, dtype=torch.float16)
    assert not decode_attention_supported(q, cos, kc96, kc96, mask, pos, 32)           # D = 96
    with pytest.raises(ValueError):
        decode_attention(q, k, v, cos, sin, kc, vc, mask.half(), pos, torch.zeros(1, dtype=torch.int32, device=DEV),
                         32, 0.1)
    rc = _lib.lib.qz_decode_attention(_lib.dtype_code(torch.float16), 1, 32, 8, 96, 64, q.data_ptr(), 32 * 96,
                                      k.data_ptr(), 8 * 96, v.data_ptr(), 8 * 96, cos.data_ptr(), sin.data_ptr(), 0,
                                      kc.data_ptr(), vc.data_ptr(), mask.data_ptr(), 0, 1, pos.data_ptr(),
                                      pos.data_ptr(), q.data_ptr(), 32 * 96, None, 0.1, _lib.stream_of(q))
    assert rc == _lib.QZ_ERR_SHAPE
    assert int(pos) == 10   # nothing ran


def _llama(D=128, seed=11):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import fuse_projection_groups, replace_with_bnb_linear

    cfg = LlamaConfig(hidden_size=16 * D // 2, intermediate_size=2048, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(seed)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    fuse_projection_groups(model)
    return model, cfg


def test_llama_decode_with_fused_attention_greedy_tokens_and_graph():
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import fuse_layer_ops, fuse_prenorm, unfuse_layer_ops

    model, cfg = _llama()
    ids = torch.randint(0, cfg.vocab_size, (1, 12), device=DEV, generator=torch.Generator(device="cuda").manual_seed(2))

    def greedy(n, max_len=40):
        cache = StaticCache(config=cfg, max_cache_len=max_len)
        out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(12, device=DEV))
        tok = out.logits[:, -1:].argmax(-1)
        toks, logits = [], []
        for i in range(n):
            pos = torch.tensor([12 + i], device=DEV)
            lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits
            logits.append(lo[:, -1].float().clone())
            tok = lo[:, -1:].argmax(-1)
            toks.append(tok)
        return torch.cat(toks, 1), logits, cache

    def three_steps(tok0, graph):
        """Steps at positions 12, 13, 14 with a fixed input token; with graph=True the third
        is a HIP-graph replay (captured after the second ran on the capture stream)."""
        cache = StaticCache(config=cfg, max_cache_len=40)
        model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(12, device=DEV))
        tok = tok0.clone()
        pos = torch.tensor([12], device=DEV)

        def step():
            return model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits

        step()
        pos.add_(1)
        if not graph:
            step()
            pos.add_(1)
            out = step()
        else:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            pos.add_(1)
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph):
                out = step()
            gph.replay()
        torch.cuda.synchronize()
        assert all(int(layer.cumulative_length) == 15 for layer in cache.layers)
        return out[:, -1].float().clone()

    try:
        with torch.no_grad():
            fuse_layer_ops(model, attention=False)
            fuse_prenorm(model)
            ref_toks, ref_logits, ref_cache = greedy(10)
            unfuse_layer_ops(model)
            n = fuse_layer_ops(model)
            assert sum("_qz_fused_attn" in m.__dict__ for m in model.modules()) == cfg.num_hidden_layers
            fuse_prenorm(model)
            toks, logits, cache = greedy(10)
            assert torch.equal(toks, ref_toks)
            for a, b in zip(logits, ref_logits):
                assert ((a - b).norm() / b.norm()).item() <= 2e-3
            for lr, lf in zip(ref_cache.layers, cache.layers):   # same cache contents and positions
                assert int(lr.cumulative_length) == int(lf.cumulative_length) == 22
                torch.testing.assert_close(lf.keys.float(), lr.keys.float(), atol=2e-2, rtol=2e-2)
            eager = three_steps(ref_toks[:, :1], graph=False)
            replay = three_steps(ref_toks[:, :1], graph=True)
            assert torch.equal(replay, eager) and n > 0
    finally:
        unfuse_layer_ops(model)

"""GPU: the RMSNorm absorbed into the grouped decode GEMV (qz_gemv_4bit_grouped_rmsnorm,
integration.fuse_prenorm).

The fused launch normalises x in its prologue with k_rmsnorm's exact arithmetic (same
per-thread chunk order, same xor butterfly, same rsqrt and roundings), so the bar is
bit-identity with the two-launch form qz_rmsnorm + qz_gemv_4bit_grouped -- for every
segment, fp16 (fp16-rounded and exact NF4 codes) and bf16 activations, K = 2048..8192 --
and, for a Llama model, bit-identical logits and greedy tokens with and without the
absorption (eager, prefill through the absorbed norm, HIP-graph replay).
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _items(Ms, K, dtype, seed, bias_seg=None, quant="nf4", dq=True):
    from quantizations_amd.core import quantize_4bit

    g = torch.Generator(device="cuda").manual_seed(seed)
    items = []
    for i, M in enumerate(Ms):
        W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(dtype)
        packed, st = quantize_4bit(W, quant_type=quant, compress_statistics=dq)
        b = (torch.randn(M, device=DEV, generator=g) * 0.1).to(dtype) if i == bias_seg else None
        items.append((packed, st, b))
    return items


@pytest.mark.parametrize("dtype,exact", [(torch.float16, None), (torch.float16, True), (torch.bfloat16, None)])
@pytest.mark.parametrize("Ms,K", [((4096, 1024, 1024), 4096), ((14336, 14336), 4096), ((2048, 512, 512), 2048),
                                  ((8192, 1024, 1024), 8192), ((3000, 8), 4096),
                                  ((28672, 28672), 8192)])   # 7168 workgroups: two launches instead
def test_grouped_gemv_rmsnorm_bit_identical_to_two_launches(dtype, exact, Ms, K):
    from quantizations_amd.core import gemv_4bit_grouped
    from quantizations_amd.layer_ops import rms_norm

    items = _items(Ms, K, dtype, seed=K + len(Ms), bias_seg=1)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 3).to(dtype)
    w = (1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).to(dtype)
    eps = 1e-5
    ref = gemv_4bit_grouped(rms_norm(x, w, eps), items, exact_codes=exact)
    got = gemv_4bit_grouped(x, items, exact_codes=exact, norm=(w, eps))
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, ref)):
        assert a.shape == b.shape and a.dtype == b.dtype
        assert torch.equal(a, b), f"segment {i}: {(a.float() - b.float()).abs().max().item()}"


@pytest.mark.parametrize("Ms,K,form", [((512, 128, 128), 4096, "grouped (norm fused)"),     # 8B q/k/v, 8-way shard
                                       ((1024, 128, 128), 8192, "grouped (norm fused)"),    # 70B q/k/v, 8-way shard
                                       ((8192, 1024, 1024), 8192, "norm launch + grouped")])  # 70B q/k/v whole
def test_grouped_rmsnorm_at_k_split_geometries(Ms, K, form):
    """Where K is split over waves: a row shard's q/k/v (few workgroups) keeps the norm fused, the
    whole Llama-3-70B q/k/v (1280 workgroups x 8192 values) takes the norm launch; bit-identical either way."""
    from quantizations_amd.core import LAST_FORM, gemv_4bit_grouped
    from quantizations_amd.layer_ops import rms_norm

    items = _items(Ms, K, torch.float16, seed=K + Ms[0], bias_seg=-1)
    g = torch.Generator(device="cuda").manual_seed(11)
    x = (torch.randn(1, 1, K, device=DEV, generator=g) * 3).half()
    w = (1.0 + 0.1 * torch.randn(K, device=DEV, generator=g)).half()
    ref = gemv_4bit_grouped(rms_norm(x, w, 1e-5), items, exact_codes=True)
    got = gemv_4bit_grouped(x, items, exact_codes=True, norm=(w, 1e-5))
    torch.cuda.synchronize()
    assert LAST_FORM["grouped"] == form
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_grouped_gemv_rmsnorm_fp4_without_double_quant(dtype):
    """Config #3's format (FP4, fp32 absmax): the other scale path of the fused launch."""
    from quantizations_amd.core import gemv_4bit_grouped
    from quantizations_amd.layer_ops import rms_norm

    items = _items((4096, 1024, 1024), 4096, dtype, seed=3, quant="fp4", dq=False)
    x = (torch.randn(1, 1, 4096, device=DEV) * 2).to(dtype)
    w = (1.0 + 0.1 * torch.randn(4096, device=DEV)).to(dtype)
    ref = gemv_4bit_grouped(rms_norm(x, w, 1e-6), items)
    got = gemv_4bit_grouped(x, items, norm=(w, 1e-6))
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_grouped_rmsnorm_entry_rejects_what_it_cannot_fuse():
    """K % 2048 != 0 / misaligned / fp32: QZ_ERR_SHAPE from the C entry, nothing launched;
    the Python wrapper then runs the two launches (same results as calling them itself)."""
    from quantizations_amd import _lib
    from quantizations_amd.core import gemv_4bit_grouped
    from quantizations_amd.layer_ops import rms_norm

    K = 1024
    items = _items((256, 64), K, torch.float16, seed=1)
    x = torch.randn(K, device=DEV).half()
    w = (1.0 + 0.1 * torch.randn(K, device=DEV)).half()
    packed, st, _ = items[0]
    am, qam, am2, code2, off, _ = st.scale_args()
    y = torch.empty(256, device=DEV, dtype=torch.float16)
    segs = (_lib.GemvSegment * 1)()
    segs[0] = _lib.GemvSegment(256, packed.data_ptr(), am, qam, am2, code2, off, 0, None, y.data_ptr())
    rc = _lib.lib.qz_gemv_4bit_grouped_rmsnorm(1, ctypes.cast(segs, ctypes.c_void_p), K, x.data_ptr(),
                                               _lib.dtype_code(x.dtype), _lib.NF4, 64, 256, None, w.data_ptr(), 1e-5,
                                               _lib.stream_of(x))
    assert rc == _lib.QZ_ERR_SHAPE
    ref = gemv_4bit_grouped(rms_norm(x, w, 1e-5), items)
    got = gemv_4bit_grouped(x, items, norm=(w, 1e-5))
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def _llama(seed=5):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import fuse_layer_ops, fuse_projection_groups, replace_with_bnb_linear

    cfg = LlamaConfig(hidden_size=2048, intermediate_size=4096, num_hidden_layers=2, num_attention_heads=16,
                      num_key_value_heads=4, vocab_size=512)
    torch.manual_seed(seed)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    with torch.no_grad():
        for m in model.modules():
            if type(m).__name__ == "LlamaRMSNorm":
                m.weight.copy_(1.0 + 0.1 * torch.randn_like(m.weight.float()).half())
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    fuse_projection_groups(model)
    fuse_layer_ops(model)
    return model, cfg


def test_llama_prenorm_logits_and_tokens_bit_identical_eager_and_graph():
    from quantizations_amd.integration import fuse_prenorm, unfuse_layer_ops, unfuse_prenorm

    model, cfg = _llama()
    try:
        _check_prenorm_model(model, cfg, fuse_prenorm, unfuse_prenorm)
    finally:
        unfuse_layer_ops(model)   # the modeling module's apply_rotary_pos_emb is process-global


def _check_prenorm_model(model, cfg, fuse_prenorm, unfuse_prenorm):
    from transformers.cache_utils import StaticCache

    ids = torch.randint(0, cfg.vocab_size, (1, 10), device=DEV, generator=torch.Generator(device="cuda").manual_seed(3))

    def greedy(n):
        cache = StaticCache(config=cfg, max_cache_len=32)
        out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(10, device=DEV))
        logits = [out.logits[:, -1].clone()]
        tok = out.logits[:, -1:].argmax(-1)
        toks = []
        for i in range(n):
            pos = torch.tensor([10 + i], device=DEV)
            lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits
            logits.append(lo[:, -1].clone())
            tok = lo[:, -1:].argmax(-1)
            toks.append(tok)
        return torch.cat(toks, 1), logits

    def graph_logits(tok0):
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
        return out[:, -1].clone()

    with torch.no_grad():
        ref_toks, ref_logits = greedy(6)
        ref_graph = graph_logits(ref_toks[:, :1])
        n = fuse_prenorm(model)
        assert n == 2 * cfg.num_hidden_layers
        probe = torch.randn(1, 1, cfg.hidden_size, device=DEV).half()
        assert model.model.layers[0].input_layernorm(probe) is probe   # absorbed norms pass x through
        toks, logits = greedy(6)
        assert torch.equal(toks, ref_toks)
        for a, b in zip(logits, ref_logits):   # prefill (norm + group) and decode (fused launch)
            assert torch.equal(a, b)
        assert torch.equal(graph_logits(ref_toks[:, :1]), ref_graph)
        unfuse_prenorm(model)
        toks2, logits2 = greedy(6)
        assert torch.equal(toks2, ref_toks) and torch.equal(logits2[-1], ref_logits[-1])

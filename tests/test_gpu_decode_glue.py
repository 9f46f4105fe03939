"""GPU: the host model's per-step glue (integration.fuse_decode_glue; csrc/layer_ops.hip
k_decode_mask, k_rope_table) -- the causal mask and the rotary cos/sin of a decode step, one launch
each instead of transformers' small torch kernels.  Not the Linear4bit path; the bar is the same
values as transformers' own code: the rotary module's forward (bit-identical inside its table),
create_causal_mask against a StaticCache, and greedy tokens of bench.py's graph decode loop."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


def _cfg(rope, max_pos=256, hidden=256, heads=4, kv=2, layers=2):
    from transformers import LlamaConfig

    kw = dict(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=layers, num_attention_heads=heads,
              num_key_value_heads=kv, vocab_size=1024, max_position_embeddings=max_pos)
    if rope == "llama3":   # Llama-3.1's scaled frequencies
        kw["rope_parameters"] = {"rope_type": "llama3", "rope_theta": 500000.0, "factor": 8.0, "low_freq_factor": 1.0,
                                 "high_freq_factor": 4.0, "original_max_position_embeddings": 64}
    else:
        kw["rope_theta"] = 500000.0
    return LlamaConfig(**kw)


@pytest.mark.parametrize("rope", ["default", "llama3"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_rope_table_equals_rotary_module(rope, dtype):
    from transformers import LlamaForCausalLM

    from quantizations_amd.integration import fuse_decode_glue, unfuse_decode_glue

    cfg = _cfg(rope, max_pos=512)
    model = LlamaForCausalLM(cfg).to(dtype).to(DEV).eval()
    rot = model.model.rotary_emb
    x = torch.empty(0, dtype=dtype, device=DEV)
    g = torch.Generator(device="cpu").manual_seed(3)
    cases = [torch.tensor([[0]]), torch.tensor([[511]]), torch.tensor([[37]]).expand(2, 1),
             torch.randint(0, 512, (3, 5), generator=g), torch.arange(512).unsqueeze(0)]
    refs = [rot(x, position_ids=p.to(DEV)) for p in cases]
    try:
        assert fuse_decode_glue(model) >= 1 and "_qz_rope_orig" in rot.__dict__
        for p, (rc, rs) in zip(cases, refs):
            c, s = rot(x, position_ids=p.to(DEV))
            assert c.dtype == dtype and c.shape == rc.shape
            assert torch.equal(c, rc) and torch.equal(s, rs)
        # outside the table: computed in-kernel (fp32 cosf/sinf), close to the module's values
        far = torch.tensor([[512, 700]], device=DEV)
        c, s = rot(x, position_ids=far)
        rc, rs = rot.__dict__["_qz_rope_orig"](x, far)
        assert torch.allclose(c.float(), rc.float(), atol=2e-3) and torch.allclose(s.float(), rs.float(), atol=2e-3)
    finally:
        unfuse_decode_glue(model)
    assert "forward" not in rot.__dict__


@pytest.mark.parametrize("batch", [1, 2])
def test_decode_mask_equals_create_causal_mask(batch):
    """After a prefill into a StaticCache, each decode step's mask from the fast path equals
    transformers' create_causal_mask (called through the original function)."""
    import sys

    from transformers import LlamaForCausalLM
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import _MASK_PATCHED, fuse_decode_glue, unfuse_decode_glue

    cfg = _cfg("default")
    cfg._attn_implementation = "sdpa"
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    modname = type(model.model).__module__
    try:
        fuse_decode_glue(model)
        assert modname in _MASK_PATCHED
        fast, orig = sys.modules[modname].create_causal_mask, _MASK_PATCHED[modname]
        cache = StaticCache(config=cfg, max_cache_len=80)
        ids = torch.randint(0, 1024, (batch, 9), device=DEV)
        with torch.no_grad():
            out = model(input_ids=ids, past_key_values=cache, use_cache=True)
            tok = out.logits[:, -1:].argmax(-1)
            for step in range(4):
                emb = model.model.embed_tokens(tok)
                pos = torch.full((batch, 1), 9 + step, device=DEV)
                kw = dict(config=cfg, inputs_embeds=emb, attention_mask=None, past_key_values=cache, position_ids=pos)
                got, ref = fast(**kw), orig(**kw)
                assert got.dtype == torch.bool and got.shape == ref.shape == (batch, 1, 1, 80)
                assert torch.equal(got, ref)
                tok = model(input_ids=tok, past_key_values=cache, position_ids=pos, use_cache=True).logits[:, -1:].argmax(-1)
            # a padding mask takes transformers' own path
            am = torch.ones(batch, 9 + 4 + 1, dtype=torch.long, device=DEV)
            kw = dict(config=cfg, inputs_embeds=emb, attention_mask=am, past_key_values=cache, position_ids=pos)
            assert torch.equal(fast(**kw), orig(**kw))
    finally:
        unfuse_decode_glue(model)
    assert modname not in _MASK_PATCHED


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_llama_decode_with_glue_equals_without(dtype):
    """bench.py's graph decode loop with the glue launches (its default) against the same model with
    transformers' own mask and rotary code: identical greedy tokens; the glue kernels ran."""
    from transformers import LlamaForCausalLM

    import bench
    from quantizations_amd import _lib
    from quantizations_amd.integration import replace_with_bnb_linear, unfuse_decode_glue, unfuse_layer_ops

    cfg = _cfg("llama3", max_pos=256, hidden=1024, heads=8, kv=2)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).to(dtype).to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    bench.prepare_decode_model(model, 0, 1, False)
    calls = {"rope": 0, "mask": 0}
    lib = _lib.lib
    rope_fn, mask_fn = lib.qz_rope_table, lib.qz_decode_mask

    def spy(name, fn):
        def f(*a):
            calls[name] += 1
            return fn(*a)
        return f
    lib.qz_rope_table, lib.qz_decode_mask = spy("rope", rope_fn), spy("mask", mask_fn)
    try:
        _, hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    finally:
        lib.qz_rope_table, lib.qz_decode_mask = rope_fn, mask_fn
    assert calls["rope"] >= 1 and calls["mask"] >= 1, calls
    unfuse_decode_glue(model)
    try:
        _, ref_hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    finally:
        unfuse_layer_ops(model)   # module-level patches (apply_rotary_pos_emb) must not leak into later tests
    assert torch.equal(hist, ref_hist)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,V", [(1, 128256), (2, 128256), (1, 1000), (3, 37), (1, 5)])
def test_greedy_step_is_torch_argmax_and_feedback(dtype, B, V):
    """layer_ops.greedy_step against torch.argmax + index_copy_ + copy_ + add_ (bench.py's loop):
    random logits, ties (first index wins), -inf rows, NaN (wins, first one), a strided row view."""
    from quantizations_amd.layer_ops import greedy_step

    g = torch.Generator(device="cuda").manual_seed(V + B)
    cases = []
    lo = torch.randn(B, 1, V, device=DEV, generator=g).to(dtype)
    cases.append(lo)
    t = lo.clone()
    t[..., V // 3] = 50.0
    t[..., V - 1] = 50.0           # tie: the first index
    cases.append(t)
    t = torch.full((B, 1, V), float("-inf"), device=DEV, dtype=dtype)
    cases.append(t)                # all -inf: index 0
    t = lo.clone()
    t[..., V // 2] = float("nan")
    t[..., V - 1] = float("nan")   # NaN beats every number, the first NaN wins
    cases.append(t)
    wide = torch.randn(B, 1, V + 24, device=DEV, generator=g).to(dtype)
    cases.append(wide[..., 8:8 + V])   # rows of stride V + 24, offset 8 elements
    H = 16
    for i, c in enumerate(cases):
        hist = torch.randint(0, 9, (B, H), device=DEV, generator=g)
        pos = torch.tensor([3 + i], device=DEV)
        tok = torch.zeros(B, 1, dtype=torch.int64, device=DEV)
        hist_r, pos_r, tok_r = hist.clone(), pos.clone(), tok.clone()
        nxt = c[:, -1:].argmax(-1)
        hist_r.index_copy_(1, pos_r, nxt.view(B, 1))
        tok_r.copy_(nxt)
        pos_r.add_(1)
        greedy_step(c[:, -1], hist, pos, tok)
        torch.cuda.synchronize()
        assert torch.equal(tok, tok_r), (i, tok, tok_r)
        assert torch.equal(hist, hist_r) and torch.equal(pos, pos_r)


@pytest.mark.parametrize("B", [1, 2])
def test_greedy_step_position_past_history(B):
    """pos == H (a graph replayed once more than hist has columns): nothing is written at column H
    -- the next row's first entry, or the guard words after the last row -- while tok and pos still
    advance."""
    from quantizations_amd.layer_ops import greedy_step

    H, V = 8, 1000
    logits = torch.randn(B, V, device=DEV, generator=torch.Generator(device="cuda").manual_seed(B))
    flat = torch.full((B * H + 4,), -7, dtype=torch.int64, device=DEV)
    hist = flat[:B * H].view(B, H)
    pos = torch.tensor([H], device=DEV)
    tok = torch.zeros(B, dtype=torch.int64, device=DEV)
    greedy_step(logits, hist, pos, tok)
    torch.cuda.synchronize()
    assert bool((flat == -7).all())
    assert torch.equal(tok, logits.argmax(-1)) and int(pos.item()) == H + 1


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,K", [(5000, 4096), (4099, 8192), (17, 4096), (1, 8192)])
def test_gemv_dense_against_fp64_and_library(dtype, M, K):
    """qz_gemv_dense (the lm_head of a decode token): fp32 accumulation rounded once -- the library's
    numerics class.  Its error against an fp64 product is the output rounding (within 5 % of
    F.linear's), and it differs from F.linear by at most one rounding step where it differs."""
    import torch.nn.functional as F

    from quantizations_amd.layer_ops import gemv_dense, gemv_dense_supported

    g = torch.Generator(device="cuda").manual_seed(M + K)
    W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(dtype)
    x = torch.randn(1, 1, K, device=DEV, generator=g).to(dtype)
    assert gemv_dense_supported(x, W)
    y = gemv_dense(x, W)
    yl = F.linear(x, W)
    ref = W.double() @ x.view(-1).double()
    assert y.shape == yl.shape == (1, 1, M) and y.dtype == dtype
    e_o = ((y.view(-1).double() - ref).norm() / ref.norm()).item()
    e_l = ((yl.view(-1).double() - ref).norm() / ref.norm()).item()
    assert e_o <= 1.05 * e_l + 1e-6, (e_o, e_l)
    ulp = torch.finfo(dtype).eps
    assert torch.all((y.float() - yl.float()).abs() <= 2 * ulp * yl.float().abs().clamp_min(1e-3))
    # two rows, a misaligned x or another width: the caller keeps F.linear
    assert not gemv_dense_supported(torch.randn(2, 1, K, device=DEV).to(dtype), W)
    assert not gemv_dense_supported(torch.randn(1, 1, K + 1, device=DEV).to(dtype)[..., 1:], W)


def test_llama_decode_dense_lm_head_tokens():
    """bench.py's graph decode of a 4096-wide model with the lm_head on qz_gemv_dense (its default)
    against F.linear: identical greedy tokens; the dense launch ran."""
    from transformers import LlamaForCausalLM

    import bench
    from quantizations_amd import _lib
    from quantizations_amd.integration import replace_with_bnb_linear, unfuse_layer_ops, unfuse_lm_head

    cfg = _cfg("llama3", max_pos=256, hidden=4096, heads=32, kv=8, layers=1)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, modules_to_not_convert=["lm_head"], quant_type="nf4",
                            compute_dtype=torch.float32)
    bench.prepare_decode_model(model, 0, 1, False)
    calls = {"n": 0}
    fn = _lib.lib.qz_gemv_dense

    def spy(*a):
        calls["n"] += 1
        return fn(*a)
    _lib.lib.qz_gemv_dense = spy
    try:
        _, hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    finally:
        _lib.lib.qz_gemv_dense = fn
    assert calls["n"] >= 1
    unfuse_lm_head(model)
    try:
        _, ref_hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
    finally:
        unfuse_layer_ops(model)
    assert torch.equal(hist, ref_hist)


def test_row_sharded_lm_head_rows_equal_the_full_launch():
    """parallel.RowShardedDenseLinear: rank r's local rows of a 128256 x 4096 fp16 lm_head on
    qz_gemv_dense are bit-identical to rows [r M/N, (r+1) M/N) of the unsharded launch (each row
    is the same dot product), for N = 2, 4, 8 (the all-gather itself: test_gpu_xgmi_rowsplit.py)."""
    import torch.nn as nn

    from quantizations_amd.layer_ops import gemv_dense
    from quantizations_amd.parallel import RowShardedDenseLinear

    M, K = 128256, 4096
    full = nn.Linear(K, M, bias=False, device=DEV, dtype=torch.float16)
    with torch.no_grad():
        full.weight.normal_(0, 0.02)
    x = torch.randn(1, 1, K, device=DEV).half()
    ref = gemv_dense(x, full.weight).view(-1)
    for world in (2, 4, 8):
        for rank in range(world):
            mod = RowShardedDenseLinear(full, rank=rank, world_size=world)
            y = gemv_dense(x, mod.weight).view(-1)
            assert torch.equal(y, ref[mod.r0:mod.r1])
            del mod

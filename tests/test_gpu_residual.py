"""GPU: the residual add in the GEMV epilogue (qz_gemv_4bit_residual, Linear4bit.forward_residual)
and the decoder layer that routes LlamaDecoderLayer's two `residual + h` adds into it
(integration.fuse_layer_ops residual=True).  The bar is bit-identity with the two-op torch form
residual + gemv: every geometry of the vector kernel (WK = 1 packed and unpacked stores, WK > 1
through LDS), the generic kernel, fp16 / bf16 / fp32, and whole-model logits."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,K,exact", [(4096, 4096, True), (4096, 14336, True), (8192, 8192, None),
                                       (1023, 4096, None), (300, 1000, None), (64, 4096, True)])
def test_gemv_residual_is_the_torch_add(dtype, M, K, exact):
    from quantizations_amd.core import gemv_4bit, quantize_4bit

    g = torch.Generator(device="cuda").manual_seed(M + K)
    W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(torch.float16)
    packed, st = quantize_4bit(W, quant_type="nf4", compress_statistics=True)
    x = torch.randn(1, 1, K, device=DEV, generator=g).to(dtype)
    r = (torch.randn(1, 1, M, device=DEV, generator=g) * 4).to(dtype)
    bias = (torch.randn(M, device=DEV, generator=g) * 0.1).to(dtype) if M == 1023 else None
    ref = r + gemv_4bit(x, packed, state=st, bias=bias, exact_codes=exact)
    got = gemv_4bit(x, packed, state=st, bias=bias, exact_codes=exact, residual=r)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.dtype == ref.dtype
    assert torch.equal(got, ref), (got.float() - ref.float()).abs().max().item()


def test_linear4bit_forward_residual_falls_back_to_two_ops():
    import quantizations_amd as qa

    lin = qa.Linear4bit(256, 128, quant_type="nf4", compute_dtype=torch.float32).to(DEV)
    x = torch.randn(1, 1, 256, device=DEV).half()
    r = torch.randn(1, 1, 128, device=DEV).half()
    assert torch.equal(lin.forward_residual(x, r), r + lin(x))           # fused epilogue
    x3 = torch.randn(1, 3, 256, device=DEV).half()                          # prefill: two ops
    r3 = torch.randn(1, 3, 128, device=DEV).half()
    assert torch.equal(lin.forward_residual(x3, r3), r3 + lin(x3))


def test_llama_residual_decoder_bit_identical_eager_and_graph():
    from transformers import LlamaConfig, LlamaForCausalLM
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import (fuse_layer_ops, fuse_prenorm, fuse_projection_groups,
                                               replace_with_bnb_linear, unfuse_layer_ops)

    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2048, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(4)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    fuse_projection_groups(model)
    ids = torch.randint(0, 512, (1, 9), device=DEV, generator=torch.Generator(device="cuda").manual_seed(1))

    def decode(graph):
        cache = StaticCache(config=cfg, max_cache_len=32)
        out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(9, device=DEV))
        tok = out.logits[:, -1:].argmax(-1)
        pos = torch.tensor([9], device=DEV)
        logits = [out.logits[:, -1].clone()]

        def step():
            return model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits

        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                lo = step()
            torch.cuda.current_stream().wait_stream(s)
            logits.append(lo[:, -1].clone())
            pos.add_(1)
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph):
                lo = step()
            for _ in range(3):
                gph.replay()
                logits.append(lo[:, -1].clone())
                pos.add_(1)
        else:
            for _ in range(4):
                lo = step()
                logits.append(lo[:, -1].clone())
                pos.add_(1)
        torch.cuda.synchronize()
        return logits

    try:
        with torch.no_grad():
            fuse_layer_ops(model, residual=False)
            fuse_prenorm(model)
            ref = decode(False)
            unfuse_layer_ops(model)
            fuse_layer_ops(model)
            assert sum("_qz_residual_decoder" in m.__dict__ for m in model.modules()) == cfg.num_hidden_layers
            fuse_prenorm(model)
            got = decode(False)
            assert all(torch.equal(a, b) for a, b in zip(got, ref))
            got_graph = decode(True)
            assert all(torch.equal(a, b) for a, b in zip(got_graph, ref))
    finally:
        unfuse_layer_ops(model)


def test_fused_attention_fallback_keeps_the_residual():
    """The residual-fused decoder passes `residual` into the patched attention; when that
    attention cannot take the one-launch path (here: a q width that disagrees with the head
    count the cache implies) its fallback must still return residual + attention (ADVICE r3:
    the early return dropped it).  Logits vs the unfused transformers model."""
    from transformers import LlamaConfig, LlamaForCausalLM
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import fuse_layer_ops, replace_with_bnb_linear, unfuse_layer_ops

    cfg = LlamaConfig(hidden_size=1024, intermediate_size=2048, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(5)
    model = LlamaForCausalLM(cfg).half().to(DEV).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    ids = torch.randint(0, 512, (1, 9), device=DEV, generator=torch.Generator(device="cuda").manual_seed(2))

    def decode():
        cache = StaticCache(config=cfg, max_cache_len=32)
        out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(9, device=DEV))
        tok = out.logits[:, -1:].argmax(-1)
        pos = torch.tensor([9], device=DEV)
        lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits
        torch.cuda.synchronize()
        return lo[:, -1].float()

    with torch.no_grad():
        ref = decode()
        try:
            fuse_layer_ops(model)   # residual-fused decoder + one-launch attention
            assert sum("_qz_residual_decoder" in m.__dict__ for m in model.modules()) == cfg.num_hidden_layers
            model.config.num_attention_heads = 16   # the fused path's head count no longer fits q
            got = decode()
        finally:
            model.config.num_attention_heads = 8
            unfuse_layer_ops(model)
    torch.testing.assert_close(got, ref, atol=3e-2, rtol=3e-2)

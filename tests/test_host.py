"""Host-side mirror of the reference interface (no GPU needed)."""
import inspect

import numpy as np
import pytest
import torch

import quantizations_amd as qa
from quantizations_amd import core, modules


def test_linear4bit_signature_matches_reference():
    # reference modules.py:86-96
    params = list(inspect.signature(modules.Linear4bit.__init__).parameters)
    assert params == ["self", "input_features", "output_features", "bias", "compute_dtype", "compress_statistics",
                      "quant_type", "quant_storage", "device"]
    p = inspect.signature(modules.Linear4bit.__init__).parameters
    assert p["bias"].default is False and p["quant_type"].default == "fp4" and p["compress_statistics"].default


def test_params4bit_signature_and_kwargs():
    params = list(inspect.signature(core.Params4bit.__new__).parameters)
    assert params[:9] == ["cls", "data", "requires_grad", "quant_state", "blocksize", "quant_type", "quant_storage",
                          "module", "bnb_quantized"]
    # transformers: Params4bit(value, requires_grad=False, **old.__dict__) must not fail on extra keys
    p = core.Params4bit(torch.zeros(4, 4), requires_grad=False, quant_type="nf4", _is_hf_initialized=True)
    assert p.quant_type == "nf4" and not p.bnb_quantized


def test_codebooks(ref_tables):
    assert np.array_equal(core.get_4bit_type("fp4", device="cpu").numpy().view(np.uint32),
                          ref_tables["fp4_lut"].view(np.uint32))
    nf4 = core.get_4bit_type("nf4", device="cpu")
    assert nf4[7] == 0 and nf4[0] == -1 and nf4[15] == 1
    with pytest.raises(NotImplementedError):
        core.get_4bit_type("int4", device="cpu")


def test_dynamic_map_matches_reference(ref_tables):
    assert np.array_equal(core.create_dynamic_map().numpy().view(np.uint32), ref_tables["dynamic_map"].view(np.uint32))


def test_quantize_requires_gpu_like_reference():
    with pytest.raises(NotImplementedError):
        core.quantize_4bit(torch.zeros(64, dtype=torch.float16))
    with pytest.raises(NotImplementedError):
        core.quantize_4bit(torch.zeros(64, dtype=torch.float16, device="meta"), quant_type="int4")


def test_gemv_argument_errors_like_reference():
    st = core.QuantState(absmax=torch.zeros(4), shape=torch.Size([8, 32]), blocksize=64, quant_type="fp4")
    with pytest.raises(ValueError, match="state cannot None"):
        core.gemv_4bit(torch.zeros(1, 1, 32), torch.zeros(1), state=None)
    with pytest.raises(ValueError, match="Dimensions of A are invalid"):
        core.gemv_4bit(torch.zeros(2, 1, 32), torch.zeros(1), state=st)
    with pytest.raises(ValueError):
        core.dequantize_4bit(torch.zeros(1), st, blocksize=96)


def test_quant_state_dict_roundtrip():
    st2 = core.QuantState(absmax=torch.rand(2), blocksize=256, code=core.create_dynamic_map(), dtype=torch.float32)
    st = core.QuantState(absmax=torch.randint(0, 255, (300,), dtype=torch.uint8), shape=torch.Size([60, 320]),
                         code=core.get_4bit_type("nf4", device="cpu"), blocksize=64, quant_type="nf4",
                         dtype=torch.float16, offset=torch.tensor(0.25), state2=st2)
    d = st.as_dict()
    assert set(k for k in d) <= set(core.QuantState.valid_qs_keys)
    back = core.QuantState.from_dict(d, device="cpu")
    assert back.nested and back.quant_type == "nf4" and back.shape == st.shape and back.dtype == torch.float16
    assert torch.equal(back.absmax, st.absmax) and torch.equal(back.state2.absmax, st2.absmax)
    assert float(back.offset) == 0.25


def test_module_needs_quantisation_before_forward():
    m = qa.Linear4bit(32, 8, quant_type="nf4")
    with pytest.raises(RuntimeError, match="not quantised"):
        m(torch.zeros(1, 1, 32, dtype=torch.float16))


def test_replace_with_bnb_linear_skips_lm_head_on_meta():
    from quantizations_amd.integration import replace_with_bnb_linear

    class Tiny(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.proj = torch.nn.Linear(64, 64)
            self.lm_head = torch.nn.Linear(64, 10)

    with torch.device("meta"):
        t = Tiny()
    # meta weights never reach .to(cuda) -> not quantised, but the module types are swapped
    replace_with_bnb_linear(t, quant_type="nf4", device="meta")
    assert isinstance(t.proj, qa.Linear4bit) and not isinstance(t.lm_head, qa.Linear4bit)
    assert t.proj.weight.quant_type == "nf4" and t.proj.weight.compress_statistics


def test_fuse_layer_ops_patches_and_restores_on_cpu():
    """fuse_layer_ops installs the HIP norm/rotary forms; on CPU tensors the kernels
    do not apply and transformers' own code runs, so logits are unchanged; unfuse
    restores the original forwards and apply_rotary_pos_emb."""
    from transformers import LlamaConfig, LlamaForCausalLM
    from transformers.cache_utils import StaticCache
    import transformers.models.llama.modeling_llama as ml

    from quantizations_amd.integration import fuse_layer_ops, unfuse_layer_ops
    from quantizations_amd.layer_ops import rms_norm_supported, rope_supported

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=97)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).eval()
    ids = torch.randint(0, 97, (1, 5))
    orig = ml.apply_rotary_pos_emb
    with torch.no_grad():
        ref = model(input_ids=ids).logits
        cache = StaticCache(config=cfg, max_cache_len=8)
        ref_pre = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(5)).logits
        p5 = torch.tensor([5])
        ref_step = model(input_ids=ids[:, :1], past_key_values=cache, cache_position=p5,
                         position_ids=p5.view(1, 1)).logits
        # norms, final norm, MLPs, decoder layers, attention modules, rope
        assert fuse_layer_ops(model, decoder=True) == 2 * 2 + 1 + 2 + 2 + 2 + 1
        cache = StaticCache(config=cfg, max_cache_len=8)     # CPU decode: the attention patch defers
        pre = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(5)).logits
        p5 = torch.tensor([5])
        step = model(input_ids=ids[:, :1], past_key_values=cache, cache_position=p5, position_ids=p5.view(1, 1)).logits
        assert ml.apply_rotary_pos_emb is not orig and ml.apply_rotary_pos_emb._qz_orig is orig
        assert fuse_layer_ops(model) == 0  # idempotent
        assert torch.equal(model(input_ids=ids).logits, ref)
        assert torch.equal(pre, ref_pre) and torch.equal(step, ref_step)
        unfuse_layer_ops(model)
    assert ml.apply_rotary_pos_emb is orig
    assert not any("forward" in m.__dict__ for m in model.modules())
    x = torch.randn(2, 64)
    assert not rms_norm_supported(x, torch.ones(64))  # CPU tensors never reach the kernel
    q = torch.randn(1, 4, 3, 16)
    assert not rope_supported(q, q, torch.randn(1, 3, 16), torch.randn(1, 3, 16))


def test_fuse_layer_ops_residual_decoder_on_cpu_is_bit_identical():
    """The default fuse_layer_ops also restates each decoder layer so that its two residual
    adds can run in the o_proj / down_proj epilogues; on CPU (no kernels) every patched
    forward defers to torch in the original operand order: logits of prefill and of a
    StaticCache decode step are bit-identical, and unfuse removes every patch."""
    from transformers import LlamaConfig, LlamaForCausalLM
    from transformers.cache_utils import StaticCache

    from quantizations_amd.integration import fuse_layer_ops, unfuse_layer_ops

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=97)
    torch.manual_seed(1)
    model = LlamaForCausalLM(cfg).eval()
    ids = torch.randint(0, 97, (1, 5))

    def run():
        cache = StaticCache(config=cfg, max_cache_len=8)
        a = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(5)).logits
        p5 = torch.tensor([5])
        b = model(input_ids=ids[:, :1], past_key_values=cache, cache_position=p5, position_ids=p5.view(1, 1)).logits
        return a, b

    with torch.no_grad():
        ref = run()
        # norms + final norm, MLPs, attention modules, rope, residual decoder layers
        assert fuse_layer_ops(model) == 2 * 2 + 1 + 2 + 2 + 1 + 2
        assert sum("_qz_residual_decoder" in m.__dict__ for m in model.modules()) == 2
        got = run()
        assert all(torch.equal(x, y) for x, y in zip(got, ref))
        unfuse_layer_ops(model)
    assert not any(k.startswith("_qz") or k == "forward" for m in model.modules() for k in m.__dict__)


def test_fuse_prenorm_absorbs_only_cuda_norms_of_plain_groups():
    """fuse_prenorm needs a Linear4bit decode group (not a row-sharded one) and a norm weight
    on the GPU: on a CPU model it absorbs nothing; a group whose compute is not the Linear4bit
    one is never given a norm; unfuse_prenorm leaves no patched forward behind."""
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import fuse_prenorm, unfuse_prenorm
    from quantizations_amd.modules import DecodeGroup, _linear4bit_group_compute

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=97)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).eval()
    for layer in model.model.layers:   # Linear4bit projections (unquantised on CPU) in decode groups
        for parent, names in ((layer.self_attn, ("q_proj", "k_proj", "v_proj")), (layer.mlp, ("gate_proj", "up_proj"))):
            members = []
            for nm in names:
                lin = getattr(parent, nm)
                q = qa.Linear4bit(lin.in_features, lin.out_features, bias=False, quant_type="nf4")
                setattr(parent, nm, q)
                members.append(q)
            grp = DecodeGroup(members, _linear4bit_group_compute)
            for q in members:
                q.__dict__["_qz_group"] = grp
    assert fuse_prenorm(model) == 0                      # norm weights on the CPU
    assert not any("_qz_absorbed_norm" in m.__dict__ for m in model.modules())
    g = model.model.layers[0].self_attn.q_proj.__dict__["_qz_group"]
    assert isinstance(g, DecodeGroup) and g.prenorm is None
    g._compute = lambda grp, x: None                     # e.g. a row-sharded group's compute
    assert fuse_prenorm(model) == 0 and g.prenorm is None
    unfuse_prenorm(model)
    assert not any("forward" in m.__dict__ for m in model.modules())


def test_fuse_layer_ops_leaves_other_rotary_forms_alone():
    """The rotary patch is limited to Llama/Mistral/Qwen2 attention modules whose
    modeling module has the half-split rotate_half.  An attention class outside
    the allow-list (here: a Cohere-style module with the interleaved
    rotate_half) keeps its own apply_rotary_pos_emb, and so does an allow-listed
    name whose module rotates interleaved."""
    import sys
    import types

    from quantizations_amd.integration import _half_split_rotate, fuse_layer_ops, unfuse_layer_ops

    def interleaved(x):  # modeling_cohere.py's rotate_half
        x1, x2 = x[..., ::2], x[..., 1::2]
        return torch.stack([-x2, x1], dim=-1).flatten(-2)

    def apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1):
        return q, k

    created = []
    for modname, clsname in (("qz_fake_cohere", "CohereAttention"), ("qz_fake_llama_like", "LlamaAttention")):
        mod = types.ModuleType(modname)
        mod.rotate_half = interleaved
        mod.apply_rotary_pos_emb = apply_rotary_pos_emb
        cls = type(clsname, (torch.nn.Module,), {"__module__": modname})
        mod.__dict__[clsname] = cls
        sys.modules[modname] = mod
        created.append((modname, cls))
    try:
        assert not _half_split_rotate(sys.modules["qz_fake_cohere"])
        import transformers.models.llama.modeling_llama as ml
        assert _half_split_rotate(ml)
        model = torch.nn.Sequential(*[cls() for _, cls in created])
        assert fuse_layer_ops(model, norm=False, mlp=False) == 0
        for modname, _ in created:
            assert sys.modules[modname].apply_rotary_pos_emb is apply_rotary_pos_emb
        unfuse_layer_ops(model)
    finally:
        for modname, _ in created:
            sys.modules.pop(modname, None)


def test_fused_route_threshold_follows_measured_crossover():
    # scripts/prefill_lowT_sweep.py on one MI355X (profiles/r2_prefill_lowT_sweep.txt)
    from quantizations_amd import core

    assert core.fused_max_tokens(4096) == 256        # 4096x4096, 4096x14336: fused wins to T = 256
    assert core.fused_max_tokens(1024) == 128        # k/v projections: to T = 128
    assert core.fused_max_tokens(14336) == 128       # gate/up: a tie at T = 128, dequant route above
    # Llama-3-70B (profiles/r6_prefill_lowT_sweep_70b.txt): q/o and down to T = 256, gate/up to 128, and
    # the k/v projections (1024 x 8192) fused at every measured T up to 512
    assert core.fused_max_tokens(8192, 8192) == 256 and core.fused_max_tokens(8192, 28672) == 256
    assert core.fused_max_tokens(28672, 8192) == 128
    assert core.fused_max_tokens(1024, 8192) == 512 and core.fused_max_tokens(1024, 4096) == 128
    assert core.PREFILL_FUSED_MAX_TOKENS is None     # no QZ_PREFILL_FUSED_MAX_T in the test env


def test_fused_route_threshold_env_override_replaces_table(monkeypatch):
    """An explicit QZ_PREFILL_FUSED_MAX_T replaces the measured table (in both directions)."""
    from quantizations_amd import core

    for v in (512, 64, 0):
        monkeypatch.setattr(core, "PREFILL_FUSED_MAX_TOKENS", v)
        assert all(core.fused_max_tokens(m, k) == v for m in (8, 1024, 4096, 14336) for k in (4096, 8192))

"""Pre-quantised checkpoints: the bnb-compatible
QuantState layout, Linear4bit state-dict hooks and safetensors round trips.

Key names are the reference's valid_qs_keys (core.py:29-42); the reference
declares them but never serialises, so the packed layout follows bitsandbytes
(non-tensor fields JSON-encoded into one uint8 tensor) -- parity unpinned
beyond the key names.  The CPU tests build statistics with the oracle (no GPU
kernel runs); the GPU test saves and reloads a quantised model."""
import json

import numpy as np
import pytest
import torch

from conftest import REPO  # noqa: F401


def _oracle_state(M, K, qt, dq, seed=0):
    import oracle
    from quantizations_amd.core import QuantState, create_dynamic_map, get_4bit_type

    W = (torch.randn(M, K, generator=torch.Generator().manual_seed(seed)) * 0.02).half()
    st = oracle.quantize_4bit(W.float().numpy(), 64, qt, double_quant=dq)
    if dq:
        st2 = QuantState(absmax=torch.from_numpy(st.absmax2), blocksize=256, code=create_dynamic_map(),
                         dtype=torch.float32)
        qs = QuantState(absmax=torch.from_numpy(st.qabsmax), shape=torch.Size([M, K]), code=get_4bit_type(qt, "cpu"),
                        blocksize=64, quant_type=qt, dtype=torch.float16, offset=torch.tensor(float(st.offset)),
                        state2=st2)
    else:
        qs = QuantState(absmax=torch.from_numpy(st.absmax_raw), shape=torch.Size([M, K]), code=get_4bit_type(qt, "cpu"),
                        blocksize=64, quant_type=qt, dtype=torch.float16)
    return torch.from_numpy(st.packed).reshape(-1, 1), qs


def _same_state(a, b):
    assert a.quant_type == b.quant_type and a.blocksize == b.blocksize and a.dtype == b.dtype
    assert tuple(a.shape) == tuple(b.shape) and a.nested == b.nested
    assert torch.equal(a.absmax.cpu(), b.absmax.cpu()) and torch.equal(a.code.cpu(), b.code.cpu())
    if a.nested:
        assert torch.equal(a.state2.absmax.cpu(), b.state2.absmax.cpu())
        assert torch.equal(a.state2.code.cpu(), b.state2.code.cpu())
        assert a.state2.blocksize == b.state2.blocksize
        assert a.offset.cpu().view(torch.int32) == b.offset.cpu().view(torch.int32)  # bit-exact fp32


@pytest.mark.parametrize("qt,dq", [("nf4", True), ("fp4", True), ("nf4", False)])
def test_quant_state_packed_layout_and_round_trip(qt, dq):
    from quantizations_amd.core import QuantState

    _, qs = _oracle_state(96, 256, qt, dq)
    d = qs.as_dict(packed=True)
    tensor_keys = {"absmax", "quant_map"} | ({"nested_absmax", "nested_quant_map"} if dq else set())
    packed_key = "quant_state.bitsandbytes__" + qt
    assert set(d) == tensor_keys | {packed_key}
    assert all(isinstance(v, torch.Tensor) for v in d.values()) and d[packed_key].dtype == torch.uint8
    meta = json.loads(bytes(d[packed_key].tolist()).decode())
    assert set(meta) | tensor_keys <= set(QuantState.valid_qs_keys)   # reference core.py:29-42
    assert meta["shape"] == [96, 256] and meta["blocksize"] == 64 and meta["dtype"] == "float16"
    _same_state(qs, QuantState.from_dict(d, device="cpu"))
    # module-prefixed keys (as they appear in a model state dict) and the unpacked form
    pref = {"model.layers.3.mlp.up_proj.weight." + k: v for k, v in d.items()}
    _same_state(qs, QuantState.from_dict(pref, device="cpu"))
    _same_state(qs, QuantState.from_dict(qs.as_dict(packed=False), device="cpu"))


def test_quant_state_rejects_incomplete():
    from quantizations_amd.core import QuantState

    _, qs = _oracle_state(8, 128, "nf4", True)
    d = qs.as_dict(packed=True)
    del d["absmax"]
    with pytest.raises(ValueError):
        QuantState.from_dict(d, device="cpu")


def _prequantized_linear(M, K, qt="nf4", bias=True, seed=0):
    from quantizations_amd.core import Params4bit
    from quantizations_amd.modules import Linear4bit

    packed, qs = _oracle_state(M, K, qt, True, seed)
    lin = Linear4bit(K, M, bias=bias, quant_type=qt, device="meta")
    lin.weight = Params4bit.from_prequantized(packed, qs.as_dict(packed=True), device="cpu", module=lin)
    if bias:
        lin.bias = torch.nn.Parameter(torch.randn(M, generator=torch.Generator().manual_seed(seed + 1)),
                                      requires_grad=False)
    return lin, packed, qs


def test_linear4bit_state_dict_round_trip_cpu():
    from quantizations_amd.modules import Linear4bit

    lin, packed, qs = _prequantized_linear(64, 256)
    sd = lin.state_dict()
    assert set(sd) == {"weight", "bias", "weight.absmax", "weight.quant_map", "weight.nested_absmax",
                       "weight.nested_quant_map", "weight.quant_state.bitsandbytes__nf4"}
    assert sd["weight"].dtype == torch.uint8 and torch.equal(sd["weight"], packed)
    fresh = Linear4bit(256, 64, bias=True, quant_type="nf4", device="meta")
    res = fresh.load_state_dict(sd, strict=True, assign=True)
    assert not res.missing_keys and not res.unexpected_keys
    assert fresh.weight.bnb_quantized and torch.equal(fresh.weight.data, packed)
    _same_state(qs, fresh.weight.quant_state)
    assert fresh.quant_state is fresh.weight.quant_state
    assert torch.equal(fresh.bias, lin.bias)


def test_safetensors_round_trip_cpu(tmp_path):
    from quantizations_amd.integration import load_quantized, save_quantized

    model = torch.nn.Sequential()
    for i in range(2):
        lin, _, _ = _prequantized_linear(32, 128, qt=("nf4", "fp4")[i], seed=i)
        model.add_module(f"l{i}", lin)
    model.add_module("head", torch.nn.Linear(32, 8))
    path = str(tmp_path / "m.safetensors")
    save_quantized(model, path)
    target = torch.nn.Sequential()
    target.add_module("l0", torch.nn.Linear(128, 32))   # plain Linear: becomes Linear4bit from the checkpoint
    target.add_module("l1", torch.nn.Linear(128, 32))
    target.add_module("head", torch.nn.Linear(32, 8))
    load_quantized(target, path, device="cpu")
    from quantizations_amd.modules import Linear4bit
    assert isinstance(target.l0, Linear4bit) and isinstance(target.l1, Linear4bit)
    assert not isinstance(target.head, Linear4bit)
    for name in ("l0", "l1"):
        a, b = getattr(model, name), getattr(target, name)
        assert torch.equal(a.weight.data, b.weight.data) and b.weight.quant_type == a.weight.quant_type
        _same_state(a.weight.quant_state, b.weight.quant_state)
    assert torch.equal(model.head.weight, target.head.weight)


@pytest.mark.gpu
def test_tiny_llama_checkpoint_round_trip_gpu(tmp_path):
    """Quantise, save, rebuild from the file (no re-quantisation), same logits bit for bit."""
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import load_quantized, replace_with_bnb_linear, save_quantized

    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=512)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).half().cuda().eval()
    replace_with_bnb_linear(model, quant_type="nf4")
    ids = torch.randint(0, 512, (1, 9), device="cuda")
    with torch.no_grad():
        ref = model(input_ids=ids).logits
    path = str(tmp_path / "tiny.safetensors")
    save_quantized(model, path)
    torch.manual_seed(123)  # different random init: everything must come from the file
    other = LlamaForCausalLM(cfg).half().cuda().eval()
    load_quantized(other, path, modules_to_not_convert=["lm_head"])
    with torch.no_grad():
        out = other(input_ids=ids).logits
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
def test_oracle_built_checkpoint_loaded_on_gpu_matches_oracle(tmp_path, orc, qt):
    """A safetensors file written from ORACLE-built quant states (packed bytes,
    qabsmax, absmax2, offset under the core.py:29-42 keys) -- no GPU kernel
    produced any of it -- loaded with load_quantized onto the GPU: Linear4bit
    decode (the fused GEMV, default fp16 table), gemv_4bit on the loaded state with fp32 x
    (fp32 codes) and with fp16 x + exact codes, and prefill all match oracle.gemv of the
    same bytes."""
    from safetensors.torch import save_file

    from quantizations_amd.core import gemv_4bit
    from quantizations_amd.integration import load_quantized
    from quantizations_amd.modules import Linear4bit

    shapes = {"up": (384, 1024), "down": (1024, 384 * 2)}
    sd, states = {}, {}
    for i, (name, (M, K)) in enumerate(shapes.items()):
        packed, qs = _oracle_state(M, K, qt, True, seed=40 + i)
        sd[f"{name}.weight"] = packed
        for k, v in qs.as_dict(packed=True).items():
            sd[f"{name}.weight.{k}"] = v
        W = (torch.randn(M, K, generator=torch.Generator().manual_seed(40 + i)) * 0.02).half()
        states[name] = orc.quantize_4bit(W.float().numpy(), 64, qt, double_quant=True)
        assert np.array_equal(packed.numpy().ravel(), states[name].packed)
    path = str(tmp_path / "oracle.safetensors")
    save_file(sd, path)

    model = torch.nn.Sequential()
    model.add_module("up", torch.nn.Linear(1024, 384, bias=False))
    model.add_module("down", torch.nn.Linear(768, 1024, bias=False))
    load_quantized(model, path, device="cuda")
    for name, (M, K) in shapes.items():
        lin = getattr(model, name)
        assert isinstance(lin, Linear4bit) and lin.weight.is_cuda and lin.weight.quant_type == qt
        o = states[name]
        x = torch.randn(1, 1, K, generator=torch.Generator().manual_seed(M)).half()
        yref = orc.gemv(x.float().numpy().ravel(), o)
        y = lin(x.cuda()).float().cpu().numpy().ravel()
        rel = np.linalg.norm(y - yref) / np.linalg.norm(yref)
        assert rel <= 1e-3, (name, rel)
        # fp32 x: the fp32 code table, fp32 output
        ye = gemv_4bit(x.float().cuda(), lin.weight, state=lin.weight.quant_state)
        rel_e = np.linalg.norm(ye.cpu().numpy().ravel() - yref) / np.linalg.norm(yref)
        assert rel_e <= 1e-5, (name, rel_e)
        # fp16 x with exact_codes=True (the exact hi + lo fp16 table): the reference value
        # rounded once to the fp16 output, plus fp32 summation noise
        yh = gemv_4bit(x.cuda(), lin.weight, state=lin.weight.quant_state, exact_codes=True)
        yh = yh.double().cpu().numpy().ravel()
        assert np.all(np.abs(yh - yref) <= 2.0 ** -11 * np.abs(yref) + 1e-5 * np.max(np.abs(yref))), name
        X = torch.randn(3, 7, K, generator=torch.Generator().manual_seed(K)).half()
        Yref = X.reshape(-1, K).double().numpy() @ orc.dequantize(o).astype(np.float16).astype(np.float64).T
        Y = lin(X.cuda()).double().cpu().numpy().reshape(-1, M)
        assert np.linalg.norm(Y - Yref) / np.linalg.norm(Yref) <= 1e-3


def test_linear4bit_deepcopy_keeps_the_4bit_state():
    """copy.deepcopy of a quantised Linear4bit (e.g. to keep an unsharded reference) keeps its
    packed bytes and QuantState -- equal values, separate tensors -- and the copy's
    Params4bit.module points to the copied module (torch's default Parameter.__deepcopy__
    would drop the state)."""
    import copy

    from quantizations_amd.modules import Linear4bit

    M, K = 128, 256
    packed, qs = _oracle_state(M, K, "nf4", True, seed=7)
    lin = Linear4bit(K, M, bias=False, quant_type="nf4", device="meta")
    from quantizations_amd.core import Params4bit
    lin.weight = Params4bit.from_prequantized(packed.reshape(-1, 1), qs.as_dict(packed=True), device="cpu", module=lin)
    twin = copy.deepcopy(lin)
    w, w2 = lin.weight, twin.weight
    assert isinstance(w2, Params4bit) and w2.bnb_quantized and w2.quant_state is not None
    assert w2.module is twin and twin.quant_state is w2.quant_state
    assert torch.equal(w2.data, w.data) and w2.data.data_ptr() != w.data.data_ptr()
    for a, b in ((w.quant_state.absmax, w2.quant_state.absmax), (w.quant_state.state2.absmax, w2.quant_state.state2.absmax),
                 (w.quant_state.offset, w2.quant_state.offset), (w.quant_state.code, w2.quant_state.code)):
        assert torch.equal(a, b) and a.data_ptr() != b.data_ptr()
    assert w2.quant_state.shape == w.quant_state.shape and w2.quant_state.quant_type == "nf4"

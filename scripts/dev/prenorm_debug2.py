"""Dev check: fused vs two-launch grouped GEMV on the model's own gate/up input."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_prenorm import _llama, _items, DEV  # noqa: E402
from transformers.cache_utils import StaticCache  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped  # noqa: E402
from quantizations_amd.layer_ops import rms_norm  # noqa: E402

model, cfg = _llama()
ids = torch.randint(0, cfg.vocab_size, (1, 10), device=DEV, generator=torch.Generator(device="cuda").manual_seed(3))
caught = []
layer = model.model.layers[1]
layer.post_attention_layernorm.register_forward_pre_hook(lambda m, a: caught.append(a[0].detach().clone()))
with torch.no_grad():
    cache = StaticCache(config=cfg, max_cache_len=32)
    out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(10, device=DEV))
    tok = out.logits[:, -1:].argmax(-1)
    pos = torch.tensor([10], device=DEV)
    model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1))
H = caught[1]
ln = layer.post_attention_layernorm
mlp = layer.mlp
items = [(mlp.gate_proj.weight, mlp.gate_proj.weight.quant_state, None), (mlp.up_proj.weight, mlp.up_proj.weight.quant_state, None)]
for exact in (None, True):
    ref = gemv_4bit_grouped(rms_norm(H, ln.weight, ln.variance_epsilon), items, exact_codes=exact)
    got = gemv_4bit_grouped(H, items, exact_codes=exact, norm=(ln.weight, ln.variance_epsilon))
    print("exact", exact, [bool(torch.equal(a, b)) for a, b in zip(got, ref)],
          [(a.float() - b.float()).abs().max().item() for a, b in zip(got, ref)])
print("H", H.shape, H.dtype, H.is_contiguous(), H.abs().max().item(), "w", ln.weight.dtype, ln.weight.is_contiguous(),
      "eps", ln.variance_epsilon)
# random inputs at this geometry
items2 = _items((4096, 4096), 2048, torch.float16, seed=11)
for t in range(5):
    x = (torch.randn(1, 1, 2048, device=DEV) * (3 + 10 * t)).half()
    w = (1.0 + 0.1 * torch.randn(2048, device=DEV)).half()
    ref = gemv_4bit_grouped(rms_norm(x, w, 1e-6), items2)
    got = gemv_4bit_grouped(x, items2, norm=(w, 1e-6))
    print("random", t, [bool(torch.equal(a, b)) for a, b in zip(got, ref)])

# x' itself through an identity weight (NF4 code 1.0, fp32 absmax 1.0: y_r = x'_r exactly)
from quantizations_amd.core import quantize_4bit  # noqa: E402
import numpy as np  # noqa: E402
K = 2048
I = torch.eye(K, device=DEV, dtype=torch.float16)
pk, st = quantize_4bit(I, quant_type="nf4", compress_statistics=False)
xi = gemv_4bit_grouped(H, [(pk, st, None)], norm=(ln.weight, ln.variance_epsilon))[0].view(-1)
xr = rms_norm(H, ln.weight, ln.variance_epsilon).view(-1)
xo = gemv_4bit_grouped(xr, [(pk, st, None)])[0].view(-1)
print("identity GEMV of the two-launch x' reproduces it:", bool(torch.equal(xo, xr)))
d = (xi != xr).nonzero().view(-1)
print("x' elements differing:", d.numel(), d[:10].tolist())
# numpy restatement of k_rmsnorm's order: thread t sums chunk t's 8 squares, xor butterfly per wave
h = H.view(-1).float().cpu().numpy().astype(np.float32)
ss = np.zeros(256, np.float32)
for t in range(256):
    acc = np.float32(0)
    for j in range(8):
        v = h[8 * t + j]
        acc = np.float32(acc + np.float32(v * v))
    ss[t] = acc
parts = []
for wv in range(4):
    v = ss[64 * wv: 64 * wv + 64].copy()
    o = 32
    while o > 0:
        v = np.array([np.float32(v[l] + v[l ^ o]) for l in range(64)], np.float32)
        o //= 2
    parts.append(v[0])
tot = np.float32(np.float32(parts[0] + parts[1]) + np.float32(parts[2] + parts[3]))
var = np.float32(np.float32(tot * np.float32(np.float32(1.0) / np.float32(K))) + np.float32(ln.variance_epsilon))
print("tot", float(tot), "var", float(var), "1/sqrt", float(np.float32(1.0) / np.sqrt(np.float64(var))))
for e in d[:5].tolist():
    print(e, "H", float(H.view(-1)[e]), "w", float(ln.weight[e]), "fused", float(xi[e]), "two-launch", float(xr[e]))

# numpy x' with the numpy rs, against both
rs_np = np.float32(1.0 / np.sqrt(np.float64(var)))
wn = ln.weight.detach().float().cpu().numpy().astype(np.float32)
hn = (h * rs_np).astype(np.float32).astype(np.float16).astype(np.float32)
xn = (wn * hn).astype(np.float32).astype(np.float16)
xi_n = xi.float().cpu().numpy().astype(np.float16)
xr_n = xr.float().cpu().numpy().astype(np.float16)
print("numpy vs fused mismatches:", int((xn != xi_n).sum()), " numpy vs two-launch:", int((xn != xr_n).sum()))
for cand in (rs_np, np.nextafter(rs_np, np.float32(2)), np.nextafter(rs_np, np.float32(0))):
    hn = (h * cand).astype(np.float32).astype(np.float16).astype(np.float32)
    xn = (wn * hn).astype(np.float32).astype(np.float16)
    print(f"rs {float(cand):.9g}: vs fused {int((xn != xi_n).sum())}, vs two-launch {int((xn != xr_n).sum())}")
# the two-launch tot: sum of squares in plain fp64 for scale
print("fp64 sum of squares", float((h.astype(np.float64) ** 2).sum()))

def emulate(order):
    ss = np.zeros(256, np.float32)
    for t in range(256):
        acc = np.float32(0)
        idx = [8 * t + j for j in range(8)] if order == "vec" else [t + 256 * j for j in range(8)]
        for e in idx:
            acc = np.float32(acc + np.float32(h[e] * h[e]))
        ss[t] = acc
    parts = []
    for wv in range(4):
        v = ss[64 * wv: 64 * wv + 64].copy()
        o = 32
        while o > 0:
            v = np.array([np.float32(v[l] + v[l ^ o]) for l in range(64)], np.float32)
            o //= 2
        parts.append(v[0])
    return np.float32(np.float32(parts[0] + parts[1]) + np.float32(parts[2] + parts[3]))


for order in ("vec", "strided"):
    t_ = emulate(order)
    var_ = np.float32(np.float32(t_ * np.float32(1.0 / K)) + np.float32(ln.variance_epsilon))
    print(order, "tot", repr(float(t_)), "var", repr(float(var_)))
w2 = ln.weight.detach().clone()
print("rms_norm(H) stable across copies:", bool(torch.equal(rms_norm(H.clone(), w2, ln.variance_epsilon), xr)))
from quantizations_amd.layer_ops import add_rms_norm  # noqa: E402
_, xa = add_rms_norm(torch.zeros_like(H), H, ln.weight.detach(), ln.variance_epsilon)
print("add_rms_norm(0, H) == rms_norm(H):", bool(torch.equal(xa.view(-1), xr)), " == fused:", bool(torch.equal(xa.view(-1), xi)))
print("ptr%16: H", H.data_ptr() % 16, "w", ln.weight.data_ptr() % 16, "w2", w2.data_ptr() % 16)
outs = [rms_norm(H, ln.weight, ln.variance_epsilon).view(-1) for _ in range(6)]
print("rms_norm(H, w) repeat-equal:", [bool(torch.equal(o, xr)) for o in outs])
outs2 = [rms_norm(H.clone(), w2, ln.variance_epsilon).view(-1) for _ in range(6)]
print("rms_norm(H', w2) vs xr:", [bool(torch.equal(o, xr)) for o in outs2], "vs fused:", [bool(torch.equal(o, xi)) for o in outs2])
torch.cuda.synchronize()

"""Debug: the test's exact sequence, printing what each path produced."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_qkv_attention import _setup, _two_launches, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_qkv_attention, qkv_attention_state  # noqa: E402
from quantizations_amd.layer_ops import decode_attention  # noqa: E402

H, Hq, Hkv, D, L = 4096, 32, 8, 128, 112
dtype = torch.float16
items, kc, vc, cos, sin, nw = _setup(H, Hq, Hkv, D, L, dtype, seed=H + L)
nrm = (nw, 1e-5)
kc2, vc2 = kc.clone(), vc.clone()
kc0, vc0 = kc.clone(), vc.clone()
p0 = L - 5
pos, pos2 = (torch.tensor([p0], dtype=torch.int64, device=DEV) for _ in range(2))
st = qkv_attention_state(Hq, Hkv, DEV)
g = torch.Generator(device="cuda").manual_seed(7)
mask = torch.zeros(1, 1, 1, L, dtype=torch.bool, device=DEV)
mask[..., : p0 + 1] = True
x = (torch.randn(1, 1, H, device=DEV, generator=g) * 2).to(dtype)
ref = _two_launches(x, items, nrm, cos, sin, kc, vc, mask, pos, Hq, True)
out = gemv_4bit_qkv_attention(x, items, nrm, cos, sin, kc2, vc2, mask, pos2, st, Hq, D ** -0.5, exact_codes=True)
torch.cuda.synchronize()
print("ref", ref.view(-1)[:4].tolist(), "out", out.view(-1)[:4].tolist(), "equal", torch.equal(out, ref))
# recompute the reference on fresh copies
q, k, v = gemv_4bit_grouped(x, items, exact_codes=True, norm=nrm)
arrive = torch.zeros(1, dtype=torch.int32, device=DEV)
r2 = decode_attention(q.view(1, 1, -1), k.view(1, 1, -1), v.view(1, 1, -1), cos, sin, kc0.clone(), vc0.clone(), mask,
                      torch.tensor([p0], dtype=torch.int64, device=DEV), arrive, Hq, D ** -0.5)
torch.cuda.synchronize()
print("ref again", r2.view(-1)[:4].tolist(), "equal ref", torch.equal(r2, ref), "equal out", torch.equal(r2, out))
print("caches equal", torch.equal(kc, kc2), torch.equal(vc, vc2), "pos", pos.item(), pos2.item(),
      "state", int(st.sum().item()))

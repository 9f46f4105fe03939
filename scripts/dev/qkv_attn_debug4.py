"""Debug: the test's 6-step loop with a per-step report."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_qkv_attention import _setup, _two_launches, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_qkv_attention, qkv_attention_state  # noqa: E402

H, Hq, Hkv, D, L = 4096, 32, 8, 128, 112
dtype = torch.float16
items, kc, vc, cos, sin, nw = _setup(H, Hq, Hkv, D, L, dtype, seed=H + L)
nrm = (nw, 1e-5)
kc2, vc2 = kc.clone(), vc.clone()
p0 = L - 5
pos, pos2 = (torch.tensor([p0], dtype=torch.int64, device=DEV) for _ in range(2))
st = qkv_attention_state(Hq, Hkv, DEV)
g = torch.Generator(device="cuda").manual_seed(7)
for step in range(6):
    mask = torch.zeros(1, 1, 1, L, dtype=torch.bool, device=DEV)
    mask[..., : min(p0 + step + 1, L)] = True
    x = (torch.randn(1, 1, H, device=DEV, generator=g) * 2).to(dtype)
    ref = _two_launches(x, items, nrm, cos, sin, kc, vc, mask, pos, Hq, True)
    out = gemv_4bit_qkv_attention(x, items, nrm, cos, sin, kc2, vc2, mask, pos2, st, Hq, D ** -0.5, exact_codes=True)
    torch.cuda.synchronize()
    d = (out.float() - ref.float()).abs().view(Hq, D).max(-1).values
    rows = [(kc[0, h] != kc2[0, h]).any(-1).nonzero().view(-1).tolist() for h in range(Hkv)]
    print(step, "p", int(pos.item()), int(pos2.item()), "equal", torch.equal(out, ref), "heads differing",
          (d > 0).nonzero().view(-1).tolist(), "k-cache rows differing per kv head", rows,
          "state", int(st.sum().item()), flush=True)

"""Debug: the failing test case step by step (core path vs two launches vs the direct C call)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_qkv_attention import _setup, _two_launches, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_qkv_attention, qkv_attention_state  # noqa: E402

H, Hq, Hkv, D, L = 4096, 32, 8, 128, 112
items, kc, vc, cos, sin, nw = _setup(H, Hq, Hkv, D, L, torch.float16, seed=H + L)
for variant in ("test", "mask_all", "pos50"):
    p0 = 50 if variant == "pos50" else L - 5
    kc1, vc1, kc2, vc2 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    pos, pos2 = (torch.tensor([p0], dtype=torch.int64, device=DEV) for _ in range(2))
    st = qkv_attention_state(Hq, Hkv, DEV)
    mask = torch.zeros(1, 1, 1, L, dtype=torch.bool, device=DEV)
    mask[..., : p0 + 1] = True
    if variant == "mask_all":
        mask[:] = True
    x = (torch.randn(1, 1, H, device=DEV, generator=torch.Generator(device="cuda").manual_seed(7)) * 2).half()
    ref = _two_launches(x, items, (nw, 1e-5), cos, sin, kc1, vc1, mask, pos, Hq, True)
    out = gemv_4bit_qkv_attention(x, items, (nw, 1e-5), cos, sin, kc2, vc2, mask, pos2, st, Hq, D ** -0.5,
                                  exact_codes=True)
    torch.cuda.synchronize()
    d = (out.float() - ref.float()).abs().view(Hq, D).max(-1).values
    print(variant, "equal", torch.equal(out, ref), "caches", torch.equal(kc1, kc2), torch.equal(vc1, vc2),
          "pos", int(pos.item()), int(pos2.item()), "per-head maxdiff", [round(v, 4) for v in d.tolist()], flush=True)

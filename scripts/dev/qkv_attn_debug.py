"""Debug: the fused q/k/v + attention launch against the two launches, piece by piece -- its q/k/v
outputs against the grouped launch's, then its attention output against decode_attention run on
ITS OWN q/k/v (caches copied)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_qkv_attention import _setup, DEV  # noqa: E402
from quantizations_amd import _lib  # noqa: E402
from quantizations_amd.core import _gemv_quant_type, gemv_4bit_grouped, qkv_attention_state, ptr  # noqa: E402
from quantizations_amd.layer_ops import decode_attention  # noqa: E402

H, Hq, Hkv, D, L = 4096, 32, 8, 128, 112
for norm in (False, True):
    items, kc, vc, cos, sin, nw = _setup(H, Hq, Hkv, D, L, torch.float16, seed=11)
    nrm = (nw, 1e-5) if norm else None
    x = torch.randn(1, 1, H, device=DEV).half()
    pos = torch.tensor([50], dtype=torch.int64, device=DEV)
    mask = torch.ones(1, 1, 1, L, dtype=torch.bool, device=DEV)
    kc2, vc2, pos2 = kc.clone(), vc.clone(), pos.clone()
    st = qkv_attention_state(Hq, Hkv, DEV)
    segs = (_lib.GemvSegment * 3)()
    ys = []
    for i, (B, s, _) in enumerate(items):
        y = torch.empty(s.shape[0], dtype=torch.float16, device=DEV)
        am, qam, am2, code2, off, _x = s.scale_args()
        segs[i] = _lib.GemvSegment(s.shape[0], ptr(B), am, qam, am2, code2, off, 0, None, ptr(y))
        ys.append(y)
    out = torch.empty(Hq * D, dtype=torch.float16, device=DEV)
    s0 = items[0][1]
    rc = _lib.lib.qz_gemv_4bit_qkv_attention(ctypes.cast(segs, ctypes.c_void_p), H, ptr(x), 0,
                                             _gemv_quant_type(s0.quant_type, True, x.dtype), 64, 256, None,
                                             ptr(nw) if norm else None, 1e-5, Hq, Hkv, D, L, ptr(cos), ptr(sin),
                                             ptr(kc2), ptr(vc2), ptr(mask), 1, ptr(pos2), ptr(out), D ** -0.5,
                                             ptr(st), _lib.stream_of(x))
    torch.cuda.synchronize()
    print("norm", norm, "rc", rc, "state sum", int(st.sum().item()), "pos", int(pos2.item()))
    ref = gemv_4bit_grouped(x, items, exact_codes=True, norm=nrm)
    for name, a, b in zip("qkv", ys, ref):
        print(f"  {name}: equal {torch.equal(a, b.view(-1))}  maxdiff {(a.float() - b.view(-1).float()).abs().max().item():.3g}")
    arrive = torch.zeros(1, dtype=torch.int32, device=DEV)
    kc3, vc3, pos3 = kc.clone(), vc.clone(), pos.clone()
    o2 = decode_attention(ys[0].view(1, 1, -1), ys[1].view(1, 1, -1), ys[2].view(1, 1, -1), cos, sin, kc3, vc3, mask,
                          pos3, arrive, Hq, D ** -0.5)
    o3 = decode_attention(ref[0].view(1, 1, -1), ref[1].view(1, 1, -1), ref[2].view(1, 1, -1), cos, sin, kc.clone(),
                          vc.clone(), mask, pos.clone(), arrive, Hq, D ** -0.5)
    torch.cuda.synchronize()
    d = (out.float() - o2.view(-1).float()).abs().view(Hq, D).max(-1).values
    print("  attention on its own q/k/v: equal", torch.equal(out, o2.view(-1)), "per-head maxdiff", d.tolist())
    print("  two-launch ref vs attention(own qkv):", torch.equal(o2, o3), " caches equal", torch.equal(kc2, kc3),
          torch.equal(vc2, vc3))

"""Dev timing, Llama-3-8B q/k/v (4096 + 1024 + 1024 rows, K = 4096) with the fused RMSNorm prologue at
QZ_GROUPED_NORM_R = 0 (the geometry's R = 2), 1, 2, 4 (rows per wave: 768 / 1536 / 768 / 384 workgroups,
each repeating the prologue; outputs bit-identical, the per-row sums do not depend on R) and the norm
launch + plain grouped launch; o_proj + residual for scale.  8 rotating weight sets, one HIP graph each."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "dev"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pair_ps_times_lib import graph_time  # noqa: E402
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd import _lib  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped  # noqa: E402
from quantizations_amd.layer_ops import rms_norm  # noqa: E402

H, KV, NC = 4096, 1024, 8
qkv = [_items((H, KV, KV), H, torch.float16, seed=1 + c) for c in range(NC)]
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(1, 1, H, device=DEV, generator=g).half()
w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).half()
outs = [torch.empty(m, device=DEV, dtype=torch.float16) for m in (H, KV, KV)]


def it(c):
    return [(*t, 0, y) for t, y in zip(qkv[c], outs)]


ref = gemv_4bit_grouped(rms_norm(x, w, 1e-5), qkv[0], exact_codes=True)
for R in (0, 1, 2, 4):
    _lib.lib.qz_gemv_set_knob(b"QZ_GROUPED_NORM_R", R)
    y = gemv_4bit_grouped(x, qkv[0], exact_codes=True, norm=(w, 1e-5))
    same = all(torch.equal(u, v) for u, v in zip(y, ref))
    t = graph_time(lambda i: gemv_4bit_grouped(x, it(i % NC), exact_codes=True, norm=(w, 1e-5)))
    print(f"8B q/k/v + fused norm, QZ_GROUPED_NORM_R={R}: {t:.2f} us (== norm launch + grouped: {same})", flush=True)
_lib.lib.qz_gemv_set_knob(b"QZ_GROUPED_NORM_R", 0)
t2 = graph_time(lambda i: gemv_4bit_grouped(rms_norm(x, w, 1e-5), it(i % NC), exact_codes=True))
t0 = graph_time(lambda i: gemv_4bit_grouped(x, it(i % NC), exact_codes=True))
print(f"8B q/k/v: norm launch + grouped {t2:.2f} us, grouped alone {t0:.2f} us", flush=True)

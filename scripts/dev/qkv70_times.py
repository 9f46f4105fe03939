"""Dev timing, Llama-3-70B attention-side launches (K = 8192): q/k/v grouped with the fused RMSNorm
prologue vs the register-held norm launch + the plain grouped launch (outputs compared bit for bit),
and o_proj (8192 x 8192) with its residual epilogue.  8 rotating weight sets, one HIP graph each."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "dev"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pair_ps_times_lib import graph_time  # noqa: E402
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit, gemv_4bit_grouped  # noqa: E402
from quantizations_amd.layer_ops import rms_norm  # noqa: E402

H, KV, NC = 8192, 1024, 8
qkv = [_items((H, KV, KV), H, torch.float16, seed=1 + c) for c in range(NC)]
o = [_items((H,), H, torch.float16, seed=100 + c)[0] for c in range(NC)]
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(1, 1, H, device=DEV, generator=g).half()
res = torch.randn(H, device=DEV, generator=g).half()
w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).half()
outs = [torch.empty(m, device=DEV, dtype=torch.float16) for m in (H, KV, KV)]
a = gemv_4bit_grouped(x, qkv[0], exact_codes=True, norm=(w, 1e-5))
b = gemv_4bit_grouped(rms_norm(x, w, 1e-5), qkv[0], exact_codes=True)
print("fused norm == norm launch + grouped:", all(torch.equal(u, v) for u, v in zip(a, b)), flush=True)


def it(c):
    return [(*t, 0, y) for t, y in zip(qkv[c], outs)]


t_fused = graph_time(lambda i: gemv_4bit_grouped(x, it(i % NC), exact_codes=True, norm=(w, 1e-5)))
t_two = graph_time(lambda i: gemv_4bit_grouped(rms_norm(x, w, 1e-5), it(i % NC), exact_codes=True))
t_plain = graph_time(lambda i: gemv_4bit_grouped(x, it(i % NC), exact_codes=True))
t_o = graph_time(lambda i: gemv_4bit(x, o[i % NC][0], state=o[i % NC][1], exact_codes=True, residual=res))
print(f"70B q/k/v: fused norm {t_fused:.2f} us, norm launch + grouped {t_two:.2f} us, grouped alone {t_plain:.2f} us;"
      f" o_proj + residual {t_o:.2f} us (b2b in one graph)", flush=True)


# (measured once with a QZ_GROUPED_NORM_WK1 knob, since removed: whole rows per wave with the fused
#  prologue at R = 4 / 2 / 1 took 16.37 / 16.96 / 23.40 us against 16.61 for the norm launch + the
#  K-split grouped launch -- profiles/r5_qkv70_forms.txt)

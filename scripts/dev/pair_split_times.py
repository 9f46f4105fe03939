"""Dev timing, Llama-3-70B MLP shapes (K = 8192): the grouped gate/up launch (R = 4, K over two waves)
against the split pair (same geometry + SiLU epilogue), and the small launches around them (the
register-held RMSNorm, the SiLU product).  8 rotating weight copies (1.9 GB, past the Infinity Cache),
a HIP graph of 32 launches over them; the pair's output is checked against grouped + silu_mul."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts", "dev"))
from pair_ps_times_lib import graph_time  # noqa: E402
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu  # noqa: E402
from quantizations_amd.layer_ops import rms_norm, silu_mul  # noqa: E402

K, M, NC = 8192, int(os.environ.get("PAIR_M", "28672")), 8
copies = [_items((M, M), K, torch.float16, seed=1 + c) for c in range(NC)]
g = torch.Generator(device="cuda").manual_seed(3)
x = (torch.randn(1, 1, K, device=DEV, generator=g)).half()
w = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).half()
outs = [torch.empty(M, device=DEV, dtype=torch.float16) for _ in range(2)]
gate, up = gemv_4bit_grouped(x, copies[0], exact_codes=True)
h = gemv_4bit_pair_silu(x, copies[0], exact_codes=True)
print(f"split pair == grouped + silu_mul: {torch.equal(h, silu_mul(gate, up))}", flush=True)
t_gr = graph_time(lambda i: gemv_4bit_grouped(x, [(*it, 0, o) for it, o in zip(copies[i % NC], outs)],
                                              exact_codes=True))
t_pr = graph_time(lambda i: gemv_4bit_pair_silu(x, copies[i % NC], exact_codes=True))
t_si = graph_time(lambda i: silu_mul(gate, up))
t_nm = graph_time(lambda i: rms_norm(x, w, 1e-5))
print(f"{M}x{K} gate/up: grouped {t_gr:.2f} us, split pair {t_pr:.2f} us, silu_mul {t_si:.2f} us, "
      f"rms_norm(K={K}) {t_nm:.2f} us (b2b in one graph)", flush=True)
# whole rows per wave (QZ_PAIR_WK1=1) without the norm, one workgroup per block, R = 4 / 2 / 8
from quantizations_amd import _lib  # noqa: E402
_lib.set_gemv_knob("QZ_PAIR_WK1", 1)
for r in (4, 2, 8):
    _lib.set_gemv_knob("QZ_PAIR_R", r)
    for ps in (0, 2, 3):
        _lib.set_gemv_knob("QZ_PAIR_PS", ps)
        t = graph_time(lambda i: gemv_4bit_pair_silu(x, copies[i % NC], exact_codes=True))
        print(f"whole-row pair R={r} QZ_PAIR_PS={ps}: {t:.2f} us", flush=True)
_lib.set_gemv_knob("QZ_PAIR_WK1", 1)
_lib.set_gemv_knob("QZ_PAIR_R", 0)
_lib.set_gemv_knob("QZ_PAIR_PS", -1)
# with the norm: the norm launch + the whole-row pair (default) against the norm fused into the
# persistent whole-row pair (QZ_PAIR_WK1=2) on the 16-copy table (QZ_PAIR_WT=0: 3 workgroups per CU
# fit) or the 256-B-entry one (64 KiB + the 16 KiB image: one workgroup per CU)
nrm = (w, 1e-5)
ref = gemv_4bit_pair_silu(x, copies[0], exact_codes=True, norm=nrm)
t = graph_time(lambda i: gemv_4bit_pair_silu(x, copies[i % NC], exact_codes=True, norm=nrm))
print(f"norm launch + whole-row pair: {t:.2f} us", flush=True)
_lib.set_gemv_knob("QZ_PAIR_WK1", 2)
for wt, ps in ((0, 3), (0, 2), (0, 4), (1, 2), (0, 0)):
    _lib.set_gemv_knob("QZ_PAIR_WT", wt)
    _lib.set_gemv_knob("QZ_PAIR_PS", ps)
    same = torch.equal(gemv_4bit_pair_silu(x, copies[0], exact_codes=True, norm=nrm), ref)
    t = graph_time(lambda i: gemv_4bit_pair_silu(x, copies[i % NC], exact_codes=True, norm=nrm))
    print(f"norm fused, whole rows, QZ_PAIR_WT={wt} QZ_PAIR_PS={ps}: {t:.2f} us (same bits: {same})", flush=True)
_lib.set_gemv_knob("QZ_PAIR_WK1", 1)
_lib.set_gemv_knob("QZ_PAIR_WT", 1)
_lib.set_gemv_knob("QZ_PAIR_PS", -1)

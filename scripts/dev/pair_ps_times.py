"""Dev timing: the Llama-3-8B gate/up pair launch (qz_gemv_4bit_pair_silu, exact codes, with and
without the fused RMSNorm) with one workgroup per row block against persistent workgroups
(QZ_PAIR_PS: 1-8 = workgroups per CU, >= 16 = the grid).  8 rotating weight copies (470 MB, past the 256 MB Infinity
Cache), a HIP graph of 64 launches over them; every variant's output is compared bit for bit with
the one-workgroup-per-block launch first."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd import _lib  # noqa: E402
from quantizations_amd.core import gemv_4bit_pair_silu  # noqa: E402


def graph_time(fn, reps=64, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


K, M, NC = 4096, int(os.environ.get("PAIR_M", "14336")), 8
copies = [_items((M, M), K, torch.float16, seed=1 + c) for c in range(NC)]
g = torch.Generator(device="cuda").manual_seed(3)
x = (torch.randn(1, 1, K, device=DEV, generator=g)).half()
w = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).half()
variants = [int(v) for v in os.environ.get("PAIR_PS", "0,2,3,4").split(",")]
for nrm in ((w, 1e-5), None) if os.environ.get("PAIR_NONORM", "1") == "1" else ((w, 1e-5),):
    ref = None
    for ps in variants:
        _lib.set_gemv_knob("QZ_PAIR_PS", ps % 1000)
        # 1000 + v: the 256-B-entry (WT) exact-code table at QZ_PAIR_PS = v; below 1000 the 16-copy one
        _lib.set_gemv_knob("QZ_PAIR_WT", 1 if ps >= 1000 else 0)
        out = [gemv_4bit_pair_silu(x, copies[c], exact_codes=True, norm=nrm) for c in range(NC)]
        if ref is None:
            ref = out
        same = all(torch.equal(a, b) for a, b in zip(out, ref))
        t = graph_time(lambda i: gemv_4bit_pair_silu(x, copies[i % NC], exact_codes=True, norm=nrm))
        print(f"pair {M}x{K} norm={nrm is not None} QZ_PAIR_PS={ps}: {t:.2f} us/launch, "
              f"bit-identical to PS=0: {same}", flush=True)
        if not same:
            sys.exit(3)
_lib.set_gemv_knob("QZ_PAIR_PS", -1)
_lib.set_gemv_knob("QZ_PAIR_WT", 1)

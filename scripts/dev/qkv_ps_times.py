"""Dev timing: the Llama-3-8B q/k/v grouped launch with the fused RMSNorm (gemv_4bit_grouped(norm=...),
exact codes) with one workgroup per row block against persistent workgroups (QZ_GROUPED_PS = per CU
or the grid, QZ_GROUPED_PS_R = rows per wave, QZ_GROUPED_WT = the 256-B-entry table).  24 rotating
weight copies (300 MB, past the 256 MB Infinity Cache), a HIP graph of 72 launches over them; every
variant's outputs are compared bit for bit with the default launch first."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped  # noqa: E402


def graph_time(fn, reps=72, iters=20):
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


K = 4096
Ms = tuple(int(v) for v in os.environ.get("QKV_MS", "4096,1024,1024").split(","))
NC = int(os.environ.get("QKV_COPIES", "24"))
copies = [_items(Ms, K, torch.float16, seed=1 + c, bias_seg=1 if c == 0 else None) for c in range(NC)]
outs = [[torch.empty(M, device=DEV, dtype=torch.float16) for M in Ms] for _ in range(NC)]
its = [[(a, b, c, 0, o) for (a, b, c), o in zip(copies[i], outs[i])] for i in range(NC)]
g = torch.Generator(device="cuda").manual_seed(3)
x = (torch.randn(1, 1, K, device=DEV, generator=g)).half()
w = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).half()
variants = os.environ.get("QKV_VARIANTS", "0:0:0,2:2:0,3:2:0,2:1:0,3:1:0,2:2:1,2:1:1,3:1:1").split(",")
ref = None
for v in variants:
    ps, r, wt, early = (v.split(":") + ["0"])[:4]
    os.environ["QZ_GROUPED_PS"], os.environ["QZ_GROUPED_PS_R"], os.environ["QZ_GROUPED_WT"] = ps, r, wt
    os.environ["QZ_GROUPED_EARLY"] = early
    res = [[t.clone() for t in gemv_4bit_grouped(x, its[c], exact_codes=True, norm=(w, 1e-5))] for c in range(NC)]
    if ref is None:
        ref = res
    same = all(torch.equal(a, b) for ra, rb in zip(res, ref) for a, b in zip(ra, rb))
    t = graph_time(lambda i: gemv_4bit_grouped(x, its[i % NC], exact_codes=True, norm=(w, 1e-5)))
    print(f"qkv {Ms}x{K} norm PS={ps} R={r} WT={wt} EARLY={early}: {t:.2f} us/launch, bit-identical to the first: {same}", flush=True)
    if not same:
        sys.exit(3)
for k in ("QZ_GROUPED_PS", "QZ_GROUPED_PS_R", "QZ_GROUPED_WT", "QZ_GROUPED_EARLY"):
    os.environ.pop(k, None)

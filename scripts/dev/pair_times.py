"""Dev timing: Llama-3-8B gate/up as the grouped launch (+ fused norm) followed by qz_silu_mul,
against the one-launch pair (qz_gemv_4bit_pair_silu), exact codes, each as a HIP graph of 64
dependent repetitions (the decode step's dependent-launch regime)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "dev"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu  # noqa: E402
from quantizations_amd.layer_ops import silu_mul  # noqa: E402


def graph_time(fn, reps=64, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
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
items = _items((14336, 14336), K, torch.float16, seed=1)
x = torch.randn(1, 1, K, device=DEV).half()
w = (1 + 0.1 * torch.randn(K, device=DEV)).half()
outs = [torch.empty(14336, device=DEV, dtype=torch.float16) for _ in range(2)]
it = [(a, b, c, 0, o) for (a, b, c), o in zip(items, outs)]
for nrm in (None, (w, 1e-5)):
    t_g = graph_time(lambda: gemv_4bit_grouped(x, it, exact_codes=True, norm=nrm))
    t_gs = graph_time(lambda: silu_mul(*gemv_4bit_grouped(x, it, exact_codes=True, norm=nrm)))
    t_p = graph_time(lambda: gemv_4bit_pair_silu(x, items, exact_codes=True, norm=nrm))
    print(f"gateup norm={nrm is not None}: grouped {t_g:.2f} us, grouped + silu_mul {t_gs:.2f} us, "
          f"pair {t_p:.2f} us", flush=True)

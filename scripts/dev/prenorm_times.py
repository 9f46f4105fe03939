"""Dev timing: grouped decode GEMV alone, RMSNorm + grouped GEMV (two launches), and the fused
launch, at the Llama-3-8B q/k/v and gate/up shapes (exact codes), each as a HIP graph of 64
dependent repetitions (the decode step's dependent-launch regime)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit_grouped  # noqa: E402
from quantizations_amd.layer_ops import rms_norm  # noqa: E402


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


for name, Ms, K in (("qkv", (4096, 1024, 1024), 4096), ("gateup", (14336, 14336), 4096),
                    ("qkv70b", (8192, 1024, 1024), 8192), ("gateup70b", (28672, 28672), 8192)):
    items = _items(Ms, K, torch.float16, seed=1)
    x = torch.randn(1, 1, K, device=DEV).half()
    w = (1 + 0.1 * torch.randn(K, device=DEV)).half()
    outs = [torch.empty(M, device=DEV, dtype=torch.float16) for M in Ms]
    it = [(a, b, c, 0, o) for (a, b, c), o in zip(items, outs)]
    t_g = graph_time(lambda: gemv_4bit_grouped(x, it, exact_codes=True))
    t_two = graph_time(lambda: gemv_4bit_grouped(rms_norm(x, w, 1e-5), it, exact_codes=True))
    t_f = graph_time(lambda: gemv_4bit_grouped(x, it, exact_codes=True, norm=(w, 1e-5)))
    print(f"{name}: grouped {t_g:.2f} us, norm + grouped {t_two:.2f} us, fused {t_f:.2f} us", flush=True)

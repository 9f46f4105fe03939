"""Low-T prefill route crossover (GPU): gemm_4bit(route="fused") -- the multi-token kernel
(T <= 16) and the 128-row tile kernel (17 <= T < 4096) -- against route="blas" (dequantize_4bit
+ the library GEMM, the reference's modules.py:62-64), whole-route times including the
dequant pass, for the four Llama-3-8B shapes (default) or the four Llama-3-70B shapes ("70b").  Sets
core.fused_max_tokens' table.
   python scripts/prefill_lowT_sweep.py [8b|70b]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import gemm_4bit, quantize_4bit  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(50_000_000)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


dev = torch.device("cuda")
out = {}
SHAPES = {"8b": [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336)],
          "70b": [(8192, 8192), (1024, 8192), (28672, 8192), (8192, 28672)]}
for (M, K) in SHAPES[sys.argv[1] if len(sys.argv) > 1 else "8b"]:
    torch.manual_seed(M + K)
    packed, st = quantize_4bit((torch.randn(M, K, device=dev) * 0.02).half(), quant_type="nf4")
    for T in (2, 8, 16, 17, 32, 64, 128, 192, 256, 384, 512):
        x = torch.randn(T, K, device=dev, dtype=torch.float16)
        f = timed(lambda: gemm_4bit(x, packed, st, route="fused"))
        b = timed(lambda: gemm_4bit(x, packed, st, route="blas"))
        r = {"fused_us": round(f, 2), "dequant_blas_us": round(b, 2), "fused_faster": f < b}
        out[f"{M}x{K} T={T}"] = r
        print(f"{M}x{K} T={T}", json.dumps(r), flush=True)
print(json.dumps(out))

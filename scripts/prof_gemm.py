"""Drive the fused prefill GEMM (core.gemm_4bit, route='fused') on one shape for
rocprofv3 passes.   python scripts/prof_gemm.py T M K [qt] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import gemm_4bit, quantize_4bit  # noqa: E402

T, M, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
qt = sys.argv[4] if len(sys.argv) > 4 else "nf4"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dev = torch.device("cuda")
torch.manual_seed(0)
packed, st = quantize_4bit((torch.randn(M, K, device=dev) * 0.02).half(), quant_type=qt)
x = torch.randn(T, K, device=dev, dtype=torch.float16)
for _ in range(iters):
    gemm_4bit(x, packed, st, route="fused")
torch.cuda.synchronize()
print(f"done {T}x{M}x{K} {qt}")

"""Both prefill routes at config #4 (T = 8 x 2048 = 16384 tokens, 4096x4096 NF4+DQ) for
rocprofv3 passes: the fused MFMA kernel, then dequantize_4bit + hipBLASLt.
   python scripts/prof_prefill.py [iters] [route,route,...]   (default fused,dequant; gemm16 = dequant +
   our 16-bit GEMM)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import gemm_4bit, quantize_4bit  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
torch.manual_seed(0)
packed, st = quantize_4bit((torch.randn(4096, 4096, device=dev) * 0.02).half(), quant_type="nf4")
x = torch.randn(16384, 4096, device=dev, dtype=torch.float16)
routes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fused", "dequant"]
for route in routes:
    for _ in range(iters):
        gemm_4bit(x, packed, st, route=route)
    torch.cuda.synchronize()
print("done")

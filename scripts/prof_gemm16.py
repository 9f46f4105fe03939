"""qz_gemm_16bit (schedule QZ_GEMM16_SCHED, default 971) and hipBLASLt (F.linear) on the same randn fp16
operands, for rocprofv3 passes: config #4's 4096 x 4096 at T = 16384 unless M K T are given.
   python scripts/prof_gemm16.py [iters] [M K T]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import gemm_16bit  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
M, K, T = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (4096, 4096, 16384)
dev = torch.device("cuda")
torch.manual_seed(0)
W = (torch.randn(M, K, device=dev) * 0.02).half()
x = torch.randn(T, K, device=dev, dtype=torch.float16)
for _ in range(iters):
    gemm_16bit(x, W)
torch.cuda.synchronize()
for _ in range(iters):
    torch.nn.functional.linear(x, W)
torch.cuda.synchronize()
print("done")

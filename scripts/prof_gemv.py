"""Drive the product GEMV (core.gemv_4bit) on one shape with rotating weight
copies, for rocprofv3 kernel-trace / PMC passes.

  python scripts/prof_gemv.py M K [qt] [iters] [copies]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import gemv_4bit, quantize_4bit  # noqa: E402

M, K = int(sys.argv[1]), int(sys.argv[2])
qt = sys.argv[3] if len(sys.argv) > 3 else "nf4"
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 200
copies = int(sys.argv[5]) if len(sys.argv) > 5 else max(2, min(64, (600 << 20) // (M * K // 2)))
dev = torch.device("cuda")
torch.manual_seed(0)
W = (torch.randn(M, K, device=dev) * 0.02).half()
packed, st = quantize_4bit(W, quant_type=qt)
del W
sets = []
for _ in range(copies):
    s2 = type(st)(absmax=st.absmax.clone(), shape=st.shape, code=st.code, blocksize=st.blocksize,
                  quant_type=st.quant_type, dtype=st.dtype, offset=st.offset, state2=st.state2)
    sets.append((packed.clone(), s2))
x = torch.randn(1, K, device=dev, dtype=torch.float16)
y = torch.empty(1, M, device=dev, dtype=torch.float16)
for i in range(iters):
    p, s = sets[i % copies]
    gemv_4bit(x, p, y, state=s)
torch.cuda.synchronize()
print(f"done {M}x{K} {qt} iters={iters} copies={copies}")

"""Counter target: the two 4096-row launches of a Llama-3-8B decode layer as the decode runs them --
q/k/v grouped with the fused input RMSNorm (4096 + 1024 + 1024 rows, K = 4096) and o_proj (4096 x
4096) with the residual epilogue, NF4 + double quant, exact codes -- over 8 rotating weight sets,
`iters` of each (eager, so rocprofv3 sees every dispatch)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_prenorm import _items, DEV  # noqa: E402
from quantizations_amd.core import gemv_4bit, gemv_4bit_grouped  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
H, KV, NC = 4096, 1024, 8
qkv = [_items((H, KV, KV), H, torch.float16, seed=1 + c) for c in range(NC)]
o = [_items((H,), H, torch.float16, seed=100 + c)[0] for c in range(NC)]
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.randn(1, 1, H, device=DEV, generator=g).half()
res = torch.randn(H, device=DEV, generator=g).half()
w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).half()
outs = [torch.empty(m, device=DEV, dtype=torch.float16) for m in (H, KV, KV)]
for i in range(iters):
    c = i % NC
    gemv_4bit_grouped(x, [(*t, 0, y) for t, y in zip(qkv[c], outs)], exact_codes=True, norm=(w, 1e-5))
    gemv_4bit(x, o[c][0], state=o[c][1], exact_codes=True, residual=res)
torch.cuda.synchronize()
print("ok", iters)

"""Prefill route crossover (GPU): for each (M, K) and token count T, the dequant
(bit-exact, ours) + qz_gemm_16bit (8-phase MFMA, ours) route vs dequant + the
library GEMM (hipBLASLt, the reference's F.linear), plus the fused kernel; and a
rel-err check of qz_gemm_16bit against an fp64 product.  Sets GEMM16_MIN_TILES.
   python scripts/prefill_route_sweep.py [T,T,...]   (default 513,1024,2048,4096,8192,16384)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import dequantize_4bit, gemm_16bit, gemm_4bit, quantize_4bit  # noqa: E402


def timed(fn, iters=10):
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
Ts = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [513, 1024, 2048, 4096, 8192, 16384]
out = {}
for (M, K) in [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336)]:
    torch.manual_seed(M + K)
    packed, st = quantize_4bit((torch.randn(M, K, device=dev) * 0.02).half(), quant_type="nf4")
    W = dequantize_4bit(packed, st).t()
    for T in Ts:
        x = torch.randn(T, K, device=dev, dtype=torch.float16)
        ref = (x.double() @ W.double().t())
        y = gemm_16bit(x, W)
        rel = float(((y.double() - ref).norm() / ref.norm()).item())
        del ref
        r = {"tiles": ((T + 255) // 256) * ((M + 255) // 256),
             "gemm16_us": round(timed(lambda: gemm_16bit(x, W)), 2),
             "blas_us": round(timed(lambda: torch.nn.functional.linear(x, W)), 2),
             "dequant_us": round(timed(lambda: dequantize_4bit(packed, st)), 2),
             "fused_us": round(timed(lambda: gemm_4bit(x, packed, st, route="fused")), 2),
             "gemm16_rel_err": float(f"{rel:.3e}")}
        r["gemm16_TFLOPs"] = round(2.0 * T * M * K / (r["gemm16_us"] * 1e-6) / 1e12, 1)
        r["blas_TFLOPs"] = round(2.0 * T * M * K / (r["blas_us"] * 1e-6) / 1e12, 1)
        out[f"{M}x{K} T={T}"] = r
        print(f"{M}x{K} T={T}", json.dumps(r), flush=True)
        del x, y
print(json.dumps(out))

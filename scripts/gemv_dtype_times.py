"""Decode GEMV launch time by activation dtype (GPU): the product gemv_4bit / grouped gate/up
launches for fp16, bf16 and fp32 x at the Llama-3-8B shapes, back-to-back on a parked stream,
8 rotating weight sets.
   python scripts/gemv_dtype_times.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd.core import gemv_4bit, gemv_4bit_grouped, quantize_4bit  # noqa: E402


def timed(fn, n, iters=200):
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(50_000_000)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters * 1e3, 3)


dev = torch.device("cuda")
out = {}
for (M, K) in [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336)]:
    sets = [quantize_4bit((torch.randn(M, K, device=dev) * 0.02).half(), quant_type="nf4") for _ in range(8)]
    row = {}
    for dt in (torch.float16, torch.bfloat16, torch.float32):
        x = torch.randn(1, K, device=dev).to(dt)
        row[str(dt).split(".")[-1]] = timed(lambda i: gemv_4bit(x, sets[i % 8][0], state=sets[i % 8][1]), 8)
    out[f"{M}x{K}"] = row
    print(f"{M}x{K}", json.dumps(row), flush=True)
    del sets
sets = [[quantize_4bit((torch.randn(14336, 4096, device=dev) * 0.02).half(), quant_type="nf4") for _ in range(2)]
        for _ in range(4)]
row = {}
for dt in (torch.float16, torch.bfloat16, torch.float32):
    x = torch.randn(1, 1, 4096, device=dev).to(dt)
    row[str(dt).split(".")[-1]] = timed(
        lambda i: gemv_4bit_grouped(x, [(p, s, None) for p, s in sets[i % 4]]), 4)
out["gate/up grouped 2x14336x4096"] = row
print("gate/up grouped", json.dumps(row), flush=True)
print(json.dumps(out))

"""k_gemm16_4d schedules vs hipBLASLt (GPU, dev measurement): config #4's three Llama-3-8B shapes at
T = 16384 (and 4096^2 at T = 4096), fp16 randn operands.  Every schedule's output is compared bit
for bit with schedule 0's; times are medians over ROUNDS rounds that interleave every route, so DVFS
drift hits all of them alike.
   python scripts/gemm16_sched_sweep.py [S,S,...]   (default 0,1,3,9,11)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd import _lib  # noqa: E402
from quantizations_amd.core import gemm_16bit  # noqa: E402

ROUNDS = int(os.environ.get("ROUNDS", "7"))
# DATA=uniform: gemm16_stamps.hip's operands (fp16 bits (h & 0x83FF) | 0x3800: |v| in [0.5, 1), random sign
# and mantissa) instead of randn -- the chip's clock under load depends on the operands' bits
DATA = os.environ.get("DATA", "randn")


def operand(rows, cols, scale):
    if DATA == "uniform":
        h = torch.randint(0, 1 << 16, (rows, cols), device="cuda", dtype=torch.int32)
        v = (h & 0x83FF) | 0x3800
        return torch.where(v >= 32768, v - 65536, v).to(torch.int16).view(torch.float16)
    return (torch.randn(rows, cols, device="cuda") * scale).half()
scheds = [int(s) for s in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 3, 9, 11]


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(20_000_000)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


dev = torch.device("cuda")
out = {}
for (M, K, T) in [(4096, 4096, 16384), (14336, 4096, 16384), (4096, 14336, 16384), (4096, 4096, 4096)]:
    torch.manual_seed(M + K + T)
    W = operand(M, K, 0.02)
    x = operand(T, K, 1.0)
    iters = max(2, int(2e12 / (2.0 * T * M * K) * 3))
    ys = {}
    for s in scheds:
        _lib.set_gemv_knob("QZ_GEMM16_SCHED", s)
        ys[s] = gemm_16bit(x, W)
    torch.cuda.synchronize()
    same = {s: bool(torch.equal(ys[s], ys[scheds[0]])) for s in scheds}
    del ys
    times = {f"s{s}": [] for s in scheds}
    times["blas"] = []
    for r in range(ROUNDS):
        for s in scheds:
            _lib.set_gemv_knob("QZ_GEMM16_SCHED", s)
            times[f"s{s}"].append(timed(lambda: gemm_16bit(x, W), iters))
        times["blas"].append(timed(lambda: torch.nn.functional.linear(x, W), iters))
    flop = 2.0 * T * M * K
    res = {"bit_identical_to_first": same}
    for k, v in times.items():
        v.sort()
        med = v[len(v) // 2]
        res[k] = {"us": round(med, 2), "TFLOPs": round(flop / (med * 1e-6) / 1e12, 1)}
    out[f"{M}x{K} T={T}"] = res
    print(f"{M}x{K} T={T}", json.dumps(res), flush=True)
    del x, W
_lib.set_gemv_knob("QZ_GEMM16_SCHED", 971)
print(json.dumps(out))

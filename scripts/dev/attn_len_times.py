"""Decode attention (Llama-3-8B / 70B heads) b2b in one HIP graph over 32 layers' caches, against the
cache length L: how much of the launch is the per-workgroup K/V cache stream (L rows x 512 B)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "dev"))
from pair_ps_times_lib import graph_time  # noqa: E402
from quantizations_amd.layer_ops import decode_attention  # noqa: E402

dev = torch.device("cuda")
for Hq, Hkv in ((32, 8), (64, 8)):
    for L in (32, 64, 112, 128):
        D, NL = 128, 32
        kcs = [torch.randn(1, Hkv, L, D, device=dev).half() for _ in range(NL)]
        vcs = [torch.randn(1, Hkv, L, D, device=dev).half() for _ in range(NL)]
        q = torch.randn(1, 1, Hq * D, device=dev).half()
        k = torch.randn(1, 1, Hkv * D, device=dev).half()
        v = torch.randn(1, 1, Hkv * D, device=dev).half()
        cos = torch.rand(1, 1, D, device=dev).half()
        sin = torch.rand(1, 1, D, device=dev).half()
        mask = torch.ones(1, 1, 1, L, dtype=torch.bool, device=dev)
        poss = [torch.tensor([0], device=dev) for _ in range(NL)]   # < 30 calls each: stays inside L
        arr = torch.zeros(1, dtype=torch.int32, device=dev)

        def f(i):
            return decode_attention(q, k, v, cos, sin, kcs[i % NL], vcs[i % NL], mask, poss[i % NL], arr, Hq, D ** -0.5)
        t = graph_time(f)
        print(f"Hq={Hq} Hkv={Hkv} L={L}: {t:.2f} us per launch", flush=True)

"""Decode attention at the head counts one rank keeps under the head-sharded row split (N = 1, 2, 4, 8;
parallel.shard_attention_heads): Llama-3-8B (32 q / 8 kv heads) and Llama-3-70B (64 / 8), D = 128, a
static cache of L = 128 positions, b2b in one HIP graph over 32 layers' caches -- the per-layer
attention row of DESIGN.md section 6's budget."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "dev"))
from pair_ps_times_lib import graph_time  # noqa: E402
from quantizations_amd.layer_ops import decode_attention  # noqa: E402

dev = torch.device("cuda")
out = {}
for model, (HQ, HKV) in (("llama3-8b", (32, 8)), ("llama3-70b", (64, 8))):
    for N in (1, 2, 4, 8):
        Hq, Hkv, D, L, NL = HQ // N, HKV // N, 128, 128, 32
        kcs = [torch.randn(1, Hkv, L, D, device=dev).half() for _ in range(NL)]
        vcs = [torch.randn(1, Hkv, L, D, device=dev).half() for _ in range(NL)]
        q = torch.randn(1, 1, Hq * D, device=dev).half()
        k = torch.randn(1, 1, Hkv * D, device=dev).half()
        v = torch.randn(1, 1, Hkv * D, device=dev).half()
        cos = torch.rand(1, 1, D, device=dev).half()
        sin = torch.rand(1, 1, D, device=dev).half()
        mask = torch.ones(1, 1, 1, L, dtype=torch.bool, device=dev)
        poss = [torch.tensor([0], device=dev) for _ in range(NL)]
        arr = torch.zeros(1, dtype=torch.int32, device=dev)

        def f(i):
            return decode_attention(q, k, v, cos, sin, kcs[i % NL], vcs[i % NL], mask, poss[i % NL], arr, Hq, D ** -0.5)
        t = graph_time(f)
        out[f"{model} N={N}"] = {"q_heads": Hq, "kv_heads": Hkv, "L": L, "us_per_launch": round(t, 2)}
        print(f"{model} N={N}: {Hq} q / {Hkv} kv heads, L={L}: {t:.2f} us per launch", flush=True)
print(json.dumps(out))

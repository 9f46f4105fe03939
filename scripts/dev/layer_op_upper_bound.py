"""Dev measurement (not a product path, wrong numerics on purpose): the bs=1 Llama-3-8B graph decode
step with the RMSNorm launches removed (norm -> identity) and/or the SiLU*up launch removed
(h = gate), i.e. the most a fusion of those ops into the neighbouring GEMVs could save.
   python scripts/dev/layer_op_upper_bound.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def run(skip_norm: bool, skip_silu: bool, steps=64, warmup=8):
    model, cfg = bench.build_model(0, 0)
    bench.prepare_decode_model(model, 0, 1, False)
    for m in model.modules():
        if skip_norm and m.__dict__.get("_qz_fused_norm"):
            m.__dict__["forward"] = lambda h: h
        if skip_silu and m.__dict__.get("_qz_fused_mlp"):
            def fwd(x, mod=m):
                g = mod.gate_proj(x)
                mod.up_proj(x)
                return mod.down_proj(g)
            m.__dict__["forward"] = fwd
    dt, _ = bench.decode_bench_graph(model, cfg, steps, warmup, 32, 1)
    del model
    torch.cuda.empty_cache()
    return dt / steps * 1e3


for sn, ss in ((False, False), (True, False), (False, True), (True, True), (False, False)):
    print(f"skip_norm={sn} skip_silu={ss}: {run(sn, ss):.4f} ms/token", flush=True)

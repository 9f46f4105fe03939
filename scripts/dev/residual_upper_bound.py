"""Dev measurement (wrong numerics on purpose): the bs=1 graph decode step with the decoder
layers' two residual adds removed, against the product layout -- the most a fusion of those
adds into the neighbouring launches could save.
   python scripts/dev/residual_upper_bound.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def run(skip_adds: bool, steps=64, warmup=8):
    model, cfg = bench.build_model(0, 0)
    bench.prepare_decode_model(model, 0, 1, False)
    if skip_adds:
        for layer in model.model.layers:
            def fwd(hidden_states, attention_mask=None, position_ids=None, past_key_values=None, use_cache=False,
                    position_embeddings=None, mod=layer, **kw):
                h = mod.input_layernorm(hidden_states)
                h, _ = mod.self_attn(hidden_states=h, attention_mask=attention_mask, position_ids=position_ids,
                                     past_key_values=past_key_values, use_cache=use_cache,
                                     position_embeddings=position_embeddings, **kw)
                h = mod.post_attention_layernorm(h)
                return mod.mlp(h)
            layer.__dict__["forward"] = fwd
    dt, _ = bench.decode_bench_graph(model, cfg, steps, warmup, 32, 1)
    del model
    torch.cuda.empty_cache()
    return dt / steps * 1e3


for sk in (False, True, False):
    print(f"skip_residual_adds={sk}: {run(sk):.4f} ms/token", flush=True)

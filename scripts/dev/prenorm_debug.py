"""Dev check: where does the prenorm model's decode differ from the reference?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_prenorm import _llama, DEV  # noqa: E402
from transformers.cache_utils import StaticCache  # noqa: E402
from quantizations_amd.integration import fuse_prenorm  # noqa: E402

model, cfg = _llama()
ids = torch.randint(0, cfg.vocab_size, (1, 10), device=DEV, generator=torch.Generator(device="cuda").manual_seed(3))
acts = {}
names = []


def hook(name):
    def f(mod, inp, out):
        o = out[0] if isinstance(out, tuple) else out
        acts.setdefault(name, []).append(o.detach().clone())
    return f


for name, mod in model.named_modules():
    if name.endswith(("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj", "input_layernorm",
                      "post_attention_layernorm")) or name in ("model.norm", "lm_head"):
        mod.register_forward_hook(hook(name))
        names.append(name)


def greedy(n):
    cache = StaticCache(config=cfg, max_cache_len=32)
    out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(10, device=DEV))
    logits = [out.logits[:, -1].clone()]
    tok = out.logits[:, -1:].argmax(-1)
    for i in range(n):
        pos = torch.tensor([10 + i], device=DEV)
        lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos.view(1, 1)).logits
        logits.append(lo[:, -1].clone())
        tok = lo[:, -1:].argmax(-1)
    return logits


with torch.no_grad():
    r1 = greedy(3)
    r2 = greedy(3)
    print("unfused decode deterministic:", [bool(torch.equal(x, y)) for x, y in zip(r1, r2)])
    acts.clear()
    a = greedy(3)
    na = {k: len(v) for k, v in acts.items()}
    print("prenorm absorbed:", fuse_prenorm(model))
    b = greedy(3)
    b2 = greedy(3)
    print("fused decode deterministic:", [bool(torch.equal(x, y)) for x, y in zip(b, b2)])
    for i, (x, y) in enumerate(zip(a, b)):
        print(f"step {i}: equal {torch.equal(x, y)} maxdiff {(x.float() - y.float()).abs().max().item():.3g}")
    for k in names:
        v = acts[k]
        n = na[k]
        for j in range(n):
            if j + n < len(v) and not torch.equal(v[j], v[j + n]):
                print(f"{k:45s} call {j}: differs, maxdiff {(v[j].float() - v[j + n].float()).abs().max().item():.3g}"
                      f" shape {tuple(v[j].shape)}")
                break

"""Headline benchmark: Llama-3-8B NF4 (double quant) batch-1 greedy decode on MI355X
(BASELINE.json configs[1]) plus the 4096x4096 decode-GEMV roofline and the
config #1 CPU dequant+matmul baseline.

  python bench.py [--gpus N] [--steps K] [--warmup W]

* Model: transformers LlamaForCausalLM with the Llama-3-8B architecture,
  random-init fp16 weights (no network -> no checkpoint), every decoder
  nn.Linear replaced by quantizations_amd.Linear4bit(quant_type="nf4",
  compress_statistics=True) through replace_with_bnb_linear; lm_head stays
  fp16 (transformers' default skip list).  A step = one generated token
  (full forward: embeddings, 32 layers with attention + KV cache, lm_head,
  argmax).  value = generated tokens / s.
* N > 1 (torchrun, one process per GPU), default: the north-star layout
   -- ONE bs=1 decode stream served by all N GPUs,
  every Linear4bit row-split (rank p keeps rows [p*M/N, (p+1)*M/N) of the
  global quant state) and its fp16 output RCCL all-gathered over xGMI
  (q/k/v and gate/up shards exchanged by one all-gather per group): strong
  scaling, global batch 1, parallelism tp{N}-rowsplit-allgather.  The
  weak-scaling layout (--weak: one bs=1 stream per GPU, global batch N,
  Megatron pairing -- q/k/v/gate/up column-parallel, o/down row-parallel +
  one all-reduce each) is measured after it and reported only as the extra
  key `weak_scaling_extra` (--no-extra-weak skips it).
* roofline: the 4096x4096 NF4+DQ fused GEMV alone, 64 rotating weight copies
  (> the 256 MiB Infinity Cache), HIP events on the launch stream around 400
  back-to-back launches (average launch duration, matches rocprofv3);
  algorithmic bytes per launch = 8,672,324.
* cpu_baseline (rank 0, N = 1): the oracle's CPU dequant + torch.matmul of one
  Linear4bit(4096,4096) NF4 layer (config #1), scaled to the 224 Linear4bit
  layers of one token.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

LLAMA3_8B = dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                 num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0, max_position_embeddings=8192,
                 rms_norm_eps=1e-5, tie_word_embeddings=False)
LLAMA3_70B = dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                  num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0, max_position_embeddings=8192,
                  rms_norm_eps=1e-5, tie_word_embeddings=False)
MODELS = {"llama3-8b": LLAMA3_8B, "llama3-70b": LLAMA3_70B}
# Linear4bit shapes of one Llama-3-8B layer (q, k, v, o, gate, up, down) as (M, K)
LAYER_SHAPES = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
GEMV_BYTES_4096 = 8_672_324  # packed 8,388,608 + qabsmax 262,144 + absmax2 4,096 + offset 4 + code2 1,024 + LUT 64
#                              + x 8,192 + y 8,192   
CAPTURE_MODE = "thread_local"  # bench --capture-mode (the RCCL watchdog thread queries events during capture)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(layers: int, seed: int, model_name: str = "llama3-8b", quant_type: str = "nf4",
                double_quant: bool = True, dtype: torch.dtype = torch.float16,
                compute_dtype: torch.dtype = torch.float32):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import replace_with_bnb_linear

    base = MODELS[model_name]
    cfg = LlamaConfig(**{**base, "num_hidden_layers": layers or base["num_hidden_layers"]})
    torch.manual_seed(seed)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg)
    torch.set_default_dtype(prev)
    model.eval()
    replace_with_bnb_linear(model, modules_to_not_convert=["lm_head"], quant_type=quant_type,
                            compress_statistics=double_quant,
                            compute_dtype=compute_dtype)
    torch.cuda.empty_cache()
    return model, cfg


@torch.inference_mode()
def decode_bench(model, cfg, steps: int, warmup: int, prompt_len: int, world: int, batch: int = 1):
    from transformers.cache_utils import DynamicCache

    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1234)
    ids = torch.randint(0, cfg.vocab_size, (batch, prompt_len), generator=g).to(dev)
    cache = DynamicCache()
    out = model(input_ids=ids, past_key_values=cache, use_cache=True)      # prefill (fused MFMA GEMM path)
    nxt = out.logits[:, -1:].argmax(-1)
    for _ in range(warmup):
        out = model(input_ids=nxt, past_key_values=cache, use_cache=True)
        nxt = out.logits[:, -1:].argmax(-1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks = []
    for _ in range(steps):
        out = model(input_ids=nxt, past_key_values=cache, use_cache=True)
        nxt = out.logits[:, -1:].argmax(-1)
        toks.append(nxt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    return dt, torch.cat(toks, dim=1)


GREEDY = "kernel"   # --greedy: the decode step's greedy pick + feedback ("kernel": layer_ops.greedy_step)


def greedy_token(logits: torch.Tensor) -> torch.Tensor:
    """argmax over the last dim ([B, 1, V] -> [B, 1]), the first maximal index as torch.argmax
    returns it, in two parallel stages when V splits into 256-wide rows: a row max with its
    first index, then the first row holding the global max.  torch's one-pass argmax reduces the
    128256 Llama-3 logits with a handful of workgroups (43.7 us of a 2 ms decode step,
    profiles/r3_decode_anatomy_fused.txt); the two stages spread it over 501."""
    V = logits.shape[-1]
    if V % 256 or V < 4096:
        return logits.argmax(-1)
    m, i = logits.reshape(*logits.shape[:-1], V // 256, 256).max(-1)   # [B, 1, V/256]
    r = m.argmax(-1, keepdim=True)                                       # first row with the max
    return (i.gather(-1, r) + r * 256).squeeze(-1)


@torch.inference_mode()
def decode_bench_graph(model, cfg, steps: int, warmup: int, prompt_len: int, world: int, batch: int = 1,
                       graph: bool = True, device: str = "cuda"):
    """Same workload as decode_bench, with the decode step captured once into a HIP
    graph (StaticCache, static token/position buffers; the graph contains the
    whole forward, the argmax and the feedback of the token into the next
    step).  One replay = one generated token per stream (`batch` streams).
    graph=False runs the identical step eagerly (the gloo CPU test of the
    multi-GPU layout drives this function with it).  Returns (seconds for the
    timed steps, token history [batch, prompt + warmup + steps + 8])."""
    from transformers.cache_utils import StaticCache

    dev = torch.device(device)
    cuda = dev.type == "cuda"
    g = torch.Generator(device="cpu").manual_seed(1234)
    ids = torch.randint(0, cfg.vocab_size, (batch, prompt_len), generator=g).to(dev)
    cache = StaticCache(config=cfg, max_cache_len=prompt_len + warmup + steps + 8)
    out = model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(prompt_len, device=dev),
                use_cache=True)
    tok = out.logits[:, -1:].argmax(-1)
    pos = torch.tensor([prompt_len], device=dev, dtype=torch.long)
    hist = torch.zeros((batch, prompt_len + warmup + steps + 8), device=dev, dtype=torch.long)
    pos_ids = pos.view(1, 1).expand(batch, 1)

    def step():
        lo = model(input_ids=tok, past_key_values=cache, cache_position=pos, position_ids=pos_ids,
                   use_cache=True).logits
        if GREEDY == "kernel" and lo.is_cuda:
            from quantizations_amd.layer_ops import greedy_step
            greedy_step(lo[:, -1], hist, pos, tok)   # argmax + the three feedback writes, one launch
            return
        nxt = greedy_token(lo[:, -1:]) if GREEDY == "two-stage" else lo[:, -1:].argmax(-1)
        hist.index_copy_(1, pos, nxt.view(batch, 1))
        tok.copy_(nxt)
        pos.add_(1)

    run = step
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(s)
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg, capture_error_mode=CAPTURE_MODE):
            step()
        run = cg.replay
        if world > 1:
            dist.barrier()   # every rank starts replaying together (in-graph exchanges wait on peers)
    for _ in range(warmup):
        run()
    if world > 1:
        dist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    if cuda:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    return dt, hist


def prepare_decode_model(model, rank: int, world: int, sharded: bool, tp_mode: str = "gather",
                         fuse: bool = True, layer_ops: str = "all", local_matmul=None, gatherer=None,
                         prenorm: bool = True, attention: bool = True, residual: bool = True,
                         mlp_pair: bool = True,
                         glue: bool = True, lm_head: bool = True, shard_head: bool = True,
                         head_sharded_attention: bool = True):
    """The bench's model layout after replace_with_bnb_linear: shard every
    Linear4bit for the multi-GPU layout (tp_mode "gather": row split + all-gather,
    "pair": Megatron column/row pairing), attach the q/k/v and gate/up decode
    groups and the one-launch layer ops (with `attention`, the decode step's rotary + cache
    update + attention as one launch), and (single-GPU layout, `prenorm`) absorb
    each layer's two RMSNorms into those groups' launches.  `local_matmul` is the CPU
    test hook of parallel.py (None = the HIP kernels).  Returns (n_groups,
    n_layer_ops); absorbed norms count as layer ops."""
    if sharded:
        if tp_mode == "pair":
            from quantizations_amd.parallel import apply_tensor_parallel
            apply_tensor_parallel(model, rank, world, local_matmul=local_matmul, gatherer=gatherer)
        else:
            from quantizations_amd.parallel import shard_attention_heads, shard_lm_head, shard_model_linear4bit
            shard_model_linear4bit(model, rank, world, local_matmul=local_matmul, gatherer=gatherer)
            if head_sharded_attention:   # q/k/v rows stay local: each rank attends over its own heads
                shard_attention_heads(model)
            if shard_head:   # the fp16 lm_head's rows too (each rank 1/N of its 1-2 GB), gathered like the rest
                shard_lm_head(model, rank, world, gatherer=gatherer,
                              dense_kernel=lm_head and layer_ops != "none")
        import gc
        gc.collect()  # replaced Linear4bit <-> Params4bit.module cycles hold the full weights until collected
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    n_groups = 0
    if fuse:
        from quantizations_amd.integration import fuse_projection_groups
        n_groups = fuse_projection_groups(model)   # q/k/v and gate/up: one grouped GEMV launch each
    n_layer_ops = 0
    if layer_ops != "none":
        from quantizations_amd.integration import fuse_layer_ops
        n_layer_ops = fuse_layer_ops(model, norm=layer_ops in ("all", "all+decoder", "norm"),
                                     rope=layer_ops in ("all", "all+decoder", "rope"),
                                     mlp=layer_ops in ("all", "all+decoder", "mlp"),
                                     decoder=layer_ops == "all+decoder",
                                     attention=attention and layer_ops in ("all", "all+decoder"),
                                     residual=residual, mlp_pair=mlp_pair)  # one launch each
    if prenorm and fuse and layer_ops in ("all", "norm"):
        from quantizations_amd.integration import fuse_prenorm
        n_layer_ops += fuse_prenorm(model)   # RMSNorm inside the q/k/v and gate/up launches
    if glue and layer_ops != "none":
        from quantizations_amd.integration import fuse_decode_glue
        n_layer_ops += fuse_decode_glue(model)   # the step's causal mask and rotary cos/sin: one launch each
    if lm_head and layer_ops != "none":
        from quantizations_amd.integration import fuse_lm_head
        n_layer_ops += fuse_lm_head(model)   # the fp16 lm_head of a decode token: qz_gemv_dense
    return n_groups, n_layer_ops


@torch.inference_mode()
def gemv_roofline(copies: int = 64, iters: int = 400):
    """Per-launch duration of the 4096x4096 NF4+DQ fused GEMV (rotating weights)."""
    from quantizations_amd import _lib
    from quantizations_amd.core import quantize_4bit

    dev = torch.device("cuda")
    torch.manual_seed(7)
    W = (torch.randn(4096, 4096, device=dev) * 0.02).to(torch.float16)
    packed, qs = quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    sets = [(packed.clone(), qs.absmax.clone(), qs.state2.absmax.clone()) for _ in range(copies)]
    x = torch.randn(4096, device=dev).to(torch.float16)
    y = torch.empty(4096, device=dev, dtype=torch.float16)
    code2, off = qs.state2.code, qs.offset
    stream = torch.cuda.current_stream().cuda_stream
    fn = _lib.lib.qz_gemv_4bit

    from quantizations_amd import core
    # what the bench model's Linear4bit (compute_dtype fp32, the reference default) launches
    # for fp16 activations: the exact codes (core.exact_codes_for)
    prod_qt = core._gemv_quant_type("nf4", core.exact_codes_for(torch.float32), torch.float16)
    alt_qt = prod_qt ^ _lib.EXACT_CODES
    qt_flags = [prod_qt]

    def launch(i):
        p, qa, a2 = sets[i % copies]
        rc = fn(4096, 4096, x.data_ptr(), _lib.DT_F16, p.data_ptr(), qt_flags[0], 64, 0, qa.data_ptr(),
                a2.data_ptr(), code2.data_ptr(), off.data_ptr(), 256, 0, 0, 0, y.data_ptr(), stream)
        if rc:
            raise RuntimeError(f"qz_gemv_4bit rc={rc}")

    for i in range(2 * copies):
        launch(i)
    torch.cuda.synchronize()

    def blocked(fn_body):
        # Park the stream behind a ~50 ms spin kernel so the host enqueues every
        # launch (and event) before the GPU reaches them: the events then time
        # GPU execution, not Python/ctypes submission latency.
        torch.cuda._sleep(100_000_000)
        fn_body()
        torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]

    def per_launch():
        for i in range(iters):
            ev[i][0].record()
            launch(i)
            ev[i][1].record()

    blocked(per_launch)
    us = [a.elapsed_time(b) * 1e3 for a, b in ev]
    # back-to-back stream throughput (kernel + inter-kernel gap), also host-decoupled
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def b2b():
        e0.record()
        for i in range(iters):
            launch(i)
        e1.record()

    blocked(b2b)
    b2b_us = e0.elapsed_time(e1) * 1e3 / iters
    # the same launches with the other NF4 code precision (exact fp32 codes as hi + lo
    # fp16 parts <-> fp16-rounded codes)
    qt_flags[0] = alt_qt
    for i in range(copies):
        launch(i)
    blocked(b2b)
    alt_us = e0.elapsed_time(e1) * 1e3 / iters
    qt_flags[0] = prod_qt
    # one-shot read floor of the same 8.39 MB packed weight (same rotation, same timing method)
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    floor_fn = _lib.lib.qz_bench_read_floor

    def floor():
        e0.record()
        for i in range(iters):
            p = sets[i % copies][0]
            rc = floor_fn(p.data_ptr(), p.numel(), sink.data_ptr(), stream)
            if rc:
                raise RuntimeError(f"qz_bench_read_floor rc={rc}")
        e1.record()

    blocked(floor)
    floor_us = e0.elapsed_time(e1) * 1e3 / iters

    # the fixed back-to-back period of an EMPTY dependent launch (same method): the
    # part of every launch's duration that moves no bytes
    empty_fn = _lib.lib.qz_bench_empty

    def empty():
        e0.record()
        for _ in range(iters):
            rc = empty_fn(sink.data_ptr(), stream)
            if rc:
                raise RuntimeError(f"qz_bench_empty rc={rc}")
        e1.record()

    blocked(empty)
    empty_us = e0.elapsed_time(e1) * 1e3 / iters
    q = statistics.quantiles(us, n=10)
    GEMV_EXTRA["per_launch_event_us_p10"], GEMV_EXTRA["per_launch_event_us_p90"] = round(q[0], 3), round(q[-1], 3)
    GEMV_EXTRA["codes"] = "exact (fp32 as hi+lo fp16)" if prod_qt & _lib.EXACT_CODES else "fp16"
    GEMV_EXTRA["other_codes_launch_us"] = round(alt_us, 3)
    return statistics.mean(us), statistics.median(us), b2b_us, floor_us, empty_us


GEMV_EXTRA = {}


@torch.inference_mode()
def gemv_in_kernel(exact: bool, copies: int = 64, samples: int = 12, burst: int = 30):
    """In-kernel duration of the 4096x4096 NF4+DQ product GEMV: the same instantiation with
    s_memrealtime stamps (libqz_diag.so, measurement-only): first wave's start to last
    wave's end of one launch, the last of `burst` back-to-back launches on a parked stream,
    median over `samples`.  None when the diagnostic library is absent."""
    import ctypes

    from quantizations_amd.core import quantize_4bit

    path = os.path.join(REPO, "quantizations_amd", "libqz_diag.so")
    if not os.path.exists(path):
        return None
    diag = ctypes.CDLL(path)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    diag.qz_diag_set_stamp_buffer.argtypes = [vp]
    diag.qz_diag_gemv_stamped.argtypes = [i32, i32, vp, vp, i32, vp, vp, vp, vp, vp, ctypes.POINTER(i32), vp]
    dev = torch.device("cuda")
    torch.manual_seed(7)
    W = (torch.randn(4096, 4096, device=dev) * 0.02).to(torch.float16)
    packed, qs = quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    sets = [(packed.clone(), qs.absmax.clone(), qs.state2.absmax.clone()) for _ in range(copies)]
    x = torch.randn(4096, device=dev).to(torch.float16)
    y = torch.empty(4096, device=dev, dtype=torch.float16)
    stamps = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)   # up to 4096 waves x 8 u64
    if diag.qz_diag_set_stamp_buffer(stamps.data_ptr()):
        raise RuntimeError("qz_diag_set_stamp_buffer failed")
    stream = torch.cuda.current_stream().cuda_stream
    nw = i32(0)

    def launch(i):
        p, qa, a2 = sets[i % copies]
        rc = diag.qz_diag_gemv_stamped(4096, 4096, x.data_ptr(), p.data_ptr(), int(exact), qa.data_ptr(),
                                       a2.data_ptr(), qs.state2.code.data_ptr(), qs.offset.data_ptr(),
                                       y.data_ptr(), ctypes.byref(nw), stream)
        if rc:
            raise RuntimeError(f"qz_diag_gemv_stamped rc={rc}")

    for i in range(2 * copies):
        launch(i)
    torch.cuda.synchronize()
    spans = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b2b = []
    for smp in range(samples):
        torch.cuda._sleep(20_000_000)
        e0.record()
        for i in range(burst):
            launch(smp * burst + i)
        e1.record()
        torch.cuda.synchronize()
        b2b.append(e0.elapsed_time(e1) * 1e3 / burst)
        st = stamps.view(-1, 8)[:nw.value].cpu()
        t0 = int(st[:, 0].min())
        spans.append((int(st[:, 4].max()) - t0) * 0.01)          # 100 MHz ticks -> us
    return {"in_kernel_us": round(statistics.median(spans), 3),
            "in_kernel_us_min": round(min(spans), 3), "in_kernel_us_max": round(max(spans), 3),
            "stamped_launch_us_avg": round(statistics.median(b2b), 3), "waves": nw.value,
            "method": "s_memrealtime (100 MHz) at each wave's start and after its stores; max end - min start of "
                      f"one launch (the last of {burst} back-to-back), median of {samples}; stamped build of the "
                      "product instantiation (libqz_diag.so)"}


@torch.inference_mode()
def gemv_parity():
    """Decode-GEMV accuracy at the Llama-3-8B shapes (NF4 + double quant): rel err
    ||y - y_ref|| / ||y_ref|| with y_ref the fp64 product of the same x with the fp32
    dequantised weight (= the reference's fp32 weight products kernels.cu:1169;
    dequantize_4bit(fp32) is pinned bit-exact to the oracle in tests/).  Each activation
    dtype has its own code table: fp16 x the fp16-rounded codes (default) or the exact
    hi + lo codes; bf16 x bf16 hi + lo codes; fp32 x the fp32 codes.  Outputs are in x's
    dtype, so the fp16/bf16 figures include the output's own rounding (bf16: 2^-9 per
    element, above the 1e-3 bar by itself; the `_vs_bf16_rounded_ref` figure removes it)."""
    from quantizations_amd.core import dequantize_4bit, gemv_4bit, quantize_4bit

    dev = torch.device("cuda")
    res = {}
    for (M, K) in [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336)]:
        torch.manual_seed(M + K)
        W = (torch.randn(M, K, device=dev) * 0.02).half()
        packed, st = quantize_4bit(W, quant_type="nf4")
        del W
        wd = dequantize_4bit(packed, st, out_dtype=torch.float32).t().double()   # [M, K]
        x = torch.randn(K, device=dev)
        row = {}
        for name, xdt, ex in (("fp16_codes_f16", torch.float16, False), ("exact_codes_f16", torch.float16, True),
                              ("bf16_codes_bf16", torch.bfloat16, None), ("fp32_codes_f32", torch.float32, None)):
            xx = x.to(xdt)
            ref = wd @ xx.double()
            y = gemv_4bit(xx.reshape(1, K), packed, state=st, exact_codes=ex).reshape(-1).double()
            row[name] = float(f"{((y - ref).norm() / ref.norm()).item():.3e}")
            if xdt == torch.bfloat16:  # net of the bf16 output's own rounding (2^-9 per element)
                rr = ref.to(torch.bfloat16).double()
                row[name + "_vs_bf16_rounded_ref"] = float(f"{((y - rr).norm() / ref.norm()).item():.3e}")
        res[f"{M}x{K}"] = row
        del wd, packed, st
    from quantizations_amd import _lib, core
    return {"rel_err_vs_fp32_weight_products": res, "tolerance": 1e-3,
            "tolerance_by_output_dtype": {"f16": 1e-3, "f32": 1e-5,
                                          "bf16": "2^-8 = 3.9e-3 (the bf16 output's own rounding, 2^-9 per element, "
                                                  "is above 1e-3); net of it (_vs_bf16_rounded_ref) 1e-3"},
            "default": {"f16_activations": "exact_codes" if core._gemv_quant_type("nf4", None, torch.float16)
                        & _lib.EXACT_CODES else "fp16_codes",
                        "bf16_activations": "bf16 hi+lo codes", "f32_activations": "fp32 codes"}}


def gemv_alg_bytes(shapes, dq: bool = True, x_bytes: int = 2, y_bytes: int = 2) -> int:
    """Algorithmic bytes of one (grouped) NF4 decode GEMV launch:
    per segment packed M*K/2 + scales (u8 codes + fp32 absmax2/256 + offset +
    code2, or fp32 absmax) + x + y, plus the 16-entry codebook once."""
    total = 64
    for m, k in shapes:
        n = m * k
        total += n // 2 + x_bytes * k + y_bytes * m
        total += (n // 64 + 4 * (n // 64 // 256) + 4 + 1024) if dq else 4 * (n // 64)
    return total


assert gemv_alg_bytes([(4096, 4096)]) == GEMV_BYTES_4096


@torch.inference_mode()
def dominant_roofline(copies: int = 8, iters: int = 100, prenorm: bool = True, pair: bool = True):
    """The decode step's longest Linear4bit launch: the grouped gate/up GEMV of a
    Llama-3-8B layer (2 x 14336x4096 NF4+DQ in ONE launch; with `prenorm`, the
    post-attention RMSNorm inside it; with `pair`, act_fn(gate) * up in its epilogue --
    as the bench decode runs it), rotating weights (8 sets = 485 MB > the 256 MiB
    Infinity Cache), same timing method."""
    from quantizations_amd.core import gemv_4bit_grouped, gemv_4bit_pair_silu, quantize_4bit

    dev = torch.device("cuda")
    torch.manual_seed(8)
    sets = []
    for _ in range(copies):
        items = []
        for _ in range(2):
            W = (torch.randn(14336, 4096, device=dev) * 0.02).to(torch.float16)
            packed, qs = quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
            items.append((packed, qs, None))
        sets.append(items)
        del W
    x = torch.randn(1, 1, 4096, device=dev).to(torch.float16)
    nw = (1.0 + 0.1 * torch.randn(4096, device=dev)).to(torch.float16)
    outs = [torch.empty(14336, device=dev, dtype=torch.float16) for _ in range(2)]
    sets = [[(p, q, b, 0, o) for (p, q, b), o in zip(items, outs)] for items in sets]
    from quantizations_amd.core import exact_codes_for

    def timed(exact, norm, pr=pair):
        nm = (nw, 1e-5) if norm else None

        def launch(i):
            if pr:
                assert gemv_4bit_pair_silu(x, [t[:3] for t in sets[i % copies]], exact_codes=exact,
                                           norm=nm) is not None
            else:
                gemv_4bit_grouped(x, sets[i % copies], exact_codes=exact, norm=nm)
        for i in range(2 * copies):
            launch(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(100_000_000)
        e0.record()
        for i in range(iters):
            launch(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / iters

    prod = exact_codes_for(torch.float32)      # the bench model's Linear4bit (compute_dtype fp32)
    us = timed(prod, prenorm)
    other_us = timed(not prod, prenorm)
    plain_us = timed(prod, False, False) if (prenorm or pair) else us
    # + the norm weight; the pair writes one [14336] product instead of the two projections
    nbytes = gemv_alg_bytes([(14336, 4096)] * 2) + (4096 * 2 if prenorm else 0) - (14336 * 2 if pair else 0)
    return {"kernel": ("k_gemv_4bit_pair gate/up + act_fn(gate) * up" if pair else "k_gemv_4bit_grouped gate/up")
                      + " 2 x 14336x4096 NF4+DQ (one launch per layer)"
                      + (", post-attention RMSNorm in its prologue" if prenorm else "")
                      + (" (persistent workgroups, 2 per CU, 256-B-entry exact-code table)" if (prenorm and pair) else ""),
            "codes": "exact (fp32 as hi+lo fp16)" if prod else "fp16",
            "launch_us_avg": round(us, 3), "algorithmic_bytes": nbytes,
            "achieved": round(nbytes / (us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "other_codes_launch_us": round(other_us, 3), "plain_grouped_launch_us": round(plain_us, 3),
            "traffic": _pmc_traffic("r5_pair_wide_pmc.json") if (prenorm and pair)
            else _pmc_traffic("r3_gateup_pmc.json"),
            "profile": ("profiles/r5_pair_wide_pmc.json (rocprofv3 FETCH/WRITE passes of THIS launch: the "
                        "persistent pair with the norm and SiLU, exact codes on the 256-B-entry table; SQ counters "
                        "profiles/r5_pair_wide_sq_counters.txt, kernel trace r5_pair_wide_trace_stats.txt)"
                        if (prenorm and pair) else
                        "profiles/r3_gateup_pmc.json (rocprofv3 kernel trace + FETCH/WRITE passes of the grouped "
                        "launch without the norm)")}


@torch.inference_mode()
def chain_roofline(copies: int = 8, layers: int = 32, reps: int = 10, shards: int = 1, model_name: str = "llama3-8b"):
    """The Linear4bit chain of a Llama-3 decoder layer as the bench decode runs it -- q/k/v
    (+ input RMSNorm) grouped, o_proj (+ residual), gate/up + SiLU (+ post-attention RMSNorm)
    paired, down_proj (+ residual) -- four dependent launches per layer, `layers` layers on
    `copies` rotating weight sets (8B: 8 x 113 MB, 70B: 8 x 428 MB, both > the 256 MiB Infinity
    Cache) captured in ONE HIP graph: algorithmic bytes / time for the chain, i.e. the
    single-launch roofline with the dependent-launch gaps of a real decode step included (the
    attention launch between q/k/v and o_proj is left out: it is not a Linear4bit; o_proj reads the
    q output in its place, so every launch still depends on the previous one).  Where the product
    takes another form (Llama-3-70B: gate/up at K = 8192 splits rows over two waves, so the split
    pair runs after a separate norm launch), the chain runs what the product runs; `gate_up_form` and
    `launches_per_layer` say which.  shards = P > 1: the same chain on ONE rank's
    rows of the row-split layout (every projection M / P rows, the launches a rank runs per layer
    at N = P; the exchanges are timed separately), for the N-GPU budget in DESIGN.md section 6."""
    from quantizations_amd.core import LAST_FORM, gemv_4bit, gemv_4bit_grouped, gemv_4bit_pair_silu, quantize_4bit
    from quantizations_amd.layer_ops import silu_mul

    base_cfg = MODELS[model_name]
    H, I = base_cfg["hidden_size"], base_cfg["intermediate_size"]
    KV = base_cfg["num_key_value_heads"] * (H // base_cfg["num_attention_heads"])
    shapes = {"q": (H, H), "k": (KV, H), "v": (KV, H), "o": (H, H), "gate": (I, H), "up": (I, H), "down": (H, I)}
    dev = torch.device("cuda")
    torch.manual_seed(11)
    base = {}
    for name, (M, K) in shapes.items():
        M //= shards
        W = (torch.randn(M, K, device=dev) * 0.02).to(torch.float16)
        base[name] = quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        del W

    def clone(pk, qs):
        st = type(qs)(absmax=qs.absmax.clone(), shape=qs.shape, code=qs.code, blocksize=qs.blocksize,
                      quant_type=qs.quant_type, dtype=qs.dtype, offset=qs.offset.clone(),
                      state2=type(qs.state2)(absmax=qs.state2.absmax.clone(), code=qs.state2.code,
                                             blocksize=qs.state2.blocksize, dtype=qs.state2.dtype))
        return pk.clone(), st
    sets = [{n: clone(*base[n]) for n in base} for _ in range(copies)]
    del base
    Hs, Is, KVs = H // shards, I // shards, KV // shards    # this rank's rows
    nw1 = (1.0 + 0.1 * torch.randn(H, device=dev)).half()
    nw2 = (1.0 + 0.1 * torch.randn(H, device=dev)).half()
    x0 = torch.randn(1, 1, H, device=dev).half()
    qkv_out = [torch.empty(Hs, device=dev, dtype=torch.float16), torch.empty(KVs, device=dev, dtype=torch.float16),
               torch.empty(KVs, device=dev, dtype=torch.float16)]
    gu_out = [torch.empty(Is, device=dev, dtype=torch.float16), torch.empty(Is, device=dev, dtype=torch.float16)]
    # stand-ins for the exchanged full vectors a rank's next launch reads (row-split: every launch
    # consumes the all-gathered [H] / [I] vector; P = 1: the previous output itself)
    full_h = torch.randn(1, 1, I, device=dev).half()
    forms = set()
    launches = []   # per layer, as the forms ran (a norm launch counts)

    def layer(x, w):
        q, _, _ = gemv_4bit_grouped(x, [(*w["q"], None, 0, qkv_out[0]), (*w["k"], None, 0, qkv_out[1]),
                                        (*w["v"], None, 0, qkv_out[2])], exact_codes=True, norm=(nw1, 1e-5))
        n = 2 if LAST_FORM.get("grouped", "").startswith("norm launch") else 1
        forms.add("q/k/v " + LAST_FORM.get("grouped", "?"))
        xo = q.view(1, 1, H) if shards == 1 else x          # o_proj reads the (gathered) attention output
        a = gemv_4bit(xo, w["o"][0], state=w["o"][1], exact_codes=True, residual=x.view(-1)[:Hs])
        xa = a if shards == 1 else x                        # ... the gathered residual stream
        h = gemv_4bit_pair_silu(xa, [(*w["gate"], None), (*w["up"], None)], exact_codes=True, norm=(nw2, 1e-5))
        if h is None:   # what the product runs where the pair launch refuses (fuse_layer_ops' MLP forward)
            g_, u_ = gemv_4bit_grouped(xa, [(*w["gate"], None, 0, gu_out[0]), (*w["up"], None, 0, gu_out[1])],
                                       exact_codes=True, norm=(nw2, 1e-5))
            h = silu_mul(g_, u_)
            forms.add("gate/up " + LAST_FORM.get("grouped", "?") + " + silu_mul")
            n += 3 if LAST_FORM.get("grouped", "").startswith("norm launch") else 2
        else:
            forms.add("gate/up " + LAST_FORM.get("pair", "?"))
            n += 2 if LAST_FORM.get("pair", "").startswith("norm launch") else 1
        launches.append(n + 2)   # + o_proj, down_proj
        xh = h if shards == 1 else full_h                   # ... the gathered h
        y = gemv_4bit(xh, w["down"][0], state=w["down"][1], exact_codes=True, residual=a.view(-1)[:Hs])
        return y if shards == 1 else x

    def chain():
        x = x0
        for i in range(layers):
            x = layer(x, sets[i % copies])
        return x
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        chain()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3 / layers)
    us = statistics.median(times)
    # algorithmic bytes per layer: the four launches' GEMV bytes, + the two norm
    # weights and the two residual reads, - the pair's second output (it writes h only)
    nbytes = (gemv_alg_bytes([(Hs, H), (KVs, H), (KVs, H)]) - 2 * (2 * H)   # q/k/v: x read once, not 3 x
              + gemv_alg_bytes([(Hs, H)]) + 2 * Hs                              # o_proj + its residual read
              + gemv_alg_bytes([(Is, H)] * 2) - 2 * H - 2 * Is                  # pair: x once, one output
              + gemv_alg_bytes([(Hs, I)]) + 2 * Hs                              # down_proj + its residual read
              + 2 * (2 * H))                                                    # the two RMSNorm weights
    del sets, g
    torch.cuda.empty_cache()
    ach = nbytes / (us * 1e-6) / 1e9
    name = "Llama-3-70B" if model_name == "llama3-70b" else "Llama-3-8B"
    return {"what": f"one {name} layer's Linear4bit chain: q/k/v+norm grouped, o_proj+residual, gate/up+SiLU+norm, "
                    "down_proj+residual, NF4+DQ exact codes, one HIP graph of "
                    f"{layers} layers over {copies} rotating weight sets"
                    + (f"; ONE rank's rows of the {shards}-way row split (exchanges not included)" if shards > 1 else ""),
            "model": model_name, "shards": shards, "gate_up_form": sorted(forms),
            "launches_per_layer": max(launches) if launches else None,
            "us_per_layer": round(us, 3), "algorithmic_bytes_per_layer": nbytes,
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "us_per_layer_min": round(min(times), 3), "us_per_layer_max": round(max(times), 3)}


def _safe(fn, *a, **k):
    """fn(*a, **k), or {"error": ...} if it raises: a rank-0 extra measurement never costs the
    headline line (and never leaves the other ranks waiting in a later collective)."""
    try:
        return fn(*a, **k)
    except Exception as e:  # noqa: BLE001 -- reported in the line
        log(f"bench: {getattr(fn, '__name__', fn)} failed: {type(e).__name__}: {e}")
        try:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        except Exception:  # noqa: BLE001
            pass
        return {"error": f"{type(e).__name__}: {e}"}


def effective_knobs() -> dict:
    """The measurement knobs in effect: the C launchers' (read once at library load,
    qz_gemv_knobs) and the Python routing switches (read at import of quantizations_amd.core),
    with every QZ_* variable set in this process's environment."""
    from quantizations_amd import _lib, core
    return {"gemv_launchers": _lib.gemv_knobs(),
            "routing": {"GEMV_EXACT_CODES": core.GEMV_EXACT_CODES, "PREFILL_GEMM16": core.PREFILL_GEMM16,
                        "GEMM16_MIN_TILES": core.GEMM16_MIN_TILES,
                        "PREFILL_FUSED_MAX_T": core._FUSED_MAX_T_ENV},
            "env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("QZ_")}}


def _pmc_traffic(name: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary under profiles/."""
    path = os.path.join(REPO, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


@torch.inference_mode()
def rowsplit_layer(rank: int, world: int, sharded: bool, M: int = 8192, K: int = 28672, calls: int = 20,
                   reps: int = 5, gatherer=None):
    """one Llama-3-70B-shaped Linear4bit (M x K NF4+DQ, bs = 1) row-split over
    the job's ranks -- each rank's GEMV on M/P rows (slices of the ONE global quant state)
    + the RCCL all-gather of the fp16 shards -- vs the same layer's unsharded GEMV on one
    GPU.  `calls` forward calls are captured into one HIP graph and replayed `reps` times;
    per-call microseconds = the slowest rank's replay time / calls (barrier + sync around)."""
    import quantizations_amd as qa
    from quantizations_amd.parallel import RowShardedLinear4bit

    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(88)
    W = (torch.randn(M, K, device=dev, generator=g) * 0.02).half()
    full = qa.Linear4bit(K, M, bias=False, quant_type="nf4", compress_statistics=True)
    full.weight = qa.Params4bit(W, requires_grad=False, quant_type="nf4", module=full, compress_statistics=True)
    del W
    full = full.to(dev)
    x = torch.randn(1, 1, K, device=dev, generator=g).half()

    def timed(fn):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg, capture_error_mode=CAPTURE_MODE):
            for _ in range(calls):
                fn()
        cg.replay()
        best = None
        for _ in range(reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cg.replay()
            torch.cuda.synchronize()
            dt = torch.tensor([time.perf_counter() - t0], device=dev)
            if world > 1:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            best = dt.item() if best is None else min(best, dt.item())
        return round(best / calls * 1e6, 2)

    out = {"layer": f"{M}x{K} NF4+DQ (Llama-3-70B down_proj shape), bs=1", "ranks": world,
           "unsharded_us": timed(lambda: full(x))}
    if sharded:
        try:
            shard = RowShardedLinear4bit(full, rank, world)
            out["rows_per_rank"] = shard.r1 - shard.r0
            out["local_gemv_us"] = timed(lambda: shard.local_forward(x))
            out["rowsplit_allgather_us"] = timed(lambda: shard(x))
            if gatherer is not None:   # the same layer through the one-shot exchange
                shard.gatherer = gatherer
                out["rowsplit_oneshot_us"] = timed(lambda: shard(x))
                got1 = shard(x).reshape(-1)
                shard.gatherer = None
                out["oneshot_equals_rccl"] = bool(torch.equal(got1, shard(x).reshape(-1)))
            ref, got = full(x).reshape(-1), shard(x).reshape(-1)
            # same products; a shard's GEMV may split K differently (fp32 summation order)
            out["bit_identical_to_unsharded"] = bool(torch.equal(got, ref))
            out["max_abs_diff_vs_unsharded"] = float((got.float() - ref.float()).abs().max())
        except Exception as e:  # reported, never fatal to the headline line
            out["error"] = f"{type(e).__name__}: {e}"
    return out


@torch.inference_mode()
def prefill_bench(T: int = 16384, iters: int = 10):
    """config #4: one prefill pass of 8 x 2048 tokens through the Llama-3-8B
    Linear4bit shapes: fused dequant+MFMA GEMM vs the reference route
    (dequantize_4bit to fp16, then a library fp16 GEMM)."""
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, quantize_4bit

    dev = torch.device("cuda")
    out = {}
    torch.manual_seed(11)
    X = torch.randn(T, 14336, device=dev, dtype=torch.float16)
    for (M, K) in [(4096, 4096), (14336, 4096), (4096, 14336)]:
        W = (torch.randn(M, K, device=dev) * 0.02).to(torch.float16)
        packed, qs = quantize_4bit(W, quant_type="nf4")
        x = X[:, :K]
        if not x.is_contiguous():
            x = x.contiguous()

        def fused():
            return gemm_4bit(x, packed, qs, route="fused")

        def own_route():
            return gemm_4bit(x, packed, qs, route="gemm16")

        def ref_route():
            return torch.nn.functional.linear(x, dequantize_4bit(packed, qs).t())

        res = {}
        for name, fn in (("fused", fused), ("dequant+gemm16", own_route), ("dequant+hipblaslt", ref_route)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            res[name] = {"ms": round(ms, 3), "TFLOP/s": round(2.0 * T * M * K / (ms * 1e-3) / 1e12, 1)}
        out[f"{M}x{K}"] = res
        del W, packed, qs
    from quantizations_amd.core import GEMM16_MIN_TILES, PREFILL_GEMM16, fused_max_tokens
    return {"tokens": T, "shapes": out, "mfma_peak_TFLOPs_f16_dense": 2500.0,
            "product_route": "fused" if T <= fused_max_tokens(4096) else
                             ("dequant+gemm16" if PREFILL_GEMM16 else "dequant+hipblaslt"),
            "note": "every route multiplies the same bit-exact dequantised weight; matmul_4bit takes the fused "
                    f"MFMA kernels up to {fused_max_tokens(4096)} tokens ({fused_max_tokens(1024)} for 1024 or "
                    f"14336 rows), above it our dequant kernel + hipBLASLt "
                    "(the reference's F.linear route) unless QZ_PREFILL_GEMM16=1 selects our 4-wave LDS-DMA MFMA GEMM "
                    f"(qz_gemm_16bit: the persistent k_gemm16_4q, >= {GEMM16_MIN_TILES} 256x256 tiles)"}


@torch.inference_mode()
def prefill_sweep(Ts=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 16384), iters=20):
    """4096x4096 NF4: fused MFMA GEMM vs dequant + library GEMM over token count T."""
    from quantizations_amd.core import dequantize_4bit, gemm_4bit, quantize_4bit

    dev = torch.device("cuda")
    torch.manual_seed(12)
    M = K = 4096
    W = (torch.randn(M, K, device=dev) * 0.02).to(torch.float16)
    packed, qs = quantize_4bit(W, quant_type="nf4")
    res = {}
    for T in Ts:
        x = torch.randn(T, K, device=dev, dtype=torch.float16)

        def fused():
            return gemm_4bit(x, packed, qs, route="fused")

        def own_route():
            return gemm_4bit(x, packed, qs, route="gemm16")

        def ref_route():
            return torch.nn.functional.linear(x, dequantize_4bit(packed, qs).t())

        row = {}
        for name, fn in (("fused", fused), ("dequant+gemm16", own_route), ("dequant+blas", ref_route)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(50_000_000)  # host enqueues every launch before the GPU reaches them
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            row[name] = round(e0.elapsed_time(e1) / iters * 1e3, 2)
        res[T] = row
    return {"shape": "4096x4096 nf4 dq", "us": res}


def _cpu_model() -> str:
    """`lscpu` model name of the host (falls back to /proc/cpuinfo)."""
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(runs: int = 20, warmups: int = 3):
    """config #1 on the host cores -- Linear4bit(4096,4096)
    NF4 + double quant, W ~ N(0, 0.02^2) fp16 (seed 0), x ~ N(0,1) fp16 (seed 1);
    the oracle's CPU restatement (absmax double-dequant + LUT dequant to fp32,
    then torch.matmul in fp32; the reference has no CPU path).  Median of
    `runs` after `warmups`, for dequant+matmul and for the matmul alone."""
    import numpy as np

    import oracle

    # the GPU box exposes the whole machine's CPUs; its share is OMP_NUM_THREADS (16)
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    W = (torch.randn(4096, 4096, generator=torch.Generator().manual_seed(0)) * 0.02).to(torch.float16)
    x16 = torch.randn(1, 1, 4096, generator=torch.Generator().manual_seed(1)).to(torch.float16)
    x = x16.float().numpy().reshape(-1)
    st = oracle.quantize_4bit(W.float().numpy(), 64, "nf4", double_quant=True)

    def timed(fn):
        for _ in range(warmups):
            fn()
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    full_s = timed(lambda: oracle.cpu_dequant_matmul(x, st))
    Wf = oracle.cpu_dequant(st)
    xt = torch.from_numpy(x).reshape(1, 4096)
    mm_s = timed(lambda: xt @ Wf.t())
    elems_per_token = LLAMA3_8B["num_hidden_layers"] * sum(m * k for m, k in LAYER_SHAPES)
    tok_s = 1.0 / (full_s * elems_per_token / (4096 * 4096))
    del np
    return {"value": round(tok_s, 5), "unit": "tokens/s", "cores": cores, "kind": "port",
            "cpu_model": _cpu_model(),
            "dequant_matmul_ms": round(full_s * 1e3, 3), "matmul_alone_ms": round(mm_s * 1e3, 3),
            "runs": runs, "warmups": warmups,
            "sample": f"config #1: Linear4bit(4096,4096) NF4+DQ, CPU dequant + torch.matmul fp32 (oracle "
                      f"restatement of kernels.cu/core.py), median of {runs} runs after {warmups} warm-ups = "
                      f"{full_s * 1e3:.1f} ms per layer ({mm_s * 1e3:.2f} ms of it the matmul alone); value = "
                      f"that layer time scaled by weight count to the 224 Linear4bit layers of one Llama-3-8B "
                      f"token (extrapolated, not a decode run)"}


def roofline_object(args, layer_ops: str) -> dict:
    """The line's `roofline` object: the 4096x4096 decode GEMV's launch period (gemv_roofline), its
    in-kernel duration, the dominant launch of the decode step and the one-launch ceiling."""
    mean_us, med_us, b2b_us, floor_us, empty_us = gemv_roofline()
    # average launch duration = HIP events around `iters` back-to-back launches on
    # the launch stream / iters; a per-launch event pair adds ~2.3 us of event
    # overhead on ROCm and disagrees with rocprofv3, so it is reported only.
    ach = GEMV_BYTES_4096 / (b2b_us * 1e-6) / 1e9
    traffic = _pmc_traffic("gemv_4096_pmc.json")
    roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "k_gemv_4bit<Tab,DQ,f16,R=2,WK=1,full-step,CL=%d> 4096x4096 NF4+DQ (LDS byte-table decode, "
                      "%s codes)" % (int(GEMV_EXTRA.get("codes", "").startswith("exact")), GEMV_EXTRA.get("codes")),
            "launch_us_avg": round(b2b_us, 3),
            "per_launch_event_us_mean": round(mean_us, 3), "per_launch_event_us_median": round(med_us, 3),
            "per_launch_event_us_p10": GEMV_EXTRA.get("per_launch_event_us_p10"),
            "per_launch_event_us_p90": GEMV_EXTRA.get("per_launch_event_us_p90"),
            "one_shot_read_floor_us": round(floor_us, 3),
            "frac_of_one_shot_floor": round(floor_us / b2b_us, 4),
            # what one launch can reach at all: an empty dependent launch's period
            # plus the 8.67 MB at peak bandwidth
            "empty_launch_us": round(empty_us, 3),
            "frac_ceiling_one_launch": round(GEMV_BYTES_4096 / ((empty_us + GEMV_BYTES_4096 / (HBM_PEAK_GBS * 1e3))
                                                                * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "codes": GEMV_EXTRA.get("codes"), "other_codes_launch_us": GEMV_EXTRA.get("other_codes_launch_us"),
            "dominant_decode_kernel": _safe(dominant_roofline,
                prenorm=bool(not args.no_prenorm and not args.no_fuse
                             and layer_ops in ("all", "norm")),
                pair=bool(not args.no_mlp_pair and not args.no_fuse and layer_ops in ("all", "all+decoder", "mlp")))}
    from quantizations_amd import _lib, core
    ink = _safe(gemv_in_kernel, bool(core._gemv_quant_type("nf4", core.exact_codes_for(torch.float32),
                                                           torch.float16) & _lib.EXACT_CODES))
    if ink is not None and "error" in ink:
        roof["in_kernel"] = ink
    elif ink is not None:
        # the kernel's own duration (stamps): what the launch period adds on top is dispatch
        roof["in_kernel"] = ink
        roof["in_kernel_us"] = ink["in_kernel_us"]
        roof["frac_in_kernel"] = round(GEMV_BYTES_4096 / (ink["in_kernel_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    return roof


def codes_desc(args, compute_dtype) -> str:
    """The decode GEMV's code table for the bench model (core._gemv_quant_type)."""
    if args.dtype == "bf16":
        return "codes as bf16 hi+lo"
    if args.quant == "fp4":
        return "FP4 codes, exact"
    from quantizations_amd import _lib, core
    exact = core._gemv_quant_type("nf4", core.exact_codes_for(compute_dtype), torch.float16) & _lib.EXACT_CODES
    return "exact NF4 codes (fp32 as hi+lo fp16)" if exact else "fp16-rounded NF4 codes"


def decode_layout(args, world: int, sharded: bool):
    """(weak, tp_mode, global batch).  Strong scaling (default): ONE global batch (bs=1)
    for any N, every Linear4bit row-split over all N GPUs + all-gather.  --weak: every
    GPU adds one bs=1 stream (global batch batch x N) and the layers are TP-paired."""
    weak = args.weak and sharded
    tp_mode = args.tp_mode or ("pair" if weak else "gather")
    return weak, tp_mode, (args.batch * world if weak else args.batch)


def parallelism_name(tp_mode: str, world: int, sharded: bool) -> str:
    if not sharded:
        return "single"
    return f"tp{world}-megatron-pair-allreduce" if tp_mode == "pair" else f"tp{world}-rowsplit-allgather"


def setup_oneshot(rank: int):
    """The one-shot IPC all-gather for the row-split layers, verified against RCCL on live
    data; (None, "rccl (...)") when it cannot be set up or disagrees."""
    try:
        from quantizations_amd.exchange import OneShotAllGather
        g = OneShotAllGather(slot_bytes=1 << 18)
        if not g.verify():
            log(f"[rank {rank}] one-shot all-gather disagrees with RCCL: using RCCL")
            g.close()
            return None, "rccl (one-shot failed verification)"
        # the process's first captured graph is the slow one (exchange.warm_graph); its success is
        # voted over every rank, so either all ranks keep the gatherer or all fall back together
        if not g.warm_graph():
            log(f"[rank {rank}] one-shot all-gather failed its warm-up graph on some rank: using RCCL")
            g.close()
            return None, "rccl (one-shot failed its warm-up graph)"
        return g, "oneshot-ipc"
    except Exception as e:  # reported in the line, never fatal to the measurement
        log(f"[rank {rank}] one-shot all-gather unavailable ({type(e).__name__}: {e}): using RCCL")
        return None, f"rccl (one-shot unavailable: {type(e).__name__})"


def launch_ranks(n: int, port: int = 0) -> int:
    """Start `n` ranks of this same command line through torch.distributed.run (one
    process per GPU, rendezvous on 127.0.0.1) and return the launcher's exit status.
    Called before any GPU work in this process."""
    import socket
    import subprocess

    if not port:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this driver
    log(f"bench: starting {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def selftest_main(args, rank: int, world: int):
    """CPU rehearsal of the N-rank entry point (tests/test_bench_entry.py): gloo instead
    of RCCL, the tiny Linear4bit Llama and the shard-local product of the TEST module
    named by --selftest (the product's local product is the HIP GEMV), and bench's own
    layout (prepare_decode_model) and decode loop (decode_bench_graph, eager on CPU).
    Prints the headline line's layout keys plus whether the greedy tokens equal the
    unsharded reference model's; exits non-zero when they do not."""
    import importlib

    hook = importlib.import_module(args.selftest)
    dist.init_process_group("gloo")
    if dist.get_world_size() != args.gpus:
        log(f"error: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
        sys.exit(2)
    sharded = world > 1 or args.force_shard
    weak, tp_mode, gbatch = decode_layout(args, world, sharded)
    cfg, model, ref = hook.tiny_model()
    n_groups, _ = prepare_decode_model(model, rank, world, sharded, tp_mode, fuse=not args.no_fuse,
                                       layer_ops="none", local_matmul=hook.local_matmul)
    dt, hist = decode_bench_graph(model, cfg, args.steps, args.warmup, args.prompt, world, gbatch,
                                  graph=False, device="cpu")
    _, ref_hist = decode_bench_graph(ref, cfg, args.steps, args.warmup, args.prompt, 1, gbatch,
                                     graph=False, device="cpu")
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    same = torch.tensor([int(torch.equal(hist, ref_hist))])
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(json.dumps({"metric": "selftest decode tokens/sec (tiny Llama, CPU, gloo)",
                          "value": round(args.steps * gbatch / float(t.item()), 3), "unit": "tokens/s",
                          "n_gpus": dist.get_world_size(), "steps": args.steps, "warmup": args.warmup,
                          "scaling": "weak" if weak else "strong",
                          "config": {"workload": "selftest-tiny-llama", "global_batch": gbatch,
                                     "parallelism": parallelism_name(tp_mode, world, sharded),
                                     "projection_groups": n_groups},
                          "selftest": {"tokens_equal_unsharded": bool(same.item())}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if not same.item():
        sys.exit(3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=32)
    ap.add_argument("--layers", type=int, default=0, help="decoder layers (0 = the model's own count)")
    ap.add_argument("--model", choices=sorted(MODELS), default="llama3-8b",
                    help="llama3-8b (configs #1-#4) or llama3-70b (config #5)")
    ap.add_argument("--quant", choices=("nf4", "fp4"), default="nf4", help="codebook (config #3: fp4 --no-dq)")
    ap.add_argument("--no-dq", action="store_true", help="fp32 absmax instead of double quant")
    ap.add_argument("--dtype", choices=("fp16", "bf16"), default="fp16",
                    help="model / activation dtype (bf16: SURVEY 8(f) row 4, the bf16 activation path)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the decode step")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--gemv-only", action="store_true", help="only the 4096x4096 roofline microbench (profiling)")
    ap.add_argument("--prefill-only", action="store_true", help="only the config #4 prefill GEMM measurement")
    ap.add_argument("--chain-only", action="store_true",
                    help="only the Linear4bit chain of one decoder layer (chain_roofline; profiling)")
    ap.add_argument("--chain-shards", type=int, default=1,
                    help="--chain-only: the chain on one rank's rows of a P-way row split")
    ap.add_argument("--dominant-only", action="store_true",
                    help="only the grouped gate/up GEMV measurement (the decode step's longest launch; profiling)")
    ap.add_argument("--no-prefill", action="store_true")
    ap.add_argument("--no-fuse", action="store_true", help="one GEMV launch per Linear4bit (no q/k/v, gate/up groups)")
    ap.add_argument("--no-layer-ops", action="store_true",
                    help="keep transformers' eager RMSNorm / rotary (8 and 10 launches) instead of layer_ops")
    ap.add_argument("--no-prenorm", action="store_true",
                    help="keep each RMSNorm as its own launch (default: absorbed into the q/k/v and gate/up "
                         "grouped GEMV launches on one GPU)")
    ap.add_argument("--no-attention", action="store_true",
                    help="keep transformers' rotary + StaticCache update + sdpa (14 launches per layer) instead of "
                         "the one-launch layer_ops.decode_attention")
    ap.add_argument("--greedy", choices=("kernel", "two-stage", "torch"), default="kernel",
                    help="the decode step's greedy pick: one launch with the token feedback (layer_ops.greedy_step), "
                         "greedy_token's two stages, or torch.argmax (the last two + index_copy/copy/add)")
    ap.add_argument("--torch-argmax", action="store_true",
                    help="the decode step's greedy pick as torch's one-pass argmax (default: greedy_token's two "
                         "stages, the same index)")
    ap.add_argument("--no-mlp-pair", action="store_true",
                    help="gate/up as the grouped launch + a separate SiLU-product launch (default: one launch)")
    ap.add_argument("--lm-head-library", action="store_true",
                    help="keep the fp16 lm_head on F.linear (hipBLASLt) instead of layer_ops.gemv_dense (its "
                         "rows stay split over the ranks; --no-shard-lm-head replicates it)")
    ap.add_argument("--replicated-attention", action="store_true",
                    help="N > 1 row-split layout: gather q/k/v and run every head's attention on every rank "
                         "(default: head-sharded -- each rank's q/k/v rows are whole heads, attended locally, "
                         "and the attention output is gathered before o_proj)")
    ap.add_argument("--no-shard-lm-head", action="store_true",
                    help="N > 1 row-split layout: keep the whole fp16 lm_head on every rank (default: each rank "
                         "its 1/N of the rows, gathered like the Linear4bit outputs)")
    ap.add_argument("--no-glue", action="store_true",
                    help="keep transformers' own causal-mask and rotary code in the decode step (default: one "
                         "launch each, integration.fuse_decode_glue; same values)")
    ap.add_argument("--no-residual", action="store_true",
                    help="keep each decoder layer's two residual adds as their own launches (default: in the "
                         "o_proj / down_proj GEMV epilogues)")
    ap.add_argument("--layer-ops", choices=("all", "all+decoder", "norm", "rope", "mlp", "none"), default="all",
                    help="which transformers ops integration.fuse_layer_ops replaces")
    ap.add_argument("--capture-mode", choices=("global", "thread_local", "relaxed"), default="thread_local",
                    help="torch.cuda.graph capture_error_mode of the decode-step capture")
    ap.add_argument("--prefill-sweep", action="store_true", help="fused vs dequant+hipBLASLt over T (4096x4096)")
    ap.add_argument("--tp-mode", choices=("pair", "gather"), default=None,
                    help="multi-GPU layout: row-split every Linear4bit + all-gather (default; the north-star "
                         "layout) or Megatron pairing (column q/k/v/gate/up + row o/down, 2 all-reduces per "
                         "layer; the --weak default)")
    ap.add_argument("--force-shard", action="store_true",
                    help="run the multi-GPU code path (process group, sharded layers, RCCL) even at world size 1")
    ap.add_argument("--batch", type=int, default=1,
                    help="decode streams (bs=1 each); with --weak the global batch is batch x N")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: weak scaling -- one bs=1 stream per GPU (global batch = batch x N), Megatron "
                         "pairing unless --tp-mode says otherwise")
    ap.add_argument("--strong", action="store_true", help="(default) N > 1: the global batch stays --batch")
    ap.add_argument("--no-extra-weak", action="store_true",
                    help="N > 1: skip the extra weak-scaling (TP-pair, global batch N) measurement")
    ap.add_argument("--allgather", choices=("oneshot", "rccl"), default="oneshot",
                    help="row-split exchange: one-shot IPC all-gather (exchange.OneShotAllGather; verified "
                         "against RCCL at setup, RCCL on any failure) or RCCL all_gather_into_tensor")
    ap.add_argument("--compute-dtype", choices=("fp32", "fp16"), default="fp32",
                    help="Linear4bit compute_dtype: fp32 = the reference default (fp16 x decoded against the "
                         "exact fp32 codes); fp16 = the fp16-rounded code table")
    ap.add_argument("--no-extra-codes", action="store_true",
                    help="N = 1: skip the second decode measurement with the other code table")
    ap.add_argument("--selftest", default=None, help=argparse.SUPPRESS)  # CPU test hook module (tests/)
    ap.add_argument("--master-port", type=int, default=0,
                    help="rendezvous port when bench.py starts the N ranks itself (0 = a free port)")
    args = ap.parse_args()
    global CAPTURE_MODE
    CAPTURE_MODE = args.capture_mode
    if args.weak and args.strong:
        ap.error("--weak and --strong are exclusive")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks here, before
        # anything touches the GPU, one child process per GPU (torch.distributed.run
        # sets RANK / LOCAL_RANK / WORLD_SIZE), and exit with the launcher's status.
        sys.exit(launch_ranks(args.gpus, args.master_port))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report a {world}-rank run "
            f"as {args.gpus} GPUs")
        sys.exit(2)
    if args.selftest:
        return selftest_main(args, rank, world)
    torch.cuda.set_device(local)
    sharded = world > 1 or args.force_shard
    if sharded:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            log(f"error: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
            sys.exit(2)
    gatherer, exchange = None, ("rccl" if sharded else None)
    if sharded and args.allgather == "oneshot":
        gatherer, exchange = setup_oneshot(rank)

    if args.gemv_only:
        mean_us, med_us, b2b_us, floor_us, empty_us = gemv_roofline()
        print(json.dumps({"gemv_4096_us_mean": mean_us, "gemv_4096_us_median": med_us, "back_to_back_us": b2b_us,
                          "read_floor_us": floor_us, "empty_launch_us": empty_us, **GEMV_EXTRA,
                          "achieved_GBs": GEMV_BYTES_4096 / (b2b_us * 1e-6) / 1e9}), flush=True)
        return

    if args.dominant_only:
        print(json.dumps(dominant_roofline()), flush=True)
        return
    if args.chain_only:
        print(json.dumps(chain_roofline(shards=args.chain_shards, model_name=args.model)), flush=True)
        return
    if args.prefill_only:
        print(json.dumps(prefill_bench()), flush=True)
        return
    if args.prefill_sweep:
        print(json.dumps(prefill_sweep()), flush=True)
        return

    layer_ops = "none" if args.no_layer_ops else args.layer_ops

    compute_dtype = torch.float32 if args.compute_dtype == "fp32" else torch.float16
    global GREEDY
    GREEDY = "torch" if args.torch_argmax else args.greedy

    def run_decode(tp_mode: str, gbatch: int, steps: int, warmup: int, cdt: torch.dtype = compute_dtype):
        t_build = time.perf_counter()
        model, cfg = build_model(args.layers, seed=0, model_name=args.model, quant_type=args.quant,
                                 double_quant=not args.no_dq,
                                 dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float16,
                                 compute_dtype=cdt)
        n_groups, n_layer_ops = prepare_decode_model(model, rank, world, sharded, tp_mode, fuse=not args.no_fuse,
                                                     layer_ops=layer_ops, gatherer=gatherer,
                                                     prenorm=not args.no_prenorm,
                                                     attention=not args.no_attention,
                                                     residual=not args.no_residual,
                                                     mlp_pair=not args.no_mlp_pair,
                                                     glue=not args.no_glue,
                                                     lm_head=not args.lm_head_library,
                                                     shard_head=not args.no_shard_lm_head,
                                                     head_sharded_attention=not args.replicated_attention)
        log(f"[rank {rank}] model ready in {time.perf_counter() - t_build:.1f}s, "
            f"{torch.cuda.memory_allocated() / 2**30:.2f} GiB ({tp_mode if sharded else 'single'}, batch {gbatch})")
        mode = "eager"
        if not args.eager:
            try:
                dt, _ = decode_bench_graph(model, cfg, steps, warmup, args.prompt, world, gbatch)
                mode = "hipgraph"
            except Exception as e:  # capture unsupported by this transformers build -> eager
                log(f"[rank {rank}] graph decode failed ({type(e).__name__}: {e}); falling back to eager")
                torch.cuda.synchronize()
        if mode == "eager":
            dt, _ = decode_bench(model, cfg, steps, warmup, args.prompt, world, gbatch)
        t = torch.tensor([dt], device="cuda")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)   # the slowest rank's time
        del model
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        return float(t.item()), mode, cfg, n_groups, n_layer_ops

    def parallelism(tp_mode: str) -> str:
        return parallelism_name(tp_mode, world, sharded)

    weak, tp_mode, gbatch = decode_layout(args, world, sharded)
    dt, mode, cfg, n_groups, n_layer_ops = run_decode(tp_mode, gbatch, args.steps, args.warmup)
    tok_s = args.steps * gbatch / dt   # tokens generated by all streams, whole job

    extra_weak = None
    if world > 1 and not weak and not args.no_extra_weak:
        # the weak-scaling layout, reported beside the headline only (extra key)
        w_steps = max(8, args.steps // 2)
        wdt, wmode, _, _, _ = run_decode("pair", args.batch * world, w_steps, args.warmup)
        extra_weak = {"value": round(w_steps * args.batch * world / wdt, 3), "unit": "tokens/s",
                      "ms_per_step": round(wdt / w_steps * 1e3, 4), "steps": w_steps, "scaling": "weak",
                      "global_batch": args.batch * world, "decode": wmode, "parallelism": parallelism("pair")}

    extra_codes = None
    if world == 1 and not sharded and not args.no_extra_codes and args.dtype == "fp16" and args.quant == "nf4":
        # the same decode with the other fp16-activation code table (reported beside the headline)
        other = torch.float16 if compute_dtype == torch.float32 else torch.float32
        c_steps = max(16, args.steps // 2)
        cdt_, cmode, _, _, _ = run_decode(tp_mode, gbatch, c_steps, args.warmup, cdt=other)
        extra_codes = {"value": round(c_steps * gbatch / cdt_, 3), "unit": "tokens/s",
                       "ms_per_step": round(cdt_ / c_steps * 1e3, 4), "steps": c_steps, "decode": cmode,
                       "compute_dtype": "fp32" if other == torch.float32 else "fp16",
                       "codes": "exact NF4 codes (fp32 as hi+lo fp16)" if other == torch.float32
                       else "fp16-rounded NF4 codes"}

    roof = None
    parity = None
    chain = None
    if rank == 0 and not args.no_roofline:
        roof = _safe(roofline_object, args, layer_ops)
        parity = _safe(gemv_parity)
        chain = _safe(chain_roofline)

    layer = None
    if not args.no_roofline:
        layer = rowsplit_layer(rank, world, sharded, gatherer=gatherer)   # every rank takes part (the all-gather)
    if gatherer is not None and gatherer.failed_anywhere():
        # a one-shot exchange gave up waiting for a peer (5 s bound): its outputs, and so the
        # measured decode, are not valid -- no line is reported (every rank takes this branch)
        log(f"[rank {rank}] error: a one-shot all-gather timed out on some rank; the measurement is invalid")
        dist.barrier()
        dist.destroy_process_group()
        sys.exit(4)

    prefill = None
    if rank == 0 and world == 1 and not args.no_prefill:
        prefill = prefill_bench()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline()

    if rank == 0:
        line = {
            # BASELINE.json's metric for the headline model; other configs name their own model/codebook
            "metric": ("decode tokens/sec Llama-3-8B NF4 bs=1; 4096×4096 GEMV GB/s vs HBM peak"
                       if (args.model, args.quant) == ("llama3-8b", "nf4") else
                       f"decode tokens/sec {'Llama-3-70B' if args.model == 'llama3-70b' else 'Llama-3-8B'} "
                       f"{args.quant.upper()} bs=1; 4096×4096 GEMV GB/s vs HBM peak"),
            "value": round(tok_s, 3), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak" if weak else "strong", "vs_baseline": None,
            "dtype": f"{'bf16' if args.dtype == 'bf16' else 'f16'} activations x 4-bit {args.quant.upper()} weights "
                     f"({codes_desc(args, compute_dtype)}), fp32 accumulate",
            "data": f"synthetic (random-init {'Llama-3-70B' if args.model == 'llama3-70b' else 'Llama-3-8B'} "
                    "architecture, random prompt)",
            "config": {"workload": f"{args.model}-{args.quant}{'' if args.no_dq else '-dq'}"
                                   f"{'-bf16' if args.dtype == 'bf16' else ''}-decode-bs1",
                       "layers": cfg.num_hidden_layers,
                       "prompt_len": args.prompt, "global_batch": gbatch, "streams_per_gpu": gbatch / world,
                       "stream_batch": 1, "decode": mode,
                       "parallelism": parallelism(tp_mode),
                       "projection_groups": n_groups, "layer_ops": n_layer_ops},
            "roofline": roof, "parity": parity, "cpu_baseline": cpu, "prefill_config4": prefill,
        }
        line["config"]["compute_dtype"] = args.compute_dtype
        line["config"]["rmsnorm_in_grouped_gemv"] = bool(not args.no_prenorm and not args.no_fuse
                                                         and layer_ops in ("all", "norm"))
        line["config"]["decode_attention"] = ("qz_decode_attention" if not args.no_attention
                                              and layer_ops in ("all", "all+decoder") else "transformers sdpa")
        line["config"]["silu_in_gate_up_launch"] = bool(not args.no_mlp_pair and not args.no_fuse
                                                        and layer_ops in ("all", "all+decoder", "mlp"))
        line["config"]["residual_in_gemv_epilogue"] = bool(not args.no_residual and not args.no_attention
                                                           and layer_ops == "all")
        line["config"]["lm_head"] = "F.linear (hipBLASLt)" if (args.lm_head_library or layer_ops == "none") \
            else "layer_ops.gemv_dense"
        line["config"]["lm_head_rows_split"] = bool(sharded and tp_mode == "gather" and not args.no_shard_lm_head)
        line["config"]["attention"] = ("head-sharded (local q/k/v heads, attention output gathered)"
                                       if sharded and tp_mode == "gather" and not args.replicated_attention
                                       else "replicated" if sharded and tp_mode == "gather" else
                                       "local heads (TP pairing)" if sharded else "single GPU")
        line["config"]["decode_glue_launches"] = bool(not args.no_glue and layer_ops != "none")
        line["config"]["greedy_argmax"] = {"kernel": "one launch with the feedback (layer_ops.greedy_step)",
                                           "two-stage": "two-stage (greedy_token)", "torch": "torch.argmax"}[GREEDY]
        line["config"]["knobs"] = _safe(effective_knobs)
        if exchange is not None:
            line["config"]["exchange"] = exchange
        if extra_codes is not None:
            line["decode_other_codes"] = extra_codes
        if chain is not None:
            line["chain_roofline"] = chain
        if layer is not None:
            line["rowsplit_layer"] = layer
        if extra_weak is not None:
            line["weak_scaling_extra"] = extra_weak
        print(json.dumps(line), flush=True)
    if sharded:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

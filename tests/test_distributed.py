"""Row-sharded Linear4bit over torch.distributed (gloo, world_size 2, CPU).

The sharding logic -- slicing the GLOBAL packed bytes, first- and second-level
scales with the right block_base -- and the all-gather reassembly are checked
end to end: each rank evaluates its shard with the oracle (test-only local
compute hook; the product's local compute is the HIP GEMV, covered on GPU) and
the gathered output must equal the oracle's full-layer output bit for bit."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full_module(M, K, qt, seed, bias):
    import oracle
    from quantizations_amd.core import QuantState, create_dynamic_map, get_4bit_type

    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(M, K, generator=g) * 0.02).to(torch.float16)
    st = oracle.quantize_4bit(W.float().numpy(), 64, qt, double_quant=True)
    st2 = QuantState(absmax=torch.from_numpy(st.absmax2), blocksize=256, code=create_dynamic_map(),
                     dtype=torch.float32)
    qs = QuantState(absmax=torch.from_numpy(st.qabsmax), shape=torch.Size([M, K]), code=get_4bit_type(qt, "cpu"),
                    blocksize=64, quant_type=qt, dtype=torch.float16, offset=torch.tensor(float(st.offset)),
                    state2=st2)
    weight = types.SimpleNamespace(data=torch.from_numpy(st.packed).reshape(-1, 1), quant_state=qs)
    b = torch.randn(M, generator=g).to(torch.float16) if bias else None
    mod = types.SimpleNamespace(weight=weight, bias=None if b is None else types.SimpleNamespace(data=b),
                                in_features=K, out_features=M)
    return mod, st, b


def _oracle_local(x, shard):
    """Test hook: evaluate a shard with the oracle through its sliced state + block_base."""
    import oracle

    st = shard.state
    rows, K = st.shape
    nb = rows * K // st.blocksize
    b = np.arange(nb) + shard.block_base
    code2 = st.state2.code.numpy()
    am = (code2[st.absmax.numpy()[b]] * st.state2.absmax.numpy()[b // st.state2.blocksize]).astype(np.float32)
    am = (am + np.float32(st.offset)).astype(np.float32)
    xs = x.reshape(-1, K).float().numpy()
    ys = [oracle.gemv_4bit(xr, shard.packed.numpy(), am, st.code.numpy(), rows, K, st.blocksize) for xr in xs]
    y = torch.from_numpy(np.stack(ys).astype(np.float32))
    if shard.bias is not None:
        y = y + shard.bias.float()
    return y.reshape(*x.shape[:-1], rows)


def _worker(rank, world, port, M, K, qt, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from quantizations_amd.parallel import RowShardedLinear4bit

        full, st, b = _full_module(M, K, qt, seed=3, bias=True)
        layer = RowShardedLinear4bit(full, local_matmul=_oracle_local)
        g = torch.Generator().manual_seed(9)
        x = torch.randn(1, T, K, generator=g).to(torch.float16)
        y = layer(x)
        xs = x.reshape(T, K).float().numpy()
        ref = np.stack([oracle.gemv(xr, st) for xr in xs]).astype(np.float32) + b.float().numpy()
        q.put((rank, bool(np.array_equal(y.reshape(T, M).numpy(), ref)), tuple(y.shape), layer.block_base))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("M,K,qt,T", [(256, 512, "nf4", 1), (256, 512, "fp4", 3), (96, 1024, "nf4", 2),
                                      (64, 640, "fp4", 1)])
def test_row_sharded_gather_matches_full_layer(M, K, qt, T):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, K, qt, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, shape, _ in res:
        assert ok, f"rank {rank}: gathered output differs from the full layer"
        assert shape == (1, T, M)
    # (64 rows x 640) / 64 = 640 blocks; rank 1 starts at block 320 -> 2nd-level block 1, base 64
    if (M, K) == (64, 640):
        assert sorted(r[3] for r in res) == [0, 64]


def test_shard_rows_rejects_unaligned():
    from quantizations_amd.core import QuantState
    from quantizations_amd.parallel import shard_rows

    qs = QuantState(absmax=torch.zeros(10), shape=torch.Size([10, 96]), blocksize=64, quant_type="fp4")
    with pytest.raises(ValueError):
        shard_rows(torch.zeros(480, dtype=torch.uint8), qs, 1, 3)   # 10 rows / 3
    with pytest.raises(ValueError):
        shard_rows(torch.zeros(480, dtype=torch.uint8), qs, 1, 2)   # row 5 * 96 not on a 64-block


def _group_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from quantizations_amd.integration import fuse_projection_groups
        from quantizations_amd.parallel import RowShardedLinear4bit

        parent = torch.nn.Module()
        refs = {}
        for i, (name, M) in enumerate((("q_proj", 256), ("k_proj", 128), ("v_proj", 128))):
            full, st, b = _full_module(M, 512, "nf4", seed=20 + i, bias=True)
            parent.add_module(name, RowShardedLinear4bit(full, local_matmul=_oracle_local))
            refs[name] = (st, b)
        assert fuse_projection_groups(parent) == 1
        g = torch.Generator().manual_seed(5)
        ok = True
        for trial in range(2):  # a fresh x must recompute the group
            x = torch.randn(1, 1, 512, generator=g).to(torch.float16)
            for name in ("q_proj", "k_proj", "v_proj"):
                y = getattr(parent, name)(x)
                st, b = refs[name]
                ref = (oracle.gemv(x.reshape(-1).float().numpy(), st).astype(np.float32)
                       + b.float().numpy()).astype(np.float16)
                ok = ok and tuple(y.shape) == (1, 1, st.packed.size * 2 // 512) and \
                    bool(np.array_equal(y.reshape(-1).numpy(), ref))
        # a small batch of decode tokens (3) runs through the group with ONE all-gather of
        # [T, sum(rows)]; a 20-token prefill bypasses it -- both keep the fp32 hook output
        for T in (3, 20):
            xp = torch.randn(1, T, 512, generator=g).to(torch.float16)
            for name in ("q_proj", "k_proj", "v_proj"):
                yp = getattr(parent, name)(xp)
                st, b = refs[name]
                refp = np.stack([oracle.gemv(r, st) for r in xp.reshape(T, 512).float().numpy()]).astype(np.float32)
                ok = ok and tuple(yp.shape) == (1, T, st.packed.size * 2 // 512) and \
                    bool(np.array_equal(yp.reshape(T, -1).numpy(), refp + b.float().numpy()))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_row_sharded_projection_group_single_gather():
    """q/k/v fused into one DecodeGroup: one grouped local GEMV + ONE all-gather
    per decode step; every member's output equals its own full layer."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok, f"rank {rank}: grouped sharded outputs differ from the full layers"


def _tp_hook(x, mod):
    """Test hook: a shard's local product from its own packed bytes + statistics
    (oracle dequant; double quant resolved exactly as the kernels do)."""
    import oracle
    from quantizations_amd.parallel import consumer_absmax

    st = mod.state
    M, K = int(st.shape[0]), int(st.shape[1])
    nb = M * K // st.blocksize
    am = consumer_absmax(st)[mod.block_base:mod.block_base + nb]
    W = torch.from_numpy(oracle.dequantize_4bit(mod.packed.numpy(), am.numpy(), M * K, st.blocksize,
                                                st.quant_type)).reshape(M, K)
    y = x.float() @ W.t()
    if mod.bias is not None:
        y = y + mod.bias.float()
    return y.to(x.dtype)


def _tiny_llama_4bit(world: int = 2):
    """A tiny fp32 Llama whose decoder linears are Linear4bit layers built from
    ORACLE-quantised weights (layer 0 NF4, layer 1 FP4, double quant), plus the
    unsharded reference model holding the oracle's dequantised weights.  world > 2: a 512-wide
    model with 8 query and 8 kv heads, so the Megatron pairing can split heads and whole scale
    blocks over up to 8 ranks."""
    import copy

    import oracle
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.core import Params4bit, QuantState, create_dynamic_map, get_4bit_type
    from quantizations_amd.modules import Linear4bit

    # world > 2: widths whose column shards keep whole 64-element scale blocks at 8 ranks
    hidden, inter, heads, kv = (128, 256, 4, 2) if world <= 2 else (512, 512, 8, 8)
    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=inter, num_hidden_layers=2, num_attention_heads=heads,
                      num_key_value_heads=kv, vocab_size=104)   # rows split over 2, 4, 8 ranks (lm_head too)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).float().eval()
    ref = copy.deepcopy(model)
    for name, lin in list(model.named_modules()):
        if not isinstance(lin, torch.nn.Linear) or name == "lm_head":
            continue
        M, K = lin.out_features, lin.in_features
        qt = "nf4" if ".layers.0." in name else "fp4"   # one format per layer: groups need it
        W = lin.weight.detach().half()
        st = oracle.quantize_4bit(W.float().numpy(), 64, qt, double_quant=True)
        qs = QuantState(absmax=torch.from_numpy(st.qabsmax), shape=torch.Size([M, K]),
                        code=get_4bit_type(qt, "cpu"), blocksize=64, quant_type=qt, dtype=torch.float16,
                        offset=torch.tensor(float(st.offset)),
                        state2=QuantState(absmax=torch.from_numpy(st.absmax2), blocksize=256,
                                          code=create_dynamic_map(), dtype=torch.float32))
        l4 = Linear4bit(K, M, bias=False, quant_type=qt, device="meta")
        l4.weight = Params4bit.from_prequantized(torch.from_numpy(st.packed).reshape(-1, 1),
                                                 qs.as_dict(packed=True), device="cpu", module=l4)
        parent = model.get_submodule(name.rsplit(".", 1)[0])
        parent._modules[name.rsplit(".", 1)[1]] = l4
        ref.get_submodule(name).weight.data.copy_(torch.from_numpy(oracle.dequantize(st)).reshape(M, K))
    return cfg, model, ref


def _tp_worker(rank, world, port, q, batch=1, oneshot=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantizations_amd.integration import fuse_projection_groups
        from quantizations_amd.parallel import RowParallelLinear4bit, apply_tensor_parallel

        cfg, model, ref = _tiny_llama_4bit()
        ag = None
        if oneshot:  # the row-parallel all-reduce as a one-shot gather of the fp32 partials + sum
            from exchange_emulation import ShmAllGather
            ag = ShmAllGather(slot_bytes=8192, tag=f"tp{port}")
        n = apply_tensor_parallel(model, rank, world, local_matmul=_tp_hook, gatherer=ag)
        groups = fuse_projection_groups(model)
        ids = torch.tensor([[5, 17, 3, 88, 41, 9], [7, 2, 60, 11, 4, 30]])[:batch]
        with torch.no_grad():
            ref_logits = ref(input_ids=ids).logits
            out = model(input_ids=ids, use_cache=True)
            # one decode step through the (column-parallel) groups and the local-head KV cache
            nxt = out.logits[:, -1:].argmax(-1)
            step = model(input_ids=nxt, past_key_values=out.past_key_values, use_cache=True).logits
            ref_step = ref(input_ids=torch.cat([ids, nxt], 1)).logits[:, -1:]
            # the bench's decode layout: StaticCache (sized lazily from the local k/v heads) with
            # explicit cache/position ids, one stream per batch row
            from transformers.cache_utils import StaticCache
            cache = StaticCache(config=cfg, max_cache_len=ids.shape[1] + 4)
            L = ids.shape[1]
            model(input_ids=ids, past_key_values=cache, cache_position=torch.arange(L), use_cache=True)
            pos = torch.tensor([L])
            st_step = model(input_ids=nxt, past_key_values=cache, cache_position=pos,
                            position_ids=pos.view(1, 1).expand(ids.shape[0], 1), use_cache=True).logits
        rel = float((out.logits - ref_logits).norm() / ref_logits.norm())
        rel_step = max(float((step - ref_step).norm() / ref_step.norm()),
                       float((st_step - ref_step).norm() / ref_step.norm()))
        o_proj = model.model.layers[0].self_attn.o_proj
        if ag is not None:
            assert ag.calls >= 4, ag.calls   # o and down of 2 layers went through it at least once
            ag.close()
        q.put((rank, n, groups, rel, rel_step, isinstance(o_proj, RowParallelLinear4bit),
               model.model.layers[0].self_attn.q_proj.packed.numel()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch,oneshot", [(1, False), (2, False), (2, True)])
def test_tensor_parallel_pairing_tiny_llama(batch, oneshot):
    """Megatron TP pairing (column q/k/v/gate/up, row o/down + all-reduce) on a
    tiny Llama over gloo world 2: logits of prefill and of a cached decode step
    equal the unsharded model's (fp32 sums in another order).  batch 2 is the
    bench's weak-scaling layout (one decode stream per GPU, TP over all GPUs); with
    `oneshot` the row-parallel all-reduce runs as the one-shot exchange's gather of the
    fp32 partials + a rank-ordered sum (the protocol rehearsed over shared memory)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.path.join(REPO, "tests") + os.pathsep + \
        os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q, batch, oneshot)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, n, groups, rel, rel_step, is_rowpar, qshape in res:
        assert n == 4 and groups == 4 and is_rowpar, (rank, n, groups)
        assert qshape == 128 * 64 // 2   # q_proj rows 64 of 128 on each rank
        assert rel < 1e-5 and rel_step < 1e-5, (rank, rel, rel_step)


def _bench_layout_worker(rank, world, port, q, tp_mode, batch, layer_ops="none"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from quantizations_amd.parallel import RowShardedLinear4bit

        cfg, model, ref = _tiny_llama_4bit(world)
        n_groups, n_ops = bench.prepare_decode_model(model, rank, world, True, tp_mode, fuse=True,
                                                     layer_ops=layer_ops, local_matmul=_tp_hook)
        if layer_ops != "none":
            # the fused decoder layer on row shards: both norms absorbed into the sharded groups, the
            # MLP's gate/up + SiLU product as one local launch + one exchange of h, the residual adds
            # handed to o_proj / down_proj (forward_residual)
            from quantizations_amd.parallel import RowShardedLinear4bit
            lay = model.model.layers[0]
            grp = lay.mlp.gate_proj.__dict__["_qz_group"]
            assert grp.prenorm is not None and lay.self_attn.q_proj.__dict__["_qz_group"].prenorm is not None
            assert "_qz_residual_decoder" in lay.__dict__
            calls = {"pair": 0, "res": 0}
            import quantizations_amd.parallel as par
            orig_pair, orig_res = par.sharded_silu_pair, RowShardedLinear4bit.forward_residual

            def pair_spy(g, x):
                calls["pair"] += 1
                return orig_pair(g, x)

            def res_spy(self, x, r):
                calls["res"] += 1
                return orig_res(self, x, r)
            par.sharded_silu_pair = pair_spy
            RowShardedLinear4bit.forward_residual = res_spy
        # bench.py's own decode loop (StaticCache, static token/position buffers, token
        # feedback), eagerly on CPU; the reference is the unsharded dequantised model
        _, hist = bench.decode_bench_graph(model, cfg, steps=5, warmup=2, prompt_len=6, world=world, batch=batch,
                                           graph=False, device="cpu")
        if layer_ops != "none":
            par.sharded_silu_pair, RowShardedLinear4bit.forward_residual = orig_pair, orig_res
            assert calls["res"] > 0 or tp_mode == "pair", calls
            assert (calls["pair"] > 0) == (batch == 1), calls
        _, ref_hist = bench.decode_bench_graph(ref, cfg, steps=5, warmup=2, prompt_len=6, world=1, batch=batch,
                                               graph=False, device="cpu")
        attn = model.model.layers[0].self_attn
        up = model.model.layers[0].mlp.up_proj
        from quantizations_amd.parallel import RowShardedDenseLinear
        # the row split: up_proj gathers its rows; head-sharded attention: q/k/v stay local, o_proj
        # gathers the heads' outputs first
        heads = all(isinstance(m, RowShardedLinear4bit) and not m.gather for m in (attn.q_proj, attn.k_proj,
                                                                                    attn.v_proj)) \
            and isinstance(attn.o_proj, RowShardedLinear4bit) and attn.o_proj.gather_input and attn.o_proj.gather
        q.put((rank, n_groups, bool(torch.equal(hist, ref_hist)), int((hist[:, 6:13] != 0).sum()),
               isinstance(up, RowShardedLinear4bit) and up.gather and heads,
               isinstance(model.get_output_embeddings(), RowShardedDenseLinear)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("tp_mode,batch,layer_ops,world", [
    ("gather", 1, "none", 2), ("pair", 2, "none", 2), ("gather", 1, "all", 2), ("pair", 1, "all", 2),
    # config #5's rank counts: the row split + exchange at 4 and 8 ranks, the weak-scaling extra at 8
    ("gather", 1, "all", 4), ("gather", 1, "all", 8), ("pair", 8, "none", 8)])
def test_bench_multi_gpu_layout_end_to_end(tp_mode, batch, layer_ops, world):
    """bench.py --gpus N exactly as the driver runs it, on gloo world N (2, 4, 8) with the
    oracle as each shard's local product: the default strong-scaling layout
    (one bs=1 stream, every Linear4bit row-split + all-gather) and the
    weak-scaling extra (two streams, Megatron pairing).  The row split runs the attention
    head-sharded (each rank's q/k/v rows are whole heads, attended locally; o_proj gathers the
    heads' outputs).  The greedy tokens of 7
    decode steps equal the unsharded model's on every rank (the row split includes the
    fp16 lm_head: RowShardedDenseLinear).  layer_ops "all": the
    fused decoder layer on the shards (absorbed norms, the sharded SiLU pair, the
    residual epilogues), as bench.py sets it up for N > 1."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.path.join(REPO, "tests") + os.pathsep + \
        os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_bench_layout_worker, args=(r, world, port, q, tp_mode, batch, layer_ops))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, n_groups, same, n_tok, gathers, head_rows in res:
        assert n_groups == 4, (rank, n_groups)
        assert same, f"rank {rank}: sharded greedy tokens differ from the unsharded model"
        assert n_tok > 0
        assert gathers == (tp_mode == "gather")     # row split + head-sharded attention
        assert head_rows == (tp_mode == "gather")   # the fp16 lm_head row-split too


def _gemv_hook(x, mod):
    """Test hook: a shard's local GEMV with the reference's fp32 weight products
    (kernels.cu:1169: code[nibble] * absmax in fp32), output in x's dtype."""
    from quantizations_amd.parallel import consumer_absmax

    st = mod.state
    M, K = int(st.shape[0]), int(st.shape[1])
    b = mod.packed.reshape(-1).numpy()
    nib = np.stack([b >> 4, b & 15], axis=1).reshape(-1)
    am = consumer_absmax(st).numpy()[mod.block_base:mod.block_base + M * K // st.blocksize]
    W = (st.code.numpy()[nib] * np.repeat(am, st.blocksize)).astype(np.float32).reshape(M, K)
    y = torch.from_numpy(x.reshape(-1, K).double().numpy() @ W.T.astype(np.float64))
    if mod.bias is not None:
        y = y + mod.bias.double()
    return y.reshape(*x.shape[:-1], M).to(x.dtype)


def _rowpar_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from quantizations_amd.parallel import RowParallelLinear4bit

        M, K = 256, 1024
        full, st, b = _full_module(M, K, "nf4", seed=31, bias=True)
        layer = RowParallelLinear4bit(full, local_matmul=_gemv_hook)
        Kp = K // world
        g = torch.Generator().manual_seed(4)
        x = (torch.randn(1, 1, K, generator=g) * 4).to(torch.float16)
        Kp = K // world
        y = layer(x[..., rank * Kp:(rank + 1) * Kp])
        # emulation: each rank's partial rounded to fp16 once, summed in fp32, rounded once
        from quantizations_amd.parallel import consumer_absmax
        qs = full.weight.quant_state
        pk = full.weight.data.reshape(-1).numpy()
        nib = np.stack([pk >> 4, pk & 15], axis=1).reshape(-1)
        W = (qs.code.numpy()[nib] * np.repeat(consumer_absmax(qs).numpy(), 64)).astype(np.float32).reshape(M, K)
        xd = x.reshape(-1).double().numpy()
        parts = [(xd[r * Kp:(r + 1) * Kp] @ W[:, r * Kp:(r + 1) * Kp].T.astype(np.float64)
                  + (b.double().numpy() if r == 0 else 0.0)).astype(np.float16) for r in range(world)]
        emu = np.sum(np.stack(parts).astype(np.float32), axis=0, dtype=np.float32).astype(np.float16)
        q.put((rank, y.dtype == torch.float16, bool(np.array_equal(y.reshape(-1).numpy(), emu))))
    finally:
        dist.destroy_process_group()


def test_row_parallel_fp32_allreduce_within_fp16_rounding():
    """Row-parallel o/down layer at world 2 with fp16 activations: each rank's
    fp16 partial is summed in fp32 and rounded to fp16 ONCE (an fp16 all-reduce
    would add one more rounding per rank beyond two).  Bit-exact against that
    emulation."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.path.join(REPO, "tests") + os.pathsep + \
        os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_rowpar_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, is_half, same in res:
        assert is_half
        assert same, f"rank {rank}: row-parallel output is not the fp32 sum of the fp16 partials"


def test_shard_attention_heads_and_tied_lm_head_rules():
    """CPU, no collective: shard_attention_heads keeps q/k/v row shards local and makes o_proj gather its
    input only where every projection's rows are whole heads on each rank (world 2: 4 q / 2 kv heads split;
    world 8: 2 kv heads of 32 do not -- left replicated); shard_lm_head refuses a head tied to the input
    embedding (the embedding stays whole, and tie_weights() would undo the split)."""
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.parallel import (RowShardedDenseLinear, RowShardedLinear4bit, shard_attention_heads,
                                            shard_lm_head, shard_model_linear4bit)

    for world, expect in ((2, 2), (8, 0)):
        cfg, model, _ = _tiny_llama_4bit(2)
        shard_model_linear4bit(model, 0, world)
        assert shard_attention_heads(model) == expect
        attn = model.model.layers[0].self_attn
        assert all(isinstance(m, RowShardedLinear4bit) for m in (attn.q_proj, attn.k_proj, attn.v_proj, attn.o_proj))
        assert attn.q_proj.gather == (expect == 0) and attn.o_proj.gather_input == (expect > 0)
        assert model.model.layers[0].mlp.up_proj.gather   # the MLP keeps the plain row split
    for tied in (False, True):
        cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=1, num_attention_heads=2,
                          num_key_value_heads=2, vocab_size=96, tie_word_embeddings=tied)
        model = LlamaForCausalLM(cfg).eval()
        assert shard_lm_head(model, 0, 2) == (not tied)
        assert isinstance(model.get_output_embeddings(), RowShardedDenseLinear) == (not tied)

"""GPU: the north-star multi-GPU layout at world size 2 on the real kernels -- every
Linear4bit of a small Llama row-split over two ranks (RowShardedLinear4bit slicing the global
quant state, block_base addressing, grouped q/k/v and gate/up shard launches) and the shards
exchanged by the one-shot all-gather (exchange.OneShotAllGather, both protocols by payload),
driven by bench.py's own decode loop (HIP-graph capture).  The box has one MI355X, so the two
ranks are two processes on it mapping each other's exchange buffers (gloo only for the setup
and barriers; RCCL cannot put two ranks on one GPU).  Each rank's logits of a teacher-forced
prefill + decode step match the unsharded model's within fp16 rounding, and both ranks'
greedy decodes agree with each other token for token.  The same for the Megatron pairing
(column-parallel q/k/v/gate/up on the local heads, row-parallel o/down whose fp32 partials the
one-shot exchange gathers and every rank sums in rank order)."""
import copy
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO
from test_distributed import _free_port

pytestmark = pytest.mark.gpu


def _model(dev, world=2):
    from transformers import LlamaConfig, LlamaForCausalLM

    from quantizations_amd.integration import replace_with_bnb_linear

    # 8 kv heads from 4 ranks on, so the Megatron pairing splits them
    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=4 if world <= 2 else 8, vocab_size=1024, max_position_embeddings=256)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).half().to(dev).eval()
    replace_with_bnb_linear(model, quant_type="nf4", compute_dtype=torch.float32)
    return cfg, model


def _worker(rank, world, port, q, layout):
    try:
        _work(rank, world, port, q, layout)
    except BaseException as e:  # report instead of leaving the peer blocked in a collective
        q.put((rank, "error", f"{type(e).__name__}: {e}"))
        raise


def _work(rank, world, port, q, layout):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        import bench
        from quantizations_amd.exchange import OneShotAllGather
        from quantizations_amd.integration import fuse_projection_groups
        from quantizations_amd.parallel import RowShardedLinear4bit, apply_tensor_parallel, shard_model_linear4bit

        dev = torch.device("cuda", 0)
        cfg, model = _model(dev, world)
        ref = copy.deepcopy(model)
        ag = OneShotAllGather(slot_bytes=1 << 18, device=dev)
        if layout.startswith("gather"):
            shard_model_linear4bit(model, rank, world, gatherer=ag)
            from quantizations_amd.parallel import shard_attention_heads, shard_lm_head
            assert shard_lm_head(model, rank, world, gatherer=ag)   # the fp16 lm_head's rows too, as bench.py
            if "heads" in layout:   # bench.py's default N > 1 layout: every rank attends over its own heads
                assert shard_attention_heads(model) == cfg.num_hidden_layers
        else:   # Megatron pairing: column q/k/v/gate/up, row o/down with the one-shot all-reduce
            apply_tensor_parallel(model, rank, world, gatherer=ag)
        n_groups = fuse_projection_groups(model)
        fuse_projection_groups(ref)
        if layout.endswith("fused"):
            # the fused decoder layer on the shards, as bench.py runs N > 1: both RMSNorms inside the
            # sharded q/k/v and gate/up launches, gate/up + SiLU as one launch on the local rows, the
            # residual adds in the o/down epilogues, the one-launch decode attention
            from quantizations_amd.integration import fuse_layer_ops, fuse_prenorm
            for m in (model, ref):
                fuse_layer_ops(m)
                assert fuse_prenorm(m) == 2 * cfg.num_hidden_layers
        lay = model.model.layers[0]
        fused_ok = (not layout.endswith("fused")) or (
            lay.mlp.gate_proj.__dict__["_qz_group"].prenorm is not None and "_qz_residual_decoder" in lay.__dict__)
        ids = torch.randint(0, cfg.vocab_size, (1, 12), generator=torch.Generator().manual_seed(5)).to(dev)
        with torch.inference_mode():
            a = model(input_ids=ids).logits.float()          # prefill: multi-token shard launches
            b = ref(input_ids=ids).logits.float()
            prefill_rel = ((a - b).norm() / b.norm()).item()
            a1 = model(input_ids=ids[:, :1]).logits.float()  # one token: grouped decode GEMVs
            b1 = ref(input_ids=ids[:, :1]).logits.float()
            decode_rel = ((a1 - b1).norm() / b1.norm()).item()
        torch.cuda.synchronize()
        dist.barrier()
        # bench.py's decode loop, HIP-graph captured, at world N; the unsharded model's greedy decode
        # (the same kernels on all rows) on this process for comparison
        _, hist = bench.decode_bench_graph(model, cfg, steps=6, warmup=2, prompt_len=8, world=world, batch=1)
        hist = hist.cpu()
        _, ref_hist = bench.decode_bench_graph(ref, cfg, steps=6, warmup=2, prompt_len=8, world=1, batch=1)
        same_as_unsharded = bool(torch.equal(hist, ref_hist.cpu()))
        allh = [None] * world
        dist.all_gather_object(allh, hist)
        q0 = model.model.layers[0].self_attn.q_proj
        q.put((rank, n_groups, prefill_rel, decode_rel, all(torch.equal(allh[0], h) for h in allh), same_as_unsharded,
               int((hist[:, 8:16] != 0).sum()), ag.failed_anywhere(), isinstance(q0, RowShardedLinear4bit),
               q0.r1 - q0.r0, q0.r0, fused_ok))
        dist.barrier()
        ag.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(420)
@pytest.mark.parametrize("layout,world", [("gather", 2), ("pair", 2), ("gather-fused", 2), ("pair-fused", 2),
                                          ("gather-fused", 4), ("gather-fused", 8), ("pair-fused", 8),
                                          ("gather-heads", 2), ("gather-heads-fused", 2), ("gather-heads-fused", 4),
                                          ("gather-heads-fused", 8)])
def test_rowsplit_oneshot_on_gpu(layout, world):
    """world 8: config #5's layout with 8 processes on the one MI355X (each mapping the 7 others'
    exchange buffers); gather layouts decode exactly the unsharded model's greedy tokens (a shard's
    rows are summed in the same order as the unsharded launch's).  gather-heads: bench.py's default
    N > 1 layout, the attention head-sharded (parallel.shard_attention_heads: local q/k/v heads, a
    KV cache of the rank's kv heads, the heads' outputs gathered before o_proj)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.path.join(REPO, "tests") + os.pathsep + \
        os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, layout)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted((q.get(timeout=360) for _ in range(world)), key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[1] != "error", f"rank {r[0]}: {r[2]}"
    for p in procs:
        assert p.exitcode == 0
    rows_exp = 512 // world
    for rank, n_groups, prefill_rel, decode_rel, same, same_ref, n_tok, failed, sharded, rows, r0, fused_ok in res:
        assert sharded and rows == rows_exp and n_groups == 4, (rank, rows, n_groups)
        assert fused_ok, "the fused layer was not installed on the shards"
        assert r0 == rows_exp * rank                 # q_proj rows [rows rank, +rows) of 512
        if layout.startswith("gather"):
            assert same_ref, f"rank {rank}: greedy tokens differ from the unsharded model's"
        assert not failed, f"rank {rank}: an exchange timed out"
        # row shards multiply the global state's exact weights; fp32 summation order and the
        # fp16 rounding of a shard launch's outputs are the only differences
        assert prefill_rel < 2e-3 and decode_rel < 2e-3, (rank, prefill_rel, decode_rel)
        assert same, "the ranks decoded different tokens"
        assert n_tok > 0

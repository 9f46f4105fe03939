"""The one-shot all-gather's host logic on CPU (gloo world 2, 4 and 8 -- config #5's ranks): the test-only shared-memory
rehearsal of comm.hip's protocol (tests/exchange_emulation.py) returns exactly what
dist.all_gather_into_tensor returns -- rank-major shard placement, both slot parities,
payloads from 16 B to the slot size -- and, as the `gatherer` of the row-split model,
yields the unsharded model's greedy tokens while every decode exchange goes through it
(larger payloads fall back to the collective)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO
from test_distributed import _free_port, _tiny_llama_4bit, _tp_hook


def _env():
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.path.join(REPO, "tests") + os.pathsep + \
        os.environ.get("PYTHONPATH", "")


def _placement_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from exchange_emulation import ShmAllGather

        from quantizations_amd.exchange import all_gather_into

        ag = ShmAllGather(slot_bytes=6144, tag=f"p{port}")
        ok, used = True, 0
        g = torch.Generator().manual_seed(rank)
        for n in (8, 16, 24, 512, 2048, 8, 3072, 2048, 4096):  # fp16 elements: 16 B .. 8 KiB (both protocols)
            x = torch.randn(n, generator=g).half()
            a = torch.empty(world * n, dtype=torch.float16)
            b = torch.empty_like(a)
            before = ag.calls
            all_gather_into(a, x, None, ag)
            used += ag.calls - before
            dist.all_gather_into_tensor(b, x)
            ok = ok and torch.equal(a, b)
        ag.close()
        q.put((rank, ok, used))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_oneshot_protocol_placement_and_parity(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    _env()
    procs = [ctx.Process(target=_placement_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, used in res:
        assert ok, f"rank {rank}: one-shot result differs from all_gather_into_tensor"
        assert used == 8, used     # 4096 elements = 8 KiB > the 6 KiB slot: the collective


def _model_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from exchange_emulation import ShmAllGather

        from quantizations_amd.integration import fuse_projection_groups
        from quantizations_amd.parallel import shard_model_linear4bit

        cfg, model, ref = _tiny_llama_4bit(world)
        ag = ShmAllGather(slot_bytes=1024, tag=f"m{port}")
        shard_model_linear4bit(model, rank, world, local_matmul=_tp_hook, gatherer=ag)
        n_groups = fuse_projection_groups(model)
        _, hist = bench.decode_bench_graph(model, cfg, steps=5, warmup=2, prompt_len=6, world=world, batch=1,
                                           graph=False, device="cpu")
        _, ref_hist = bench.decode_bench_graph(ref, cfg, steps=5, warmup=2, prompt_len=6, world=1, batch=1,
                                               graph=False, device="cpu")
        q.put((rank, n_groups, bool(torch.equal(hist, ref_hist)), ag.calls))
        ag.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_row_split_model_through_oneshot_gatherer(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    _env()
    procs = [ctx.Process(target=_model_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, n_groups, same, calls in res:
        assert n_groups == 4
        assert same, f"rank {rank}: tokens differ from the unsharded model"
        # 2 layers x (q/k/v group + o + gate/up group + down) per decode step, 7 decode steps
        assert calls >= 2 * 4 * 7, calls

"""GPU: the one-shot all-gather (comm.hip k_allgather_oneshot through exchange.OneShotAllGather)
between 2, 4 and 8 processes -- ranks on the box's one MI355X, each mapping the others'
uncached exchange buffers through a hipIpc handle (on an 8-GPU node the same code maps
the peers' buffers over xGMI).  Every call's rank-major result equals the concatenation
of both ranks' shards, over payload sizes from 16 B to the slot size, both slot parities,
both protocols (flags, tagged granules) interleaved, eager launches and a HIP-graph replay;
no wait ever times out."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO
from test_distributed import _free_port

pytestmark = pytest.mark.gpu


def _shard(rank, call, n):
    g = torch.Generator().manual_seed(1000 * call + rank)
    return torch.randn(n, generator=g).half()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        from quantizations_amd.exchange import OneShotAllGather

        dev = torch.device("cuda", 0)
        ag = OneShotAllGather(slot_bytes=1 << 18, device=dev)   # bench.setup_oneshot's slot
        bad = []
        # fp16 elements: 16 B .. 64 KiB, and the row-split lm_head's logits (128256 / N rows: N = 2, 8)
        sizes = [8, 16, 1024, 7168, 32768, 8, 4096, 14336, 64128, 16032]
        for call in range(24):
            n = sizes[call % len(sizes)]
            x = _shard(rank, call, n).to(dev)
            out = torch.empty(world * n, dtype=torch.float16, device=dev)
            ag(out, x, (0, 1, 2)[call % 3])   # by size, flag protocol, tagged granules
            exp = torch.cat([_shard(r, call, n) for r in range(world)])
            if not torch.equal(out.cpu(), exp):
                bad.append(call)
        ag.warm_graph()   # the throwaway first graph bench.setup_oneshot captures (collective)
        # graph capture: fixed buffers, four calls per replay
        n = 2048
        xs = [torch.empty(n, dtype=torch.float16, device=dev) for _ in range(4)]
        outs = [torch.empty(world * n, dtype=torch.float16, device=dev) for _ in range(4)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for x, o in zip(xs, outs):
                ag(o, x)
        torch.cuda.synchronize()
        for rep in range(3):
            for i, x in enumerate(xs):
                x.copy_(_shard(rank, 100 + 10 * rep + i, n))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                exp = torch.cat([_shard(r, 100 + 10 * rep + i, n) for r in range(world)])
                if not torch.equal(o.cpu(), exp):
                    bad.append(("graph", rep, i))
        q.put((rank, bad, ag.failed(), int(ag.epoch[0].item())))
        dist.barrier()
        ag.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(420)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_oneshot_allgather_processes_one_gpu(world):
    """world 8 is config #5's rank count: 8 processes on the one MI355X, each mapping the 7
    others' buffers (the 8-rank granule regions, the epoch ticket at 8 writers)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    os.environ["PYTHONPATH"] = REPO + os.pathsep + os.path.join(REPO, "tests") + os.pathsep + \
        os.environ.get("PYTHONPATH", "")
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=360) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    for rank, bad, failed, epoch in res:
        assert not failed, f"rank {rank}: a peer's signal timed out"
        assert not bad, f"rank {rank}: wrong all-gather results at {bad}"
        # 24 eager calls + warm_graph (2 eager, 3 replays x 2) + 3 replays x 4 (capture runs nothing)
        assert epoch == 24 + 2 + 3 * 2 + 3 * 4, epoch

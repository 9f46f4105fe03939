"""Per-call time of the one-shot all-gather by protocol and payload (one MI355X: world 1, or
two processes on the same GPU with --world 2), 50 calls captured in one HIP graph, and the
RCCL all_gather_into_tensor at world 1 for comparison.  Prints one JSON line per rank 0.

  python scripts/exchange_times.py [--world 2]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timed(fn, calls=50, reps=5, all_reps=None):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    best = None
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        if all_reps is not None:
            all_reps.append(round(dt / calls * 1e6, 2))
    return round(best / calls * 1e6, 2)


def worker(rank, world, port, backend, reverse=False, granules_first=False, warm=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    from quantizations_amd.exchange import OneShotAllGather
    dev = torch.device("cuda", 0)
    ag = OneShotAllGather(slot_bytes=1 << 17, device=dev)
    res = {}
    if warm:  # a throwaway graph of flag-protocol calls before anything is timed
        xw = torch.randn(512, device=dev).half()
        ow = torch.empty(world * 512, device=dev, dtype=torch.float16)
        timed(lambda: ag(ow, xw, 1), reps=2)
    sizes = (256, 1024, 2048, 4096, 7168, 16384, 65536)
    order = list(reversed(sizes)) if reverse else list(sizes)
    for nbytes in order:
        n = nbytes // 2
        x = torch.randn(n, device=dev).half()
        out = torch.empty(world * n, device=dev, dtype=torch.float16)
        fr, gr = [], []
        if granules_first:
            row = {"granules": timed(lambda: ag(out, x, 2), all_reps=gr)}
            row["flags"] = timed(lambda: ag(out, x, 1), all_reps=fr)
        else:
            row = {"flags": timed(lambda: ag(out, x, 1), all_reps=fr), "granules": timed(lambda: ag(out, x, 2), all_reps=gr)}
        row["flags_reps"], row["granules_reps"] = fr, gr
        if world == 1:
            row["rccl"] = timed(lambda: dist.all_gather_into_tensor(out, x))
        res[nbytes] = row
    if rank == 0:
        print(json.dumps({"world": world, "order": "descending" if reverse else "ascending",
                          "first": "granules" if granules_first else "flags", "warm_graph": warm, "us_per_call": res,
                          "failed": ag.failed()}), flush=True)
    dist.barrier()
    ag.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--reverse", action="store_true", help="measure the payload sizes largest first")
    ap.add_argument("--granules-first", action="store_true", help="time the granule protocol before the flags one")
    ap.add_argument("--warm", action="store_true", help="replay a throwaway flag-protocol graph before timing")
    a = ap.parse_args()
    import socket
    sk = socket.socket(); sk.bind(("127.0.0.1", 0)); port = sk.getsockname()[1]; sk.close()
    if a.world == 1:
        worker(0, 1, port, "nccl", a.reverse, a.granules_first, a.warm)
    else:
        mp.start_processes(worker, args=(a.world, port, "gloo", a.reverse, a.granules_first, a.warm), nprocs=a.world, join=True, start_method="spawn")

"""Dev probe: per-launch period of the empty launch, the one-shot read floor and
the 4096^2 NF4+DQ GEMV, launched back-to-back on a parked stream vs replayed
from one HIP graph (how the decode step runs).  Rotating weight copies."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizations_amd import _lib  # noqa: E402
from quantizations_amd.core import quantize_4bit  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(7)
    W = (torch.randn(4096, 4096, device=dev) * 0.02).to(torch.float16)
    packed, qs = quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    copies = 64
    sets = [(packed.clone(), qs.absmax.clone(), qs.state2.absmax.clone()) for _ in range(copies)]
    x = torch.randn(4096, device=dev).to(torch.float16)
    y = torch.empty(4096, device=dev, dtype=torch.float16)
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    code2, off = qs.state2.code, qs.offset
    L = _lib.lib

    def gemv(i, stream):
        p, qa, a2 = sets[i % copies]
        rc = L.qz_gemv_4bit(4096, 4096, x.data_ptr(), _lib.DT_F16, p.data_ptr(), _lib.NF4, 64, 0, qa.data_ptr(),
                            a2.data_ptr(), code2.data_ptr(), off.data_ptr(), 256, 0, 0, 0, y.data_ptr(), stream)
        assert rc == 0

    def floor(i, stream):
        p = sets[i % copies][0]
        assert L.qz_bench_read_floor(p.data_ptr(), p.numel(), sink.data_ptr(), stream) == 0

    def empty(i, stream):
        assert L.qz_bench_empty(sink.data_ptr(), stream) == 0

    n = 128
    out = {}
    for name, fn in (("empty", empty), ("floor", floor), ("gemv", gemv)):
        s = torch.cuda.current_stream().cuda_stream
        for i in range(n):
            fn(i, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = []
        for _ in range(5):
            torch.cuda._sleep(100_000_000)
            e0.record()
            for i in range(n):
                fn(i, s)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / n)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            fn(0, cs.cuda_stream)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cs):
            for i in range(n):
                fn(i, torch.cuda.current_stream().cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        gres = []
        for _ in range(5):
            torch.cuda._sleep(100_000_000)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            gres.append(e0.elapsed_time(e1) * 1e3 / n)
        out[name] = {"stream_us": round(sorted(res)[2], 3), "graph_us": round(sorted(gres)[2], 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

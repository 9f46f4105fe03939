"""Price each phase of k_decode_attn (measurement only): the QZ_ATTN_ABL builds of
layer_ops.hip (scripts/dev/build_attn_abl.sh) launched at the bench's decode shape
(B 1, Hq 32, Hkv 8, D 128, L 112, fp16), back-to-back and as a 32-launch HIP graph
(the decode step's 32 layers, one replay ~ one token's attention launches)."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def run(abl, B=1, Hq=32, Hkv=8, D=128, L=112, p=60):
    lib = ctypes.CDLL(os.path.join(HERE, "attn_abl", f"libattn_{abl}.so"))
    f = lib.qz_decode_attention
    f.restype = ctypes.c_int
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, Hq * D, device=dev, generator=g).half()
    k = torch.randn(B, Hkv * D, device=dev, generator=g).half()
    v = torch.randn(B, Hkv * D, device=dev, generator=g).half()
    cos = torch.rand(1, D, device=dev, generator=g).half()
    sin = torch.rand(1, D, device=dev, generator=g).half()
    caches = [(torch.randn(B, Hkv, L, D, device=dev, generator=g).half(),
               torch.randn(B, Hkv, L, D, device=dev, generator=g).half()) for _ in range(32)]
    mask = torch.zeros(1, L, dtype=torch.bool, device=dev)
    mask[:, : p + 1] = True
    pos = torch.tensor([p], dtype=torch.int64, device=dev)
    arrive = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.float16)
    vp = ctypes.c_void_p
    P = lambda t: vp(t.data_ptr())

    def launch(i, stream):
        kc, vc = caches[i % 32]
        rc = f(0, B, Hq, Hkv, D, L, P(q), ctypes.c_longlong(Hq * D), P(k), ctypes.c_longlong(Hkv * D), P(v),
               ctypes.c_longlong(Hkv * D), P(cos), P(sin), ctypes.c_longlong(0), P(kc), P(vc), P(mask),
               ctypes.c_longlong(0), ctypes.c_longlong(1), P(pos), P(arrive), P(out), ctypes.c_longlong(Hq * D),
               vp(0), ctypes.c_float(D ** -0.5), vp(stream))
        assert rc == 0, rc

    s = torch.cuda.current_stream()
    for i in range(200):
        launch(i, s.cuda_stream)
    torch.cuda.synchronize()
    n = 2000
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        launch(i, s.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    b2b = e0.elapsed_time(e1) * 1e3 / n
    gs = torch.cuda.Stream()
    gs.wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(gs):
        graph.capture_begin()
        for i in range(32):
            launch(i, gs.cuda_stream)
        graph.capture_end()
    torch.cuda.synchronize()
    for _ in range(20):
        graph.replay()
    torch.cuda.synchronize()
    reps = 200
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    gr = e0.elapsed_time(e1) * 1e3 / reps / 32
    return {"abl": abl, "back_to_back_us": round(b2b, 3), "graph_us_per_launch": round(gr, 3)}


if __name__ == "__main__":
    for a in [int(x) for x in (sys.argv[1:] or ["0", "1", "2", "4", "8", "16", "32"])]:
        print(json.dumps(run(a)), flush=True)

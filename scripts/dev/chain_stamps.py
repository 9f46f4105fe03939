"""Stage timeline of the persistent MLP chain (csrc/chain.hip) from its diagnostic build
(libqz_diag.so, qz_diag_mlp_chain_stamped): wave 0 of every workgroup stamps s_memrealtime
(100 MHz) at the chain's stage points; the last of `burst` back-to-back launches over 8 rotating
Llama-3-8B (or --model llama3-70b) weight sets is read back and each point is printed as
p10 / p50 / p90 / max over workgroups, in microseconds from the first workgroup's start.

  python scripts/dev/chain_stamps.py [--model llama3-70b] [--burst 24] [--samples 5]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

POINTS = ["start", "stage A done", "h1 drained", "barrier 0 passed", "x' in LDS", "stage B done",
          "barrier 1 passed", "act in LDS", "stage C done (wave 0)", "all waves done"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--burst", type=int, default=24)
    ap.add_argument("--samples", type=int, default=5)
    a = ap.parse_args()
    import bench
    from quantizations_amd import _lib
    from quantizations_amd.core import _gemv_quant_type, mlp_chain_state, quantize_4bit

    cfg = bench.MODELS[a.model]
    H, I = cfg["hidden_size"], cfg["intermediate_size"]
    dev = torch.device("cuda")
    torch.manual_seed(3)
    sets = []
    for _ in range(8):
        d = {}
        for name, (M, K) in (("o", (H, H)), ("gate", (I, H)), ("up", (I, H)), ("down", (H, I))):
            W = (torch.randn(M, K, device=dev) * 0.02).half()
            d[name] = quantize_4bit(W, quant_type="nf4", compress_statistics=True)
            del W
        sets.append(d)
    x = torch.randn(H, device=dev).half()
    res = torch.randn(H, device=dev).half()
    nw = (1 + 0.1 * torch.randn(H, device=dev)).half()
    h1 = torch.empty(H, device=dev, dtype=torch.float16)
    act = torch.empty(I, device=dev, dtype=torch.float16)
    out = torch.empty(H, device=dev, dtype=torch.float16)
    st = mlp_chain_state(dev)
    stamps = torch.zeros(4096 * 12, dtype=torch.int64, device=dev)
    diag = ctypes.CDLL(os.path.join(REPO, "quantizations_amd", "libqz_diag.so"))
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    diag.qz_diag_mlp_chain_stamped.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, ctypes.c_float, vp, vp,
                                               vp, vp, vp, ctypes.POINTER(i32), vp]
    grid = i32(0)
    qt = _gemv_quant_type("nf4", True, torch.float16)
    stream = torch.cuda.current_stream().cuda_stream
    segs_all = []
    for d in sets:
        segs = (_lib.GemvSegment * 4)()
        for i, name in enumerate(("o", "gate", "up", "down")):
            p, s = d[name]
            am, qam, am2, code2, off, _ = s.scale_args()
            segs[i] = _lib.GemvSegment(s.shape[0], p.data_ptr(), am, qam, am2, code2, off, 0, None, None)
        segs_all.append(segs)

    def launch(i):
        segs = segs_all[i % len(segs_all)]
        base = ctypes.cast(segs, ctypes.c_void_p).value
        sz = ctypes.sizeof(_lib.GemvSegment)
        rc = diag.qz_diag_mlp_chain_stamped(base, base + sz, base + 2 * sz, base + 3 * sz, x.data_ptr(),
                                            res.data_ptr(), 0, qt, 64, 256, nw.data_ptr(), 1e-5, h1.data_ptr(),
                                            act.data_ptr(), out.data_ptr(), st.data_ptr(), stamps.data_ptr(),
                                            ctypes.byref(grid), stream)
        if rc:
            raise RuntimeError(f"qz_diag_mlp_chain_stamped rc={rc}")

    for i in range(16):
        launch(i)
    torch.cuda.synchronize()
    rows = []
    for smp in range(a.samples):
        torch.cuda._sleep(20_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.burst):
            launch(smp * a.burst + i)
        e1.record()
        torch.cuda.synchronize()
        per = e0.elapsed_time(e1) * 1e3 / a.burst
        s = stamps.view(-1, 12)[:grid.value].cpu().double()
        t0 = s[:, 0].min()
        rel = (s - t0) * 0.01
        print(f"sample {smp}: {grid.value} workgroups, {per:.2f} us per launch (b2b); failed={bool(st[-32].item())}")
        for k, name in enumerate(POINTS):
            col = sorted(rel[:, k].tolist())
            q = lambda f: col[min(int(f * len(col)), len(col) - 1)]
            print(f"  {k} {name:24s} p10 {q(.1):7.2f}  p50 {q(.5):7.2f}  p90 {q(.9):7.2f}  max {col[-1]:7.2f}")
        rows.append(per)
    print(f"median per-launch {statistics.median(rows):.2f} us")


if __name__ == "__main__":
    main()

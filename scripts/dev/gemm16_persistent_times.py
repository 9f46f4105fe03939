"""(Ran against commit 68449ff, which had k_gemm16_4e and qz_gemm_16bit_persistent; both removed after
the measurement, profiles/r5_gemm16_persistent_times.txt.)  Config #4 shapes (T = 16384): qz_gemm_16bit (k_gemm16_4d) vs its persistent epilogue-overlap twin
(k_gemm16_4e) vs F.linear (hipBLASLt) on the same fp16 operands; outputs of the two kernels compared."""
import torch
import torch.nn.functional as F

from quantizations_amd import _lib


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / it


dev = torch.device("cuda")
T = 16384
for M, K in ((4096, 4096), (14336, 4096), (4096, 14336)):
    X = torch.randn(T, K, device=dev).half()
    W = (torch.randn(M, K, device=dev) * 0.02).half()
    Y1 = torch.empty(T, M, device=dev, dtype=torch.float16)
    Y2 = torch.empty_like(Y1)
    st = torch.cuda.current_stream().cuda_stream
    f1 = lambda: _lib.check(_lib.lib.qz_gemm_16bit(T, M, K, X.data_ptr(), K, 0, W.data_ptr(), None, Y1.data_ptr(), M, st), "4d")
    f2 = lambda: _lib.check(_lib.lib.qz_gemm_16bit_persistent(T, M, K, X.data_ptr(), K, 0, W.data_ptr(), None, Y2.data_ptr(), M, st), "4e")
    f3 = lambda: F.linear(X, W)
    fl = 2.0 * T * M * K
    r = {}
    for rep in range(2):
        for name, f in (("4d", f1), ("4e", f2), ("hipBLASLt", f3)):
            t = timeit(f)
            r.setdefault(name, []).append(fl / t / 1e6)
    f1(); f2(); torch.cuda.synchronize()
    same = torch.equal(Y1, Y2)
    print(f"{M}x{K} T={T}: " + ", ".join(f"{n} {'/'.join(f'{v:.0f}' for v in vs)} TF/s" for n, vs in r.items())
          + f"; 4e == 4d: {same}", flush=True)
    del X, W, Y1, Y2

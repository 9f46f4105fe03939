"""lm_head shapes (128256 x 4096 / 8192, fp16 and bf16): F.linear (hipBLASLt) vs qz_gemv_dense vs the
nt read floor of the same bytes; relative error of both against an fp64 product."""
import torch
import torch.nn.functional as F

from quantizations_amd import _lib


def timeit(fn, it=40):
    for _ in range(5):
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
sink = torch.zeros(64, dtype=torch.int32, device=dev)
for K in (4096, 8192):
    for dt in (torch.float16, torch.bfloat16):
        M = 128256
        W = (torch.randn(M, K, device=dev) * 0.02).to(dt)
        x = torch.randn(1, 1, K, device=dev).to(dt)
        y = torch.empty(M, device=dev, dtype=dt)
        st = torch.cuda.current_stream().cuda_stream
        code = _lib.dtype_code(dt)
        ours = lambda: _lib.check(_lib.lib.qz_gemv_dense(M, K, x.data_ptr(), code, W.data_ptr(), y.data_ptr(), st), "dense")
        lib = lambda: F.linear(x, W)
        floor = lambda: _lib.lib.qz_bench_read_floor(W.data_ptr(), M * K * 2, sink.data_ptr(), st)
        t_o, t_l, t_f = timeit(ours), timeit(lib), timeit(floor)
        ref = (W.double() @ x.view(-1).double())
        yl = lib().view(-1)
        ours(); torch.cuda.synchronize()
        e_o = ((y.double() - ref).norm() / ref.norm()).item()
        e_l = ((yl.double() - ref).norm() / ref.norm()).item()
        diff = (y != yl).float().mean().item()
        am = (y.float().argmax().item(), yl.float().argmax().item())
        gb = M * K * 2 / 1e9
        print(f"K={K} {str(dt)[6:]}: ours {t_o:.1f} us ({gb / t_o * 1e6 / 1e3:.2f} TB/s)  hipBLASLt {t_l:.1f} us "
              f"({gb / t_l * 1e6 / 1e3:.2f})  nt read floor {t_f:.1f} us ({gb / t_f * 1e6 / 1e3:.2f}); rel err ours "
              f"{e_o:.2e} lib {e_l:.2e}; outputs differing {diff:.4f}; argmax {am}", flush=True)
        del W

import os, sys, torch
sys.path.insert(0, os.getcwd())
from quantizations_amd.core import gemm_16bit
dev = torch.device("cuda")
for (T, M, K) in [(256, 256, 64), (256, 256, 128), (256, 256, 256), (512, 256, 4096), (4096, 4096, 4096)]:
    torch.manual_seed(0)
    x = torch.randn(T, K, device=dev, dtype=torch.float16)
    W = (torch.randn(M, K, device=dev) * 0.02).half()
    y = gemm_16bit(x, W)
    ref = x.double() @ W.double().t()
    bad = ~torch.isfinite(y)
    err = (y.double() - ref).abs()
    print(T, M, K, "nonfinite", int(bad.sum()), "maxerr", float(err[~bad].max()) if (~bad).any() else None,
          "rel", float(((y.double() - ref).norm() / ref.norm())))
    if bad.any():
        idx = bad.nonzero()
        print("  bad rows(t)", sorted(set(idx[:, 0].tolist()))[:20], "cols(m)", sorted(set(idx[:, 1].tolist()))[:20])
    big = err > 1e-2
    if big.any():
        idx = big.nonzero()
        print("  err rows(t)", sorted(set(idx[:, 0].tolist()))[:16], "cols(m)", sorted(set(idx[:, 1].tolist()))[:16], int(big.sum()))

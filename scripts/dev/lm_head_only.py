"""One qz_gemv_dense launch per iteration at the Llama-3-8B lm_head shape (128256 x 4096 fp16), for
rocprofv3 passes (kernel trace / FETCH_SIZE / WRITE_SIZE): does the launch move its 1.05 GB once?"""
import torch

from quantizations_amd.layer_ops import gemv_dense

dev = torch.device("cuda")
W = (torch.randn(128256, 4096, device=dev) * 0.02).half()
x = torch.randn(1, 1, 4096, device=dev).half()
for _ in range(20):
    y = gemv_dense(x, W)
torch.cuda.synchronize()
print("ok", float(y.float().abs().sum()))

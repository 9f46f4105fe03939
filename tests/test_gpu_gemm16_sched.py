"""GPU: every k_gemm16_4d schedule qz_gemm_16bit can launch (QZ_GEMM16_SCHED: the split-release
step schedule, the permuted-W-row register epilogue, the unstaged last steps, the asm step, the persistent form) gives the SAME bits as
schedule 0, which test_gpu_edges.py checks against fp64 of the bit-exact dequantised weight (each
output element sums its k products in the same order under every schedule; only the issue order of
the LDS reads / DMAs and the epilogue path differ).  Ragged T and M tiles, 1-4-step K loops, bias,
fp16 and bf16."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda")
# 512 |: the persistent k_gemm16_4q (one workgroup per CU, the next tile's steps 0 / 1 staged by the
# last two steps of a tile) where K / 64 is even, else the non-persistent schedule; 963 = 707 | 256:
# W's k-half 1 fragments read (and its image refilled) before X's; 971 = 963 | 8: non-temporal stores
SCHEDS = [1, 2, 3, 9, 11, 25, 27, 65, 67, 193, 195, 579, 707, 963, 971]


@pytest.fixture
def sched_knob():
    from quantizations_amd import _lib

    before = _lib.gemv_knobs().get("QZ_GEMM16_SCHED", 971)
    yield lambda s: _lib.set_gemv_knob("QZ_GEMM16_SCHED", s)
    _lib.set_gemv_knob("QZ_GEMM16_SCHED", before)


@pytest.mark.parametrize("T,M,K", [(4096, 1024, 4096), (4100, 1032, 256), (300, 264, 192), (37, 264, 64),
                                   (257, 1032, 128), (1, 8, 64), (512, 520, 4160),
                                   # > 256 tiles: persistent workgroups walk 2 tiles (grouped order; ragged)
                                   (8192, 4096, 128), (4100, 4104, 256)])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm16_schedules_bit_identical(sched_knob, T, M, K, dtype, bias):
    from quantizations_amd.core import gemm_16bit

    g = torch.Generator(device="cuda").manual_seed(T * 7 + M + K)
    W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(dtype)
    X = torch.randn(T, K, device=DEV, generator=g).to(dtype)
    bv = (torch.randn(M, device=DEV, generator=g) * 0.1).to(dtype) if bias else None
    sched_knob(0)
    ref = gemm_16bit(X, W, bv)
    assert ref is not None
    wd = W.double()
    exp = X.double() @ wd.t() + (bv.double() if bias else 0.0)
    rel = ((ref.double() - exp).norm() / exp.norm()).item()
    assert rel <= (1e-3 if dtype == torch.float16 else 4e-3)
    for s in SCHEDS:
        sched_knob(s)
        y = gemm_16bit(X, W, bv)
        torch.cuda.synchronize()
        ndiff = int((y != ref).sum().item())
        assert ndiff == 0, f"schedule {s}: {ndiff} of {y.numel()} outputs differ from schedule 0"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("T,M,K", [(4096, 1024, 4096), (300, 264, 256), (8192, 4096, 128)])
def test_gemm16_strided_activation_rows(sched_knob, T, M, K, dtype):
    """X as a column slice of a wider tensor (row stride K + 64, the C-ABI's ldx > K): the DMA
    offsets of the default persistent schedule and of schedule 0 give the same bits as on the
    contiguous copy."""
    from quantizations_amd.core import gemm_16bit

    g = torch.Generator(device="cuda").manual_seed(T + M + K)
    W = (torch.randn(M, K, device=DEV, generator=g) * 0.02).to(dtype)
    Xw = torch.randn(T, K + 64, device=DEV, generator=g).to(dtype)
    X = Xw[:, :K]
    assert X.stride(0) == K + 64
    for s in (0, 971):
        sched_knob(s)
        y_strided = gemm_16bit(X, W)
        y_contig = gemm_16bit(X.contiguous(), W)
        torch.cuda.synchronize()
        assert torch.equal(y_strided, y_contig), f"schedule {s}"

"""The C-ABI library: loads without a GPU and exports exactly what
include/quantizations.h declares (no compute calls here)."""
import ctypes
import os
import re
import subprocess

from conftest import REPO

HEADER = os.path.join(REPO, "include", "quantizations.h")
LIB = os.path.join(REPO, "quantizations_amd", "libquantizations.so")

REFERENCE_FIVE = ["cgemm_4bit_inference_naive_fp32", "cquantize_blockwise_fp16_fp4", "cdequantize_blockwise_fp16_fp4",
                  "cquantize_blockwise_fp32", "cdequantize_blockwise_fp32"]  # pythonInterface.cpp:154-164


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|long long)\s+\**\s*(\w+)\s*\(", src, flags=re.M)))


def test_header_declares_reference_names():
    names = declared()
    for n in REFERENCE_FIVE:
        assert n in names and n + "_stream" in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: __graft_entry__.build()"
    lib = ctypes.CDLL(LIB)
    for n in declared():
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, flags=re.M))
    assert set(declared()) <= exported
    # extern "C": no mangled duplicates of the reference names
    assert not any(n.startswith("_Z") and "cgemm_4bit" in n for n in exported)


def test_python_binding_matches_header():
    from quantizations_amd import _lib

    assert sorted(_lib.SIGNATURES) == declared()


def test_version_callable_without_gpu():
    from quantizations_amd import _lib

    assert _lib.lib.qz_version() == 100
    assert _lib.lib.qz_absmax_mean_workspace(262144) == 256


def test_argument_errors_are_reported_not_launched():
    # null pointers / bad blocksize are rejected before any HIP call
    from quantizations_amd import _lib

    L = _lib.lib
    assert L.qz_quantize_4bit(0, 0, 64, 64, 0, 0, 0, 0) == -1
    assert L.qz_quantize_4bit(1, 0, 64, 48, 0, 1, 1, 0) == -2
    assert L.qz_quantize_4bit(1, 9, 64, 64, 0, 1, 1, 0) == -4
    assert L.qz_gemv_4bit(4, 64, 1, 0, 1, 0, 64, 1, 1, 1, 1, 1, 256, 0, 0, 0, 1, 0) == -1  # both scale sources
    assert L.cgemm_4bit_inference_naive_fp32(8, 2, 64, 1, 1, 1, 1, 1, 8, 32, 8, 64) == -3  # n != 1
    # layer ops: negative sizes / odd head_dim are rejected before any launch
    assert L.qz_rmsnorm(1, 0, -1, 64, 64, 1, 1e-6, 1, 64, 0) == -1
    assert L.qz_rmsnorm(1, 0, 4, 64, 32, 1, 1e-6, 1, 64, 0) == -1  # ldx < K
    assert L.qz_rmsnorm(1, 0, 0, 64, 64, 1, 1e-6, 1, 64, 0) == 0    # empty: nothing to do
    s3 = (ctypes.c_longlong * 3)(0, 0, 0)
    s2 = (ctypes.c_longlong * 2)(0, 0)
    assert L.qz_rope_qk(0, 1, 1, 127, 1, 1, s3, 1, s3, 1, 1, s3, 1, s3, 1, 1, s2, 0) == -3
    assert L.qz_rope_qk(0, 1, 1, 128, 1, 1, s3, 1, s3, 1, 1, s3, 1, s3, 0, 1, s2, 0) == -1
    assert L.qz_silu_mul(1, 1, 0, -1, 1, 0) == -1
    assert L.qz_silu_mul(0, 1, 0, 16, 1, 0) == -1
    assert L.qz_silu_mul(1, 1, 9, 16, 1, 0) == -4
    assert L.qz_add_rmsnorm(1, 0, 0, 4, 64, 64, 1, 1e-6, 1, 1, 64, 0) == -1  # residual required
    assert L.qz_add_rmsnorm(1, 1, 0, 4, 64, 64, 1, 1e-6, 0, 1, 64, 0) == -1  # sum output required


def test_gemm16_and_gemm4_guards_without_gpu():
    # qz_gemm_16bit_ok is a pure host check; shape/dtype/null errors return before any launch
    from quantizations_amd import _lib

    L = _lib.lib
    assert L.qz_gemm_16bit_ok(256, 256, 4096, 16, 4096, 16, 16, 256) == 1
    assert L.qz_gemm_16bit_ok(256, 256, 4100, 16, 4100, 16, 16, 256) == 0   # K % 64
    assert L.qz_gemm_16bit_ok(256, 260, 4096, 16, 4096, 16, 16, 260) == 0   # M % 8
    assert L.qz_gemm_16bit_ok(256, 256, 4096, 8, 4096, 16, 16, 256) == 0    # X not 16-B aligned
    assert L.qz_gemm_16bit_ok(256, 256, 4096, 16, 4000, 16, 16, 256) == 0   # ldx < K
    assert L.qz_gemm_16bit(1, 8, 100, 16, 100, 1, 16, 0, 16, 8, 0) == -3    # K % 64: shape error
    assert L.qz_gemm_16bit(1, 8, 64, 16, 64, 7, 16, 0, 16, 8, 0) == -4      # dtype
    assert L.qz_gemm_16bit(1, 8, 64, 0, 64, 1, 16, 0, 16, 8, 0) == -1       # null X
    assert L.qz_gemm_16bit(0, 8, 64, 16, 64, 1, 16, 0, 16, 8, 0) == 0       # empty: nothing to do

// dequantize.hip -- 4-bit -> fp16/bf16/fp32 and 8-bit blockwise dequantisation.
//
// 4-bit: reference kernels.cu:554-560 (FP4 through dDequantizeFP4Tree, so the
// zero code 8 gives -0.0) and the NF4 codebook; the per-block scale comes
// either from an fp32 absmax or, fused, from the double-quantised statistics
// (core.py:613-617 without the intermediate fp32 absmax tensor).
// 8-bit: kernels.cu:549-553 (+ core.py:468 offset when given).
// Both are HBM-streaming kernels: 16 B/lane loads, 16-32 B/lane stores.
#include "common.h"

namespace qz {

template <int QT, int ODT>
__global__ __launch_bounds__(256) void k_dequantize_4bit(const unsigned char *__restrict__ A, long long n,
                                                         int blocksize, ScaleSrc sc, void *__restrict__ out) {
  // each thread: 8 packed bytes = 16 elements, all inside one scale block
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long e0 = t * 16;
  if (e0 >= n) return;
  const long long blk = e0 / blocksize;
  const float am = sc.qabsmax ? dq_scale(sc, blk, *sc.offset) : sc.absmax[blk];
  const long long nbytes = (n + 1) >> 1;
  uint32_t w[2];
  if (e0 + 16 <= n) {
    const uint2 v = *reinterpret_cast<const uint2 *>(A + (e0 >> 1));
    w[0] = v.x;
    w[1] = v.y;
  } else {
    unsigned char b[8];
    for (int j = 0; j < 8; ++j) b[j] = ((e0 >> 1) + j) < nbytes ? A[(e0 >> 1) + j] : 0;
    w[0] = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
    w[1] = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
  }
  float v[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t byte = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
    const uint32_t hi = byte >> 4, lo = byte & 0xFu;
    if constexpr (QT == QZ_NF4) {
      v[2 * j] = __fmul_rn(kNF4[hi], am);
      v[2 * j + 1] = __fmul_rn(kNF4[lo], am);
    } else {
      v[2 * j] = dequant_fp4_tree(hi, am);
      v[2 * j + 1] = dequant_fp4_tree(lo, am);
    }
  }
  if (e0 + 16 <= n) {
    if constexpr (ODT == QZ_DT_F32) {
      float4 *o = reinterpret_cast<float4 *>(reinterpret_cast<float *>(out) + e0);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    } else {
      uint32_t pk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (ODT == QZ_DT_F16) {
          pk[j] = cvt_pk_f16_rne(v[2 * j], v[2 * j + 1]);
        } else {
          const uint16_t a = __bfloat16_as_ushort(__float2bfloat16(v[2 * j]));
          const uint16_t b = __bfloat16_as_ushort(__float2bfloat16(v[2 * j + 1]));
          pk[j] = (uint32_t)a | ((uint32_t)b << 16);
        }
      }
      uint4 *o = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(out) + e0);
      o[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      o[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    }
  } else {
    for (int j = 0; j < 16 && e0 + j < n; ++j) store_f32<ODT>(out, e0 + j, v[j]);
  }
}

__global__ __launch_bounds__(256) void k_dequantize_8bit(const float *__restrict__ code,
                                                         const unsigned char *__restrict__ A,
                                                         const float *__restrict__ absmax, long long n, int blocksize,
                                                         const float *__restrict__ offset, float *__restrict__ out) {
  __shared__ float smem_code[256];
  smem_code[threadIdx.x] = code[threadIdx.x];
  __syncthreads();
  const float off = offset ? *offset : 0.0f;
  const long long e0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e0 >= n) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long long e = e0 + j;
    if (e < n) {
      float v = __fmul_rn(smem_code[A[e]], absmax[e / blocksize]);
      if (offset) v = __fadd_rn(v, off);
      out[e] = v;
    }
  }
}

}  // namespace qz

using namespace qz;

extern "C" int qz_dequantize_4bit(const unsigned char *A, long long n, int quant_type, int blocksize,
                                  const float *absmax, const unsigned char *qabsmax, const float *absmax2,
                                  const float *code2, const float *offset, int blocksize2, void *out, int out_dtype,
                                  void *stream) {
  if (!A || !out || n < 0) return QZ_ERR_ARG;
  if (!valid_blocksize(blocksize)) return QZ_ERR_BLOCKSIZE;
  if ((absmax == nullptr) == (qabsmax == nullptr)) return QZ_ERR_ARG;
  if (qabsmax && (!absmax2 || !code2 || !offset || blocksize2 <= 0)) return QZ_ERR_ARG;
  if (quant_type != QZ_FP4 && quant_type != QZ_NF4) return QZ_ERR_DTYPE;
  if (n == 0) return QZ_OK;
  ScaleSrc sc{absmax, qabsmax, absmax2, code2, offset, blocksize2};
  const long long threads = (n + 15) / 16;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
#define QZ_DQ4(QT, ODT) hipLaunchKernelGGL((k_dequantize_4bit<QT, ODT>), grid, dim3(256), 0, s, A, n, blocksize, sc, out)
  if (quant_type == QZ_FP4) {
    switch (out_dtype) {
      case QZ_DT_F16: QZ_DQ4(QZ_FP4, QZ_DT_F16); break;
      case QZ_DT_BF16: QZ_DQ4(QZ_FP4, QZ_DT_BF16); break;
      case QZ_DT_F32: QZ_DQ4(QZ_FP4, QZ_DT_F32); break;
      default: return QZ_ERR_DTYPE;
    }
  } else {
    switch (out_dtype) {
      case QZ_DT_F16: QZ_DQ4(QZ_NF4, QZ_DT_F16); break;
      case QZ_DT_BF16: QZ_DQ4(QZ_NF4, QZ_DT_BF16); break;
      case QZ_DT_F32: QZ_DQ4(QZ_NF4, QZ_DT_F32); break;
      default: return QZ_ERR_DTYPE;
    }
  }
#undef QZ_DQ4
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" int qz_dequantize_blockwise_8bit(const float *code, const unsigned char *A, const float *absmax,
                                            long long n, int blocksize, const float *offset, float *out,
                                            void *stream) {
  if (!code || !A || !absmax || !out || n < 0) return QZ_ERR_ARG;
  if (!valid_blocksize(blocksize)) return QZ_ERR_BLOCKSIZE;
  if (n == 0) return QZ_OK;
  const long long threads = (n + 3) / 4;
  hipLaunchKernelGGL(k_dequantize_8bit, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     code, A, absmax, n, blocksize, offset, out);
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

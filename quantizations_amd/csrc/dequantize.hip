// dequantize.hip -- 4-bit -> fp16/bf16/fp32 and 8-bit blockwise dequantisation.
//
// 4-bit: reference kernels.cu:554-560 (FP4 through dDequantizeFP4Tree, so the
// zero code 8 gives -0.0) and the NF4 codebook; the per-block scale comes
// either from an fp32 absmax or, fused, from the double-quantised statistics
// (core.py:613-617 without the intermediate fp32 absmax tensor).
// 8-bit: kernels.cu:549-553 (+ core.py:468 offset when given).
// Both are HBM-streaming kernels.  4-bit: 32 codes per thread (one 16-B
// load, 64-B fp16/bf16 or 128-B fp32 stores); for 16-bit outputs the codes go
// through the per-block table of exact weights fp16/bf16(code * absmax)
// (decode.h, shared with the fused GEMM), so each weight costs a few v_perm
// instead of a product and a convert.
#include "common.h"
#include "decode.h"

namespace qz {

typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));

template <int QT, int ODT>
__global__ __launch_bounds__(256) void k_dequantize_4bit_v32(const unsigned char *__restrict__ A, long long n,
                                                             int bs_log2, ScaleSrc sc, int bs2_log2,
                                                             void *__restrict__ out) {
  // thread t: elements [32 t, 32 t + 32) -- always inside one scale block (blocksize >= 32)
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long e0 = t * 32;
  // every thread of the workgroup has 32 in-range codes: the LDS-transposed store path (uniform branch)
  const bool full_block = ((long long)blockIdx.x + 1) * 256 * 32 <= n;
  if (e0 >= n) return;
  const long long blk = e0 >> bs_log2;
  float am;
  if (sc.qabsmax) am = __fadd_rn(__fmul_rn(sc.code2[sc.qabsmax[blk]], sc.absmax2[blk >> bs2_log2]), *sc.offset);
  else am = sc.absmax[blk];
  if (e0 + 32 <= n) {
    const v4u_t wv = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(A + (e0 >> 1)));
    const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
    if constexpr (ODT == QZ_DT_F32) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t byte = (w[d] >> (8 * j)) & 0xFFu;
          const uint32_t hi = byte >> 4, lo = byte & 0xFu;
          if constexpr (QT == QZ_NF4) {
            v[2 * j] = __fmul_rn(kNF4[hi], am);
            v[2 * j + 1] = __fmul_rn(kNF4[lo], am);
          } else {
            v[2 * j] = dequant_fp4_tree(hi, am);
            v[2 * j + 1] = dequant_fp4_tree(lo, am);
          }
        }
        v4u_t *o = reinterpret_cast<v4u_t *>(reinterpret_cast<float *>(out) + e0 + 8 * d);
        o[0] = v4u_t{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
        o[1] = v4u_t{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])};
      }
    } else {
      uint32_t tab[8];
      block_table<QT, ODT>(am, tab);
      v4u_t v[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t N[4];
        decode_codes_natural(w[d], tab, N);
        v[d] = v4u_t{N[0], N[1], N[2], N[3]};
      }
      if (full_block) {
        // transpose through LDS so each store instruction writes 1 KiB contiguous per wave
        __shared__ v4u_t s_out[256 * 4];
#pragma unroll
        for (int d = 0; d < 4; ++d) s_out[threadIdx.x * 4 + d] = v[d];
        __syncthreads();
        v4u_t *o = reinterpret_cast<v4u_t *>(reinterpret_cast<uint16_t *>(out) + (long long)blockIdx.x * 256 * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i * 256 + threadIdx.x] = s_out[i * 256 + threadIdx.x];
      } else {
        v4u_t *o = reinterpret_cast<v4u_t *>(reinterpret_cast<uint16_t *>(out) + e0);
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = v[d];
      }
    }
    return;
  }
  // ragged tail (n % 32 != 0): element by element, reference indexing
  for (long long e = e0; e < n; ++e) {
    const uint32_t byte = A[e >> 1];
    const uint32_t nib = (e & 1) ? (byte & 0xFu) : (byte >> 4);
    float v;
    if constexpr (QT == QZ_NF4) v = __fmul_rn(kNF4[nib], am);
    else v = dequant_fp4_tree(nib, am);
    store_f32<ODT>(out, e, v);
  }
}

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
  hipStream_t s = (hipStream_t)stream;
  int bs2l = 0;
  if (qabsmax) {
    while ((1 << bs2l) < blocksize2) ++bs2l;
    if ((1 << bs2l) != blocksize2) return QZ_ERR_BLOCKSIZE;
  }
  int bsl = 0;
  while ((1 << bsl) < blocksize) ++bsl;
  const bool wide = (reinterpret_cast<uintptr_t>(A) % 16) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0;
  if (wide) {  // 32 codes per thread, table decode
    const long long threads = (n + 31) / 32;
    const dim3 grid((unsigned)((threads + 255) / 256));
#define QZ_DQ32(QT, ODT) \
  hipLaunchKernelGGL((k_dequantize_4bit_v32<QT, ODT>), grid, dim3(256), 0, s, A, n, bsl, sc, bs2l, out)
    if (quant_type == QZ_FP4) {
      switch (out_dtype) {
        case QZ_DT_F16: QZ_DQ32(QZ_FP4, QZ_DT_F16); break;
        case QZ_DT_BF16: QZ_DQ32(QZ_FP4, QZ_DT_BF16); break;
        case QZ_DT_F32: QZ_DQ32(QZ_FP4, QZ_DT_F32); break;
        default: return QZ_ERR_DTYPE;
      }
    } else {
      switch (out_dtype) {
        case QZ_DT_F16: QZ_DQ32(QZ_NF4, QZ_DT_F16); break;
        case QZ_DT_BF16: QZ_DQ32(QZ_NF4, QZ_DT_BF16); break;
        case QZ_DT_F32: QZ_DQ32(QZ_NF4, QZ_DT_F32); break;
        default: return QZ_ERR_DTYPE;
      }
    }
#undef QZ_DQ32
    QZ_LAUNCH_CHECK();
    return QZ_OK;
  }
  const long long threads = (n + 15) / 16;
  const dim3 grid((unsigned)((threads + 255) / 256));
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

// quantize.hip -- load-time quantisation kernels for gfx950.
//
//  * 4-bit blockwise pack (FP4 / NF4), reference kernels.cu:340-478 (FP4 case)
//  * deterministic fp64 mean of the block absmax (core.py:563, fixed order)
//  * 8-bit blockwise quantisation with the dynamic code (double quant,
//    kernels.cu:340-478 General8bit + kernels.cu:166-237 dQuantize)
//
// All are byte/integer-exact against oracle/oracle.c: the decision trees use
// fp32 compares, scales are 1.0f/amax (correctly rounded: hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt), products are __fmul_rn.
#include "common.h"

namespace qz {

// Max over `tpb` consecutive threads (tpb a power of two <= 256); every thread
// of the group receives the result.  `red` is >= 4 floats of LDS.
__device__ __forceinline__ float group_max(float v, int tpb, float *red) {
  const int lim = tpb < kWave ? tpb : kWave;
  for (int off = 1; off < lim; off <<= 1) v = fmaxf(v, __shfl_xor(v, off));
  if (tpb > kWave) {
    const int wave = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) red[wave] = v;
    __syncthreads();
    const int wpg = tpb / kWave;  // waves per group (2 or 4)
    const int g0 = (wave / wpg) * wpg;
    v = red[g0];
    for (int w = 1; w < wpg; ++w) v = fmaxf(v, red[g0 + w]);
    __syncthreads();
  }
  return v;
}

// ---------------------------------------------------------------------------
// 4-bit pack.  Each thread owns BPT output bytes (2*BPT consecutive inputs);
// TPB = min(blocksize/2/BPT, 256) threads share one quantisation block.
// ---------------------------------------------------------------------------
template <int DT, int QT>
__global__ __launch_bounds__(256) void k_quantize_4bit(const void *__restrict__ A, long long n, int blocksize,
                                                       int bpt, float *__restrict__ absmax,
                                                       unsigned char *__restrict__ out) {
  __shared__ float red[4];
  const int tpb = blocksize / 2 / bpt;
  const int blocks_per_wg = 256 / tpb;
  const long long qblock = (long long)blockIdx.x * blocks_per_wg + threadIdx.x / tpb;
  const int tig = threadIdx.x % tpb;
  const long long start = qblock * blocksize;

  // every thread of the workgroup takes part in the reduction (no early exit)
  float m = -3.402823466e+38f;
  for (int j = 0; j < 2 * bpt; ++j) {
    const long long e = start + (long long)tig * 2 * bpt + j;
    const float v = e < n ? load_f32<DT>(A, e) : 0.0f;  // BlockLoad pads with 0 (kernels.cu:410)
    m = fmaxf(m, fabsf(v));
  }
  m = group_max(m, tpb, red);
  if (start >= n) return;
  if (tig == 0) absmax[qblock] = m;
  const float s = 1.0f / m;
  for (int j = 0; j < bpt; ++j) {
    const long long e = start + (long long)tig * 2 * bpt + 2 * j;
    if (e >= n) break;
    const float x0 = __fmul_rn(load_f32<DT>(A, e), s);
    const float x1 = __fmul_rn(e + 1 < n ? load_f32<DT>(A, e + 1) : 0.0f, s);
    uint32_t q0, q1;
    if constexpr (QT == QZ_NF4) {
      q0 = quantize_nf4(x0);
      q1 = quantize_nf4(x1);
    } else {
      q0 = quantize_fp4(x0);
      q1 = quantize_fp4(x1);
    }
    out[e >> 1] = (unsigned char)((q0 << 4) | q1);  // high nibble = even element (kernels.cu:467)
  }
}

// ---------------------------------------------------------------------------
// dQuantize<0> (kernels.cu:183-237) over the LDS copy of the sorted code.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t quantize_8bit(const float *code, float x) {
  int pivot = 127, upper_pivot = 255, lower_pivot = 0;
  float lower = -1.0f, upper = 1.0f;
  float val = code[pivot];
  for (int i = 64; i > 0; i >>= 1) {
    if (x > val) {
      lower_pivot = pivot;
      lower = val;
      pivot += i;
    } else {
      upper_pivot = pivot;
      upper = val;
      pivot -= i;
    }
    val = code[pivot];
  }
  if (upper_pivot == 255) upper = code[upper_pivot];
  if (lower_pivot == 0) lower = code[lower_pivot];
  if (x > val) {
    const float mid = __fmul_rn(__fadd_rn(upper, val), 0.5f);
    return x > mid ? upper_pivot : pivot;
  }
  const float mid = __fmul_rn(__fadd_rn(lower, val), 0.5f);
  return x < mid ? lower_pivot : pivot;
}

// 8-bit blockwise quantisation; EPT elements per thread, TPB = blocksize/EPT.
__global__ __launch_bounds__(256) void k_quantize_8bit(const float *__restrict__ code, const float *__restrict__ A,
                                                       long long n, int blocksize, int ept,
                                                       const float *__restrict__ subtract,
                                                       float *__restrict__ absmax, unsigned char *__restrict__ out) {
  __shared__ float smem_code[256];
  __shared__ float red[4];
  smem_code[threadIdx.x] = code[threadIdx.x];
  const float off = subtract ? *subtract : 0.0f;
  const int tpb = blocksize / ept;
  const int blocks_per_wg = 256 / tpb;
  const long long qblock = (long long)blockIdx.x * blocks_per_wg + threadIdx.x / tpb;
  const int tig = threadIdx.x % tpb;
  const long long start = qblock * blocksize;
  float m = -3.402823466e+38f;
  for (int j = 0; j < ept; ++j) {
    const long long e = start + (long long)tig * ept + j;
    float v = 0.0f;
    if (e < n) v = subtract ? __fsub_rn(A[e], off) : A[e];
    m = fmaxf(m, fabsf(v));
  }
  __syncthreads();  // smem_code visible
  m = group_max(m, tpb, red);
  if (start >= n) return;
  if (tig == 0) absmax[qblock] = m;
  const float s = 1.0f / m;
  for (int j = 0; j < ept; ++j) {
    const long long e = start + (long long)tig * ept + j;
    if (e >= n) break;
    const float v = subtract ? __fsub_rn(A[e], off) : A[e];
    out[e] = (unsigned char)quantize_8bit(smem_code, __fmul_rn(v, s));
  }
}

// ---------------------------------------------------------------------------
// Deterministic mean (oracle.c orc_absmax_mean): fp64, chunks of 1024 summed
// by 256 lanes (4 sequential adds each) and a halving tree; chunk sums again.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double tree256(double v, double *s) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (int stride = 128; stride > 0; stride >>= 1) {
    if ((int)threadIdx.x < stride) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + stride];
    __syncthreads();
  }
  return s[0];
}

__global__ __launch_bounds__(256) void k_mean_partial(const float *__restrict__ a, long long n,
                                                      double *__restrict__ partial) {
  __shared__ double s[256];
  const long long base = (long long)blockIdx.x * 1024;
  double acc = 0.0;
  for (int j = 0; j < 4; ++j) {
    const long long idx = base + j * 256 + threadIdx.x;
    if (idx < n) acc = acc + (double)a[idx];
  }
  const double tot = tree256(acc, s);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_mean_final(const double *__restrict__ partial, long long nc, long long n,
                                                    float *__restrict__ offset) {
  __shared__ double s[256];
  double acc = 0.0;
  for (long long idx = threadIdx.x; idx < nc; idx += 256) acc = acc + partial[idx];
  const double tot = tree256(acc, s);
  if (threadIdx.x == 0) *offset = (float)(tot / (double)n);
}

}  // namespace qz

using namespace qz;

extern "C" int qz_quantize_4bit(const void *A, int a_dtype, long long n, int blocksize, int quant_type, float *absmax,
                                unsigned char *out, void *stream) {
  if (!A || !absmax || !out || n < 0) return QZ_ERR_ARG;
  if (!valid_blocksize(blocksize)) return QZ_ERR_BLOCKSIZE;
  if (quant_type != QZ_FP4 && quant_type != QZ_NF4) return QZ_ERR_DTYPE;
  if (n == 0) return QZ_OK;
  const int bpt = blocksize / 2 > 256 ? blocksize / 512 : 1;
  const int tpb = blocksize / 2 / bpt;
  const long long nblocks = (n + blocksize - 1) / blocksize;
  const long long grid = (nblocks + (256 / tpb) - 1) / (256 / tpb);
  hipStream_t s = (hipStream_t)stream;
#define QZ_Q4(DT, QT) \
  hipLaunchKernelGGL((k_quantize_4bit<DT, QT>), dim3((unsigned)grid), dim3(256), 0, s, A, n, blocksize, bpt, absmax, out)
  if (quant_type == QZ_FP4) {
    switch (a_dtype) {
      case QZ_DT_F16: QZ_Q4(QZ_DT_F16, QZ_FP4); break;
      case QZ_DT_BF16: QZ_Q4(QZ_DT_BF16, QZ_FP4); break;
      case QZ_DT_F32: QZ_Q4(QZ_DT_F32, QZ_FP4); break;
      default: return QZ_ERR_DTYPE;
    }
  } else {
    switch (a_dtype) {
      case QZ_DT_F16: QZ_Q4(QZ_DT_F16, QZ_NF4); break;
      case QZ_DT_BF16: QZ_Q4(QZ_DT_BF16, QZ_NF4); break;
      case QZ_DT_F32: QZ_Q4(QZ_DT_F32, QZ_NF4); break;
      default: return QZ_ERR_DTYPE;
    }
  }
#undef QZ_Q4
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" long long qz_absmax_mean_workspace(long long n) { return n <= 0 ? 1 : (n + 1023) / 1024; }

extern "C" int qz_absmax_mean(const float *absmax, long long n, double *workspace, float *offset, void *stream) {
  if (!absmax || !workspace || !offset || n <= 0) return QZ_ERR_ARG;
  const long long nc = (n + 1023) / 1024;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_mean_partial, dim3((unsigned)nc), dim3(256), 0, s, absmax, n, workspace);
  hipLaunchKernelGGL(k_mean_final, dim3(1), dim3(256), 0, s, workspace, nc, n, offset);
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" int qz_quantize_blockwise_8bit(const float *code, const float *A, long long n, int blocksize,
                                          const float *subtract, float *absmax, unsigned char *out, void *stream) {
  if (!code || !A || !absmax || !out || n < 0) return QZ_ERR_ARG;
  if (!valid_blocksize(blocksize)) return QZ_ERR_BLOCKSIZE;
  if (n == 0) return QZ_OK;
  const int ept = blocksize > 256 ? blocksize / 256 : 1;
  const int tpb = blocksize / ept;
  const long long nblocks = (n + blocksize - 1) / blocksize;
  const long long grid = (nblocks + (256 / tpb) - 1) / (256 / tpb);
  hipLaunchKernelGGL(k_quantize_8bit, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, code, A, n, blocksize,
                     ept, subtract, absmax, out);
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

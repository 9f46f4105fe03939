// gemm.hip -- fused 4-bit dequantise + MFMA GEMM for batched prefill on gfx950.
//
// Replaces the reference prefill (modules.py:62-64): a full-weight dequant
// kernel that writes M*K fp16 to HBM (kernels.cu:554-560), a cast to fp32 and
// an fp32 SGEMM (F.linear).  Here Y[T, M] = X[T, K] . W[M, K]^T (+ bias) runs
// in one kernel:
//   * a 256-thread workgroup owns a 128 (tokens) x 128 (features) output tile
//     and walks K in steps of 64 -- exactly one scale block (blocksize 64) per
//     weight row per step;
//   * the 128 x 64 weight tile arrives as 4 KiB of packed nibbles (16 B per
//     thread), is decoded in registers to the UNSCALED codebook values in fp16
//     (v_perm byte tables, as in gemv.hip) and written to LDS; X (128 x 64
//     fp16) is staged next to it; both images use a 16-B-chunk XOR swizzle so
//     the ds_read_b128 operand fetches are conflict-free;
//   * each wave computes 64 x 64 with v_mfma_f32_16x16x32_f16 into a per-step
//     accumulator, and the step result is folded into the running fp32 sum
//     with one FMA by the per-column (weight row) scale of that step -- the
//     block absmax (double quant rebuilt in kernel) times the codebook factor.
// Requires K % 64 == 0 and blocksize % 64 == 0 (every Llama shape); other
// shapes return QZ_ERR_SHAPE and the host falls back to dequant + GEMM.
#include "common.h"

namespace qz {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kBT = 128, kBM = 128, kBK = 64;

__device__ __forceinline__ uint32_t gperm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// 8 nibbles -> 4 natural-order half2 (e_2j, e_2j+1) of the unscaled codebook
// (FP4: values x12, exact; 16-entry: fp16 of the codebook).
template <int QT>
__device__ __forceinline__ void decode_nat(uint32_t w, const uint32_t (&t)[8], uint32_t (&P)[4]) {
  if constexpr (QT == QZ_FP4) {
    const uint32_t hh = gperm(t[1], t[0], (w >> 4) & 0x07070707u) | (w & 0x80808080u);
    const uint32_t hl = gperm(t[1], t[0], w & 0x07070707u) | ((w << 4) & 0x80808080u);
    P[0] = gperm(hh, hl, 0x000C040Cu);
    P[1] = gperm(hh, hl, 0x010C050Cu);
    P[2] = gperm(hh, hl, 0x020C060Cu);
    P[3] = gperm(hh, hl, 0x030C070Cu);
  } else {
    // AND-combined 8-entry lookups (see decode_lut16 in gemv.hip)
    uint32_t ah = ((w >> 4) & 0x0F0F0F0Fu) | (w & 0x80808080u);
    asm("" : "+v"(ah));
    const uint32_t bh = ah ^ 0x88888888u;
    const uint32_t lh = gperm(t[1], t[0], ah) & gperm(t[3], t[2], bh);
    const uint32_t hh = gperm(t[5], t[4], ah) & gperm(t[7], t[6], bh);
    uint32_t al = (w & 0x0F0F0F0Fu) | ((w << 4) & 0x80808080u);
    asm("" : "+v"(al));
    const uint32_t bl = al ^ 0x88888888u;
    const uint32_t ll = gperm(t[1], t[0], al) & gperm(t[3], t[2], bl);
    const uint32_t hl = gperm(t[5], t[4], al) & gperm(t[7], t[6], bl);
    const uint32_t q0 = gperm(hh, lh, 0x05010400u);  // (e0, e2)
    const uint32_t q1 = gperm(hh, lh, 0x07030602u);  // (e4, e6)
    const uint32_t q2 = gperm(hl, ll, 0x05010400u);  // (e1, e3)
    const uint32_t q3 = gperm(hl, ll, 0x07030602u);  // (e5, e7)
    P[0] = gperm(q2, q0, 0x05040100u);               // (e0, e1)
    P[1] = gperm(q2, q0, 0x07060302u);               // (e2, e3)
    P[2] = gperm(q3, q1, 0x05040100u);               // (e4, e5)
    P[3] = gperm(q3, q1, 0x07060302u);               // (e6, e7)
  }
}

// LDS image: [row][64 halfs] = 128-B rows; 16-B chunk c of row r is stored
// at chunk position c ^ ((r >> 1) & 7): the 16 rows one ds_read_b128 lane
// group touches land on 16 distinct 16-B bank slots.
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

struct GemmParams {
  const void *X;
  const unsigned char *B;
  ScaleSrc sc;
  const void *bias;
  void *Y;
  int T, M, K, ldx, ldy;
  int bs_log2, bs2_log2;
  float lut_scale;
  uint32_t tab[8];
};

template <int QT, bool DQ>
__global__ __launch_bounds__(256) void k_gemm_4bit_f16(GemmParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char s_x[kBT * 128];
  __shared__ __attribute__((aligned(16))) unsigned char s_w[kBM * 128];
  __shared__ float s_scale[kBM];
  __shared__ float s_code2[DQ ? 256 : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wt = wave >> 1, wm = wave & 1;
  const int t0 = blockIdx.y * kBT;
  const int m0 = blockIdx.x * kBM;
  const int row_bytes = p.K >> 1;

  float offset = 0.0f;
  if constexpr (DQ) {
    s_code2[tid] = p.sc.code2[tid];
    offset = *p.sc.offset;
  }
  uint32_t tab[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) tab[i] = p.tab[i];

  f4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  // weight-tile ownership: thread -> (row wr, 32-element half wh)
  const int wr = tid >> 1, wh = tid & 1;
  const int wrow = m0 + wr;
  const bool wrow_ok = wrow < p.M;
  const int fr = lane & 15, fk = lane >> 4;  // MFMA fragment row / k-group

  for (int k0 = 0; k0 < p.K; k0 += kBK) {
    // ---- issue this step's global loads ----
    v4u xv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int r = c >> 3, kc = c & 7;
      const int t = t0 + r;
      xv[i] = t < p.T ? *reinterpret_cast<const v4u *>(reinterpret_cast<const uint16_t *>(p.X) + (size_t)t * p.ldx +
                                                       k0 + 8 * kc)
                      : v4u{0u, 0u, 0u, 0u};
    }
    v4u wv = v4u{0u, 0u, 0u, 0u};
    uint32_t q = 0;
    float a = 0.0f;
    if (wrow_ok) {
      wv = __builtin_nontemporal_load(
          reinterpret_cast<const v4u *>(p.B + (size_t)wrow * row_bytes + (k0 >> 1) + 16 * wh));
      const long long b = ((long long)wrow * p.K + k0) >> p.bs_log2;
      if constexpr (DQ) {
        q = p.sc.qabsmax[b];
        a = p.sc.absmax2[b >> p.bs2_log2];
      } else {
        a = p.sc.absmax[b];
      }
    }
    __syncthreads();  // previous step's LDS reads are done; s_code2 staged

    // ---- decode W to LDS, copy X to LDS ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<v4u *>(s_x + lds_off(c >> 3, c & 7)) = xv[i];
    }
    {
      const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t P[4];
        decode_nat<QT>(w[d], tab, P);
        *reinterpret_cast<v4u *>(s_w + lds_off(wr, 4 * wh + d)) = v4u{P[0], P[1], P[2], P[3]};
      }
      if (wh == 0) {
        float am;
        if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[q], a), offset);
        else am = a;
        s_scale[wr] = wrow_ok ? am * p.lut_scale : 0.0f;
      }
    }
    __syncthreads();

    // ---- MFMA: per-step product, then scaled fold into acc ----
    f4_t part[4][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      h8_t af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const h8_t *>(s_x + lds_off(64 * wt + 16 * i + fr, 4 * kk + fk));
        bf[i] = *reinterpret_cast<const h8_t *>(s_w + lds_off(64 * wm + 16 * i + fr, 4 * kk + fk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          part[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], kk == 0 ? f4_t{0.f, 0.f, 0.f, 0.f}
                                                                                    : part[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float sc = s_scale[64 * wm + 16 * j + fr];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaf(part[i][j][r], sc, acc[i][j][r]);
    }
  }

  // ---- epilogue: C/D map col = lane & 15, row = 4 * (lane >> 4) + r ----
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + 64 * wm + 16 * j + fr;
    if (m >= p.M) continue;
    const float bv = p.bias ? __half2float(reinterpret_cast<const __half *>(p.bias)[m]) : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + 64 * wt + 16 * i + 4 * fk + r;
        if (t < p.T)
          reinterpret_cast<uint16_t *>(p.Y)[(size_t)t * p.ldy + m] = f32_to_f16_bits(acc[i][j][r] + bv);
      }
  }
}

static void gemm_tables(int quant_type, uint32_t tab[8], float *lut_scale) {
  for (int i = 0; i < 8; ++i) tab[i] = 0;
  if (quant_type == QZ_FP4) {
    const uint8_t hb[8] = {0x00, 0x2C, 0x48, 0x4A, 0x44, 0x46, 0x40, 0x42};  // fp16 hi bytes of {0,1/16,8,12,4,6,2,3}
    for (int i = 0; i < 8; ++i) tab[i >> 2] |= (uint32_t)hb[i] << (8 * (i & 3));
    *lut_scale = 1.0f / 12.0f;
    return;
  }
  static const float nf4[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                                -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                                0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                                0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                                0.7229568362236023f, 1.0f};
  for (int i = 0; i < 16; ++i) {
    const uint16_t h = __half_as_ushort(__float2half_rn(nf4[i]));
    tab[i >> 2] |= (uint32_t)(h & 0xFF) << (8 * (i & 3));
    tab[4 + (i >> 2)] |= (uint32_t)(h >> 8) << (8 * (i & 3));
  }
  *lut_scale = 1.0f;
}

static int ilog2g(long long v) {
  int l = 0;
  while ((1LL << l) < v) ++l;
  return (1LL << l) == v ? l : -1;
}

}  // namespace qz

using namespace qz;

extern "C" int qz_gemm_4bit(int T, int M, int K, const void *X, int ldx, int dtype, const unsigned char *B,
                            int quant_type, int blocksize, const float *absmax, const unsigned char *qabsmax,
                            const float *absmax2, const float *code2, const float *offset, int blocksize2,
                            const void *bias, void *Y, int ldy, void *stream) {
  if (!X || !B || !Y || T < 0 || M < 0 || K < 0) return QZ_ERR_ARG;
  if ((absmax == nullptr) == (qabsmax == nullptr)) return QZ_ERR_ARG;
  const bool dq = qabsmax != nullptr;
  if (dq && (!absmax2 || !code2 || !offset)) return QZ_ERR_ARG;
  if (quant_type != QZ_FP4 && quant_type != QZ_NF4) return QZ_ERR_DTYPE;
  if (dtype != QZ_DT_F16) return QZ_ERR_DTYPE;
  const int bsl = ilog2g(blocksize), bs2l = dq ? ilog2g(blocksize2) : 0;
  if (bsl < 6 || bs2l < 0) return QZ_ERR_BLOCKSIZE;
  if (K % kBK != 0 || ldx < K || ldy < M || (ldx % 8) != 0 ||
      (reinterpret_cast<uintptr_t>(X) % 16) != 0 || (reinterpret_cast<uintptr_t>(B) % 16) != 0)
    return QZ_ERR_SHAPE;
  if (T == 0 || M == 0) return QZ_OK;
  GemmParams p;
  p.X = X;
  p.B = B;
  p.sc = ScaleSrc{absmax, qabsmax, absmax2, code2, offset, blocksize2};
  p.bias = bias;
  p.Y = Y;
  p.T = T;
  p.M = M;
  p.K = K;
  p.ldx = ldx;
  p.ldy = ldy;
  p.bs_log2 = bsl;
  p.bs2_log2 = bs2l;
  gemm_tables(quant_type, p.tab, &p.lut_scale);
  const dim3 grid((unsigned)((M + kBM - 1) / kBM), (unsigned)((T + kBT - 1) / kBT));
  hipStream_t s = (hipStream_t)stream;
  if (quant_type == QZ_FP4) {
    if (dq) hipLaunchKernelGGL((k_gemm_4bit_f16<QZ_FP4, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_gemm_4bit_f16<QZ_FP4, false>), grid, dim3(256), 0, s, p);
  } else {
    if (dq) hipLaunchKernelGGL((k_gemm_4bit_f16<QZ_NF4, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_gemm_4bit_f16<QZ_NF4, false>), grid, dim3(256), 0, s, p);
  }
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

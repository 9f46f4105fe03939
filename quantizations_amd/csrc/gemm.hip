// gemm.hip -- fused 4-bit dequantise + MFMA GEMM for batched prefill on gfx950.
//
// Replaces the reference prefill (modules.py:62-64): a full-weight dequant
// kernel that writes M*K fp16 to HBM (kernels.cu:554-560), a cast to fp32 and
// an fp32 SGEMM (F.linear).  Here Y[T, M] = X[T, K] . W[M, K]^T (+ bias) runs
// in one kernel (plus a tiny reduce kernel when K is split):
//
//   * A 256-thread workgroup owns a BT (tokens: 64 or 128) x 128 (weight rows)
//     output tile and walks its K range in steps of 64 = one scale block per
//     weight row (blocksize >= 64).
//   * The W operand is BIT-IDENTICAL to the reference's dequantised fp16/bf16
//     weight (dequantize_4bit, kernels.cu:554-560 -> our k_dequantize_4bit):
//     each thread owns 32 codes of one (row, block) and first builds that
//     block's 16-entry table fp16(code[i] * absmax) (fp32 product, RNE store;
//     FP4 negatives by sign flip, so code 8 is -0.0 as in the tree), then
//     decodes its nibbles through the table with the AND-combined v_perm
//     lookups of gemv.hip.  The GEMM therefore differs from "dequantise, then
//     fp32 GEMM" only in fp32 summation order.
//   * Software pipeline: the next K-step's X and W bytes are loaded into
//     registers before this step's MFMAs; after them the registers are decoded
//     into the other half of a double-buffered LDS image.  One barrier per step.
//   * Within every 16-byte (8-element) chunk both operands are stored in the
//     pair order (e0,e2),(e4,e6),(e1,e3),(e5,e7) that the decode produces; the
//     dot product over K is order-free, so W needs no re-interleave.
//   * LDS images are [row][64 elements] with a 16-B-chunk XOR swizzle so the
//     ds_read_b128 operand fetches are conflict-free.
//   * v_mfma_f32_16x16x32_{f16,bf16}, fp32 accumulation straight in the MFMA
//     accumulators (no per-block fold: the scale is inside W).
//   * Small T: the K range is split over gridDim.z workgroups that write fp32
//     partial tiles to a caller-provided workspace; k_gemm_reduce sums them
//     (+ bias) into Y.  The library never allocates.
// Requires K % 64 == 0, blocksize >= 64 (every Llama shape); other shapes
// return QZ_ERR_SHAPE and the host falls back to dequantize + library GEMM.
#include "common.h"
#include "decode.h"
#include "gemm16_asm_step.h"

namespace qz {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef __bf16 b8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kBM = 128, kBK = 64;

// natural 8-element chunk (x0..x7 as 4 pairs) -> (x0,x2),(x4,x6),(x1,x3),(x5,x7)
__device__ __forceinline__ v4u pair_order(const v4u r) {
  return v4u{gperm(r.y, r.x, 0x05040100u), gperm(r.w, r.z, 0x05040100u), gperm(r.y, r.x, 0x07060302u),
             gperm(r.w, r.z, 0x07060302u)};
}

// LDS image: [row][64 elements] = 128-B rows; 16-B chunk c of row r lives at
// chunk position c ^ ((r >> 1) & 7): the 16 rows one ds_read_b128 lane group
// touches land on distinct 16-B bank slots.
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

struct GemmParams {
  const void *X;
  const unsigned char *B;
  ScaleSrc sc;
  const void *bias;
  void *Y;
  float *ws;          // split-K partials [nsplit][T][M] fp32, or nullptr
  long long block_base;  // first scale block (row-sharded weights; multi-token kernel only, else 0)
  int T, M, K, ldx, ldy;
  int bs_log2, bs2_log2;
  int k_split;        // K elements per split (multiple of 64)
};

template <int QT, bool DQ, int DT, int BT>
__global__ __launch_bounds__(256) void k_gemm_4bit(GemmParams p) {
  constexpr int WT = BT / 64;       // waves along T (1 or 2)
  constexpr int WM = 4 / WT;        // waves along M (4 or 2)
  constexpr int TI = 4;             // 16-token fragments per wave (64 tokens)
  constexpr int MJ = kBM / WM / 16; // 16-row fragments per wave (2 or 4)
  constexpr int XC = BT / 32;       // 16-B X chunks per thread per step
  __shared__ __attribute__((aligned(16))) unsigned char s_x[2][BT * 128];
  __shared__ __attribute__((aligned(16))) unsigned char s_w[2][kBM * 128];
  __shared__ float s_code2[DQ ? 256 : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave / WM, wm = wave % WM;
  const int m0 = blockIdx.x * kBM;
  const int t0 = blockIdx.y * BT;
  const int kbeg = blockIdx.z * p.k_split;
  const int kend = min(p.K, kbeg + p.k_split);
  const int nsteps = (kend - kbeg) / kBK;
  const uint32_t row_bytes = (uint32_t)p.K >> 1;

  float offset = 0.0f;
  if constexpr (DQ) {
    s_code2[tid] = p.sc.code2[tid];
    offset = *p.sc.offset;
  }

  // weight ownership: thread -> (row wr, 32-code half wh of the 64-code step)
  const int wr = tid >> 1, wh = tid & 1;
  const int wrow = min(m0 + wr, p.M - 1);  // clamped: rows >= M are computed and never stored
  const unsigned char *wptr = p.B + (size_t)wrow * row_bytes + 16 * wh;
  const uint32_t blk_row = (uint32_t)(((long long)wrow * p.K) >> p.bs_log2);  // K % 64 == 0, blocksize >= 64

  // ---- staged registers of one K-step ----
  v4u xv[XC];
  v4u wv;
  uint32_t q = 0;
  float a = 0.0f;
  auto load_step = [&](int k0) {
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int c = tid + 256 * i;
      const int t = t0 + (c >> 3);
      xv[i] = t < p.T ? *reinterpret_cast<const v4u *>(reinterpret_cast<const uint16_t *>(p.X) +
                                                      (size_t)t * p.ldx + k0 + 8 * (c & 7))
                      : v4u{0u, 0u, 0u, 0u};
    }
    wv = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(wptr + (k0 >> 1)));
    const uint32_t b = blk_row + ((uint32_t)k0 >> p.bs_log2);
    if constexpr (DQ) {
      q = p.sc.qabsmax[b];
      a = p.sc.absmax2[b >> p.bs2_log2];
    } else {
      a = p.sc.absmax[b];
    }
  };
  auto store_step = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<v4u *>(s_x[buf] + lds_off(c >> 3, c & 7)) = pair_order(xv[i]);
    }
    float am;
    if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[q], a), offset);  // core.py:467-468
    else am = a;
    uint32_t t[8];
    block_table<QT, DT>(am, t);
    const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t P[4];
      decode_codes(w[d], t, P);
      *reinterpret_cast<v4u *>(s_w[buf] + lds_off(wr, 4 * wh + d)) = v4u{P[0], P[1], P[2], P[3]};
    }
  };

  f4_t acc[TI][MJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;  // MFMA fragment row / k-group
  if (nsteps > 0) {
    load_step(kbeg);
    if constexpr (DQ) __syncthreads();  // s_code2 staged
    store_step(0);
    __syncthreads();
  }
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) load_step(kbeg + (s + 1) * kBK);  // in flight during this step's MFMAs
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4u af[TI], bf[MJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        af[i] = *reinterpret_cast<const v4u *>(s_x[cur] + lds_off(64 * wt + 16 * i + fr, 4 * kk + fk));
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        bf[j] = *reinterpret_cast<const v4u *>(s_w[cur] + lds_off((kBM / WM) * wm + 16 * j + fr, 4 * kk + fk));
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
          if constexpr (DT == QZ_DT_F16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, af[i]),
                                                               __builtin_bit_cast(h8_t, bf[j]), acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, af[i]),
                                                                __builtin_bit_cast(b8_t, bf[j]), acc[i][j], 0, 0, 0);
        }
    }
    if (more) store_step(cur ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }

  // ---- epilogue: C/D map col (weight row) = lane & 15, row (token) = 4 * (lane >> 4) + r ----
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int m = m0 + (kBM / WM) * wm + 16 * j + fr;
    if (m >= p.M) continue;
    if (p.ws) {  // split-K partial
      float *ws = p.ws + (size_t)blockIdx.z * p.T * p.M;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = t0 + 64 * wt + 16 * i + 4 * fk + r;
          if (t < p.T) ws[(size_t)t * p.M + m] = acc[i][j][r];
        }
      continue;
    }
    const float bv = p.bias ? load_f32<DT>(p.bias, m) : 0.0f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + 64 * wt + 16 * i + 4 * fk + r;
        if (t < p.T) store_f32<DT>(p.Y, (long long)t * p.ldy + m, acc[i][j][r] + bv);
      }
  }
}

// Large-T prefill: 256 x 256 output tile (256 tokens x 256 weight rows), 8
// waves as 2 (tokens) x 4 (rows), each wave 128 tokens x 64 rows = 4 x 8
// v_mfma_f32_16x16x32 accumulators, K-step 64 (one scale block per row).
//   * X (the B operand) goes global -> LDS with global_load_lds_dwordx4 (no
//     VGPRs, no VALU): the LDS image is lane-linear per wave instruction, so the
//     16-B-chunk XOR swizzle of lds_off() is applied to the per-lane SOURCE
//     address (the read applies the same involution).
//   * W (the A operand) is register-staged: a thread owns 32 codes of one
//     (row, block); its packed bytes and scale for step s+1 are loaded while
//     step s multiplies, then decoded -- through the exact per-block table, in
//     natural element order to match X -- into the other LDS buffer.  The W
//     operand is bit-identical to dequantize_4bit's.
//   * One barrier per K-step (its vmcnt(0) retires the next step's X DMA and W loads).
//   * Epilogue through LDS: accumulators (+ bias) -> fp16/bf16 rows of 128 B
//     per wave, then 16-B coalesced stores of Y rows.
//   * XCD-aware tile order: each XCD walks a contiguous range of tiles (token
//     tile major), so the tiles in flight on one XCD share X/W k-slices in its L2.
constexpr int kBigT = 256, kBigM = 256;
constexpr int kBigStage = kBigT * 128;              // one buffer of X or W: 256 rows x 64 elements x 2 B
constexpr int kBigLds = 4 * kBigStage;              // X[2] + W[2] = 128 KiB
constexpr int kBigERow = 144;                       // epilogue image row: 64 outputs x 2 B + 16 B pad
constexpr int kBigMinT = 4096;  // below this the 128-row tile kernel (with split-K) is faster (gemm_micro)

// V (schedule variant, microbenchmark A/B): 0 = decode after the step's MFMAs with a
// scheduling fence per fragment half; 1 = no fences; 2 = decode between the two k-halves;
// 3 = every K-loop global read is an LDS DMA: packed W and its scales land in a 3-deep LDS
// ring two steps ahead of their decode, which then sits between the step's MFMA halves
// with no global-load wait; one counted vmcnt per step leaves the newest W DMA in flight.
// 4 = variant 3 without the decode (microbenchmark timing only: wrong results).
constexpr int kBigWp = 8192;                    // V3: packed W of one step (256 rows x 32 B)
constexpr int kBigWpOff = kBigLds;              // V3: Wp[3]
constexpr int kBigScOff = kBigWpOff + 3 * kBigWp;  // V3: scale dwords [3][2][256]
template <int V> constexpr int big_code2_off() { return V >= 3 ? kBigScOff + 3 * 2048 : kBigLds; }
template <int QT, bool DQ, int DT, int V = 0>
__global__ __launch_bounds__(512) void k_gemm_4bit_big(GemmParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[big_code2_off<V>() + (DQ ? 1024 : 0)];
  typedef __attribute__((address_space(3))) void *lds_ptr_t;
  typedef __attribute__((address_space(1))) void *glb_ptr_t;
  float *s_code2 = reinterpret_cast<float *>(smem + big_code2_off<V>());
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 2, wm = wave & 3;

  // XCD-aware, bijective tile order (blocks are dealt to the 8 XCDs round-robin)
  const int tiles_m = (p.M + kBigM - 1) / kBigM;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (wg % tiles_m) * kBigM, t0 = (wg / tiles_m) * kBigT;
  const int nsteps = p.K / kBK;

  // X staging: instruction i of wave w fills LDS rows 8*(8i + w) .. +8 (1 KiB, lane-linear);
  // lane l lands in row 8*(8i+w) + l/8, 16-B slot l%8, which holds chunk slot ^ ((row >> 1) & 7)
  // (32-bit byte offsets from the uniform X base: the host guarantees T * ldx * 2 < 2^32)
  const unsigned char *xbase = reinterpret_cast<const unsigned char *>(p.X);
  uint32_t xoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (8 * i + wave) + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    xoff[i] = ((uint32_t)min(t0 + row, p.T - 1) * (uint32_t)p.ldx + 8u * chunk) * 2u;
  }
  auto stage_x = [&](int step, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((glb_ptr_t)(xbase + xoff[i] + (uint32_t)step * (kBK * 2)),
                                       (lds_ptr_t)(smem + buf * kBigStage + (8 * i + wave) * 1024), 16, 0, 0);
  };

  // W staging: thread -> (row wr, 32-code half wh of the 64-code step)
  const int wr = tid >> 1, wh = tid & 1;
  const int wrow = min(m0 + wr, p.M - 1);  // clamped rows are computed and never stored
  const unsigned char *wptr = p.B + (size_t)wrow * ((uint32_t)p.K >> 1) + 16 * wh;
  const uint32_t blk_row = (uint32_t)(((long long)wrow * p.K) >> p.bs_log2);
  struct WStage {
    v4u w;
    uint32_t q;
    float a;
  };
  auto load_w = [&](WStage &st, int step) {
    const int k0 = step * kBK;
    st.w = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(wptr + (k0 >> 1)));
    const uint32_t b = blk_row + ((uint32_t)k0 >> p.bs_log2);
    if constexpr (DQ) {
      st.q = p.sc.qabsmax[b];
      st.a = p.sc.absmax2[b >> p.bs2_log2];
    } else {
      st.q = 0u;
      st.a = p.sc.absmax[b];
    }
  };
  float offset = 0.0f;
  auto store_w = [&](const WStage &st, int buf) {
    float am;
    if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[st.q], st.a), offset);  // core.py:467-468
    else am = st.a;
    uint32_t t[8];
    block_table<QT, DT>(am, t);
    const uint32_t w[4] = {st.w.x, st.w.y, st.w.z, st.w.w};
    unsigned char *sw = smem + (2 + buf) * kBigStage;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t N[4];
      decode_codes_natural(w[d], t, N);
      *reinterpret_cast<v4u *>(sw + lds_off(wr, 4 * wh + d)) = v4u{N[0], N[1], N[2], N[3]};
    }
  };

  // V3: W DMA of one step -- thread tid's 16 packed bytes (lane-linear: row tid/2, half tid%2),
  // and one scale dword per row: threads 0-255 the q dword (DQ; fp32 absmax otherwise), threads
  // 256-511 the absmax2 entry (DQ; fp32 absmax otherwise) of row tid % 256
  const int srow = tid & 255;
  const uint32_t blk_row_s = (uint32_t)(((long long)min(m0 + srow, p.M - 1) * p.K) >> p.bs_log2);
  auto dma_w = [&](int step, int pb) {
    const int k0 = step * kBK;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(wptr + (k0 >> 1)),
                                     (lds_ptr_t)(smem + kBigWpOff + pb * kBigWp + wave * 1024), 16, 0, 0);
    const uint32_t b = blk_row_s + ((uint32_t)k0 >> p.bs_log2);
    const void *src;
    if constexpr (DQ) src = tid < 256 ? (const void *)(p.sc.qabsmax + (b & ~3u)) : (const void *)(p.sc.absmax2 + (b >> p.bs2_log2));
    else src = p.sc.absmax + b;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)src, (lds_ptr_t)(smem + kBigScOff + pb * 2048 + wave * 256), 4, 0, 0);
  };
  auto decode_w = [&](int step, int pb, int db) {
    const v4u wv = *reinterpret_cast<const v4u *>(smem + kBigWpOff + pb * kBigWp + tid * 16);
    const unsigned char *sc = smem + kBigScOff + pb * 2048;
    float am;
    if constexpr (DQ) {
      const uint32_t b = blk_row + ((uint32_t)(step * kBK) >> p.bs_log2);
      const uint32_t q = (*reinterpret_cast<const uint32_t *>(sc + wr * 4) >> (8 * (b & 3))) & 255u;
      am = __fadd_rn(__fmul_rn(s_code2[q], *reinterpret_cast<const float *>(sc + 1024 + wr * 4)), offset);
    } else {
      am = *reinterpret_cast<const float *>(sc + 1024 + wr * 4);
    }
    WStage st{wv, 0u, am};
    if constexpr (V == 4) {  // microbenchmark ablation: no decode, the packed bytes go to LDS as they are
      unsigned char *sw = smem + (2 + db) * kBigStage;
      const uint32_t a = __float_as_uint(am);
#pragma unroll
      for (int d = 0; d < 4; ++d)
        *reinterpret_cast<v4u *>(sw + lds_off(wr, 4 * wh + d)) = v4u{wv.x ^ a, wv.y, wv.z, wv.w};
    } else if constexpr (DQ) {  // store_w rebuilds am from (q, a): pass the rebuilt scale through unchanged
      uint32_t t[8];
      block_table<QT, DT>(am, t);
      const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
      unsigned char *sw = smem + (2 + db) * kBigStage;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t N[4];
        decode_codes_natural(w[d], t, N);
        *reinterpret_cast<v4u *>(sw + lds_off(wr, 4 * wh + d)) = v4u{N[0], N[1], N[2], N[3]};
      }
    } else {
      store_w(st, db);
    }
  };

  f4_t acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f4_t{0.f, 0.f, 0.f, 0.f};
  // Fragment addresses: every fragment row is 16 * n + fr, so the chunk swizzle ((row >> 1) & 7)
  // is (fr >> 1) & 7 for all of them and chunk 4 * kk + fk lands at slot (fk ^ swz) ^ 4 * kk:
  // one lane offset per kk, everything else a compile-time / wave-uniform offset (no per-fragment
  // address registers live across the K loop).
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t frag_lane[2] = {(uint32_t)(fr * 128 + ((fk ^ ((fr >> 1) & 7)) << 4)),
                                 (uint32_t)(fr * 128 + (((fk ^ ((fr >> 1) & 7)) ^ 4) << 4))};
  auto mfma_half = [&](int buf, int kk) {
    const unsigned char *sx = smem + buf * kBigStage + (128 * wt) * 128;
    const unsigned char *sw = smem + (2 + buf) * kBigStage + (64 * wm) * 128;
    {
      v4u aw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) aw[j] = *reinterpret_cast<const v4u *>(sw + frag_lane[kk] + 16 * j * 128);
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {  // token fragments in two halves: 16 fewer live VGPRs
        v4u bx[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          bx[i] = *reinterpret_cast<const v4u *>(sx + frag_lane[kk] + 16 * (4 * ih + i) * 128);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            f4_t &c = acc[j][4 * ih + i];
            if constexpr (DT == QZ_DT_F16)
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, aw[j]), __builtin_bit_cast(h8_t, bx[i]),
                                                         c, 0, 0, 0);
            else
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, aw[j]),
                                                          __builtin_bit_cast(b8_t, bx[i]), c, 0, 0, 0);
          }
        if constexpr (V == 0) __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // W is prefetched one step ahead into ONE register set: step s issues W(s+1)'s loads right
  // after X(s+1)'s DMA, multiplies buffer s & 1, then decodes W(s+1) into the other buffer.
  // (A two-set ring needs the loop unrolled by two; its extra live registers spilled the
  // accumulators.)
  if constexpr (V >= 3) {
    stage_x(0, 0);
    dma_w(0, 0);
    if (nsteps > 1) dma_w(1, 1);
    if (nsteps > 2) dma_w(2, 2);
    if constexpr (DQ) {
      if (tid < 256) s_code2[tid] = p.sc.code2[tid];
      offset = *p.sc.offset;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    decode_w(0, 0, 0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      const int cur = s & 1;
      const bool more = s + 1 < nsteps, w3 = s + 3 < nsteps;
      if (more) stage_x(s + 1, cur ^ 1);
      if (w3) dma_w(s + 3, (s + 3) % 3);
      mfma_half(cur, 0);
      if (more) decode_w(s + 1, (s + 1) % 3, cur ^ 1);
      mfma_half(cur, 1);
      if (more) {  // X(s+1) and W(s+2) landed (only W(s+3)'s two DMAs may still fly), LDS writes done
        if (w3) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
  } else {
  WStage ws;
  stage_x(0, 0);
  load_w(ws, 0);
  if constexpr (DQ) {
    if (tid < 256) s_code2[tid] = p.sc.code2[tid];
    offset = *p.sc.offset;
  }
  __syncthreads();
  store_w(ws, 0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) {
      stage_x(s + 1, cur ^ 1);
      load_w(ws, s + 1);
    }
    mfma_half(cur, 0);
    if (V == 2 && more) store_w(ws, cur ^ 1);
    mfma_half(cur, 1);
    if (more) {
      if (V != 2) store_w(ws, cur ^ 1);
      __syncthreads();  // X(s+1) DMA + W(s+1) decode visible to every wave; buffer cur free
    }
  }
  }

  // ---- epilogue: lane holds weight rows 16j + 4*fk + r (r = 0..3) of token 16i + fr ----
  __syncthreads();  // every wave is done with the staging buffers
  unsigned char *ew = smem + wave * (64 * kBigERow);
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = min(m0 + 64 * wm + 16 * j + 4 * fk + r, p.M - 1);
      bv[j][r] = p.bias ? load_f32<DT>(p.bias, m) : 0.0f;
    }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f4_t v = acc[j][4 * h + i];
        const uint32_t lo = cvt_pk16<DT>(v[0] + bv[j][0], v[1] + bv[j][1]);
        const uint32_t hi = cvt_pk16<DT>(v[2] + bv[j][2], v[3] + bv[j][3]);
        *reinterpret_cast<uint2 *>(ew + (16 * i + fr) * kBigERow + (16 * j + 4 * fk) * 2) = uint2{lo, hi};
      }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int qd = lane + 64 * it, tok = qd >> 3, c16 = qd & 7;
      const v4u v = *reinterpret_cast<const v4u *>(ew + tok * kBigERow + c16 * 16);
      const int t = t0 + 128 * wt + 64 * h + tok, m = m0 + 64 * wm + 8 * c16;
      if (t < p.T && m < p.M)
        *reinterpret_cast<v4u *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m) = v;
    }
  }
}

// Large-T prefill, staggered two-group schedule ("8-phase"; guide section 5 template,
// re-derived for a W operand that is DECODED into LDS, not copied):
//   * same 256 x 256 tile, 8 waves as 2 (tokens: wave group g = wave >> 2) x 4
//     (rows), 128 tokens x 64 rows per wave, K-step 64 = one scale block per row,
//     same LDS images / swizzle / epilogue as k_gemm_4bit_big;
//   * a K-step is 4 phases, one C quadrant (64 tokens x 32 rows = 16 MFMAs) each.
//     A phase is [read segment] s_barrier [16 MFMAs] s_barrier; group 1 starts one
//     barrier late, so in every barrier interval one group runs MFMAs while the
//     other (the wave on the same SIMD) issues its fragment ds_reads, its share of
//     the next step's W decode and its staging DMAs -- the decode's VALU and the
//     LDS traffic hide under the other group's matrix work;
//   * quadrant order (rows lo, tok lo), (rows hi, tok lo), (rows hi, tok hi),
//     (rows lo, tok hi): each phase loads only the fragments that change
//     (12, 4, 8, 4 ds_read_b128);
//   * staging (all LDS DMA, issued in phase 0 of step s): X(s+1) into the other X
//     buffer (free: every wave passed its last read of step s-1 one barrier
//     earlier) and the packed bytes + scales of W(s+2) into a 2-slot ring; phase
//     3 of step s retires them with vmcnt(0) before its barrier, so step s+1 reads
//     them after >= 1 barrier (the RAW rule of the guide);
//   * W(s+1) is decoded during step s, one packed dword (8 codes -> 16 B of the
//     exact fp16/bf16 image) per thread per phase, into the other W buffer; the
//     per-(row, block) table is built in phase 0.  Phase 3 waits lgkmcnt(0) before
//     its barrier, so the image is complete before any wave reads it.
// SK (schedule knobs; the product uses 1): 1 = keep the rows-lo W fragments live from phase 0
// to phase 3 instead of re-reading them (+2 % fused); 2 = one static s_setprio for group 1
// instead of per-cluster flips, 4 = no s_setprio (both slower: profiles/r2_gemm_sk.txt);
// 8 = v_mfma_f32_32x32x16 instead of 16x16x32 (same results bit for bit, 7-11 % slower:
// profiles/r2_gemm_mfma32.txt); 16 = no DMA at all and 32 = every step DMAs the k-slice of step 0
// (microbenchmark timing only: the LDS -> MFMA skeleton, and the schedule with L2-resident
// operands); 64 = grouped (4 token x 8 row tiles per XCD) tile order; 128 = plain W staged
// through registers; 256 = plain W in three buffers, staged two steps ahead one piece per phase.
// V (microbenchmark A/B, timing only except 0, 2 and 5): 0 = product; 1 = no decode
// (packed bytes copied); 2 = no group stagger; 3 = as 1 without the W/scale DMAs;
// 4 = as 3 without the X DMAs (the LDS -> MFMA skeleton alone); 5 = a plain fp16 GEMM on the
// same schedule (B = fp16 [M, K], staged by DMA like X; no decode).
#ifdef QZ_STAMPS8P
__device__ unsigned long long g_qz_stamp8p[2 * 8 * 16];
#endif
// scheduling hint for one MFMA segment: NM x {1 MFMA, N VALU} (the decode's VALU goes into the
// issue slots the MFMAs leave free instead of queueing after the last one)
template <int N, int NM = 16> __device__ __forceinline__ void interleave_mfma_valu() {
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, N, 0);
  }
}
constexpr int kPlainW = 5;  // k_gemm_4bit_8p variant: B is a dense 16-bit [M, K] weight (qz_gemm_16bit)
constexpr int k8pX = 0, k8pW = 2 * kBigStage, k8pWp = 4 * kBigStage, k8pSc = k8pWp + 2 * kBigWp;
constexpr int k8pCode2 = k8pSc + 2 * 2048;
template <int QT, bool DQ, int DT, int V = 0, int SK = 0>
__global__ __launch_bounds__(512) void k_gemm_4bit_8p(GemmParams p) {
  // SK & 256 (plain W): three W buffers (k8pW .. 160 KiB, over the unused packed-W/scale rings)
  constexpr bool kW3 = V == kPlainW && (SK & 256) != 0;
  __shared__ __attribute__((aligned(16))) unsigned char smem[kW3 ? 163840 : k8pCode2 + (DQ ? 1024 : 0)];
  typedef __attribute__((address_space(3))) void *lds_ptr_t;
  typedef __attribute__((address_space(1))) void *glb_ptr_t;
  float *s_code2 = reinterpret_cast<float *>(smem + k8pCode2);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 2, wm = wave & 3;

  // XCD-aware, bijective tile order (as k_gemm_4bit_big)
  const int tiles_m = (p.M + kBigM - 1) / kBigM;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm = wg % tiles_m, tt = wg / tiles_m;
  if constexpr ((SK & 64) != 0) {
    // grouped order: the tiles of one XCD in flight together cover 4 token tiles x 8 row tiles
    // (X and W k-slices each shared by 8 resp. 4 of them in that XCD's L2) instead of 2 x 16
    const int tiles_t = (p.T + kBigT - 1) / kBigT;
    if (tiles_m % 8 == 0 && tiles_t % 4 == 0) {
      const int grp = wg / (4 * tiles_m), r = wg % (4 * tiles_m);
      tt = 4 * grp + (r % 32) / 8;
      tm = 8 * (r / 32) + r % 8;
    }
  }
  const int m0 = tm * kBigM, t0 = tt * kBigT;
  const int nsteps = p.K / kBK;
  constexpr uint32_t kStepB = (SK & 32) ? 0u : (uint32_t)(kBK * 2);  // SK & 32: timing only

  // ---- staging (LDS DMA only) ----
  const unsigned char *xbase = reinterpret_cast<const unsigned char *>(p.X);
  uint32_t xoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (8 * i + wave) + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    xoff[i] = ((uint32_t)min(t0 + row, p.T - 1) * (uint32_t)p.ldx + 8u * chunk) * 2u;
  }
  // instruction i of every wave stages token quarter i (rows 64 i .. 64 i + 63 of the tile)
  auto stage_xq = [&](int step, int buf, int i) {
    if constexpr (V == 4 || (SK & 16) != 0) return;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(xbase + xoff[i] + (uint32_t)step * kStepB),
                                     (lds_ptr_t)(smem + k8pX + buf * kBigStage + (8 * i + wave) * 1024), 16, 0, 0);
  };
  // V == kPlainW (qz_gemm_16bit): B is a dense 16-bit [M, K] weight staged by DMA like X, one
  // step ahead into the other W buffer -- the schedule as a plain GEMM, no decode
  uint32_t woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (8 * i + wave) + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    woff[i] = ((uint32_t)min(m0 + row, p.M - 1) * (uint32_t)p.K + 8u * chunk) * 2u;
  }
  // SK & 128: W through registers instead (global_load_dwordx4 in phase 0, ds_write_b128 in
  // phase 2's MFMA segment) -- no LDS-DMA issue for W
  v4u wreg[4];
  auto load_wf_regs = [&](int step) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      wreg[i] = *reinterpret_cast<const v4u *>(p.B + woff[i] + (uint32_t)step * kStepB);
  };
  auto write_wf_regs = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<v4u *>(smem + k8pW + buf * kBigStage + (8 * i + wave) * 1024 + lane * 16) = wreg[i];
  };
  auto stage_wf_piece = [&](int step, int buf, int i) {
    if constexpr ((SK & 16) != 0) return;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(p.B + woff[i] + (uint32_t)step * kStepB),
                                     (lds_ptr_t)(smem + k8pW + buf * kBigStage + (8 * i + wave) * 1024), 16, 0, 0);
  };
  auto stage_wf = [&](int step, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) stage_wf_piece(step, buf, i);
  };
  const int wr = tid >> 1, wh = tid & 1;  // decode ownership: row wr, 32-code half wh
  const int wrow = min(m0 + wr, p.M - 1);
  const unsigned char *wptr = p.B + (size_t)wrow * ((uint32_t)p.K >> 1) + 16 * wh;
  const uint32_t blk_row = (uint32_t)(((long long)wrow * p.K) >> p.bs_log2);
  const int srow = tid & 255;
  const uint32_t blk_row_s = (uint32_t)(((long long)min(m0 + srow, p.M - 1) * p.K) >> p.bs_log2);
  auto dma_w = [&](int step, int slot) {
    if constexpr (V >= 3) return;  // (V 5 stages its fp16 W in stage_wf)
    const int k0 = step * kBK;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(wptr + (k0 >> 1)),
                                     (lds_ptr_t)(smem + k8pWp + slot * kBigWp + wave * 1024), 16, 0, 0);
    const uint32_t b = blk_row_s + ((uint32_t)k0 >> p.bs_log2);
    const void *src;
    if constexpr (DQ)
      src = tid < 256 ? (const void *)(p.sc.qabsmax + (b & ~3u)) : (const void *)(p.sc.absmax2 + (b >> p.bs2_log2));
    else
      src = p.sc.absmax + b;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)src, (lds_ptr_t)(smem + k8pSc + slot * 2048 + wave * 256), 4, 0, 0);
  };
  float offset = 0.0f;
  // the exact per-(row, block) table of step `step` (its packed bytes + scales sit in `slot`):
  // read_scale issues the LDS reads (ahead of the phase's fragment reads), make_table the VALU
  struct ScaleWords {
    uint32_t q;
    float a;
  };
  auto read_scale = [&](int slot) {
    const unsigned char *sc = smem + k8pSc + slot * 2048;
    return ScaleWords{DQ ? *reinterpret_cast<const uint32_t *>(sc + wr * 4) : 0u,
                      *reinterpret_cast<const float *>(sc + 1024 + wr * 4)};
  };
  auto make_table = [&](int step, const ScaleWords &sw, uint32_t (&t)[8]) {
    float am;
    if constexpr (DQ) {
      const uint32_t b = blk_row + ((uint32_t)(step * kBK) >> p.bs_log2);
      const uint32_t q = (sw.q >> (8 * (b & 3))) & 255u;
      am = __fadd_rn(__fmul_rn(s_code2[q], sw.a), offset);   // core.py:467-468
    } else {
      am = sw.a;
    }
    block_table<QT, DT>(am, t);
  };
  auto read_packed = [&](int slot, int d) {
    return *reinterpret_cast<const uint32_t *>(smem + k8pWp + slot * kBigWp + tid * 16 + 4 * d);
  };
  // packed dword d of this thread's 16 bytes -> 8 exact 16-bit weights -> W image chunk 4 wh + d
  auto decode_dword = [&](uint32_t w, int buf, int d, const uint32_t (&t)[8]) {
    if constexpr (V == kPlainW) return;
    unsigned char *dst = smem + k8pW + buf * kBigStage + lds_off(wr, 4 * wh + d);
    if constexpr (V == 1 || V == 3 || V == 4) {
      *reinterpret_cast<v4u *>(dst) = v4u{w, w ^ t[0], w, w};
    } else {
      uint32_t N[4];
      decode_codes_natural(w, t, N);
      *reinterpret_cast<v4u *>(dst) = v4u{N[0], N[1], N[2], N[3]};
    }
  };

  // ---- fragments (as k_gemm_4bit_big: one lane offset per k-half) ----
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t frag_lane[2] = {(uint32_t)(fr * 128 + ((fk ^ ((fr >> 1) & 7)) << 4)),
                                 (uint32_t)(fr * 128 + (((fk ^ ((fr >> 1) & 7)) ^ 4) << 4))};
  f4_t acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f4_t{0.f, 0.f, 0.f, 0.f};
  v4u xf[2][4];  // X fragments of the current token half: [kk][i]
  // W fragments [kk][j] of row half 0 (wfA) and 1 (wfB); without SK & 1 both names are one set
  // (reloaded in phase 3), with it rows-lo stay live from phase 0 to phase 3
  v4u wfA[2][2], wfB0[2][2];
  v4u(&wfB)[2][2] = (SK & 1) ? wfB0 : wfA;
  // SK & 8: the same quadrants on v_mfma_f32_32x32x16 (8 MFMAs of 32 cycles per phase instead of
  // 16 of 16: half the MFMA issue slots, so more room for the other group's reads and the decode).
  // A/B lane (r32 = lane % 32, h32 = lane / 32) holds row r32, k = 8 h32 .. +8 of a k16 substep q
  // (chunk 2q + h32); the swizzle of lds_off keeps every ds_read_b128 lane group conflict-free.
  // D: lane holds column (token) r32, rows 8g + 4 h32 + r in register 4g + r.
  constexpr bool kMF32 = (SK & 8) != 0;
  typedef float f16v_t __attribute__((ext_vector_type(16)));
  const int r32 = lane & 31, h32 = lane >> 5;
  uint32_t fl32[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) fl32[q] = (uint32_t)(r32 * 128 + (((2 * q + h32) ^ ((r32 >> 1) & 7)) << 4));
  f16v_t acc32[kMF32 ? 2 : 1][kMF32 ? 4 : 1];
  if constexpr (kMF32) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[j][i][e] = 0.0f;
  }
  v4u xf32[4][2], wfA32[4], wfB32_0[4];
  v4u(&wfB32)[4] = (SK & 1) ? wfB32_0 : wfA32;
  auto load_x = [&](int buf, int th) {
    const unsigned char *sx = smem + k8pX + buf * kBigStage + (128 * wt + 64 * th) * 128;
    if constexpr (kMF32) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) xf32[q][i] = *reinterpret_cast<const v4u *>(sx + 32 * i * 128 + fl32[q]);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) xf[kk][i] = *reinterpret_cast<const v4u *>(sx + frag_lane[kk] + 16 * i * 128);
  };
  auto load_w = [&](int buf, int rh) {
    const unsigned char *sw = smem + k8pW + buf * kBigStage + (64 * wm + 32 * rh) * 128;
    if constexpr (kMF32) {
      v4u(&wf32)[4] = rh ? wfB32 : wfA32;
#pragma unroll
      for (int q = 0; q < 4; ++q) wf32[q] = *reinterpret_cast<const v4u *>(sw + fl32[q]);
      return;
    }
    v4u(&wf)[2][2] = rh ? wfB : wfA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) wf[kk][j] = *reinterpret_cast<const v4u *>(sw + frag_lane[kk] + 16 * j * 128);
  };
  auto mfma_quadrant = [&](int rh, int th) {
    if constexpr (kMF32) {
      v4u(&wf32)[4] = rh ? wfB32 : wfA32;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          f16v_t &c = acc32[rh][2 * th + i];
          if constexpr (DT == QZ_DT_F16)
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, wf32[q]),
                                                       __builtin_bit_cast(h8_t, xf32[q][i]), c, 0, 0, 0);
          else
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8_t, wf32[q]),
                                                        __builtin_bit_cast(b8_t, xf32[q][i]), c, 0, 0, 0);
        }
      return;
    }
    v4u(&wf)[2][2] = rh ? wfB : wfA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f4_t &c = acc[2 * rh + j][4 * th + i];
          if constexpr (DT == QZ_DT_F16)
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, wf[kk][j]),
                                                       __builtin_bit_cast(h8_t, xf[kk][i]), c, 0, 0, 0);
          else
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, wf[kk][j]),
                                                        __builtin_bit_cast(b8_t, xf[kk][i]), c, 0, 0, 0);
        }
  };

  // ---- prologue: X(0), X(1), W(0) and W(1) staged; W(0) decoded ----
#pragma unroll
  for (int i = 0; i < 4; ++i) stage_xq(0, 0, i);
  dma_w(0, 0);
  if (nsteps > 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) stage_xq(1, 1, i);
    dma_w(1, 1);
  }
  if constexpr (DQ) {
    if (tid < 256) s_code2[tid] = p.sc.code2[tid];
    offset = *p.sc.offset;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (V == kPlainW) {
    stage_wf(0, 0);
    if constexpr (kW3) {
      if (nsteps > 1) stage_wf(1, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    uint32_t t[8];
    make_table(0, read_scale(0), t);
#pragma unroll
    for (int d = 0; d < 4; ++d) decode_dword(read_packed(0, d), 0, d, t);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  if (V != 2 && wt == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier interval behind
  if constexpr ((SK & 2) != 0) {  // static priority for the younger half (guide T5, static form)
    if (wt == 1) __builtin_amdgcn_s_setprio(1);
  }
#ifdef QZ_STAMPS8P
  unsigned long long st8[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#define QZ_ST8(k)                                                                       \
  do {                                                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                     \
    st8[k] = s == 10 ? now_ : st8[k];                                                 \
  } while (0)
#else
#define QZ_ST8(k) do {} while (0)
#endif
  // A phase: [read segment: LDS reads + DMA issue only, no waits] s_barrier [lgkmcnt(0);
  // 16 MFMAs with this phase's share of the W(s+1) decode interleaved] s_barrier.
  int wb3 = 0;  // kW3: W buffer of step s (s % 3)
  for (int s = 0; s < nsteps; ++s) {
    const int b = s & 1;
    const int wb = kW3 ? wb3 : b;
    const int wb2 = kW3 ? (wb3 == 0 ? 2 : wb3 - 1) : 0;  // kW3: buffer of step s + 2
    const bool dma = s + 2 < nsteps;    // stage X(s+2) (into this step's buffer, quarter by quarter as
                                        // its last reader passes) and W(s+2)'s packed bytes + scales
    const int ps = (s + 1) & 1;         // ring slot of W(s+1)'s packed bytes
    uint32_t t[8], w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    ScaleWords sw{0u, 0.0f};
    QZ_ST8(0);
    // ---------------- phase 0: quadrant (rows lo, tokens lo) ----------------
    // decode inputs are read unconditionally: in the last step they are stale ring bytes, decoded
    // into the idle W buffer and never read (keeps the MFMA segments straight-line, so the
    // decode VALU interleaves with the MFMAs)
    if constexpr (V != kPlainW) {
      sw = read_scale(ps);
      w0 = read_packed(ps, 0);
    }
    if constexpr (V >= 3) sw.q = sw.q & 0u;
    load_w(wb, 0);
    load_x(b, 0);
    if constexpr (kW3) {
      if (dma) stage_wf_piece(s + 2, wb2, 0);       // W(s+2): one piece per phase
    } else if constexpr (V == kPlainW && (SK & 128) != 0) {
      load_wf_regs(min(s + 1, nsteps - 1));         // written in phase 2 (stale in the last step)
    } else if constexpr (V == kPlainW) {
      if (s + 1 < nsteps) stage_wf(s + 1, b ^ 1);  // retired by this step's phase-3 vmcnt(4)
    } else if (dma) {
      dma_w(s + 2, s & 1);
    }
    __builtin_amdgcn_s_barrier();
    QZ_ST8(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(1);
    mfma_quadrant(0, 0);
    if constexpr (V != kPlainW) make_table(s + 1, sw, t);
    decode_dword(w0, b ^ 1, 0, t);
    if constexpr (kMF32) interleave_mfma_valu<8, 8>(); else interleave_mfma_valu<4>();
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(0);
    QZ_ST8(2);
    __builtin_amdgcn_s_barrier();
    // ---------------- phase 1: (rows hi, tokens lo) ----------------
    if constexpr (V != kPlainW) {
      w1 = read_packed(ps, 1);
      w2 = read_packed(ps, 2);
    }
    load_w(wb, 1);
    if (dma) {  // quarters 0 (group 0, tokens lo) and 2 (group 1, tokens lo): last read in phase 0
      stage_xq(s + 2, b, 0);
      stage_xq(s + 2, b, 2);
      if constexpr (kW3) stage_wf_piece(s + 2, wb2, 1);
    }
    __builtin_amdgcn_s_barrier();
    QZ_ST8(3);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(1);
    mfma_quadrant(1, 0);
    decode_dword(w1, b ^ 1, 1, t);
    decode_dword(w2, b ^ 1, 2, t);
    if constexpr (kMF32) interleave_mfma_valu<8, 8>(); else interleave_mfma_valu<4>();
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(0);
    QZ_ST8(4);
    __builtin_amdgcn_s_barrier();
    // ---------------- phase 2: (rows hi, tokens hi) ----------------
    if constexpr (V != kPlainW) w3 = read_packed(ps, 3);
    load_x(b, 1);
    if constexpr (kW3) {
      if (dma) stage_wf_piece(s + 2, wb2, 2);
    }
    __builtin_amdgcn_s_barrier();
    QZ_ST8(5);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(1);
    mfma_quadrant(1, 1);
    if constexpr (V == kPlainW && (SK & 128) != 0) write_wf_regs(b ^ 1);
    decode_dword(w3, b ^ 1, 3, t);
    if constexpr (kMF32) interleave_mfma_valu<4, 8>(); else interleave_mfma_valu<2>();
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(0);
    // the W(s+1) image is complete: every wave's stores retired before this barrier (>= 3
    // barriers before step s+1's first read of it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    QZ_ST8(6);
    __builtin_amdgcn_s_barrier();
    // ---------------- phase 3: (rows lo, tokens hi); retire the step's staging ----------------
    if constexpr ((SK & 1) == 0) load_w(wb, 0);
    if (dma) {  // quarters 1 and 3 (tokens hi): last read in phase 2
      stage_xq(s + 2, b, 1);
      stage_xq(s + 2, b, 3);
      if constexpr (kW3) stage_wf_piece(s + 2, wb2, 3);
    }
    // retire X(s+1) and W(s+2)'s bytes; X(s+2)'s four quarter DMAs may stay in flight
    // (kW3: W is staged two steps ahead too: this step's 8 DMAs stay in flight)
    if (dma) {
      if constexpr (kW3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    QZ_ST8(7);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(1);
    mfma_quadrant(0, 1);
    if constexpr ((SK & 6) == 0) __builtin_amdgcn_s_setprio(0);
    QZ_ST8(8);
    __builtin_amdgcn_s_barrier();
    wb3 = wb3 == 2 ? 0 : wb3 + 1;
  }
  if (V != 2 && wt == 0) __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
#ifdef QZ_STAMPS8P
  if ((V == 0 || V == kPlainW) && lane == 0 && nsteps > 10 && (blockIdx.x == 0 || blockIdx.x == 100)) {
    for (int k = 0; k < 9; ++k) g_qz_stamp8p[((blockIdx.x ? 1 : 0) * 8 + wave) * 16 + k] = st8[k];
  }
#endif

  // ---- epilogue (as k_gemm_4bit_big): lane holds weight rows 16j + 4fk + r of token 16i + fr ----
  __syncthreads();
  unsigned char *ew = smem + wave * (64 * kBigERow);
  float bv[4][4];
  if constexpr (!kMF32) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = min(m0 + 64 * wm + 16 * j + 4 * fk + r, p.M - 1);
        bv[j][r] = p.bias ? load_f32<DT>(p.bias, m) : 0.0f;
      }
  } else {  // bv[jm * 2 + ... ]: rows 32 jm + 8 g + 4 h32 + r -> bv[2 jm + g / 2][...]: indexed below
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = 0.0f;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if constexpr (kMF32) {
#pragma unroll
      for (int jm = 0; jm < 2; ++jm)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f16v_t &v = acc32[jm][2 * h + i];
            const int row = 32 * jm + 8 * g + 4 * h32;
            float b4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
              b4[r] = p.bias ? load_f32<DT>(p.bias, min(m0 + 64 * wm + row + r, p.M - 1)) : 0.0f;
            const uint32_t lo = cvt_pk16<DT>(v[4 * g] + b4[0], v[4 * g + 1] + b4[1]);
            const uint32_t hi = cvt_pk16<DT>(v[4 * g + 2] + b4[2], v[4 * g + 3] + b4[3]);
            *reinterpret_cast<uint2 *>(ew + (32 * i + r32) * kBigERow + row * 2) = uint2{lo, hi};
          }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f4_t v = acc[j][4 * h + i];
          const uint32_t lo = cvt_pk16<DT>(v[0] + bv[j][0], v[1] + bv[j][1]);
          const uint32_t hi = cvt_pk16<DT>(v[2] + bv[j][2], v[3] + bv[j][3]);
          *reinterpret_cast<uint2 *>(ew + (16 * i + fr) * kBigERow + (16 * j + 4 * fk) * 2) = uint2{lo, hi};
        }
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int qd = lane + 64 * it, tok = qd >> 3, c16 = qd & 7;
      const v4u v = *reinterpret_cast<const v4u *>(ew + tok * kBigERow + c16 * 16);
      const int t = t0 + 128 * wt + 64 * h + tok, m = m0 + 64 * wm + 8 * c16;
      if (t < p.T && m < p.M)
        *reinterpret_cast<v4u *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_gemm16_4w: 256 x 256 tile, 4 waves (one per SIMD), each wave a 128-token x 128-row quadrant.
//
// Why not the 8-wave schedule for a dense 16-bit B: with 8 waves a step re-reads the staged tile
// 3x from LDS (each wave its 128 x 64 X and 64 x 64 W slices: 192 KB per 256 x 256 x 64 step);
// four 128 x 128 quadrants read 128 KB, the ratio hipBLASLt's MT256x256x64 tile runs at.  The
// 8-wave skeleton with no staging at all peaks at 1.58 PFLOP/s (gemm_micro SK 17,
// profiles/r2_gemm_nodma.txt) and its LDS-DMA staging costs a further 20 %.
//
// Registers per lane: 64 accumulators (8 x 8 16x16 tiles, the 256 AGPRs); the X fragments of
// the current and the next k-half (2 x 32); a 4-slot ring of W fragments streamed two MFMA rows
// ahead (16); the step-after-next's global bytes (16 x 16 B staging, global_load_dwordx4: no
// LDS-DMA issue cost).  A k-half is 8 rows j of 8 MFMAs (acc[j][*] += W_j . X_*), each row
// pinned by sched_barrier together with its share of the memory work:
//   half (s, 0): row j also writes staging chunk j (step s+1) into buffer (s+1)&1, refills it
//                with step s+2 (a whole step of latency cover), reads X fragment j of k-half 1
//                and W fragment j+2 (k-half 1 past 7); lgkmcnt(0); s_barrier
//   half (s, 1): row j reads X fragment j of step s+1's k-half 0 (buffer (s+1)&1) and the next W
//                fragment; s_barrier
// Buffer (s+1)&1 is rewritten in half (s, 0): its last reads were in half (s-1, 1) (behind the
// barrier ending it); buffer s&1 is rewritten in half (s+1, 0), behind the barrier ending (s, 1).
// The last steps load/write clamped (stale) data instead of branching.
constexpr int k4wT = 256, k4wM = 256;
constexpr int k4wStage = 256 * 128;                 // one buffer of X or W: 256 rows x 64 x 2 B
constexpr int k4wERow = 272;                        // epilogue image row: 128 outputs x 2 B + 16 B
constexpr int k4wLds = (4 * k4wStage > 4 * 128 * k4wERow) ? 4 * k4wStage : 4 * 128 * k4wERow;
template <int DT, int SK = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_gemm16_4w(GemmParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[k4wLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 1, wm = wave & 1;

  // XCD-aware, bijective tile order (as k_gemm_4bit_big)
  const int tiles_m = (p.M + k4wM - 1) / k4wM;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (wg % tiles_m) * k4wM, t0 = (wg / tiles_m) * k4wT;
  const int nsteps = p.K / kBK;

  // staging: thread t moves 16-B chunk (t & 7) of rows 32 c + t / 8, c = 0..7, of X and of W
  const unsigned char *xg = reinterpret_cast<const unsigned char *>(p.X);
  uint32_t xo[8], wo[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int row = 32 * c + (tid >> 3), ch = tid & 7;
    xo[c] = ((uint32_t)min(t0 + row, p.T - 1) * (uint32_t)p.ldx + 8u * ch) * 2u;
    wo[c] = ((uint32_t)min(m0 + row, p.M - 1) * (uint32_t)p.K + 8u * ch) * 2u;
  }
  const uint32_t lo = (uint32_t)lds_off(tid >> 3, tid & 7);  // + 4 KiB per c: same swizzle
  v4u xs[8], ws[8];
  // SK (timing only, gemm_micro): 1 = no staging in the loop, 2 = no fragment reads in the loop,
  // 4 = every step stages step 0 (L2-resident operands); 8 = LDS-DMA staging (rows 0..3 of half 0);
  // 16 = global loads only, 32 = LDS stores only
  typedef __attribute__((address_space(3))) void *lds_ptr_t;
  typedef __attribute__((address_space(1))) void *glb_ptr_t;
  const uint32_t dsw = 16u * (uint32_t)((tid & 7) ^ ((tid >> 4) & 7)) - 16u * (uint32_t)(tid & 7);
  auto dma = [&](int step, int buf, int c) {
    const uint32_t kb = (SK & 4) ? 0u : (uint32_t)step * (kBK * 2);
    unsigned char *bx = smem + buf * (2 * k4wStage) + 4096 * c + wave * 1024;
    // (dsw wraps: add the 32-bit offsets first, then to the pointer)
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(xg + (uint32_t)(xo[c] + dsw + kb)), (lds_ptr_t)bx, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(p.B + (uint32_t)(wo[c] + dsw + kb)), (lds_ptr_t)(bx + k4wStage), 16,
                                     0, 0);
  };
  auto gload = [&](int step, int c) {
    const uint32_t kb = (SK & 4) ? 0u : (uint32_t)step * (kBK * 2);
    xs[c] = *reinterpret_cast<const v4u *>(xg + xo[c] + kb);
    ws[c] = *reinterpret_cast<const v4u *>(p.B + wo[c] + kb);
  };
  auto swrite = [&](int buf, int c) {
    unsigned char *bx = smem + buf * (2 * k4wStage);
    *reinterpret_cast<v4u *>(bx + lo + 4096 * c) = xs[c];
    *reinterpret_cast<v4u *>(bx + k4wStage + lo + 4096 * c) = ws[c];
  };

  // fragments: lane (fr, fk) of a 16 x 32 operand holds row fr, k 8 fk .. +8 of the k-half
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t fl[2] = {(uint32_t)(fr * 128 + ((fk ^ ((fr >> 1) & 7)) << 4)),
                          (uint32_t)(fr * 128 + (((fk ^ ((fr >> 1) & 7)) ^ 4) << 4))};
  v4u xf[2][8], wr[4];
  auto xread = [&](int buf, int kk, int i) {
    xf[kk][i] = *reinterpret_cast<const v4u *>(smem + buf * (2 * k4wStage) + (128 * wt + 16 * i) * 128 + fl[kk]);
  };
  auto wread = [&](int buf, int kk, int j) {  // W fragment j of k-half kk into ring slot (8 kk + j) & 3
    wr[j & 3] = *reinterpret_cast<const v4u *>(smem + buf * (2 * k4wStage) + k4wStage + (128 * wm + 16 * j) * 128 +
                                               fl[kk]);
  };
  f4_t acc[8][8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f4_t{0.f, 0.f, 0.f, 0.f};
  auto mfma_row = [&](int kk, int j) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (DT == QZ_DT_F16)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, wr[j & 3]),
                                                           __builtin_bit_cast(h8_t, xf[kk][i]), acc[j][i], 0, 0, 0);
      else
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, wr[j & 3]),
                                                            __builtin_bit_cast(b8_t, xf[kk][i]), acc[j][i], 0, 0, 0);
    }
  };

  // ---- prologue: step 0 in buffer 0, step 1 in the staging registers, k-half 0's X + W 0, 1 read ----
#pragma unroll
  for (int c = 0; c < 8; ++c) gload(0, c);
#pragma unroll
  for (int c = 0; c < 8; ++c) swrite(0, c);
#pragma unroll
  for (int c = 0; c < 8; ++c) gload(min(1, nsteps - 1), c);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) xread(0, 0, i);
  wread(0, 0, 0);
  wread(0, 0, 1);

  for (int s = 0; s < nsteps; ++s) {
    const int b = s & 1;
    const int s2 = min(s + 2, nsteps - 1);
    // ---- half (s, 0) ----
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((SK & 8) != 0) {
        if (j < 4) {
          dma(min(s + 1, nsteps - 1), b ^ 1, 2 * j);
          dma(min(s + 1, nsteps - 1), b ^ 1, 2 * j + 1);
        }
      } else if constexpr ((SK & 16) != 0) {  // loads only: the registers consumed by an empty asm
        asm volatile("" ::"v"(xs[j]), "v"(ws[j]));
        gload(s2, j);
      } else if constexpr ((SK & 32) != 0) {  // LDS stores only (stale registers)
        swrite(b ^ 1, j);
      } else if constexpr ((SK & 1) == 0) {
        swrite(b ^ 1, j);
        gload(s2, j);
      }
      if constexpr ((SK & 2) == 0) {
        xread(b, 1, j);
        if (j < 6) wread(b, 0, j + 2); else wread(b, 1, j - 6);
      }
      mfma_row(0, j);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((SK & 8) != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- half (s, 1) ----
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((SK & 2) == 0) {
        xread(b ^ 1, 0, j);
        if (j < 6) wread(b, 1, j + 2); else wread(b ^ 1, 0, j - 6);
      }
      mfma_row(1, j);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // ---- epilogue: quadrant -> LDS image [128 tokens][128 rows] (+ bias) -> coalesced rows ----
  __syncthreads();
  unsigned char *ew = smem + wave * (128 * k4wERow);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bv[r] = p.bias ? load_f32<DT>(p.bias, min(m0 + 128 * wm + 16 * j + 4 * fk + r, p.M - 1)) : 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f4_t v = acc[j][i];
      const uint32_t l2 = cvt_pk16<DT>(v[0] + bv[0], v[1] + bv[1]);
      const uint32_t h2 = cvt_pk16<DT>(v[2] + bv[2], v[3] + bv[3]);
      *reinterpret_cast<uint2 *>(ew + (16 * i + fr) * k4wERow + (16 * j + 4 * fk) * 2) = uint2{l2, h2};
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int qd = lane + 64 * it, tok = qd >> 4, c16 = qd & 15;
    const v4u v = *reinterpret_cast<const v4u *>(ew + tok * k4wERow + c16 * 16);
    const int t = t0 + 128 * wt + tok, m = m0 + 128 * wm + 8 * c16;
    if (t < p.T && m < p.M) *reinterpret_cast<v4u *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// k_gemm16_4d: the 4-wave 256 x 256 tile (each wave a 128-token x 128-row quadrant, the 256
// accumulator registers in AGPRs) staged ONLY by LDS DMA, two steps ahead with two buffers.
//
// A wave holds a whole step's fragments in registers (X and W, both k-halves: 128 VGPRs), so a
// buffer is free for the next DMA as soon as every wave has read it -- not when its MFMAs are
// done.  Step s (buffer b = s & 1) is three segments:
//   A: k-half 0 MFMAs of rows 0-3 (32) with the 16 ds_read_b128 of k-half 1 from buffer b;
//      lgkmcnt(0) + s_barrier: every wave has buffer b in registers
//   B: k-half 0 MFMAs of rows 4-7 (32) with the 16 DMAs of step s + 2 into buffer b;
//      vmcnt(16) (this wave's step s + 1 DMAs, issued one step earlier, have landed) + s_barrier
//   C: k-half 1 MFMAs (64) with the 16 ds_read_b128 of step s + 1's k-half 0 from buffer b ^ 1
// so a DMA has ~1.5 steps of MFMAs to land, nothing but the staging bytes goes through LDS,
// and the loop carries no VALU address arithmetic: the DMAs are buffer loads whose per-lane
// part (row, swizzled chunk) is a fixed VGPR and whose k offset is a scalar (soffset).
// Rows past T or M are clamped (their outputs are not stored); the LDS image and fragment
// addresses are those of k_gemm16_4w (16-B chunk XOR swizzle applied to the DMA source).
// compile-time loop: f(std::integral_constant<int, 0>{}) .. f(<N - 1>) (a 128-iteration body
// is past the unroller's budget for #pragma unroll, and every index below must be a constant)
template <typename F, int... Ns>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, Ns...>) {
  (f(std::integral_constant<int, Ns>{}), ...);
}
template <int N, typename F> __device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
constexpr int k4dBuf = 2 * k4wStage;  // X image + W image of one step
constexpr int k4dLds = (2 * k4dBuf > 4 * 128 * k4wERow) ? 2 * k4dBuf : 4 * 128 * k4wERow;

// Split-release step schedule (S = 1): what each wave issues after the c-th of a step's 128
// MFMAs (16x16x32).  The buffer being read is released per OPERAND: once every wave holds its
// k-half-1 X fragments the X image takes step s + 2's DMAs, the W image once the W fragments are
// in; every LDS read has >= 6 MFMAs of cover before the lgkmcnt(0) that precedes a barrier; the
// one vmcnt wait (13: this step's DMAs issued so far) sits 34 MFMAs before the end, so the 16
// reads of step s + 1's k-half 0 spread over the rest of the step.  Codes: 1+i read X(k-half 1)
// i; 9+j read W(k-half 1) j; 17+i read X(next, k-half 0) i; 25+j read W(next) j; 33+c DMA X
// piece c; 41+c DMA W piece c; 49 lgkmcnt(0) + barrier; 50 vmcnt(13) + barrier.
struct Gemm4Sched {
  unsigned char ev[129];
};
constexpr Gemm4Sched gemm4_sched_split() {
  Gemm4Sched t{};
  const int rx1[8] = {1, 3, 5, 7, 9, 11, 13, 15};
  const int rw1[8] = {25, 28, 31, 34, 37, 39, 41, 43};
  const int dx[8] = {23, 26, 29, 32, 35, 53, 56, 59};
  const int dw[8] = {62, 65, 86, 88, 90, 97, 101, 125};
  const int rx0[8] = {94, 95, 96, 98, 99, 103, 104, 105};
  const int rw0[8] = {106, 107, 110, 113, 115, 118, 121, 124};
  for (int i = 0; i < 8; ++i) {
    t.ev[rx1[i]] = (unsigned char)(1 + i);
    t.ev[rw1[i]] = (unsigned char)(9 + i);
    t.ev[rx0[i]] = (unsigned char)(17 + i);
    t.ev[rw0[i]] = (unsigned char)(25 + i);
    t.ev[dx[i]] = (unsigned char)(33 + i);
    t.ev[dw[i]] = (unsigned char)(41 + i);
  }
  t.ev[21] = 49;
  t.ev[51] = 49;
  t.ev[92] = 50;
  return t;
}
constexpr Gemm4Sched kGemm4Split = gemm4_sched_split();
// The same schedule with every read / DMA one MFMA later where that slot is free (the waits stay):
// S & 16 gives it to the waves on odd SIMDs, so the two SIMD pairs do not hit the LDS and the
// address path in the same cycles
constexpr Gemm4Sched gemm4_sched_shift(Gemm4Sched a) {
  Gemm4Sched t{};
  for (int c = 128; c >= 1; --c) {
    const int e = a.ev[c];
    if (e == 0) continue;
    if (e < 49 && c + 1 <= 128 && a.ev[c + 1] == 0 && t.ev[c + 1] == 0 && c + 1 != 92 && c + 1 != 21 && c + 1 != 51)
      t.ev[c + 1] = (unsigned char)e;
    else
      t.ev[c] = (unsigned char)e;
  }
  return t;
}
constexpr Gemm4Sched kGemm4SplitB = gemm4_sched_shift(kGemm4Split);
constexpr int gemm4_sched_count(int code) {
  int n = 0;
  for (int c = 0; c < 129; ++c) n += kGemm4Split.ev[c] == code;
  return n;
}
constexpr int gemm4_sched_dmas_before(int c0) {
  int n = 0;
  for (int c = 0; c < c0; ++c) n += kGemm4Split.ev[c] >= 33 && kGemm4Split.ev[c] < 49;
  return n;
}
static_assert(gemm4_sched_count(0) == 129 - 51, "k_gemm16_4d split schedule: 51 events, one per slot");
constexpr int gemm4_sched_b_count(int code) {
  int n = 0;
  for (int c = 0; c < 129; ++c) n += kGemm4SplitB.ev[c] == code;
  return n;
}
constexpr int gemm4_sched_b_dmas_before(int c0) {
  int n = 0;
  for (int c = 0; c < c0; ++c) n += kGemm4SplitB.ev[c] >= 33 && kGemm4SplitB.ev[c] < 49;
  return n;
}
static_assert(gemm4_sched_b_count(0) == 129 - 51 && kGemm4SplitB.ev[128] == 0, "shifted schedule: 51 events");
static_assert(gemm4_sched_b_dmas_before(92) == 13 && kGemm4SplitB.ev[21] == 49 && kGemm4SplitB.ev[51] == 49 &&
              kGemm4SplitB.ev[92] == 50, "shifted schedule: the waits unchanged");
static_assert(gemm4_sched_dmas_before(92) == 13, "k_gemm16_4d split schedule: vmcnt(13) at the wait");

// QZ_STAMPS_G16 (microbenchmark builds only): s_memtime of each wave of workgroups 0-7 at the
// kernel start, after the prologue barrier, around the waits of step kStampStep, the loop end and
// the epilogue end -- where a step's cycles go
#ifdef QZ_STAMPS_G16
__device__ unsigned long long g_qz_stamp_g16[8 * 4 * 16];
constexpr int kStampStep = 20;
#define QZ_G16_STAMP(k) do { if (blockIdx.x < 8) g_qz_stamp_g16[(blockIdx.x * 4 + wave) * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define QZ_G16_STAMP_AT(k, st) do { if ((st) == kStampStep) QZ_G16_STAMP(k); } while (0)
#else
#define QZ_G16_STAMP(k) do { } while (0)
#define QZ_G16_STAMP_AT(k, st) do { } while (0)
#endif
template <int DT, int SK = 0, int P1 = 32, int P2 = 96, int S = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_gemm16_4d(GemmParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[k4dLds];
  typedef __attribute__((address_space(3))) void *lds_ptr_t;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 1, wm = wave & 1;
  QZ_G16_STAMP(0);
  QZ_G16_STAMP(0);

  // XCD-aware, bijective tile order (as k_gemm_4bit_big)
  const int tiles_m = (p.M + k4wM - 1) / k4wM;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm = wg % tiles_m, tt = wg / tiles_m;
  if constexpr ((SK & 64) != 0) {
    // grouped order: the 32 tiles an XCD runs together cover 4 token tiles x 8 row tiles
    const int tiles_t = (p.T + k4wT - 1) / k4wT;
    if (tiles_m % 8 == 0 && tiles_t % 4 == 0) {
      const int grp = wg / (4 * tiles_m), r = wg % (4 * tiles_m);
      tt = 4 * grp + (r % 32) / 8;
      tm = 8 * (r / 32) + r % 8;
    }
  }
  const int m0 = tm * k4wM, t0 = tt * k4wT;
  const int nsteps = p.K / kBK;

  // DMA c (0..7) of a thread moves 16-B chunk (tid & 7) of rows 32 c + tid / 8 of X and of W;
  // wave w's instruction c fills LDS rows 32 c + 8 w .. + 7 (1 KiB, lane-linear)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(p.X), (short)0, (int)((uint32_t)p.T * (uint32_t)p.ldx * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char *>(p.B), (short)0, (int)((uint32_t)p.M * (uint32_t)p.K * 2u), 0x00020000);
  const uint32_t sw = (uint32_t)((tid & 7) ^ ((tid >> 4) & 7));
  // S & 2: the W image's swizzle is chunk ^ f(row), f = row bits (1, 3, 4) -> chunk bits
  // (0, 1, 2), the one that keeps the permuted W fragment rows below conflict-free
  constexpr bool kPerm = (S & 2) != 0;
  const int wr = tid >> 3;
  const uint32_t sww = kPerm ? (uint32_t)((tid & 7) ^ (((wr >> 1) & 1) | (((wr >> 3) & 1) << 1) | (((wr >> 4) & 1) << 2)))
                             : sw;
  uint32_t xo[8], wo[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int row = 32 * c + (tid >> 3);
    xo[c] = ((uint32_t)min(t0 + row, p.T - 1) * (uint32_t)p.ldx + 8u * sw) * 2u;
    wo[c] = ((uint32_t)min(m0 + row, p.M - 1) * (uint32_t)p.K + 8u * sww) * 2u;
  }
  // h = 0: X rows, h = 1: W rows
  auto dma_half = [&](int step, int buf, int c, int h) {
    const int kb = (SK & 4) ? 0 : step * (kBK * 2);
    unsigned char *d = smem + buf * k4dBuf + 4096 * c + 1024 * wave;
    if (h == 0) __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)d, 16, xo[c], kb, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(d + k4wStage), 16, wo[c], kb, 0, 0);
  };
  auto dma = [&](int step, int buf, int c) {
    dma_half(step, buf, c, 0);
    dma_half(step, buf, c, 1);
  };

  // fragments: lane (fr, fk) of a 16 x 32 operand holds row fr, k 8 fk .. +8 of the k-half
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t fl[2] = {(uint32_t)(fr * 128 + ((fk ^ ((fr >> 1) & 7)) << 4)),
                          (uint32_t)(fr * 128 + (((fk ^ ((fr >> 1) & 7)) ^ 4) << 4))};
  // S & 2: W fragment j's lane fr reads row 32 (j / 2) + 8 (fr / 4) + 4 (j % 2) + fr % 4 of the
  // wave's 128 rows, so a lane's accumulators of fragments 2J and 2J + 1 hold 8 CONSECUTIVE
  // output rows: the epilogue stores them as one 16-B vector straight from the registers.
  const int fwz = ((fr >> 1) & 1) | (((fr >> 2) & 1) << 1) | (((fr >> 3) & 1) << 2);
  const uint32_t wl[2] = {(uint32_t)((8 * (fr >> 2) + (fr & 3)) * 128 + ((fk ^ fwz) << 4)),
                          (uint32_t)((8 * (fr >> 2) + (fr & 3)) * 128 + (((fk ^ fwz) ^ 4) << 4))};
  v4u xf[2][8], wf[2][8];
  // fragment reads: X tile i / W tile j of k-half kk from buffer buf
  auto read_x = [&](int buf, int kk, int i) {
    xf[kk][i] = *reinterpret_cast<const v4u *>(smem + buf * k4dBuf + fl[kk] + (128 * wt + 16 * i) * 128);
  };
  auto read_w = [&](int buf, int kk, int j) {
    const unsigned char *bw = smem + buf * k4dBuf + k4wStage;
    if constexpr (kPerm)
      wf[kk][j] = *reinterpret_cast<const v4u *>(bw + wl[kk] + (128 * wm + 32 * (j >> 1) + 4 * (j & 1)) * 128);
    else
      wf[kk][j] = *reinterpret_cast<const v4u *>(bw + fl[kk] + (128 * wm + 16 * j) * 128);
  };
  // SK & 32: v_mfma_f32_32x32x16 (64 MFMAs of 32 cycles per step instead of 128 of 16: half the
  // MFMA issue holds, more issue room for the DMAs and reads).  A/B lane (r32, h32) holds row
  // r32, k = 8 h32 .. +8 of k16 slice 2 kk + q (chunk 2 (2 kk + q) + h32, same swizzle); the 8
  // fragments of a k-half per operand are [q][tile].  D: lane holds token r32 of its 32-token
  // tile, rows 8 g + 4 h32 + r (register 4 g + r).
  constexpr bool kM32 = (SK & 32) != 0;
  constexpr int kNM = kM32 ? 64 : 128;  // MFMAs per step
  typedef float f16v_t __attribute__((ext_vector_type(16)));
  const int r32 = lane & 31, h32 = lane >> 5;
  uint32_t fl32[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) fl32[q] = (uint32_t)(r32 * 128 + (((2 * q + h32) ^ ((r32 >> 1) & 7)) << 4));
  // read g of a k-half, in the order the MFMAs consume them.  16x16x32: W fragment 0, the 8 X
  // fragments (tokens 16 i ..), W fragments 1-7.  32x32x16, per k16 slice q (8 reads): W tile 0,
  // X tiles 0-3, W tiles 1-3 -> stored as xf[kk][4 q + i], wf[kk][4 q + j]
  auto frag_read = [&](int buf, int kk, int g) {
    const unsigned char *bs = smem + buf * k4dBuf;
    if constexpr (kM32) {
      const int q = g >> 3, h = g & 7;
      const uint32_t o = fl32[2 * kk + q];
      if (h >= 1 && h <= 4)
        xf[kk][4 * q + h - 1] = *reinterpret_cast<const v4u *>(bs + (128 * wt + 32 * (h - 1)) * 128 + o);
      else {
        const int j = h == 0 ? 0 : h - 4;
        wf[kk][4 * q + j] = *reinterpret_cast<const v4u *>(bs + k4wStage + (128 * wm + 32 * j) * 128 + o);
      }
      return;
    }
    if (g >= 1 && g <= 8) read_x(buf, kk, g - 1);
    else read_w(buf, kk, g == 0 ? 0 : g - 8);
  };
  f4_t acc[kM32 ? 1 : 8][kM32 ? 1 : 8];
  f16v_t acc32[kM32 ? 4 : 1][kM32 ? 4 : 1];
  if constexpr (kM32) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[j][i][e] = 0.0f;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = f4_t{0.f, 0.f, 0.f, 0.f};
  }
  // MFMA n of k-half kk.  16x16x32 (n < 64): row fragment j = n / 8, token fragment i = n % 8.
  // 32x32x16 (n < 32): slice q = n / 16, row tile j = (n / 4) % 4, token tile i = n % 4.
  // SK & 16: as inline asm with the accumulator tied to one AGPR quad ("+a").
  auto mfma = [&](int kk, int n) {
    if constexpr (kM32) {
      const int q = n >> 4, j = (n >> 2) & 3, i = n & 3;
      if constexpr (DT == QZ_DT_F16)
        acc32[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8_t, wf[kk][4 * q + j]),
                                                             __builtin_bit_cast(h8_t, xf[kk][4 * q + i]), acc32[j][i],
                                                             0, 0, 0);
      else
        acc32[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8_t, wf[kk][4 * q + j]),
                                                              __builtin_bit_cast(b8_t, xf[kk][4 * q + i]),
                                                              acc32[j][i], 0, 0, 0);
      return;
    }
    const int j = n >> 3, i = n & 7;
    if constexpr ((SK & 16) != 0) {
      if constexpr (DT == QZ_DT_F16)
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[j][i]) : "v"(wf[kk][j]), "v"(xf[kk][i]));
      else
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j][i]) : "v"(wf[kk][j]), "v"(xf[kk][i]));
    } else if constexpr (DT == QZ_DT_F16) {
      acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, wf[kk][j]),
                                                         __builtin_bit_cast(h8_t, xf[kk][i]), acc[j][i], 0, 0, 0);
    } else {
      acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, wf[kk][j]),
                                                          __builtin_bit_cast(b8_t, xf[kk][i]), acc[j][i], 0, 0, 0);
    }
  };
  // ---- prologue: steps 0 and 1 in flight, step 0's k-half 0 in registers ----
#pragma unroll
  for (int c = 0; c < 8; ++c) dma(0, 0, c);
#pragma unroll
  for (int c = 0; c < 8; ++c) dma(min(1, nsteps - 1), 1, c);
  __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
  __builtin_amdgcn_s_barrier();
  QZ_G16_STAMP(1);
#pragma unroll
  for (int g = 0; g < 16; ++g) frag_read(0, 0, g);
  if constexpr ((SK & 16) != 0) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

  // One loop body for every step (a peeled tail split the accumulators between AGPRs and
  // VGPRs): the last two steps stage clamped copies of the last step into buffers nobody reads
  // again, and the last step reads a k-half it does not use.  The kNM MFMAs of a step (k-half 0
  // then 1) carry, pinned in program order by sched_barrier:
  //   [0, P1)    the 16 k-half 1 fragment reads of buffer b;  lgkmcnt(0) + s_barrier
  //   [P1, P2)   step s + 2's 16 DMAs into buffer b;  vmcnt(16) + s_barrier
  //   [P2, kNM)  step s + 1's 16 k-half 0 fragment reads of buffer b ^ 1
  // (P2 >= kNM / 2: the k-half 0 registers are free; every DMA has a whole step of MFMAs to land.)
  static_assert(P1 % 16 == 0 && P1 > 0 && P1 <= kNM / 2 && (P2 - P1) % 16 == 0 && P2 > P1 && P2 >= kNM / 2 &&
                P2 < kNM && (kNM - P2) % 16 == 0, "k_gemm16_4d segment bounds");
  constexpr int kR1 = P1 / 16, kD = (P2 - P1) / 16, kR0 = (kNM - P2) / 16;
  static_assert(S == 0 || !kM32, "the split-release schedule and the W permutation are written for 16x16x32");
  static_assert((S & 8) == 0 || (S & 1) != 0, "the rotated loop is the split-release schedule's");
  // MFMA n of step s (buffer s & 1) and the event the split-release table puts after it, every
  // MFMA pinned in program order
  auto split_mfma = [&](auto nc, int s, auto tb) {
    constexpr int n = decltype(nc)::value;
    constexpr bool kB = decltype(tb)::value;
    const int b = s & 1;
    const int s2 = min(s + 2, nsteps - 1);
    if constexpr (n == 0) QZ_G16_STAMP_AT(2, s);
    if constexpr (n == 0) QZ_G16_STAMP_AT(9, s - 1);
    __builtin_amdgcn_sched_barrier(0);
    mfma(n / 64, n % 64);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int e = kB ? kGemm4SplitB.ev[n + 1] : kGemm4Split.ev[n + 1];
    if constexpr (e >= 1 && e <= 8) read_x(b, 1, e - 1);
    else if constexpr (e >= 9 && e <= 16) read_w(b, 1, e - 9);
    else if constexpr (e >= 17 && e <= 24) read_x(b ^ 1, 0, e - 17);
    else if constexpr (e >= 25 && e <= 32) read_w(b ^ 1, 0, e - 25);
    else if constexpr (e >= 33 && e <= 40) {
      if constexpr ((SK & 1) == 0) dma_half(s2, b, e - 33, 0);
    } else if constexpr (e >= 41 && e <= 48) {
      if constexpr ((SK & 1) == 0) dma_half(s2, b, e - 41, 1);
    } else if constexpr (e == 49) {
      QZ_G16_STAMP_AT(n < 40 ? 3 : 5, s);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      QZ_G16_STAMP_AT(n < 40 ? 4 : 6, s);
    } else if constexpr (e == 50) {
      QZ_G16_STAMP_AT(7, s);
      // vmcnt(13): the 13 DMAs this step has issued may stay in flight
      __builtin_amdgcn_s_waitcnt((SK & 1) ? 0xC07F : 0x0F7D);
      __builtin_amdgcn_s_barrier();
      QZ_G16_STAMP_AT(8, s);
    }
  };
  if constexpr ((S & 64) != 0) {
    // Each step ONE hand-ordered instruction stream (gemm16_asm_step.h, generated by
    // scripts/gen/gemm16_asm_step.py): the same MFMAs on the same accumulators in the same order
    // (bit-identical), the reads / DMAs / waits / barriers exactly where the schedule puts them, and no
    // wait the compiler would add.  S & 128: the library's two event orders, by the SIMD's low bit
    // (else kGemm4Split's); S & 2: the permuted W rows of the register epilogue.  Two buffers
    // alternate: a step reads its k-half 1 fragments from buffer b, the next step's k-half 0 from
    // b ^ 1, and refills b by DMA.
    typedef __attribute__((address_space(3))) unsigned char lds_uc;
    const uint32_t sb = (uint32_t)(uintptr_t)(lds_uc *)smem;
    // HW_ID bits 4..5: this wave's SIMD; DUAL runs the library's L1 order on odd SIMDs, L0 on even
    const uint32_t simd_odd = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg((0 << 11) | (4 << 6) | 4) & 1);
    uint32_t xb1[2], wb1[2], xb0[2], wb0[2], mb[2];
#pragma unroll
    for (int buf = 0; buf < 2; ++buf) {
      const uint32_t bb = sb + (uint32_t)(buf * k4dBuf);
      xb1[buf] = bb + fl[1] + (uint32_t)(128 * wt) * 128u;
      xb0[buf] = bb + fl[0] + (uint32_t)(128 * wt) * 128u;
      wb1[buf] = bb + (uint32_t)k4wStage + (kPerm ? wl[1] : fl[1]) + (uint32_t)(128 * wm) * 128u;
      wb0[buf] = bb + (uint32_t)k4wStage + (kPerm ? wl[0] : fl[0]) + (uint32_t)(128 * wm) * 128u;
      mb[buf] = __builtin_amdgcn_readfirstlane(bb + 1024u * (uint32_t)wave);
    }
#define QZ_G16_ASM_OPS(B_)                                                                                        \
  : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]), "+a"(acc[0][4]), "+a"(acc[0][5]),          \
    "+a"(acc[0][6]), "+a"(acc[0][7]), "+a"(acc[1][0]), "+a"(acc[1][1]), "+a"(acc[1][2]), "+a"(acc[1][3]),          \
    "+a"(acc[1][4]), "+a"(acc[1][5]), "+a"(acc[1][6]), "+a"(acc[1][7]), "+a"(acc[2][0]), "+a"(acc[2][1]),          \
    "+a"(acc[2][2]), "+a"(acc[2][3]), "+a"(acc[2][4]), "+a"(acc[2][5]), "+a"(acc[2][6]), "+a"(acc[2][7]),          \
    "+a"(acc[3][0]), "+a"(acc[3][1]), "+a"(acc[3][2]), "+a"(acc[3][3]), "+a"(acc[3][4]), "+a"(acc[3][5]),          \
    "+a"(acc[3][6]), "+a"(acc[3][7]), "+a"(acc[4][0]), "+a"(acc[4][1]), "+a"(acc[4][2]), "+a"(acc[4][3]),          \
    "+a"(acc[4][4]), "+a"(acc[4][5]), "+a"(acc[4][6]), "+a"(acc[4][7]), "+a"(acc[5][0]), "+a"(acc[5][1]),          \
    "+a"(acc[5][2]), "+a"(acc[5][3]), "+a"(acc[5][4]), "+a"(acc[5][5]), "+a"(acc[5][6]), "+a"(acc[5][7]),          \
    "+a"(acc[6][0]), "+a"(acc[6][1]), "+a"(acc[6][2]), "+a"(acc[6][3]), "+a"(acc[6][4]), "+a"(acc[6][5]),          \
    "+a"(acc[6][6]), "+a"(acc[6][7]), "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),          \
    "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]),                                            \
    "+v"(xf[0][0]), "+v"(xf[0][1]), "+v"(xf[0][2]), "+v"(xf[0][3]), "+v"(xf[0][4]), "+v"(xf[0][5]),                \
    "+v"(xf[0][6]), "+v"(xf[0][7]), "+v"(wf[0][0]), "+v"(wf[0][1]), "+v"(wf[0][2]), "+v"(wf[0][3]),                \
    "+v"(wf[0][4]), "+v"(wf[0][5]), "+v"(wf[0][6]), "+v"(wf[0][7]), "=&v"(xf[1][0]), "=&v"(xf[1][1]),                \
    "=&v"(xf[1][2]), "=&v"(xf[1][3]), "=&v"(xf[1][4]), "=&v"(xf[1][5]), "=&v"(xf[1][6]), "=&v"(xf[1][7]),                \
    "=&v"(wf[1][0]), "=&v"(wf[1][1]), "=&v"(wf[1][2]), "=&v"(wf[1][3]), "=&v"(wf[1][4]), "=&v"(wf[1][5]),                \
    "=&v"(wf[1][6]), "=&v"(wf[1][7])                                                                                  \
  : "v"(xb1[B_]), "v"(wb1[B_]), "v"(xb0[(B_) ^ 1]), "v"(wb0[(B_) ^ 1]), "v"(xo[0]), "v"(xo[1]), "v"(xo[2]),         \
    "v"(xo[3]), "v"(xo[4]), "v"(xo[5]), "v"(xo[6]), "v"(xo[7]), "v"(wo[0]), "v"(wo[1]), "v"(wo[2]), "v"(wo[3]),     \
    "v"(wo[4]), "v"(wo[5]), "v"(wo[6]), "v"(wo[7]), "s"(rx), "s"(rw), "s"(soff), "s"(mb[B_]), "s"(simd_odd)       \
  : "memory", "m0", "scc"
#define QZ_G16_ASM_PICK(SCH_, B_)                                                                                 \
  do {                                                                                                             \
    if constexpr (DT == QZ_DT_F16 && !kPerm) asm volatile(QZ_GEMM16_ASM_##SCH_##_NAT_F16 QZ_G16_ASM_OPS(B_));     \
    else if constexpr (DT == QZ_DT_F16) asm volatile(QZ_GEMM16_ASM_##SCH_##_PERM_F16 QZ_G16_ASM_OPS(B_));        \
    else if constexpr (!kPerm) asm volatile(QZ_GEMM16_ASM_##SCH_##_NAT_BF16 QZ_G16_ASM_OPS(B_));                  \
    else asm volatile(QZ_GEMM16_ASM_##SCH_##_PERM_BF16 QZ_G16_ASM_OPS(B_));                                       \
  } while (0)
#define QZ_G16_ASM_LOOP(SCH_)                                                                                     \
  do {                                                                                                             \
    int s = 0;                                                                                                     \
    for (; s + 1 < nsteps; s += 2) {                                                                               \
      {                                                                                                            \
        const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)min(s + 2, nsteps - 1) * (uint32_t)(kBK * 2)); \
        QZ_G16_ASM_PICK(SCH_, 0);                                                                                  \
      }                                                                                                            \
      {                                                                                                            \
        const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)min(s + 3, nsteps - 1) * (uint32_t)(kBK * 2)); \
        QZ_G16_ASM_PICK(SCH_, 1);                                                                                  \
      }                                                                                                            \
    }                                                                                                              \
    if (s < nsteps) {                                                                                              \
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)min(s + 2, nsteps - 1) * (uint32_t)(kBK * 2)); \
      QZ_G16_ASM_PICK(SCH_, 0);                                                                                    \
    }                                                                                                              \
  } while (0)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 is reserved: the compiler sets it before each of its own uses
    if constexpr ((S & 128) != 0) QZ_G16_ASM_LOOP(DUAL);
    else QZ_G16_ASM_LOOP(SPLIT);
#pragma clang diagnostic pop
#undef QZ_G16_ASM_LOOP
#undef QZ_G16_ASM_PICK
#undef QZ_G16_ASM_OPS
  } else if constexpr ((S & 8) != 0) {
    // Rotated loop: an iteration runs MFMAs [kRot, 128) of step s and [0, kRot) of step s + 1, so
    // the loop header sits right after a lgkmcnt(0) + barrier -- the compiler's conservative wait at
    // a loop header then finds no LDS read outstanding (at the step boundary it waited for every
    // read of step s + 1's k-half 0, ~100 cycles of the MFMA pipe per step).  Step 0's head and the
    // last step's tail are peeled.
    constexpr int kRot = 51;
    static_assert(kGemm4Split.ev[kRot] == 49, "rotate at a lgkmcnt(0) + barrier");
    auto steps = [&](auto tb) {
      static_for<kRot>([&](auto nc) { split_mfma(nc, 0, tb); });
      for (int s = 0; s + 1 < nsteps; ++s) {
        static_for<128 - kRot>([&](auto nc) {
          split_mfma(std::integral_constant<int, kRot + decltype(nc)::value>{}, s, tb);
        });
        static_for<kRot>([&](auto nc) { split_mfma(nc, s + 1, tb); });
      }
      static_for<128 - kRot>([&](auto nc) {
        split_mfma(std::integral_constant<int, kRot + decltype(nc)::value>{}, nsteps - 1, tb);
      });
    };
    if constexpr ((S & 16) != 0) {
      // HW_ID bit 4: the low bit of this wave's SIMD
      if (__builtin_amdgcn_s_getreg((0 << 11) | (4 << 6) | 4) & 1) steps(std::true_type{});
      else steps(std::false_type{});
    } else {
      steps(std::false_type{});
    }
  } else
  for (int s = 0; s < nsteps; ++s) {
    const int b = s & 1;
    const int s2 = min(s + 2, nsteps - 1);
    static_for<kNM>([&](auto nc) {
      constexpr int n = decltype(nc)::value;
      if constexpr ((S & 1) != 0) {
        split_mfma(nc, s, std::false_type{});
        return;
      }
      if constexpr (n == 0) QZ_G16_STAMP_AT(2, s);
      if constexpr (n == 0) QZ_G16_STAMP_AT(9, s - 1);
      mfma(n / (kNM / 2), n % (kNM / 2));
      if constexpr (n < P1) {
        if constexpr ((n + 1) % kR1 == 0) {
          if constexpr ((SK & 2) == 0) frag_read(b, 1, (n + 1) / kR1 - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (n == P1 - 1) {
          QZ_G16_STAMP_AT(3, s);
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
          __builtin_amdgcn_s_barrier();
          QZ_G16_STAMP_AT(4, s);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if constexpr (n < P2) {
        if constexpr ((n + 1 - P1) % kD == 0) {
          constexpr int d = (n + 1 - P1) / kD - 1;
          if constexpr ((SK & 1) == 0) dma_half(s2, b, d >> 1, d & 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (n == P2 - 1) {
          QZ_G16_STAMP_AT(7, s);
          __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
          __builtin_amdgcn_s_barrier();
          QZ_G16_STAMP_AT(8, s);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if constexpr ((n + 1 - P2) % kR0 == 0) {
        if constexpr ((SK & 2) == 0) frag_read(b ^ 1, 0, (n + 1 - P2) / kR0 - 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  }
  if constexpr ((SK & 16) != 0) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  QZ_G16_STAMP(10);
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
  QZ_G16_STAMP(11);

  if constexpr (kPerm) {
    // ---- epilogue straight from the accumulators: fragments 2J, 2J + 1 of token tile i give a
    // lane 8 consecutive rows of one token -> one 16-B store (16 tokens x 64 B per instruction)
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      const int m = m0 + 128 * wm + 32 * J + 8 * fk;
      float bv[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) bv[r] = p.bias ? load_f32<DT>(p.bias, min(m + r, p.M - 1)) : 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = t0 + 128 * wt + 16 * i + fr;
        const f4_t lo = acc[2 * J][i], hi = acc[2 * J + 1][i];
        const v4u o = v4u{cvt_pk16<DT>(lo[0] + bv[0], lo[1] + bv[1]), cvt_pk16<DT>(lo[2] + bv[2], lo[3] + bv[3]),
                          cvt_pk16<DT>(hi[0] + bv[4], hi[1] + bv[5]), cvt_pk16<DT>(hi[2] + bv[6], hi[3] + bv[7])};
        if constexpr ((SK & 128) != 0) {  // timing only: no global stores
          if (o.x == 0x7FFF7FFFu && o.y == 0x12345678u) *reinterpret_cast<v4u *>(p.Y) = o;
          continue;
        }
        if (t < p.T && m < p.M) *reinterpret_cast<v4u *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m) = o;
      }
    }
    QZ_G16_STAMP(12);
    return;
  }

  // ---- epilogue: quadrant -> LDS image [128 tokens][128 rows] (+ bias) -> coalesced rows ----
  __syncthreads();
  unsigned char *ew = smem + wave * (128 * k4wERow);
  if constexpr (kM32) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = 32 * j + 8 * g + 4 * h32;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = p.bias ? load_f32<DT>(p.bias, min(m0 + 128 * wm + row + r, p.M - 1)) : 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f16v_t &v = acc32[j][i];
          const uint32_t l2 = cvt_pk16<DT>(v[4 * g] + bv[0], v[4 * g + 1] + bv[1]);
          const uint32_t h2 = cvt_pk16<DT>(v[4 * g + 2] + bv[2], v[4 * g + 3] + bv[3]);
          *reinterpret_cast<uint2 *>(ew + (32 * i + r32) * k4wERow + row * 2) = uint2{l2, h2};
        }
      }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        bv[r] = p.bias ? load_f32<DT>(p.bias, min(m0 + 128 * wm + 16 * j + 4 * fk + r, p.M - 1)) : 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f4_t v = acc[j][i];
        const uint32_t l2 = cvt_pk16<DT>(v[0] + bv[0], v[1] + bv[1]);
        const uint32_t h2 = cvt_pk16<DT>(v[2] + bv[2], v[3] + bv[3]);
        *reinterpret_cast<uint2 *>(ew + (16 * i + fr) * k4wERow + (16 * j + 4 * fk) * 2) = uint2{l2, h2};
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int qd = lane + 64 * it, tok = qd >> 4, c16 = qd & 15;
    const v4u v = *reinterpret_cast<const v4u *>(ew + tok * k4wERow + c16 * 16);
    const int t = t0 + 128 * wt + tok, m = m0 + 128 * wm + 8 * c16;
    if constexpr ((SK & 128) != 0) {  // timing only: no global stores (the image is still read)
      if (v.x == 0x7FFF7FFFu && v.y == 0x12345678u) *reinterpret_cast<v4u *>(p.Y) = v;
      continue;
    }
    if (t < p.T && m < p.M) *reinterpret_cast<v4u *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m) = v;
  }
  QZ_G16_STAMP(12);
}

// ---------------------------------------------------------------------------------------------
// k_gemm16_4q: k_gemm16_4d<..., S = 64 | 2 (| 128)>'s hand-ordered asm step in a PERSISTENT
// workgroup (one per CU, as the library's MT256x256x64 kernel runs) that walks tiles id, id + grid,
// ... in the grouped XCD-aware order.  A tile's last two steps stage the NEXT tile's steps 0 and 1,
// so the k-half 0 fragments of its first step are in registers when the tile ends; the epilogue
// stores the permuted accumulators straight from the registers (no LDS, no barrier) and the next
// tile's first step starts its k-half 0 MFMAs from 0 (*_FIRST) instead of zeroing 256 AGPRs.  Same
// MFMAs in the same order per output as k_gemm16_4d: bit-identical.  Host contract: nsteps = K / 64
// even (every tile starts on buffer 0), grid <= tiles.  S & 128: DUAL (the library's two event
// orders by SIMD parity), else SPLIT.
struct Gemm4qOffs {
  uint32_t x[8], w[8];
};
template <int DT, int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_gemm16_4q(GemmParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * k4dBuf];
  typedef __attribute__((address_space(3))) void *lds_ptr_t;
  typedef __attribute__((address_space(3))) unsigned char lds_uc;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 1, wm = wave & 1;
  const int tiles_m = (p.M + k4wM - 1) / k4wM, tiles_t = (p.T + k4wT - 1) / k4wT;
  const int ntiles = tiles_m * tiles_t;
  const int nsteps = p.K / kBK;
  auto tile_of = [&](int id, int &m0, int &t0) {
    const int q8 = ntiles >> 3, r8 = ntiles & 7, xcd = id & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
    int tm = wg % tiles_m, tt = wg / tiles_m;
    if (tiles_m % 8 == 0 && tiles_t % 4 == 0) {
      const int grp = wg / (4 * tiles_m), r = wg % (4 * tiles_m);
      tt = 4 * grp + (r % 32) / 8;
      tm = 8 * (r / 32) + r % 8;
    }
    m0 = tm * k4wM;
    t0 = tt * k4wT;
  };
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(p.X), (short)0, (int)((uint32_t)p.T * (uint32_t)p.ldx * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char *>(p.B), (short)0, (int)((uint32_t)p.M * (uint32_t)p.K * 2u), 0x00020000);
  // k_gemm16_4d's DMA pieces and swizzles (X: chunk ^ row bits 1..3; W: the S & 2 one)
  const int wr = tid >> 3;
  const uint32_t sw = (uint32_t)((tid & 7) ^ ((tid >> 4) & 7));
  const uint32_t sww = (uint32_t)((tid & 7) ^ (((wr >> 1) & 1) | (((wr >> 3) & 1) << 1) | (((wr >> 4) & 1) << 2)));
  auto offs_of = [&](int m0, int t0, Gemm4qOffs &o) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int row = 32 * c + wr;
      o.x[c] = ((uint32_t)min(t0 + row, p.T - 1) * (uint32_t)p.ldx + 8u * sw) * 2u;
      o.w[c] = ((uint32_t)min(m0 + row, p.M - 1) * (uint32_t)p.K + 8u * sww) * 2u;
    }
  };
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t fl[2] = {(uint32_t)(fr * 128 + ((fk ^ ((fr >> 1) & 7)) << 4)),
                          (uint32_t)(fr * 128 + (((fk ^ ((fr >> 1) & 7)) ^ 4) << 4))};
  const int fwz = ((fr >> 1) & 1) | (((fr >> 2) & 1) << 1) | (((fr >> 3) & 1) << 2);
  const uint32_t wl[2] = {(uint32_t)((8 * (fr >> 2) + (fr & 3)) * 128 + ((fk ^ fwz) << 4)),
                          (uint32_t)((8 * (fr >> 2) + (fr & 3)) * 128 + (((fk ^ fwz) ^ 4) << 4))};
  v4u xf[2][8], wf[2][8];
  f4_t acc[8][8];
  const uint32_t sb = (uint32_t)(uintptr_t)(lds_uc *)smem;
  const uint32_t simd_odd = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg((0 << 11) | (4 << 6) | 4) & 1);
  uint32_t xb1[2], wb1[2], xb0[2], wb0[2], mb[2];
#pragma unroll
  for (int buf = 0; buf < 2; ++buf) {
    const uint32_t bb = sb + (uint32_t)(buf * k4dBuf);
    xb1[buf] = bb + fl[1] + (uint32_t)(128 * wt) * 128u;
    xb0[buf] = bb + fl[0] + (uint32_t)(128 * wt) * 128u;
    wb1[buf] = bb + (uint32_t)k4wStage + wl[1] + (uint32_t)(128 * wm) * 128u;
    wb0[buf] = bb + (uint32_t)k4wStage + wl[0] + (uint32_t)(128 * wm) * 128u;
    mb[buf] = __builtin_amdgcn_readfirstlane(bb + 1024u * (uint32_t)wave);
  }

  int id = blockIdx.x;
  if (id >= ntiles) return;
  int m0, t0, nm0 = 0, nt0 = 0;
  tile_of(id, m0, t0);
  Gemm4qOffs cur, nxt;
  offs_of(m0, t0, cur);
  // ---- first tile: steps 0 and 1 in flight, step 0's k-half 0 in registers ----
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    unsigned char *d = smem + 4096 * c + 1024 * wave;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)d, 16, cur.x[c], 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(d + k4wStage), 16, cur.w[c], 0, 0, 0);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    unsigned char *d = smem + k4dBuf + 4096 * c + 1024 * wave;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)d, 16, cur.x[c], kBK * 2, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(d + k4wStage), 16, cur.w[c], kBK * 2, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    xf[0][i] = *reinterpret_cast<const v4u *>(smem + fl[0] + (128 * wt + 16 * i) * 128);
    wf[0][i] = *reinterpret_cast<const v4u *>(smem + k4wStage + wl[0] + (128 * wm + 32 * (i >> 1) + 4 * (i & 1)) * 128);
  }

  // A_: "+a" for a step that accumulates, "=a" for a tile's first (*_FIRST: the previous tile's
  // sums are dead once stored, so nothing carries the accumulators across the epilogue).  The k-half 1
  // fragments are written (early, while the inputs are still read) before a step uses them: "=&v",
  // so they are dead between steps; the k-half 0 ones carry over to the next step: "+v".
#define QZ_G16Q_OPS(B_, O_, A_)                                                                                       \
  : A_(acc[0][0]), A_(acc[0][1]), A_(acc[0][2]), A_(acc[0][3]), A_(acc[0][4]), A_(acc[0][5]),          \
    A_(acc[0][6]), A_(acc[0][7]), A_(acc[1][0]), A_(acc[1][1]), A_(acc[1][2]), A_(acc[1][3]),          \
    A_(acc[1][4]), A_(acc[1][5]), A_(acc[1][6]), A_(acc[1][7]), A_(acc[2][0]), A_(acc[2][1]),          \
    A_(acc[2][2]), A_(acc[2][3]), A_(acc[2][4]), A_(acc[2][5]), A_(acc[2][6]), A_(acc[2][7]),          \
    A_(acc[3][0]), A_(acc[3][1]), A_(acc[3][2]), A_(acc[3][3]), A_(acc[3][4]), A_(acc[3][5]),          \
    A_(acc[3][6]), A_(acc[3][7]), A_(acc[4][0]), A_(acc[4][1]), A_(acc[4][2]), A_(acc[4][3]),          \
    A_(acc[4][4]), A_(acc[4][5]), A_(acc[4][6]), A_(acc[4][7]), A_(acc[5][0]), A_(acc[5][1]),          \
    A_(acc[5][2]), A_(acc[5][3]), A_(acc[5][4]), A_(acc[5][5]), A_(acc[5][6]), A_(acc[5][7]),          \
    A_(acc[6][0]), A_(acc[6][1]), A_(acc[6][2]), A_(acc[6][3]), A_(acc[6][4]), A_(acc[6][5]),          \
    A_(acc[6][6]), A_(acc[6][7]), A_(acc[7][0]), A_(acc[7][1]), A_(acc[7][2]), A_(acc[7][3]),          \
    A_(acc[7][4]), A_(acc[7][5]), A_(acc[7][6]), A_(acc[7][7]),                                            \
    "+v"(xf[0][0]), "+v"(xf[0][1]), "+v"(xf[0][2]), "+v"(xf[0][3]), "+v"(xf[0][4]), "+v"(xf[0][5]),                \
    "+v"(xf[0][6]), "+v"(xf[0][7]), "+v"(wf[0][0]), "+v"(wf[0][1]), "+v"(wf[0][2]), "+v"(wf[0][3]),                \
    "+v"(wf[0][4]), "+v"(wf[0][5]), "+v"(wf[0][6]), "+v"(wf[0][7]), "=&v"(xf[1][0]), "=&v"(xf[1][1]),                \
    "=&v"(xf[1][2]), "=&v"(xf[1][3]), "=&v"(xf[1][4]), "=&v"(xf[1][5]), "=&v"(xf[1][6]), "=&v"(xf[1][7]),                \
    "=&v"(wf[1][0]), "=&v"(wf[1][1]), "=&v"(wf[1][2]), "=&v"(wf[1][3]), "=&v"(wf[1][4]), "=&v"(wf[1][5]),                \
    "=&v"(wf[1][6]), "=&v"(wf[1][7])                                                                                  \
  : "v"(xb1[B_]), "v"(wb1[B_]), "v"(xb0[(B_) ^ 1]), "v"(wb0[(B_) ^ 1]), "v"(O_.x[0]), "v"(O_.x[1]), "v"(O_.x[2]),   \
    "v"(O_.x[3]), "v"(O_.x[4]), "v"(O_.x[5]), "v"(O_.x[6]), "v"(O_.x[7]), "v"(O_.w[0]), "v"(O_.w[1]), "v"(O_.w[2]), \
    "v"(O_.w[3]), "v"(O_.w[4]), "v"(O_.w[5]), "v"(O_.w[6]), "v"(O_.w[7]), "s"(rx), "s"(rw), "s"(soff), "s"(mb[B_]),  \
    "s"(simd_odd)                                                                                                   \
  : "memory", "m0", "scc"
  // one step on buffer B_ whose DMAs fetch step DS_ of the tile O_ describes
#define QZ_G16Q_STEP(SCH_, B_, O_, DS_, A_)                                                                       \
  do {                                                                                                             \
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(DS_) * (uint32_t)(kBK * 2));                  \
    if constexpr (DT == QZ_DT_F16) asm volatile(QZ_GEMM16_ASM_##SCH_##_F16 QZ_G16Q_OPS(B_, O_, A_));              \
    else asm volatile(QZ_GEMM16_ASM_##SCH_##_BF16 QZ_G16Q_OPS(B_, O_, A_));                                       \
  } while (0)
  // a tile: step 0 from zero, steps 1 .. nsteps - 3 staging this tile's steps + 2, the last two
  // staging the next tile's steps 0 and 1
#define QZ_G16Q_TILE(SCH_)                                                                                        \
  do {                                                                                                             \
    if (nsteps > 2) {                                                                                              \
      QZ_G16Q_STEP(SCH_##_PERM_FIRST, 0, cur, 2, "=a");                                                                  \
      QZ_G16Q_STEP(SCH_##_PERM, 1, cur, 3, "+a");                                                                        \
      for (int s = 2; s + 2 < nsteps; s += 2) {                                                                    \
        QZ_G16Q_STEP(SCH_##_PERM, 0, cur, s + 2, "+a");                                                                  \
        QZ_G16Q_STEP(SCH_##_PERM, 1, cur, s + 3, "+a");                                                                  \
      }                                                                                                            \
      QZ_G16Q_STEP(SCH_##_PERM, 0, nxt, 0, "+a");                                                                        \
    } else {                                                                                                       \
      QZ_G16Q_STEP(SCH_##_PERM_FIRST, 0, nxt, 0, "=a");                                                                  \
    }                                                                                                              \
    QZ_G16Q_STEP(SCH_##_PERM, 1, nxt, 1, "+a");                                                                          \
  } while (0)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 is reserved: the compiler sets it before each of its own uses
  for (;;) {
    const int nid = id + (int)gridDim.x;
    const bool more = nid < ntiles;
    if (more) {
      tile_of(nid, nm0, nt0);
      offs_of(nm0, nt0, nxt);
    } else {
      nxt = cur;  // clamped copies of this tile's steps 0 and 1 into buffers nobody reads again
    }
    if constexpr ((S & 256) != 0) QZ_G16Q_TILE(DUALW);   // W's k-half 1 reads and refill first
    else if constexpr ((S & 128) != 0) QZ_G16Q_TILE(DUAL);
    else QZ_G16Q_TILE(SPLIT);
    // the MFMA results' read-after-write wait before the accumulators are read (the asm's own
    // tail covers most of it)
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    // ---- epilogue straight from the accumulators (k_gemm16_4d's S & 2 one): 16-B stores of 8
    // consecutive rows; the next tile's first step overwrites the accumulators ----
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      const int m = m0 + 128 * wm + 32 * J + 8 * fk;
      float bv[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) bv[r] = p.bias ? load_f32<DT>(p.bias, min(m + r, p.M - 1)) : 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = t0 + 128 * wt + 16 * i + fr;
        const f4_t lo = acc[2 * J][i], hi = acc[2 * J + 1][i];
        const v4u o = v4u{cvt_pk16<DT>(lo[0] + bv[0], lo[1] + bv[1]), cvt_pk16<DT>(lo[2] + bv[2], lo[3] + bv[3]),
                          cvt_pk16<DT>(hi[0] + bv[4], hi[1] + bv[5]), cvt_pk16<DT>(hi[2] + bv[6], hi[3] + bv[7])};
        if (t < p.T && m < p.M) {
          v4u *dst = reinterpret_cast<v4u *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m);
          if constexpr ((S & 8) != 0) __builtin_nontemporal_store(o, dst);   // S & 8: streaming stores
          else *dst = o;
        }
      }
    }
    if (!more) break;
    id = nid;
    m0 = nm0;
    t0 = nt0;
    cur = nxt;
  }
#pragma clang diagnostic pop
#undef QZ_G16Q_TILE
#undef QZ_G16Q_STEP
#undef QZ_G16Q_OPS
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): the clamped DMAs land before the workgroup ends
}

// ---------------------------------------------------------------------------------------------
// k_gemm16_4p: k_gemm16_4d's step (P1 = 16, P2 = 112, 16x16x32) in a persistent workgroup that
// walks tiles id, id + grid, ... (grouped XCD-aware order).  The last two steps of a tile stage
// the NEXT tile's steps 0 and 1, so its k-half 0 fragments are in registers when the tile ends,
// and the epilogue stores straight from the accumulators (8-B stores: 16 tokens x 32 B per
// instruction, merged in L2) without the LDS image -- no prologue wait, no epilogue barrier.
struct Gemm4pOffs {
  uint32_t x[8], w[8];
};
template <int DT, int SK = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_gemm16_4p(GemmParams p) {
  constexpr int P1 = 16, P2 = 112;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * k4dBuf];
  typedef __attribute__((address_space(3))) void *lds_ptr_t;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave >> 1, wm = wave & 1;
  const int tiles_m = (p.M + k4wM - 1) / k4wM, tiles_t = (p.T + k4wT - 1) / k4wT;
  const int ntiles = tiles_m * tiles_t;
  const int nsteps = p.K / kBK;
  // tile id -> (m0, t0): XCD-aware bijection, then the grouped order (4 token x 8 row tiles)
  auto tile_of = [&](int id, int &m0, int &t0) {
    const int q8 = ntiles >> 3, r8 = ntiles & 7, xcd = id & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
    int tm = wg % tiles_m, tt = wg / tiles_m;
    if (tiles_m % 8 == 0 && tiles_t % 4 == 0) {
      const int grp = wg / (4 * tiles_m), r = wg % (4 * tiles_m);
      tt = 4 * grp + (r % 32) / 8;
      tm = 8 * (r / 32) + r % 8;
    }
    m0 = tm * k4wM;
    t0 = tt * k4wT;
  };
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(p.X), (short)0, (int)((uint32_t)p.T * (uint32_t)p.ldx * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char *>(p.B), (short)0, (int)((uint32_t)p.M * (uint32_t)p.K * 2u), 0x00020000);
  const uint32_t sw = (uint32_t)((tid & 7) ^ ((tid >> 4) & 7));
  // per-lane DMA offsets of a tile (rows clamped into the tensors)
  typedef Gemm4pOffs Offs;
  auto offs_of = [&](int m0, int t0, Offs &o) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int row = 32 * c + (tid >> 3);
      o.x[c] = ((uint32_t)min(t0 + row, p.T - 1) * (uint32_t)p.ldx + 8u * sw) * 2u;
      o.w[c] = ((uint32_t)min(m0 + row, p.M - 1) * (uint32_t)p.K + 8u * sw) * 2u;
    }
  };
  auto dma_half = [&](const Offs &o, int step, int buf, int c, int h) {
    const int kb = step * (kBK * 2);
    unsigned char *d = smem + buf * k4dBuf + 4096 * c + 1024 * wave;
    if (h == 0) __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)d, 16, o.x[c], kb, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(d + k4wStage), 16, o.w[c], kb, 0, 0);
  };
  const int fr = lane & 15, fk = lane >> 4;
  const uint32_t fl[2] = {(uint32_t)(fr * 128 + ((fk ^ ((fr >> 1) & 7)) << 4)),
                          (uint32_t)(fr * 128 + (((fk ^ ((fr >> 1) & 7)) ^ 4) << 4))};
  v4u xf[2][8], wf[2][8];
  auto frag_read = [&](int buf, int kk, int g) {
    const unsigned char *bx = smem + buf * k4dBuf + fl[kk];
    const int wj = g == 0 ? 0 : g - 8;
    if (g >= 1 && g <= 8) xf[kk][g - 1] = *reinterpret_cast<const v4u *>(bx + (128 * wt + 16 * (g - 1)) * 128);
    else wf[kk][wj] = *reinterpret_cast<const v4u *>(bx + k4wStage + (128 * wm + 16 * wj) * 128);
  };
  f4_t acc[8][8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f4_t{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](int kk, int n) {
    const int j = n >> 3, i = n & 7;
    if constexpr (DT == QZ_DT_F16)
      acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, wf[kk][j]),
                                                         __builtin_bit_cast(h8_t, xf[kk][i]), acc[j][i], 0, 0, 0);
    else
      acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, wf[kk][j]),
                                                          __builtin_bit_cast(b8_t, xf[kk][i]), acc[j][i], 0, 0, 0);
  };

  int id = blockIdx.x;
  if (id >= ntiles) return;
  int m0, t0, nm0 = 0, nt0 = 0;
  tile_of(id, m0, t0);
  Offs cur, nxt;
  offs_of(m0, t0, cur);
  // ---- first tile: steps 0 and 1 in flight, step 0's k-half 0 in registers ----
#pragma unroll
  for (int c = 0; c < 8; ++c) { dma_half(cur, 0, 0, c, 0); dma_half(cur, 0, 0, c, 1); }
#pragma unroll
  for (int c = 0; c < 8; ++c) { dma_half(cur, min(1, nsteps - 1), 1, c, 0); dma_half(cur, min(1, nsteps - 1), 1, c, 1); }
  __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int g = 0; g < 16; ++g) frag_read(0, 0, g);

  int gs = 0;  // global step: buffer parity across tiles
  for (;;) {
    const int nid = id + (int)gridDim.x;
    const bool more = nid < ntiles;
    if (more) {
      tile_of(nid, nm0, nt0);
      offs_of(nm0, nt0, nxt);
    } else {
      nxt = cur;
    }
    for (int s = 0; s < nsteps; ++s, ++gs) {
      const int b = gs & 1;
      // DMA source: step s + 2 of this tile, else step s + 2 - nsteps of the next (clamped
      // copies of this tile's last step after the last tile)
      const bool into_next = s + 2 >= nsteps;
      const Offs &so = into_next ? nxt : cur;
      const int s2 = into_next ? (more ? s + 2 - nsteps : nsteps - 1) : s + 2;
      static_for<128>([&](auto nc) {
        constexpr int n = decltype(nc)::value;
        mfma(n >> 6, n & 63);
        if constexpr (n < P1) {
          frag_read(b, 1, n);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (n == P1 - 1) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
          }
        } else if constexpr (n < P2) {
          if constexpr ((n + 1 - P1) % 6 == 0) {
            constexpr int d = (n + 1 - P1) / 6 - 1;
            dma_half(so, s2, b, d >> 1, d & 1);
            __builtin_amdgcn_sched_barrier(0);
          }
          if constexpr (n == P2 - 1) {
            __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {
          frag_read(b ^ 1, 0, n - P2);
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    }
    // ---- epilogue: accumulators (+ bias) -> Y, 8 B per lane per store; then zero them ----
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + 128 * wm + 16 * j + 4 * fk;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = p.bias ? load_f32<DT>(p.bias, min(m + r, p.M - 1)) : 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = t0 + 128 * wt + 16 * i + fr;
        const f4_t v = acc[j][i];
        const uint2 o = uint2{cvt_pk16<DT>(v[0] + bv[0], v[1] + bv[1]), cvt_pk16<DT>(v[2] + bv[2], v[3] + bv[3])};
        if ((SK & 128) == 0 && t < p.T && m < p.M)
          *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(p.Y) + (size_t)t * p.ldy + m) = o;
        acc[j][i] = f4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (!more) break;
    id = nid;
    m0 = nm0;
    t0 = nt0;
    cur = nxt;
  }
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
}

// Multi-token GEMV for 2 <= T <= 16 (small-batch decode, short prefills).
// A 512-thread workgroup owns 16 weight rows; its 8 waves split K and meet in
// LDS (no workspace, no second launch).  Per 256-element chunk, lane
// (r = l % 16, g = l / 16) of a wave loads the 32 B of row r holding codes
// 64g .. 64g+63 -- one whole scale block, and with its 3 neighbours a full
// 128-B line of the row -- builds that block's exact 16-bit table and decodes
// its 8 dwords into the A fragments of 8 v_mfma_f32_16x16x32 (A = weights, M
// dimension; B = the T tokens, N dimension, zero-padded to 16).  Every token
// rides on the same decode: T tokens cost about one GEMV.
//
// The B fragments (lane (c, g) of MFMA j needs x[c][64g + 8j .. +8]) touch 64
// different lines per wave instruction when loaded straight from memory.
// TB > 0 (production): the wave instead stages its chunk of X -- TB token
// rows x 512 B, loaded with plain coalesced 16-B loads (two token rows per
// wave instruction) together with the weights -- into a wave-private LDS
// image in the decode's pair order, and reads the fragments from there
// (ds_read_b128, rows padded to 528 B: conflict-free); lanes c >= T read a
// zero row.  TB = 0: the direct fragment loads (kept for the microbenchmark).
constexpr int kMtChunk = 256, kMtWaves = 8;
constexpr int kMtXRow = kMtChunk * 2 + 16;  // padded LDS row of one token's chunk of X
template <int QT, bool DQ, int DT, int TB = 0, int W = kMtWaves>
__device__ __forceinline__ void mt_body(const GemmParams &p, const int block) {
  constexpr int XL = TB > 0 ? (TB + 1) / 2 : 1;  // staging loads per lane per chunk (two token rows each)
  __shared__ float s_code2[DQ ? 256 : 1];
  __shared__ f4_t s_red[W][64];
  __shared__ __attribute__((aligned(16))) unsigned char s_xs[TB > 0 ? W * (TB + 1) * kMtXRow : 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int m0 = block * 16;
  const int nch = p.K / kMtChunk;
  const int ch0 = wave * nch / W, ch1 = (wave + 1) * nch / W;
  const int wrow = min(m0 + r, p.M - 1);
  const uint32_t row_bytes = (uint32_t)p.K >> 1;
  const unsigned char *wptr = p.B + (size_t)wrow * row_bytes + 32 * g;
  const long long ebase = (long long)wrow * p.K + 64 * g;
  const bool tok = r < p.T;  // as a B-operand lane, lane l carries token c = l % 16
  const uint16_t *xrow = reinterpret_cast<const uint16_t *>(p.X) + (size_t)min(r, p.T - 1) * p.ldx + 64 * g;
  // TB > 0: staging lane map -- load i covers token rows 2i, 2i+1; lane l -> row 2i + l/32, 16-B piece l % 32
  unsigned char *xs = s_xs + (TB > 0 ? wave * (TB + 1) * kMtXRow : 0);
  const int spc = lane & 31, shalf = lane >> 5;
  const uint16_t *xstage = reinterpret_cast<const uint16_t *>(p.X) + 8 * spc;
  // fragment reads: token row c (< T) or the zero row TB
  const uint32_t frag_off = (uint32_t)((tok ? r : TB) * kMtXRow + g * 128);

  // two NAMED stages (a dynamically indexed register array would live in scratch)
  struct Stage {
    v4u w[2];
    v4u x[XL];
    uint32_t q;
    float a;
    int ch;
  };
  auto load = [&](Stage &st, int ch) {
    const v4u *wp = reinterpret_cast<const v4u *>(wptr + ch * (kMtChunk / 2));
    st.w[0] = __builtin_nontemporal_load(wp);
    st.w[1] = __builtin_nontemporal_load(wp + 1);
    st.ch = ch;
    const uint32_t b = (uint32_t)(p.block_base + ((ebase + ch * kMtChunk) >> p.bs_log2));
    if constexpr (DQ) {
      st.q = p.sc.qabsmax[b];
      st.a = p.sc.absmax2[b >> p.bs2_log2];
    } else {
      st.q = 0u;
      st.a = p.sc.absmax[b];
    }
    if constexpr (TB > 0) {
#pragma unroll
      for (int i = 0; i < XL; ++i) {  // rows >= T re-read row T-1 (never stored to LDS)
        const int t = min(2 * i + shalf, p.T - 1);
        st.x[i] = *reinterpret_cast<const v4u *>(xstage + (size_t)t * p.ldx + ch * kMtChunk);
      }
    }
  };
  f4_t acc = f4_t{0.f, 0.f, 0.f, 0.f};
  float offset = 0.0f;
  auto consume = [&](const Stage &st) {
    v4u bfr[8];
    if constexpr (TB > 0) {
      // stage this chunk's X rows (pair order) into the wave's image, then read the fragments
#pragma unroll
      for (int i = 0; i < XL; ++i) {
        const int t = 2 * i + shalf;
        if (t < p.T) *reinterpret_cast<v4u *>(xs + t * kMtXRow + spc * 16) = pair_order(st.x[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) bfr[j] = *reinterpret_cast<const v4u *>(xs + frag_off + j * 16);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const v4u xv = *reinterpret_cast<const v4u *>(xrow + st.ch * kMtChunk + 8 * j);
        bfr[j] = tok ? pair_order(xv) : v4u{0u, 0u, 0u, 0u};
      }
    }
    float am;
    if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[st.q], st.a), offset);
    else am = st.a;
    uint32_t t[8];
    block_table<QT, DT>(am, t);
    const uint32_t w[8] = {st.w[0].x, st.w[0].y, st.w[0].z, st.w[0].w, st.w[1].x, st.w[1].y, st.w[1].z, st.w[1].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t P[4];
      decode_codes(w[j], t, P);
      const v4u af = v4u{P[0], P[1], P[2], P[3]};
      if constexpr (DT == QZ_DT_F16)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8_t, af), __builtin_bit_cast(h8_t, bfr[j]),
                                                     acc, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8_t, af), __builtin_bit_cast(b8_t, bfr[j]),
                                                      acc, 0, 0, 0);
    }
  };
  Stage s0, s1;
  if (ch0 < ch1) load(s0, ch0);  // first HBM requests go out before anything else
  if constexpr (TB > 0) {  // the wave's zero row (B columns of absent tokens)
    for (int i = lane; i < kMtXRow / 4; i += 64) reinterpret_cast<uint32_t *>(xs + TB * kMtXRow)[i] = 0u;
  }
  if constexpr (DQ) {
    if (tid < 256) s_code2[tid] = p.sc.code2[tid];
    offset = *p.sc.offset;
    __syncthreads();
  }
  for (int ch = ch0; ch < ch1; ch += 2) {  // ping-pong: the next stage is in flight during each decode
    if (ch + 1 < ch1) load(s1, ch + 1);
    __builtin_amdgcn_sched_barrier(0);
    consume(s0);
    if (ch + 1 >= ch1) break;
    if (ch + 2 < ch1) load(s0, ch + 2);
    __builtin_amdgcn_sched_barrier(0);
    consume(s1);
  }
  // K-split partials meet in LDS; C/D map: lane l holds rows 4g+i (i = 0..3) for token l % 16
  s_red[wave][lane] = acc;
  __syncthreads();
  if (tid < 256) {
    const int l = tid & 63, i = tid >> 6;  // (lane slot, row-in-quad)
    const int c = l & 15, m = m0 + 4 * (l >> 4) + i;
    if (c < p.T && m < p.M) {
      float v = 0.0f;
#pragma unroll
      for (int w = 0; w < W; ++w) v += s_red[w][l][i];
      if (p.bias) v += load_f32<DT>(p.bias, m);
      store_f32<DT>(p.Y, (long long)c * p.ldy + m, v);
    }
  }
}

template <int QT, bool DQ, int DT, int TB, int W = kMtWaves>
__global__ __launch_bounds__(64 * W) void k_gemv_4bit_mt(GemmParams p) {
  mt_body<QT, DQ, DT, TB, W>(p, blockIdx.x);
}

// token bucket of the staged multi-token kernel: LDS image rows per wave
static int mt_bucket(int T) { return T <= 2 ? 2 : T <= 4 ? 4 : T <= 8 ? 8 : 16; }

// Grouped multi-token launch: the 2..16-token counterpart of
// k_gemv_4bit_grouped (q/k/v, gate/up of one layer over a small batch in ONE
// grid).  Segment i owns workgroups [start[i], start[i+1]); every segment's
// output is bit-identical to its own k_gemv_4bit_mt launch.
constexpr int kMtMaxSeg = 4;
struct GemmGroup {
  GemmParams seg[kMtMaxSeg];
  int start[kMtMaxSeg];
  int nseg;
};

template <int QT, bool DQ, int DT, int TB>
__global__ __launch_bounds__(64 * kMtWaves) void k_gemv_4bit_mt_grouped(GemmGroup g) {
  const int b = blockIdx.x;
  int s = 0;
#pragma unroll
  for (int i = 1; i < kMtMaxSeg; ++i)
    if (i < g.nseg && b >= g.start[i]) s = i;
  s = __builtin_amdgcn_readfirstlane(s);
  const GemmParams seg = g.seg[s];
  mt_body<QT, DQ, DT, TB>(seg, b - g.start[s]);
}

// Y[t, m] = sum_z ws[z][t][m] (+ bias[m]); 4 consecutive m per thread.
template <int DT>
__global__ __launch_bounds__(256) void k_gemm_reduce(const float *__restrict__ ws, int nsplit, int T, int M,
                                                     const void *bias, void *Y, int ldy) {
  const long long i4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long long n = (long long)T * M;
  if (i4 >= n) return;
  const int t = (int)(i4 / M), m = (int)(i4 % M);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < nsplit; ++z) {
    const float4 v = *reinterpret_cast<const float4 *>(ws + (size_t)z * n + i4);
    s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float b = bias ? load_f32<DT>(bias, m + j) : 0.0f;
    store_f32<DT>(Y, (long long)t * ldy + m + j, s[j] + b);
  }
}

static int ilog2g(long long v) {
  int l = 0;
  while ((1LL << l) < v) ++l;
  return (1LL << l) == v ? l : -1;
}

// Tile / split choice: BT = 64 tokens for T <= 64, else 128; K is split over
// up to 16 workgroups (>= 4 K-steps each) until the grid has >= 512 workgroups
// (2 per CU), as long as the fp32 partials fit the caller's workspace.
static void gemm_plan(int T, int M, int K, long long ws_bytes, int *bt, int *nsplit, int *k_split) {
  *bt = T <= 64 ? 64 : 128;
  const long long tiles = (long long)((M + kBM - 1) / kBM) * ((T + *bt - 1) / *bt);
  const int steps = K / kBK;
  int s = 1;
  while (tiles * s < 512 && s * 2 <= 16 && steps / (s * 2) >= 4 &&
         (long long)(s * 2) * T * M * 4 <= ws_bytes)
    s *= 2;
  const int per = (steps + s - 1) / s;
  *nsplit = (steps + per - 1) / per;
  *k_split = per * kBK;
}

}  // namespace qz

using namespace qz;

static bool mt_ok(int T, int K) { return T >= 2 && T <= 16 && K % kMtChunk == 0; }

// QZ_GEMM16_SCHED (read once at load, reported and set through qz_gemv_knobs / qz_gemv_set_knob):
// the k_gemm16_4d schedule qz_gemm_16bit launches -- 0: P1/P2 segments; S bits: 1 split-release
// schedule, 2 permuted W rows + 16-B register epilogue, 8 the split schedule's loop rotated, 16 (with 8)
// the waves on odd SIMDs run the schedule one MFMA later, 64 (with 1) each step one hand-ordered asm
// stream (gemm16_asm_step.h), 128 (with 64) the library's two event orders by SIMD parity, 512 (with
// 64 | 2) the persistent k_gemm16_4q where K / 64 is even, 256 (with 512) W's k-half 1 fragments
// read and its image refilled before X's, 8 (with 512 | 256) the epilogue's stores non-temporal where
// K <= 8192 (the output is not re-read by this launch; it stops evicting the X / W k-slices that other
// tiles re-read).
// Default 971 = 512 | 256 | 128 | 64 | 8 | 2 | 1
namespace qz {
int &gemm16_sched();  // gemv.hip: QZ_GEMM16_SCHED
}

extern "C" int qz_gemm_16bit_ok(int T, int M, int K, const void *X, int ldx, const void *W, const void *Y, int ldy);

// Dense 16-bit GEMM (k_gemm16_4d: 4 waves, 256 x 256 tile, LDS-DMA staging two steps ahead): the
// second half of the large-T prefill route "dequantise once (qz_dequantize_4bit, bit-exact), then
// GEMM" (modules.py:62-64's own structure, both halves hand-written for gfx950).
extern "C" int qz_gemm_16bit(int T, int M, int K, const void *X, int ldx, int dtype, const void *W, const void *bias,
                             void *Y, int ldy, void *stream) {
  if (!X || !W || !Y || T < 0 || M < 0 || K < 0) return QZ_ERR_ARG;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_DTYPE;
  if (T == 0 || M == 0) return QZ_OK;
  if (!qz_gemm_16bit_ok(T, M, K, X, ldx, W, Y, ldy)) return QZ_ERR_SHAPE;
  GemmParams p{};
  p.X = X;
  p.B = reinterpret_cast<const unsigned char *>(W);
  p.bias = bias;
  p.Y = Y;
  p.T = T;
  p.M = M;
  p.K = K;
  p.ldx = ldx;
  p.ldy = ldy;
  p.k_split = K;
  const unsigned g = (unsigned)(((M + k4wM - 1) / k4wM) * ((T + k4wT - 1) / k4wT));
  hipStream_t s = (hipStream_t)stream;
  const int sched = gemm16_sched();
  // S & 512: the persistent form (k_gemm16_4q), one workgroup per CU, when every tile starts on
  // buffer 0 (K / 64 even); otherwise the schedule's non-persistent kernel
  if ((sched & 512) != 0 && (K / kBK) % 2 == 0) {
    const unsigned gq = std::min(g, (unsigned)device_cus());
    // bit 8: non-temporal output stores where the output is large against the K loop (K <= 8192:
    // measured faster at K = 4096, slower at 14336 -- profiles/r6_gemm16_nt_store_sweeps.txt)
    const bool nt_out = K <= 8192;
#define QZ_G16Q(DT_, S_) hipLaunchKernelGGL((k_gemm16_4q<DT_, S_>), dim3(gq), dim3(256), 0, s, p)
    if (dtype == QZ_DT_F16) {
      if ((sched & 264) == 264 && nt_out) QZ_G16Q(QZ_DT_F16, 392);
      else if (sched & 256) QZ_G16Q(QZ_DT_F16, 384);
      else if (sched & 128) QZ_G16Q(QZ_DT_F16, 128);
      else QZ_G16Q(QZ_DT_F16, 0);
    } else {
      if ((sched & 264) == 264 && nt_out) QZ_G16Q(QZ_DT_BF16, 392);
      else if (sched & 256) QZ_G16Q(QZ_DT_BF16, 384);
      else if (sched & 128) QZ_G16Q(QZ_DT_BF16, 128);
      else QZ_G16Q(QZ_DT_BF16, 0);
    }
#undef QZ_G16Q
    QZ_LAUNCH_CHECK();
    return QZ_OK;
  }
  // the non-persistent schedule (bit 8 of a persistent schedule is its store policy, not 4d's rotation)
  const int s4d = (sched & 512) ? (sched & 255 & ~8) : (sched & 255);
#define QZ_G16(DT_, S_) hipLaunchKernelGGL((k_gemm16_4d<DT_, 64, 16, 112, S_>), dim3(g), dim3(256), 0, s, p)
#define QZ_G16S(DT_)                   \
  switch (s4d) {                       \
    case 1: QZ_G16(DT_, 1); break;     \
    case 2: QZ_G16(DT_, 2); break;     \
    case 3: QZ_G16(DT_, 3); break;     \
    case 9: QZ_G16(DT_, 9); break;     \
    case 11: QZ_G16(DT_, 11); break;   \
    case 25: QZ_G16(DT_, 25); break;   \
    case 27: QZ_G16(DT_, 27); break;   \
    case 65: QZ_G16(DT_, 65); break;   \
    case 67: QZ_G16(DT_, 67); break;   \
    case 193: QZ_G16(DT_, 193); break; \
    case 195: QZ_G16(DT_, 195); break; \
    default: QZ_G16(DT_, 0); break;    \
  }
  if (dtype == QZ_DT_F16) {
    QZ_G16S(QZ_DT_F16)
  } else {
    QZ_G16S(QZ_DT_BF16)
  }
#undef QZ_G16S
#undef QZ_G16
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" int qz_gemm_16bit_ok(int T, int M, int K, const void *X, int ldx, const void *W, const void *Y, int ldy) {
  return T > 0 && M > 0 && K > 0 && K % kBK == 0 && M % 8 == 0 && ldx >= K && ldx % 8 == 0 && ldy >= M &&
         ldy % 8 == 0 && (reinterpret_cast<uintptr_t>(X) % 16) == 0 && (reinterpret_cast<uintptr_t>(W) % 16) == 0 &&
         (reinterpret_cast<uintptr_t>(Y) % 16) == 0 && (long long)T * ldx * 2 < (1LL << 32) &&
         (long long)M * K * 2 < (1LL << 32);
}

extern "C" long long qz_gemm_4bit_workspace_size(int T, int M, int K) {
  if (T <= 0 || M <= 0 || K <= 0 || K % kBK != 0) return 0;
  if (mt_ok(T, K)) return 0;  // the multi-token kernel reduces in LDS
  int bt, ns, ks;
  gemm_plan(T, M, K, (long long)1 << 62, &bt, &ns, &ks);
  return ns > 1 ? (long long)ns * T * M * 4 : 0;
}

extern "C" int qz_gemm_4bit(int T, int M, int K, const void *X, int ldx, int dtype, const unsigned char *B,
                            int quant_type, int blocksize, const float *absmax, const unsigned char *qabsmax,
                            const float *absmax2, const float *code2, const float *offset, int blocksize2,
                            const void *bias, void *Y, int ldy, float *workspace, long long workspace_bytes,
                            void *stream) {
  if (!X || !B || !Y || T < 0 || M < 0 || K < 0) return QZ_ERR_ARG;
  if ((absmax == nullptr) == (qabsmax == nullptr)) return QZ_ERR_ARG;
  const bool dq = qabsmax != nullptr;
  if (dq && (!absmax2 || !code2 || !offset)) return QZ_ERR_ARG;
  if (quant_type != QZ_FP4 && quant_type != QZ_NF4) return QZ_ERR_DTYPE;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_DTYPE;
  const int bsl = ilog2g(blocksize), bs2l = dq ? ilog2g(blocksize2) : 0;
  if (bsl < 6 || bs2l < 0) return QZ_ERR_BLOCKSIZE;
  if (K % kBK != 0 || ldx < K || ldy < M || (ldx % 8) != 0 || (M % 4) != 0 ||
      (reinterpret_cast<uintptr_t>(X) % 16) != 0 || (reinterpret_cast<uintptr_t>(B) % 16) != 0 ||
      (long long)M * K / blocksize >= (1LL << 32))
    return QZ_ERR_SHAPE;
  if (T == 0 || M == 0) return QZ_OK;
  if (workspace_bytes < 0 || (workspace_bytes > 0 && !workspace)) return QZ_ERR_ARG;
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
  p.block_base = 0;
  int bt, nsplit;
  hipStream_t s = (hipStream_t)stream;
  if (mt_ok(T, K)) {  // 2..16 tokens: multi-token MFMA GEMV, one launch
    p.ws = nullptr;
    p.k_split = K;
    const dim3 grid((unsigned)((M + 15) / 16));
    const int tb = mt_bucket(T);
#define QZ_MTB(QT_, DQ_, DT_, TB_) \
  hipLaunchKernelGGL((k_gemv_4bit_mt<QT_, DQ_, DT_, TB_>), grid, dim3(64 * kMtWaves), 0, s, p)
#define QZ_MT(QT_, DQ_, DT_)                                             \
  do {                                                                   \
    if (tb == 2) QZ_MTB(QT_, DQ_, DT_, 2);                               \
    else if (tb == 4) QZ_MTB(QT_, DQ_, DT_, 4);                          \
    else if (tb == 8) QZ_MTB(QT_, DQ_, DT_, 8);                          \
    else QZ_MTB(QT_, DQ_, DT_, 16);                                      \
  } while (0)
#define QZ_MT_DT(QT_, DQ_) \
  do { if (dtype == QZ_DT_F16) QZ_MT(QT_, DQ_, QZ_DT_F16); else QZ_MT(QT_, DQ_, QZ_DT_BF16); } while (0)
    if (quant_type == QZ_FP4) {
      if (dq) QZ_MT_DT(QZ_FP4, true); else QZ_MT_DT(QZ_FP4, false);
    } else {
      if (dq) QZ_MT_DT(QZ_NF4, true); else QZ_MT_DT(QZ_NF4, false);
    }
#undef QZ_MT_DT
#undef QZ_MT
#undef QZ_MTB
    QZ_LAUNCH_CHECK();
    return QZ_OK;
  }
  if (T >= kBigMinT && (M % 8) == 0 && (ldy % 8) == 0 && (reinterpret_cast<uintptr_t>(Y) % 16) == 0 &&
      (long long)T * ldx * 2 < (1LL << 32)) {  // large T: the 256 x 256 tile kernel
    p.ws = nullptr;
    p.k_split = K;
    const unsigned g = (unsigned)(((M + kBigM - 1) / kBigM) * ((T + kBigT - 1) / kBigT));
#define QZ_BIG(QT_, DQ_, DT_) hipLaunchKernelGGL((k_gemm_4bit_8p<QT_, DQ_, DT_, 0, 1>), dim3(g), dim3(512), 0, s, p)
#define QZ_BIG_DT(QT_, DQ_) \
  do { if (dtype == QZ_DT_F16) QZ_BIG(QT_, DQ_, QZ_DT_F16); else QZ_BIG(QT_, DQ_, QZ_DT_BF16); } while (0)
    if (quant_type == QZ_FP4) {
      if (dq) QZ_BIG_DT(QZ_FP4, true); else QZ_BIG_DT(QZ_FP4, false);
    } else {
      if (dq) QZ_BIG_DT(QZ_NF4, true); else QZ_BIG_DT(QZ_NF4, false);
    }
#undef QZ_BIG_DT
#undef QZ_BIG
    QZ_LAUNCH_CHECK();
    return QZ_OK;
  }
  gemm_plan(T, M, K, workspace ? workspace_bytes : 0, &bt, &nsplit, &p.k_split);
  p.ws = nsplit > 1 ? workspace : nullptr;
  const dim3 grid((unsigned)((M + kBM - 1) / kBM), (unsigned)((T + bt - 1) / bt), (unsigned)nsplit);
#define QZ_GEMM(QT_, DQ_, DT_, BT_) hipLaunchKernelGGL((k_gemm_4bit<QT_, DQ_, DT_, BT_>), grid, dim3(256), 0, s, p)
#define QZ_GEMM_BT(QT_, DQ_, DT_) \
  do { if (bt == 64) QZ_GEMM(QT_, DQ_, DT_, 64); else QZ_GEMM(QT_, DQ_, DT_, 128); } while (0)
#define QZ_GEMM_DT(QT_, DQ_) \
  do { if (dtype == QZ_DT_F16) QZ_GEMM_BT(QT_, DQ_, QZ_DT_F16); else QZ_GEMM_BT(QT_, DQ_, QZ_DT_BF16); } while (0)
  if (quant_type == QZ_FP4) {
    if (dq) QZ_GEMM_DT(QZ_FP4, true); else QZ_GEMM_DT(QZ_FP4, false);
  } else {
    if (dq) QZ_GEMM_DT(QZ_NF4, true); else QZ_GEMM_DT(QZ_NF4, false);
  }
#undef QZ_GEMM_DT
#undef QZ_GEMM_BT
#undef QZ_GEMM
  QZ_LAUNCH_CHECK();
  if (nsplit > 1) {
    const long long n4 = ((long long)T * M) / 4;
    const unsigned g = (unsigned)((n4 + 255) / 256);
    if (dtype == QZ_DT_F16)
      hipLaunchKernelGGL((k_gemm_reduce<QZ_DT_F16>), dim3(g), dim3(256), 0, s, workspace, nsplit, T, M, bias, Y, ldy);
    else
      hipLaunchKernelGGL((k_gemm_reduce<QZ_DT_BF16>), dim3(g), dim3(256), 0, s, workspace, nsplit, T, M, bias, Y, ldy);
    QZ_LAUNCH_CHECK();
  }
  return QZ_OK;
}

extern "C" int qz_gemm_4bit_grouped(int nseg, const qz_gemv_segment *segs, int T, int K, const void *X, int ldx,
                                    int dtype, int quant_type, int blocksize, int blocksize2, void *stream) {
  if (nseg < 1 || nseg > QZ_GEMV_MAX_SEGMENTS || !segs || !X || T < 0 || K < 0) return QZ_ERR_ARG;
  if (quant_type != QZ_FP4 && quant_type != QZ_NF4) return QZ_ERR_DTYPE;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_DTYPE;
  const bool dq = segs[0].qabsmax != nullptr;
  const int bsl = ilog2g(blocksize), bs2l = dq ? ilog2g(blocksize2) : 0;
  if (bsl < 6 || bs2l < 0) return QZ_ERR_BLOCKSIZE;
  if (!mt_ok(T, K) || ldx < K || (ldx % 8) != 0 || (reinterpret_cast<uintptr_t>(X) % 16) != 0) return QZ_ERR_SHAPE;
  GemmGroup g;
  g.nseg = nseg;
  int blocks = 0;
  for (int i = 0; i < nseg; ++i) {
    const qz_gemv_segment &q = segs[i];
    if (!q.B || !q.y || q.M < 0) return QZ_ERR_ARG;
    if ((q.absmax == nullptr) == (q.qabsmax == nullptr) || (q.qabsmax != nullptr) != dq) return QZ_ERR_ARG;
    if (dq && (!q.absmax2 || !q.code2 || !q.offset)) return QZ_ERR_ARG;
    if ((q.M % 4) != 0 || (reinterpret_cast<uintptr_t>(q.B) % 16) != 0 || q.block_base < 0 ||
        q.block_base + (long long)q.M * K / blocksize >= (1LL << 32))
      return QZ_ERR_SHAPE;
    GemmParams &p = g.seg[i];
    p.X = X;
    p.B = q.B;
    p.sc = ScaleSrc{q.absmax, q.qabsmax, q.absmax2, q.code2, q.offset, blocksize2};
    p.bias = q.bias;
    p.Y = q.y;
    p.ws = nullptr;
    p.block_base = q.block_base;
    p.T = T;
    p.M = q.M;
    p.K = K;
    p.ldx = ldx;
    p.ldy = q.M;
    p.bs_log2 = bsl;
    p.bs2_log2 = bs2l;
    p.k_split = K;
    g.start[i] = blocks;
    blocks += (q.M + 15) / 16;
  }
  for (int i = nseg; i < kMtMaxSeg; ++i) g.start[i] = blocks;
  if (blocks == 0 || T == 0) return QZ_OK;
  hipStream_t s = (hipStream_t)stream;
  const int tb = mt_bucket(T);
#define QZ_MTGB(QT_, DQ_, DT_, TB_) \
  hipLaunchKernelGGL((k_gemv_4bit_mt_grouped<QT_, DQ_, DT_, TB_>), dim3(blocks), dim3(64 * kMtWaves), 0, s, g)
#define QZ_MTG(QT_, DQ_, DT_)                                            \
  do {                                                                   \
    if (tb == 2) QZ_MTGB(QT_, DQ_, DT_, 2);                              \
    else if (tb == 4) QZ_MTGB(QT_, DQ_, DT_, 4);                         \
    else if (tb == 8) QZ_MTGB(QT_, DQ_, DT_, 8);                         \
    else QZ_MTGB(QT_, DQ_, DT_, 16);                                     \
  } while (0)
#define QZ_MTG_DT(QT_, DQ_) \
  do { if (dtype == QZ_DT_F16) QZ_MTG(QT_, DQ_, QZ_DT_F16); else QZ_MTG(QT_, DQ_, QZ_DT_BF16); } while (0)
  if (quant_type == QZ_FP4) {
    if (dq) QZ_MTG_DT(QZ_FP4, true); else QZ_MTG_DT(QZ_FP4, false);
  } else {
    if (dq) QZ_MTG_DT(QZ_NF4, true); else QZ_MTG_DT(QZ_NF4, false);
  }
#undef QZ_MTG_DT
#undef QZ_MTG
#undef QZ_MTGB
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

// gemv.hip -- fused 4-bit dequantise + GEMV for batch-1 decode on gfx950.
//
// Replaces the reference decode chain (modules.py:56-61 -> core.py:426-504):
// absmax double-dequant kernel + `+= offset` + kgemm_4bit_inference_naive
// (kernels.cu:1061-1219) + two cast kernels, with ONE launch.
//
// Layout (unchanged bnb/reference format): W is [M, K] row-major, two 4-bit
// codes per byte, high nibble = even element; one scale per `blocksize`
// consecutive flat elements; with double quant the scale is rebuilt in kernel
// as code2[q] * absmax2[b / 256] + offset (two roundings, as core.py:467-468).
//
// Work decomposition (wave64-first): a K-STEP is 1 KiB of one row = 2048
// elements; lane l of a wave owns bytes [16 l, 16 l + 16) of the step, i.e.
// 32 consecutive elements that always sit inside one scale block.  A wave
// handles R rows of one step at a time, so its 64 B slice of x (fp16) is
// loaded once and reused R times; the NW waves of a workgroup are split WK
// ways along K (steps s = wk, wk+WK, ...) and RG = NW/WK ways along rows, and
// the WK partial sums meet in LDS.  Weight loads are 16 B/lane (1 KiB per wave
// instruction, fully coalesced) and non-temporal: each byte is read exactly
// once per call.
//
// Nibble decode: a workgroup first writes a 256-entry table to LDS: entry b =
// the two codes of packed byte b, i.e. exactly the operand pair that v_dot2
// multiplies with the natural-order x pair.  Decoding a byte is then one
// address computation and one LDS read; the table is stored in bank-private
// copies (lane l reads its own copy), so the random byte values never conflict.
// Any 16-entry codebook works (NF4, FP4 x12 with the sign in bit 3, a runtime LUT).
// Products: v_dot2c_f32_f16 (fp16 x fp16 exact products, fp32 accumulate);
// per 32-element chunk the fp32 dot is scaled by the block absmax with one
// FMA.  bf16 x is dotted RAW against bf16 hi + lo code pairs (v_dot2c_f32_bf16)
// and fp32 x RAW against fp32 codes (v_fma_f32): no conversion of x.
// Exact codes (CL, fp16 x): each code c is stored as c * 2^S = ch + cl, two fp16
// values (~2^-23 relative: fp32-class), in a 64-bit table entry (hi pair, lo
// pair) read with one ds_read_b64, and the dot takes ch*x + cl*x.  S (power of
// two, from max|code|) is undone on the output.
//
// The variants this file once carried for measurement only (register v_perm
// decodes, MFMA tile / diagonal decodes, the streaming form, step rings, the
// next-launch prefetch, fp32-code FMA forms, ablation bits) lost on every decode
// shape and were removed in round 5; DESIGN.md section 4.1 / 11 keeps their numbers
// and the git history their code.
#include "gemv_core.h"

namespace qz {

static int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}
static Knobs read_knobs() {
  Knobs k;
  k.wide8 = env_int("QZ_GEMV_WIDE8", 1) != 0;
  const int nr = env_int("QZ_GROUPED_NORM_R", 0);
  k.norm_r = (nr == 1 || nr == 2 || nr == 4) ? nr : 0;
  const int pr = env_int("QZ_PAIR_R", 0);
  k.pair_r = (pr == 2 || pr == 3 || pr == 4 || pr == 6 || pr == 8) ? pr : 0;
  k.pair_wt = env_int("QZ_PAIR_WT", 1) != 0;
  k.pair_ps = env_int("QZ_PAIR_PS", -1);
  k.pair_wk1 = env_int("QZ_PAIR_WK1", 2);
  return k;
}
static Knobs g_knobs = read_knobs();   // at library load
Knobs &gemv_knobs() { return g_knobs; }
// QZ_GEMM16_SCHED: the k_gemm16_4d / k_gemm16_4q schedule qz_gemm_16bit launches (gemm.hip); 971 =
// the persistent asm-step form with the library's dual event order, W's fragments read and refilled
// first, non-temporal output stores: the fastest measured (all bit-identical)
static int g_gemm16_sched = env_int("QZ_GEMM16_SCHED", 971);
int &gemm16_sched() { return g_gemm16_sched; }

template <bool DQ, int DT, int R, int WK, int NW, bool FS, bool CL, bool WT, bool TWO, int STAMP = 0>
__global__ __launch_bounds__(NW * 64) void k_gemv_4bit(GemvParams p) {
  gemv_body<DQ, DT, R, WK, NW, FS, CL, WT, false, false, TWO, false, STAMP>(p, blockIdx.x);
}

template <bool DQ, int DT, int R, int WK, bool FS, bool CL, bool NRM, bool TWO>
__global__ __launch_bounds__(256) void k_gemv_4bit_grouped(GemvGroup g) {
  const int b = blockIdx.x;
  int s = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < g.nseg && b >= g.start[i]) s = i;
  s = __builtin_amdgcn_readfirstlane(s);
  // copy the segment out before load_params launders it: loads through a
  // computed kernarg address are not invariant, so interleaving them with the
  // laundering asm would serialise them (one s_waitcnt per field)
  const GemvParams seg = g.seg[s];
  const int start = g.start[s];
  gemv_body<DQ, DT, R, WK, 4, FS, CL, false, NRM, false, TWO, false>(seg, b - start);
}

// LlamaMLP's gate/up pair (gemv_body PAIR): one launch computes act_fn(gate_proj(x)) * up_proj(x)
template <bool DQ, int DT, int R, bool CL, bool NRM, bool TWO, bool PS = false, bool WT = false>
__global__ __launch_bounds__(256) void k_gemv_4bit_pair(GemvGroup g) {
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
  const GemvParams seg = g.seg[wave >> 1];
  gemv_body<DQ, DT, R, 1, 4, true, CL, WT, NRM, true, TWO, PS>(seg, blockIdx.x, g.seg);
}

// Generic path for shapes the vector kernel does not cover (K % 32 != 0,
// odd K, blocksize < 32): one wave per row, flat element addressing exactly
// as the reference (e = r*K + k, byte e>>1, high nibble for even e).
template <bool DQ, int DT>
__global__ __launch_bounds__(256) void k_gemv_4bit_generic(GemvParams p, int quant_type) {
  __shared__ float s_lut[16];
  if (threadIdx.x < 16) s_lut[threadIdx.x] = p.lut ? p.lut[threadIdx.x] : 0.0f;
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1);
  const int row = blockIdx.x * 4 + threadIdx.x / kWave;
  if (row >= p.M) return;
  const float offset = DQ ? *p.sc.offset : 0.0f;
  float acc = 0.0f;
  for (int k = lane; k < p.K; k += kWave) {
    const long long e = (long long)row * p.K + k;
    const uint32_t byte = p.B[e >> 1];
    const uint32_t nib = (e & 1) ? (byte & 0xFu) : (byte >> 4);
    const long long b = p.block_base + (e >> p.bs_log2);
    float am;
    if constexpr (DQ) am = __fadd_rn(__fmul_rn(p.sc.code2[p.sc.qabsmax[b]], p.sc.absmax2[b >> p.bs2_log2]), offset);
    else am = p.sc.absmax[b];
    float c;
    if (p.lut) c = s_lut[nib];
    else if (quant_type == QZ_NF4) c = kNF4[nib];
    else c = (nib & 8u ? -1.0f : 1.0f) * dequant_fp4_tree(nib & 7u, 1.0f);
    acc = fmaf(load_f32<DT>(p.x, k), __fmul_rn(c, am), acc);
  }
  acc = wave_sum_last(acc);
  if (lane == kWave - 1) {
    if (p.bias) acc += load_f32<DT>(p.bias, row);
    store_f32<DT>(p.y, row, add_res<DT>(acc, p.res, row));
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

template <bool DQ, int DT, bool FS, bool CL>
static void launch_vec(const GemvParams &p, int R, int WK, hipStream_t s) {
  const int RG = 4 / WK;
  const unsigned grid = (unsigned)((p.M + R * RG - 1) / (R * RG));
#define QZ_GV(RR, WW, TWO_) \
  hipLaunchKernelGGL((k_gemv_4bit<DQ, DT, RR, WW, 4, FS, CL, false, (WW == 1 && TWO_)>), dim3(grid), dim3(256), 0, s, p)
#define QZ_GV_RW(TWO_)                        \
  do {                                        \
    if (R == 4 && WK == 2) QZ_GV(4, 2, TWO_); \
    else if (R == 4) QZ_GV(4, 1, TWO_);       \
    else if (R == 2) QZ_GV(2, 1, TWO_);       \
    else if (WK == 1) QZ_GV(1, 1, TWO_);      \
    else if (WK == 2) QZ_GV(1, 2, TWO_);      \
    else QZ_GV(1, 4, TWO_);                   \
  } while (0)
  if constexpr (FS) {
    if (two_steps(p.K, WK, true)) { QZ_GV_RW(true); return; }
  }
  // exact codes, K >= 14336 (down_proj: 7 or more K-steps per wave): 8-wave workgroups sharing one
  // 256-B-entry table (conflict-free, v_perm addresses): 4096 x 14336 8.92 -> 8.70 us, 8192 x 28672
  // (R = 4) 29.2 -> 25.5 us (profiles/r4_gemv_8wave_wide_table.txt); the per-row sums are the same
  if constexpr (FS && CL && DT == QZ_DT_F16) {
    if (WK == 1 && (R == 2 || R == 4) && p.K >= 14336 && gemv_knobs().wide8) {
      const unsigned g8 = (unsigned)((p.M + R * 8 - 1) / (R * 8));
      if (R == 4) hipLaunchKernelGGL((k_gemv_4bit<DQ, DT, 4, 1, 8, FS, CL, true, false>), dim3(g8), dim3(512), 0, s, p);
      else hipLaunchKernelGGL((k_gemv_4bit<DQ, DT, 2, 1, 8, FS, CL, true, false>), dim3(g8), dim3(512), 0, s, p);
      return;
    }
  }
  QZ_GV_RW(false);
#undef QZ_GV_RW
#undef QZ_GV
}

template <bool DQ, bool FS, bool CL>
static int dispatch_dt(const GemvParams &p, int dtype, int R, int WK, hipStream_t s) {
  switch (dtype) {
    case QZ_DT_F16: launch_vec<DQ, QZ_DT_F16, FS, CL>(p, R, WK, s); return QZ_OK;
    case QZ_DT_BF16:
      if constexpr (!CL) { launch_vec<DQ, QZ_DT_BF16, FS, false>(p, R, WK, s); return QZ_OK; }
      break;
    case QZ_DT_F32:
      if constexpr (!CL) { launch_vec<DQ, QZ_DT_F32, FS, false>(p, R, WK, s); return QZ_OK; }
      break;
  }
  return QZ_ERR_DTYPE;
}

template <bool CL>
static int dispatch_tab(const GemvParams &p, int dtype, bool dq, bool fs, int R, int WK, hipStream_t s) {
  if (fs) return dq ? dispatch_dt<true, true, CL>(p, dtype, R, WK, s) : dispatch_dt<false, true, CL>(p, dtype, R, WK, s);
  return dq ? dispatch_dt<true, false, CL>(p, dtype, R, WK, s) : dispatch_dt<false, false, CL>(p, dtype, R, WK, s);
}

}  // namespace qz

using namespace qz;

static int gemv_impl(int M, int K, const void *x, int dtype, const unsigned char *B, int quant_type, int blocksize,
                     const float *absmax, const unsigned char *qabsmax, const float *absmax2, const float *code2,
                     const float *offset, int blocksize2, long long block_base, const float *lut, const void *bias,
                     const void *res, void *y, void *stream) {
  GemvParams p;
  bool vec_ok;
  const int st = make_params(M, K, x, dtype, B, quant_type, blocksize, absmax, qabsmax, absmax2, code2, offset,
                             blocksize2, block_base, lut, bias, y, &p, &vec_ok);
  if (st != QZ_OK) return st;
  p.res = res;
  if (M == 0) return QZ_OK;
  const bool dq = qabsmax != nullptr;
  hipStream_t s = (hipStream_t)stream;
  // bf16 x always decodes with bf16 hi + lo codes and fp32 x with fp32 codes: the exact-code (CL)
  // variant is the fp16-activation option only
  const bool cl = exact_codes(quant_type, lut) && dtype == QZ_DT_F16;
  quant_type &= ~QZ_EXACT_CODES;

  if (!vec_ok) {
    const unsigned grid = (unsigned)((M + 3) / 4);
    if (K == 0) return QZ_ERR_SHAPE;
#define QZ_GG(DQ_, DT_) \
  hipLaunchKernelGGL((k_gemv_4bit_generic<DQ_, DT_>), dim3(grid), dim3(256), 0, s, p, quant_type)
    if (dq) {
      if (dtype == QZ_DT_F16) QZ_GG(true, QZ_DT_F16); else if (dtype == QZ_DT_BF16) QZ_GG(true, QZ_DT_BF16); else QZ_GG(true, QZ_DT_F32);
    } else {
      if (dtype == QZ_DT_F16) QZ_GG(false, QZ_DT_F16); else if (dtype == QZ_DT_BF16) QZ_GG(false, QZ_DT_BF16); else QZ_GG(false, QZ_DT_F32);
    }
#undef QZ_GG
    QZ_LAUNCH_CHECK();
    return QZ_OK;
  }

  int R, WK;
  choose_geometry(M, K, dtype, &R, &WK);
  set_tables(quant_type, lut, cl, dtype, &p);
  const bool fs = full_steps(K, blocksize, blocksize2, dq, block_base);
  const int rc = cl ? dispatch_tab<true>(p, dtype, dq, fs, R, WK, s) : dispatch_tab<false>(p, dtype, dq, fs, R, WK, s);
  if (rc != QZ_OK) return rc;
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" int qz_gemv_4bit(int M, int K, const void *x, int dtype, const unsigned char *B, int quant_type,
                            int blocksize, const float *absmax, const unsigned char *qabsmax, const float *absmax2,
                            const float *code2, const float *offset, int blocksize2, long long block_base,
                            const float *lut, const void *bias, void *y, void *stream) {
  return gemv_impl(M, K, x, dtype, B, quant_type, blocksize, absmax, qabsmax, absmax2, code2, offset, blocksize2,
                   block_base, lut, bias, nullptr, y, stream);
}

extern "C" int qz_gemv_4bit_residual(int M, int K, const void *x, int dtype, const unsigned char *B, int quant_type,
                                     int blocksize, const float *absmax, const unsigned char *qabsmax,
                                     const float *absmax2, const float *code2, const float *offset, int blocksize2,
                                     long long block_base, const float *lut, const void *bias, const void *residual,
                                     void *y, void *stream) {
  if (!residual) return QZ_ERR_ARG;
  return gemv_impl(M, K, x, dtype, B, quant_type, blocksize, absmax, qabsmax, absmax2, code2, offset, blocksize2,
                   block_base, lut, bias, residual, y, stream);
}

// nw != nullptr: x is first RMSNorm'd with weight nw / epsilon eps, bit-identically to qz_rmsnorm
// (the pre-norm of q/k/v and gate/up fused into their grouped launch)
static int gemv_grouped_impl(int nseg, const qz_gemv_segment *segs, int K, const void *x, int dtype, int quant_type,
                             int blocksize, int blocksize2, const float *lut, const void *nw, float eps, void *stream) {
  if (nseg < 1 || nseg > QZ_GEMV_MAX_SEGMENTS || !segs) return QZ_ERR_ARG;
  GemvGroup g;
  g.nseg = nseg;
  const bool cl = exact_codes(quant_type, lut) && dtype == QZ_DT_F16;
  bool all_vec = true;
  long long total_m = 0;
  const bool dq = segs[0].qabsmax != nullptr;
  for (int i = 0; i < nseg; ++i) {
    const qz_gemv_segment &q = segs[i];
    bool v;
    const int st = make_params(q.M, K, x, dtype, q.B, quant_type, blocksize, q.absmax, q.qabsmax, q.absmax2, q.code2,
                               q.offset, blocksize2, q.block_base, lut, q.bias, q.y, &g.seg[i], &v);
    if (st != QZ_OK) return st;
    if ((q.qabsmax != nullptr) != dq) return QZ_ERR_ARG;  // one launch = one scale format
    all_vec = all_vec && v;
    total_m += q.M;
  }
  if (total_m == 0) return QZ_OK;
  if (nw) {  // the fused pre-norm takes full-step 16-bit single-token launches only
    if (!all_vec || total_m > INT32_MAX || (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) || K % 8 != 0 || K > 16384 ||
        ((uintptr_t)x | (uintptr_t)nw) % 16 != 0)
      return QZ_ERR_SHAPE;
    for (int i = 0; i < nseg; ++i) {
      if (!full_steps(K, blocksize, blocksize2, dq, segs[i].block_base)) return QZ_ERR_SHAPE;
      g.seg[i].nw = nw;
      g.seg[i].eps = eps;
    }
  }
  if (!all_vec || total_m > INT32_MAX) {  // odd shapes: one launch per segment (same results)
    for (int i = 0; i < nseg; ++i) {
      const qz_gemv_segment &q = segs[i];
      const int rc = qz_gemv_4bit(q.M, K, x, dtype, q.B, quant_type, blocksize, q.absmax, q.qabsmax, q.absmax2,
                                  q.code2, q.offset, blocksize2, q.block_base, lut, q.bias, q.y, stream);
      if (rc != QZ_OK) return rc;
    }
    return QZ_OK;
  }
  int R, WK;
  choose_geometry((int)total_m, K, dtype, &R, &WK);
  // QZ_GROUPED_NORM_R (knob): rows per wave of the fused pre-norm launch where the geometry keeps
  // whole rows per wave (WK = 1: the same per-row sums)
  if (nw && gemv_knobs().norm_r && WK == 1) R = gemv_knobs().norm_r;
  const int rows_per_block = R * (4 / WK);
  int blocks = 0;
  for (int i = 0; i < nseg; ++i) {
    set_tables(quant_type & ~QZ_EXACT_CODES, lut, cl, dtype, &g.seg[i]);
    g.start[i] = blocks;
    blocks += (g.seg[i].M + rows_per_block - 1) / rows_per_block;
  }
  for (int i = nseg; i < kMaxSeg; ++i) g.start[i] = blocks;
  g.total = blocks;
  // every workgroup repeats the norm prologue (x and the norm weight from L2, two barriers, 8 KiB
  // more LDS): past ~4096 workgroups it costs more than the separate launch saves (measured:
  // Llama-3-70B gate/up, 7168 workgroups, 74.6 us fused vs 58.6 us for the two launches;
  // profiles/r3_prenorm_launch_times.txt)
  if (nw && blocks > kNormMaxBlocks) return QZ_ERR_SHAPE;
  // where K is split over waves and the prologue is large (the Llama-3-70B q/k/v: 1280 workgroups
  // each normalising 8192 values) the norm launch + the plain grouped launch beat the fused prologue
  // (16.41 vs 17.23 us, profiles/r5_qkv70_forms.txt): the caller runs the two launches.  A row
  // shard's q/k/v (Llama-3-8B at N = 8: 384 workgroups x 4096) keeps it fused (round 4's form).
  if (nw && WK != 1 && (long long)blocks * K > kNormSplitMaxValues) return QZ_ERR_SHAPE;
  bool all_fs = true;
  for (int i = 0; i < nseg; ++i) all_fs = all_fs && full_steps(K, blocksize, blocksize2, dq, segs[i].block_base);
  hipStream_t s = (hipStream_t)stream;
  const bool two = two_steps(K, WK, all_fs || nw);
  const size_t lds = nw ? (size_t)K * 2 : 0;
#define QZ_GR1(DQ_, DT_, RR, WW, FS_, CL_, NRM_)                                                            \
  do {                                                                                                    \
    if (FS_ && two && WW == 1)                                                                            \
      hipLaunchKernelGGL((k_gemv_4bit_grouped<DQ_, DT_, RR, WW, FS_, CL_, NRM_, (FS_ && WW == 1)>), dim3(blocks), \
                         dim3(256), lds, s, g);                                                           \
    else hipLaunchKernelGGL((k_gemv_4bit_grouped<DQ_, DT_, RR, WW, FS_, CL_, NRM_, false>), dim3(blocks),      \
                            dim3(256), lds, s, g);                                                        \
  } while (0)
#define QZ_GR_RW(DQ_, DT_, FS_, CL_, NRM_)                                                                  \
  do {                                                                                                    \
    if (R == 4 && WK == 2) QZ_GR1(DQ_, DT_, 4, 2, FS_, CL_, NRM_);                                        \
    else if (R == 4) QZ_GR1(DQ_, DT_, 4, 1, FS_, CL_, NRM_);                                              \
    else if (R == 2) QZ_GR1(DQ_, DT_, 2, 1, FS_, CL_, NRM_);                                              \
    else if (WK == 1) QZ_GR1(DQ_, DT_, 1, 1, FS_, CL_, NRM_);                                             \
    else if (WK == 2) QZ_GR1(DQ_, DT_, 1, 2, FS_, CL_, NRM_);                                             \
    else QZ_GR1(DQ_, DT_, 1, 4, FS_, CL_, NRM_);                                                          \
  } while (0)
#define QZ_GR_DT(DQ_, FS_)                                                                                  \
  do {                                                                                                    \
    if (dtype == QZ_DT_F16) { if (cl) QZ_GR_RW(DQ_, QZ_DT_F16, FS_, true, false); else QZ_GR_RW(DQ_, QZ_DT_F16, FS_, false, false); } \
    else if (dtype == QZ_DT_BF16) QZ_GR_RW(DQ_, QZ_DT_BF16, FS_, false, false);                         \
    else QZ_GR_RW(DQ_, QZ_DT_F32, FS_, false, false);                                                    \
  } while (0)
  if (nw) {
    if (dtype == QZ_DT_F16) {
      if (dq) { if (cl) QZ_GR_RW(true, QZ_DT_F16, true, true, true); else QZ_GR_RW(true, QZ_DT_F16, true, false, true); }
      else { if (cl) QZ_GR_RW(false, QZ_DT_F16, true, true, true); else QZ_GR_RW(false, QZ_DT_F16, true, false, true); }
    } else {
      if (dq) QZ_GR_RW(true, QZ_DT_BF16, true, false, true); else QZ_GR_RW(false, QZ_DT_BF16, true, false, true);
    }
  } else if (all_fs) { if (dq) QZ_GR_DT(true, true); else QZ_GR_DT(false, true); }
  else { if (dq) QZ_GR_DT(true, false); else QZ_GR_DT(false, false); }
#undef QZ_GR_DT
#undef QZ_GR_RW
#undef QZ_GR1
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" int qz_gemv_4bit_grouped(int nseg, const qz_gemv_segment *segs, int K, const void *x, int dtype,
                                    int quant_type, int blocksize, int blocksize2, const float *lut, void *stream) {
  return gemv_grouped_impl(nseg, segs, K, x, dtype, quant_type, blocksize, blocksize2, lut, nullptr, 0.0f, stream);
}

extern "C" int qz_gemv_4bit_grouped_rmsnorm(int nseg, const qz_gemv_segment *segs, int K, const void *x, int dtype,
                                            int quant_type, int blocksize, int blocksize2, const float *lut,
                                            const void *norm_weight, float eps, void *stream) {
  if (!norm_weight || !x) return QZ_ERR_ARG;
  return gemv_grouped_impl(nseg, segs, K, x, dtype, quant_type, blocksize, blocksize2, lut, norm_weight, eps, stream);
}

// the persistent exact-code pair on the 256-B-entry table (64 KiB: 32 bank-private copies of each 8-B
// entry, v_perm addresses), 2 workgroups per CU
template <bool DQ, int DT, int R, bool CL, bool NRM>
static void launch_pair_wt(unsigned grid, size_t lds, hipStream_t s, const GemvGroup &g, bool two) {
  if constexpr (CL && NRM && DT == QZ_DT_F16 && (R == 2 || R == 4)) {
    if (two) hipLaunchKernelGGL((k_gemv_4bit_pair<DQ, DT, R, CL, NRM, true, true, true>), dim3(grid), dim3(256), lds, s, g);
    else hipLaunchKernelGGL((k_gemv_4bit_pair<DQ, DT, R, CL, NRM, false, true, true>), dim3(grid), dim3(256), lds, s, g);
  }
}

// the persistent pair in its step-loop form (K != 4096): with the fused norm only -- without one
// the persistence buys nothing (the knob's grid then runs one workgroup per block)
template <bool DQ, int DT, int R, bool CL, bool NRM>
static void launch_pair_ps_loop(unsigned grid, int blocks, size_t lds, hipStream_t s, const GemvGroup &g) {
  if constexpr (NRM)
    hipLaunchKernelGGL((k_gemv_4bit_pair<DQ, DT, R, CL, NRM, false, true>), dim3(grid), dim3(256), lds, s, g);
  else
    hipLaunchKernelGGL((k_gemv_4bit_pair<DQ, DT, R, CL, NRM, false>), dim3(blocks), dim3(256), lds, s, g);
}

// LlamaMLP's act_fn(gate_proj(x)) * up_proj(x) (modeling_llama.py:175, hidden_act "silu") in one
// launch: segs[0] = gate, segs[1] = up (equal M; their y are not written), h = the [M] product
extern "C" int qz_gemv_4bit_pair_silu(const qz_gemv_segment *segs, int K, const void *x, int dtype, int quant_type,
                                      int blocksize, int blocksize2, const float *lut, const void *norm_weight,
                                      float eps, void *h, void *stream) {
  if (!segs || !h || !x) return QZ_ERR_ARG;
  if (segs[0].M != segs[1].M) return QZ_ERR_SHAPE;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_SHAPE;
  GemvGroup g;
  g.nseg = 2;
  const bool cl = exact_codes(quant_type, lut) && dtype == QZ_DT_F16;
  const bool dq = segs[0].qabsmax != nullptr;
  for (int i = 0; i < 2; ++i) {
    const qz_gemv_segment &q = segs[i];
    bool v;
    const int st = make_params(q.M, K, x, dtype, q.B, quant_type, blocksize, q.absmax, q.qabsmax, q.absmax2, q.code2,
                               q.offset, blocksize2, q.block_base, lut, q.bias, h, &g.seg[i], &v);
    if (st != QZ_OK) return st;
    if ((q.qabsmax != nullptr) != dq || !v || !full_steps(K, blocksize, blocksize2, dq, q.block_base))
      return QZ_ERR_SHAPE;
    set_tables(quant_type & ~QZ_EXACT_CODES, lut, cl, dtype, &g.seg[i]);
    g.seg[i].nw = norm_weight;
    g.seg[i].eps = eps;
  }
  const int M = segs[0].M;
  if (M == 0) return QZ_OK;
  if (norm_weight && (K % 8 != 0 || K > 16384 || ((uintptr_t)x | (uintptr_t)norm_weight) % 16 != 0))
    return QZ_ERR_SHAPE;
  // the geometry qz_gemv_4bit_grouped takes for the pair's 2M rows (same per-row summation order,
  // so the same bits where it keeps whole rows per wave).  Single-row waves (R = 1: small row shards,
  // e.g. Llama-3-8B gate/up over 8 ranks) take the pair launch too
  int R, WK;
  choose_geometry(2 * M, K, dtype, &R, &WK);
  if (WK != 1) {
    // K split over waves in the grouped launch (the K = 8192 layers of Llama-3-70B; small pairs):
    // the pair keeps whole rows per wave -- the same products in another fp32 summation order
    // (faster: 28672 x 8192 gate/up 52-55 us against 57-59 for the grouped launch and 60-61 for a
    // split-K pair, profiles/r5_pair_k8192_forms.txt), with the norm fused in persistent workgroups
    // at 3 per CU (54.6 us against 55.7 for the norm launch + the pair, 58.2 on the 64 KiB table
    // that fits once per CU: profiles/r5_pair70_norm_forms.txt).  QZ_PAIR_WK1=1: the norm as its own
    // launch (QZ_ERR_SHAPE with a norm: the caller runs it first); 0: these geometries declined
    const int wk1 = gemv_knobs().pair_wk1;
    if (wk1 == 0 || (norm_weight && wk1 != 2)) return QZ_ERR_SHAPE;
    WK = 1;
  }
  if (gemv_knobs().pair_r) R = gemv_knobs().pair_r;   // knob; the per-row sums do not depend on R
  const int blocks = (M + 2 * R - 1) / (2 * R);
  if (norm_weight && blocks > kNormMaxBlocks) return QZ_ERR_SHAPE;
  for (int i = 2; i < kMaxSeg; ++i) g.start[i] = 0;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = norm_weight ? (size_t)K * 2 : 0;
  const bool two = two_steps(K, 1, true);
  // Persistent workgroups (gemv_body PS) for two-step launches with the fused RMSNorm: every
  // workgroup normalises x once for several row blocks instead of once per block (measured,
  // profiles/r4_pair_persistent.txt: 14336 rows 19.5 -> 16.4 us, 7168 rows 13.9 -> 10.4 us, the
  // N = 4 / 8 shards 8.9 -> 7.4 and 7.9 -> 6.3 us; without the norm the one-block-per-workgroup
  // launch stays faster).  Grid: 3 workgroups per CU (what the 43 KiB LDS image admits), the best
  // or within 4 % of the best of 2 / 3 / 4 per CU and of blocks / 2 at every shape.
  // With exact codes and R = 2 / 4 the persistent pair takes the 256-B-entry table (64 KiB: 32
  // bank-private copies of each 8-B entry, one v_perm per address, no bank conflicts) at 2
  // workgroups per CU: 16.2-16.8 -> 15.1 us for 14336 rows, 10.8 -> 10.6 for 7168
  // (profiles/r4_pair_persistent_wide_table.txt), from 3 blocks per workgroup on (at the N = 4
  // shard, 896 blocks, the 16-copy table at 3 per CU is 3 % faster)
  // The persistent grid must be resident at once (a second round of persistent workgroups repeats the
  // whole block loop): workgroups per CU = what the LDS admits -- the byte table (32 KiB, 64 KiB for
  // the 256-B-entry one), the normalised image (2K bytes) and ~4 KiB of partials -- capped at 3.  At
  // K = 8192 the wide table + image (84 KiB) fits once, so the wide table is taken only where two fit.
  const int cus = device_cus();
  const size_t img = norm_weight ? (size_t)K * 2 : 0;
  const int per_cu_wt = (int)std::min<size_t>(3, kLdsPerCU / (2 * kTabDwords * 4 + img + 4096));
  const int per_cu = (int)std::min<size_t>(3, kLdsPerCU / (kTabDwords * 4 + img + 4096));
  const bool wt_ok = cl && norm_weight && (R == 2 || R == 4) && blocks >= 3 * 2 * cus && per_cu_wt >= 2 &&
                     gemv_knobs().pair_wt;
  int pgrid_i = 0;
  if (gemv_knobs().pair_ps >= 0) {
    const int ps = gemv_knobs().pair_ps;
    pgrid_i = ps <= 0 ? 0 : ps <= 8 ? cus * ps : ps;
  } else if (norm_weight) {
    pgrid_i = (wt_ok ? 2 : per_cu) * cus;
  }
  const unsigned pgrid = (unsigned)max(pgrid_i, 1);
  const bool persist = pgrid_i > 0 && pgrid_i < blocks;   // the two-step form or the step loop (K != 4096)
  const bool pair_wt = persist && wt_ok;
#define QZ_PS(DQ_, DT_, RR, CL_, NRM_)                                                                               \
  do {                                                                                                              \
    if (pair_wt) launch_pair_wt<DQ_, DT_, RR, CL_, NRM_>(pgrid, lds, s, g, two);                                        \
    else if (persist && two) hipLaunchKernelGGL((k_gemv_4bit_pair<DQ_, DT_, RR, CL_, NRM_, true, true>), dim3(pgrid), \
                                                dim3(256), lds, s, g);                                              \
    else if (persist) launch_pair_ps_loop<DQ_, DT_, RR, CL_, NRM_>(pgrid, blocks, lds, s, g);                      \
    else if (two) hipLaunchKernelGGL((k_gemv_4bit_pair<DQ_, DT_, RR, CL_, NRM_, true>), dim3(blocks), dim3(256),    \
                                     lds, s, g);                                                                    \
    else hipLaunchKernelGGL((k_gemv_4bit_pair<DQ_, DT_, RR, CL_, NRM_, false>), dim3(blocks), dim3(256), lds, s, g); \
  } while (0)
#define QZ_PS_R(DQ_, DT_, CL_, NRM_)                  \
  do {                                                \
    if (R == 4) QZ_PS(DQ_, DT_, 4, CL_, NRM_);        \
    else if (R == 8) QZ_PS(DQ_, DT_, 8, CL_, NRM_);   \
    else if (R == 6) QZ_PS(DQ_, DT_, 6, CL_, NRM_);   \
    else if (R == 3) QZ_PS(DQ_, DT_, 3, CL_, NRM_);   \
    else if (R == 1) QZ_PS(DQ_, DT_, 1, CL_, NRM_);   \
    else QZ_PS(DQ_, DT_, 2, CL_, NRM_);               \
  } while (0)
#define QZ_PS_N(DQ_, DT_, CL_)                                                         \
  do {                                                                                 \
    if (norm_weight) QZ_PS_R(DQ_, DT_, CL_, true); else QZ_PS_R(DQ_, DT_, CL_, false); \
  } while (0)
  if (dtype == QZ_DT_F16) {
    if (dq) { if (cl) QZ_PS_N(true, QZ_DT_F16, true); else QZ_PS_N(true, QZ_DT_F16, false); }
    else { if (cl) QZ_PS_N(false, QZ_DT_F16, true); else QZ_PS_N(false, QZ_DT_F16, false); }
  } else {
    if (dq) QZ_PS_N(true, QZ_DT_BF16, false); else QZ_PS_N(false, QZ_DT_BF16, false);
  }
#undef QZ_PS_N
#undef QZ_PS_R
#undef QZ_PS
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

// The launch-geometry knobs in effect (read once at library load) as a JSON object, for the bench
// line's config.  Returns the length written (excluding the NUL), or the length needed if n is too small.
extern "C" int qz_gemv_knobs(char *buf, int n) {
  char tmp[320];
  const int len = snprintf(tmp, sizeof(tmp),
                           "{\"QZ_GEMV_WIDE8\": %d, \"QZ_GROUPED_NORM_R\": %d, \"QZ_PAIR_R\": %d, \"QZ_PAIR_WT\": %d, "
                           "\"QZ_PAIR_PS\": %d, \"QZ_PAIR_WK1\": %d, \"QZ_GEMM16_SCHED\": %d, \"cus\": %d}",
                           gemv_knobs().wide8, gemv_knobs().norm_r, gemv_knobs().pair_r, gemv_knobs().pair_wt,
                           gemv_knobs().pair_ps, gemv_knobs().pair_wk1, gemm16_sched(), device_cus());
  if (buf && n > len) memcpy(buf, tmp, (size_t)len + 1);
  return len;
}

// Sets one knob (the names of qz_gemv_knobs; values as the environment variable would give them),
// for measurements and tests that compare launch forms.  Returns QZ_OK or QZ_ERR_ARG.
extern "C" int qz_gemv_set_knob(const char *name, int value) {
  if (!name) return QZ_ERR_ARG;
  Knobs &k = gemv_knobs();
  if (!strcmp(name, "QZ_GEMV_WIDE8")) k.wide8 = value != 0;
  else if (!strcmp(name, "QZ_GROUPED_NORM_R")) k.norm_r = (value == 1 || value == 2 || value == 4) ? value : 0;
  else if (!strcmp(name, "QZ_PAIR_R")) k.pair_r = (value == 2 || value == 3 || value == 4 || value == 6 || value == 8) ? value : 0;
  else if (!strcmp(name, "QZ_PAIR_WT")) k.pair_wt = value != 0;
  else if (!strcmp(name, "QZ_PAIR_PS")) k.pair_ps = value;
  else if (!strcmp(name, "QZ_PAIR_WK1")) k.pair_wk1 = value;
  else if (!strcmp(name, "QZ_GEMM16_SCHED")) gemm16_sched() = value;
  else return QZ_ERR_ARG;
  return QZ_OK;
}

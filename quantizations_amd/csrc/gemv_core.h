// gemv_core.h -- the decode GEMV's device core (byte tables, step loads, the GEMV body) and the
// host-side geometry / argument helpers of gemv.hip (the per-layer launches), also built into the
// measurement-only diag library and the microbenchmarks.  See gemv.hip's header for the design.
#pragma once
#include "common.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace qz {

// Bank-private table copies: 32 copies of a 4-B entry (fp16 codes) or 16 copies
// of an 8-B entry (exact / bf16 / fp32 codes) -- 128 B per byte value, 32 KiB.
// A ds_read_b32 serves each 32-lane half of the wave in one LDS cycle when its
// lanes hit distinct banks (MI355X_MICROARCH.md, LDS table): copy j lives wholly in
// bank j (dword e*32 + j) and lane l reads copy l % 32.  With 8-B entries a
// 32-lane group holds two lanes per copy, which collide only when their byte
// values have the same parity (1.5-way on average).  WT ("wide table"): 256 B per
// byte value (64 / 32 copies), 64 KiB, every copy bank-private, and the lookup
// address is one v_perm.
constexpr int kTabCopies = 32;
constexpr int kTabDwords = 256 * kTabCopies;  // 32 KiB
constexpr int kTabCopiesCL = 16;

// The byte tables of the built-in codebooks, computed at compile time and stored
// once in device memory with each entry repeated 4 times (one 16-B store covers
// 4 bank copies): a workgroup fills its LDS image with plain 16-B copies.
constexpr uint16_t f16_bits_rne_c(float f) {  // normal-range values and +-0 only
  const uint32_t u = __builtin_bit_cast(uint32_t, f);
  const uint32_t sign = (u >> 16) & 0x8000u, au = u & 0x7FFFFFFFu;
  if (au == 0) return (uint16_t)sign;
  const uint32_t e = (au >> 23) - 127u + 15u, m = au & 0x7FFFFFu;
  uint32_t h = (e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1u;
  return (uint16_t)(sign | h);
}
struct ByteTable {
  uint32_t v[256 * 4];
};
constexpr ByteTable make_byte_table(const uint16_t (&c)[16]) {
  ByteTable t{};
  for (int e = 0; e < 256; ++e)
    for (int k = 0; k < 4; ++k) t.v[4 * e + k] = (uint32_t)c[e >> 4] | ((uint32_t)c[e & 15] << 16);
  return t;
}
// NF4 codebook q_data (reference kernels.cu:851)
constexpr float kNF4Host[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                                -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                                0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                                0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                                0.7229568362236023f, 1.0f};
constexpr ByteTable make_nf4_table() {
  uint16_t c[16] = {};
  for (int i = 0; i < 16; ++i) c[i] = f16_bits_rne_c(kNF4Host[i]);
  return make_byte_table(c);
}
// FP4 x12: magnitudes {0, 1/16, 8, 12, 4, 6, 2, 3} (exact fp16), sign in code bit 3 (code 8 = -0.0)
constexpr uint16_t kFP4x12Bits[16] = {0x0000, 0x2C00, 0x4800, 0x4A00, 0x4400, 0x4600, 0x4000, 0x4200,
                                      0x8000, 0xAC00, 0xC800, 0xCA00, 0xC400, 0xC600, 0xC000, 0xC200};
// exact NF4 codes (CL): c * 2^14 = hi + lo (fp16 each), entries {hi pair, lo pair} x 2
constexpr int kNF4ExactShift = 14;
constexpr float f16_value_c(uint16_t h) {  // normal-range values and +-0 only
  const float sgn = (h & 0x8000u) ? -1.0f : 1.0f;
  const int e = (h >> 10) & 31;
  if (e == 0) return sgn * 0.0f;
  float v = 1.0f + (float)(h & 0x3FFu) / 1024.0f;
  for (int i = 15; i < e; ++i) v *= 2.0f;
  for (int i = e; i < 15; ++i) v *= 0.5f;
  return sgn * v;
}
constexpr ByteTable make_nf4_exact_table() {
  uint16_t hi[16] = {}, lo[16] = {};
  for (int i = 0; i < 16; ++i) {
    const float c = kNF4Host[i] * (float)(1 << kNF4ExactShift);  // exact (power of two)
    hi[i] = f16_bits_rne_c(c);
    lo[i] = f16_bits_rne_c(c - f16_value_c(hi[i]));               // the residual is exact in fp32
  }
  ByteTable t{};
  for (int e = 0; e < 256; ++e) {
    const uint32_t h = (uint32_t)hi[e >> 4] | ((uint32_t)hi[e & 15] << 16);
    const uint32_t l = (uint32_t)lo[e >> 4] | ((uint32_t)lo[e & 15] << 16);
    t.v[4 * e + 0] = h; t.v[4 * e + 1] = l; t.v[4 * e + 2] = h; t.v[4 * e + 3] = l;
  }
  return t;
}
// bf16 activations: the codes as bf16 hi + lo pairs -- c = hi + lo to ~2^-16 -- dotted straight
// against the raw bf16 x pairs with v_dot2c_f32_bf16 (bf16 has fp32's exponent range: no
// pre-scale).  Entries {hi pair, lo pair}, the CL geometry.
constexpr uint16_t bf16_bits_rne_c(float f) {  // finite values
  const uint32_t u = __builtin_bit_cast(uint32_t, f);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
constexpr float bf16_value_c(uint16_t b) { return __builtin_bit_cast(float, (uint32_t)b << 16); }
constexpr ByteTable make_bf16_table(const float (&c)[16]) {
  uint16_t hi[16] = {}, lo[16] = {};
  for (int i = 0; i < 16; ++i) {
    hi[i] = bf16_bits_rne_c(c[i]);
    lo[i] = bf16_bits_rne_c(c[i] - bf16_value_c(hi[i]));        // the residual is exact in fp32
  }
  ByteTable t{};
  for (int e = 0; e < 256; ++e) {
    const uint32_t h = (uint32_t)hi[e >> 4] | ((uint32_t)hi[e & 15] << 16);
    const uint32_t l = (uint32_t)lo[e >> 4] | ((uint32_t)lo[e & 15] << 16);
    t.v[4 * e + 0] = h; t.v[4 * e + 1] = l; t.v[4 * e + 2] = h; t.v[4 * e + 3] = l;
  }
  return t;
}
// FP4 x12 magnitudes {0, 1/16, 8, 12, 4, 6, 2, 3} are exact in bf16 (lo = 0); out_scale 1/12
constexpr float kFP4x12Host[16] = {0.0f, 0.0625f, 8.0f, 12.0f, 4.0f, 6.0f, 2.0f, 3.0f,
                                   -0.0f, -0.0625f, -8.0f, -12.0f, -4.0f, -6.0f, -2.0f, -3.0f};
// fp32 activations: entries {code[e >> 4], code[e & 15]} as fp32 -- the reference's own fp32
// quant_map values (kernels.cu:1115-1120) -- multiplied into the raw fp32 x by v_fma_f32
constexpr ByteTable make_f32_table(const float (&c)[16]) {
  ByteTable t{};
  for (int e = 0; e < 256; ++e) {
    const uint32_t a = __builtin_bit_cast(uint32_t, c[e >> 4]), b = __builtin_bit_cast(uint32_t, c[e & 15]);
    t.v[4 * e + 0] = a; t.v[4 * e + 1] = b; t.v[4 * e + 2] = a; t.v[4 * e + 3] = b;
  }
  return t;
}
static __device__ const ByteTable g_byte_tab_nf4 = make_nf4_table();
static __device__ const ByteTable g_byte_tab_nf4x = make_nf4_exact_table();
static __device__ const ByteTable g_byte_tab_fp4 = make_byte_table(kFP4x12Bits);
static __device__ const ByteTable g_byte_tab_nf4_bf = make_bf16_table(kNF4Host);
static __device__ const ByteTable g_byte_tab_fp4_bf = make_bf16_table(kFP4x12Host);
static __device__ const ByteTable g_byte_tab_nf4_f32 = make_f32_table(kNF4Host);
static __device__ const ByteTable g_byte_tab_fp4_f32 = make_f32_table(kFP4x12Host);
static_assert(bf16_bits_rne_c(0.07958029955625534f) == 0x3DA3, "bf16 RNE of an NF4 code");
static_assert(f16_bits_rne_c(0.07958029955625534f) == 0x2D18, "fp16 RNE of an NF4 code");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// v rounded to the storage format of DT (the conversions store_f32 uses), back as fp32
template <int DT> __device__ __forceinline__ float round_store(float v) {
  if constexpr (DT == QZ_DT_F16) return __half2float(__ushort_as_half(f32_to_f16_bits(v)));
  else if constexpr (DT == QZ_DT_BF16) return __bfloat162float(__float2bfloat16(v));
  else return v;
}
// LlamaDecoderLayer's `residual + h` on the projection output h as torch stores it (rounded), the
// sum rounded again by the store
template <int DT> __device__ __forceinline__ float add_res(float o, const void *res, long long row) {
  return res ? __fadd_rn(load_f32<DT>(res, row), round_store<DT>(o)) : o;
}

// two outputs in the 16-bit format of DT, element 0 in the low half (each converted exactly as
// store_f32 converts it)
template <int DT> __device__ __forceinline__ uint32_t pack16(float a, float b) {
  if constexpr (DT == QZ_DT_F16) {
    return (uint32_t)f32_to_f16_bits(a) | ((uint32_t)f32_to_f16_bits(b) << 16);
  } else {
    return (uint32_t)__builtin_bit_cast(uint16_t, __float2bfloat16(a)) |
           ((uint32_t)__builtin_bit_cast(uint16_t, __float2bfloat16(b)) << 16);
  }
}

struct GemvParams {
  const unsigned char *B;
  const void *x;
  ScaleSrc sc;
  const void *bias;
  void *y;
  const float *lut;  // runtime 16-entry codebook (always decoded exactly) or nullptr
  long long block_base;
  int M, K;
  int bs_log2, bs2_log2;
  float out_scale;
  int tabsel;        // built-in byte table: 0 = NF4, 1 = FP4 (x12), 2 = exact NF4 (CL)
  const void *nw;    // fused pre-norm (NRM): the RMSNorm weight [K], or nullptr
  float eps;         //   and its epsilon
  const void *res;   // residual [M] added after the output rounding (y = round(round(x W^T) + res)), or nullptr
};

__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, a), __builtin_bit_cast(h2_t, b), c, false);
}

// Kernel arguments are read ONCE at entry and laundered through an empty asm:
// the compiler then keeps them in SGPRs instead of re-fetching them from the
// kernarg segment at each use (every re-fetch is a serialized scalar-cache miss
// on the critical path of a ~us kernel).
template <typename T> __device__ __forceinline__ T keep_s(T v) {
  asm volatile("" : "+s"(v));
  return v;
}
template <typename T> __device__ __forceinline__ T *keep_sp(T *v) {
  // launder as a GLOBAL (address space 1) pointer so that loads through the
  // result are still selected as global_load (a generic pointer would become
  // flat_load, which drains both vmcnt and lgkmcnt at every wait)
  typedef __attribute__((address_space(1))) T *gptr;
  gptr g = (gptr)v;
  asm volatile("" : "+s"(g));
  return (T *)g;
}

// Diagnostic timeline stamps (measurement-only builds: diag_stamps.hip and scripts/microbench
// define QZ_STAMPS and instantiate STAMP != 0).  The product library compiles none of this.  Per
// wave: s_memrealtime (100 MHz, chip-wide) at fixed points, stored once at the end by lane 0 with
// the wave's XCC / HW ids.  STAMP 1: all points; STAMP 2 ("light"): only the start (0) and end
// (4) stamps, so the schedule between them is the product's (bench.py's in-kernel time).
#ifdef QZ_STAMPS
__device__ unsigned long long *g_qz_stamp;
#define QZ_STAMP_DECL unsigned long long qz_st_[6] = {0, 0, 0, 0, 0, 0}
#define QZ_STAMP(k)                                                                  \
  do {                                                                               \
    if constexpr ((STAMP & 3) != 0 && ((STAMP & 3) == 1 || (k) == 0 || (k) == 4)) {  \
      __builtin_amdgcn_sched_barrier(0);                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(qz_st_[k])::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                             \
    }                                                                                \
  } while (0)
#define QZ_STAMP_FLUSH(wave_id)                                                      \
  do {                                                                               \
    if constexpr ((STAMP & 3) != 0) {                                                \
      uint32_t xcc, hw;                                                              \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));             \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));               \
      qz_st_[5] = ((unsigned long long)xcc << 32) | hw;                              \
      if ((threadIdx.x & 63) == 0) {                                                 \
        if constexpr ((STAMP & 3) == 2) {                                            \
          g_qz_stamp[(size_t)(wave_id) * 8 + 0] = qz_st_[0];                         \
          g_qz_stamp[(size_t)(wave_id) * 8 + 4] = qz_st_[4];                         \
        } else {                                                                     \
          for (int k_ = 0; k_ < 6; ++k_) g_qz_stamp[(size_t)(wave_id) * 8 + k_] = qz_st_[k_]; \
        }                                                                            \
      }                                                                              \
    }                                                                                \
  } while (0)
#else
#define QZ_STAMP_DECL
#define QZ_STAMP(k) do {} while (0)
#define QZ_STAMP_FLUSH(wave_id) do {} while (0)
#endif

__device__ __forceinline__ GemvParams load_params(const GemvParams &in) {
  GemvParams p;
  p.B = keep_sp(in.B);
  p.x = keep_sp(in.x);
  p.sc.absmax = keep_sp(in.sc.absmax);
  p.sc.qabsmax = keep_sp(in.sc.qabsmax);
  p.sc.absmax2 = keep_sp(in.sc.absmax2);
  p.sc.code2 = keep_sp(in.sc.code2);
  p.sc.offset = keep_sp(in.sc.offset);
  p.sc.bs2 = keep_s(in.sc.bs2);
  p.bias = keep_sp(in.bias);
  p.y = keep_sp(in.y);
  p.lut = keep_sp(in.lut);
  p.block_base = keep_s(in.block_base);
  p.M = keep_s(in.M);
  p.K = keep_s(in.K);
  p.bs_log2 = keep_s(in.bs_log2);
  p.bs2_log2 = keep_s(in.bs2_log2);
  p.out_scale = keep_s(in.out_scale);
  p.tabsel = keep_s(in.tabsel);
  p.res = keep_sp(in.res);
  p.nw = keep_sp(in.nw);
  p.eps = keep_s(in.eps);
  return p;
}

// Dot of one lane's 16-byte weight chunk (32 codes) with its x slice through the LDS byte
// table.  `jb` selects the lane's bank-private copy; the address of byte m is
// (byte << 7) | jb (WT: one v_perm builds (byte << 8) | jb).  W (wide entries: CL / bf16):
// each entry holds a {hi pair, lo pair} and the dot adds lo x x.
template <bool W, bool WT = false, bool BF = false>
__device__ __forceinline__ float chunk_dot_tab(const u32x4 &wv, const uint32_t (&xh)[16], const uint32_t *s_tab,
                                               uint32_t jb) {
  static_assert(!BF || W, "bf16 entries use the 64-bit table geometry");
  const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  uint32_t v[16], vl[W ? 16 : 1];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t a[4];
    if constexpr (WT) {
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = __builtin_amdgcn_perm(w[d], jb, 0x0C0C0000u | ((4u + m) << 8));
    } else {
      a[0] = ((w[d] << 7) & 0x7F80u) | jb;
      a[1] = ((w[d] >> 1) & 0x7F80u) | jb;
      a[2] = ((w[d] >> 9) & 0x7F80u) | jb;
      a[3] = ((w[d] >> 17) & 0x7F80u) | jb;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if constexpr (W) {
        const u32x2 e = *reinterpret_cast<const u32x2 *>(tb + a[m]);
        v[4 * d + m] = e.x;
        vl[4 * d + m] = e.y;
      } else {
        v[4 * d + m] = *reinterpret_cast<const uint32_t *>(tb + a[m]);
      }
    }
  }
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float &acc = (i & 1) ? s1 : s0;
    if constexpr (BF) {  // bf16 code pairs (hi, lo) against the raw bf16 x pair
      acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, v[i]), __builtin_bit_cast(bf16x2_t, xh[i]),
                                            acc, false);
      acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, vl[i]), __builtin_bit_cast(bf16x2_t, xh[i]),
                                            acc, false);
      continue;
    }
    acc = dot2(v[i], xh[i], acc);
    if constexpr (W) acc = dot2(vl[i], xh[i], acc);   // code residual x x
  }
  return s0 + s1;
}

// fp32 x: byte m of the lane's chunk holds elements 2m (high nibble) and 2m + 1; its 64-bit
// entry {code_hi, code_lo} (fp32) goes into two v_fma_f32 with the raw x.  Same
// 128-B-per-byte-value geometry as the CL table.
__device__ __forceinline__ float chunk_dot_tab_f32(const u32x4 &wv, const uint32_t (&xr)[32], const uint32_t *s_tab,
                                                   uint32_t jb) {
  const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t a[4] = {((w[d] << 7) & 0x7F80u) | jb, ((w[d] >> 1) & 0x7F80u) | jb,
                           ((w[d] >> 9) & 0x7F80u) | jb, ((w[d] >> 17) & 0x7F80u) | jb};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const u32x2 e = *reinterpret_cast<const u32x2 *>(tb + a[m]);
      const int k = 2 * (4 * d + m);
      float &acc = (m & 1) ? s1 : s0;
      acc = fmaf(__uint_as_float(e.x), __uint_as_float(xr[k]), acc);
      acc = fmaf(__uint_as_float(e.y), __uint_as_float(xr[k + 1]), acc);
    }
  }
  return s0 + s1;
}

// Sum over the 64 lanes, result valid in lane 63 only: an inclusive row scan
// (row_shr 1, 2, 4, 8) then row_bcast:15 / row_bcast:31 -- six DPP adds, no
// readlane round trips through SGPRs.
template <int CTRL, int ROWS> __device__ __forceinline__ float dpp_add_rows(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wave_sum_last(float v) {
  v = dpp_add_rows<0x111, 0xF>(v);  // row_shr:1
  v = dpp_add_rows<0x112, 0xF>(v);  // row_shr:2
  v = dpp_add_rows<0x114, 0xF>(v);  // row_shr:4
  v = dpp_add_rows<0x118, 0xF>(v);  // row_shr:8
  v = dpp_add_rows<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  v = dpp_add_rows<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
  return v;
}

// Fills the LDS byte table from a precomputed device table entry `v` (entry
// e = threadIdx.x, already repeated 4 times: one 16-B store covers 4 bank
// copies).  The stores of a thread are rotated by its lane so that each
// 8-lane store group covers all 32 banks.  (Loading 8 pieces per thread to
// make every store address an immediate offset was measured slower: the
// extra loads delay the first weight loads.)
template <int PIECES = kTabCopies / 4>
__device__ __forceinline__ void store_byte_table_entry(uint32_t *s_tab, const u32x4 &v,
                                                       const uint32_t e = threadIdx.x) {
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    const uint32_t piece = (e + (uint32_t)i) & (PIECES - 1);
    reinterpret_cast<u32x4 *>(s_tab)[e * PIECES + piece] = v;
  }
}

// Exponent S (power of two) for a runtime codebook: max|code| * 2^S lies in
// [2^14, 2^15), so every code c * 2^S splits into two normal fp16 values
// ch + cl with ~2^-23 relative error (an all-zero or non-finite book: S = 0).
__device__ __forceinline__ int lut_shift(const float *lut) {
  float mx = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fabsf(lut[i]));
  const int E = (int)(__float_as_uint(mx) >> 23);
  if (mx == 0.0f || E == 255) return 0;
  return max(-100, min(141 - E, 100));
}

// Builds the CL (exact-code) byte table from a runtime fp32 codebook: entry
// e = {hi pair, lo pair} of (code[e >> 4], code[e & 15]) * 2^S.
template <int NT, int PIECES = kTabCopies / 4>
__device__ __forceinline__ void build_byte_table_exact(uint32_t *s_tab, const float *lut, int S) {
  for (int e = threadIdx.x; e < 256; e += NT) {
    const float ca = ldexpf(lut[e >> 4], S), cb = ldexpf(lut[e & 15], S);
    const uint32_t h = cvt_pk_f16_rne(ca, cb);
    const float ra = ca - (float)__builtin_bit_cast(_Float16, (uint16_t)(h & 0xFFFFu));
    const float rb = cb - (float)__builtin_bit_cast(_Float16, (uint16_t)(h >> 16));
    const uint32_t l = cvt_pk_f16_rne(ra, rb);
    store_byte_table_entry<PIECES>(s_tab, u32x4{h, l, h, l}, (uint32_t)e);
  }
}

// Builds the bf16 byte table from a runtime fp32 codebook: entry e = {hi pair, lo pair} of
// (code[e >> 4], code[e & 15]) as bf16 hi + lo (c = hi + lo to ~2^-16).
template <int NT, int PIECES = kTabCopies / 4>
__device__ __forceinline__ void build_byte_table_bf16(uint32_t *s_tab, const float *lut) {
  for (int e = threadIdx.x; e < 256; e += NT) {
    const float ca = lut[e >> 4], cb = lut[e & 15];
    const uint32_t ha = __builtin_bit_cast(uint16_t, (__bf16)ca), hb = __builtin_bit_cast(uint16_t, (__bf16)cb);
    const float ra = ca - __builtin_bit_cast(float, ha << 16), rb = cb - __builtin_bit_cast(float, hb << 16);
    const uint32_t la = __builtin_bit_cast(uint16_t, (__bf16)ra), lb = __builtin_bit_cast(uint16_t, (__bf16)rb);
    const uint32_t h = ha | (hb << 16), l = la | (lb << 16);
    store_byte_table_entry<PIECES>(s_tab, u32x4{h, l, h, l}, (uint32_t)e);
  }
}

// The fp32 byte table from a runtime codebook: entry e = {code[e >> 4], code[e & 15]}.
template <int NT, int PIECES = kTabCopies / 4>
__device__ __forceinline__ void build_byte_table_f32(uint32_t *s_tab, const float *lut) {
  for (int e = threadIdx.x; e < 256; e += NT) {
    const uint32_t a = __float_as_uint(lut[e >> 4]), b = __float_as_uint(lut[e & 15]);
    store_byte_table_entry<PIECES>(s_tab, u32x4{a, b, a, b}, (uint32_t)e);
  }
}

// One step's worth of loads for R rows.  Branch-free: out-of-range rows and
// the inactive tail lanes of the last step read a clamped in-bounds address
// and are zeroed at compute time, so the compiler issues every load up front
// (no exec-masked regions, no lazily re-read kernel arguments).  The lane's x
// slice (32 activations) is loaded raw, so the loads retire in issue order; NOX:
// x comes from an LDS image instead (the fused pre-norm).
template <bool DQ, int DT, int R, bool NOX, bool FS> struct StepLoads {
  static constexpr int kXWords = DT == QZ_DT_F32 ? 32 : 16;  // raw x dwords per lane
  u32x4 wv[R];
  uint32_t q[R];    // DQ: 8-bit scale code
  float a[R];       // DQ: absmax2 entry; else: fp32 absmax
  uint32_t xr[kXWords];
  int xb;  // first activation index of this lane's chunk
  bool on;

  __device__ __forceinline__ void load_x(const void *x, uint32_t e0) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(x) +
                                                     e0 * (DT == QZ_DT_F32 ? 4u : 2u));
#pragma unroll
    for (int i = 0; i < kXWords / 4; ++i) {
      const u32x4 v = p[i];
      xr[4 * i] = v.x; xr[4 * i + 1] = v.y; xr[4 * i + 2] = v.z; xr[4 * i + 3] = v.w;
    }
  }

  // All offsets are 32-bit unsigned (the launcher guarantees M*K < 2^32): the
  // loads then use the SGPR-base + 32-bit VGPR offset form, with no 64-bit
  // VALU address arithmetic per load.
  __device__ __forceinline__ void issue(const GemvParams &p, int row0, int s, int lane, int row_bytes) {
    if constexpr (FS) {
      issue_full(p, row0, s, lane, row_bytes);
      return;
    }
    const uint32_t boff_raw = ((uint32_t)s << 10) + ((uint32_t)lane << 4);
    on = boff_raw < (uint32_t)row_bytes;
    const uint32_t boff = on ? boff_raw : 0u;
    xb = 2 * (int)boff;
    if constexpr (!NOX) load_x(p.x, 2u * boff);
    // per row: weights then that row's scale, so row r can be consumed while
    // rows > r are still in flight (vmcnt retires in issue order)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t row = (uint32_t)min(row0 + r, p.M - 1);  // wave-uniform
      const unsigned char *rowp = p.B + (size_t)row * (uint32_t)row_bytes;
      wv[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rowp + boff));
      const uint32_t b = (uint32_t)p.block_base + ((row * (uint32_t)p.K + 2u * boff) >> p.bs_log2);
      if constexpr (DQ) {
        q[r] = p.sc.qabsmax[b];
        a[r] = p.sc.absmax2[b >> p.bs2_log2];
      } else {
        a[r] = p.sc.absmax[b];
      }
    }
  }

  // Full-step form (host-checked: K % 2048 == 0, K % blocksize == 0, and the
  // step's blocks share one absmax2 entry): every lane is in range, the
  // row's first scale block is a wave-uniform SGPR base, the lane's block
  // offset is one VGPR shared by all R rows, and the double-quant absmax2
  // entry of a (row, step) is ONE scalar load.
  __device__ __forceinline__ void issue_full(const GemvParams &p, int row0, int s, int lane, int row_bytes) {
    const uint32_t boff = ((uint32_t)s << 10) + ((uint32_t)lane << 4);
    on = true;
    xb = 2 * (int)boff;
    if constexpr (!NOX) load_x(p.x, 2u * boff);
    const uint32_t lb = (2u * boff) >> p.bs_log2;                 // lane's block within the row
    const uint32_t sb = ((uint32_t)s << 11) >> p.bs_log2;         // step's first block within the row
    const uint32_t bpr = (uint32_t)p.K >> p.bs_log2;              // blocks per row
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t row = (uint32_t)min(row0 + r, p.M - 1);  // wave-uniform
      const unsigned char *rowp = p.B + (size_t)row * (uint32_t)row_bytes;
      wv[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rowp + boff));
      const uint32_t rb = (uint32_t)p.block_base + row * bpr;    // wave-uniform
      if constexpr (DQ) {
        q[r] = (p.sc.qabsmax + rb)[lb];
        typedef const __attribute__((address_space(4))) float *cfp;
        a[r] = ((cfp)p.sc.absmax2)[(rb + sb) >> p.bs2_log2];
      } else {
        a[r] = (p.sc.absmax + rb)[lb];
      }
    }
  }
};

// Fused pre-norm (NRM): the bit-exact sum of squares of k_rmsnorm (layer_ops.hip): thread t adds
// the squares of 16-B chunks t, t + 256, ... in element order, then the xor butterfly of the wave
template <int DT> __device__ __forceinline__ float norm_chunk_ss(const u32x4 &v, float ss) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t b = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
    const float h = DT == QZ_DT_F16 ? __half2float(__ushort_as_half((unsigned short)b)) : __uint_as_float(b << 16);
    ss = __fadd_rn(ss, __fmul_rn(h, h));
  }
  return ss;
}
__device__ __forceinline__ float norm_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// x' = storage(w * storage(x * rs)) for the 8 elements of a 16-B chunk (k_rmsnorm's second pass)
template <int DT> __device__ __forceinline__ u32x4 norm_chunk_apply(const u32x4 &xv, const u32x4 &wv, float rs) {
  const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w}, ww[4] = {wv.x, wv.y, wv.z, wv.w};
  uint32_t o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    float r2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t xb = (xw[d] >> (16 * h)) & 0xFFFFu, wb = (ww[d] >> (16 * h)) & 0xFFFFu;
      // x * rs rounded to fp32, then to the storage dtype (torch's two roundings; the asm keeps
      // hipcc from folding the multiply into one v_fma_mix rounding), then the weight product
      float xs = __fmul_rn(DT == QZ_DT_F16 ? __half2float(__ushort_as_half((unsigned short)xb)) : __uint_as_float(xb << 16),
                           rs);
      asm volatile("" : "+v"(xs));
      if constexpr (DT == QZ_DT_F16) {
        const float hn = __half2float(__float2half_rn(xs));
        r2[h] = __fmul_rn(__half2float(__ushort_as_half((unsigned short)wb)), hn);
      } else {
        const float hn = __bfloat162float(__float2bfloat16(xs));
        r2[h] = __fmul_rn(__uint_as_float(wb << 16), hn);
      }
      asm volatile("" : "+v"(r2[h]));
    }
    if constexpr (DT == QZ_DT_F16)
      o[d] = (uint32_t)__half_as_ushort(__float2half_rn(r2[0])) | ((uint32_t)__half_as_ushort(__float2half_rn(r2[1])) << 16);
    else
      o[d] = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(r2[0])) |
             ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(r2[1])) << 16);
  }
  return u32x4{o[0], o[1], o[2], o[3]};
}
// LDS image of x' (NRM): step s's 2048 activations in a 4 KiB block, lane l's 64-B slice at 64 l,
// its 16-B chunk i at position i ^ ((l >> 2) & 3) -- the four ds_read_b128 of a step are then
// conflict-free in every lane group
__device__ __forceinline__ uint32_t norm_x_off(uint32_t chunk) {  // chunk = element / 8
  const uint32_t s = chunk >> 8, l = (chunk >> 2) & 63u, i = chunk & 3u;
  return (s << 12) + (l << 6) + ((i ^ ((l >> 2) & 3u)) << 4);
}

// Grouped launch: up to kMaxSeg GEMVs that share x and K (q/k/v, gate/up of
// one decoder layer) in ONE grid.  Segment i owns row blocks
// [start[i], start[i+1]); each segment keeps its own weights, statistics,
// offset, bias and output, so every output is bit-identical to its own
// qz_gemv_4bit launch with the same geometry.  total = all segments' blocks.
constexpr int kMaxSeg = 4;
struct GemvGroup {
  GemvParams seg[kMaxSeg];
  int start[kMaxSeg];
  int nseg;
  int total;
};

// The decode GEMV body.
//  DQ: double-quantised scales; DT: activation dtype; R rows per wave; WK waves along K; NW waves
//  per workgroup; FS: full-step loads (host-checked); CL: exact codes (fp16 x); WT: the 256-B-entry
//  table; NRM: x is RMSNorm'd in the prologue (bit-identical to qz_rmsnorm) into an LDS image;
//  PAIR (LlamaMLP's gate/up): waves 0-1 take R-row groups of pair[0] (gate_proj), waves 2-3 the
//  same rows of pair[1] (up_proj), and the epilogue stores act_fn(gate) * up (k_silu_mul's
//  arithmetic) into pair[0].y, the input of down_proj; TWO: the wave owns exactly two K-steps
//  (host-checked) and runs them as straight-line code -- issue, barrier, issue step 2, decode,
//  decode -- with no loop whose shared dominator would take the waits of step 1's scale codes above
//  step 2's issue (profiles/r4_gemv_two_step.txt); PS (pair launches with the norm): persistent
//  workgroups -- each takes row blocks blockIdx.x, + gridDim.x, ..., so its prologue (byte table,
//  code2, the normalised x) is paid once, and the next block's first step is issued before the
//  current block's epilogue.
template <bool DQ, int DT, int R, int WK, int NW, bool FS, bool CL, bool WT, bool NRM, bool PAIR, bool TWO, bool PS,
          int STAMP = 0>
__device__ __forceinline__ void gemv_body(const GemvParams &p_in, const int block, const GemvParams *pair = nullptr) {
  static_assert(!NRM || (NW == 4 && FS && DT != QZ_DT_F32), "fused pre-norm: 4 waves, full steps, 16-bit activations");
  static_assert(!PAIR || (NW == 4 && WK == 1 && DT != QZ_DT_F32), "pair: 4 waves, WK = 1, 16-bit activations");
  static_assert(!PS || (PAIR && FS), "persistent form: pair launches, full steps");
  static_assert(!TWO || (FS && WK == 1), "two-step form: full steps, whole rows per wave");
  static_assert(!CL || DT == QZ_DT_F16, "exact codes are the fp16-activation table");
  static_assert(NW * 64 >= 256, "one byte-table entry per thread");
  constexpr int kPieces = WT ? 16 : kTabCopies / 4;
  QZ_STAMP_DECL;
  QZ_STAMP(0);
  const GemvParams p = load_params(p_in);
  constexpr int RG = NW / WK;
  constexpr bool kBF = DT == QZ_DT_BF16;    // bf16 code pairs hi + lo in 64-bit entries
  constexpr bool kF32 = DT == QZ_DT_F32;    // fp32 code table, v_fma_f32
  constexpr bool kWide = CL || kBF || kF32; // 64-bit entries
  __shared__ float s_code2[PAIR ? 2 : 1][DQ ? 256 : 1];   // PAIR: each weight's own double-quant code
  __shared__ float s_part[NW][R];
  __shared__ float s_part2[PS ? 2 : 1][NW][R];   // PS: by block parity (no barrier after the reads)
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[(WT ? 2 : 1) * kTabDwords];
  extern __shared__ __attribute__((aligned(16))) unsigned char s_x[];

  const int lane = threadIdx.x & (kWave - 1);
  // wave-uniform by construction; readfirstlane makes it provable, so the step
  // loop compiles to scalar branches instead of exec-masked divergent flow
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int wk = wave % WK;
  const int rg = wave / WK;
  int row0 = PAIR ? (block * 2 + (wave & 1)) * R : (block * RG + rg) * R;
  const int cb = PAIR ? (wave >> 1) : 0;   // this wave's code2 table
  const int row_bytes = p.K >> 1;
  const int nsteps = (row_bytes + 1023) >> 10;

  // 1. the double-quant code table load goes out first (it gates the barrier)
  float c2 = 0.0f, c2b = 0.0f, offset = 0.0f;
  if constexpr (DQ) {
    if constexpr (PAIR) {
      c2 = keep_sp(pair[0].sc.code2)[threadIdx.x];
      c2b = keep_sp(pair[1].sc.code2)[threadIdx.x];
    } else if (NW * 64 == 256 || threadIdx.x < 256) {
      c2 = p.sc.code2[threadIdx.x & 255];
    }
    offset = *p.sc.offset;
  }
  // 1b. the precomputed byte-table entry of this thread (issued before the
  // weights, so waiting for it does not wait for the first HBM step)
  u32x4 tab_entry = {0u, 0u, 0u, 0u};
  if (!p.lut && threadIdx.x < 256) {
    const ByteTable *bt = kF32 ? (p.tabsel ? &g_byte_tab_fp4_f32 : &g_byte_tab_nf4_f32)
                          : kBF ? (p.tabsel ? &g_byte_tab_fp4_bf : &g_byte_tab_nf4_bf)
                                : (CL ? &g_byte_tab_nf4x : (p.tabsel ? &g_byte_tab_fp4 : &g_byte_tab_nf4));
    tab_entry = reinterpret_cast<const u32x4 *>(bt->v)[threadIdx.x];
  }
  // 1c. NRM: this thread's chunks of x and of the norm weight (L2-resident), ahead of the
  // weights.  The first kNHeld chunks (K <= 4096: all of them) stay in registers across the
  // barrier; later ones are read again after it (registers would cost occupancy)
  constexpr int kNChunks = NRM ? 8 : 1;   // up to 8 x 256 chunks of 8: K <= 16384
  constexpr int kNHeld = NRM ? 2 : 1;
  u32x4 nx[kNChunks], nwh[kNHeld];
  const int n_nchunk = p.K >> 3;
  if constexpr (NRM) {
#pragma unroll
    for (int i = 0; i < kNChunks; ++i) {
      const int c = (int)threadIdx.x + 256 * i;
      if (c < n_nchunk) nx[i] = reinterpret_cast<const u32x4 *>(p.x)[c];
    }
#pragma unroll
    for (int i = 0; i < kNHeld; ++i) {
      const int c = (int)threadIdx.x + 256 * i;
      if (c < n_nchunk) nwh[i] = reinterpret_cast<const u32x4 *>(p.nw)[c];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // 2. this wave's first step of HBM traffic
  typedef StepLoads<DQ, DT, R, NRM, FS> Loads;
  Loads cur, other;
  int s = wk;
  cur.issue(p, row0, s < nsteps ? s : 0, lane, row_bytes);
  const bool have = s < nsteps;
  const int n_my = have ? (nsteps - wk + WK - 1) / WK : 0;  // this wave's steps: s = wk, wk + WK, ...
  // 3. stage the code table (waits only for the code load: it was issued first)
  if constexpr (DQ) {
    if (NW * 64 == 256 || threadIdx.x < 256) s_code2[0][threadIdx.x & 255] = c2;
    if constexpr (PAIR) s_code2[PAIR ? 1 : 0][threadIdx.x] = c2b;
  }
  __shared__ float s_nss[NRM ? 4 : 1];
  if constexpr (NRM) {  // sum of squares: per thread in chunk order, per wave by the xor butterfly
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < kNChunks; ++i)
      if ((int)threadIdx.x + 256 * i < n_nchunk) ss = norm_chunk_ss<DT>(nx[i], ss);
    ss = norm_wave_sum(ss);
    if (lane == 0) s_nss[wave] = ss;
  }
  // output scale: the codebook's (FP4 x12: 1/12; exact NF4: 2^-14), or for a
  // runtime codebook (fp16 x: always exact codes) 2^-S of its in-kernel split
  float out_scale = p.out_scale;
  if constexpr (kF32) {
    if (p.lut) {
      out_scale = 1.0f;
      build_byte_table_f32<NW * 64, kPieces>(s_tab, p.lut);
    } else if (threadIdx.x < 256) {
      store_byte_table_entry<kPieces>(s_tab, tab_entry);
    }
  } else if constexpr (kBF) {
    if (p.lut) {
      out_scale = 1.0f;
      build_byte_table_bf16<NW * 64, kPieces>(s_tab, p.lut);
    } else if (threadIdx.x < 256) {
      store_byte_table_entry<kPieces>(s_tab, tab_entry);
    }
  } else if constexpr (CL) {
    if (p.lut) {
      const int S = lut_shift(p.lut);
      out_scale = ldexpf(1.0f, -S);
      build_byte_table_exact<NW * 64, kPieces>(s_tab, p.lut, S);
    } else if (threadIdx.x < 256 && (STAMP & 48) == 0) {
      store_byte_table_entry<kPieces>(s_tab, tab_entry);
    }
  } else if (threadIdx.x < 256) {   // fp16 codes: the built-in books only (a runtime book is exact)
    store_byte_table_entry<kPieces>(s_tab, tab_entry);
  }
  // STAMP & 16 / 32 (microbenchmark ablations, wrong results): no byte-table stores / also no
  // prologue barrier
  if constexpr ((STAMP & 32) == 0) __syncthreads();
  if constexpr (NRM) {  // rs as k_rmsnorm (torch MeanOps: sum * (1/N), then rsqrt(var + eps)); x' -> LDS
    const float tot = __fadd_rn(__fadd_rn(s_nss[0], s_nss[1]), __fadd_rn(s_nss[2], s_nss[3]));
    const float rs = rsqrtf(__fadd_rn(__fmul_rn(tot, 1.0f / (float)p.K), p.eps));
#pragma unroll
    for (int i = 0; i < kNChunks; ++i) {
      const int c = (int)threadIdx.x + 256 * i;
      if (c < n_nchunk) {
        const u32x4 xv = i < kNHeld ? nx[i] : reinterpret_cast<const u32x4 *>(p.x)[c];
        const u32x4 wv = i < kNHeld ? nwh[i < kNHeld ? i : 0] : reinterpret_cast<const u32x4 *>(p.nw)[c];
        *reinterpret_cast<u32x4 *>(s_x + norm_x_off((uint32_t)c)) = norm_chunk_apply<DT>(xv, wv, rs);
      }
    }
    __syncthreads();
  }
  QZ_STAMP(1);
  const uint32_t jb = WT ? (kWide ? (uint32_t)(lane & 31) << 3 : (uint32_t)lane << 2)
                        : (kWide ? (uint32_t)(lane & (kTabCopiesCL - 1)) << 3 : (uint32_t)(lane & 31) << 2);

  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;

  auto consume = [&](const Loads &c) {
    if constexpr (NRM) {
      auto &xr = const_cast<Loads &>(c).xr;
      const uint32_t c0 = (uint32_t)c.xb >> 3;  // the lane's first chunk
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(s_x + norm_x_off(c0 + (uint32_t)i));
        xr[4 * i] = v.x; xr[4 * i + 1] = v.y; xr[4 * i + 2] = v.z; xr[4 * i + 3] = v.w;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float am;
      if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[cb][c.q[r]], c.a[r]), offset);
      else am = c.a[r];
      am = c.on ? am : 0.0f;
      float d;
      if constexpr (kF32) {
        d = chunk_dot_tab_f32(c.wv[r], c.xr, s_tab, jb);
      } else {
        d = chunk_dot_tab<kWide, WT, kBF>(c.wv[r], c.xr, s_tab, jb);
      }
      acc[r] = fmaf(d, am, acc[r]);
    }
  };
  // Ping-pong over two named load sets, whole pairs per iteration.  No path
  // may consume `other` where another path consumes `cur`: hipcc would merge
  // the two tails into one block fed by register COPIES, and copying a
  // register whose load is in flight forces vmcnt(0) -- the prefetch is then
  // waited for before the current step is decoded.  Every consume(cur) below
  // reads the same registers on every path, so no copies are needed.  The next
  // step's loads are issued UNCONDITIONALLY before the current step is consumed
  // (a conditional prefetch makes hipcc's waitcnt pass pick the count valid on
  // both paths -- vmcnt(0) -- which serialises HBM traffic with the decode).
  if constexpr (PS) {
    // the pair epilogue of block `blk` (the one after the loop below, with s_part by parity)
    auto pair_out = [&](int blk, int par) {
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
      if (lane == kWave - 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float o = v[r] * out_scale;
          if (p.bias) o += load_f32<DT>(p.bias, min(row0 + r, p.M - 1));
          s_part2[par][wave][r] = o;
        }
      }
      __syncthreads();
      if ((int)threadIdx.x < 2 * R) {
        const int g2 = threadIdx.x / R, r = threadIdx.x % R;
        const int row = (blk * 2 + g2) * R + r;
        if (row < p.M) {
          const float gv = round_store<DT>(s_part2[par][g2][r]), uv = round_store<DT>(s_part2[par][2 + g2][r]);
          const float a = round_store<DT>(__fdiv_rn(gv, __fadd_rn(1.0f, expf(-gv))));
          store_f32<DT>(keep_sp(pair[0].y), row, __fmul_rn(a, uv));
        }
      }
    };
    const int nblocks = (p.M + 2 * R - 1) / (2 * R);
    int blk = block;
    for (int it = 0;; ++it) {
      if constexpr (TWO) {
        other.issue(p, row0, s + WK, lane, row_bytes);
        __builtin_amdgcn_sched_barrier(0);
        consume(cur);
        consume(other);
      } else {
        // n_my steps (WK = 1: every step of the row), cur = step 0 issued: the early ping-pong --
        // `other` one step ahead, each set re-issued right after it is consumed
        const int n = n_my;
        other.issue(p, row0, n >= 2 ? 1 : 0, lane, row_bytes);
        __builtin_amdgcn_sched_barrier(0);
        int j = 0, ss = 0;
        for (; j + 3 < n; j += 2) {
          consume(cur);
          cur.issue(p, row0, ss + 2, lane, row_bytes);
          __builtin_amdgcn_sched_barrier(0);
          consume(other);
          other.issue(p, row0, ss + 3, lane, row_bytes);
          __builtin_amdgcn_sched_barrier(0);
          ss += 2;
        }
        if (n - j == 3) {
          consume(cur);
          cur.issue(p, row0, ss + 2, lane, row_bytes);
          __builtin_amdgcn_sched_barrier(0);
          consume(other);
          consume(cur);
        } else if (n - j == 2) {
          consume(cur);
          consume(other);
        } else {
          consume(cur);
        }
      }
      const int nb = blk + (int)gridDim.x;   // workgroup-uniform
      if (nb >= nblocks) {
        pair_out(blk, it & 1);
        break;
      }
      const int nrow0 = (nb * 2 + (wave & 1)) * R;
      cur.issue(p, nrow0, s, lane, row_bytes);   // the next block's first step, ahead of this epilogue
      __builtin_amdgcn_sched_barrier(0);
      pair_out(blk, it & 1);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.0f;
      blk = nb;
      row0 = nrow0;
    }
    return;
  } else if constexpr (TWO) {
    other.issue(p, row0, s + WK, lane, row_bytes);
    __builtin_amdgcn_sched_barrier(0);
    consume(cur);
    QZ_STAMP(2);
    consume(other);
  } else if (have) {
    const int n = n_my;
    int j = 0;
    for (; j + 2 < n; j += 2) {
      other.issue(p, row0, s + WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the decode
      consume(cur);
      cur.issue(p, row0, s + 2 * WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      consume(other);
      s += 2 * WK;
    }
    if (n - j == 2) {
      other.issue(p, row0, s + WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      consume(cur);
      QZ_STAMP(2);
      consume(other);
    } else {
      consume(cur);
    }
  }

  QZ_STAMP(3);
  if constexpr (PAIR) {  // gate (waves 0-1) and up (waves 2-3) of the same rows meet in LDS
    float v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
    if (lane == kWave - 1) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float o = v[r] * out_scale;
        if (p.bias) o += load_f32<DT>(p.bias, min(row0 + r, p.M - 1));
        s_part[wave][r] = o;
      }
    }
    __syncthreads();
    if ((int)threadIdx.x < 2 * R) {
      const int g2 = threadIdx.x / R, r = threadIdx.x % R;
      const int row = (block * 2 + g2) * R + r;
      if (row < p.M) {
        // h = act_fn(gate) * up on the projections as torch stores them; k_silu_mul's
        // x / (1 + exp(-x)) rounded, then the product rounded by the store
        const float gv = round_store<DT>(s_part[g2][r]), uv = round_store<DT>(s_part[2 + g2][r]);
        const float a = round_store<DT>(__fdiv_rn(gv, __fadd_rn(1.0f, expf(-gv))));
        store_f32<DT>(keep_sp(pair[0].y), row, __fmul_rn(a, uv));
      }
    }
    return;
  }
  if constexpr (WK == 1) {  // the wave owns whole rows: lane 63 reduces and stores them
    float v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
    if (lane == kWave - 1) {
      // 16-bit outputs of a row pair inside M go out as one dword (row0 is even for even R)
      constexpr bool kPack = DT != QZ_DT_F32 && R % 2 == 0;
      const bool pack = kPack && row0 + R <= p.M && (reinterpret_cast<uintptr_t>(p.y) & 3u) == 0;
      if (pack) {
#pragma unroll
        for (int r = 0; r < R; r += 2) {
          float o0 = v[r] * out_scale, o1 = v[r + 1] * out_scale;
          if (p.bias) {
            o0 += load_f32<DT>(p.bias, row0 + r);
            o1 += load_f32<DT>(p.bias, row0 + r + 1);
          }
          o0 = add_res<DT>(o0, p.res, row0 + r);
          o1 = add_res<DT>(o1, p.res, row0 + r + 1);
          reinterpret_cast<uint32_t *>(p.y)[(row0 + r) >> 1] = pack16<DT>(o0, o1);
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int row = row0 + r;
          if (row < p.M) {
            float o = v[r] * out_scale;
            if (p.bias) o += load_f32<DT>(p.bias, row);
            o = add_res<DT>(o, p.res, row);
            store_f32<DT>(p.y, row, o);
          }
        }
      }
    }
    QZ_STAMP(4);
    QZ_STAMP_FLUSH(block * NW + wave);
    return;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float v = wave_sum_last(acc[r]);
    if (lane == kWave - 1) s_part[wave][r] = v;
  }
  __syncthreads();
  if ((int)threadIdx.x < RG * R) {
    const int g = threadIdx.x / R, r = threadIdx.x % R;
    const int row = (block * RG + g) * R + r;
    if (row < p.M) {
      float v = 0.0f;
#pragma unroll
      for (int k = 0; k < WK; ++k) v += s_part[g * WK + k][r];
      v *= out_scale;
      if (p.bias) v += load_f32<DT>(p.bias, row);
      store_f32<DT>(p.y, row, add_res<DT>(v, p.res, row));
    }
  }
}

// ---------------------------------------------------------------------------
// host side: knobs, geometry, argument checks
// ---------------------------------------------------------------------------

// Measurement knobs of the launch geometry.  Read ONCE, when the library is loaded (a variable
// set later changes nothing; qz_gemv_set_knob changes one explicitly), and reported by
// qz_gemv_knobs() -- bench.py copies that into its line's config, so a stray variable on a box
// cannot change what is measured unseen.
struct Knobs {
  int wide8;    // QZ_GEMV_WIDE8=0: long-K exact-code GEMVs on 4-wave workgroups (default: 8 waves, 256-B table)
  int norm_r;   // QZ_GROUPED_NORM_R=1|2|4: rows per wave of the normed grouped launch (0 = geometry's)
  int pair_r;   // QZ_PAIR_R=2|3|4|6|8: rows per wave of the pair launch (0 = geometry's)
  int pair_wt;  // QZ_PAIR_WT=0: the persistent pair keeps the 16-copy exact table (default 1)
  int pair_ps;  // QZ_PAIR_PS: 0 = one workgroup per block, 1..8 = workgroups per CU, >= 16 = the grid; -1 = default
  int pair_wk1; // QZ_PAIR_WK1: where the grouped geometry splits K over waves (K = 8192), the pair launch
                // 2 (default): keeps whole rows per wave, the norm fused (persistent, as many per CU as the
                // LDS admits); 1: whole rows, a norm declined (the caller runs the norm launch first);
                // 0: declines these geometries (round 4: grouped launch + SiLU launch)
};
constexpr int kNormMaxBlocks = 4096;
// fused norm prologue at K-split geometries: at most this many normalised values over all workgroups
constexpr long long kNormSplitMaxValues = 1LL << 23;
constexpr size_t kLdsPerCU = 160 * 1024;   // gfx950: LDS per compute unit
// the knobs the library read at load (gemv.hip); qz_gemv_set_knob changes one explicitly
Knobs &gemv_knobs();

static int ilog2(long long v) {
  int l = 0;
  while ((1LL << l) < v) ++l;
  return (1LL << l) == v ? l : -1;
}

// Geometries choose_geometry can return: (R, WK) in {(4,1), (4,2), (2,1), (1,1), (1,2), (1,4)}.
// two_steps(K, WK): every wave owns exactly two full K-steps (the straight-line TWO form;
// profiles/r4_gemv_two_step.txt).  WK = 1 only: at K = 8192, WK = 2 (the Llama-3-70B q/k/v and o
// shapes, R = 4) hipcc gave the straight-line body 259-278 VGPRs against 130 for the loop form --
// one wave per SIMD (profiles/r4_bench_70b_two_step_regression.txt)
static inline bool two_steps(int K, int WK, bool fs) { return fs && WK == 1 && K == 2 * 2048; }

// Geometry (WK = waves along K, R = rows per wave) for the byte-table decode,
// from the measured shape sweep in DESIGN.md section 4.1:
//  * > 64 Mi weights (gate/up groups, 8192x28672, ...): R=4 -- more bytes in
//    flight per wave and fewer x/scale loads per weight byte;
//  * smaller: R=2;
//  * WK=1 (a wave owns whole rows: no cross-wave reduction), then R halves /
//    WK doubles until the grid has >= 2048 waves, so small-M slices (TP
//    shards, 1024-row k/v projections) still fill the 256 CUs.
//  * fp32 x (128 B of x per lane per step, twice the weight bytes of a row pair): R=4 down to
//    1024 waves (profiles/r2_gemv_f32_R.txt: 4096^2 6.36 -> 5.87 us, 14336x4096 17.9 -> 13.9).
static void choose_geometry(int M, int K, int dtype, int *R, int *WK) {
  const int nsteps = ((K >> 1) + 1023) >> 10;
  const bool f32 = dtype == QZ_DT_F32;
  // (exactly 64 Mi weights -- the Llama-3-70B o_proj, 8192 x 8192 -- takes R = 2 with whole rows:
  //  10.37 vs 10.85 us at R = 4, WK = 2, profiles/r5_pair_k8192_forms.txt geom8k)
  *R = (f32 || (long long)M * K > (1LL << 26)) ? 4 : 2;
  *WK = 1;
  // * 4 K-steps per row (K = 8192, the Llama-3-70B q/k/v, o and gate/up) at R=4: two waves per
  //   row, two steps each (profiles/r2_gemv_wk70.txt: 10240x8192 14.0 -> 11.3 us, 8192^2 11.0 ->
  //   9.4, 57344x8192 55.1 -> 51.5; K = 4096 and 14336 keep WK = 1)
  if (*R == 4 && nsteps == 4 && !f32) *WK = 2;
  const long long min_waves = f32 ? 1024 : 2048;
  while ((long long)((M + *R - 1) / *R) * (*WK) < min_waves) {
    if (*R > 1) *R >>= 1;
    else if (*WK < 4 && *WK * 2 <= nsteps) *WK <<= 1;
    else break;
  }
}

// Full-step kernels (StepLoads::issue_full) need every K-step (2048 weights)
// in range and aligned to scale blocks, and each step's blocks inside one
// double-quant group.
static bool full_steps(int K, int blocksize, int blocksize2, bool dq, long long block_base) {
  if (K % 2048 != 0 || K % blocksize != 0) return false;
  const long long step_blocks = blocksize >= 2048 ? 1 : 2048 / blocksize;
  if (block_base % step_blocks != 0) return false;
  return !dq || blocksize2 % step_blocks == 0;
}

// The byte table a launch uses and the scale it undoes on the output.  bf16 / fp32 x: the NF4 or
// FP4 x12 code table of that dtype; fp16 x: fp16-rounded NF4 (tabsel 0), FP4 x12 (1) or the exact
// NF4 codes x 2^14 (CL, 2).  A runtime codebook is converted in kernel (out_scale set there).
static void set_tables(int quant_type, const float *lut, bool cl, int dtype, GemvParams *p) {
  const bool fp4 = !lut && quant_type == QZ_FP4;
  p->tabsel = fp4 ? 1 : (cl && dtype == QZ_DT_F16 ? 2 : 0);
  p->out_scale = fp4 ? 1.0f / 12.0f : 1.0f;
  if (dtype == QZ_DT_F16 && cl && !lut) p->out_scale = 1.0f / (float)(1 << kNF4ExactShift);
}

// Exact codes: a runtime codebook is always decoded exactly (the reference
// ABI's fp32 quant_map); QZ_EXACT_CODES asks for it with the built-in NF4 book.
// The built-in FP4 book x12 is exact in fp16 already.
static bool exact_codes(int quant_type_flags, const float *lut) {
  if (lut) return true;
  return (quant_type_flags & QZ_EXACT_CODES) && (quant_type_flags & ~QZ_EXACT_CODES) == QZ_NF4;
}

// Validates one GEMV's arguments and fills its kernel parameters (everything
// except the decode tables).  Returns QZ_OK or a negative status.
static int make_params(int M, int K, const void *x, int dtype, const unsigned char *B, int quant_type, int blocksize,
                       const float *absmax, const unsigned char *qabsmax, const float *absmax2, const float *code2,
                       const float *offset, int blocksize2, long long block_base, const float *lut, const void *bias,
                       void *y, GemvParams *p, bool *vec_ok) {
  if (!x || !B || !y || M < 0 || K < 0) return QZ_ERR_ARG;
  quant_type &= ~QZ_EXACT_CODES;
  if ((absmax == nullptr) == (qabsmax == nullptr)) return QZ_ERR_ARG;
  const bool dq = qabsmax != nullptr;
  if (dq && (!absmax2 || !code2 || !offset)) return QZ_ERR_ARG;
  if (quant_type != QZ_FP4 && quant_type != QZ_NF4) return QZ_ERR_DTYPE;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16 && dtype != QZ_DT_F32) return QZ_ERR_DTYPE;
  const int bsl = ilog2(blocksize);
  const int bs2l = dq ? ilog2(blocksize2) : 0;
  if (bsl < 1 || bs2l < 0) return QZ_ERR_BLOCKSIZE;
  p->B = B;
  p->x = x;
  p->sc = ScaleSrc{absmax, qabsmax, absmax2, code2, offset, blocksize2};
  p->bias = bias;
  p->y = y;
  p->lut = lut;
  p->block_base = block_base;
  p->M = M;
  p->K = K;
  p->bs_log2 = bsl;
  p->bs2_log2 = bs2l;
  p->out_scale = 1.0f;
  p->tabsel = 0;
  p->nw = nullptr;
  p->eps = 0.0f;
  p->res = nullptr;
  *vec_ok = K > 0 && (K % 32) == 0 && blocksize >= 32 && (reinterpret_cast<uintptr_t>(B) % 16) == 0 &&
            (reinterpret_cast<uintptr_t>(x) % 16) == 0 &&
            (long long)M * K + 2LL * 1024 < (1LL << 32) &&            // 32-bit element offsets
            block_base + (long long)M * K / blocksize < (1LL << 32);   // 32-bit block indices
  return QZ_OK;
}

}  // namespace qz

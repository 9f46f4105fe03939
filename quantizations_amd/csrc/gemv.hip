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
// loaded once and reused R times; the 4 waves of a 256-thread workgroup are
// split WK ways along K (steps s = wk, wk+WK, ...) and RG = 4/WK ways along
// rows, and the WK partial sums meet in LDS.  Weight loads are 16 B/lane
// (1 KiB per wave instruction, fully coalesced) and non-temporal: each byte
// is read exactly once per call.
//
// Nibble decode (production: kModeTab).  A workgroup first writes a 256-entry
// table to LDS: entry b = the two fp16 codes of packed byte b, i.e. exactly
// the half2 operand that v_dot2 multiplies with the natural-order x pair.
// Decoding a byte is then one address computation (2 VALU) and one
// ds_read_b32; the table is stored 32 times, copy j wholly inside bank j, and
// lane l reads copy l % 32, so the random byte values never conflict.  Any
// 16-entry codebook works (NF4, FP4 x12 with the sign in bit 3, a runtime LUT).
// The older register-only decodes are kept for the microbenchmarks:
//  * kModeFP4: the 8 FP4 magnitudes x12 have zero low bytes, so one v_perm
//    per 4 nibbles yields the fp16 high bytes and the sign bit is OR-ed in.
//  * kModeLUT16: two 8-entry v_perm lookups per fp16 byte plane, AND-combined
//    on bit 3, then pairs (e0,e2),(e4,e6),(e1,e3),(e5,e7).  ~3.5 VALU ops per
//    weight, half of them half-rate v_perm: VALU-issue-bound on gfx950.
// Products: v_dot2_f32_f16 (fp16 x fp16 exact products, fp32 accumulate);
// per 32-element chunk the fp32 dot is scaled by the block absmax with one
// FMA.  On the product byte-table path bf16 x is dotted RAW against bf16 hi + lo
// code pairs (v_dot2c_f32_bf16, kRawBF) and fp32 x RAW against fp32 codes
// (v_fma_f32, kRawF32): no conversion of x.  Only the register-decode modes
// (microbenchmarks) still split fp32/bf16 x into hi+lo fp16 halves after a
// per-lane power-of-two pre-scale that puts the chunk's largest |x| in
// [2^14, 2^15) (kScaled; undone exactly on the fp32 dot).
// Exact codes (CL): a runtime codebook (`lut`, the reference ABI's fp32
// quant_map, kernels.cu:1115-1120) is NOT rounded to fp16: each code c is
// stored as c * 2^S = ch + cl, two fp16 values (~2^-23 relative: fp32-class),
// in a 64-bit table entry (hi pair, lo pair) read with one ds_read_b64, and
// the dot takes ch*x + cl*x.  S (power of two, from max|code|) is undone on
// the output.
#include "common.h"

#include <cstdlib>
#include <utility>

namespace qz {

enum {
  kModeFP4 = 0,    // sign/magnitude FP4: 8-entry x12 table in VALU
  kModeLUT16 = 1,  // any 16-entry codebook (NF4): AND-combined v_perm lookups in VALU
  kModeRaw = 2,    // benchmark-only: no decode
  kModeTab = 3     // any 16-entry codebook: byte -> half2 table in LDS, bank-private copies
};

// kModeTab: one LDS entry per packed BYTE value holds the two decoded fp16
// codes (element 2m in the low half, 2m+1 in the high half) -- exactly the
// operand of v_dot2 against the natural-order x pair, so the decode is one
// address computation + one ds_read_b32 per two weights and NO v_perm.  A
// ds_read_b32 serves each 32-lane half of the wave in one LDS cycle when its
// lanes hit distinct banks (MI355X_MICROARCH.md, LDS table); byte values are
// random, so the table is stored 32 times, copy j entirely in bank j
// (dword e*32 + j), and lane l reads copy l % 32: never a bank conflict.
constexpr int kTabCopies = 32;
constexpr int kTabDwords = 256 * kTabCopies;  // 32 KiB
// CL (exact codes): 64-bit entries (hi pair, lo pair), 16 copies -> the same
// 128 B per byte value and 32 KiB, so the byte -> address computation and the
// occupancy are unchanged.  Lane l reads copy l % 16: a ds_read_b64 lane group
// (32 lanes, bank = dword mod 64) then holds two lanes per copy, which collide
// only when their byte values have the same parity (entry stride 32 dwords):
// 1.5-way on average.
constexpr int kTabCopiesCL = 16;

// The byte tables of the two built-in codebooks, computed at compile time and
// stored once in device memory with each entry repeated 4 times (one 16-B
// store per 4 bank copies): a workgroup fills its LDS image with 8 plain
// 16-B copies per thread instead of decoding 256 entries.
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
// bf16 activations (round 2): the codes as bf16 hi + lo pairs -- c = hi + lo to ~2^-16 --
// dotted straight against the raw bf16 x pairs with v_dot2c_f32_bf16 (no x conversion, no
// pre-scale: bf16 has fp32's exponent range).  Entries {hi pair, lo pair}, the CL geometry.
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
__device__ const ByteTable g_byte_tab_nf4 = make_nf4_table();
__device__ const ByteTable g_byte_tab_nf4x = make_nf4_exact_table();
__device__ const ByteTable g_byte_tab_fp4 = make_byte_table(kFP4x12Bits);
__device__ const ByteTable g_byte_tab_nf4_bf = make_bf16_table(kNF4Host);
// fp32 activations (round 2): entries {code[e >> 4], code[e & 15]} as fp32 -- the reference's
// own fp32 quant_map values (kernels.cu:1115-1120) -- multiplied into the raw fp32 x by v_fma_f32
constexpr ByteTable make_f32_table(const float (&c)[16]) {
  ByteTable t{};
  for (int e = 0; e < 256; ++e) {
    const uint32_t a = __builtin_bit_cast(uint32_t, c[e >> 4]), b = __builtin_bit_cast(uint32_t, c[e & 15]);
    t.v[4 * e + 0] = a; t.v[4 * e + 1] = b; t.v[4 * e + 2] = a; t.v[4 * e + 3] = b;
  }
  return t;
}
__device__ const ByteTable g_byte_tab_fp4_bf = make_bf16_table(kFP4x12Host);
__device__ const ByteTable g_byte_tab_nf4_f32 = make_f32_table(kNF4Host);
__device__ const ByteTable g_byte_tab_fp4_f32 = make_f32_table(kFP4x12Host);
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
  const float *lut;  // runtime 16-entry codebook (kModeLUT16) or nullptr
  long long block_base;
  int M, K;
  int bs_log2, bs2_log2;
  float out_scale;
  int tabsel;        // kModeTab: 0 = NF4, 1 = FP4 (x12), 2 = exact NF4 (CL) precomputed byte table;
                     // lut != nullptr builds an exact (CL) table in kernel
  uint32_t tab[8];
  uint32_t tab_lo[8];  // exact codes (CL): fp16 byte planes of the lo parts (the hi parts are tab)
  const void *nw;    // fused pre-norm (NRM): the RMSNorm weight [K], or nullptr
  float eps;         //   and its epsilon
  const void *res;   // residual [M] added after the output rounding (y = round(round(x W^T) + res)), or nullptr
  // prefetch (PF): the first pf_chunks KiB of each of pf_rows rows (stride pf_row_bytes) of the NEXT
  // launch's packed weight, read into the caches (Infinity Cache) once this launch's own loads are out
  const unsigned char *pf;
  uint32_t pf_row_bytes;
  int pf_rows, pf_chunks;
};

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, a), __builtin_bit_cast(h2_t, b), c, false);
}

// Kernel arguments are read ONCE at entry and laundered through an empty asm:
// the compiler then keeps them in SGPRs instead of re-fetching them from the
// kernarg segment at each use (every re-fetch is a serialized scalar-cache miss
// on the critical path of a ~µs kernel).
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

// Diagnostic timeline stamps (dev builds only: scripts/microbench defines
// QZ_STAMPS and instantiates ABL & 512).  The product library compiles none of
// this.  Per wave: s_memrealtime (100 MHz, chip-wide) at fixed points, stored
// once at the end by lane 0 with the wave's XCC / HW ids.
#ifdef QZ_STAMPS
__device__ unsigned long long *g_qz_stamp;
#define QZ_STAMP_DECL unsigned long long qz_st_[6] = {0, 0, 0, 0, 0, 0}
// ABL & 8192 ("light"): only the start (0) and end (4) stamps, flushed as two stores, so the
// instrumentation leaves the kernel's schedule between them untouched (bench.py's in-kernel time)
#define QZ_STAMP(k)                                                                  \
  do {                                                                               \
    if constexpr ((ABL & 512) != 0 && ((ABL & 8192) == 0 || (k) == 0 || (k) == 4)) { \
      __builtin_amdgcn_sched_barrier(0);                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(qz_st_[k])::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                             \
    }                                                                                \
  } while (0)
#define QZ_STAMP_FLUSH(wave_id)                                                      \
  do {                                                                               \
    if constexpr ((ABL & 512) != 0) {                                                \
      uint32_t xcc, hw;                                                              \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));             \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));               \
      qz_st_[5] = ((unsigned long long)xcc << 32) | hw;                              \
      if ((threadIdx.x & 63) == 0) {                                                 \
        if constexpr ((ABL & 8192) != 0) {                                           \
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
#pragma unroll
  for (int i = 0; i < 8; ++i) p.tab[i] = keep_s(in.tab[i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) p.tab_lo[i] = keep_s(in.tab_lo[i]);
  p.nw = keep_sp(in.nw);
  p.eps = keep_s(in.eps);
  p.pf = keep_sp(in.pf);
  p.pf_row_bytes = keep_s(in.pf_row_bytes);
  p.pf_rows = keep_s(in.pf_rows);
  p.pf_chunks = keep_s(in.pf_chunks);
  return p;
}

// FP4: 8 nibbles -> 4 half2 in natural order P[j] = (e_2j, e_2j+1), values x12.
__device__ __forceinline__ void decode_fp4(uint32_t w, uint32_t t0, uint32_t t1, uint32_t (&P)[4]) {
  const uint32_t hh = perm(t1, t0, (w >> 4) & 0x07070707u) | (w & 0x80808080u);
  const uint32_t hl = perm(t1, t0, w & 0x07070707u) | ((w << 4) & 0x80808080u);
  P[0] = perm(hh, hl, 0x000C040Cu);
  P[1] = perm(hh, hl, 0x010C050Cu);
  P[2] = perm(hh, hl, 0x020C060Cu);
  P[3] = perm(hh, hl, 0x030C070Cu);
}

// 16-entry codebook: 8 nibbles -> (e0,e2),(e4,e6),(e1,e3),(e5,e7).
// Each fp16 byte plane is a 16-entry lookup done as two 8-entry v_perm
// lookups AND-ed together: the selector byte is the nibble with its bit 3
// copied to bit 7, so entries 0-7 index the first table directly and
// entries 8-15 give a selector >= 0x88, which v_perm maps to 0xFF; XOR 0x88
// swaps the roles for the second table.  (v_perm, v_bfi and v_dot2c issue at
// half rate on gfx950; this form needs no mask perm and no v_bfi.)
__device__ __forceinline__ void decode_lut16(uint32_t w, const uint32_t (&t)[8], uint32_t (&P)[4]) {
  uint32_t ah = ((w >> 4) & 0x0F0F0F0Fu) | (w & 0x80808080u);   // high nibbles (even elements)
  asm("" : "+v"(ah));  // keep the XOR below a full-rate v_xor (not a re-associated v_bitop3)
  const uint32_t bh = ah ^ 0x88888888u;
  const uint32_t lh = perm(t[1], t[0], ah) & perm(t[3], t[2], bh);
  const uint32_t hh = perm(t[5], t[4], ah) & perm(t[7], t[6], bh);
  uint32_t al = (w & 0x0F0F0F0Fu) | ((w << 4) & 0x80808080u);   // low nibbles (odd elements)
  asm("" : "+v"(al));
  const uint32_t bl = al ^ 0x88888888u;
  const uint32_t ll = perm(t[1], t[0], al) & perm(t[3], t[2], bl);
  const uint32_t hl = perm(t[5], t[4], al) & perm(t[7], t[6], bl);
  P[0] = perm(hh, lh, 0x05010400u);
  P[1] = perm(hh, lh, 0x07030602u);
  P[2] = perm(hl, ll, 0x05010400u);
  P[3] = perm(hl, ll, 0x07030602u);
}

// x slice of one lane for one step: 32 activations, loaded raw (so that the
// loads retire in issue order without forcing early waits) and turned into
// 16 half2 "hi" (+ "lo" for fp32/bf16 activations) in the pair order of MODE
// only at compute time.
template <int MODE, int DT> struct XSlice {
  // fp32 x needs the lo part; a bf16 value (8-bit significand) pre-scaled into fp16's range is
  // exact in the hi part, and whatever it loses below fp16's smallest subnormal its lo part
  // (rtz of a residual < 2^-24) loses too: bf16 lo is identically zero, so it is not formed
  // the byte-table decode takes bf16 x raw against bf16 code pairs (kRawBF) and fp32 x raw
  // against fp32 codes (kRawF32): no conversion at all
  static constexpr bool kRawBF = DT == QZ_DT_BF16 && MODE == kModeTab;
  static constexpr bool kRawF32 = DT == QZ_DT_F32 && MODE == kModeTab;
  static constexpr bool kSplit = DT == QZ_DT_F32 && !kRawF32;
  static constexpr bool kScaled = DT != QZ_DT_F16 && !kRawBF && !kRawF32;
  static constexpr int kWords = DT == QZ_DT_F32 ? 32 : 16;  // raw dwords per lane
  uint32_t raw[kWords];

  __device__ __forceinline__ void load(const void *x, uint32_t e0) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(x) +
                                                     e0 * (DT == QZ_DT_F32 ? 4u : 2u));
#pragma unroll
    for (int i = 0; i < kWords / 4; ++i) {
      const u32x4 v = p[i];
      raw[4 * i] = v.x; raw[4 * i + 1] = v.y; raw[4 * i + 2] = v.z; raw[4 * i + 3] = v.w;
    }
  }

  __device__ __forceinline__ void load_lds(const unsigned char *lds_x, int e0) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(lds_x + e0 * (DT == QZ_DT_F32 ? 4 : 2));
#pragma unroll
    for (int i = 0; i < kWords / 4; ++i) {
      const u32x4 v = p[i];
      raw[4 * i] = v.x; raw[4 * i + 1] = v.y; raw[4 * i + 2] = v.z; raw[4 * i + 3] = v.w;
    }
  }

  // hi/lo half2 operands, pair order of MODE.  fp32/bf16: the chunk is first
  // scaled by 2^se so that its largest |x| lies in [2^14, 2^15) (hi = rtz
  // never saturates, lo never flushes); usc = 2^-se undoes it on the dot.
  __device__ __forceinline__ void prepare(uint32_t (&hi)[16], uint32_t (&lo)[kSplit ? 16 : 1], float &usc) const {
    usc = 1.0f;
    if constexpr (kRawF32) {
      return;  // chunk_dot_tab_f32 reads raw[] itself
    } else if constexpr (kRawBF) {
#pragma unroll
      for (int i = 0; i < 16; ++i) hi[i] = raw[i];
    } else if constexpr (DT == QZ_DT_F16) {
      if constexpr (MODE == kModeFP4 || MODE == kModeTab) {
#pragma unroll
        for (int i = 0; i < 16; ++i) hi[i] = raw[i];
      } else {
#pragma unroll
        for (int d = 0; d < 4; ++d) {  // per 8 elements: (x0,x2),(x4,x6),(x1,x3),(x5,x7)
          hi[4 * d + 0] = perm(raw[4 * d + 1], raw[4 * d + 0], 0x05040100u);
          hi[4 * d + 1] = perm(raw[4 * d + 3], raw[4 * d + 2], 0x05040100u);
          hi[4 * d + 2] = perm(raw[4 * d + 1], raw[4 * d + 0], 0x07060302u);
          hi[4 * d + 3] = perm(raw[4 * d + 3], raw[4 * d + 2], 0x07060302u);
        }
      }
    } else {
      float f[32];
      if constexpr (DT == QZ_DT_F32) {
#pragma unroll
        for (int i = 0; i < 32; ++i) f[i] = __uint_as_float(raw[i]);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          f[2 * i] = __uint_as_float(raw[i] << 16);
          f[2 * i + 1] = __uint_as_float(raw[i] & 0xFFFF0000u);
        }
      }
      // chunk max |x| (v_max3_f32 with abs modifiers; NaN is ignored here and
      // still propagates through the dot), its biased exponent E, se = 141 - E
      float mx = 0.0f;
#pragma unroll
      for (int i = 0; i < 32; i += 2) mx = fmaxf(mx, fmaxf(fabsf(f[i]), fabsf(f[i + 1])));
      const int E = (int)(__float_as_uint(mx) >> 23);
      const int se = min(141 - E, 100);                    // in [-114, 100]: both scales are normal
      const float sc = __uint_as_float((uint32_t)(127 + se) << 23);
      usc = __uint_as_float((uint32_t)(127 - se) << 23);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        int a[4], b[4];
        if constexpr (MODE == kModeFP4 || MODE == kModeTab) {
          a[0] = 0; b[0] = 1; a[1] = 2; b[1] = 3; a[2] = 4; b[2] = 5; a[3] = 6; b[3] = 7;
        } else {
          a[0] = 0; b[0] = 2; a[1] = 4; b[1] = 6; a[2] = 1; b[2] = 3; a[3] = 5; b[3] = 7;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // hi = rtz(f s) (|f s| < 2^15), lo = rtz(f s - hi); f s - hi is exact
          const float fa = f[8 * d + a[j]] * sc, fb = f[8 * d + b[j]] * sc;
          const auto h = __builtin_amdgcn_cvt_pkrtz(fa, fb);
          hi[4 * d + j] = __builtin_bit_cast(uint32_t, h);
          if constexpr (kSplit) {
            const float ra = fa - (float)h.x, rb = fb - (float)h.y;
            lo[4 * d + j] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(ra, rb));
          }
        }
      }
    }
  }
};

// dot of one lane's 16-byte weight chunk (32 codes) with its x slice
template <int MODE, bool SPLIT>
__device__ __forceinline__ float chunk_dot(const u32x4 &wv, const uint32_t (&hi)[16],
                                           const uint32_t (&lo)[SPLIT ? 16 : 1], const uint32_t (&t)[8]) {
  const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t P[4];
    if constexpr (MODE == kModeFP4) {
      decode_fp4(w[d], t[0], t[1], P);
    } else if constexpr (MODE == kModeLUT16) {
      decode_lut16(w[d], t, P);
    } else {
      P[0] = w[d]; P[1] = w[d] ^ 1u; P[2] = w[d] ^ 2u; P[3] = w[d] ^ 3u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j & 1) s1 = dot2(P[j], hi[4 * d + j], s1);
      else s0 = dot2(P[j], hi[4 * d + j], s0);
      if constexpr (SPLIT) {
        if (j & 1) s1 = dot2(P[j], lo[4 * d + j], s1);
        else s0 = dot2(P[j], lo[4 * d + j], s0);
      }
    }
  }
  return s0 + s1;
}

// kModeTab: dot of one lane's 16-byte chunk through the LDS byte table.
// `jb` selects the lane's bank-private copy: 4 * (lane % 32), or for CL
// (64-bit exact-code entries) 8 * (lane % 16).  Both tables use 128 B per
// byte value, so the address of byte m is (byte << 7) | jb either way.
// (ABL: benchmark-only ablations -- 16 replaces the dot products by integer
// adds, 32 replaces the table reads by the addresses themselves.)
template <bool SPLIT, int ABL = 0, bool CL = false, bool WT = false, bool BF = false>
__device__ __forceinline__ float chunk_dot_tab(const u32x4 &wv, const uint32_t (&hi)[16],
                                               const uint32_t (&lo)[SPLIT ? 16 : 1], const uint32_t *s_tab,
                                               uint32_t jb) {
  static_assert(!BF || CL, "bf16 entries use the 64-bit (CL) table geometry");
  const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  uint32_t v[16], vl[CL ? 16 : 1];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    // byte m of w, times the stride of one entry (128 B; WT: 256 B), plus the copy.  WT builds
    // the address with ONE v_perm: byte 0 = the lane's copy offset jb (< 256), byte 1 = byte m
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
      if constexpr ((ABL & 32) != 0) {
        v[4 * d + m] = a[m];
        if constexpr (CL) vl[4 * d + m] = a[m] ^ 1u;
      } else if constexpr (CL) {
        const u32x2 e = *reinterpret_cast<const u32x2 *>(tb + a[m]);
        v[4 * d + m] = e.x;
        vl[4 * d + m] = e.y;
      } else {
        v[4 * d + m] = *reinterpret_cast<const uint32_t *>(tb + a[m]);
      }
    }
  }
  if constexpr ((ABL & 16) != 0) {
    uint32_t u0 = 0, u1 = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i & 1) u1 += v[i] ^ hi[i];
      else u0 += v[i] ^ hi[i];
    }
    return (float)(u0 + u1);
  }
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float &acc = (i & 1) ? s1 : s0;
    if constexpr (BF) {  // bf16 code pairs (hi, lo) against the raw bf16 x pair
      acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, v[i]), __builtin_bit_cast(bf16x2_t, hi[i]),
                                            acc, false);
      acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, vl[i]), __builtin_bit_cast(bf16x2_t, hi[i]),
                                            acc, false);
      continue;
    }
    acc = dot2(v[i], hi[i], acc);
    if constexpr (CL) acc = dot2(vl[i], hi[i], acc);   // code residual x x_hi
    if constexpr (SPLIT) acc = dot2(v[i], lo[i], acc);  // code_hi x x residual
  }
  return s0 + s1;
}

// fp32 x (kRawF32): byte m of the lane's chunk holds elements 2m (high nibble) and 2m + 1;
// its 64-bit entry {code_hi, code_lo} (fp32) goes into two v_fma_f32 with the raw x.  Same
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

// Exact codes by mixed-precision FMA (FM, round 4): the byte table holds the two codes as fp32
// (the kRawF32 table: the reference's fp32 quant_map values, kernels.cu:1115-1120) and each
// goes into one v_fma_mix_f32 with its raw fp16 activation, the half picked by op_sel -- no x
// conversion, no hi/lo code split.  Per packed byte: one ds_read_b64 and two full-rate FMAs
// (the hi + lo table needs two half-rate v_dot2c).  The products are fp32 (an fp16 x an fp32
// code, rounded once), as the reference's fp32 FMA chain (kernels.cu:1169-1210).
// Addresses: AD = 0 builds (byte << 7) | jb with two VALU (the 16-copy, 128-B-entry table);
// AD = 1 is the 256-B-entry table (WT: 32 bank-private copies, no conflicts) addressed by ONE
// v_mov_b32_sdwa that writes the byte into bits 8..15 of a register whose byte 0 holds the
// lane's copy offset jb for the whole kernel (`ad`, initialised once; bytes 2-3 stay zero).
template <int M_> __device__ __forceinline__ void sdwa_byte1(uint32_t &a, uint32_t w) {
  if constexpr (M_ == 0) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(a) : "v"(w));
  else if constexpr (M_ == 1) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(a) : "v"(w));
  else if constexpr (M_ == 2) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a) : "v"(w));
  else asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(a) : "v"(w));
}
template <int AD>
__device__ __forceinline__ float chunk_dot_tab_fm(const u32x4 &wv, const uint32_t (&xr)[16], const uint32_t *s_tab,
                                                  uint32_t jb, uint32_t (&ad)[16]) {
  const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t a[4];
    if constexpr (AD == 1) {
      sdwa_byte1<0>(ad[4 * d + 0], w[d]);
      sdwa_byte1<1>(ad[4 * d + 1], w[d]);
      sdwa_byte1<2>(ad[4 * d + 2], w[d]);
      sdwa_byte1<3>(ad[4 * d + 3], w[d]);
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = ad[4 * d + m];
    } else {
      a[0] = ((w[d] << 7) & 0x7F80u) | jb;
      a[1] = ((w[d] >> 1) & 0x7F80u) | jb;
      a[2] = ((w[d] >> 9) & 0x7F80u) | jb;
      a[3] = ((w[d] >> 17) & 0x7F80u) | jb;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const u32x2 e = *reinterpret_cast<const u32x2 *>(tb + a[m]);
      const uint32_t xv = xr[4 * d + m];   // x[2j] in the low half, x[2j + 1] in the high half
      // written out: left to itself hipcc SLP-packs the scalar FMAs into v_pk_fma_f32 fed by
      // v_cvt_f32_f16 + v_mov copies (twice the VALU)
      asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(s[(2 * m) & 3]) : "v"(xv), "v"(e.x));
      asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(s[(2 * m + 1) & 3]) : "v"(xv), "v"(e.y));
    }
  }
  return (s[0] + s[1]) + (s[2] + s[3]);
}

// Exact codes against fp32 x (XF, round 4): the fp16 x of a step is widened to fp32 once (shared by
// the wave's R rows) and each packed byte's fp32 code pair {code(hi nibble), code(lo nibble)} (the
// kRawF32 table) meets its x pair in full-rate fp32 FMAs: PK = 0 two v_fma_f32, PK = 1 one
// v_pk_fma_f32.  The products are fp32 (exact code x exact x, rounded once), as the reference's fp32
// FMA chain (kernels.cu:1169-1210).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
template <int PK>
__device__ __forceinline__ float chunk_dot_tab_xf(const u32x4 &wv, const f32x2_t (&xf)[16], const uint32_t *s_tab,
                                                  uint32_t jb) {
  const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  f32x2_t s2[2] = {f32x2_t{0.0f, 0.0f}, f32x2_t{0.0f, 0.0f}};
  float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t a[4] = {((w[d] << 7) & 0x7F80u) | jb, ((w[d] >> 1) & 0x7F80u) | jb,
                           ((w[d] >> 9) & 0x7F80u) | jb, ((w[d] >> 17) & 0x7F80u) | jb};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x2_t e = *reinterpret_cast<const f32x2_t *>(tb + a[m]);
      if constexpr (PK) {
        asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(s2[m & 1]) : "v"(e), "v"(xf[4 * d + m]));
      } else {
        // written out: hipcc would SLP-pack the pair into v_pk_fma_f32 (+ register copies), which
        // issues no faster than the two full-rate FMAs it replaces
        const float ex = e.x, ey = e.y, xx = xf[4 * d + m].x, xy = xf[4 * d + m].y;
        asm("v_fmac_f32 %0, %1, %2" : "+v"(s[(2 * m) & 3]) : "v"(ex), "v"(xx));
        asm("v_fmac_f32 %0, %1, %2" : "+v"(s[(2 * m + 1) & 3]) : "v"(ey), "v"(xy));
      }
    }
  }
  if constexpr (PK) return (s2[0].x + s2[1].x) + (s2[0].y + s2[1].y);
  return (s[0] + s[1]) + (s[2] + s[3]);
}

// compile-time loop: f(std::integral_constant<int, 0>{}) .. f(<N - 1>)
template <typename F, int... Ns>
__device__ __forceinline__ void gv_static_for_impl(F &&f, std::integer_sequence<int, Ns...>) {
  (f(std::integral_constant<int, Ns>{}), ...);
}
template <int N, typename F> __device__ __forceinline__ void gv_static_for(F &&f) {
  gv_static_for_impl(f, std::make_integer_sequence<int, N>{});
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

// Builds the kModeTab byte table from the 16-entry fp16 byte planes t[8]
// (every thread of the workgroup takes part; the caller synchronises).
template <int NT, int PIECES = kTabCopies / 4>
__device__ __forceinline__ void build_byte_table(uint32_t *s_tab, const uint32_t (&t)[8]) {
  for (int e = threadIdx.x; e < 256; e += NT) {
    uint32_t P[4];
    decode_lut16((uint32_t)e, t, P);  // byte 0 = e: P[0].lo = code[e >> 4], P[2].lo = code[e & 15]
    const uint32_t v = (P[0] & 0xFFFFu) | (P[2] << 16);
    const u32x4 q = {v, v, v, v};
    // 128 B per entry; rotate the 16-B pieces by lane so that each 8-lane
    // store group covers all 32 banks
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = (i + (int)threadIdx.x) & (PIECES - 1);
      reinterpret_cast<u32x4 *>(s_tab)[e * PIECES + piece] = q;
    }
  }
}

// Fills the LDS byte table from a precomputed device table entry `v` (entry
// e = threadIdx.x, already repeated 4 times: one 16-B store covers 4 bank
// copies).  The 8 stores of a thread are rotated by its lane so that each
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
// e = {hi pair, lo pair} of (code[e >> 4], code[e & 15]) * 2^S, 16 copies.
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
// (code[e >> 4], code[e & 15]) as bf16 hi + lo (c = hi + lo to ~2^-16), 16 copies.
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

// The fp32 byte table from a runtime codebook: entry e = {code[e >> 4], code[e & 15]}, 16 copies.
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
// (no exec-masked regions, no lazily re-read kernel arguments).
template <int MODE, bool DQ, int DT, int R, bool XL, int ABL = 0, bool FS = false> struct StepLoads {
  u32x4 wv[R];
  uint32_t q[R];    // DQ: 8-bit scale code
  float a[R];       // DQ: absmax2 entry; else: fp32 absmax
  XSlice<MODE, DT> xs;
  int xb;  // first activation index of this lane's chunk
  bool on;

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
    if constexpr (!XL && !(ABL & 2)) xs.load(p.x, 2u * boff);
    if constexpr (ABL & 2) {
#pragma unroll
      for (int i = 0; i < XSlice<MODE, DT>::kWords; ++i) xs.raw[i] = 0x3C003C00u ^ boff;
    }
    // per row: weights then that row's scale, so row r can be consumed while
    // rows > r are still in flight (vmcnt retires in issue order)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t row = (uint32_t)min(row0 + r, p.M - 1);  // wave-uniform
      const unsigned char *rowp = p.B + (size_t)row * (uint32_t)row_bytes;
      wv[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rowp + boff));
      const uint32_t b = (uint32_t)p.block_base + ((row * (uint32_t)p.K + 2u * boff) >> p.bs_log2);
      if constexpr (ABL & 1) {
        q[r] = b & 255u;
        a[r] = 1.0f;
      } else if constexpr (DQ) {
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
    // ABL & 2048 (microbenchmark only): every wave reads its own one of 64 copies of x
    const void *xp = (ABL & 2048) ? (const void *)((const char *)p.x + (size_t)((row0 / R) & 63) * p.K * 2) : p.x;
    if constexpr (!XL && !(ABL & 2)) xs.load(xp, 2u * boff);
    const uint32_t lb = (2u * boff) >> p.bs_log2;                 // lane's block within the row
    const uint32_t sb = ((uint32_t)s << 11) >> p.bs_log2;         // step's first block within the row
    const uint32_t bpr = (uint32_t)p.K >> p.bs_log2;              // blocks per row
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t row = (uint32_t)min(row0 + r, p.M - 1);  // wave-uniform
      const unsigned char *rowp = p.B + (size_t)row * (uint32_t)row_bytes;
      wv[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rowp + boff));
      const uint32_t rb = (uint32_t)p.block_base + row * bpr;    // wave-uniform
      if constexpr (ABL & 1) {
        q[r] = lb & 255u;
        a[r] = 1.0f;
      } else if constexpr (DQ) {
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

template <int MODE, bool DQ, int DT, int R, int WK, int NW = 4, bool XL = false, int ABL = 0, bool FS = false,
          bool CL = false, bool WT = false, bool NRM = false, bool PAIR = false, int FMV = 0, int OPT = 0,
          bool PF = false, bool PS = false, int NSW = 0, bool GPS = false>
__device__ __forceinline__ void gemv_body(const GemvParams &p_in, const int block,
                                          const GemvParams *pair = nullptr, const GemvGroup *grp = nullptr) {
  // NRM: x is RMSNorm'd in the prologue (bit-identical to qz_rmsnorm) into an LDS image
  static_assert(!NRM || (NW == 4 && FS && !XL && MODE == kModeTab && (DT == QZ_DT_F16 || DT == QZ_DT_BF16)),
                "fused pre-norm: 4 waves, full steps, 16-bit activations");
  // PAIR (LlamaMLP's gate/up): waves 0-1 take R-row groups of pair[0] (gate_proj), waves 2-3 the
  // same rows of pair[1] (up_proj); the epilogue stores act_fn(gate) * up (k_silu_mul's
  // arithmetic) for those rows into pair[0].y, the input of down_proj
  static_assert(!PAIR || (NW == 4 && WK == 1 && MODE == kModeTab && DT != QZ_DT_F32), "pair: 4 waves, WK = 1");
  // WT ("wide table"): 256 B per byte value -- 64 copies of a 4-B entry, or 32 copies of an
  // 8-B exact entry, 64 KiB -- so the lookup address is one v_perm and every copy is bank-private
  constexpr int kPieces = WT ? 16 : kTabCopies / 4;
  static_assert(!CL || MODE == kModeTab, "exact codes need the byte-table decode");
  QZ_STAMP_DECL;
  QZ_STAMP(0);
  const GemvParams p = load_params(p_in);
  constexpr int RG = NW / WK;
  constexpr bool kSplit = XSlice<MODE, DT>::kSplit;   // fp32 x: hi + lo parts
  // bf16 x (byte-table decode): bf16 code pairs hi + lo in 64-bit entries, the CL geometry
  constexpr bool kBF = XSlice<MODE, DT>::kRawBF;
  constexpr bool kF32 = XSlice<MODE, DT>::kRawF32;    // fp32 x: fp32 code table, v_fma_f32
  constexpr bool kWide = CL || kBF || kF32;
  // FMV (exact codes, fp16 x): 0 = hi + lo fp16 code pairs by v_dot2c; 1 = fp32 codes by
  // v_fma_mix_f32 (chunk_dot_tab_fm), two-VALU addresses; 2 = the same on the 256-B-entry (WT)
  // table with one-SDWA addresses
  constexpr bool kFM = CL && DT == QZ_DT_F16 && (FMV == 1 || FMV == 2);
  // FMV 3 / 4: fp32 codes against x widened to fp32 once per step, v_fma_f32 / v_pk_fma_f32
  // (chunk_dot_tab_xf); the 128-B-entry kRawF32 table, two-VALU addresses
  constexpr bool kXF = CL && DT == QZ_DT_F16 && (FMV == 3 || FMV == 4);
  static_assert(FMV != 2 || WT, "SDWA addresses index the 256-B-entry table");
  // OPT (round 4): bit 0 = issue the wave's second K-step before the prologue barrier (both steps
  // of a K = 4096 row in flight from the start); bit 1 = build the fp16 byte-table entry from the
  // SGPR byte planes (tab / tab_lo) instead of loading it (no global load gates the barrier)
  constexpr bool kEarly = (OPT & 1) != 0;
  constexpr bool kSTab = (OPT & 2) != 0 && MODE == kModeTab && !kBF && !kF32 && !kFM;
  // bit 2: the scale codes / absmax2 of a step become visible only inside consume() (an empty asm),
  // so hipcc cannot hoist their use -- and the vmcnt wait it needs -- above the next step's issue
  constexpr bool kLaunder = (OPT & 4) != 0;
  // bit 3: the wave owns exactly two K-steps (host-checked): straight-line code -- issue, barrier,
  // issue step 2, decode, decode -- with no loop whose shared dominator would take the waits of
  // step 1's scale codes above step 2's issue (hipcc did: the product's K = 4096 waves waited for
  // ALL of step 1 before issuing step 2)
  constexpr bool kTwo = (OPT & 8) != 0;
  // PS (round 4, pair launches): persistent workgroups -- the grid is smaller than the row blocks and
  // each workgroup takes blocks blockIdx.x, + gridDim.x, ..., so its prologue (byte table, code2,
  // the fused RMSNorm of x into LDS) is paid once for all of them; the next block's first step is
  // issued before the current block's epilogue
  static_assert(!PS || (PAIR && kTwo && !kEarly && !PF), "persistent form: two-step pair launches");
  // GPS (round 4, grouped launches with the fused norm): the same persistence over the blocks of all
  // segments; a workgroup that crosses into another segment re-stages that segment's code2 table
  static_assert(!GPS || (!PAIR && !PS && kTwo && !kEarly && !PF && WK == 1 && NW == 4), "grouped persistent form");
  // bits 4 / 5 (round 4): a ring of 3 / 4 step buffers for waves that own exactly NSW K-steps
  // (host-checked; K = 14336: Llama-3-8B down_proj, 7 steps), straight-line: step i + D - 1 is
  // issued before step i is decoded, so D - 1 steps stay in flight instead of one
  constexpr int kRing = (OPT & 32) ? 4 : (OPT & 16) ? 3 : 0;
  static_assert(kRing == 0 || (NSW >= 2 && !kEarly && !kTwo && !PS && !PF), "ring: a fixed step count");
  constexpr bool kScaled = XSlice<MODE, DT>::kScaled; // fp32/bf16 x: per-chunk power-of-two pre-scale
  constexpr int XB = DT == QZ_DT_F32 ? 4 : 2;
  __shared__ float s_code2[PAIR ? 2 : 1][DQ ? 256 : 1];   // PAIR: each weight's own double-quant code
  __shared__ float s_part[NW][R];
  __shared__ float s_part2[PS ? 2 : 1][NW][R];   // PS: by block parity (no barrier after the reads)
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[MODE == kModeTab ? (WT ? 2 : 1) * kTabDwords : 1];
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

  // ABL & 32768 (microbenchmark, timing only: WRONG outputs): a prologue without memory -- the
  // byte table from the SGPR planes, code2 / offset replaced by constants -- to price the
  // prologue's global loads (which queue behind the CU's HBM requests)
  constexpr bool kNoPro = (ABL & 32768) != 0;
  // 1. the double-quant code table load goes out first (it gates the barrier)
  float c2 = 0.0f, c2b = 0.0f, offset = 0.0f;
  if constexpr (DQ && !kNoPro) {
    if constexpr (PAIR) {
      c2 = keep_sp(pair[0].sc.code2)[threadIdx.x];
      c2b = keep_sp(pair[1].sc.code2)[threadIdx.x];
    } else if (NW * 64 == 256 || threadIdx.x < 256) {
      c2 = p.sc.code2[threadIdx.x & 255];
    }
    offset = *p.sc.offset;
  } else if constexpr (DQ) {
    c2 = (float)(threadIdx.x & 255) * (1.0f / 256.0f);
  }
  // 1b. the precomputed byte-table entry of this thread (issued before the
  // weights, so waiting for it does not wait for the first HBM step)
  u32x4 tab_entry = {0u, 0u, 0u, 0u};
  if constexpr (kSTab) {
    if (!p.lut && threadIdx.x < 256) {
      uint32_t P[4], tp[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) tp[i] = p.tab[i];
      decode_lut16((uint32_t)threadIdx.x, tp, P);
      const uint32_t h = (P[0] & 0xFFFFu) | (P[2] << 16);
      if constexpr (CL) {
#pragma unroll
        for (int i = 0; i < 8; ++i) tp[i] = p.tab_lo[i];
        decode_lut16((uint32_t)threadIdx.x, tp, P);
        const uint32_t l = (P[0] & 0xFFFFu) | (P[2] << 16);
        tab_entry = u32x4{h, l, h, l};
      } else {
        tab_entry = u32x4{h, h, h, h};
      }
    }
  } else if constexpr (kNoPro && MODE == kModeTab) {
    uint32_t P[4], tp[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) tp[i] = p.tab[i];
    decode_lut16((uint32_t)threadIdx.x, tp, P);
    const uint32_t h = (P[0] & 0xFFFFu) | (P[2] << 16);
    tab_entry = u32x4{h, h, h, h};
  } else if constexpr (MODE == kModeTab && (ABL & 64) == 0) {
    static_assert(NW * 64 >= 256, "one byte-table entry per thread");
    if (!p.lut && threadIdx.x < 256) {
      const ByteTable *bt = (kF32 || kFM || kXF) ? (p.tabsel ? &g_byte_tab_fp4_f32 : &g_byte_tab_nf4_f32)
                            : kBF ? (p.tabsel ? &g_byte_tab_fp4_bf : &g_byte_tab_nf4_bf)
                                  : (CL ? &g_byte_tab_nf4x : (p.tabsel ? &g_byte_tab_fp4 : &g_byte_tab_nf4));
      tab_entry = reinterpret_cast<const u32x4 *>(bt->v)[threadIdx.x];
    }
  }
  // 1c. XL: this thread's share of x (<= kXLChunks 16-B chunks), also ahead of the weights
  constexpr int kXLChunks = XL ? 8 : 1;
  u32x4 xr[kXLChunks];
  const int x_nchunk = (p.K * XB) >> 4;
  if constexpr (XL) {
#pragma unroll
    for (int i = 0; i < kXLChunks; ++i) {
      const int c = (int)threadIdx.x + i * NW * 64;
      if (c < x_nchunk) xr[i] = reinterpret_cast<const u32x4 *>(p.x)[c];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // 1d. NRM: this thread's chunks of x and of the norm weight (L2-resident), ahead of the
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
  StepLoads<MODE, DQ, DT, R, XL || NRM, ABL, FS> cur, other;
  int s = wk;
  cur.issue(p, row0, s < nsteps ? s : 0, lane, row_bytes);
  const bool have = s < nsteps;
  const int n_my = have ? (nsteps - wk + WK - 1) / WK : 0;  // this wave's steps: s = wk, wk + WK, ...
  if constexpr (kEarly) {
    // unconditional (a clamped step when there is no second one): a conditional issue makes hipcc's
    // waitcnt before the table stores count only the loads common to both paths, i.e. wait for step 0
    other.issue(p, row0, n_my >= 2 ? s + WK : (s < nsteps ? s : 0), lane, row_bytes);
  }
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
  if constexpr (XL) {  // x -> LDS (the launcher guarantees K * XB <= kXLChunks * 16 * NW * 64)
#pragma unroll
    for (int i = 0; i < kXLChunks; ++i) {
      const int c = (int)threadIdx.x + i * NW * 64;
      if (c < x_nchunk) reinterpret_cast<u32x4 *>(s_x)[c] = xr[i];
    }
  }
  uint32_t t[8];
  if (MODE != kModeTab && p.lut) {  // register decodes (microbenchmarks): runtime codebook -> fp16 byte planes
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t h = __half_as_ushort(__float2half_rn(p.lut[i]));
      t[i >> 2] |= (h & 0xFFu) << (8 * (i & 3));
      t[4 + (i >> 2)] |= (h >> 8) << (8 * (i & 3));
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = p.tab[i];
  }
  // output scale: the codebook's (FP4 x12: 1/12; exact NF4: 2^-14), or for a
  // runtime codebook (always exact codes) 2^-S of its in-kernel split
  float out_scale = p.out_scale;
  if constexpr (MODE == kModeTab && (ABL & 64) == 0) {
    if constexpr (kF32 || kFM || kXF) {
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
      } else if (threadIdx.x < 256) {
        store_byte_table_entry<kPieces>(s_tab, tab_entry);
      }
    } else {
      if (p.lut) build_byte_table<NW * 64, kPieces>(s_tab, t);
      else if (threadIdx.x < 256) store_byte_table_entry<kPieces>(s_tab, tab_entry);
    }
  }
  if constexpr ((DQ || XL || MODE == kModeTab) && (ABL & 128) == 0) __syncthreads();
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
  uint32_t ad[16];   // FMV = 2: per-byte address registers, byte 0 = jb for the whole kernel
#pragma unroll
  for (int i = 0; i < 16; ++i) ad[i] = jb;

  // Steady state: the next step's loads are issued UNCONDITIONALLY before the
  // current step is consumed, and the last step is peeled after the loop.  (A
  // conditional prefetch makes hipcc's waitcnt pass pick the count valid on
  // both paths -- vmcnt(0) -- which waits for the prefetch itself and
  // serialises HBM traffic with the decode.)
  typedef StepLoads<MODE, DQ, DT, R, XL || NRM, ABL, FS> Loads;
  auto consume = [&](const Loads &c) {
    if constexpr (kLaunder) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        asm volatile("" : "+v"(const_cast<Loads &>(c).q[r]));
        asm volatile("" : "+v"(const_cast<Loads &>(c).a[r]));
      }
    }
    if constexpr (XL) const_cast<Loads &>(c).xs.load_lds(s_x, c.xb);
    if constexpr (NRM) {
      auto &raw = const_cast<Loads &>(c).xs.raw;
      const uint32_t c0 = (uint32_t)c.xb >> 3;  // the lane's first chunk
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(s_x + norm_x_off(c0 + (uint32_t)i));
        raw[4 * i] = v.x; raw[4 * i + 1] = v.y; raw[4 * i + 2] = v.z; raw[4 * i + 3] = v.w;
      }
    }
    uint32_t hi[16], lo[kSplit ? 16 : 1];
    float usc;
    c.xs.prepare(hi, lo, usc);
    f32x2_t xf[kXF ? 16 : 1];
    if constexpr (kXF) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const auto h = __builtin_bit_cast(h2_t, hi[i]);
        xf[i] = f32x2_t{(float)h.x, (float)h.y};
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float am;
      if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[cb][c.q[r]], c.a[r]), offset);
      else am = c.a[r];
      am = c.on ? am : 0.0f;
      if constexpr (kScaled) am *= usc;  // exact: a power of two (the lane's x pre-scale)
      float d;
      if constexpr (kF32) d = chunk_dot_tab_f32(c.wv[r], c.xs.raw, s_tab, jb);
      else if constexpr (kFM) d = chunk_dot_tab_fm<FMV == 2 ? 1 : 0>(c.wv[r], hi, s_tab, jb, ad);
      else if constexpr (kXF) d = chunk_dot_tab_xf<FMV == 4 ? 1 : 0>(c.wv[r], xf, s_tab, jb);
      else if constexpr (MODE == kModeTab) d = chunk_dot_tab<kSplit, ABL, kWide, WT, kBF>(c.wv[r], hi, lo, s_tab, jb);
      else d = chunk_dot<MODE, kSplit>(c.wv[r], hi, lo, t);
      acc[r] = fmaf(d, am, acc[r]);
    }
  };
  // Ping-pong over two named load sets, whole pairs per iteration.  No path
  // may consume `other` where another path consumes `cur`: hipcc would merge
  // the two tails into one block fed by register COPIES, and copying a
  // register whose load is in flight forces vmcnt(0) -- the prefetch is then
  // waited for before the current step is decoded.  Every consume(cur) below
  // reads the same registers on every path, so no copies are needed.
  // PF: this wave's share of the next launch's first K-steps, issued after its own last loads (so no
  // wait for its own data waits for them); the values are discarded after the stores
  constexpr int kPfMax = PF ? 4 : 1;
  uint32_t pfv[kPfMax];
  auto prefetch = [&]() {
    if constexpr (PF) {
      const int W = (int)gridDim.x * NW, gw = block * NW + wave;
      const int items = p.pf_rows * p.pf_chunks;
#pragma unroll
      for (int i = 0; i < kPfMax; ++i) {
        const int it = min(gw + i * W, items - 1);
        const int r = it / p.pf_chunks, ck = it - r * p.pf_chunks;
        const uint32_t off = (uint32_t)r * p.pf_row_bytes + ((uint32_t)ck << 10) + ((uint32_t)lane << 4);
        pfv[i] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p.pf + off));
      }
    }
  };
  if constexpr (GPS) {
    auto seg_of = [&](int b) {
      int sg = 0;
#pragma unroll
      for (int i = 1; i < kMaxSeg; ++i)
        if (i < grp->nseg && b >= grp->start[i]) sg = i;
      return __builtin_amdgcn_readfirstlane(sg);
    };
    auto store_rows = [&](const GemvParams &q, int r0) {
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
      if (lane == kWave - 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int row = r0 + r;
          if (row < q.M) {
            float o = v[r] * out_scale;
            if (q.bias) o += load_f32<DT>(q.bias, row);
            o = add_res<DT>(o, q.res, row);
            store_f32<DT>(q.y, row, o);
          }
        }
      }
    };
    const int total = grp->total;
    int blk = (int)blockIdx.x;
    int sg = seg_of(blk);
    GemvParams q = p;
    for (int it = 0;; ++it) {
      other.issue(q, row0, s + WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      consume(cur);
      consume(other);
      const int nb = blk + (int)gridDim.x;   // workgroup-uniform
      if (nb >= total) {
        store_rows(q, row0);
        break;
      }
      const int ns = seg_of(nb);
      const GemvParams qn = load_params(grp->seg[ns]);
      const int nrow0 = ((nb - grp->start[ns]) * RG + rg) * R;
      cur.issue(qn, nrow0, s, lane, row_bytes);   // the next block's first step, ahead of this epilogue
      __builtin_amdgcn_sched_barrier(0);
      store_rows(q, row0);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.0f;
      if (ns != sg) {   // another segment: its own code2 table and offset
        if constexpr (DQ) {
          __syncthreads();   // every wave has decoded the old segment's blocks
          s_code2[0][threadIdx.x & 255] = qn.sc.code2[threadIdx.x & 255];
          offset = *qn.sc.offset;
          __syncthreads();
        }
        sg = ns;
      }
      q = qn;
      blk = nb;
      row0 = nrow0;
    }
    return;
  } else if constexpr (kRing > 0) {
    Loads third, fourth;
    auto sel = [&](auto K) -> Loads & {
      constexpr int k = decltype(K)::value;
      if constexpr (k == 0) return cur;
      else if constexpr (k == 1) return other;
      else if constexpr (k == 2) return third;
      else return fourth;
    };
    gv_static_for<NSW>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i == 0) {
        gv_static_for<kRing - 1>([&](auto J) {
          constexpr int j = decltype(J)::value + 1;
          if constexpr (j < NSW) sel(std::integral_constant<int, j % kRing>{}).issue(p, row0, s + j * WK, lane, row_bytes);
        });
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (i + kRing - 1 < NSW) {
        constexpr int j = i + kRing - 1;
        sel(std::integral_constant<int, j % kRing>{}).issue(p, row0, s + j * WK, lane, row_bytes);
        __builtin_amdgcn_sched_barrier(0);
      }
      consume(sel(std::integral_constant<int, i % kRing>{}));
    });
  } else if constexpr (PS) {
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
      other.issue(p, row0, s + WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      consume(cur);
      consume(other);
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
  } else if constexpr (kTwo && !kEarly) {
    other.issue(p, row0, s + WK, lane, row_bytes);
    prefetch();
    __builtin_amdgcn_sched_barrier(0);
    consume(cur);
    QZ_STAMP(2);
    consume(other);
  } else if (kEarly && have) {
    // `other` already holds step s + WK (n >= 2); at the loop top cur = step j, other = j + 1
    const int n = n_my;
    int j = 0;
    for (; j + 3 < n; j += 2) {
      consume(cur);
      cur.issue(p, row0, s + 2 * WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      consume(other);
      other.issue(p, row0, s + 3 * WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      s += 2 * WK;
    }
    if (n - j == 3) {
      consume(cur);
      cur.issue(p, row0, s + 2 * WK, lane, row_bytes);
      __builtin_amdgcn_sched_barrier(0);
      consume(other);
      consume(cur);
    } else if (n - j == 2) {
      consume(cur);
      QZ_STAMP(2);
      consume(other);
    } else {
      consume(cur);
    }
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
      prefetch();
      __builtin_amdgcn_sched_barrier(0);
      consume(cur);
      QZ_STAMP(2);
      consume(other);
    } else {
      prefetch();
      consume(cur);
    }
  }

  if constexpr ((ABL & 4) != 0) {  // benchmark-only: no reduction, no store
#pragma unroll
    for (int r = 0; r < R; ++r) asm volatile("" ::"v"(acc[r]));
    return;
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
    for (int r = 0; r < R; ++r) v[r] = (ABL & 8) ? acc[r] : wave_sum_last(acc[r]);
    if (lane == kWave - 1) {
      // 16-bit outputs of a row pair inside M go out as one dword (row0 is even for even R)
      constexpr bool kPack = DT != QZ_DT_F32 && R % 2 == 0 && (ABL & (1024 | 4096)) == 0;  // 4096: A/B knob
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
            if constexpr ((ABL & 1024) != 0 && DT == QZ_DT_F16)  // microbenchmark: non-temporal y store
              __builtin_nontemporal_store((uint16_t)f32_to_f16_bits(o), reinterpret_cast<uint16_t *>(p.y) + row);
            else
              store_f32<DT>(p.y, row, o);
          }
        }
      }
    }
    QZ_STAMP(4);
    QZ_STAMP_FLUSH(block * NW + wave);
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < kPfMax; ++i) asm volatile("" ::"v"(pfv[i]));
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float v = (ABL & 8) ? acc[r] : wave_sum_last(acc[r]);
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

template <int MODE, bool DQ, int DT, int R, int WK, int NW = 4, bool XL = false, int ABL = 0, bool FS = false,
          bool CL = false, bool WT = false, int FMV = 0, int OPT = 0, bool PF = false, int NSW = 0>
__global__ __launch_bounds__(NW * 64) void k_gemv_4bit(GemvParams p) {
  gemv_body<MODE, DQ, DT, R, WK, NW, XL, ABL, FS, CL, WT, false, false, FMV, OPT, PF, false, NSW>(p, blockIdx.x);
}

// Streaming ("persistent") form for rows of exactly NS K-steps (K = 2048 * NS, full-step
// loads, fp16 x): a grid of at most the resident workgroups, each wave walks the row groups
// u = gw, gw + W, gw + 2W, ... (gw = its global wave id, W = waves in the grid), R rows per
// group.  The LDS byte table is filled once per workgroup, the wave's x slices of every step
// stay in registers for all its row groups (x is loaded once per wave, not once per row group),
// and the loads of group u + W are issued before group u is decoded, so the HBM stream of a
// wave never stops between its row groups: only its last group has a serial decode tail.
// Set A always holds step 0 of a group, set B step 1 (NS = 2).
template <bool DQ, int R, bool CL, int ABL = 0>
__device__ __forceinline__ void gemv_stream2_body(const GemvParams &p_in, int nunits) {
  constexpr int NS = 2;
  static_assert(NS == 2, "two named load sets, one per K-step");
  typedef StepLoads<kModeTab, DQ, QZ_DT_F16, R, true, ABL, true> Loads;   // XL = true: no x loads
  const GemvParams p = load_params(p_in);
  __shared__ float s_code2[DQ ? 256 : 1];
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabDwords];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int W = (int)gridDim.x * 4;
  const int gw = (int)blockIdx.x * 4 + wave;
  const int row_bytes = p.K >> 1;
  // 1. the code table and this thread's byte-table entry go out first
  float c2 = 0.0f, offset = 0.0f;
  if constexpr (DQ) {
    c2 = p.sc.code2[threadIdx.x & 255];
    offset = *p.sc.offset;
  }
  const ByteTable *bt = CL ? &g_byte_tab_nf4x : (p.tabsel ? &g_byte_tab_fp4 : &g_byte_tab_nf4);
  const u32x4 tab_entry = reinterpret_cast<const u32x4 *>(bt->v)[threadIdx.x];
  // 2. the wave's first row group (both steps), then x (64 B per lane per step)
  Loads A, B;
  const int u0 = gw < nunits ? gw : nunits - 1;
  A.issue(p, u0 * R, 0, lane, row_bytes);
  B.issue(p, u0 * R, 1, lane, row_bytes);
  XSlice<kModeTab, QZ_DT_F16> x0, x1;
  x0.load(p.x, 2u * ((uint32_t)lane << 4));
  x1.load(p.x, 2u * ((1u << 10) + ((uint32_t)lane << 4)));
  if constexpr (DQ) s_code2[threadIdx.x & 255] = c2;
  store_byte_table_entry(s_tab, tab_entry);
  __syncthreads();
  const uint32_t jb = CL ? (uint32_t)(lane & (kTabCopiesCL - 1)) << 3 : (uint32_t)(lane & 31) << 2;
  float acc[R];
  auto consume = [&](const Loads &c, const XSlice<kModeTab, QZ_DT_F16> &xs) {
    uint32_t lo[1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float am;
      if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[c.q[r]], c.a[r]), offset);
      else am = c.a[r];
      const float d = chunk_dot_tab<false, ABL, CL>(c.wv[r], xs.raw, lo, s_tab, jb);
      acc[r] = fmaf(d, am, acc[r]);
    }
  };
  auto finish = [&](int row0) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = wave_sum_last(acc[r]);
    if (lane == kWave - 1) {
      if constexpr (R % 2 == 0) {
        if (row0 + R <= p.M && (reinterpret_cast<uintptr_t>(p.y) & 3u) == 0) {
#pragma unroll
          for (int r = 0; r < R; r += 2) {
            float o0 = acc[r] * p.out_scale, o1 = acc[r + 1] * p.out_scale;
            if (p.bias) {
              o0 += load_f32<QZ_DT_F16>(p.bias, row0 + r);
              o1 += load_f32<QZ_DT_F16>(p.bias, row0 + r + 1);
            }
            reinterpret_cast<uint32_t *>(p.y)[(row0 + r) >> 1] = pack16<QZ_DT_F16>(o0, o1);
          }
          return;
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (row0 + r < p.M) {
          float o = acc[r] * p.out_scale;
          if (p.bias) o += load_f32<QZ_DT_F16>(p.bias, row0 + r);
          store_f32<QZ_DT_F16>(p.y, row0 + r, o);
        }
      }
    }
  };
  if (gw >= nunits) return;
  const int n = (nunits - gw + W - 1) / W;   // this wave's row groups
  int u = gw;
  for (int i = 0; i + 1 < n; ++i) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    consume(A, x0);
    A.issue(p, (u + W) * R, 0, lane, row_bytes);
    __builtin_amdgcn_sched_barrier(0);
    consume(B, x1);
    finish(u * R);
    B.issue(p, (u + W) * R, 1, lane, row_bytes);
    __builtin_amdgcn_sched_barrier(0);
    u += W;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  consume(A, x0);
  consume(B, x1);
  finish(u * R);
}

template <bool DQ, int R, bool CL, int ABL = 0>
__global__ __launch_bounds__(256) void k_gemv_4bit_stream2(GemvParams p, int nunits) {
  gemv_stream2_body<DQ, R, CL, ABL>(p, nunits);
}

// ---------------------------------------------------------------------------
// MFMA-product decode GEMV (round 4, experimental: k_gemv_4bit_mf).  The byte table's
// entries ARE v_mfma_f32_16x16x32_f16 operand fragments: a lane's 16 packed bytes decode
// through the table into 32 codes = four 8-code fragments with no VALU after the LDS read,
// so the matrix pipe takes the products and the VALU keeps only the table addresses.
//  * a wave owns a 16-row tile: lane l reads row (l & 15), 16-B chunk g = l >> 4 of each 64-B
//    row segment; one load instruction covers 16 rows x 128 elements (1 KiB);
//  * the codes are the B operand (lane l supplies B[k = 8 g + jj][n = l & 15]: weight row n,
//    codes 8j..8j+7 of chunk g for MFMA j) and x is a "diagonal" A operand: A[m][8 g + jj] =
//    x of chunk g if m == g, else 0 -- the lanes with (l & 15) == (l >> 4) load x, the others
//    load zeros (a zero buffer, so no select and no exec mask);
//  * so C[m = g][n = row] is chunk g's unscaled dot of that row, which the 16x16 C layout puts
//    in lane `row` (0..15), register g: each of lanes 0..15 scales its row's four chunks by
//    their blocks' absmax and keeps ONE running sum -- no cross-lane reduction;
//  * exact codes add the lo fragments into the same C (hi + lo = the fp32 code to ~2^-23);
//  * NWK waves split K; the per-row partials meet in LDS.
// ---------------------------------------------------------------------------
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));
__device__ const uint32_t g_mf_zeros[512] = {};   // the inactive lanes' A fragments (2 KiB of zeros)

template <bool CL, bool WT, int NWK, int NL>
__global__ __launch_bounds__(NWK * 64) void k_gemv_4bit_mf(GemvParams p_in) {
  const GemvParams p = load_params(p_in);
  constexpr int kPieces = WT ? 16 : kTabCopies / 4;
  static_assert(NL % 2 == 0 && NL <= 8, "2 NL qabsmax bytes per row come as whole dwords");
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[(WT ? 2 : 1) * kTabDwords];
  __shared__ float s_code2[256];
  __shared__ float s_part[NWK][16];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int row0 = blockIdx.x * 16;
  const int rl = lane & 15, g = lane >> 4;           // this lane's row in the tile, its 16-B chunk
  const uint32_t row_bytes = (uint32_t)p.K >> 1;
  // 1. code2 and the table entry (the barrier waits for them), then every weight load
  float c2 = 0.0f;
  if (threadIdx.x < 256) c2 = p.sc.code2[threadIdx.x];
  const float offset = *p.sc.offset;
  u32x4 tab_entry = {0u, 0u, 0u, 0u};
  if (threadIdx.x < 256) tab_entry = reinterpret_cast<const u32x4 *>((CL ? &g_byte_tab_nf4x : &g_byte_tab_nf4)->v)[threadIdx.x];
  const uint32_t kb0 = (uint32_t)(wave * NL) * 64u;  // this wave's first byte within a row
  const unsigned char *rowp = p.B + (size_t)(uint32_t)(row0 + rl) * row_bytes;
  u32x4 wv[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i)
    wv[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rowp + kb0 + 64u * i + 16u * g));
  // x: A fragment (i, j) = 16 B at 4 kb0 + 64 g + 256 i + 16 j in the diagonal lanes, zeros elsewhere
  typedef const __attribute__((address_space(1))) char *gcp;   // global, not flat, loads
  u32x4 xa[NL][4];
#pragma unroll
  for (int i = 0; i < NL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) xa[i][j] = u32x4{0u, 0u, 0u, 0u};
  if (rl == g) {   // four lanes load x (exec-masked: a quarter KiB per load, not a KiB of zeros)
    const gcp xbase = (gcp)p.x + 4u * kb0 + 64u * (uint32_t)g;
#pragma unroll
    for (int i = 0; i < NL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        xa[i][j] = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(xbase + 256 * i + 16 * j);
  }
  // scales of row (row0 + rl): its 2 NL blocks of this wave's range as NL / 2 dwords of qabsmax
  const uint32_t bpr = (uint32_t)p.K >> p.bs_log2;
  const uint32_t b0 = (uint32_t)p.block_base + (uint32_t)(row0 + rl) * bpr + ((2u * kb0) >> p.bs_log2);
  uint32_t qv[NL / 2];
#pragma unroll
  for (int t = 0; t < NL / 2; ++t) qv[t] = reinterpret_cast<const uint32_t *>(p.sc.qabsmax + b0)[t];
  const float a2 = p.sc.absmax2[b0 >> p.bs2_log2];    // the 2 NL blocks share one (host-checked)
  if (threadIdx.x < 256) {
    s_code2[threadIdx.x] = c2;
    store_byte_table_entry<kPieces>(s_tab, tab_entry);
  }
  __syncthreads();
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  const uint32_t jb = WT ? (uint32_t)(lane & 31) << 3 : (uint32_t)(lane & 15) << 3;
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t w[4] = {wv[i].x, wv[i].y, wv[i].z, wv[i].w};
    uint32_t hi[16], lo[16];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t a;
        if constexpr (WT) a = __builtin_amdgcn_perm(w[d], jb, 0x0C0C0000u | ((4u + m) << 8));
        else a = ((m == 0 ? (w[d] << 7) : (w[d] >> (8 * m - 7))) & 0x7F80u) | jb;
        if constexpr (CL) {
          const u32x2 e = *reinterpret_cast<const u32x2 *>(tb + a);
          hi[4 * d + m] = e.x;
          lo[4 * d + m] = e.y;
        } else {
          hi[4 * d + m] = *reinterpret_cast<const uint32_t *>(tb + a);
        }
      }
    }
    float4_t c = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const half8_t af = __builtin_bit_cast(half8_t, xa[i][j]);
      const u32x4 bh = {hi[4 * j], hi[4 * j + 1], hi[4 * j + 2], hi[4 * j + 3]};
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, __builtin_bit_cast(half8_t, bh), c, 0, 0, 0);
      if constexpr (CL) {
        const u32x4 bl = {lo[4 * j], lo[4 * j + 1], lo[4 * j + 2], lo[4 * j + 3]};
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, __builtin_bit_cast(half8_t, bl), c, 0, 0, 0);
      }
    }
    // chunks 0, 1 of load i lie in block 2 i, chunks 2, 3 in block 2 i + 1 (bytes of qv)
    const uint32_t qw = qv[i >> 1];
    const float am0 = __fadd_rn(__fmul_rn(s_code2[(qw >> (16 * (i & 1))) & 0xFFu], a2), offset);
    const float am1 = __fadd_rn(__fmul_rn(s_code2[(qw >> (16 * (i & 1) + 8)) & 0xFFu], a2), offset);
    acc = fmaf(__fadd_rn(c[0], c[1]), am0, acc);
    acc = fmaf(__fadd_rn(c[2], c[3]), am1, acc);
  }
  if (lane < 16) s_part[wave][lane] = acc;
  __syncthreads();
  if (threadIdx.x < 16) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < NWK; ++w) v += s_part[w][threadIdx.x];
    const int row = row0 + (int)threadIdx.x;
    float o = v * p.out_scale;
    if (p.bias) o += load_f32<QZ_DT_F16>(p.bias, row);
    store_f32<QZ_DT_F16>(p.y, row, o);
  }
}

// ---------------------------------------------------------------------------
// MFMA-diagonal decode GEMV (round 4, experimental: k_gemv_4bit_dg).  The product GEMV's memory
// layout -- a wave reads ONE row per load instruction, contiguously -- with the products on
// the matrix pipe:
//  * a segment is 1024 elements (512 B) of a row; lane l owns its 16-element chunk
//    c(l) = 4 (l & 15) + (l >> 4), i.e. 8 B at 8 c(l): one dwordx2 per lane per segment;
//  * v_mfma_f32_16x16x32_f16 with the lane's codes as A (A[m = l & 15][k = 8 (l >> 4) + jj])
//    and the lane's OWN x as B (B[k = 8 (l >> 4) + jj][n = l & 15]): C[m][n] sums the four k
//    groups g of lanes m + 16 g (codes) against lanes n + 16 g (x), so the diagonal m == n is
//    sum_g codes(chunk 4 m + g) . x(chunk 4 m + g) = the dot of scale block m of the segment
//    (chunks 4m..4m+3 = elements 64m..64m+63): one absmax per diagonal element;
//  * exact codes: an A fragment is two table entries as they land from two ds_read_b64,
//    {hi pair, lo pair} of bytes 2f and 2f + 1 = codes (ch, ch, cl, cl, ch, ch, cl, cl), and B
//    the matching x pairs doubled (x, x, x, x of 4f..4f+3 as (x0 x1 x0 x1 x2 x3 x2 x3)) -- built
//    once per segment and shared by the R rows;
//  * the diagonal C[m][m] sits in lane m + 16 (m >> 2), register m & 3: every lane scales its
//    four C registers by its block's absmax into four running sums per row and keeps the one
//    with index m & 3 at the end; 16 lanes x NWK waves meet in LDS.
// ---------------------------------------------------------------------------
template <bool CL, int R, int NSEG, int NWK>
__global__ __launch_bounds__(NWK * 64) void k_gemv_4bit_dg(GemvParams p_in) {
  const GemvParams p = load_params(p_in);
  constexpr int kPieces = 16;   // the 256-B-entry (WT) table: 32 bank-private 8-B copies, one v_perm per address
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[2 * kTabDwords];
  __shared__ float s_code2[256];
  __shared__ float s_red[NWK][R][16];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int row0 = blockIdx.x * R;
  const int m = lane & 15;                                   // this lane's C column = its diagonal row
  const uint32_t c = 4u * (uint32_t)m + ((uint32_t)lane >> 4);  // this lane's 16-element chunk of a segment
  const uint32_t row_bytes = (uint32_t)p.K >> 1;
  // 1. code2 and the table entry first (the barrier waits for them)
  float c2 = 0.0f;
  if (threadIdx.x < 256) c2 = p.sc.code2[threadIdx.x];
  const float offset = *p.sc.offset;
  u32x4 tab_entry = {0u, 0u, 0u, 0u};
  if (threadIdx.x < 256) tab_entry = reinterpret_cast<const u32x4 *>((CL ? &g_byte_tab_nf4x : &g_byte_tab_nf4)->v)[threadIdx.x];
  // 2. weights (R rows x NSEG segments), x (the lane's chunk of each segment), scale codes
  const uint32_t seg0 = (uint32_t)(wave * NSEG);               // this wave's first segment of the row
  u32x2 wv[NSEG][R];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const unsigned char *rp = p.B + (size_t)(uint32_t)(row0 + r) * row_bytes + (seg0 + sg) * 512u + 8u * c;
      wv[sg][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(rp));
    }
  u32x4 xr[NSEG][2];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    const u32x4 *xp = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(p.x) + ((seg0 + sg) * 1024u + 16u * c) * 2u);
    xr[sg][0] = xp[0];
    xr[sg][1] = xp[1];
  }
  const uint32_t bpr = (uint32_t)p.K >> p.bs_log2;             // 64-element blocks per row
  uint32_t qb[NSEG][R];
  float a2[NSEG][R];
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t b = (uint32_t)p.block_base + (uint32_t)(row0 + r) * bpr + (seg0 + sg) * 16u;   // the segment's first block
      qb[sg][r] = p.sc.qabsmax[b + (uint32_t)m];
      typedef const __attribute__((address_space(4))) float *cfp;
      a2[sg][r] = ((cfp)p.sc.absmax2)[b >> p.bs2_log2];        // one per (row, segment): 16 | 256
    }
  if (threadIdx.x < 256) {
    s_code2[threadIdx.x] = c2;
    store_byte_table_entry<kPieces>(s_tab, tab_entry);
  }
  __syncthreads();
  const unsigned char *tb = reinterpret_cast<const unsigned char *>(s_tab);
  const uint32_t jb = (uint32_t)(lane & 31) << 3;
  float4_t acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = float4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int sg = 0; sg < NSEG; ++sg) {
    const uint32_t X[8] = {xr[sg][0].x, xr[sg][0].y, xr[sg][0].z, xr[sg][0].w,
                           xr[sg][1].x, xr[sg][1].y, xr[sg][1].z, xr[sg][1].w};
    half8_t bfr[CL ? 4 : 2];
#pragma unroll
    for (int f = 0; f < (CL ? 4 : 2); ++f) {
      const u32x4 b = CL ? u32x4{X[2 * f], X[2 * f], X[2 * f + 1], X[2 * f + 1]}
                         : u32x4{X[4 * f], X[4 * f + 1], X[4 * f + 2], X[4 * f + 3]};
      bfr[f] = __builtin_bit_cast(half8_t, b);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t w[2] = {wv[sg][r].x, wv[sg][r].y};
      float4_t cc = {0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (CL) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const uint32_t wd = w[f >> 1];
          const uint32_t b0 = (uint32_t)(2 * (f & 1)), b1 = b0 + 1u;
          const u32x2 e0 = *reinterpret_cast<const u32x2 *>(tb + __builtin_amdgcn_perm(wd, jb, 0x0C0C0000u | ((4u + b0) << 8)));
          const u32x2 e1 = *reinterpret_cast<const u32x2 *>(tb + __builtin_amdgcn_perm(wd, jb, 0x0C0C0000u | ((4u + b1) << 8)));
          const u32x4 a = {e0.x, e0.y, e1.x, e1.y};
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8_t, a), bfr[f], cc, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          uint32_t h[4];
#pragma unroll
          for (int t = 0; t < 4; ++t)
            h[t] = *reinterpret_cast<const uint32_t *>(tb + __builtin_amdgcn_perm(w[f], jb, 0x0C0C0000u | ((4u + t) << 8)));
          const u32x4 a = {h[0], h[1], h[2], h[3]};
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8_t, a), bfr[f], cc, 0, 0, 0);
        }
      }
      const float am = __fadd_rn(__fmul_rn(s_code2[qb[sg][r]], a2[sg][r]), offset);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[r][k] = fmaf(cc[k], am, acc[r][k]);
    }
  }
  // the diagonal: lane l keeps register m & 3 if m >> 2 == l >> 4 (its block's dot), else nothing
  const bool diag = (m >> 2) == (lane >> 4);
  const int k3 = m & 3;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float v = k3 == 0 ? acc[r][0] : k3 == 1 ? acc[r][1] : k3 == 2 ? acc[r][2] : acc[r][3];
    if (diag) s_red[wave][r][m] = v;
  }
  __syncthreads();
  if (threadIdx.x < R * 16) {   // thread (r, b): the NWK partials of block column b of row r, then 16 lanes
    const int r = threadIdx.x >> 4, b = threadIdx.x & 15;
    float v = 0.0f;
#pragma unroll
    for (int wk = 0; wk < NWK; ++wk) v += s_red[wk][r][b];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
    if (b == 0) {
      const int row = row0 + r;
      float o = v * p.out_scale;
      if (p.bias) o += load_f32<QZ_DT_F16>(p.bias, row);
      store_f32<QZ_DT_F16>(p.y, row, o);
    }
  }
}


template <int MODE, bool DQ, int DT, int R, int WK, bool FS, bool CL, bool NRM = false, int OPT = 0, bool GPS = false,
          bool WT = false>
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
  gemv_body<MODE, DQ, DT, R, WK, 4, false, 0, FS, CL, WT, NRM, false, 0, OPT, false, false, 0, GPS>(seg, b - start,
                                                                                                 nullptr, &g);
}

// QZ_GROUPED_PS / QZ_GROUPED_WT (measurement knobs): persistent workgroups for the two-step grouped
// launch with the fused norm (optionally on the 256-B-entry exact-code table)
template <bool DQ, int DT, int R, bool CL, bool WT>
static void launch_grouped_ps(unsigned grid, size_t lds, hipStream_t s, const GemvGroup &g) {
  if constexpr ((DT == QZ_DT_F16 || DT == QZ_DT_BF16) && (R == 1 || R == 2 || R == 4) && (!WT || (CL && DT == QZ_DT_F16)))
    hipLaunchKernelGGL((k_gemv_4bit_grouped<kModeTab, DQ, DT, R, 1, true, CL, true, 8, true, WT>), dim3(grid), dim3(256),
                       lds, s, g);
}

// LlamaMLP's gate/up pair (gemv_body PAIR): one launch computes act_fn(gate_proj(x)) * up_proj(x)
template <int MODE, bool DQ, int DT, int R, bool FS, bool CL, bool NRM, int OPT = 0, bool PS = false, bool WT = false>
__global__ __launch_bounds__(256) void k_gemv_4bit_pair(GemvGroup g) {
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
  const GemvParams seg = g.seg[wave >> 1];
  gemv_body<MODE, DQ, DT, R, 1, 4, false, 0, FS, CL, WT, NRM, true, 0, OPT, false, PS>(seg, blockIdx.x, g.seg);
}

// QZ_PAIR_WT (measurement knob): the persistent exact-code pair on the 256-B-entry table (64 KiB: 32
// bank-private copies of each 8-B entry, v_perm addresses), 2 workgroups per CU
template <bool DQ, int DT, int R, bool CL, bool NRM>
static void launch_pair_wt(unsigned grid, size_t lds, hipStream_t s, const GemvGroup &g) {
  if constexpr (CL && NRM && DT == QZ_DT_F16 && (R == 2 || R == 4))
    hipLaunchKernelGGL((k_gemv_4bit_pair<kModeTab, DQ, DT, R, true, CL, NRM, 8, true, true>), dim3(grid), dim3(256), lds,
                       s, g);
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
// host-side table construction
// ---------------------------------------------------------------------------
static uint16_t f32_to_f16_bits(float f) {
  return __half_as_ushort(__float2half_rn(f));  // host-side RNE conversion (hip_fp16.h)
}

static void build_tables(int mode, int quant_type, uint32_t tab[8], float *out_scale) {
  for (int i = 0; i < 8; ++i) tab[i] = 0;
  if (mode == kModeTab && quant_type == QZ_FP4) {
    // 16-entry planes of the signed FP4 codebook x12: magnitudes {0, 1/16, 8, 12, 4, 6, 2, 3}
    // are exact fp16 values with zero low bytes; codes 8..15 carry the sign (code 8 = -0.0)
    const uint8_t hb[8] = {0x00, 0x2C, 0x48, 0x4A, 0x44, 0x46, 0x40, 0x42};
    for (int i = 0; i < 16; ++i) {
      const uint32_t h = (uint32_t)hb[i & 7] | (i >= 8 ? 0x80u : 0u);
      tab[4 + (i >> 2)] |= h << (8 * (i & 3));
    }
    *out_scale = 1.0f / 12.0f;
    return;
  }
  if (mode == kModeFP4) {
    // magnitudes x12 for codes 0..7: {0, 1/16, 8, 12, 4, 6, 2, 3}, fp16 high bytes (low bytes are 0)
    const uint8_t hb[8] = {0x00, 0x2C, 0x48, 0x4A, 0x44, 0x46, 0x40, 0x42};
    for (int i = 0; i < 8; ++i) tab[i >> 2] |= (uint32_t)hb[i] << (8 * (i & 3));
    *out_scale = 1.0f / 12.0f;
    return;
  }
  static const float nf4[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                                -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                                0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                                0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                                0.7229568362236023f, 1.0f};
  (void)quant_type;
  for (int i = 0; i < 16; ++i) {
    const uint16_t h = f32_to_f16_bits(nf4[i]);
    tab[i >> 2] |= (uint32_t)(h & 0xFF) << (8 * (i & 3));
    tab[4 + (i >> 2)] |= (uint32_t)(h >> 8) << (8 * (i & 3));
  }
  *out_scale = 1.0f;
}

// Exact NF4 codes (CL) as fp16 byte planes: hi = fp16(c * 2^14) in `hi`, lo = fp16(c * 2^14 - hi)
// in `lo` (the kernel's SGPR-built table, OPT & 2; the same values as g_byte_tab_nf4x)
static void build_exact_planes(uint32_t hi[8], uint32_t lo[8]) {
  for (int i = 0; i < 8; ++i) hi[i] = lo[i] = 0;
  for (int i = 0; i < 16; ++i) {
    const float c = kNF4Host[i] * (float)(1 << kNF4ExactShift);
    const uint16_t h = f32_to_f16_bits(c);
    const uint16_t l = f32_to_f16_bits(c - __half2float(__ushort_as_half(h)));
    hi[i >> 2] |= (uint32_t)(h & 0xFF) << (8 * (i & 3));
    hi[4 + (i >> 2)] |= (uint32_t)(h >> 8) << (8 * (i & 3));
    lo[i >> 2] |= (uint32_t)(l & 0xFF) << (8 * (i & 3));
    lo[4 + (i >> 2)] |= (uint32_t)(l >> 8) << (8 * (i & 3));
  }
}

static int ilog2(long long v) {
  int l = 0;
  while ((1LL << l) < v) ++l;
  return (1LL << l) == v ? l : -1;
}

// Geometries choose_geometry can return: (R, WK) in {(4,1), (4,2), (2,1), (1,1), (1,2), (1,4)}.
// two_steps(K, WK): every wave owns exactly two full K-steps (gemv_body OPT 8, the straight-line
// form: step 2 issued right after the prologue barrier; profiles/r4_gemv_two_step.txt).  WK = 1
// only: at K = 8192, WK = 2 (the Llama-3-70B q/k/v and o shapes, R = 4) hipcc gives the
// straight-line body 259-278 VGPRs against 130 for the loop form -- one wave per SIMD
// (profiles/r4_bench_70b_two_step_regression.txt)
static inline bool two_steps(int K, int WK, bool fs) { return fs && WK == 1 && K == 2 * 2048; }

template <int MODE, bool DQ, int DT, bool FS, bool CL>
static void launch_vec(const GemvParams &p, int R, int WK, hipStream_t s) {
  const int RG = 4 / WK;
  const unsigned grid = (unsigned)((p.M + R * RG - 1) / (R * RG));
#define QZ_GV(RR, WW, OPT_) \
  hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, DT, RR, WW, 4, false, 0, FS, CL, false, 0, (WW == 1 ? OPT_ : 0)>), dim3(grid), \
                     dim3(256), 0, s, p)
#define QZ_GV_RW(OPT_)                        \
  do {                                        \
    if (R == 4 && WK == 2) QZ_GV(4, 2, OPT_); \
    else if (R == 4) QZ_GV(4, 1, OPT_);       \
    else if (R == 2) QZ_GV(2, 1, OPT_);       \
    else if (WK == 1) QZ_GV(1, 1, OPT_);      \
    else if (WK == 2) QZ_GV(1, 2, OPT_);      \
    else QZ_GV(1, 4, OPT_);                   \
  } while (0)
  if constexpr (FS) {
    if (two_steps(p.K, WK, true)) { QZ_GV_RW(8); return; }
  }
  // exact codes, K >= 14336 (down_proj: 7 or more K-steps per wave): 8-wave workgroups sharing one
  // 256-B-entry table (conflict-free, v_perm addresses): 4096 x 14336 8.92 -> 8.70 us, 8192 x 28672
  // (R = 4) 29.2 -> 25.5 us (profiles/r4_gemv_8wave_wide_table.txt); the per-row sums are the same
  if constexpr (FS && CL && DT == QZ_DT_F16 && MODE == kModeTab) {
    const char *w8 = getenv("QZ_GEMV_WIDE8");   // measurement knob (read per call): 0 = off
    if (WK == 1 && (R == 2 || R == 4) && p.K >= 14336 && !(w8 && atoi(w8) == 0)) {
      const unsigned g8 = (unsigned)((p.M + R * 8 - 1) / (R * 8));
      if (R == 4) hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, DT, 4, 1, 8, false, 0, FS, CL, true>), dim3(g8), dim3(512), 0, s, p);
      else hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, DT, 2, 1, 8, false, 0, FS, CL, true>), dim3(g8), dim3(512), 0, s, p);
      return;
    }
  }
  QZ_GV_RW(0);
#undef QZ_GV_RW
#undef QZ_GV
}

template <int MODE, bool DQ, bool FS, bool CL>
static int dispatch_dt(const GemvParams &p, int dtype, int R, int WK, hipStream_t s) {
  switch (dtype) {
    case QZ_DT_F16: launch_vec<MODE, DQ, QZ_DT_F16, FS, CL>(p, R, WK, s); return QZ_OK;
    case QZ_DT_BF16: launch_vec<MODE, DQ, QZ_DT_BF16, FS, CL>(p, R, WK, s); return QZ_OK;
    case QZ_DT_F32: launch_vec<MODE, DQ, QZ_DT_F32, FS, CL>(p, R, WK, s); return QZ_OK;
  }
  return QZ_ERR_DTYPE;
}

template <bool CL>
static int dispatch_tab(const GemvParams &p, int dtype, bool dq, bool fs, int R, int WK, hipStream_t s) {
  if (fs) return dq ? dispatch_dt<kModeTab, true, true, CL>(p, dtype, R, WK, s)
                    : dispatch_dt<kModeTab, false, true, CL>(p, dtype, R, WK, s);
  return dq ? dispatch_dt<kModeTab, true, false, CL>(p, dtype, R, WK, s)
            : dispatch_dt<kModeTab, false, false, CL>(p, dtype, R, WK, s);
}

}  // namespace qz

using namespace qz;

// Geometry (WK = waves along K, R = rows per wave) for the byte-table decode,
// from the measured shape sweep in DESIGN.md section 4.1 (scripts/gpu_sessions/run24.sh):
//  * >= 64 Mi weights (gate/up groups, 8192x28672, ...): R=4 -- more bytes in
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
  *R = (f32 || (long long)M * K >= (1LL << 26)) ? 4 : 2;
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

// Decode tables for the byte-table kernel: the 16-entry codebook as fp16 byte
// planes (a runtime `lut` is converted in kernel, so its planes stay zero).
// Exact codes (CL): the built-in NF4 table holds code * 2^14 as hi + lo.
static void set_tables(int quant_type, const float *lut, bool cl, int dtype, GemvParams *p) {
  build_tables(kModeTab, lut ? QZ_NF4 : quant_type, p->tab, &p->out_scale);
  if (dtype == QZ_DT_BF16 || dtype == QZ_DT_F32) {  // bf16 / fp32 code tables: NF4 codes, FP4 x12
    const bool fp4 = !lut && quant_type == QZ_FP4;
    p->tabsel = fp4 ? 1 : 0;
    p->out_scale = fp4 ? 1.0f / 12.0f : 1.0f;
    return;
  }
  p->tabsel = (!lut && quant_type == QZ_FP4) ? 1 : (cl ? 2 : 0);
  for (int i = 0; i < 8; ++i) p->tab_lo[i] = 0;
  if (lut) p->out_scale = 1.0f;
  else if (cl) {
    p->out_scale = 1.0f / (float)(1 << kNF4ExactShift);
    build_exact_planes(p->tab, p->tab_lo);
  }
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
  p->nw = nullptr;
  p->eps = 0.0f;
  p->res = nullptr;
  p->pf = nullptr;
  p->pf_row_bytes = 0;
  p->pf_rows = 0;
  p->pf_chunks = 0;
  *vec_ok = K > 0 && (K % 32) == 0 && blocksize >= 32 && (reinterpret_cast<uintptr_t>(B) % 16) == 0 &&
            (reinterpret_cast<uintptr_t>(x) % 16) == 0 &&
            (long long)M * K + 2LL * 1024 < (1LL << 32) &&            // 32-bit element offsets
            block_base + (long long)M * K / blocksize < (1LL << 32);   // 32-bit block indices
  return QZ_OK;
}

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
  // bf16 x always decodes with bf16 hi + lo codes (~2^-16) and fp32 x with fp32 codes: the
  // exact-code (CL) variant is the fp16-activation option only
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
constexpr int kNormMaxBlocks = 4096;
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
  // QZ_GROUPED_NORM_R (measurement knob, read once): rows per wave of the fused pre-norm launch
  // (1, 2, 4) where the geometry keeps whole rows per wave (WK = 1: the same per-row sums)
  static const int norm_r = [] {
    const char *e = getenv("QZ_GROUPED_NORM_R");
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 2 || v == 4 ? v : 0;
  }();
  if (nw && norm_r && WK == 1) R = norm_r;
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
  bool all_fs = true;
  for (int i = 0; i < nseg; ++i) all_fs = all_fs && full_steps(K, blocksize, blocksize2, dq, segs[i].block_base);
  hipStream_t s = (hipStream_t)stream;
  const bool two = two_steps(K, WK, all_fs || nw);
#define QZ_GR1(DQ_, DT_, RR, WW, FS_, OPT_)                                                                    \
  do {                                                                                                      \
    if (cl) hipLaunchKernelGGL((k_gemv_4bit_grouped<kModeTab, DQ_, DT_, RR, WW, FS_, true, false, OPT_>),   \
                               dim3(blocks), dim3(256), 0, s, g);                                           \
    else hipLaunchKernelGGL((k_gemv_4bit_grouped<kModeTab, DQ_, DT_, RR, WW, FS_, false, false, OPT_>),     \
                            dim3(blocks), dim3(256), 0, s, g);                                              \
  } while (0)
#define QZ_GR(DQ_, DT_, RR, WW, FS_)                                 \
  do {                                                               \
    if (FS_ && two) QZ_GR1(DQ_, DT_, RR, WW, FS_, (FS_ && WW == 1 ? 8 : 0));    \
    else QZ_GR1(DQ_, DT_, RR, WW, FS_, 0);                           \
  } while (0)
#define QZ_GR_RW(DQ_, DT_, FS_)                                      \
  do {                                                               \
    if (R == 4 && WK == 2) QZ_GR(DQ_, DT_, 4, 2, FS_);               \
    else if (R == 4) QZ_GR(DQ_, DT_, 4, 1, FS_);                     \
    else if (R == 2) QZ_GR(DQ_, DT_, 2, 1, FS_);                     \
    else if (WK == 1) QZ_GR(DQ_, DT_, 1, 1, FS_);                    \
    else if (WK == 2) QZ_GR(DQ_, DT_, 1, 2, FS_);                    \
    else QZ_GR(DQ_, DT_, 1, 4, FS_);                                 \
  } while (0)
#define QZ_GR_DT(DQ_, FS_)                                           \
  do {                                                               \
    if (dtype == QZ_DT_F16) QZ_GR_RW(DQ_, QZ_DT_F16, FS_);           \
    else if (dtype == QZ_DT_BF16) QZ_GR_RW(DQ_, QZ_DT_BF16, FS_);    \
    else QZ_GR_RW(DQ_, QZ_DT_F32, FS_);                              \
  } while (0)
  // QZ_GROUPED_EARLY=1 (measurement knob, read per call): the normed two-step launch issues its second
  // K-step before the prologue barriers (OPT 1 | 8) instead of after them
  const char *gee = getenv("QZ_GROUPED_EARLY");
  const bool g_early = gee && atoi(gee) == 1;
#define QZ_GN(DQ_, DT_, RR, WW, CL_)                                                                          \
  do {                                                                                                        \
    if (two && g_early && WW == 1)                                                                            \
      hipLaunchKernelGGL((k_gemv_4bit_grouped<kModeTab, DQ_, DT_, RR, WW, true, CL_, true, (WW == 1 ? 9 : 0)>), dim3(blocks), \
                         dim3(256), (size_t)K * 2, s, g);                                                     \
    else if (two) hipLaunchKernelGGL((k_gemv_4bit_grouped<kModeTab, DQ_, DT_, RR, WW, true, CL_, true, (WW == 1 ? 8 : 0)>), \
                                dim3(blocks), dim3(256), (size_t)K * 2, s, g);                                \
    else hipLaunchKernelGGL((k_gemv_4bit_grouped<kModeTab, DQ_, DT_, RR, WW, true, CL_, true>), dim3(blocks),  \
                            dim3(256), (size_t)K * 2, s, g);                                                  \
  } while (0)
#define QZ_GN_RW(DQ_, DT_, CL_)                                      \
  do {                                                               \
    if (R == 4 && WK == 2) QZ_GN(DQ_, DT_, 4, 2, CL_);               \
    else if (R == 4) QZ_GN(DQ_, DT_, 4, 1, CL_);                     \
    else if (R == 2) QZ_GN(DQ_, DT_, 2, 1, CL_);                     \
    else if (WK == 1) QZ_GN(DQ_, DT_, 1, 1, CL_);                    \
    else if (WK == 2) QZ_GN(DQ_, DT_, 1, 2, CL_);                    \
    else QZ_GN(DQ_, DT_, 1, 4, CL_);                                 \
  } while (0)
  // QZ_GROUPED_PS (measurement knob, read per call): persistent workgroups for the two-step grouped
  // launch with the fused norm: 1..8 per CU, >= 16 the grid; QZ_GROUPED_PS_R rows per wave (1, 2, 4)
  // and QZ_GROUPED_WT=1 the 256-B-entry exact-code table
  if (nw && two && WK == 1) {
    const char *gpe = getenv("QZ_GROUPED_PS");
    const int gps = gpe ? atoi(gpe) : 0;
    if (gps > 0) {
      int Rg = R;
      if (const char *gre = getenv("QZ_GROUPED_PS_R")) {
        const int v = atoi(gre);
        if (v == 1 || v == 2 || v == 4) Rg = v;
      }
      GemvGroup g2 = g;
      int gb = 0;
      for (int i = 0; i < nseg; ++i) {
        g2.start[i] = gb;
        gb += (g2.seg[i].M + 4 * Rg - 1) / (4 * Rg);
      }
      for (int i = nseg; i < kMaxSeg; ++i) g2.start[i] = gb;
      g2.total = gb;
      const unsigned ggrid = (unsigned)(gps <= 8 ? 256 * gps : gps);
      const char *gwe = getenv("QZ_GROUPED_WT");
      const bool gwt = gwe && atoi(gwe) == 1 && cl && dtype == QZ_DT_F16;
      if ((int)ggrid < gb) {
        const size_t lds = (size_t)K * 2;
#define QZ_GP(DQ_, DT_, RR)                                                                                 \
  do {                                                                                                      \
    if (gwt) launch_grouped_ps<DQ_, DT_, RR, true, true>(ggrid, lds, s, g2);                                \
    else if (cl) launch_grouped_ps<DQ_, DT_, RR, true, false>(ggrid, lds, s, g2);                           \
    else launch_grouped_ps<DQ_, DT_, RR, false, false>(ggrid, lds, s, g2);                                  \
  } while (0)
#define QZ_GP_R(DQ_, DT_)                                                                                   \
  do {                                                                                                      \
    if (Rg == 4) QZ_GP(DQ_, DT_, 4); else if (Rg == 2) QZ_GP(DQ_, DT_, 2); else QZ_GP(DQ_, DT_, 1);        \
  } while (0)
        if (dtype == QZ_DT_F16) { if (dq) QZ_GP_R(true, QZ_DT_F16); else QZ_GP_R(false, QZ_DT_F16); }
        else { if (dq) QZ_GP_R(true, QZ_DT_BF16); else QZ_GP_R(false, QZ_DT_BF16); }
#undef QZ_GP_R
#undef QZ_GP
        QZ_LAUNCH_CHECK();
        return QZ_OK;
      }
    }
  }
  if (nw) {
    if (dtype == QZ_DT_F16) {
      if (dq) { if (cl) QZ_GN_RW(true, QZ_DT_F16, true); else QZ_GN_RW(true, QZ_DT_F16, false); }
      else { if (cl) QZ_GN_RW(false, QZ_DT_F16, true); else QZ_GN_RW(false, QZ_DT_F16, false); }
    } else {
      if (dq) QZ_GN_RW(true, QZ_DT_BF16, false); else QZ_GN_RW(false, QZ_DT_BF16, false);
    }
  } else if (all_fs) { if (dq) QZ_GR_DT(true, true); else QZ_GR_DT(false, true); }
  else { if (dq) QZ_GR_DT(true, false); else QZ_GR_DT(false, false); }
#undef QZ_GN_RW
#undef QZ_GN
#undef QZ_GR_DT
#undef QZ_GR_RW
#undef QZ_GR
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
  // so the same bits); the epilogue needs whole rows per wave: splits along K (WK > 1, e.g. the
  // K = 8192 layers) are left to the two-launch form.  Single-row waves (R = 1: small row shards,
  // e.g. Llama-3-8B gate/up over 8 ranks) take the pair launch too
  int R, WK;
  choose_geometry(2 * M, K, dtype, &R, &WK);
  if (WK != 1) return QZ_ERR_SHAPE;
  // QZ_PAIR_R (measurement knob, read once): rows per wave for the pair launch (2, 3, 4, 6, 8); the per-row
  // sums do not depend on R, so neither do the bits
  static const int pair_r = [] {
    const char *e = getenv("QZ_PAIR_R");
    const int v = e ? atoi(e) : 0;
    return v == 2 || v == 3 || v == 4 || v == 6 || v == 8 ? v : 0;
  }();
  if (pair_r) R = pair_r;
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
  // or within 4 % of the best of 2 / 3 / 4 per CU and of blocks / 2 at every shape.  QZ_PAIR_PS
  // (measurement knob, read per call) overrides: 1..8 = workgroups per CU, >= 16 = the grid, 0 = one
  // workgroup per block
  // With exact codes and R = 2 / 4 the persistent pair takes the 256-B-entry table (64 KiB: 32
  // bank-private copies of each 8-B entry, one v_perm per address, no bank conflicts) at 2
  // workgroups per CU: 16.2-16.8 -> 15.1 us for 14336 rows, 10.8 -> 10.6 for 7168
  // (profiles/r4_pair_persistent_wide_table.txt); QZ_PAIR_WT=0 (knob, read per call) keeps the 16-copy table
  const char *wte = getenv("QZ_PAIR_WT");
  // (from 3 blocks per workgroup on: at the N = 4 shard, 896 blocks, the 16-copy table at 3 per CU is
  // 3 % faster)
  const bool wt_ok = cl && norm_weight && (R == 2 || R == 4) && blocks >= 3 * 512 && !(wte && atoi(wte) == 0);
  const char *pse = getenv("QZ_PAIR_PS");
  int pgrid_i = 0;
  if (pse) {
    const int ps = atoi(pse);
    pgrid_i = ps <= 0 ? 0 : ps <= 8 ? 256 * ps : ps;
  } else if (norm_weight) {
    pgrid_i = (wt_ok ? 2 : 3) * 256;
  }
  const unsigned pgrid = (unsigned)max(pgrid_i, 1);
  const bool persist = two && pgrid_i > 0 && pgrid_i < blocks;
  const bool pair_wt = persist && wt_ok;
#define QZ_PS(DQ_, DT_, RR, CL_, NRM_)                                                                               \
  do {                                                                                                              \
    if (pair_wt) launch_pair_wt<DQ_, DT_, RR, CL_, NRM_>(pgrid, lds, s, g);                                        \
    else if (persist) hipLaunchKernelGGL((k_gemv_4bit_pair<kModeTab, DQ_, DT_, RR, true, CL_, NRM_, 8, true>), dim3(pgrid), \
                                    dim3(256), lds, s, g);                                                          \
    else if (two) hipLaunchKernelGGL((k_gemv_4bit_pair<kModeTab, DQ_, DT_, RR, true, CL_, NRM_, 8>), dim3(blocks),    \
                                     dim3(256), lds, s, g);                                                         \
    else hipLaunchKernelGGL((k_gemv_4bit_pair<kModeTab, DQ_, DT_, RR, true, CL_, NRM_>), dim3(blocks), dim3(256), lds, \
                            s, g);                                                                                  \
  } while (0)
#define QZ_PS_R(DQ_, DT_, CL_, NRM_)           \
  do {                                          \
    if (R == 4) QZ_PS(DQ_, DT_, 4, CL_, NRM_);  \
    else if (R == 8) QZ_PS(DQ_, DT_, 8, CL_, NRM_);  \
    else if (R == 6) QZ_PS(DQ_, DT_, 6, CL_, NRM_);  \
    else if (R == 3) QZ_PS(DQ_, DT_, 3, CL_, NRM_);  \
    else if (R == 1) QZ_PS(DQ_, DT_, 1, CL_, NRM_);  \
    else QZ_PS(DQ_, DT_, 2, CL_, NRM_);         \
  } while (0)
#define QZ_PS_N(DQ_, DT_, CL_)                                                      \
  do {                                                                              \
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

// attn_core.h -- the decode attention of one query head as a device function over caller-provided
// LDS (layer_ops.hip: k_decode_attn).
//
// Decode attention with a static KV cache (LlamaAttention.forward, modeling_llama.py:243-281, for
// one new token per sequence): rotary of q and k, the cache update of StaticLayer.update
// (cache_utils.py:455-487: keys/values[:, :, p] = k, v and p += 1) and the masked GQA
// softmax(q k^T * scale) v of sdpa_attention_forward -- in eager torch 14 launches per layer (rope,
// arange, two int64 adds, two index_copy_, two repeat_kv copies, the bool-mask conversion,
// attn_fwd).  One workgroup of 256 threads takes ONE query head over kAttnChunk key positions (the
// G workgroups of a kv head read its cache rows G times, from L2: the per-workgroup serial work --
// the scores and P V, measured at 3.2 and 3.3 us of a 10.1 us launch with G = 4 heads per
// workgroup, profiles/r3_attn_ablation_g4.txt -- is what bounds a decode step's attention, not
// bandwidth); nsplit > 1 leaves per-chunk partials (max, sum, unnormalised output) that
// k_decode_attn_combine merges.
// Numerics: q and k are rotated with k_rope_qk's per-op rounding (the cache receives the
// bit-identical k), scores and probabilities stay fp32 (SDPA's flash kernel rounds the
// probabilities to the storage dtype before P V; this kernel does not), output rounded once.
#pragma once
#include "common.h"

namespace qz {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kAttnChunk = 128;  // key positions per workgroup
// QZ_ATTN_ABL (measurement builds only, scripts/dev/attn_ablation.py; 0 in the product): drop one
// phase to price it -- 1 the arrival atomic, 2 the cache row loads, 4 P V, 8 the scores,
// 16 the softmax exponentials, 32 everything after the loads
#ifndef QZ_ATTN_ABL
#define QZ_ATTN_ABL 0
#endif
constexpr int kAttnAbl = QZ_ATTN_ABL;
constexpr int kAttnMaxG = 8;     // query heads per kv head
constexpr int kAttnSpecL = 512;  // caches read before their mask arrives (speculatively) up to this length

struct DecodeAttnArgs {
  const void *q, *k, *v;     // projection outputs, row b at b * {qs, ks, vs} elements, head-major
  long long qs, ks, vs;
  const void *cos, *sin;     // [B or 1, D], row b at b * cs (cs = 0: one row for all)
  long long cs;
  void *kc, *vc;             // caches [B, Hkv, L, D], contiguous
  const unsigned char *mask;  // bool, element (b, j) at b * mb + j * mj
  long long mb, mj;
  long long *pos;            // write position p (StaticLayer.cumulative_length), advanced by one
  unsigned int *arrive;      // arrival counter, zero between launches
  void *out;                 // [B, Hq * D], row b at b * os
  long long os;
  float *part;               // nsplit > 1: [B, Hkv, nsplit, G, D + 2]
  int Hkv, G, L, nsplit;
  float scale;
};

// The fp32 value is pinned in a register first: otherwise hipcc folds a preceding __fmul_rn
// into the conversion (v_fma_mixlo_f16 a, b, 0), rounding the exact product to 16 bits ONCE,
// where torch rounds it to fp32 and then to the storage dtype (a different result whenever
// that double rounding differs, ~1 element in 1000 of an RMSNorm output).
template <int DT> __device__ __forceinline__ float round_dt(float v) {
  if constexpr (DT == QZ_DT_F32) return v;
  asm volatile("" : "+v"(v));
  if constexpr (DT == QZ_DT_F16) return __half2float(__float2half_rn(v));
  else return __bfloat162float(__float2bfloat16(v));
}

// storage bits of a value (the RNE conversions store_f32 uses) and back
template <int DT> __device__ __forceinline__ uint32_t bits_dt(float v) {
  if constexpr (DT == QZ_DT_F16) return f32_to_f16_bits(v);
  else return __bfloat16_as_ushort(__float2bfloat16(v));
}
template <int DT> __device__ __forceinline__ float from_bits(uint32_t u) {
  if constexpr (DT == QZ_DT_F16) return __half2float(__ushort_as_half((unsigned short)(u & 0xFFFFu)));
  else return __uint_as_float(u << 16);
}

template <int DT> __device__ __forceinline__ float dot2_dt(uint32_t a, uint32_t b, float c) {
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
  if constexpr (DT == QZ_DT_F16)
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b), c, false);
  else
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b16x2, a), __builtin_bit_cast(b16x2, b), c, false);
}

// LDS of one head's attention.  `v` is the staged v rows, kAttnChunk x H2 words with the word
// columns XOR-swizzled by (position & 31): a thread writes its half row at one column across 32
// consecutive positions per instruction, so an unswizzled 64-word row put every lane of a write
// group on one bank (profiles/r5_attn_vpad_ab.txt: 6.80 -> 6.43 us per launch with the rows
// spread); the P V reads (one row, consecutive columns) stay conflict-free.  The rest is small.
template <int D> struct AttnLds {
  static constexpr int H2 = D / 2;
  static constexpr int NSUB = kWave / H2;
  static constexpr int kVBytes = kAttnChunk * H2 * 4;
  // small-region offsets (bytes, 16-B aligned)
  static constexpr int oQh = 0;                               // rotated q, raw [H2 words]
  static constexpr int oSc = oQh + H2 * 4;                    // half-row partial scores [2][kAttnChunk]
  static constexpr int oP = oSc + 2 * kAttnChunk * 4;         // probabilities [kAttnChunk]
  static constexpr int oKn = oP + kAttnChunk * 4;             // the new rotated k, raw [H2]
  static constexpr int oVn = oKn + H2 * 4;                    // the new v, raw [H2]
  static constexpr int oOk = oVn + H2 * 4;                    // mask bytes [kAttnChunk]
  static constexpr int oPv = oOk + kAttnChunk;                // P V partials [4 NSUB][D]
  static constexpr int oMl = oPv + 4 * NSUB * D * 4;          // max, sum
  static constexpr int kSmallBytes = oMl + 16;
  uint32_t *v;
  unsigned char *small;
  __device__ uint32_t *qh() const { return reinterpret_cast<uint32_t *>(small + oQh); }
  __device__ float *sc() const { return reinterpret_cast<float *>(small + oSc); }
  __device__ float *p() const { return reinterpret_cast<float *>(small + oP); }
  __device__ uint32_t *kn() const { return reinterpret_cast<uint32_t *>(small + oKn); }
  __device__ uint32_t *vn() const { return reinterpret_cast<uint32_t *>(small + oVn); }
  __device__ unsigned char *ok() const { return small + oOk; }
  __device__ float *pv() const { return reinterpret_cast<float *>(small + oPv); }
  __device__ float *ml() const { return reinterpret_cast<float *>(small + oMl); }
  __device__ uint32_t &vw(int pos, int col) const { return v[pos * H2 + (col ^ (pos & 31))]; }
};

// One query head `hq` of sequence `b` over key chunk `split`, by the 256 threads of the calling
// workgroup (q, k and v come from a previous launch: plain loads).  Returns the position p it read (the caller advances *a.pos once every head is done).
template <int DT, int D>
__device__ __forceinline__ long long decode_attn_head(const DecodeAttnArgs &a, int split, int hq, int b,
                                                      const AttnLds<D> &S) {
  constexpr int ES = DT == QZ_DT_F32 ? 4 : 2;
  static_assert(ES == 2, "16-bit activations and caches");
  constexpr int H2 = D / 2;      // rotary half; also the share of a row one thread dots
  constexpr int NW = H2 / 2;     // 32-bit words of half a row
  constexpr int NSUB = kWave / H2;  // P V: lane groups per wave (D = 128: 1, D = 64: 2)
  uint32_t *s_qh = S.qh(), *s_kn = S.kn(), *s_vn = S.vn();
  float *s_p = S.p(), *s_pv = S.pv(), *s_ml = S.ml();
  float *s_sc = S.sc();
  unsigned char *s_ok = S.ok();

  const int t = threadIdx.x;
  const int G = a.G, L = a.L;
  const int h = hq / G, gq = hq - h * G;                     // kv head, query head within it
  const int j0 = split * kAttnChunk;
  const long long crow = ((long long)b * a.Hkv + h) * L;     // first cache row of (b, h)
  const int pos_i = t & (kAttnChunk - 1), half = t >> 7;     // this thread's key position / row half
  const long long j = j0 + pos_i;
  const bool in_l = j < L;

  // 0. Every global load goes out before anything waits (a decode step's attention is bound by
  //    latency, not bandwidth): p, the q / cos / sin / new k and v operands of the rotary
  //    (threads below H2: one pair each), then the mask byte and the half rows of k and v at
  //    position j -- whatever the mask says (a masked row is dropped after it arrives) -- for
  //    caches up to kAttnSpecL positions; a longer cache is read after its mask, so a long
  //    static cache early in a sequence does not stream its masked rows.
  const long long p = *a.pos;
  const bool rt = t < H2;
  float x1 = 0.f, x2 = 0.f, c1 = 0.f, c2 = 0.f, s1 = 0.f, s2 = 0.f, k1 = 0.f, k2 = 0.f;
  uint32_t vnew = 0u;
  if (rt) {
    const char *cb = reinterpret_cast<const char *>(a.cos) + (long long)b * a.cs * ES;
    const char *sb = reinterpret_cast<const char *>(a.sin) + (long long)b * a.cs * ES;
    const char *qb = reinterpret_cast<const char *>(a.q) + ((long long)b * a.qs + (long long)hq * D) * ES;
    const char *kb = reinterpret_cast<const char *>(a.k) + ((long long)b * a.ks + (long long)h * D) * ES;
    const char *vb = reinterpret_cast<const char *>(a.v) + ((long long)b * a.vs + (long long)h * D) * ES;
    x1 = load_f32<DT>(qb, t); x2 = load_f32<DT>(qb, t + H2);
    k1 = load_f32<DT>(kb, t); k2 = load_f32<DT>(kb, t + H2);
    vnew = reinterpret_cast<const uint32_t *>(vb)[t];  // elements 2t, 2t + 1
    c1 = load_f32<DT>(cb, t); c2 = load_f32<DT>(cb, t + H2);
    s1 = load_f32<DT>(sb, t); s2 = load_f32<DT>(sb, t + H2);
  }
  const unsigned char mk = in_l ? a.mask[(long long)b * a.mb + j * a.mj] : (unsigned char)0;
  u32x4 kr[NW / 4], vr[NW / 4];
  const bool spec = L <= kAttnSpecL;
  const u32x4 *kp = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(a.kc) + ((crow + j) * D + half * H2) * ES);
  const u32x4 *vp = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(a.vc) + ((crow + j) * D + half * H2) * ES);
  if (in_l && spec && (kAttnAbl & 2) == 0) {
#pragma unroll
    for (int i = 0; i < NW / 4; ++i) kr[i] = kp[i];
#pragma unroll
    for (int i = 0; i < NW / 4; ++i) vr[i] = vp[i];
  } else {
#pragma unroll
    for (int i = 0; i < NW / 4; ++i) kr[i] = vr[i] = u32x4{0u, 0u, 0u, 0u};
  }
  __builtin_amdgcn_sched_barrier(0);

  // 1. rotary of this query head (and, in the chunk holding p, of the new key), k_rope_qk's
  //    arithmetic: q*cos + cat(-x2, x1)*sin with every torch op rounded to the storage dtype.  The
  //    G query heads of one kv head all rotate the new key (bit-identical values); the first of
  //    them writes the cache rows.
  auto rope = [&](float u1, float u2, float &lo, float &hi) {
    lo = from_bits<DT>(bits_dt<DT>(__fadd_rn(round_dt<DT>(__fmul_rn(u1, c1)), round_dt<DT>(__fmul_rn(-u2, s1)))));
    hi = from_bits<DT>(bits_dt<DT>(__fadd_rn(round_dt<DT>(__fmul_rn(u2, c2)), round_dt<DT>(__fmul_rn(u1, s2)))));
  };
  const bool mine = p >= j0 && p < j0 + kAttnChunk && p < L;  // this chunk holds the new token
  if (rt) {
    float lo, hi;
    rope(x1, x2, lo, hi);
    reinterpret_cast<uint16_t *>(s_qh)[t] = (uint16_t)bits_dt<DT>(lo);
    reinterpret_cast<uint16_t *>(s_qh)[t + H2] = (uint16_t)bits_dt<DT>(hi);
    if (mine) {
      rope(k1, k2, lo, hi);
      if (gq == 0) {
        char *kd = reinterpret_cast<char *>(a.kc) + (crow + p) * D * ES;
        char *vd = reinterpret_cast<char *>(a.vc) + (crow + p) * D * ES;
        store_f32<DT>(kd, t, lo);
        store_f32<DT>(kd, t + H2, hi);
        reinterpret_cast<uint32_t *>(vd)[t] = vnew;
      }
      s_vn[t] = vnew;
      // the rotated k as raw elements: element e in the 16-bit half e % 2 of s_kn[e / 2]
      reinterpret_cast<uint16_t *>(s_kn)[t] = (uint16_t)bits_dt<DT>(lo);
      reinterpret_cast<uint16_t *>(s_kn)[t + H2] = (uint16_t)bits_dt<DT>(hi);
    }
  }
  __syncthreads();
  if constexpr ((kAttnAbl & 32) != 0) {
    if (t < 2 * H2) { float acc = 0.f;
#pragma unroll
      for (int i = 0; i < NW / 4; ++i) acc += __uint_as_float(kr[i].x ^ vr[i].y);
      reinterpret_cast<float *>(a.out)[t] = acc + __uint_as_float(s_qh[t & (H2 - 1)]); }
    return p;
  }

  // 2. half-row dot products: thread t scores position t % 128 over dims [H2 * (t / 128), + H2)
  //    and stages that half of the position's v row in LDS (zeros where masked / past L)
  {
    const bool ok = mk != 0;
    if (!spec && ok && j != p) {  // long cache: the rows the mask keeps, read now
#pragma unroll
      for (int i = 0; i < NW / 4; ++i) kr[i] = kp[i];
#pragma unroll
      for (int i = 0; i < NW / 4; ++i) vr[i] = vp[i];
    }
    uint32_t kw[NW], vw[NW];
    if (ok && j == p) {
#pragma unroll
      for (int i = 0; i < NW; ++i) { kw[i] = s_kn[half * NW + i]; vw[i] = s_vn[half * NW + i]; }
    } else {
#pragma unroll
      for (int i = 0; i < NW / 4; ++i) {
        kw[4 * i] = kr[i].x; kw[4 * i + 1] = kr[i].y; kw[4 * i + 2] = kr[i].z; kw[4 * i + 3] = kr[i].w;
        vw[4 * i] = vr[i].x; vw[4 * i + 1] = vr[i].y; vw[4 * i + 2] = vr[i].z; vw[4 * i + 3] = vr[i].w;
      }
      if (!ok) {
#pragma unroll
        for (int i = 0; i < NW; ++i) kw[i] = vw[i] = 0u;
      }
    }
    if (half == 0) s_ok[pos_i] = ok ? 1 : 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) S.vw(pos_i, half * NW + i) = vw[i];
    if constexpr ((kAttnAbl & 8) == 0) {
      // both operands are storage-dtype values: v_dot2 of the raw pairs, products exact in fp32
      const uint32_t *qw = &s_qh[half * NW];
      float acc0 = 0.0f, acc1 = 0.0f;  // two chains: even / odd words
#pragma unroll
      for (int i = 0; i < NW; i += 2) {
        acc0 = dot2_dt<DT>(kw[i], qw[i], acc0);
        acc1 = dot2_dt<DT>(kw[i + 1], qw[i + 1], acc1);
      }
      s_sc[half * kAttnChunk + pos_i] = __fadd_rn(acc0, acc1);
    }
  }
  __syncthreads();

  // 3. softmax statistics of the chunk: wave 0, two positions per lane
  if (t < kWave) {
    float s[2], m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pi = 2 * t + r;
      s[r] = s_ok[pi] ? __fmul_rn(__fadd_rn(s_sc[pi], s_sc[kAttnChunk + pi]), a.scale) : -INFINITY;
      m = fmaxf(m, s[r]);
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, kWave));
    float l = 0.0f, e[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      e[r] = s[r] == -INFINITY ? 0.0f : ((kAttnAbl & 16) ? s[r] - m : expf(s[r] - m));
      l += e[r];
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) l += __shfl_xor(l, o, kWave);
    s_p[2 * t] = e[0];
    s_p[2 * t + 1] = e[1];
    if (t == 0) { s_ml[0] = m; s_ml[1] = l; }
  }
  __syncthreads();

  // 4. P V: wave w takes positions [32 w, 32 w + 32), lane group ps of the wave every NSUB-th of
  //    them, lane pl one output pair; the 4 * NSUB slice partials meet in LDS
  {
    const int w = t / kWave, lane = t & (kWave - 1), pl = lane % H2, ps = lane / H2;
    float e0 = 0.0f, e1 = 0.0f;
    if constexpr ((kAttnAbl & 4) == 0) {
      // a fixed trip count, fully unrolled (every LDS read issued before the FMAs wait): rows
      // past L are zero in the v image and s_p
#pragma unroll
      for (int i = 0; i < 32 / NSUB; ++i) {
        const int q = 32 * w + ps + NSUB * i;
        const float pr = s_p[q];
        const uint32_t vv = S.vw(q, pl);
        e0 = fmaf(pr, from_bits<DT>(vv), e0);
        e1 = fmaf(pr, from_bits<DT>(vv >> 16), e1);
      }
    }
    s_pv[(w * NSUB + ps) * D + 2 * pl] = e0;
    s_pv[(w * NSUB + ps) * D + 2 * pl + 1] = e1;
  }
  __syncthreads();
  if (t < D) {
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 4 * NSUB; ++i) acc += s_pv[i * D + t];
    // a full cache (p >= L) has no slot for the new token: HF's StaticLayer.update fails on the
    // out-of-range index_copy_; here the output is NaN (never a silently stale attention)
    if (p >= L) acc = __builtin_nanf("");
    if (a.nsplit == 1) {
      char *ob = reinterpret_cast<char *>(a.out) + ((long long)b * a.os + (long long)hq * D) * ES;
      store_f32<DT>(ob, t, __fdiv_rn(acc, s_ml[1]));
    } else {
      float *pp = a.part + ((((long long)b * a.Hkv + h) * a.nsplit + split) * G + gq) * (D + 2);
      pp[t] = acc;
      if (t == 0) { pp[D] = s_ml[0]; pp[D + 1] = s_ml[1]; }
    }
  }
  return p;
}

}  // namespace qz

// qkv_attn.hip -- a decode token's q/k/v projections (+ the input RMSNorm) AND its attention in ONE
// launch (round 5).
//
// Per Llama layer the decode step ran q/k/v (grouped GEMV, norm in its prologue), then the
// attention launch (k_decode_attn: one workgroup per query head), then o_proj.  The attention
// launch is latency-bound (6.4 us in a graph for ~2 us of arithmetic: the launch, one memory round
// trip for q/k/v and the cache rows, four barriers; profiles/r3_attn_ablation_g1.txt).  Here the
// grouped GEMV's workgroups store their rows write-through (sc1) and count them per head with
// agent-scope atomics; the LAST workgroup to store a query head's rows runs that head's attention
// (attn_core.h, bit-identical arithmetic, q/k/v read at agent scope) in the LDS its decode used.
//
// Visibility: the q / k / v rows live in UNCACHED device memory (the caller's buffers, e.g.
// core._qkv_scratch: hipDeviceMallocUncached).  In cached (hipMalloc) memory the readers were served
// lines of the PREVIOUS call's rows at the same addresses -- behind write-through stores, agent-scope
// loads and even an agent-scope acquire -- with three workgroups per CU (the guide's measured sc1
// hand-offs hold for one per CU); uncached lines cannot go stale.  The stores stay write-through and
// the loads agent-scope, so the protocol does not depend on the memory type beyond that.
//
// Ordering and progress: the grid is laid out k, v, q (segments in that order), so every k and v
// workgroup is dispatched before any q workgroup.  A query head's attention needs its kv head's k
// and v rows too: the q workgroup that completes the head waits (bounded, s_sleep) for the kv
// head's counter -- k/v workgroups never wait on anything, and they were dispatched first, so the
// wait ends; if it ever gave up, a status word is set (the host can read it) instead of hanging.
// Each head's counter expects D / rows-per-block q arrivals; each kv head's 2 D / rows-per-block.
// The last head to finish advances the cache position and zeroes every counter for the next call
// (HIP-graph replays reuse the same words).  Outputs equal the grouped launch + qz_decode_attention
// bit for bit (tests/test_gpu_qkv_attention.py).
#include "gemv_core.h"
#include "attn_core.h"

namespace qz {

constexpr int kQaLine = 32;                 // counter words, one 128-B line each
constexpr unsigned kQaSpinLimit = 1u << 20;

struct QkvAttnArgs {
  DecodeAttnArgs a;
  unsigned *cnt;            // [Hq] head counters, [Hkv] kv-head counters, done, status (one line each)
  int Hq;
  int seg_q;                // segment index of q in the grid (k = 0, v = 1, q = 2)
  int rows_per_block;
  unsigned q_expected, kv_expected;
};

__device__ __forceinline__ unsigned qa_add(unsigned *w) {
  return __hip_atomic_fetch_add((gu32_t *)w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned qa_load(const unsigned *w) {
  return __hip_atomic_load((const gu32_t *)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void qa_store(unsigned *w, unsigned v) {
  __hip_atomic_store((gu32_t *)w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DT, int D> struct QkvAttnTail {
  static constexpr bool kActive = true;
  const QkvAttnArgs *qa;
  int seg;     // 0 k, 1 v, 2 q
  int block;   // row block within the segment

  __device__ void operator()(unsigned char *big, unsigned char *small) const {
    // this wave's write-through row stores have landed; then every wave of the workgroup is past
    // its decode (the byte table and the image are free) and past its stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int s_head;
    unsigned *cnt = qa->cnt;
    const int Hq = qa->Hq, Hkv = qa->a.Hkv, G = qa->a.G;
    const int head = block * qa->rows_per_block / D;   // the q head (seg q) or kv head (seg k / v)
    if (threadIdx.x == 0) {
      int go = -1;
      if (seg == qa->seg_q) {
        if (qa_add(cnt + head * kQaLine) == qa->q_expected - 1u) go = head;
      } else {
        qa_add(cnt + (Hq + head) * kQaLine);
      }
      s_head = go;
    }
    __syncthreads();
    const int hq = s_head;
    if (hq < 0) return;
    // this workgroup stored the head's last q rows: wait for its kv head's k and v rows
    if (threadIdx.x == 0) {
      const unsigned *kvc = cnt + (Hq + hq / G) * kQaLine;
      unsigned n = 0;
      while (qa_load(kvc) < qa->kv_expected && ++n < kQaSpinLimit) __builtin_amdgcn_s_sleep(1);
      if (n >= kQaSpinLimit) qa_store(cnt + (Hq + Hkv + 1) * kQaLine, 1u);
    }
    __syncthreads();
    const AttnLds<D> S{reinterpret_cast<uint32_t *>(big), small};
    const long long p = decode_attn_head<DT, D, true>(qa->a, 0, hq, 0, S);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned *done = cnt + (Hq + Hkv) * kQaLine;
      if (qa_add(done) == (unsigned)Hq - 1u) {
        // every head has read p and every workgroup has counted itself: advance, then re-arm
        if (p < qa->a.L) *qa->a.pos = p + 1;
        for (int i = 0; i < Hq + Hkv; ++i) qa_store(cnt + i * kQaLine, 0u);
        qa_store(done, 0u);
      }
    }
  }
};

template <bool DQ, int DT, int R, bool FS, bool CL, bool NRM, bool TWO, int D>
__global__ __launch_bounds__(256) void k_gemv_4bit_qkv_attn(GemvGroup g, QkvAttnArgs qa) {
  const int b = blockIdx.x;
  int s = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < g.nseg && b >= g.start[i]) s = i;
  s = __builtin_amdgcn_readfirstlane(s);
  const GemvParams seg = g.seg[s];
  const int start = g.start[s];
  const QkvAttnTail<DT, D> tail{&qa, s, b - start};
  gemv_body<DQ, DT, R, 1, 4, FS, CL, false, NRM, false, TWO, false, 0, QkvAttnTail<DT, D>>(seg, b - start, nullptr,
                                                                                        tail);
}

template <bool DQ, int DT, bool CL, bool NRM, int D>
static void launch_qkv_attn(int R, bool two, unsigned blocks, size_t lds, hipStream_t s, const GemvGroup &g,
                            const QkvAttnArgs &qa) {
  if (R == 4) {
    if (two) hipLaunchKernelGGL((k_gemv_4bit_qkv_attn<DQ, DT, 4, true, CL, NRM, true, D>), dim3(blocks), dim3(256), lds, s, g, qa);
    else hipLaunchKernelGGL((k_gemv_4bit_qkv_attn<DQ, DT, 4, true, CL, NRM, false, D>), dim3(blocks), dim3(256), lds, s, g, qa);
  } else {
    if (two) hipLaunchKernelGGL((k_gemv_4bit_qkv_attn<DQ, DT, 2, true, CL, NRM, true, D>), dim3(blocks), dim3(256), lds, s, g, qa);
    else hipLaunchKernelGGL((k_gemv_4bit_qkv_attn<DQ, DT, 2, true, CL, NRM, false, D>), dim3(blocks), dim3(256), lds, s, g, qa);
  }
}

template <bool DQ, int DT, bool CL, int D>
static void launch_qkv_attn_n(bool nrm, int R, bool two, unsigned blocks, size_t lds, hipStream_t s,
                              const GemvGroup &g, const QkvAttnArgs &qa) {
  if (nrm) launch_qkv_attn<DQ, DT, CL, true, D>(R, two, blocks, lds, s, g, qa);
  else launch_qkv_attn<DQ, DT, CL, false, D>(R, two, blocks, lds, s, g, qa);
}

}  // namespace qz

using namespace qz;

extern "C" int qz_qkv_attention_state_words(int Hq, int Hkv) {
  if (Hq <= 0 || Hkv <= 0) return 0;
  return (Hq + Hkv + 2) * kQaLine;
}

extern "C" int qz_gemv_4bit_qkv_attention(const qz_gemv_segment *segs, int K, const void *x, int dtype, int quant_type,
                                          int blocksize, int blocksize2, const float *lut, const void *norm_weight,
                                          float eps, int Hq, int Hkv, int D, int L, const void *cos, const void *sin,
                                          void *k_cache, void *v_cache, const void *mask, long long mask_j,
                                          long long *pos, void *out, float scale, unsigned *state, void *stream) {
  if (!segs || !x || !cos || !sin || !k_cache || !v_cache || !mask || !pos || !out || !state) return QZ_ERR_ARG;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_SHAPE;
  if (Hq <= 0 || Hkv <= 0 || Hq % Hkv != 0 || Hq / Hkv > kAttnMaxG || (D != 64 && D != 128)) return QZ_ERR_SHAPE;
  if (L <= 0 || L > kAttnChunk) return QZ_ERR_SHAPE;   // one key chunk per head (no combine pass)
  if (segs[0].M != Hq * D || segs[1].M != Hkv * D || segs[2].M != Hkv * D) return QZ_ERR_SHAPE;
  if (((uintptr_t)k_cache | (uintptr_t)v_cache) % 16 != 0) return QZ_ERR_SHAPE;
  if (norm_weight && (K % 8 != 0 || K > 16384 || ((uintptr_t)x | (uintptr_t)norm_weight) % 16 != 0))
    return QZ_ERR_SHAPE;
  // the grid in the order k, v, q (k / v workgroups dispatched before any q workgroup)
  const int order[3] = {1, 2, 0};
  GemvGroup g;
  g.nseg = 3;
  const bool cl = exact_codes(quant_type, lut) && dtype == QZ_DT_F16;
  const bool dq = segs[0].qabsmax != nullptr;
  long long total_m = 0;
  for (int i = 0; i < 3; ++i) {
    const qz_gemv_segment &q = segs[order[i]];
    bool v;
    const int st = make_params(q.M, K, x, dtype, q.B, quant_type, blocksize, q.absmax, q.qabsmax, q.absmax2, q.code2,
                               q.offset, blocksize2, q.block_base, lut, q.bias, q.y, &g.seg[i], &v);
    if (st != QZ_OK) return st;
    if ((q.qabsmax != nullptr) != dq || !v || !q.y || (reinterpret_cast<uintptr_t>(q.y) & 3u) ||
        !full_steps(K, blocksize, blocksize2, dq, q.block_base))
      return QZ_ERR_SHAPE;
    set_tables(quant_type & ~QZ_EXACT_CODES, lut, cl, dtype, &g.seg[i]);
    g.seg[i].nw = norm_weight;
    g.seg[i].eps = eps;
    total_m += q.M;
  }
  int R, WK;
  choose_geometry((int)total_m, K, dtype, &R, &WK);
  if (norm_weight && gemv_knobs().norm_r && WK == 1) R = gemv_knobs().norm_r;
  const int rpb = R * 4;
  // whole rows per wave, packed row pairs, and every workgroup's rows inside one head
  if (WK != 1 || (R != 2 && R != 4) || D % rpb != 0) return QZ_ERR_SHAPE;
  int blocks = 0;
  for (int i = 0; i < 3; ++i) {
    g.start[i] = blocks;
    blocks += g.seg[i].M / rpb;
  }
  for (int i = 3; i < kMaxSeg; ++i) g.start[i] = blocks;
  g.total = blocks;
  if (norm_weight && blocks > kNormMaxBlocks) return QZ_ERR_SHAPE;
  QkvAttnArgs qa{};
  DecodeAttnArgs &a = qa.a;
  a.q = segs[0].y; a.k = segs[1].y; a.v = segs[2].y;
  a.qs = (long long)Hq * D; a.ks = a.vs = (long long)Hkv * D;
  a.cos = cos; a.sin = sin; a.cs = 0;
  a.kc = k_cache; a.vc = v_cache;
  a.mask = reinterpret_cast<const unsigned char *>(mask); a.mb = 0; a.mj = mask_j;
  a.pos = pos; a.arrive = nullptr; a.out = out; a.os = (long long)Hq * D; a.part = nullptr;
  a.Hkv = Hkv; a.G = Hq / Hkv; a.L = L; a.nsplit = 1; a.scale = scale;
  qa.cnt = state;
  qa.Hq = Hq;
  qa.seg_q = 2;
  qa.rows_per_block = rpb;
  qa.q_expected = (unsigned)(D / rpb);
  qa.kv_expected = (unsigned)(2 * D / rpb);
  const bool two = two_steps(K, 1, true);
  const size_t small = D == 128 ? (size_t)AttnLds<128>::kSmallBytes : (size_t)AttnLds<64>::kSmallBytes;
  const size_t lds = std::max(norm_weight ? (size_t)K * 2 : (size_t)0, small);
  hipStream_t s = (hipStream_t)stream;
  const unsigned nb = (unsigned)blocks;
  const bool nrm = norm_weight != nullptr;
#define QZ_QA(DQ_, DT_, CL_)                                                                  \
  do {                                                                                        \
    if (D == 128) launch_qkv_attn_n<DQ_, DT_, CL_, 128>(nrm, R, two, nb, lds, s, g, qa);      \
    else launch_qkv_attn_n<DQ_, DT_, CL_, 64>(nrm, R, two, nb, lds, s, g, qa);                \
  } while (0)
  if (dtype == QZ_DT_F16) {
    if (dq) { if (cl) QZ_QA(true, QZ_DT_F16, true); else QZ_QA(true, QZ_DT_F16, false); }
    else { if (cl) QZ_QA(false, QZ_DT_F16, true); else QZ_QA(false, QZ_DT_F16, false); }
  } else {
    if (dq) QZ_QA(true, QZ_DT_BF16, false); else QZ_QA(false, QZ_DT_BF16, false);
  }
#undef QZ_QA
  return QZ_OK;
}

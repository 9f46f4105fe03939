// layer_ops.hip -- the small ops that sit around the 4-bit projections of a
// Llama decoder layer, each as ONE launch (integration.fuse_layer_ops):
//
//  * RMSNorm, which feeds q/k/v and gate/up (modeling_llama.py:62-67).  In eager
//    torch it is 8 launches (cast, pow, mean, add, rsqrt, mul, cast, mul);
//  * rotary position embedding of q and k (modeling_llama.py:130-160), ~10
//    launches (2 x {mul, slice-neg, cat, mul, add});
//  * SiLU(gate) * up, the input of down_proj (modeling_llama.py:175), 2 launches;
//  * residual add + post-attention RMSNorm (LlamaDecoderLayer.forward:317-321).
//
// At batch-1 decode each of those launches moves a few KiB, so the step is
// bound by the fixed cost of a dependent launch (~1.55 us), not
// by bytes.  Numerics follow torch's elementwise opmath exactly: fp32 compute,
// rounding to the storage dtype after every op that torch stores.  The only
// freedom taken is RMSNorm's fp32 sum order (torch's reduction tree is not
// specified), so RMSNorm is checked to a tolerance and rotary bit-exactly.
#include "attn_core.h"

namespace qz {
namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// One 256-thread workgroup per row.  VEC: 16-B loads of 16 / sizeof(elem)
// elements (host-checked alignment, K a multiple of the vector width); the
// second pass re-reads x from L1/L2 (8 KiB per fp16 Llama-3-8B row).
// ADD (LlamaDecoderLayer.forward:317-321, `residual + h` then the norm): the
// normalised value is h' = round(x + r), written to `sum` as the new residual;
// both passes recompute h' from x and r (same rounding, no read-after-write).
template <int DT, bool VEC, bool ADD>
__global__ __launch_bounds__(256) void k_rmsnorm(const void *__restrict__ x, const void *__restrict__ r, int K,
                                                 long long ldx, const void *__restrict__ w, float eps,
                                                 void *__restrict__ y, void *__restrict__ sum, long long ldy) {
  constexpr int ES = DT == QZ_DT_F32 ? 4 : 2;
  constexpr int V = VEC ? 16 / ES : 1;
  __shared__ float s_part[4];
  const long long row = blockIdx.x;
  const char *xr = reinterpret_cast<const char *>(x) + row * ldx * ES;
  const char *rr = ADD ? reinterpret_cast<const char *>(r) + row * ldx * ES : nullptr;
  char *yr = reinterpret_cast<char *>(y) + row * ldy * ES;
  char *sr = ADD ? reinterpret_cast<char *>(sum) + row * ldy * ES : nullptr;
  const int nv = K / V;
  auto value = [&](long long e) {
    if constexpr (ADD) return round_dt<DT>(__fadd_rn(load_f32<DT>(rr, e), load_f32<DT>(xr, e)));
    else return load_f32<DT>(xr, e);
  };

  float ss = 0.0f;
  for (int i = threadIdx.x; i < nv; i += 256) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float h = value((long long)i * V + j);
      ss = __fadd_rn(ss, __fmul_rn(h, h));
    }
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = __fadd_rn(__fadd_rn(s_part[0], s_part[1]), __fadd_rn(s_part[2], s_part[3]));
  // torch MeanOps: sum * (1/N) in fp32; then rsqrt(var + eps)
  const float rs = rsqrtf(__fadd_rn(__fmul_rn(tot, 1.0f / (float)K), eps));
  for (int i = threadIdx.x; i < nv; i += 256) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const long long e = (long long)i * V + j;
      const float v = value(e);
      if constexpr (ADD) store_f32<DT>(sr, e, v);                     // the new residual stream
      const float h = round_dt<DT>(__fmul_rn(v, rs));                  // hidden.to(input_dtype)
      float o = __fmul_rn(load_f32<DT>(w, e), h);                      // weight * hidden (exact for
      asm volatile("" : "+v"(o));                                      // 16-bit dtypes; pinned anyway)
      store_f32<DT>(yr, e, o);
    }
  }
}

// k_rmsnorm's VEC arithmetic for rows of at most 2048 vectors (K <= 16384 at 16 bits, 8192 at fp32):
// every thread's vectors of x (and r) and of the weight are loaded up front and held in registers,
// so a row costs one memory round trip before the reduction instead of one per loop iteration and
// pass (the Llama-3-70B norm, K = 8192: 8.3 us as the loop, profiles/r5_pair_k8192_ab.txt).  Same
// per-thread element order, same reduction, same roundings: bit-identical to k_rmsnorm.
// gridDim.y > 1 (a few rows, e.g. one decode token): workgroup (row, sl) of the gridDim.y slices
// computes the row's whole sum of squares (the same bits in every slice) but loads the weight for,
// and writes, only the chunks c with c % gridDim.y == sl -- one CU streams only ~25 GB/s, so the
// row's output is spread over several CUs
template <int DT, bool ADD>
__global__ __launch_bounds__(256) void k_rmsnorm_held(const void *__restrict__ x, const void *__restrict__ r, int K,
                                                      long long ldx, const void *__restrict__ w, float eps,
                                                      void *__restrict__ y, void *__restrict__ sum, long long ldy) {
  constexpr int ES = DT == QZ_DT_F32 ? 4 : 2;
  constexpr int V = 16 / ES;
  constexpr int NC = 8;
  __shared__ float s_part[4];
  const long long row = blockIdx.x;
  const uint4 *xr = reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(x) + row * ldx * ES);
  const uint4 *rr = ADD ? reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(r) + row * ldx * ES) : nullptr;
  const uint4 *wr = reinterpret_cast<const uint4 *>(w);
  uint4 *yr = reinterpret_cast<uint4 *>(reinterpret_cast<char *>(y) + row * ldy * ES);
  uint4 *sr = ADD ? reinterpret_cast<uint4 *>(reinterpret_cast<char *>(sum) + row * ldy * ES) : nullptr;
  const int nv = K / V;
  uint4 xa[NC], ra[ADD ? NC : 1], wa[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = (int)threadIdx.x + 256 * c;
    if (i < nv) {
      xa[c] = xr[i];
      if constexpr (ADD) ra[c] = rr[i];
    }
  }
  const int nsl = (int)gridDim.y, sl = (int)blockIdx.y;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = (int)threadIdx.x + 256 * c;
    if (i < nv && c % nsl == sl) wa[c] = wr[i];
  }
  float h[NC][V];
  float ss = 0.0f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if ((int)threadIdx.x + 256 * c < nv) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float xe = load_f32<DT>(&xa[c], j);
        if constexpr (ADD) h[c][j] = round_dt<DT>(__fadd_rn(load_f32<DT>(&ra[c < (ADD ? NC : 1) ? c : 0], j), xe));
        else h[c][j] = xe;
        ss = __fadd_rn(ss, __fmul_rn(h[c][j], h[c][j]));
      }
    }
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = __fadd_rn(__fadd_rn(s_part[0], s_part[1]), __fadd_rn(s_part[2], s_part[3]));
  const float rs = rsqrtf(__fadd_rn(__fmul_rn(tot, 1.0f / (float)K), eps));
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = (int)threadIdx.x + 256 * c;
    if (i < nv && c % nsl == sl) {
      uint4 ov, sv;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if constexpr (ADD) store_f32<DT>(&sv, j, h[c][j]);
        const float hn = round_dt<DT>(__fmul_rn(h[c][j], rs));
        float o = __fmul_rn(load_f32<DT>(&wa[c], j), hn);
        asm volatile("" : "+v"(o));
        store_f32<DT>(&ov, j, o);
      }
      if constexpr (ADD) sr[i] = sv;
      yr[i] = ov;
    }
  }
}

struct RopeArgs {
  const void *x[2];
  void *o[2];
  long long xs[2][3], os[2][3];  // (b, h, s) element strides
  int H[2];
  long long rows_q;              // B*Hq*S: rows of q, then B*Hk*S rows of k
  long long pairs;               // total (row, d < D/2) pairs
  const void *cos, *sin;
  long long cb, cs;
  int S, half;
};

// One thread per (row, d) pair: it writes out[d] and out[d + D/2].
template <int DT>
__global__ __launch_bounds__(256) void k_rope_qk(RopeArgs a) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= a.pairs) return;
  const long long row_all = idx / a.half;
  const int d = (int)(idx - row_all * a.half);
  const int t = row_all >= a.rows_q ? 1 : 0;
  const long long row = row_all - (t ? a.rows_q : 0);
  const int H = a.H[t];
  const long long s = row % a.S, bh = row / a.S, h = bh % H, b = bh / H;
  const long long xo = b * a.xs[t][0] + h * a.xs[t][1] + s * a.xs[t][2] + d;
  const long long oo = b * a.os[t][0] + h * a.os[t][1] + s * a.os[t][2] + d;
  const long long co = b * a.cb + s * a.cs + d;
  const float x1 = load_f32<DT>(a.x[t], xo), x2 = load_f32<DT>(a.x[t], xo + a.half);
  const float c1 = load_f32<DT>(a.cos, co), c2 = load_f32<DT>(a.cos, co + a.half);
  const float s1 = load_f32<DT>(a.sin, co), s2 = load_f32<DT>(a.sin, co + a.half);
  // q*cos + cat(-x2, x1)*sin, every torch op rounded to the storage dtype
  const float lo = __fadd_rn(round_dt<DT>(__fmul_rn(x1, c1)), round_dt<DT>(__fmul_rn(-x2, s1)));
  const float hi = __fadd_rn(round_dt<DT>(__fmul_rn(x2, c2)), round_dt<DT>(__fmul_rn(x1, s2)));
  store_f32<DT>(a.o[t], oo, lo);
  store_f32<DT>(a.o[t], oo + a.half, hi);
}

// LlamaMLP's act_fn(gate) * up (modeling_llama.py:175) for hidden_act "silu":
// torch's silu is x / (1 + exp(-x)) in fp32, rounded to the storage dtype, then
// the product of the two stored values rounded again.  One thread per element.
template <int DT>
__global__ __launch_bounds__(256) void k_silu_mul(const void *__restrict__ g, const void *__restrict__ u, long long n,
                                                  void *__restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = load_f32<DT>(g, i);
  const float a = round_dt<DT>(__fdiv_rn(x, __fadd_rn(1.0f, expf(-x))));
  store_f32<DT>(y, i, __fmul_rn(a, load_f32<DT>(u, i)));
}

// k_silu_mul on 16-B vectors (n a multiple of the vector, 16-B aligned operands): the same
// per-element arithmetic, one load of each operand per thread
template <int DT>
__global__ __launch_bounds__(256) void k_silu_mul_vec(const void *__restrict__ g, const void *__restrict__ u,
                                                      long long nvec, void *__restrict__ y) {
  constexpr int V = DT == QZ_DT_F32 ? 4 : 8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  const uint4 gv = reinterpret_cast<const uint4 *>(g)[i];
  const uint4 uv = reinterpret_cast<const uint4 *>(u)[i];
  uint4 ov;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const float x = load_f32<DT>(&gv, j);
    const float a = round_dt<DT>(__fdiv_rn(x, __fadd_rn(1.0f, expf(-x))));
    store_f32<DT>(&ov, j, __fmul_rn(a, load_f32<DT>(&uv, j)));
  }
  reinterpret_cast<uint4 *>(y)[i] = ov;
}

// ---------------------------------------------------------------------------
// Decode attention with a static KV cache: one query head per workgroup, the body in attn_core.h.
// Grid (nsplit, Hq, B).
template <int DT, int D>
__global__ __launch_bounds__(256) void k_decode_attn(DecodeAttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_v[kAttnChunk * (D / 2)];
  __shared__ __attribute__((aligned(16))) unsigned char s_small[AttnLds<D>::kSmallBytes];
  const AttnLds<D> S{s_v, s_small};
  const long long p = decode_attn_head<DT, D>(a, blockIdx.x, blockIdx.y, blockIdx.z, S);
  // the last workgroup to arrive advances the cache position (every workgroup has read p)
  __syncthreads();
  if (threadIdx.x == 0 && (kAttnAbl & 1) == 0) {
    const unsigned int total = gridDim.x * gridDim.y * gridDim.z;
    if (atomicAdd(a.arrive, 1u) == total - 1u) {
      if (p < a.L) *a.pos = p + 1;   // a full cache keeps its position (every later call is NaN too)
      atomicExch(a.arrive, 0u);
    }
  }
}

// nsplit > 1: merge the chunk partials of one (b, kv head) -- out = sum_s e^(m_s - M) o_s /
// sum_s e^(m_s - M) l_s with M = max_s m_s; empty chunks (m_s = -inf) weigh nothing
template <int DT, int D>
__global__ __launch_bounds__(256) void k_decode_attn_combine(DecodeAttnArgs a) {
  constexpr int ES = 2;
  const int h = blockIdx.x, b = blockIdx.y, G = a.G;
  const float *base = a.part + ((long long)b * a.Hkv + h) * a.nsplit * G * (D + 2);
  for (int o = threadIdx.x; o < G * D; o += 256) {
    const int g = o / D, d = o - g * D;
    float M = -INFINITY;
    for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, base[((long long)s * G + g) * (D + 2) + D]);
    float num = 0.0f, den = 0.0f;
    for (int s = 0; s < a.nsplit; ++s) {
      const float *pp = base + ((long long)s * G + g) * (D + 2);
      const float ms = pp[D];
      const float wgt = ms == -INFINITY ? 0.0f : expf(ms - M);
      num = fmaf(wgt, pp[d], num);
      den = fmaf(wgt, pp[D + 1], den);
    }
    char *ob = reinterpret_cast<char *>(a.out) + ((long long)b * a.os + (long long)(h * G + g) * D) * ES;
    store_f32<DT>(ob, d, __fdiv_rn(num, den));
  }
}

template <int DT, int D>
void launch_decode_attn(const DecodeAttnArgs &a, int B, hipStream_t s) {
  hipLaunchKernelGGL((k_decode_attn<DT, D>), dim3(a.nsplit, a.Hkv * a.G, B), dim3(256), 0, s, a);
  if (a.nsplit > 1) hipLaunchKernelGGL((k_decode_attn_combine<DT, D>), dim3(a.Hkv, B), dim3(256), 0, s, a);
}

template <int DT, bool ADD>
void launch_rmsnorm(bool vec, long long rows, const void *x, const void *r, int K, long long ldx, const void *w,
                    float eps, void *y, void *sum, long long ldy, hipStream_t s) {
  const dim3 g((unsigned)rows), b(256);
  constexpr int V = DT == QZ_DT_F32 ? 4 : 8;
  if (vec && K / V <= 256 * 8) {
    // a few rows: each row's chunks over up to 8 workgroups (one per 256-vector chunk)
    const int nc = (K / V + 255) / 256;
    const int nsl = rows * nc <= 64 ? nc : 1;
    hipLaunchKernelGGL((k_rmsnorm_held<DT, ADD>), dim3((unsigned)rows, (unsigned)nsl), b, 0, s, x, r, K, ldx, w, eps,
                       y, sum, ldy);
  }
  else if (vec) hipLaunchKernelGGL((k_rmsnorm<DT, true, ADD>), g, b, 0, s, x, r, K, ldx, w, eps, y, sum, ldy);
  else hipLaunchKernelGGL((k_rmsnorm<DT, false, ADD>), g, b, 0, s, x, r, K, ldx, w, eps, y, sum, ldy);
}

int rmsnorm_entry(const void *x, const void *r, int dtype, long long rows, int K, long long ldx, const void *weight,
                  float eps, void *y, void *sum, long long ldy, void *stream) {
  if (rows < 0 || K < 0) return QZ_ERR_ARG;
  if (rows == 0 || K == 0) return 0;
  if (!x || !weight || !y || ldx < K || ldy < K) return QZ_ERR_ARG;
  if ((r != nullptr) != (sum != nullptr)) return QZ_ERR_ARG;
  if (rows > 0x7FFFFFFFLL) return QZ_ERR_SHAPE;
  const int es = dtype == QZ_DT_F32 ? 4 : 2;
  const int v = 16 / es;
  const bool vec = K % v == 0 && ldx % v == 0 && ldy % v == 0 &&
                   ((uintptr_t)x | (uintptr_t)y | (uintptr_t)weight | (uintptr_t)r | (uintptr_t)sum) % 16 == 0;
  hipStream_t s = (hipStream_t)stream;
  const bool add = r != nullptr;
#define QZ_NORM(DT_)                                                                       \
  (add ? launch_rmsnorm<DT_, true>(vec, rows, x, r, K, ldx, weight, eps, y, sum, ldy, s) \
       : launch_rmsnorm<DT_, false>(vec, rows, x, r, K, ldx, weight, eps, y, sum, ldy, s))
  switch (dtype) {
    case QZ_DT_F16: QZ_NORM(QZ_DT_F16); break;
    case QZ_DT_BF16: QZ_NORM(QZ_DT_BF16); break;
    case QZ_DT_F32: QZ_NORM(QZ_DT_F32); break;
    default: return QZ_ERR_DTYPE;
  }
#undef QZ_NORM
  return (int)hipGetLastError();
}

// ---- decode-step glue of the host model (one launch each instead of the 7-9 small torch kernels
// transformers' LlamaModel.forward issues per step; the Linear4bit layers are not touched) ----
// causal mask of one new token per sequence against a static cache: masking_utils.sdpa_mask with
// causal_mask_function and kv_offset 0 -- kv position j is visible iff j <= q_offset, the cache's
// cumulative length before this token (a device int64, read in-kernel: graph-capturable)
__global__ __launch_bounds__(256) void k_decode_mask(const long long *q_off, long long n, int L,
                                                      unsigned char *mask) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  mask[i] = (long long)(i % L) <= q_off[0] ? 1 : 0;
}

// rotary cos/sin of the step's positions, looked up in [T, D] tables the model's own rotary module
// computed for positions 0..T-1 (the same values, bit for bit); a position outside the table is
// computed here from inv_freq (fp32 product, cosf/sinf, * scale, rounded to the dtype)
struct RopeTableArgs {
  const long long *pos;
  long long pb, ps;                 // position_ids strides (batch, sequence)
  const void *cos_t, *sin_t;        // [T, D]
  const float *inv_freq;            // [D / 2]
  void *cos, *sin;                  // [B, S, D], contiguous
  long long n, T;
  int S, D;
  float scale;
};
template <int DT> __global__ __launch_bounds__(256) void k_rope_table(RopeTableArgs a) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const long long bs = i / a.D;
  const int d = (int)(i - bs * a.D);
  const long long b = bs / a.S, sq = bs - b * a.S;
  const long long p = a.pos[b * a.pb + sq * a.ps];
  if (p >= 0 && p < a.T) {
    if constexpr (DT == QZ_DT_F32) {
      reinterpret_cast<float *>(a.cos)[i] = reinterpret_cast<const float *>(a.cos_t)[p * a.D + d];
      reinterpret_cast<float *>(a.sin)[i] = reinterpret_cast<const float *>(a.sin_t)[p * a.D + d];
    } else {
      reinterpret_cast<uint16_t *>(a.cos)[i] = reinterpret_cast<const uint16_t *>(a.cos_t)[p * a.D + d];
      reinterpret_cast<uint16_t *>(a.sin)[i] = reinterpret_cast<const uint16_t *>(a.sin_t)[p * a.D + d];
    }
    return;
  }
  const float f = __fmul_rn(a.inv_freq[d % (a.D / 2)], (float)p);
  store_f32<DT>(a.cos, i, __fmul_rn(cosf(f), a.scale));
  store_f32<DT>(a.sin, i, __fmul_rn(sinf(f), a.scale));
}

// greedy pick + feedback of a decode step (bench.py's loop: next = argmax(logits[b]);
// hist[b, *pos] = next; tok[b] = next; *pos += 1) in two launches: a partial pass in which each
// workgroup reduces 2048 logits of a row (one 16-B vector per thread: one CU reads only ~25 GB/s, a
// single workgroup over 128256 logits took 21 us), then one workgroup reduces the partials and
// writes the feedback.  torch.argmax's order: the largest value, NaN above every number, the first
// index among equals (a total order on (value, index), so any reduction tree gives the same pick)
constexpr int kGreedyChunk = 2048;
__device__ __forceinline__ bool greedy_better(float v, long long i, float w, long long j) {
  const bool vn = v != v, wn = w != w;
  if (vn || wn) return vn && (!wn || i < j);
  return v > w || (v == w && i < j);
}
// (best, bi) over the workgroup (256 threads) -> thread 0; bi == none marks "no element"
__device__ __forceinline__ void greedy_reduce_wg(float &best, long long &bi, long long none, float *s_v,
                                                 long long *s_i) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int o = 32; o > 0; o >>= 1) {
    const float w = __shfl_xor(best, o);
    const long long j = __shfl_xor(bi, o);
    if (j != none && (bi == none || greedy_better(w, j, best, bi))) { best = w; bi = j; }
  }
  if (lane == 0) { s_v[wave] = best; s_i[wave] = bi; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (s_i[w] != none && (bi == none || greedy_better(s_v[w], s_i[w], best, bi))) { best = s_v[w]; bi = s_i[w]; }
  }
  __syncthreads();
}
template <int DT>
__global__ __launch_bounds__(256) void k_greedy_partial(const void *logits, long long row, long long V, int nb,
                                                        float *pv, long long *pi, bool vec) {
  __shared__ float s_v[4];
  __shared__ long long s_i[4];
  const int tid = threadIdx.x, b = blockIdx.y;
  const long long base = (long long)blockIdx.x * kGreedyChunk;
  const long long end = base + kGreedyChunk < V ? base + kGreedyChunk : V;
  const void *lr = reinterpret_cast<const unsigned char *>(logits) + (size_t)b * row * (DT == QZ_DT_F32 ? 4 : 2);
  float best = -__builtin_inff();
  long long bi = V;   // no element yet
  constexpr int E = DT == QZ_DT_F32 ? 4 : 8;   // elements per 16-B vector
  if (vec) {
    // 2048 / E vectors per workgroup: at most 256 / (8 / E) per thread, in increasing index order
    typedef uint32_t w4_t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int u = 0; u < kGreedyChunk / E / 256; ++u) {
      const long long i0 = base + (long long)(tid + 256 * u) * E;
      if (i0 < end) {
        const w4_t r = *reinterpret_cast<const w4_t *>(reinterpret_cast<const unsigned char *>(lr) +
                                                        i0 * (DT == QZ_DT_F32 ? 4 : 2));
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint32_t w = r[DT == QZ_DT_F32 ? e : e >> 1];
          float v;
          if constexpr (DT == QZ_DT_F32) v = __uint_as_float(w);
          else if constexpr (DT == QZ_DT_F16) v = __half2float(__ushort_as_half((unsigned short)((e & 1) ? w >> 16 : w & 0xFFFFu)));
          else v = __uint_as_float((e & 1) ? (w & 0xFFFF0000u) : (w << 16));
          if (v > best || (v != v && best == best) || bi == V) { best = v; bi = i0 + e; }
        }
      }
    }
  } else {
    for (long long i = base + tid; i < end; i += 256) {
      const float v = load_f32<DT>(lr, i);
      if (v > best || (v != v && best == best) || bi == V) { best = v; bi = i; }
    }
  }
  greedy_reduce_wg(best, bi, V, s_v, s_i);
  if (tid == 0) {
    pv[(size_t)b * nb + blockIdx.x] = best;
    pi[(size_t)b * nb + blockIdx.x] = bi;
  }
}
__global__ __launch_bounds__(256) void k_greedy_final(int B, long long V, int nb, const float *pv,
                                                      const long long *pi, long long *hist, long long hist_row,
                                                      long long hist_len, long long *pos, long long *tok) {
  __shared__ float s_v[4];
  __shared__ long long s_i[4];
  const int tid = threadIdx.x;
  const long long p = *pos;
  for (int b = 0; b < B; ++b) {
    float best = -__builtin_inff();
    long long bi = V;
    for (int c = tid; c < nb; c += 256) {
      const float v = pv[(size_t)b * nb + c];
      const long long i = pi[(size_t)b * nb + c];
      if (i != V && (bi == V || greedy_better(v, i, best, bi))) { best = v; bi = i; }
    }
    greedy_reduce_wg(best, bi, V, s_v, s_i);
    if (tid == 0) {
      // a position past the history (a graph replayed more often than hist has columns) writes
      // nothing there: the token and the position still advance
      if (p >= 0 && p < hist_len) hist[(size_t)b * hist_row + p] = bi;
      tok[b] = bi;
    }
  }
  if (tid == 0) *pos = p + 1;
}

// ---- the host model's fp16 / bf16 lm_head for one decode token (not 4-bit: transformers keeps it
// in the model dtype): y[m] = sum_k W[m, k] x[k], fp32 accumulation, rounded once.  Each wave owns
// R rows; lane l reads the 16-B chunks l, l + 64, ... of a row (KCH = K / 512 of them) with
// non-temporal loads, all R * KCH in flight before the first dot product; x's chunks stay in
// registers; a butterfly over the 64 lanes ends each row ----
template <int DT, int KCH, int R>
__global__ __launch_bounds__(256) void k_gemv_dense(const void *__restrict__ W, const void *__restrict__ x, int M,
                                                    int K, void *__restrict__ y) {
  typedef uint32_t w4_t __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long row0 = ((long long)blockIdx.x * 4 + wave) * R;
  if (row0 >= M) return;
  w4_t xv[KCH];
#pragma unroll
  for (int j = 0; j < KCH; ++j) xv[j] = reinterpret_cast<const w4_t *>(x)[lane + 64 * j];
  w4_t wv[R][KCH];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long long row = row0 + r < M ? row0 + r : M - 1;
    const w4_t *wr = reinterpret_cast<const w4_t *>(reinterpret_cast<const uint16_t *>(W) + row * K);
#pragma unroll
    for (int j = 0; j < KCH; ++j) wv[r][j] = __builtin_nontemporal_load(wr + lane + 64 * j);
  }
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float a = 0.0f;
#pragma unroll
    for (int j = 0; j < KCH; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) a = dot2_dt<DT>(wv[r][j][e], xv[j][e], a);
    acc[r] = a;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[r] += __shfl_xor(acc[r], o);
  }
  if (lane < R && row0 + lane < M) {
    float v = acc[0];
#pragma unroll
    for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
    store_f32<DT>(y, row0 + lane, v);
  }
}

}  // namespace
}  // namespace qz

using namespace qz;

extern "C" int qz_rmsnorm(const void *x, int dtype, long long rows, int K, long long ldx, const void *weight,
                          float eps, void *y, long long ldy, void *stream) {
  return rmsnorm_entry(x, nullptr, dtype, rows, K, ldx, weight, eps, y, nullptr, ldy, stream);
}

extern "C" int qz_add_rmsnorm(const void *x, const void *residual, int dtype, long long rows, int K, long long ldx,
                              const void *weight, float eps, void *sum, void *y, long long ldy, void *stream) {
  if (!residual || !sum) return QZ_ERR_ARG;
  return rmsnorm_entry(x, residual, dtype, rows, K, ldx, weight, eps, y, sum, ldy, stream);
}

extern "C" int qz_rope_qk(int dtype, int B, int S, int D, const void *q, int Hq, const long long *q_str, void *q_out,
                          const long long *qo_str, const void *k, int Hk, const long long *k_str, void *k_out,
                          const long long *ko_str, const void *cos, const void *sin, const long long *cs_str,
                          void *stream) {
  if (B < 0 || S < 0 || D < 0 || Hq < 0 || Hk < 0) return QZ_ERR_ARG;
  if ((D & 1) != 0) return QZ_ERR_SHAPE;
  if (B == 0 || S == 0 || D == 0 || Hq + Hk == 0) return 0;
  if (!q_str || !qo_str || !k_str || !ko_str || !cs_str || !cos || !sin) return QZ_ERR_ARG;
  if ((Hq > 0 && (!q || !q_out)) || (Hk > 0 && (!k || !k_out))) return QZ_ERR_ARG;
  RopeArgs a{};
  a.x[0] = q; a.x[1] = k; a.o[0] = q_out; a.o[1] = k_out;
  for (int i = 0; i < 3; ++i) {
    a.xs[0][i] = q_str[i]; a.os[0][i] = qo_str[i]; a.xs[1][i] = k_str[i]; a.os[1][i] = ko_str[i];
  }
  a.H[0] = Hq; a.H[1] = Hk;
  a.rows_q = (long long)B * Hq * S;
  a.half = D / 2;
  a.pairs = (a.rows_q + (long long)B * Hk * S) * a.half;
  a.cos = cos; a.sin = sin; a.cb = cs_str[0]; a.cs = cs_str[1]; a.S = S;
  const long long blocks = (a.pairs + 255) / 256;
  if (blocks > 0x7FFFFFFFLL) return QZ_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case QZ_DT_F16: hipLaunchKernelGGL((k_rope_qk<QZ_DT_F16>), dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case QZ_DT_BF16: hipLaunchKernelGGL((k_rope_qk<QZ_DT_BF16>), dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case QZ_DT_F32: hipLaunchKernelGGL((k_rope_qk<QZ_DT_F32>), dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    default: return QZ_ERR_DTYPE;
  }
  return (int)hipGetLastError();
}

extern "C" int qz_silu_mul(const void *gate, const void *up, int dtype, long long n, void *y, void *stream) {
  if (n < 0) return QZ_ERR_ARG;
  if (n == 0) return 0;
  if (!gate || !up || !y) return QZ_ERR_ARG;
  const long long blocks = (n + 255) / 256;
  if (blocks > 0x7FFFFFFFLL) return QZ_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int v = dtype == QZ_DT_F32 ? 4 : 8;
  if (n % v == 0 && ((uintptr_t)gate | (uintptr_t)up | (uintptr_t)y) % 16 == 0) {
    const long long nvec = n / v;
    const dim3 gv((unsigned)((nvec + 255) / 256)), bv(256);
    switch (dtype) {
      case QZ_DT_F16: hipLaunchKernelGGL((k_silu_mul_vec<QZ_DT_F16>), gv, bv, 0, s, gate, up, nvec, y); break;
      case QZ_DT_BF16: hipLaunchKernelGGL((k_silu_mul_vec<QZ_DT_BF16>), gv, bv, 0, s, gate, up, nvec, y); break;
      case QZ_DT_F32: hipLaunchKernelGGL((k_silu_mul_vec<QZ_DT_F32>), gv, bv, 0, s, gate, up, nvec, y); break;
      default: return QZ_ERR_DTYPE;
    }
    return (int)hipGetLastError();
  }
  const dim3 grid((unsigned)blocks), blk(256);
  switch (dtype) {
    case QZ_DT_F16: hipLaunchKernelGGL((k_silu_mul<QZ_DT_F16>), grid, blk, 0, s, gate, up, n, y); break;
    case QZ_DT_BF16: hipLaunchKernelGGL((k_silu_mul<QZ_DT_BF16>), grid, blk, 0, s, gate, up, n, y); break;
    case QZ_DT_F32: hipLaunchKernelGGL((k_silu_mul<QZ_DT_F32>), grid, blk, 0, s, gate, up, n, y); break;
    default: return QZ_ERR_DTYPE;
  }
  return (int)hipGetLastError();
}

extern "C" int qz_decode_attention(int dtype, int B, int Hq, int Hkv, int D, int L, const void *q, long long q_row,
                                   const void *k, long long k_row, const void *v, long long v_row, const void *cos,
                                   const void *sin, long long cs_row, void *k_cache, void *v_cache,
                                   const void *mask, long long mask_b, long long mask_j, long long *pos,
                                   unsigned int *arrive, void *out, long long out_row, float *work, float scale,
                                   void *stream) {
  if (B < 0 || Hq < 0 || Hkv < 0 || D < 0 || L < 0) return QZ_ERR_ARG;
  if (B == 0 || Hq == 0) return 0;
  if (Hkv == 0 || Hq % Hkv != 0 || Hq / Hkv > kAttnMaxG || (D != 64 && D != 128) || L == 0) return QZ_ERR_SHAPE;
  if (B > 65535 || Hq > 65535) return QZ_ERR_SHAPE;
  if (!q || !k || !v || !cos || !sin || !k_cache || !v_cache || !mask || !pos || !arrive || !out) return QZ_ERR_ARG;
  if (q_row < (long long)Hq * D || k_row < (long long)Hkv * D || v_row < (long long)Hkv * D || cs_row < 0 ||
      out_row < (long long)Hq * D)
    return QZ_ERR_ARG;
  // 16-B row loads of the caches; 4-B words of v
  if (((uintptr_t)k_cache | (uintptr_t)v_cache) % 16 != 0 || ((uintptr_t)v % 4) != 0 || (v_row % 2) != 0)
    return QZ_ERR_ARG;
  DecodeAttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.qs = q_row; a.ks = k_row; a.vs = v_row;
  a.cos = cos; a.sin = sin; a.cs = cs_row;
  a.kc = k_cache; a.vc = v_cache;
  a.mask = reinterpret_cast<const unsigned char *>(mask); a.mb = mask_b; a.mj = mask_j;
  a.pos = pos; a.arrive = arrive; a.out = out; a.os = out_row; a.part = work;
  a.Hkv = Hkv; a.G = Hq / Hkv; a.L = L; a.nsplit = (L + kAttnChunk - 1) / kAttnChunk; a.scale = scale;
  if (a.nsplit > 1 && !work) return QZ_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case QZ_DT_F16: D == 64 ? launch_decode_attn<QZ_DT_F16, 64>(a, B, s) : launch_decode_attn<QZ_DT_F16, 128>(a, B, s); break;
    case QZ_DT_BF16: D == 64 ? launch_decode_attn<QZ_DT_BF16, 64>(a, B, s) : launch_decode_attn<QZ_DT_BF16, 128>(a, B, s); break;
    default: return QZ_ERR_DTYPE;
  }
  return (int)hipGetLastError();
}

extern "C" int qz_decode_mask(const long long *q_offset, int B, int L, void *mask, void *stream) {
  if (B < 0 || L < 0) return QZ_ERR_ARG;
  if (B == 0 || L == 0) return 0;
  if (!q_offset || !mask) return QZ_ERR_ARG;
  const long long n = (long long)B * L, blocks = (n + 255) / 256;
  if (blocks > 0x7FFFFFFFLL) return QZ_ERR_SHAPE;
  hipLaunchKernelGGL(k_decode_mask, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, q_offset, n, L,
                     reinterpret_cast<unsigned char *>(mask));
  return (int)hipGetLastError();
}

extern "C" int qz_rope_table(int dtype, int B, int S, int D, const long long *pos, long long pos_b, long long pos_s,
                             const void *cos_table, const void *sin_table, long long T, const float *inv_freq,
                             float scale, void *cos, void *sin, void *stream) {
  if (B < 0 || S < 0 || D < 0 || T < 0) return QZ_ERR_ARG;
  if ((D & 1) != 0) return QZ_ERR_SHAPE;
  if (B == 0 || S == 0 || D == 0) return 0;
  if (!pos || !inv_freq || !cos || !sin || (T > 0 && (!cos_table || !sin_table))) return QZ_ERR_ARG;
  RopeTableArgs a{};
  a.pos = pos; a.pb = pos_b; a.ps = pos_s;
  a.cos_t = cos_table; a.sin_t = sin_table; a.inv_freq = inv_freq;
  a.cos = cos; a.sin = sin;
  a.n = (long long)B * S * D; a.T = T; a.S = S; a.D = D; a.scale = scale;
  const long long blocks = (a.n + 255) / 256;
  if (blocks > 0x7FFFFFFFLL) return QZ_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case QZ_DT_F16: hipLaunchKernelGGL((k_rope_table<QZ_DT_F16>), dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case QZ_DT_BF16: hipLaunchKernelGGL((k_rope_table<QZ_DT_BF16>), dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case QZ_DT_F32: hipLaunchKernelGGL((k_rope_table<QZ_DT_F32>), dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    default: return QZ_ERR_DTYPE;
  }
  return (int)hipGetLastError();
}

extern "C" long long qz_greedy_step_work_bytes(int B, long long V) {
  if (B <= 0 || V <= 0) return 0;
  return (long long)B * ((V + kGreedyChunk - 1) / kGreedyChunk) * 16;
}

extern "C" int qz_greedy_step(const void *logits, int dtype, int B, long long V, long long row, long long *hist,
                              long long hist_row, long long hist_len, long long *pos, long long *tok, void *work,
                              void *stream) {
  if (B < 0 || V < 0 || row < 0 || hist_row < 0 || hist_len < 0) return QZ_ERR_ARG;
  if (B == 0) return 0;
  if (V == 0 || !logits || !hist || !pos || !tok || !work || row < V || (B > 1 && hist_row < hist_len))
    return QZ_ERR_ARG;
  const long long nbl = (V + kGreedyChunk - 1) / kGreedyChunk;
  if (nbl > 0x7FFFFFFFLL || B > 65535) return QZ_ERR_SHAPE;
  const int nb = (int)nbl;
  float *pv = reinterpret_cast<float *>(work);
  long long *pi = reinterpret_cast<long long *>(reinterpret_cast<unsigned char *>(work) + (size_t)B * nb * 8);
  hipStream_t s = (hipStream_t)stream;
  const int esz = dtype == QZ_DT_F32 ? 4 : 2;
  const bool vec = (V * esz) % 16 == 0 && (row * esz) % 16 == 0 && (uintptr_t)logits % 16 == 0;
  const dim3 g((unsigned)nb, (unsigned)B);
  switch (dtype) {
    case QZ_DT_F16: hipLaunchKernelGGL((k_greedy_partial<QZ_DT_F16>), g, dim3(256), 0, s, logits, row, V, nb, pv, pi, vec); break;
    case QZ_DT_BF16: hipLaunchKernelGGL((k_greedy_partial<QZ_DT_BF16>), g, dim3(256), 0, s, logits, row, V, nb, pv, pi, vec); break;
    case QZ_DT_F32: hipLaunchKernelGGL((k_greedy_partial<QZ_DT_F32>), g, dim3(256), 0, s, logits, row, V, nb, pv, pi, vec); break;
    default: return QZ_ERR_DTYPE;
  }
  hipLaunchKernelGGL(k_greedy_final, dim3(1), dim3(256), 0, s, B, V, nb, pv, pi, hist, hist_row, hist_len, pos, tok);
  return (int)hipGetLastError();
}

extern "C" int qz_gemv_dense(int M, int K, const void *x, int dtype, const void *W, void *y, void *stream) {
  if (M < 0 || K < 0) return QZ_ERR_ARG;
  if (M == 0) return 0;
  if (!x || !W || !y) return QZ_ERR_ARG;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_DTYPE;
  if ((K != 4096 && K != 8192) || ((uintptr_t)x | (uintptr_t)W) % 16 != 0) return QZ_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  if (K == 4096) {
    const dim3 g((unsigned)((M + 15) / 16));
    if (dtype == QZ_DT_F16) hipLaunchKernelGGL((k_gemv_dense<QZ_DT_F16, 8, 4>), g, dim3(256), 0, s, W, x, M, K, y);
    else hipLaunchKernelGGL((k_gemv_dense<QZ_DT_BF16, 8, 4>), g, dim3(256), 0, s, W, x, M, K, y);
  } else {
    const dim3 g((unsigned)((M + 7) / 8));
    if (dtype == QZ_DT_F16) hipLaunchKernelGGL((k_gemv_dense<QZ_DT_F16, 16, 2>), g, dim3(256), 0, s, W, x, M, K, y);
    else hipLaunchKernelGGL((k_gemv_dense<QZ_DT_BF16, 16, 2>), g, dim3(256), 0, s, W, x, M, K, y);
  }
  return (int)hipGetLastError();
}

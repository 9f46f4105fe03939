// chain.hip -- the MLP half of a Llama decoder layer as ONE persistent launch (round 5):
//
//   h1  = residual + o_proj(x_attn)                         o_proj + the first residual add
//   act = act_fn(gate_proj(rms(h1))) * up_proj(rms(h1))     post-attention RMSNorm, gate/up, SiLU
//   out = h1 + down_proj(act)                               down_proj + the second residual add
//
// (modeling_llama.py:316-322 with the Linear4bit layers of the reference path, modules.py:124-151
// -> kernels.cu:1061-1219).  Before, these were three dependent launches (o_proj + residual, the
// persistent gate/up pair with the norm in its prologue and SiLU in its epilogue, down_proj +
// residual), each paying a launch boundary, its ramp and its drain.  Here one grid of one 8-wave
// workgroup per CU runs the three stages back to back; the two all-to-all dependencies (every
// gate/up row needs all of h1, every down row all of act) are grid barriers, and each wave issues
// its next stage's first weight loads BEFORE it waits at the barrier (weights do not depend on
// the activations), so HBM keeps streaming across the stage boundary.
//
// Every output is bit-identical to the three-launch form: each wave owns whole rows (WK = 1),
// lane l always owns bytes [16 l, 16 l + 16) of each 1-KiB K-step, steps are accumulated in order
// with the same fma chain and reduced by the same DPP tree (gemv_core.h), the norm is k_rmsnorm's
// exact summation order, and the SiLU product is k_silu_mul's arithmetic.
//
// Inter-workgroup hand-off (MI355X_MICROARCH.md, visibility: "Valid forms", first table row;
// cdna_hip_programming.md Guideline 16): the handed-off vectors (h1, act) are stored write-through
// (sc1) by the workgroup that computes them; every storing wave drains its stores
// (s_waitcnt vmcnt(0)) before the workgroup barrier, after which ONE lane adds to the barrier's
// counter (agent-scope atomic, sharded 8 ways over 128-B lines); one wave polls every shard with
// relaxed agent (sc1) loads, with s_sleep, and EVERY load of handed-off bytes is an sc1 load
// (buffer loads with aux = sc1), so no acquire fence is needed.  The counters never reset: launch e
// (the epoch word, advanced by the last workgroup to finish, read at entry) waits for (e + 1) x P
// arrivals, so the launch is HIP-graph capturable with fixed arguments.  Every spin is bounded: a
// workgroup that gives up sets the status word and still arrives everywhere, so the grid always
// drains (the outputs of that call are then invalid; qz_mlp_chain_status reports it).
#include "gemv_core.h"

#include <type_traits>

namespace qz {

typedef __attribute__((address_space(1))) unsigned gu32_t;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;

// sync state: int32 words, each on its own 128-B line; caller-allocated, zeroed once
constexpr int kChLine = 32;
constexpr int kChEpoch = 0;                         // launches completed
constexpr int kChDone = kChLine;                    // finishing ticket of the current launch
constexpr int kChBar = 2 * kChLine;                 // [barrier b][shard s] at kChBar + (8 b + s) * kChLine
constexpr int kChStatus = kChBar + 16 * kChLine;    // nonzero: a spin gave up
constexpr int kChWords = kChStatus + kChLine;
constexpr int kChNW = 8;                            // waves per workgroup (one workgroup per CU)
constexpr unsigned kChSpinLimit = 1u << 18;         // polls (each >= one sc1 round trip + s_sleep)
constexpr int kChMaxK = 8192;                       // the normed stage's K (norm image + chunk registers)
constexpr int kChMaxI = 28672;                      // down_proj's K (its LDS image of act)

__device__ __forceinline__ unsigned ld_agent(const unsigned *p) {
  return __hip_atomic_load((const gu32_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 B of a handed-off vector, write-through coherent (buffer load, aux = sc1)
__device__ __forceinline__ u32x4 ld16_sc1(const void *base, uint32_t byte_off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)0x7FFFFFF0, 0x00020000);
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16));
}
__device__ __forceinline__ void st16_sc1(void *base, uint32_t byte_off, const u32x4 &v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)0x7FFFFFF0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r,
                                         (int)byte_off, 0, 16);
}

// a 16-bit value of DT (its bits) as fp32
template <int DT> __device__ __forceinline__ float bits16_f32(uint32_t b) {
  if constexpr (DT == QZ_DT_F16) return __half2float(__ushort_as_half((unsigned short)b));
  else return __uint_as_float(b << 16);
}

// The chain's arguments: the four projections (x / y / res of each set by the host: o.x = the
// attention output, o.res = the residual stream, o.y = h1; gate.y = up.y = act; down.x = act,
// down.res = h1, down.y = out), the norm, and the sync state.
struct ChainArgs {
  GemvParams o, gate, up, down;
  const void *nw;
  float eps;
  unsigned *state;
};

// What a stage's step loop reads, laundered into SGPRs once per stage (only these: the whole
// GemvParams of three stages would not fit the SGPR file); the epilogue reads its few fields
// (y, res, bias, out_scale) from the kernel arguments where it needs them.
struct StageParams {
  const unsigned char *B;
  const void *x;
  const unsigned char *qabsmax;
  const float *absmax;   // absmax2 with double quant, else the fp32 absmax
  uint32_t block_base;
  int M, K, bs_log2, bs2_log2;
};
template <bool DQ> __device__ __forceinline__ StageParams load_stage(const GemvParams &in) {
  StageParams p;
  p.B = keep_sp(in.B);
  p.x = keep_sp(in.x);
  p.qabsmax = DQ ? keep_sp(in.sc.qabsmax) : nullptr;
  p.absmax = keep_sp(DQ ? in.sc.absmax2 : in.sc.absmax);
  p.block_base = keep_s((uint32_t)in.block_base);
  p.M = keep_s(in.M);
  p.K = keep_s(in.K);
  p.bs_log2 = keep_s(in.bs_log2);
  p.bs2_log2 = keep_s(in.bs2_log2);
  return p;
}

// One K-step of R rows (full-step form: the host checked K % 2048 == 0 and the scale geometry).
// XS: where x comes from -- 0 plain global loads (written before this launch), 1 the workgroup's LDS
// image (the normalised h1), 2 handed-off global data (act), read with sc1 loads.
template <bool DQ, int R, int XS> struct ChainLoads {
  u32x4 wv[R];
  uint32_t q[R];
  float a[R];
  uint32_t xr[16];
  uint32_t boff;

  __device__ __forceinline__ void issue_w(const StageParams &p, int row0, int s, int lane) {
    boff = ((uint32_t)s << 10) + ((uint32_t)lane << 4);
    const uint32_t row_bytes = (uint32_t)p.K >> 1;
    const uint32_t lb = (2u * boff) >> p.bs_log2;
    const uint32_t sb = ((uint32_t)s << 11) >> p.bs_log2;
    const uint32_t bpr = (uint32_t)p.K >> p.bs_log2;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t row = (uint32_t)min(row0 + r, p.M - 1);
      wv[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p.B + (size_t)row * row_bytes + boff));
      const uint32_t rb = p.block_base + row * bpr;
      if constexpr (DQ) {
        q[r] = (p.qabsmax + rb)[lb];
        typedef const __attribute__((address_space(4))) float *cfp;
        a[r] = ((cfp)p.absmax)[(rb + sb) >> p.bs2_log2];
      } else {
        a[r] = (p.absmax + rb)[lb];
      }
    }
  }
  // the lane's 32 activations of the step (64 B), fp16/bf16
  __device__ __forceinline__ void issue_x(const StageParams &p) {
    if constexpr (XS == 0) {
      const u32x4 *px = reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(p.x) + 2u * 2u * boff);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 v = px[i];
        xr[4 * i] = v.x; xr[4 * i + 1] = v.y; xr[4 * i + 2] = v.z; xr[4 * i + 3] = v.w;
      }
    } else if constexpr (XS == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 v = ld16_sc1(p.x, 4u * boff + 16u * (uint32_t)i);
        xr[4 * i] = v.x; xr[4 * i + 1] = v.y; xr[4 * i + 2] = v.z; xr[4 * i + 3] = v.w;
      }
    }
  }
  __device__ __forceinline__ void issue(const StageParams &p, int row0, int s, int lane) {
    if constexpr (XS != 1) {   // x first, then the rows (vmcnt retires in issue order)
      boff = ((uint32_t)s << 10) + ((uint32_t)lane << 4);
      issue_x(p);
    }
    issue_w(p, row0, s, lane);
  }
};

// Arrive at barrier b (after every wave of the workgroup drained its stores and reached the
// workgroup barrier): one agent-scope add to this workgroup's shard.
__device__ __forceinline__ void chain_arrive(unsigned *st, int b) {
  __hip_atomic_fetch_add((gu32_t *)(st + kChBar + (8 * b + (int)(blockIdx.x & 7)) * kChLine), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}
// The sum of barrier b's 8 shards (lanes 0..7 load one each; the total is wave-uniform)
__device__ __forceinline__ unsigned chain_poll(const unsigned *st, int b, int lane) {
  unsigned v = 0;
  if (lane < 8) v = ld_agent(st + kChBar + (8 * b + lane) * kChLine);
  v += __shfl_xor(v, 1, 8);
  v += __shfl_xor(v, 2, 8);
  v += __shfl_xor(v, 4, 8);
  return __builtin_amdgcn_readfirstlane(v);
}

// Diagnostic stage stamps (measurement-only builds: diag_stamps.hip defines QZ_STAMPS and
// instantiates STAMP = 1; the product library compiles none of this): wave 0 of every workgroup
// records s_memrealtime (100 MHz, chip-wide) at fixed points, stored at the end by lane 0.
#ifdef QZ_STAMPS
__device__ unsigned long long *g_qz_chain_stamp;
#define CH_STAMP(k)                                                                              \
  do {                                                                                           \
    if constexpr (STAMP != 0) {                                                                  \
      if (wave == 0) {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ch_st_[k])::"memory");   \
        __builtin_amdgcn_sched_barrier(0);                                                       \
      }                                                                                          \
    }                                                                                            \
  } while (0)
#define CH_STAMP_FLUSH()                                                                         \
  do {                                                                                           \
    if constexpr (STAMP != 0) {                                                                  \
      if (threadIdx.x == 0)                                                                      \
        for (int k_ = 0; k_ < 12; ++k_) g_qz_chain_stamp[(size_t)blockIdx.x * 12 + k_] = ch_st_[k_]; \
    }                                                                                            \
  } while (0)
#else
#define CH_STAMP(k) do {} while (0)
#define CH_STAMP_FLUSH() do {} while (0)
#endif

template <bool DQ, int DT, bool CL, int R, int STAMP = 0>
__global__ __launch_bounds__(kChNW * 64, 1) void k_mlp_chain(ChainArgs c) {
  static_assert(DT == QZ_DT_F16 || DT == QZ_DT_BF16, "16-bit activations");
  static_assert(!CL || DT == QZ_DT_F16, "exact codes are the fp16-activation table");
  static_assert(R == 2 || R == 4, "rows per wave: the act stores are whole 16-B pieces");
  constexpr int NW = kChNW;
  constexpr bool kBF = DT == QZ_DT_BF16;
  constexpr bool kWide = CL || kBF;
  constexpr int kPieces = 16;                    // the 256-B-entry table (WT): conflict-free, v_perm addresses
  __shared__ float s_code2[4][DQ ? 256 : 1];     // o, gate, up, down
  __shared__ float s_part[2][NW][R];             // gate/up partials by block parity
  __shared__ float s_nss[4];
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[2 * kTabDwords];
  extern __shared__ __attribute__((aligned(16))) unsigned char s_x[];   // the normalised h1 (stage B)

  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
#ifdef QZ_STAMPS
  unsigned long long ch_st_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
  CH_STAMP(0);
  const int P = (int)gridDim.x;
  const int W = P * NW;
  const int gw = (int)blockIdx.x * NW + wave;
  unsigned *const st = keep_sp(c.state);
  const unsigned epoch = __builtin_amdgcn_readfirstlane(ld_agent(st + kChEpoch));
  const unsigned target = (epoch + 1u) * (unsigned)P;   // arrivals of this launch at each barrier
  bool ok = true;

  // --- prologue: the four code2 tables, offsets, this thread's byte-table entry (all L2-resident),
  // then stage A's first step
  float c2a = 0.0f, c2b = 0.0f;
  if constexpr (DQ) {
    const int t = (int)threadIdx.x & 255;
    if (threadIdx.x < 256) {
      c2a = keep_sp(c.o.sc.code2)[t];
      c2b = keep_sp(c.gate.sc.code2)[t];
    } else {
      c2a = keep_sp(c.up.sc.code2)[t];
      c2b = keep_sp(c.down.sc.code2)[t];
    }
  }
  u32x4 tab_entry = {0u, 0u, 0u, 0u};
  if (threadIdx.x < 256) {
    const ByteTable *bt = kBF ? (c.o.tabsel ? &g_byte_tab_fp4_bf : &g_byte_tab_nf4_bf)
                              : (CL ? &g_byte_tab_nf4x : (c.o.tabsel ? &g_byte_tab_fp4 : &g_byte_tab_nf4));
    tab_entry = reinterpret_cast<const u32x4 *>(bt->v)[threadIdx.x];
  }

  const StageParams pa = load_stage<DQ>(c.o);
  const int nsA = pa.K >> 11;
  const int unitsA = pa.M / R;
  typedef ChainLoads<DQ, R, 0> LoadsA;
  LoadsA a_cur, a_oth;
  int u = gw;
  a_cur.issue(pa, min(u, unitsA - 1) * R, 0, lane);

  if constexpr (DQ) {
    const int t = (int)threadIdx.x & 255;
    if (threadIdx.x < 256) { s_code2[0][t] = c2a; s_code2[1][t] = c2b; }
    else { s_code2[2][t] = c2a; s_code2[3][t] = c2b; }
  }
  if (threadIdx.x < 256) store_byte_table_entry<kPieces>(s_tab, tab_entry);
  __syncthreads();
  const uint32_t jb = kWide ? (uint32_t)(lane & 31) << 3 : (uint32_t)lane << 2;

  // acc[r] += chunk . x * scale for one step of R rows (the gemv_body consume, per stage)
  float acc[R];
  auto consume = [&](auto &ld, int tbl, float offset) {
    typedef typename std::remove_reference<decltype(ld)>::type L;
    (void)sizeof(L);
    if constexpr (std::is_same<L, ChainLoads<DQ, R, 1>>::value) {   // x' from the LDS image
      const uint32_t c0 = (2u * ld.boff) >> 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(s_x + norm_x_off(c0 + (uint32_t)i));
        ld.xr[4 * i] = v.x; ld.xr[4 * i + 1] = v.y; ld.xr[4 * i + 2] = v.z; ld.xr[4 * i + 3] = v.w;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float am;
      if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[tbl][ld.q[r]], ld.a[r]), offset);
      else am = ld.a[r];
      const float d = chunk_dot_tab<kWide, true, kBF>(ld.wv[r], ld.xr, s_tab, jb);
      acc[r] = fmaf(d, am, acc[r]);
    }
  };
  // n K-steps of one unit, cur = step 0 and oth = step 1 already issued (oth clamped when n == 1)
  auto run_steps = [&](auto &cur, auto &oth, const StageParams &p, int row0, int n, int tbl, float offset) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    int j = 0, s = 0;
    for (; j + 3 < n; j += 2) {
      consume(cur, tbl, offset);
      cur.issue(p, row0, s + 2, lane);
      __builtin_amdgcn_sched_barrier(0);
      consume(oth, tbl, offset);
      oth.issue(p, row0, s + 3, lane);
      __builtin_amdgcn_sched_barrier(0);
      s += 2;
    }
    if (n - j == 3) {
      consume(cur, tbl, offset);
      cur.issue(p, row0, s + 2, lane);
      __builtin_amdgcn_sched_barrier(0);
      consume(oth, tbl, offset);
      consume(cur, tbl, offset);
    } else if (n - j == 2) {
      consume(cur, tbl, offset);
      consume(oth, tbl, offset);
    } else {
      consume(cur, tbl, offset);
    }
  };

  // ============ stage A: h1 = residual + o_proj(x), units of R rows per wave ============
  {
    const float offA = DQ ? *keep_sp(c.o.sc.offset) : 0.0f;
    a_oth.issue(pa, min(u, unitsA - 1) * R, min(1, nsA - 1), lane);
    for (;;) {
      run_steps(a_cur, a_oth, pa, min(u, unitsA - 1) * R, nsA, 0, offA);
      const int nu = u + W;
      if (nu < unitsA) {   // the next unit's first two steps, ahead of this epilogue
        a_cur.issue(pa, nu * R, 0, lane);
        a_oth.issue(pa, nu * R, min(1, nsA - 1), lane);
        __builtin_amdgcn_sched_barrier(0);
      }
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
      if (lane == kWave - 1 && u < unitsA) {
        const int row0 = u * R;
        uint32_t pk[R / 2];
#pragma unroll
        for (int r = 0; r < R; r += 2) {
          float o0 = v[r] * c.o.out_scale, o1 = v[r + 1] * c.o.out_scale;
          if (c.o.bias) {
            o0 += load_f32<DT>(c.o.bias, row0 + r);
            o1 += load_f32<DT>(c.o.bias, row0 + r + 1);
          }
          o0 = add_res<DT>(o0, c.o.res, row0 + r);
          o1 = add_res<DT>(o1, c.o.res, row0 + r + 1);
          pk[r / 2] = pack16<DT>(o0, o1);
        }
        // h1 is handed off: write-through (sc1) stores
        if constexpr (R == 2) {
          __hip_atomic_store((gu32_t *)c.o.y + (row0 >> 1), pk[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          __hip_atomic_store((gu64_t *)c.o.y + (row0 >> 2), (unsigned long long)pk[0] | ((unsigned long long)pk[1] << 32),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (nu >= unitsA) break;
      u = nu;
    }
  }

  CH_STAMP(1);   // stage A done
  // ============ barrier 0 (h1 published) + stage B's first block ============
  const bool is_up = wave >= 4;
  const int rg = wave & 3;
  // gate_proj (waves 0-3) or up_proj (waves 4-7): equal M and K, both write act
  const StageParams pb = load_stage<DQ>(is_up ? c.up : c.gate);
  const int nsB = pb.K >> 11;
  const int nblocksB = pb.M / (4 * R);
  typedef ChainLoads<DQ, R, 1> LoadsB;
  LoadsB b_cur, b_oth;
  int blk = (int)blockIdx.x;
  // the normalised-h1 prologue's own inputs that do not depend on h1: the norm weight chunks
  const int K = pb.K;
  const int nchunk = K >> 3;                      // 16-B chunks of the vector
  u32x4 nwv[kChMaxK / 8 / (NW * 64)];
#pragma unroll
  for (int i = 0; i < kChMaxK / 8 / (NW * 64); ++i) {
    const int ch = (int)threadIdx.x + i * NW * 64;
    if (ch < nchunk) nwv[i] = reinterpret_cast<const u32x4 *>(c.nw)[ch];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its h1 stores have completed
  __syncthreads();
  CH_STAMP(2);   // every wave drained its h1 stores
  if (threadIdx.x == 0) chain_arrive(st, 0);
  unsigned seen = chain_poll(st, 0, lane);
  b_cur.issue_w(pb, (min(blk, nblocksB - 1) * 4 + rg) * R, 0, lane);
  b_oth.issue_w(pb, (min(blk, nblocksB - 1) * 4 + rg) * R, min(1, nsB - 1), lane);
  if (wave == 0) {
    for (unsigned spins = 0; (int)(seen - target) < 0;) {
      if (++spins > kChSpinLimit) { ok = false; break; }
      __builtin_amdgcn_s_sleep(2);
      seen = chain_poll(st, 0, lane);
    }
  }
  __syncthreads();

  CH_STAMP(3);   // barrier 0 passed
  // ============ stage B: x' = RMSNorm(h1) into LDS (k_rmsnorm's order), then the gate/up pair ============
  {
    // threads 0..255 (k_rmsnorm's 256-thread order): chunks t, t + 256, ... squared in element order;
    // the raw chunks go to their slots of the x' image, then every thread normalises its chunks in place
    const void *h1p = keep_sp(c.o.y);
    float ss = 0.0f;
    if (threadIdx.x < 256) {
#pragma unroll
      for (int i = 0; i < kChMaxK / 8 / 256; ++i) {
        const int ch = (int)threadIdx.x + 256 * i;
        if (ch < nchunk) {
          const u32x4 hv = ld16_sc1(h1p, (uint32_t)ch * 16u);
          *reinterpret_cast<u32x4 *>(s_x + norm_x_off((uint32_t)ch)) = hv;
          ss = norm_chunk_ss<DT>(hv, ss);
        }
      }
      ss = norm_wave_sum(ss);
      if (lane == 0) s_nss[wave] = ss;
    }
    __syncthreads();
    const float tot = __fadd_rn(__fadd_rn(s_nss[0], s_nss[1]), __fadd_rn(s_nss[2], s_nss[3]));
    const float rs = rsqrtf(__fadd_rn(__fmul_rn(tot, 1.0f / (float)K), c.eps));
#pragma unroll
    for (int i = 0; i < kChMaxK / 8 / (NW * 64); ++i) {
      const int ch = (int)threadIdx.x + i * NW * 64;
      if (ch < nchunk) {
        u32x4 *slot = reinterpret_cast<u32x4 *>(s_x + norm_x_off((uint32_t)ch));
        *slot = norm_chunk_apply<DT>(*slot, nwv[i], rs);
      }
    }
    __syncthreads();
  }
  CH_STAMP(4);   // x' in LDS
  {
    const float offB = DQ ? *keep_sp((is_up ? c.up : c.gate).sc.offset) : 0.0f;
    const int tbl = is_up ? 2 : 1;
    const float osc = c.gate.out_scale;   // gate and up share the codebook
    for (int it = 0;; ++it) {
      const int row0 = (min(blk, nblocksB - 1) * 4 + rg) * R;
      run_steps(b_cur, b_oth, pb, row0, nsB, tbl, offB);
      const int nb = blk + P;
      if (nb < nblocksB) {   // the next block's first two steps, ahead of this epilogue
        b_cur.issue_w(pb, (nb * 4 + rg) * R, 0, lane);
        b_oth.issue_w(pb, (nb * 4 + rg) * R, min(1, nsB - 1), lane);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int par = it & 1;
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
      if (lane == kWave - 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float o = v[r] * osc;
          const void *bias = is_up ? c.up.bias : c.gate.bias;
          if (bias) o += load_f32<DT>(bias, row0 + r);
          s_part[par][wave][r] = o;
        }
      }
      __syncthreads();
      if (wave == 0 && blk < nblocksB) {
        // lanes 0 .. 4R-1: rows blk*4R + lane of h = act_fn(gate) * up (k_silu_mul's arithmetic on the
        // projections as torch stores them), gathered into whole 16-B pieces, stored write-through
        uint32_t hb = 0;
        if (lane < 4 * R) {
          const int g = lane / R, r = lane % R;
          const float gv = round_store<DT>(s_part[par][g][r]), uv = round_store<DT>(s_part[par][4 + g][r]);
          const float a = round_store<DT>(__fdiv_rn(gv, __fadd_rn(1.0f, expf(-gv))));
          hb = pack16<DT>(__fmul_rn(a, uv), 0.0f) & 0xFFFFu;
        }
#pragma unroll
        for (int pc = 0; pc < R / 2; ++pc) {   // piece pc: rows 8 pc .. 8 pc + 7 of the block
          uint32_t w[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            w[k] = (uint32_t)__builtin_amdgcn_readlane(hb, 8 * pc + 2 * k) |
                   ((uint32_t)__builtin_amdgcn_readlane(hb, 8 * pc + 2 * k + 1) << 16);
          if (lane == 0) st16_sc1(c.gate.y, (uint32_t)(blk * 4 * R + 8 * pc) * 2u, u32x4{w[0], w[1], w[2], w[3]});
        }
      }
      if (nb >= nblocksB) break;
      blk = nb;
    }
  }

  CH_STAMP(5);   // stage B done
  // ============ barrier 1 (act published) + stage C's first unit ============
  const StageParams pd = load_stage<DQ>(c.down);
  const int nsC = pd.K >> 11;
  const int unitsC = pd.M / R;
  typedef ChainLoads<DQ, R, 1> LoadsC;   // x = the workgroup's LDS image of act
  LoadsC c_cur, c_oth;
  u = gw;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its act stores have completed
  __syncthreads();
  if (threadIdx.x == 0) chain_arrive(st, 1);
  seen = chain_poll(st, 1, lane);
  c_cur.issue_w(pd, min(u, unitsC - 1) * R, 0, lane);     // weights only: act is not published yet
  c_oth.issue_w(pd, min(u, unitsC - 1) * R, min(1, nsC - 1), lane);
  if (wave == 0) {
    for (unsigned spins = 0; (int)(seen - target) < 0;) {
      if (++spins > kChSpinLimit) { ok = false; break; }
      __builtin_amdgcn_s_sleep(2);
      seen = chain_poll(st, 1, lane);
    }
  }
  __syncthreads();

  CH_STAMP(6);   // barrier 1 passed
  // ============ stage C: out = h1 + down_proj(act) ============
  {
    // act (handed off) into the workgroup's LDS image once, with sc1 loads, in the norm image's
    // conflict-free layout (every wave then reads its x slices from LDS, as stage B does: sc1 loads
    // bypass L1, and every wave reading its slices of act from the fabric moved 8x the bytes)
    const int nchunkC = pd.K >> 3;
    const void *actp = keep_sp(c.down.x);
#pragma unroll
    for (int i = 0; i < kChMaxI / 8 / (NW * 64); ++i) {
      const int ch = (int)threadIdx.x + i * NW * 64;
      if (ch < nchunkC)
        *reinterpret_cast<u32x4 *>(s_x + norm_x_off((uint32_t)ch)) = ld16_sc1(actp, (uint32_t)ch * 16u);
    }
    __syncthreads();
    CH_STAMP(7);   // act in LDS
    const float offC = DQ ? *keep_sp(c.down.sc.offset) : 0.0f;
    for (;;) {
      run_steps(c_cur, c_oth, pd, min(u, unitsC - 1) * R, nsC, 3, offC);
      const int nu = u + W;
      if (nu < unitsC) {
        c_cur.issue(pd, nu * R, 0, lane);
        c_oth.issue(pd, nu * R, min(1, nsC - 1), lane);
        __builtin_amdgcn_sched_barrier(0);
      }
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = wave_sum_last(acc[r]);
      if (lane == kWave - 1 && u < unitsC) {
        const int row0 = u * R;
        // the residual h1 is handed off: sc1 load of the R values
        uint32_t hres[R / 2];
        if constexpr (R == 2) {
          hres[0] = __hip_atomic_load((const gu32_t *)c.down.res + (row0 >> 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          const unsigned long long h = __hip_atomic_load((const gu64_t *)c.down.res + (row0 >> 2), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
          hres[0] = (uint32_t)h;
          hres[1] = (uint32_t)(h >> 32);
        }
#pragma unroll
        for (int r = 0; r < R; r += 2) {
          float o0 = v[r] * c.down.out_scale, o1 = v[r + 1] * c.down.out_scale;
          if (c.down.bias) {
            o0 += load_f32<DT>(c.down.bias, row0 + r);
            o1 += load_f32<DT>(c.down.bias, row0 + r + 1);
          }
          // residual + h: h rounded as torch stores it, the sum rounded by the store (add_res)
          o0 = __fadd_rn(bits16_f32<DT>(hres[r / 2] & 0xFFFFu), round_store<DT>(o0));
          o1 = __fadd_rn(bits16_f32<DT>(hres[r / 2] >> 16), round_store<DT>(o1));
          reinterpret_cast<uint32_t *>(c.down.y)[(row0 + r) >> 1] = pack16<DT>(o0, o1);
        }
      }
      if (nu >= unitsC) break;
      u = nu;
    }
  }

  CH_STAMP(8);   // stage C done (wave 0)
  // ============ finish: the last workgroup advances the epoch ============
  __syncthreads();
  CH_STAMP(9);   // every wave done
  CH_STAMP_FLUSH();
  if (threadIdx.x == 0) {
    if (!ok) __hip_atomic_store((gu32_t *)(st + kChStatus), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned t = __hip_atomic_fetch_add((gu32_t *)(st + kChDone), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)P - 1u) {
      __hip_atomic_store((gu32_t *)(st + kChDone), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32_t *)(st + kChEpoch), epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// the grid: one workgroup per CU (the dynamic LDS request keeps a second one off every CU), all
// resident -- the grid barriers need every workgroup running; 0 if the device cannot hold it
template <bool DQ, int DT, bool CL, int R, int STAMP = 0>
static int chain_grid(size_t lds) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(&k_mlp_chain<DQ, DT, CL, R, STAMP>),
                                                   kChNW * 64, lds) != hipSuccess || occ < 1)
    return 0;
  return device_cus();
}

}  // namespace qz

using namespace qz;

extern "C" int qz_mlp_chain_state_words(void) { return kChWords; }

// Validates the chain's arguments and fills its kernel arguments; *H_, *I_ the widths.  QZ_OK or a status.
static int chain_args(const qz_gemv_segment *o, const qz_gemv_segment *gate, const qz_gemv_segment *up,
                      const qz_gemv_segment *down, const void *x, const void *residual, int dtype, int quant_type,
                      int blocksize, int blocksize2, const void *norm_weight, float eps, void *h1, void *act, void *out,
                      unsigned *state, ChainArgs *c, bool *cl_, bool *dq_, size_t *lds_) {
  if (!o || !gate || !up || !down || !x || !residual || !norm_weight || !h1 || !act || !out || !state)
    return QZ_ERR_ARG;
  if (dtype != QZ_DT_F16 && dtype != QZ_DT_BF16) return QZ_ERR_SHAPE;
  const int H = o->M, I = gate->M;
  if (up->M != I || down->M != H || H <= 0 || I <= 0) return QZ_ERR_SHAPE;
  const bool cl = exact_codes(quant_type, nullptr) && dtype == QZ_DT_F16;
  const bool dq = o->qabsmax != nullptr;
  const qz_gemv_segment *segs[4] = {o, gate, up, down};
  GemvParams *ps[4] = {&c->o, &c->gate, &c->up, &c->down};
  const int Ks[4] = {H, H, H, I};
  const void *xs[4] = {x, nullptr, nullptr, act};
  void *ys[4] = {h1, act, act, out};
  const void *rs[4] = {residual, nullptr, nullptr, h1};
  for (int i = 0; i < 4; ++i) {
    const qz_gemv_segment &q = *segs[i];
    bool v;
    // x of gate/up is the norm image (not read from memory): validate with h1 in its place
    const int stt = make_params(q.M, Ks[i], xs[i] ? xs[i] : h1, dtype, q.B, quant_type, blocksize, q.absmax,
                                q.qabsmax, q.absmax2, q.code2, q.offset, blocksize2, q.block_base, nullptr, q.bias,
                                ys[i], ps[i], &v);
    if (stt != QZ_OK) return stt;
    if ((q.qabsmax != nullptr) != dq || !v || !full_steps(Ks[i], blocksize, blocksize2, dq, q.block_base))
      return QZ_ERR_SHAPE;
    set_tables(quant_type & ~QZ_EXACT_CODES, nullptr, cl, dtype, ps[i]);
    ps[i]->x = xs[i];
    ps[i]->res = rs[i];
  }
  // shapes: whole R-row units everywhere (R = 2), 16-B act pieces per pair block, the LDS images
  constexpr int R = 2;
  if (H % (4 * R) || I % (4 * R) || H > kChMaxK || I > kChMaxI || H % 2048 || I % 2048 ||
      ((uintptr_t)x | (uintptr_t)residual | (uintptr_t)norm_weight | (uintptr_t)h1 | (uintptr_t)act | (uintptr_t)out) % 16)
    return QZ_ERR_SHAPE;
  c->nw = norm_weight;
  c->eps = eps;
  c->state = state;
  *cl_ = cl;
  *dq_ = dq;
  // dynamic LDS: the x' image of stage B (H * 2 B), then stage C's act image (I * 2 B), at least
  // 24 KiB so that the workgroup's whole request (64 KiB table + 4 KiB code tables + this) exceeds
  // half the CU's 160 KiB: one workgroup per CU
  *lds_ = max(max((size_t)H * 2, (size_t)I * 2), (size_t)24 << 10);
  return QZ_OK;
}

template <int STAMP>
static int chain_launch(const ChainArgs &c, int dtype, bool cl, bool dq, size_t lds, hipStream_t s, int *grid_out) {
  constexpr int R = 2;
  int grid = 0;
#define QZ_CH(DQ_, DT_, CL_)                                                                                 \
  do {                                                                                                     \
    grid = chain_grid<DQ_, DT_, CL_, R, STAMP>(lds);                                                       \
    if (grid < 8) return QZ_ERR_SHAPE;                                                                     \
    hipLaunchKernelGGL((k_mlp_chain<DQ_, DT_, CL_, R, STAMP>), dim3(grid), dim3(kChNW * 64), lds, s, c);   \
  } while (0)
  if (dtype == QZ_DT_F16) {
    if (dq) { if (cl) QZ_CH(true, QZ_DT_F16, true); else QZ_CH(true, QZ_DT_F16, false); }
    else { if (cl) QZ_CH(false, QZ_DT_F16, true); else QZ_CH(false, QZ_DT_F16, false); }
  } else {
    if (dq) QZ_CH(true, QZ_DT_BF16, false); else QZ_CH(false, QZ_DT_BF16, false);
  }
#undef QZ_CH
  QZ_LAUNCH_CHECK();
  if (grid_out) *grid_out = grid;
  return QZ_OK;
}

extern "C" int qz_mlp_chain(const qz_gemv_segment *o, const qz_gemv_segment *gate, const qz_gemv_segment *up,
                            const qz_gemv_segment *down, const void *x, const void *residual, int dtype,
                            int quant_type, int blocksize, int blocksize2, const void *norm_weight, float eps,
                            void *h1, void *act, void *out, unsigned *state, void *stream) {
  ChainArgs c;
  bool cl, dq;
  size_t lds;
  const int rc = chain_args(o, gate, up, down, x, residual, dtype, quant_type, blocksize, blocksize2, norm_weight, eps,
                            h1, act, out, state, &c, &cl, &dq, &lds);
  if (rc != QZ_OK) return rc;
  return chain_launch<0>(c, dtype, cl, dq, lds, (hipStream_t)stream, nullptr);
}

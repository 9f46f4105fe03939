// Standalone GEMV microbenchmark (dev tool, not shipped): one-shot HBM read
// floor for an 8 MiB weight vs k_gemv_4bit variants, rotating 64 weight copies
// so the 256 MiB Infinity Cache never serves repeats.  Run under
// `rocprofv3 --kernel-trace --stats` for kernel-only durations; the printed
// numbers are hipEvent back-to-back averages (kernel + launch gap).
#define QZ_STAMPS 1
#include "../../quantizations_amd/csrc/gemv.hip"

namespace qz {
// Experimental straight-line variant (measured slower than k_gemv_4bit on
// every decode shape in the round-1 sweep; kept here for reference).  Decode shapes: every wave owns R whole rows
// (WK = 1) and walks exactly NSW = K / 2048 steps, fully unrolled over two
// named load sets.  Without runtime control flow hipcc's waitcnt pass sees
// the exact issue order, so step i+1's HBM loads stay in flight while step i
// is decoded (the runtime-loop kernel above keeps only ~half a step in
// flight: its loop-join waits are conservative).
template <int MODE, bool DQ, int DT, int R, int NSW, int NW = 4>
__global__ __launch_bounds__(NW * 64) void k_gemv_4bit_sl(GemvParams p_in) {
  const GemvParams p = load_params(p_in);
  constexpr bool kSplit = DT != QZ_DT_F16;
  __shared__ float s_code2[DQ ? 256 : 1];

  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int row0 = (blockIdx.x * NW + wave) * R;
  const int row_bytes = p.K >> 1;

  float c2 = 0.0f, offset = 0.0f;
  if constexpr (DQ) {
    if (NW * 64 == 256 || threadIdx.x < 256) c2 = p.sc.code2[threadIdx.x & 255];
    offset = *p.sc.offset;
  }
  StepLoads<MODE, DQ, DT, R, false, 0> ld[2];
  ld[0].issue(p, row0, 0, lane, row_bytes);
  if constexpr (NSW > 1) ld[1].issue(p, row0, 1, lane, row_bytes);
  if constexpr (DQ) {
    if (NW * 64 == 256 || threadIdx.x < 256) s_code2[threadIdx.x & 255] = c2;
    __syncthreads();
  }
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = p.tab[i];

  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;

#pragma unroll
  for (int i = 0; i < NSW; ++i) {
    StepLoads<MODE, DQ, DT, R, false, 0> &c = ld[i & 1];
    uint32_t hi[16], lo[kSplit ? 16 : 1];
    float usc;
    c.xs.prepare(hi, lo, usc);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float am;
      if constexpr (DQ) am = __fadd_rn(__fmul_rn(s_code2[c.q[r]], c.a[r]), offset);
      else am = c.a[r];
      am = c.on ? am : 0.0f;
      acc[r] = fmaf(chunk_dot<MODE, kSplit>(c.wv[r], hi, lo, t), am, acc[r]);
    }
    if (i + 2 < NSW) {
      __builtin_amdgcn_sched_barrier(0);
      c.issue(p, row0, i + 2, lane, row_bytes);  // refill the set just consumed
      __builtin_amdgcn_sched_barrier(0);
    }
  }

#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float v = wave_sum_last(acc[r]);
    const int row = row0 + r;
    if (lane == kWave - 1 && row < p.M) {
      float o = v * p.out_scale;
      if (p.bias) o += load_f32<DT>(p.bias, row);
      store_f32<DT>(p.y, row, o);
    }
  }
}

}  // namespace qz

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>
#include <string>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

template <int T, int L>
__global__ __launch_bounds__(T) void k_read_floor(const unsigned char *__restrict__ p, long long bytes, uint32_t *sink) {
  const long long nchunk = bytes / 16;
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const long long c = ((long long)blockIdx.x * L + i) * T + threadIdx.x;
    if (c < nchunk) {
      v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p) + c);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int T, int L>
__global__ __launch_bounds__(T) void k_read_floor_store(const unsigned char *__restrict__ p, long long bytes, uint32_t *out) {
  const long long nchunk = bytes / 16;
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const long long c = ((long long)blockIdx.x * L + i) * T + threadIdx.x;
    if (c < nchunk) {
      v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p) + c);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if ((threadIdx.x & 63) < 2) out[(blockIdx.x * T + threadIdx.x) / 32] = acc;  // 2 rows' worth per wave
}

template <int T, int L>
__global__ __launch_bounds__(T) void k_read_floor_store_nt(const unsigned char *__restrict__ p, long long bytes, uint32_t *out) {
  const long long nchunk = bytes / 16;
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const long long c = ((long long)blockIdx.x * L + i) * T + threadIdx.x;
    if (c < nchunk) {
      v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p) + c);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if ((threadIdx.x & 63) < 2) __builtin_nontemporal_store(acc, out + (blockIdx.x * T + threadIdx.x) / 32);
}

// one-shot floor with timeline stamps (start, data back, end) per wave
__global__ __launch_bounds__(256) void k_floor_stamp(const unsigned char *__restrict__ p, long long bytes, uint32_t *sink) {
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p) + (c < bytes / 16 ? c : 0));
  uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (acc == 0x12345678u) sink[0] = acc;
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *o = qz::g_qz_stamp + (size_t)(blockIdx.x * 4 + threadIdx.x / 64) * 8;
    o[0] = t0; o[1] = t1; o[2] = t1; o[3] = t1; o[4] = t1; o[5] = ((unsigned long long)xcc << 32) | hw;
  }
}

// park the stream (~20 ms) so the host has enqueued a whole round before the GPU reaches it
__global__ void k_spin(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

// random packed weights (a constant fill would make every LDS lookup a broadcast)
__global__ void k_fill_random(uint32_t *p, long long n, uint32_t seed) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    p[i] = h;
  }
}

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 4096;
  const int NC = 64, ITERS = 100;
  const size_t pbytes = (size_t)M * K / 2, nb = (size_t)M * K / 64;
  std::vector<unsigned char *> P(NC), Q(NC);
  std::vector<float *> A2(NC), A(NC);
  for (int i = 0; i < NC; ++i) {
    CK(hipMalloc(&P[i], pbytes)); CK(hipMalloc(&Q[i], nb)); CK(hipMalloc(&A2[i], (nb / 256 + 1) * 4));
    CK(hipMalloc(&A[i], nb * 4));
    hipLaunchKernelGGL(k_fill_random, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(P[i]),
                       (long long)(pbytes / 4), 0x1234u + i);
    CK(hipMemset(Q[i], 0x40, nb));
    CK(hipMemset(A2[i], 0x3C, (nb / 256 + 1) * 4)); CK(hipMemset(A[i], 0x3C, nb * 4));
  }
  float *code2, *off; void *x, *y; uint32_t *sink;
  CK(hipMalloc(&code2, 1024)); CK(hipMemset(code2, 0x3C, 1024)); CK(hipMalloc(&off, 4)); CK(hipMemset(off, 0, 4));
  // x: 64 copies (ABL & 2048 gives every wave its own)
  CK(hipMalloc(&x, (size_t)K * 4 * 64)); CK(hipMemset(x, 0x3C, (size_t)K * 4 * 64));
  CK(hipMalloc(&y, M * 4)); CK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));

  // Variants are registered, then timed in interleaved rounds (rule 24 of the
  // guide): every round runs each variant for ITERS back-to-back launches;
  // median and min over rounds are reported.
  struct Variant { std::string name; std::function<void(int)> launch; std::vector<double> us; };
  std::vector<Variant> vs;
  auto timeit = [&](const char *name, auto launch) { vs.push_back({name, launch, {}}); };
#define FLOOR(T, L) timeit("floor T=" #T " L=" #L, [&](int i) { \
    const long long nchunk = pbytes / 16; const unsigned g = (unsigned)((nchunk + (long long)T * L - 1) / ((long long)T * L)); \
    hipLaunchKernelGGL((k_read_floor<T, L>), dim3(g), dim3(T), 0, 0, P[i % NC], (long long)pbytes, sink); })
  const bool sweep = argc > 4 && std::string(argv[4]) == "sweep";
  FLOOR(256, 1); FLOOR(256, 2);
  uint32_t *fout; CK(hipMalloc(&fout, 1 << 24));
  timeit("floor+store T=256 L=2", [&](int i) { const long long nchunk = pbytes / 16;
    const unsigned g = (unsigned)((nchunk + 511) / 512);
    hipLaunchKernelGGL((k_read_floor_store<256, 2>), dim3(g), dim3(256), 0, 0, P[i % NC], (long long)pbytes, fout); });

  GemvParams p{};
  p.sc = ScaleSrc{nullptr, nullptr, nullptr, code2, off, 256};
  p.x = x; p.y = y; p.M = M; p.K = K; p.bs_log2 = 6; p.bs2_log2 = 8; p.lut = nullptr; p.bias = nullptr;
  build_tables(kModeLUT16, QZ_NF4, p.tab, &p.out_scale);
#define GVN(MODE, DQ, R, WK, NW) timeit("gemv mode=" #MODE " dq=" #DQ " R=" #R " WK=" #WK " NW=" #NW, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; \
    if (DQ) { q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; } else { q.sc.absmax = A[i % NC]; } \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, QZ_DT_F16, R, WK, NW>), dim3(g), dim3(NW * 64), 0, 0, q); })
#define GV(MODE, DQ, R, WK) GVN(MODE, DQ, R, WK, 4)
  // full-control variant: x staged in LDS (XL) and ablation bits (ABL: 1 no scale loads,
  // 2 no x loads, 4 no reduction/store)
#define GVF(MODE, DQ, R, WK, NW, XL, ABL) timeit("gemvF mode=" #MODE " R=" #R " WK=" #WK " NW=" #NW " XL=" #XL " ABL=" #ABL, [&](int i) { \
    GemvParams q = p; q.B = P[i % NC]; \
    if (DQ) { q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; } else { q.sc.absmax = A[i % NC]; } \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, QZ_DT_F16, R, WK, NW, XL, ABL>), dim3(g), dim3(NW * 64), XL ? K * 2 : 0, 0, q); })
  const bool ablate = argc > 4 && std::string(argv[4]) == "ablate";
  const bool small = argc > 4 && std::string(argv[4]) == "small";
  const bool r8 = argc > 4 && std::string(argv[4]) == "r8";
  const bool tab = argc > 4 && std::string(argv[4]) == "tab";
  if (tab) {  // LDS byte-table decode (kModeTab = 3) vs the v_perm decode (kModeLUT16 = 1)
    GV(1, true, 2, 1); GV(1, true, 4, 2);
    GV(3, true, 1, 1); GV(3, true, 2, 1); GV(3, true, 4, 1); GV(3, true, 2, 2); GV(3, true, 4, 2); GV(3, true, 1, 2);
    GVN(3, true, 2, 1, 8); GVN(3, true, 4, 2, 8); GVN(3, true, 2, 2, 8);
  }
  const bool tabab = argc > 4 && std::string(argv[4]) == "tabab";
  if (tabab) {  // what bounds the table decode: 16 = no dot2c, 32 = no LDS reads, 3 = no scale/x loads, 4 = no reduction
    GV(3, true, 2, 1); GV(3, true, 4, 2);
    GVF(3, true, 2, 1, 4, false, 16); GVF(3, true, 4, 2, 4, false, 16);
    GVF(3, true, 2, 1, 4, false, 32); GVF(3, true, 4, 2, 4, false, 32);
    GVF(3, true, 2, 1, 4, false, 48); GVF(3, true, 4, 2, 4, false, 48);
    GVF(3, true, 2, 1, 4, false, 3); GVF(3, true, 4, 2, 4, false, 3);
    GVF(3, true, 2, 1, 4, false, 51); GVF(3, true, 4, 2, 4, false, 51);
    GVF(2, true, 2, 1, 4, false, 3); GVF(2, true, 4, 2, 4, false, 3);
    // 64 = no table build; mode 2 with 32 KiB of idle dynamic LDS (occupancy of the table kernel)
    GVF(3, true, 2, 1, 4, false, 115); GVF(3, true, 4, 2, 4, false, 115);
    GVF(3, true, 2, 1, 4, false, 64); GVF(3, true, 4, 2, 4, false, 64);
#define GVL(MODE, DQ, R, WK, NW, ABL, LDSB) timeit("gemvL mode=" #MODE " R=" #R " WK=" #WK " NW=" #NW " ABL=" #ABL " lds=" #LDSB, [&](int i) { \
    GemvParams q = p; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, QZ_DT_F16, R, WK, NW, false, ABL>), dim3(g), dim3(NW * 64), LDSB, 0, q); })
    GVL(2, true, 2, 1, 4, 3, 32768); GVL(2, true, 4, 2, 4, 3, 32768);
    GVL(2, true, 2, 1, 4, 3, 16384); GVL(2, true, 4, 2, 4, 3, 16384);
  }
  const bool tabx = argc > 4 && std::string(argv[4]) == "tabx";
  if (tabx) {  // table decode: x traffic per weight byte (R = 8 rows per wave, x staged in LDS)
    GV(3, true, 2, 1); GV(3, true, 4, 1); GV(3, true, 4, 2); GV(3, true, 8, 1); GV(3, true, 8, 2);
    GVF(3, true, 2, 1, 4, true, 0); GVF(3, true, 4, 1, 4, true, 0); GVF(3, true, 4, 2, 4, true, 0);
    GVF(3, true, 8, 1, 4, true, 0);
    GVF(3, true, 2, 1, 8, true, 0); GVF(3, true, 4, 1, 8, true, 0); GVF(3, true, 4, 2, 8, true, 0);
  }
  const bool tabfs = argc > 4 && std::string(argv[4]) == "tabfs";
#define GVS(MODE, DQ, R, WK, NW) timeit("gemvS mode=" #MODE " dq=" #DQ " R=" #R " WK=" #WK " NW=" #NW " full-step", [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; \
    if (DQ) { q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; } else { q.sc.absmax = A[i % NC]; } \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, QZ_DT_F16, R, WK, NW, false, 0, true>), dim3(g), dim3(NW * 64), 0, 0, q); })
#define GVX(MODE, R, WK, NW) timeit("gemvX mode=" #MODE " R=" #R " WK=" #WK " NW=" #NW " full-step x-in-LDS", [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<MODE, true, QZ_DT_F16, R, WK, NW, true, 0, true>), dim3(g), dim3(NW * 64), K * 2, 0, q); })
  const bool tabxl = argc > 4 && std::string(argv[4]) == "tabxl";
  if (tabxl) {
    GVS(3, true, 2, 1, 4); GVS(3, true, 4, 1, 4); GVX(3, 2, 1, 4); GVX(3, 4, 1, 4); GVX(3, 1, 1, 4);
    GVX(3, 2, 1, 8); GVX(3, 4, 1, 8); GVX(3, 1, 1, 8); GVX(3, 2, 2, 8);
  }
  if (tabfs) {  // byte-table decode: generic vs full-step loads
    GV(3, true, 2, 1); GV(3, true, 4, 1); GVS(3, true, 2, 1, 4); GVS(3, true, 4, 1, 4);
    GVS(3, true, 1, 1, 4); GVS(3, true, 2, 1, 8); GVS(3, true, 4, 1, 8); GVS(3, false, 2, 1, 4); GVS(3, false, 4, 1, 4);
  }
  const bool skel = argc > 4 && std::string(argv[4]) == "skel";
  if (skel) {  // what the GEMV skeleton costs over a bare streaming read
    // 7: loads only; 3: + DPP reduction + store; 11: + store without reduction; 259: + lane-63 reduction + store
    GVF(2, false, 2, 1, 4, false, 7); GVF(2, false, 2, 1, 4, false, 3); GVF(2, false, 2, 1, 4, false, 11);
    GVF(2, false, 2, 1, 4, false, 259);
    // table kernel: 115 = no decode work at all; +128 = no prologue barrier; +256 = lane-63 reduction
    GVF(3, false, 2, 1, 4, false, 115); GVF(3, false, 2, 1, 4, false, 243); GVF(3, false, 2, 1, 4, false, 371);
    GVF(3, true, 2, 1, 4, false, 0); GVF(3, true, 2, 1, 4, false, 256);
    GVS(3, true, 2, 1, 4);
  }
  const bool cl = argc > 4 && std::string(argv[4]) == "cl";
#define GVC(R, ABL, CL_) timeit("gemvFS tab dq R=" #R " ABL=" #ABL " CL=" #CL_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, ABL, true, CL_>), dim3(g), dim3(256), 0, 0, q); })
  if (cl) {  // exact-code (CL) table vs fp16 codes; non-temporal y stores; store drain on the floor kernel
    timeit("floor+store-nt T=256 L=2", [&](int i) { const long long nchunk = pbytes / 16;
      const unsigned g = (unsigned)((nchunk + 511) / 512);
      hipLaunchKernelGGL((k_read_floor_store_nt<256, 2>), dim3(g), dim3(256), 0, 0, P[i % NC], (long long)pbytes, fout); });
    GVC(2, 0, false); GVC(2, 0, true); GVC(2, 1024, false); GVC(2, 1024, true); GVC(4, 0, true); GVC(1, 0, true);
  }
  const bool clsweep = argc > 4 && std::string(argv[4]) == "clsweep";
#define GVCS(R, WK, NW) timeit("gemvFS CL R=" #R " WK=" #WK " NW=" #NW, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384; \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, WK, NW, false, 0, true, true>), dim3(g), dim3(NW * 64), 0, 0, q); })
#define GVW(R, CL_, WT_) timeit("gemvFS R=" #R " CL=" #CL_ " WT=" #WT_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, 0, true, CL_, WT_>), dim3(g), dim3(256), 0, 0, q); })
  const bool wt = argc > 4 && std::string(argv[4]) == "wt";
  if (wt) {  // wide (256 B per entry) table: one v_perm per lookup address, bank-private copies
    GVW(2, false, false); GVW(2, false, true); GVW(2, true, false); GVW(2, true, true); GVW(4, true, false); GVW(4, true, true);
  }
  if (clsweep) {  // exact-code full-step kernel: waves per workgroup, rows per wave, K split
    GVCS(2, 1, 4); GVCS(2, 2, 4); GVCS(1, 2, 4); GVCS(1, 1, 4); GVCS(4, 1, 4); GVCS(4, 2, 4);
    GVCS(2, 1, 8); GVCS(2, 2, 8); GVCS(1, 2, 8); GVCS(4, 2, 8); GVCS(2, 4, 8); GVCS(1, 4, 4);
  }
  const bool tabab2 = argc > 4 && std::string(argv[4]) == "tabab2";
#define GVFS(R, ABL) timeit("gemvFS tab dq R=" #R " ABL=" #ABL, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, ABL, true>), dim3(g), dim3(256), 0, 0, q); })
#define GVB(R, DT_, NAME) timeit("gemvFS tab dq R=" #R " x=" NAME, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, DT_, R, 1, 4, false, 0, true>), dim3(g), dim3(256), 0, 0, q); })
  const bool bf16 = argc > 4 && std::string(argv[4]) == "bf16";
  if (bf16) {  // activation dtype: rows per wave for bf16 x (its per-lane convert is shared by R rows)
    GVB(2, QZ_DT_F16, "f16"); GVB(4, QZ_DT_F16, "f16");
    GVB(1, QZ_DT_BF16, "bf16"); GVB(2, QZ_DT_BF16, "bf16"); GVB(4, QZ_DT_BF16, "bf16");
    GVB(2, QZ_DT_F32, "f32"); GVB(4, QZ_DT_F32, "f32");
  }
#define GVK(R, WK) timeit("gemvFS tab dq R=" #R " WK=" #WK, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    const unsigned g = (unsigned)((M + R * (4 / WK) - 1) / (R * (4 / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, WK, 4, false, 0, true>), dim3(g), dim3(256), 0, 0, q); })
  const bool wk = argc > 4 && std::string(argv[4]) == "wk";
  if (wk) {  // K split over waves for long rows (more waves per SIMD when M / R is small)
    GVK(4, 1); GVK(4, 2); GVK(2, 1); GVK(2, 2); GVK(4, 4);
  }
  const bool pk = argc > 4 && std::string(argv[4]) == "pack";
  if (pk) {  // y stores: packed row pairs (product) vs one 16-bit store per row (ABL 4096)
    GVFS(2, 0); GVFS(2, 4096); GVFS(4, 0); GVFS(4, 4096); GVFS(8, 0);
  }
  const bool xcopy = argc > 4 && std::string(argv[4]) == "xcopy";
  if (xcopy) {  // x hot-spot test: every wave reads its own copy of x (ABL 2048)
    GVFS(2, 0); GVFS(2, 2048); GVFS(4, 0); GVFS(4, 2048); GVFS(1, 0); GVFS(1, 2048);
  }
  if (tabab2) {  // full-step table kernel ablations: 1 no scale loads, 2 no x loads, 4 no reduce/store,
                 // 8 no DPP reduction, 16 no dots, 32 no LDS reads, 64 no table build, 128 no prologue barrier
    GVFS(2, 0); GVFS(2, 1); GVFS(2, 2); GVFS(2, 3); GVFS(2, 4); GVFS(2, 16); GVFS(2, 32); GVFS(2, 48);
    GVFS(2, 112); GVFS(2, 115); GVFS(2, 119); GVFS(2, 2 + 16 + 32);
    GVFS(4, 0); GVFS(4, 2); GVFS(4, 3); GVFS(1, 0); GVFS(1, 2);
  }
  if (r8) {  // 8 rows per wave (half the x traffic per weight byte) vs the production geometries
    GV(1, true, 4, 2); GV(1, true, 2, 1); GV(1, true, 8, 1); GV(1, true, 8, 2); GV(1, true, 8, 4);
    GVN(1, true, 8, 1, 8); GVN(1, true, 8, 2, 8);
  }
  if (small) {  // geometry around the 4096^2 headline launch (workgroup size too)
    GVN(1, true, 2, 1, 4); GVN(1, true, 1, 1, 4); GVN(1, true, 1, 2, 4); GVN(1, true, 2, 2, 4);
    GVN(1, true, 2, 1, 8); GVN(1, true, 1, 1, 8); GVN(1, true, 1, 2, 8); GVN(1, true, 2, 2, 8);
    GVN(1, true, 2, 1, 16); GVN(1, true, 1, 1, 16); GVN(1, true, 1, 2, 16); GVN(1, true, 2, 2, 16);
    GVN(2, true, 2, 1, 4); GVN(2, true, 1, 1, 16);
    GVF(2, true, 2, 1, 4, false, 3); GVF(2, true, 2, 1, 4, false, 7);
  }
  if (ablate) {
    GV(1, true, 4, 2); GV(1, true, 2, 1); GV(0, true, 4, 2); GV(2, true, 4, 2);
    GVF(1, true, 4, 2, 4, false, 1); GVF(1, true, 4, 2, 4, false, 2); GVF(1, true, 4, 2, 4, false, 3);
    GVF(2, true, 4, 2, 4, false, 3); GVF(1, true, 4, 2, 4, true, 0); GVF(1, true, 2, 1, 4, true, 0);
    GVN(1, true, 4, 2, 8); GVN(1, true, 4, 4, 8); GVN(1, true, 2, 2, 8); GVN(1, true, 4, 1, 8);
    GVN(1, true, 2, 1, 8); GVN(1, true, 4, 8, 8);
  }
  const bool nopro = argc > 4 && std::string(argv[4]) == "nopro";
  if (nopro) {  // price of the prologue's global loads (ABL 32768: timing only, wrong outputs)
    GVFS(2, 0); GVFS(2, 32768); GVFS(4, 0); GVFS(4, 32768); GVFS(1, 0); GVFS(1, 32768);
  }
  const bool wt8 = argc > 4 && std::string(argv[4]) == "wt8";
#define GVWN(R, NW, CL_, WT_) timeit("gemvFS R=" #R " NW=" #NW " CL=" #CL_ " WT=" #WT_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384; \
    const unsigned g = (unsigned)((M + R * NW - 1) / (R * NW)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, NW, false, 0, true, CL_, WT_>), dim3(g), dim3(NW * 64), 0, 0, q); })
  if (wt8) {  // exact codes: conflict-free 64 KiB table (WT) shared by 8 waves vs the 16-copy table at 4 waves
    GVWN(4, 4, false, false); GVWN(4, 4, true, false); GVWN(4, 8, true, true); GVWN(4, 4, true, true);
    GVWN(2, 4, false, false); GVWN(2, 4, true, false); GVWN(2, 8, true, true); GVWN(2, 8, true, false);
    GVWN(1, 8, true, true);
  }
  // outputs of every registered variant from the first whose name holds `ref` on, against it
  auto check_outputs = [&](const char *ref) {
      std::vector<uint16_t> hx(K);
      uint32_t st = 12345u;
      for (int k = 0; k < K; ++k) {
        st = st * 1664525u + 1013904223u;
        hx[k] = (uint16_t)(0x3000u + ((st >> 8) & 0x0FFFu)) | ((st >> 30) << 15);
      }
      CK(hipMemcpy(x, hx.data(), K * 2, hipMemcpyHostToDevice));
      std::vector<std::vector<uint16_t>> outs;
      size_t v0 = 0;
      while (v0 < vs.size() && vs[v0].name.find(ref) == std::string::npos) ++v0;
      for (size_t vi = v0; vi < vs.size(); ++vi) {
        CK(hipMemset(y, 0, M * 4));
        vs[vi].launch(0);
        CK(hipDeviceSynchronize());
        std::vector<uint16_t> hy(M);
        CK(hipMemcpy(hy.data(), y, M * 2, hipMemcpyDeviceToHost));
        outs.push_back(hy);
      }
      for (size_t o = 1; o < outs.size(); ++o) {
        int diff = 0, maxulp = 0;
        for (int r = 0; r < M; ++r) {
          const int d = std::abs((int)(int16_t)outs[o][r] - (int)(int16_t)outs[0][r]);
          if (d) ++diff;
          maxulp = std::max(maxulp, d);
        }
        printf("check %-40s vs product CL: %d of %d fp16 outputs differ, max %d ulp\n", vs[v0 + o].name.c_str(), diff, M,
               maxulp);
      }
      CK(hipMemset(x, 0x3C, (size_t)K * 4 * 64));
  };
  const bool fm = argc > 4 && std::string(argv[4]) == "fm";
  // exact codes (CL): FMV 0 = hi + lo fp16 code pairs by v_dot2c (round-3 product); 1 = fp32 codes
  // by v_fma_mix_f32, two-VALU addresses, 16-copy table; 2 = the same, 256-B entries + SDWA addresses
#define GVM(R, NW, WT_, FMV_) timeit("gemvFS CL R=" #R " NW=" #NW " WT=" #WT_ " FMV=" #FMV_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.out_scale = (FMV_) ? 1.0f : 1.0f / 16384; q.tabsel = 0; \
    const unsigned g = (unsigned)((M + R * NW - 1) / (R * NW)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, NW, false, 0, true, true, WT_, FMV_>), dim3(g), dim3(NW * 64), 0, 0, q); })
  if (fm) {
    GVFS(2, 0);                                      // fp16 codes (reference point)
    GVM(2, 4, false, 0); GVM(2, 4, false, 1); GVM(2, 4, true, 1); GVM(2, 4, true, 2);
    GVM(4, 4, false, 0); GVM(4, 4, false, 1); GVM(4, 4, true, 2);
    GVM(1, 4, false, 1); GVM(1, 4, true, 2);
    GVM(2, 8, true, 2); GVM(4, 8, true, 2); GVM(1, 8, true, 2);
    check_outputs("FMV=0");
  }
  const bool early = argc > 4 && std::string(argv[4]) == "early";
  // OPT 1: the second K-step issued before the prologue barrier; 2: byte table built from SGPR planes
#define GVO(R, CL_, OPT_) timeit("gemvFS R=" #R " CL=" #CL_ " OPT=" #OPT_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.tabsel = (CL_) ? 2 : 0; \
    if (CL_) { q.out_scale = 1.0f / 16384; build_exact_planes(q.tab, q.tab_lo); } \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, 0, true, CL_, false, 0, OPT_>), dim3(g), dim3(256), 0, 0, q); })
  // FMV 3 / 4: fp32 codes against x widened to fp32 once per step (v_fma_f32 / v_pk_fma_f32)
  const bool xf = argc > 4 && std::string(argv[4]) == "xf";
#define GVX(R, FMV_, OPT_) timeit("gemvFS CL R=" #R " FMV=" #FMV_ " OPT=" #OPT_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.out_scale = (FMV_) ? 1.0f : 1.0f / 16384; q.tabsel = (FMV_) ? 0 : 2; \
    if (!(FMV_)) build_exact_planes(q.tab, q.tab_lo); \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, 0, true, true, false, FMV_, OPT_>), dim3(g), dim3(256), 0, 0, q); })
  if (xf) {
    GVFS(2, 0);                                      // fp16 codes (reference point)
    if (K == 4096) {
      GVX(2, 0, 8); GVX(2, 3, 8); GVX(2, 4, 8); GVX(4, 0, 8); GVX(4, 3, 8); GVX(4, 4, 8); GVX(1, 3, 8); GVX(1, 4, 8);
    }
    GVX(2, 0, 0); GVX(2, 3, 0); GVX(2, 4, 0); GVX(4, 0, 0); GVX(4, 3, 0); GVX(4, 4, 0); GVX(1, 4, 0);
    check_outputs("FMV=0 OPT=0");
  }
  // OPT 16 / 32: a ring of 3 / 4 step buffers for waves owning exactly NSW steps (K = 2048 NSW, WK = 1)
  const bool ring = argc > 4 && std::string(argv[4]) == "ring";
#define GVR(R, OPT_, NSW_) timeit("gemvFS CL R=" #R " OPT=" #OPT_ " NSW=" #NSW_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.tabsel = 2; q.out_scale = 1.0f / 16384; build_exact_planes(q.tab, q.tab_lo); \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, 0, true, true, false, 0, OPT_, false, NSW_>), dim3(g), dim3(256), 0, 0, q); })
  if (ring && K == 14336) {
    GVO(2, true, 0); GVR(2, 16, 7); GVR(2, 32, 7); GVO(4, true, 0); GVR(4, 16, 7); GVR(4, 32, 7); GVO(1, true, 0); GVR(1, 16, 7); GVR(1, 32, 7);
    check_outputs("R=2 CL=true OPT=0");
  }
  if (ring && K == 28672) {
    GVO(2, true, 0); GVR(2, 16, 14); GVR(2, 32, 14); GVO(4, true, 0); GVR(4, 16, 14); GVR(4, 32, 14);
    check_outputs("R=2 CL=true OPT=0");
  }
  if (ring && K == 8192) {
    GVO(2, true, 0); GVR(2, 16, 4); GVR(2, 32, 4); GVO(4, true, 0); GVR(4, 16, 4);
    check_outputs("R=2 CL=true OPT=0");
  }
  // 8-wave workgroups sharing one 256-B-entry exact-code table (WT) vs the product (4 waves, 16-copy table)
  const bool nw8 = argc > 4 && std::string(argv[4]) == "nw8";
#define GVW(R, NW, WT_, OPT_) timeit("gemvFS CL R=" #R " NW=" #NW " WT=" #WT_ " OPT=" #OPT_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.tabsel = 2; q.out_scale = 1.0f / 16384; build_exact_planes(q.tab, q.tab_lo); \
    const unsigned g = (unsigned)((M + R * NW - 1) / (R * NW)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, NW, false, 0, true, true, WT_, 0, OPT_>), dim3(g), dim3(NW * 64), 0, 0, q); })
  if (nw8) {
    if (K == 4096) {
      GVW(2, 4, false, 8); GVW(2, 8, true, 8); GVW(2, 8, false, 8); GVW(2, 4, true, 8); GVW(4, 8, true, 8); GVW(1, 8, true, 8);
      check_outputs("R=2 NW=4 WT=false OPT=8");
    } else {
      GVW(2, 4, false, 0); GVW(2, 8, true, 0); GVW(2, 8, false, 0); GVW(2, 4, true, 0); GVW(4, 8, true, 0); GVW(1, 8, true, 0);
      GVW(4, 4, false, 0);
      check_outputs("R=2 NW=4 WT=false OPT=0");
    }
  }
  const bool two = argc > 4 && std::string(argv[4]) == "two";
  if (two && K == 4096) {  // OPT 8: straight-line two-step waves (K = 4096, WK = 1)
    GVO(2, true, 0); GVO(2, true, 8); GVO(2, true, 10); GVO(2, false, 0); GVO(2, false, 8); GVO(4, true, 0);
    GVO(4, true, 8); GVO(1, true, 0); GVO(1, true, 8);
    check_outputs("R=2 CL=true OPT=0");
  }
  if (early) {
    GVO(2, true, 0); GVO(2, true, 1); GVO(2, true, 2); GVO(2, true, 3);
    GVO(2, false, 0); GVO(2, false, 1); GVO(2, false, 3);
    GVO(4, true, 0); GVO(4, true, 1); GVO(4, true, 3);
    GVO(1, true, 0); GVO(1, true, 3);
    check_outputs("R=2 CL=true OPT=0");
  }
  const bool mf = argc > 4 && std::string(argv[4]) == "mf";
  // MFMA-product GEMV (k_gemv_4bit_mf, K = 4096 only): 16-row tiles, 8 waves split K, 4 loads each
#define GVMF(CL_, WT_) timeit("mf CL=" #CL_ " WT=" #WT_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.out_scale = (CL_) ? 1.0f / 16384 : 1.0f; \
    hipLaunchKernelGGL((k_gemv_4bit_mf<CL_, WT_, 8, 4>), dim3(M / 16), dim3(512), 0, 0, q); })
#define GVXL(R) timeit("gemvXL CL R=" #R " (x staged in LDS)", [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, true, 0, true, true>), dim3(g), dim3(256), K * 2, 0, q); })
  const bool pf = argc > 4 && std::string(argv[4]) == "pf";
  // launch i prefetches the first CHUNKS KiB of every row of launch i + 1's weights (the next copy)
#define GVPF(R, CHUNKS) timeit("gemvFS CL R=" #R " prefetch next chunks=" #CHUNKS, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384; \
    q.pf = P[(i + 1) % NC]; q.pf_row_bytes = (uint32_t)(K / 2); q.pf_rows = M; q.pf_chunks = CHUNKS; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, R, 1, 4, false, 0, true, true, false, 0, 0, true>), dim3(g), dim3(256), 0, 0, q); })
  if (pf) {
    GVO(2, true, 0); GVPF(2, 1); GVPF(2, 2); GVO(4, true, 0); GVPF(4, 1);
    check_outputs("R=2 CL=true OPT=0");
  }
  const bool dg = argc > 4 && std::string(argv[4]) == "dg";
  // MFMA-diagonal GEMV (k_gemv_4bit_dg, K = 1024 NSEG NWK): the product's row-contiguous loads
#define GVDG(CL_, R, NSEG, NWK) timeit("dg CL=" #CL_ " R=" #R " NSEG=" #NSEG " NWK=" #NWK, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.out_scale = (CL_) ? 1.0f / 16384 : 1.0f; \
    hipLaunchKernelGGL((k_gemv_4bit_dg<CL_, R, NSEG, NWK>), dim3(M / R), dim3(NWK * 64), 0, 0, q); })
  if (dg && K == 4096) {
    GVO(2, true, 0); GVO(2, false, 0);
    GVDG(true, 8, 1, 4); GVDG(false, 8, 1, 4); GVDG(true, 4, 1, 4); GVDG(true, 2, 1, 4); GVDG(true, 4, 2, 2);
    check_outputs("R=2 CL=true OPT=0");
  }
  if (mf && K == 4096) {
    GVO(2, true, 0); GVO(2, false, 0);
    GVMF(true, false); GVMF(true, true); GVMF(false, false);
    GVXL(2); GVXL(4); GVXL(1);
    check_outputs("R=2 CL=true OPT=0");
  }
  const bool stream = argc > 4 && std::string(argv[4]) == "stream";
#define GVST(R, G, CL_) timeit("stream2 R=" #R " wgs=" #G " CL=" #CL_, [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    if (CL_) q.out_scale = 1.0f / 16384; q.tabsel = 0; \
    const int nunits = (M + R - 1) / R; const int g = std::min((int)(G), (nunits + 3) / 4); \
    hipLaunchKernelGGL((k_gemv_4bit_stream2<true, R, CL_>), dim3(g), dim3(256), 0, 0, q, nunits); })
  if (stream) {  // persistent streaming form (K = 4096 rows) vs the production full-step kernel
    GVFS(2, 0); GVFS(4, 0); GVC(4, 0, true);
    GVST(4, 1024, false); GVST(4, 768, false); GVST(4, 512, false); GVST(4, 896, false);
    GVST(2, 1024, false); GVST(2, 768, false); GVST(2, 512, false);
    GVST(1, 1024, false); GVST(8, 1024, false); GVST(8, 512, false);
    GVST(4, 1024, true); GVST(4, 768, true); GVST(2, 1024, true);
  }
  if (!ablate && !small && !r8 && !tab && !tabab && !tabx && !tabfs && !tabxl && !skel && !tabab2 && !cl && !clsweep && !wt && !xcopy && !bf16 && !pk && !wk && !stream && !nopro && !wt8 && !fm && !early && !mf && !dg && !pf && !two && !xf && !ring && !nw8) {
  GV(1, true, 1, 1); GV(1, true, 2, 1); GV(1, true, 4, 1);
  GV(1, true, 1, 2); GV(1, true, 2, 2); GV(1, true, 4, 2);
  GV(1, true, 1, 4); GV(1, true, 2, 4); GV(1, true, 4, 4);
  if (!sweep) { GV(1, false, 2, 2); GV(2, true, 2, 2); }
#define SL(MODE, R, NSW) timeit("sl mode=" #MODE " R=" #R " NSW=" #NSW, [&](int i) { \
    GemvParams q = p; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4)); \
    hipLaunchKernelGGL((k_gemv_4bit_sl<MODE, true, QZ_DT_F16, R, NSW>), dim3(g), dim3(256), 0, 0, q); })
  const int nsw = K / 2048;
  if (nsw == 2) { SL(1, 1, 2); SL(1, 2, 2); SL(1, 4, 2); }
  if (nsw == 4) { SL(1, 1, 4); SL(1, 2, 4); SL(1, 4, 4); }
  if (nsw == 7) { SL(1, 1, 7); SL(1, 2, 7); SL(1, 4, 7); }
  if (nsw == 14) { SL(1, 1, 14); SL(1, 2, 14); SL(1, 4, 14); }
  build_tables(kModeFP4, QZ_FP4, p.tab, &p.out_scale);
  GV(0, true, 2, 2); GV(0, true, 4, 2); GV(0, true, 2, 4);
  if (nsw == 2) { SL(0, 2, 2); SL(0, 4, 2); }
  if (nsw == 4) { SL(0, 2, 4); SL(0, 4, 4); }
  if (nsw == 7) { SL(0, 2, 7); SL(0, 4, 7); }
  if (nsw == 14) { SL(0, 2, 14); SL(0, 4, 14); }
  }
  const bool stamps = argc > 4 && std::string(argv[4]) == "stamps";
  if (stamps) {  // timeline of one steady-state launch (the last of 30 back-to-back), 12 samples each
    const int NWAVES = 1 << 16;
    unsigned long long *sbuf;
    CK(hipMalloc(&sbuf, (size_t)NWAVES * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_qz_stamp), &sbuf, sizeof(sbuf)));
    std::vector<unsigned long long> h((size_t)NWAVES * 8);
    auto run = [&](const char *name, int nwaves, std::function<void(int)> launch) {
      printf("== stamps: %s (%d waves); us from the first wave's start\n", name, nwaves);
      printf("   start p50/p90/max | t1 p50/p90/max | t2 p50/p90/max | t3 p50/max | end p50/p90/max\n");
      for (int smp = 0; smp < 12; ++smp) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 200000LL);
        for (int i = 0; i < 30; ++i) launch(smp * 30 + i);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), sbuf, (size_t)nwaves * 64, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int w = 0; w < nwaves; ++w) t0 = std::min(t0, h[(size_t)w * 8]);
        std::vector<double> c[5];
        for (int w = 0; w < nwaves; ++w)
          for (int k = 0; k < 5; ++k) c[k].push_back((h[(size_t)w * 8 + k] - t0) * 0.01);
        for (int k = 0; k < 5; ++k) std::sort(c[k].begin(), c[k].end());
        auto q = [&](int k, double f) { return c[k][std::min((size_t)(f * nwaves), (size_t)nwaves - 1)]; };
        printf("   %5.2f %5.2f %5.2f | %5.2f %5.2f %5.2f | %5.2f %5.2f %5.2f | %5.2f %5.2f | %5.2f %5.2f %5.2f\n",
               q(0, .5), q(0, .9), q(0, 1), q(1, .5), q(1, .9), q(1, 1), q(2, .5), q(2, .9), q(2, 1), q(3, .5), q(3, 1),
               q(4, .5), q(4, .9), q(4, 1));
        if (smp == 11) {  // per-XCC start / end medians of the last sample
          for (int x = 0; x < 8; ++x) {
            std::vector<double> s0, s4;
            for (int w = 0; w < nwaves; ++w)
              if ((int)(h[(size_t)w * 8 + 5] >> 32) == x) {
                s0.push_back((h[(size_t)w * 8] - t0) * 0.01);
                s4.push_back((h[(size_t)w * 8 + 4] - t0) * 0.01);
              }
            if (s0.empty()) continue;
            std::sort(s0.begin(), s0.end()); std::sort(s4.begin(), s4.end());
            printf("   xcc %d: %zu waves, start med %.2f max %.2f, end med %.2f max %.2f\n", x, s0.size(),
                   s0[s0.size() / 2], s0.back(), s4[s4.size() / 2], s4.back());
          }
        }
      }
    };
    {
      const long long nchunk = pbytes / 16;
      const unsigned g = (unsigned)((nchunk + 255) / 256);
      run("floor T=256 L=1", g * 4, [&](int i) {
        hipLaunchKernelGGL(k_floor_stamp, dim3(g), dim3(256), 0, 0, P[i % NC], (long long)pbytes, sink); });
    }
    {
      const int R = 2;
      const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4));
      run("gemv tab DQ R=2 full-step", g * 4, [&, pt = p](int i) {
        GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC];
        hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, 2, 1, 4, false, 512, true>), dim3(g), dim3(256), 0, 0, q); });
      run("gemv tab DQ R=2 full-step exact codes (product)", g * 4, [&, pt = p](int i) {
        GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384;
        hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, 2, 1, 4, false, 512, true, true>), dim3(g), dim3(256), 0, 0, q); });
      run("gemv tab DQ R=2 full-step exact codes, second step before the barrier (OPT 1)", g * 4, [&, pt = p](int i) {
        GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384;
        hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, 2, 1, 4, false, 512, true, true, false, 0, 1>), dim3(g), dim3(256), 0, 0, q); });
      run("gemv tab DQ R=2 full-step exact codes, straight-line two steps (OPT 8)", g * 4, [&, pt = p](int i) {
        GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384;
        hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, 2, 1, 4, false, 512, true, true, false, 0, 8>), dim3(g), dim3(256), 0, 0, q); });
      run("gemv tab DQ R=2 full-step exact codes, SGPR table (OPT 2)", g * 4, [&, pt = p](int i) {
        GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; q.out_scale = 1.0f / 16384;
        build_exact_planes(q.tab, q.tab_lo);
        hipLaunchKernelGGL((k_gemv_4bit<3, true, QZ_DT_F16, 2, 1, 4, false, 512, true, true, false, 0, 2>), dim3(g), dim3(256), 0, 0, q); });
    }
    return 0;
  }
  const int ROUNDS = argc > 3 ? atoi(argv[3]) : 9;
  for (auto &v : vs) { for (int i = 0; i < NC; ++i) v.launch(i); }
  CK(hipDeviceSynchronize());
  for (int r = 0; r < ROUNDS; ++r)
    for (auto &v : vs) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 2000000LL);  // host enqueues the round meanwhile
      CK(hipEventRecord(e0));
      for (int i = 0; i < ITERS; ++i) v.launch(i);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / ITERS);
    }
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2], mn = v.us[0];
    printf("%-48s median %7.3f  min %7.3f us/launch (b2b)  %7.1f GB/s @median\n", v.name.c_str(), med, mn,
           pbytes / med / 1e3);
  }
  return 0;
}

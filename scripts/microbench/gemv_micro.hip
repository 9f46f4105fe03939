// Standalone GEMV microbenchmark (dev tool, not shipped): one-shot HBM read floor for the
// weight bytes vs the product k_gemv_4bit geometries, rotating 64 weight copies so the 256 MiB
// Infinity Cache never serves repeats.  Printed numbers are hipEvent back-to-back averages
// (kernel + launch gap) over interleaved rounds; `stamps` prints in-kernel wave timelines.
//
//   gemv_micro M K [rounds] [geom|geom8k|stamps]
//
// The losing experiment variants of rounds 1-4 (register v_perm decodes, MFMA decodes, the
// streaming form, step rings, next-launch prefetch, ablation bits) were removed from the product
// source in round 5; their numbers stay in profiles/ and DESIGN.md, their code in git history.
#define QZ_STAMPS 1
#include "../../quantizations_amd/csrc/gemv.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

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

// one-shot floor with timeline stamps (start, data back) per wave
__global__ __launch_bounds__(256) void k_floor_stamp(const unsigned char *__restrict__ p, long long bytes, uint32_t *sink) {
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p) + (c < bytes / 16 ? c : 0));
  uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (acc == 0x12345678u) sink[0] = acc;
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *o = qz::g_qz_stamp + (size_t)(blockIdx.x * 4 + threadIdx.x / 64) * 8;
    o[0] = t0; o[1] = t1; o[2] = t1; o[3] = t1; o[4] = t1; o[5] = 0;
  }
}

// park the stream so the host has enqueued a whole round before the GPU reaches it
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
  const int ROUNDS = argc > 3 ? atoi(argv[3]) : 9;
  const std::string mode = argc > 4 ? argv[4] : "geom";
  const int NC = 64, ITERS = 100;
  const size_t pbytes = (size_t)M * K / 2, nb = (size_t)M * K / 64;
  std::vector<unsigned char *> P(NC), Q(NC);
  std::vector<float *> A2(NC);
  for (int i = 0; i < NC; ++i) {
    CK(hipMalloc(&P[i], pbytes)); CK(hipMalloc(&Q[i], nb)); CK(hipMalloc(&A2[i], (nb / 256 + 1) * 4));
    hipLaunchKernelGGL(k_fill_random, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(P[i]),
                       (long long)(pbytes / 4), 0x1234u + i);
    CK(hipMemset(Q[i], 0x40, nb));
    CK(hipMemset(A2[i], 0x3C, (nb / 256 + 1) * 4));
  }
  float *code2, *off; void *x, *y; uint32_t *sink;
  CK(hipMalloc(&code2, 1024)); CK(hipMemset(code2, 0x3C, 1024)); CK(hipMalloc(&off, 4)); CK(hipMemset(off, 0, 4));
  CK(hipMalloc(&x, (size_t)K * 4)); CK(hipMemset(x, 0x3C, (size_t)K * 4));
  CK(hipMalloc(&y, M * 4)); CK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));

  GemvParams p{};
  p.sc = ScaleSrc{nullptr, nullptr, nullptr, code2, off, 256};
  p.x = x; p.y = y; p.M = M; p.K = K; p.bs_log2 = 6; p.bs2_log2 = 8; p.lut = nullptr; p.bias = nullptr;

  struct Variant { std::string name; std::function<void(int)> launch; std::vector<double> us; };
  std::vector<Variant> vs;
  auto timeit = [&](const std::string &name, std::function<void(int)> launch) { vs.push_back({name, launch, {}}); };
  timeit("floor T=256 L=1", [&](int i) {
    const long long nchunk = pbytes / 16; const unsigned g = (unsigned)((nchunk + 255) / 256);
    hipLaunchKernelGGL((k_read_floor<256, 1>), dim3(g), dim3(256), 0, 0, P[i % NC], (long long)pbytes, sink); });
  // the product kernel at a given geometry: CL = exact codes (tabsel 2, out_scale 2^-14), TWO only at K = 4096
#define GV(R, WK, NW, CL_, WT_, TWO_) timeit("gemv R=" #R " WK=" #WK " NW=" #NW " CL=" #CL_ " WT=" #WT_ " TWO=" #TWO_, \
    [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.tabsel = (CL_) ? 2 : 0; q.out_scale = (CL_) ? 1.0f / 16384 : 1.0f; \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<true, QZ_DT_F16, R, WK, NW, true, CL_, WT_, TWO_>), dim3(g), dim3(NW * 64), 0, 0, q); })
#define GVA(R, NW, ABL) timeit("gemv R=" #R " NW=" #NW " CL TWO abl=" #ABL, \
    [&, pt = p](int i) { \
    GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    q.tabsel = 2; q.out_scale = 1.0f / 16384; \
    const unsigned g = (unsigned)((M + R * NW - 1) / (R * NW)); \
    hipLaunchKernelGGL((k_gemv_4bit<true, QZ_DT_F16, R, 1, NW, true, true, false, true, ABL>), dim3(g), dim3(NW * 64), 0, 0, q); })
  const bool two = K == 4096;
  if (mode == "abl") {  // K = 4096 only: the prologue's table stores (16) and barrier (32) ablated (wrong results)
    GVA(2, 4, 0); GVA(2, 4, 16); GVA(2, 4, 48);
    GV(2, 1, 4, true, true, true); GV(2, 1, 8, true, true, true); GV(1, 1, 8, true, true, true);
    GV(4, 1, 8, true, true, true); GV(1, 1, 4, true, false, true);
  }
  if (mode == "nw16") {  // 16-wave workgroups sharing one wide table (4 waves per SIMD) vs the product's 8
    GV(2, 1, 8, true, true, false); GV(1, 1, 16, true, true, false); GV(2, 1, 16, true, true, false);
    GV(1, 1, 8, true, true, false); GV(4, 1, 16, true, true, false);
  }
  if (mode == "geom") {
    if (two) {
      GV(2, 1, 4, true, false, true); GV(2, 1, 4, false, false, true); GV(4, 1, 4, true, false, true);
      GV(1, 1, 4, true, false, true);
    }
    GV(2, 1, 4, true, false, false); GV(4, 1, 4, true, false, false); GV(4, 2, 4, true, false, false);
    GV(2, 1, 8, true, true, false); GV(4, 1, 8, true, true, false); GV(2, 1, 4, false, false, false);
  }
  if (mode == "geom8k") {  // K = 8192 (Llama-3-70B q/k/v, o, gate/up): K split over 2 / 4 waves, 8-wave tables
    GV(4, 2, 4, true, false, false); GV(2, 2, 4, true, false, false); GV(1, 2, 4, true, false, false);
    GV(2, 4, 4, true, false, false); GV(4, 4, 4, true, false, false); GV(4, 1, 4, true, false, false);
    GV(2, 1, 4, true, false, false); GV(4, 2, 8, true, true, false); GV(2, 2, 8, true, true, false);
    GV(4, 1, 8, true, true, false); GV(2, 1, 8, true, true, false); GV(4, 4, 8, true, true, false);
  }
  if (mode == "stamps") {  // timeline of one steady-state launch (the last of 30 back-to-back), 12 samples each
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
      }
    };
    {
      const long long nchunk = pbytes / 16;
      const unsigned g = (unsigned)((nchunk + 255) / 256);
      run("floor T=256 L=1", g * 4, [&](int i) {
        hipLaunchKernelGGL(k_floor_stamp, dim3(g), dim3(256), 0, 0, P[i % NC], (long long)pbytes, sink); });
    }
    const int R = 2;
    const unsigned g = (unsigned)((M + R * 4 - 1) / (R * 4));
    run("gemv R=2 full-step exact codes (product geometry)", g * 4, [&, pt = p](int i) {
      GemvParams q = pt; q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC];
      q.tabsel = 2; q.out_scale = 1.0f / 16384;
      if (two) hipLaunchKernelGGL((k_gemv_4bit<true, QZ_DT_F16, 2, 1, 4, true, true, false, true, 1>), dim3(g), dim3(256), 0, 0, q);
      else hipLaunchKernelGGL((k_gemv_4bit<true, QZ_DT_F16, 2, 1, 4, true, true, false, false, 1>), dim3(g), dim3(256), 0, 0, q); });
    return 0;
  }
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
    printf("%-56s median %7.3f  min %7.3f us/launch (b2b)  %7.1f GB/s @median\n", v.name.c_str(), med, mn,
           pbytes / med / 1e3);
  }
  return 0;
}

// Dev microbenchmark (not shipped): k_gemm16_4d schedules at config #4's shapes, times and in-kernel
// s_memtime stamps of step 20 (QZ_STAMPS_G16): where a step's cycles go.
//   gemm16_stamps [M K T]
#ifndef NO_STAMPS
#define QZ_STAMPS_G16
#endif
#include "../../quantizations_amd/csrc/gemm.hip"
namespace qz { int &gemm16_sched() { static int v = 971; return v; } }  // the library keeps it in gemv.hip

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_spin(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
__global__ void k_fill_h(uint16_t *p, long long n, uint32_t seed) {   // fp16 in [-1, 1)
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    p[i] = (uint16_t)((h & 0x83FF) | 0x3800 | ((h >> 16) & 0x0400 ? 0x0000 : 0x0000));
  }
}

int main(int argc, char **argv) {
  const int M = argc > 3 ? atoi(argv[1]) : 4096, K = argc > 3 ? atoi(argv[2]) : 4096, T = argc > 3 ? atoi(argv[3]) : 16384;
  void *X, *W, *Y;
  CK(hipMalloc(&X, (size_t)T * K * 2)); CK(hipMalloc(&W, (size_t)M * K * 2)); CK(hipMalloc(&Y, (size_t)T * M * 2));
  hipLaunchKernelGGL(k_fill_h, dim3(2048), dim3(256), 0, 0, (uint16_t *)X, (long long)T * K, 9u);
  hipLaunchKernelGGL(k_fill_h, dim3(2048), dim3(256), 0, 0, (uint16_t *)W, (long long)M * K, 5u);
  GemmParams p{};
  p.X = X; p.Y = Y; p.B = (const unsigned char *)W; p.bias = nullptr;
  p.T = T; p.M = M; p.K = K; p.ldx = K; p.ldy = M; p.k_split = K;
  const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256));
  struct V { std::string n; std::function<void()> f; std::vector<double> us; unsigned long long st[8 * 4 * 16]; };
  std::vector<V> vs;
#define ADD(SK_, S_) vs.push_back({"SK=" #SK_ " S=" #S_, [=]() { hipLaunchKernelGGL((k_gemm16_4d<QZ_DT_F16, SK_, 16, 112, S_>), dim3(g), dim3(256), 0, 0, p); }, {}, {}})
#define ADDQ(S_) vs.push_back({"4q S=" #S_, [=]() { hipLaunchKernelGGL((k_gemm16_4q<QZ_DT_F16, S_>), dim3(std::min(g, 256u)), dim3(256), 0, 0, p); }, {}, {}})
  ADD(64, 0); ADD(65, 0); ADDQ(0); ADDQ(128); ADDQ(384); ADDQ(392);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto &v : vs) v.f();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 9; ++r)
    for (auto &v : vs) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 200000LL);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 4; ++i) v.f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / 4);
#ifndef NO_STAMPS
      CK(hipMemcpyFromSymbol(v.st, HIP_SYMBOL(g_qz_stamp_g16), sizeof(v.st)));
#endif
    }
  printf("M=%d K=%d T=%d fp16 (SK 65 = no DMAs: stale LDS, timing only)\n", M, K, T);
  printf("stamp columns (cycles, medians over 8 workgroups x 4 waves): prologue = start->after prologue barrier;"
         " step 20 from its start: wait1 before/after, wait2 before/after, wait3 before/after, next step start;"
         " loop end -> after vmcnt(0); epilogue\n");
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    auto col = [&](int a, int b) {
      std::vector<long long> d;
      for (int w = 0; w < 32; ++w) {
        const unsigned long long *q = v.st + w * 16;
        if (q[a] && q[b]) d.push_back((long long)(q[b] - q[a]));
      }
      if (d.empty()) return -1LL;
      std::sort(d.begin(), d.end());
      return d[d.size() / 2];
    };
    printf("%-12s %9.2f us %7.1f TF/s | prologue %6lld | w1 %5lld->%5lld w2 %5lld->%5lld w3 %5lld->%5lld step %5lld | tail %5lld epi %5lld\n",
           v.n.c_str(), med, 2.0 * T * M * K / (med * 1e-6) / 1e12, col(0, 1), col(2, 3), col(2, 4), col(2, 5), col(2, 6),
           col(2, 7), col(2, 8), col(2, 9), col(10, 11), col(11, 12));
  }
  return 0;
}

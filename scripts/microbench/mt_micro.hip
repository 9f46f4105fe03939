// Dev microbenchmark (not shipped): the multi-token decode kernel (2..16
// tokens) with B fragments loaded straight from memory (TB = 0) vs staged
// through a wave-private LDS image (TB = token bucket), NF4 + double quant,
// 16 rotating weight copies, stream parked behind a spin kernel.
#include "../../quantizations_amd/csrc/gemm.hip"
namespace qz { int &gemm16_sched() { static int v = 0; return v; } }  // the library keeps it in gemv.hip

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>
#include <string>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_spin(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
__global__ void k_fill(uint32_t *p, long long n, uint32_t seed) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;
    p[i] = h;
  }
}

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 4096;
  const int NC = 16, ITERS = 50, ROUNDS = 7;
  const size_t pbytes = (size_t)M * K / 2, nb = (size_t)M * K / 64;
  std::vector<unsigned char *> P(NC), Q(NC);
  std::vector<float *> A2(NC);
  for (int i = 0; i < NC; ++i) {
    CK(hipMalloc(&P[i], pbytes)); CK(hipMalloc(&Q[i], nb)); CK(hipMalloc(&A2[i], (nb / 256 + 1) * 4));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(P[i]), (long long)(pbytes / 4), 7u + i);
    CK(hipMemset(Q[i], 0x40, nb)); CK(hipMemset(A2[i], 0x3C, (nb / 256 + 1) * 4));
  }
  float *code2, *off; void *X, *Y;
  CK(hipMalloc(&code2, 1024)); CK(hipMemset(code2, 0x3C, 1024)); CK(hipMalloc(&off, 4)); CK(hipMemset(off, 0, 4));
  CK(hipMalloc(&X, 16 * K * 2)); CK(hipMemset(X, 0x3C, 16 * K * 2)); CK(hipMalloc(&Y, 16 * M * 2));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { std::string n; std::function<void(int)> f; std::vector<double> us; };
  std::vector<V> vs;
  GemmParams p{};
  p.X = X; p.Y = Y; p.sc = ScaleSrc{nullptr, nullptr, nullptr, code2, off, 256};
  p.M = M; p.K = K; p.ldx = K; p.ldy = M; p.bs_log2 = 6; p.bs2_log2 = 8; p.k_split = K; p.block_base = 0;
  const unsigned grid = (unsigned)((M + 15) / 16);
#define MT(T_, TB_) vs.push_back({"mt T=" #T_ " TB=" #TB_, [&, pt = p](int i) { GemmParams q = pt; q.T = T_; \
    q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    hipLaunchKernelGGL((k_gemv_4bit_mt<QZ_NF4, true, QZ_DT_F16, TB_>), dim3(grid), dim3(512), 0, 0, q); }, {}})
  const bool waves = argc > 3 && std::string(argv[3]) == "waves";
  // waves-per-workgroup variants (K split W ways inside the workgroup; W = 8 is the product)
#define MTW(T_, TB_, W_) vs.push_back({"mt T=" #T_ " TB=" #TB_ " W=" #W_, [&, pt = p](int i) { GemmParams q = pt; q.T = T_; \
    q.B = P[i % NC]; q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; \
    hipLaunchKernelGGL((k_gemv_4bit_mt<QZ_NF4, true, QZ_DT_F16, TB_, W_>), dim3(grid), dim3(64 * W_), 0, 0, q); }, {}})
  if (waves) {
    MTW(2, 2, 4); MTW(2, 2, 8); MTW(2, 2, 16); MTW(8, 8, 4); MTW(8, 8, 8); MTW(8, 8, 16);
  } else {
    MT(2, 0); MT(2, 2); MT(4, 0); MT(4, 4); MT(8, 0); MT(8, 8); MT(16, 0); MT(16, 16); MT(3, 4); MT(5, 8);
  }
  for (auto &v : vs) for (int i = 0; i < NC; ++i) v.f(i);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < ROUNDS; ++r)
    for (auto &v : vs) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 1000000LL);
      CK(hipEventRecord(e0));
      for (int i = 0; i < ITERS; ++i) v.f(i);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / ITERS);
    }
  printf("M=%d K=%d\n", M, K);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    printf("%-20s median %7.3f  min %7.3f us/launch\n", v.n.c_str(), v.us[v.us.size() / 2], v.us[0]);
  }
  return 0;
}

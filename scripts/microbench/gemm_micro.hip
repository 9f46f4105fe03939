// Dev microbenchmark (not shipped): prefill GEMM kernels on a 4096x4096 (or
// M x K) NF4 + double-quant weight: the 128-row tile kernel (k_gemm_4bit) vs
// the 256x256 tile kernel (k_gemm_4bit_big), random operands, stream parked.
#ifdef STAMPS
#define QZ_STAMPS8P
#endif
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
__global__ void k_fill(uint32_t *p, long long n, uint32_t seed, uint32_t mask, uint32_t orv) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    p[i] = (h & mask) | orv;
  }
}

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 4096;
  const int ROUNDS = 5;
  const size_t pbytes = (size_t)M * K / 2, nb = (size_t)M * K / 64;
  unsigned char *B, *Q; float *A2, *code2, *off; void *X, *Y;
  const int TMAX = 16384;
  CK(hipMalloc(&B, pbytes)); CK(hipMalloc(&Q, nb)); CK(hipMalloc(&A2, (nb / 256 + 1) * 4));
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(B), (long long)(pbytes / 4), 3u, ~0u, 0u);
  CK(hipMemset(Q, 0x40, nb)); CK(hipMemset(A2, 0, (nb / 256 + 1) * 4));
  // absmax2 = 0.01 (0x3C23D70A), code2 = 1.0f: scales ~0.01
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(A2), (long long)(nb / 256 + 1), 0u, 0u, 0x3C23D70Au);
  CK(hipMalloc(&code2, 1024)); hipLaunchKernelGGL(k_fill, dim3(1), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(code2), 256LL, 0u, 0u, 0x3F800000u);
  CK(hipMalloc(&off, 4)); CK(hipMemset(off, 0, 4));
  // random fp16 activations in [-1, 1): sign random, exponent 14 or less
  CK(hipMalloc(&X, (size_t)TMAX * K * 2));
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(X), (long long)TMAX * K / 2, 9u, 0xBBFFBBFFu, 0u);
  CK(hipMalloc(&Y, (size_t)TMAX * M * 2));
  void *W16;  // fp16 weights for the plain-GEMM schedule variant (V = 5)
  CK(hipMalloc(&W16, (size_t)M * K * 2));
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(W16), (long long)M * K / 2, 5u, 0xBBFFBBFFu, 0u);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  GemmParams p{};
  p.X = X; p.Y = Y; p.B = B; p.sc = ScaleSrc{nullptr, Q, A2, code2, off, 256};
  p.M = M; p.K = K; p.ldx = K; p.ldy = M; p.bs_log2 = 6; p.bs2_log2 = 8; p.k_split = K; p.block_base = 0; p.ws = nullptr;
  p.bias = nullptr;
  struct V { std::string n; int T; std::function<void()> f; std::vector<double> us; };
  std::vector<V> vs;
  const int Ts[] = {4096, 16384};
  for (int T : Ts) {
    vs.push_back({"old128 T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T;
      hipLaunchKernelGGL((k_gemm_4bit<QZ_NF4, true, QZ_DT_F16, 128>), dim3((M + 127) / 128, (T + 127) / 128, 1), dim3(256), 0, 0, q); }, {}});
#define BIGV(V_) vs.push_back({"big256 V=" #V_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
      const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256)); \
      hipLaunchKernelGGL((k_gemm_4bit_big<QZ_NF4, true, QZ_DT_F16, V_>), dim3(g), dim3(512), 0, 0, q); }, {}})
#define P8V(V_) vs.push_back({"8phase V=" #V_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
      const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256)); \
      hipLaunchKernelGGL((k_gemm_4bit_8p<QZ_NF4, true, QZ_DT_F16, V_>), dim3(g), dim3(512), 0, 0, q); }, {}})
#define PLV(SK_) vs.push_back({"plain fp16 GEMM SK=" #SK_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
        q.B = reinterpret_cast<const unsigned char *>(W16); \
        const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256)); \
        hipLaunchKernelGGL((k_gemm_4bit_8p<QZ_NF4, false, QZ_DT_F16, 5, SK_>), dim3(g), dim3(512), 0, 0, q); }, {}})
#define P4W(SK_) vs.push_back({"4wave fp16 GEMM SK=" #SK_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
      q.B = reinterpret_cast<const unsigned char *>(W16); const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256)); \
      hipLaunchKernelGGL((k_gemm16_4w<QZ_DT_F16, SK_>), dim3(g), dim3(256), 0, 0, q); }, {}})
#define P4D(SK_, P1_, P2_) vs.push_back({"4wave-dma fp16 GEMM SK=" #SK_ " P=" #P1_ "," #P2_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
      q.B = reinterpret_cast<const unsigned char *>(W16); const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256)); \
      hipLaunchKernelGGL((k_gemm16_4d<QZ_DT_F16, SK_, P1_, P2_>), dim3(g), dim3(256), 0, 0, q); }, {}})
#define P4P(SK_) vs.push_back({"4wave-persistent fp16 GEMM SK=" #SK_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
      q.B = reinterpret_cast<const unsigned char *>(W16); const unsigned g = (unsigned)std::min(((M + 255) / 256) * ((T + 255) / 256), 256); \
      hipLaunchKernelGGL((k_gemm16_4p<QZ_DT_F16, SK_>), dim3(g), dim3(256), 0, 0, q); }, {}})
#define P8S(SK_) vs.push_back({"8phase V=0 SK=" #SK_ " T=" + std::to_string(T), T, [=]() { GemmParams q = p; q.T = T; \
        const unsigned g = (unsigned)(((M + 255) / 256) * ((T + 255) / 256)); \
        hipLaunchKernelGGL((k_gemm_4bit_8p<QZ_NF4, true, QZ_DT_F16, 0, SK_>), dim3(g), dim3(512), 0, 0, q); }, {}})
    if (T >= 4096) { PLV(1); P4D(64, 16, 112); P4P(0); P4P(128); }
  }
  for (auto &v : vs) v.f();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < ROUNDS; ++r)
    for (auto &v : vs) {
      const int it = v.T >= 4096 ? 3 : 10;
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 500000LL);
      CK(hipEventRecord(e0));
      for (int i = 0; i < it; ++i) v.f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / it);
    }
  printf("M=%d K=%d NF4+DQ f16, random operands\n", M, K);
  {  // grouped tile order (SK 65) vs SK 1: same tiles, must be bit-identical
    void *Y2; CK(hipMalloc(&Y2, (size_t)4096 * M * 2));
    GemmParams q = p; q.T = 4096;
    const unsigned g = (unsigned)(((M + 255) / 256) * ((4096 + 255) / 256));
    for (int plain = 0; plain < 2; ++plain) {
      GemmParams a = q, b2 = q; b2.Y = Y2;
      if (plain) { a.B = b2.B = reinterpret_cast<const unsigned char *>(W16); }
      if (plain) {
        hipLaunchKernelGGL((k_gemm_4bit_8p<QZ_NF4, false, QZ_DT_F16, 5, 1>), dim3(g), dim3(512), 0, 0, a);
        hipLaunchKernelGGL((k_gemm16_4p<QZ_DT_F16, 0>), dim3(std::min(g, 256u)), dim3(256), 0, 0, b2);
      } else {
        hipLaunchKernelGGL((k_gemm_4bit_8p<QZ_NF4, true, QZ_DT_F16, 0, 1>), dim3(g), dim3(512), 0, 0, a);
        hipLaunchKernelGGL((k_gemm_4bit_8p<QZ_NF4, true, QZ_DT_F16, 0, 65>), dim3(g), dim3(512), 0, 0, b2);
      }
      CK(hipDeviceSynchronize());
      std::vector<uint16_t> h1((size_t)4096 * M), h2((size_t)4096 * M);
      CK(hipMemcpy(h1.data(), Y, h1.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), Y2, h2.size() * 2, hipMemcpyDeviceToHost));
      double maxd = 0, maxv = 0; size_t ndiff = 0;
      for (size_t i = 0; i < h1.size(); ++i) {
        const float a1 = (float)__builtin_bit_cast(_Float16, h1[i]), a2 = (float)__builtin_bit_cast(_Float16, h2[i]);
        maxd = std::max(maxd, (double)std::fabs(a1 - a2)); maxv = std::max(maxv, (double)std::fabs(a1));
        ndiff += h1[i] != h2[i];
      }
      printf("check %s: 4wave-persistent(plain)/SK65(fused) vs 8phase SK1 max|diff| %.4g (max|y| %.4g), %zu of %zu elements differ\n", plain ? "plain" : "fused",
             maxd, maxv, ndiff, h1.size());
    }
  }
#ifdef STAMPS
  {
    unsigned long long h[2 * 8 * 16];
    CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_qz_stamp8p), sizeof(h)));
    printf("stamps (step 10, shader clocks rel. to wave 0's first stamp): per phase [read-seg, wait barrier1, mfma, wait barrier2]\n");
    for (int wgi = 0; wgi < 2; ++wgi)
      for (int w = 0; w < 8; ++w) {
        const unsigned long long *q = h + (wgi * 8 + w) * 16, base = h[wgi * 8 * 16];
        printf("wg%d w%d:", wgi, w);
        for (int k = 0; k < 9; ++k) printf(" %6lld", (long long)(q[k] - base));
        printf("\n");
      }
  }
#endif
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-20s median %9.2f us  %7.1f TFLOP/s\n", v.n.c_str(), med, 2.0 * v.T * M * K / (med * 1e-6) / 1e12);
  }
  return 0;
}

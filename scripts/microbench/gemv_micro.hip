// Standalone GEMV microbenchmark (dev tool, not shipped): one-shot HBM read
// floor for an 8 MiB weight vs k_gemv_4bit variants, rotating 64 weight copies
// so the 256 MiB Infinity Cache never serves repeats.  Run under
// `rocprofv3 --kernel-trace --stats` for kernel-only durations; the printed
// numbers are hipEvent back-to-back averages (kernel + launch gap).
#include "../../quantizations_amd/csrc/gemv.hip"

#include <cstdio>
#include <cstdlib>
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

int main(int argc, char **argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 4096;
  const int NC = 64, ITERS = 300;
  const size_t pbytes = (size_t)M * K / 2, nb = (size_t)M * K / 64;
  std::vector<unsigned char *> P(NC), Q(NC);
  std::vector<float *> A2(NC), A(NC);
  for (int i = 0; i < NC; ++i) {
    CK(hipMalloc(&P[i], pbytes)); CK(hipMalloc(&Q[i], nb)); CK(hipMalloc(&A2[i], (nb / 256 + 1) * 4));
    CK(hipMalloc(&A[i], nb * 4));
    CK(hipMemset(P[i], 0x5A + i, pbytes)); CK(hipMemset(Q[i], 0x40, nb));
    CK(hipMemset(A2[i], 0x3C, (nb / 256 + 1) * 4)); CK(hipMemset(A[i], 0x3C, nb * 4));
  }
  float *code2, *off; void *x, *y; uint32_t *sink;
  CK(hipMalloc(&code2, 1024)); CK(hipMemset(code2, 0x3C, 1024)); CK(hipMalloc(&off, 4)); CK(hipMemset(off, 0, 4));
  CK(hipMalloc(&x, K * 4)); CK(hipMemset(x, 0x3C, K * 4)); CK(hipMalloc(&y, M * 4)); CK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));

  auto timeit = [&](const char *name, auto launch) {
    for (int i = 0; i < 2 * NC; ++i) launch(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < ITERS; ++i) launch(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / ITERS;
    printf("%-44s %8.3f us/launch (b2b)  %7.1f GB/s of %zu B\n", name, us, pbytes / us / 1e3, pbytes);
  };

#define FLOOR(T, L) timeit("floor T=" #T " L=" #L, [&](int i) { \
    const long long nchunk = pbytes / 16; const unsigned g = (unsigned)((nchunk + (long long)T * L - 1) / ((long long)T * L)); \
    hipLaunchKernelGGL((k_read_floor<T, L>), dim3(g), dim3(T), 0, 0, P[i % NC], (long long)pbytes, sink); })
  FLOOR(256, 1); FLOOR(256, 2); FLOOR(256, 4); FLOOR(256, 8); FLOOR(512, 4); FLOOR(1024, 2); FLOOR(1024, 4);

  GemvParams p{};
  p.sc = ScaleSrc{nullptr, nullptr, nullptr, code2, off, 256};
  p.x = x; p.y = y; p.M = M; p.K = K; p.bs_log2 = 6; p.bs2_log2 = 8; p.lut = nullptr; p.bias = nullptr;
  build_tables(kModeLUT16, QZ_NF4, p.tab, &p.out_scale);
#define GVN(MODE, DQ, R, WK, NW) timeit("gemv mode=" #MODE " dq=" #DQ " R=" #R " WK=" #WK " NW=" #NW, [&](int i) { \
    GemvParams q = p; q.B = P[i % NC]; \
    if (DQ) { q.sc.qabsmax = Q[i % NC]; q.sc.absmax2 = A2[i % NC]; } else { q.sc.absmax = A[i % NC]; } \
    const unsigned g = (unsigned)((M + R * (NW / WK) - 1) / (R * (NW / WK))); \
    hipLaunchKernelGGL((k_gemv_4bit<MODE, DQ, QZ_DT_F16, R, WK, NW>), dim3(g), dim3(NW * 64), 0, 0, q); })
#define GV(MODE, DQ, R, WK) GVN(MODE, DQ, R, WK, 4)
  GV(1, true, 4, 2); GV(1, true, 2, 2); GV(1, true, 1, 2); GV(1, true, 4, 1); GV(1, true, 2, 1); GV(1, true, 1, 1);
  GV(1, false, 4, 2); GV(1, false, 2, 2); GV(1, false, 2, 1);
  GV(2, true, 2, 1); GV(2, false, 2, 1); GV(2, false, 1, 1); GV(2, false, 4, 1); GV(2, false, 2, 2);
  GVN(2, false, 2, 1, 8); GVN(2, false, 2, 1, 16); GVN(1, true, 2, 1, 8); GVN(1, true, 2, 1, 16); GVN(1, true, 1, 1, 16);
  GVN(1, true, 2, 2, 8); GVN(1, true, 4, 1, 16);
  build_tables(kModeFP4, QZ_FP4, p.tab, &p.out_scale);
  GV(0, true, 4, 2); GV(0, true, 2, 2); GV(0, true, 1, 2);
  return 0;
}

// Dev microbenchmark (not shipped): what a single launch that streams the
// 4096^2 GEMV's 8.4 MB costs on MI355X, decomposed -- empty launches, one-shot
// read floors over several geometries / load kinds, and the write drain of an
// 8 KB result.  64 rotating buffers (> the 256 MiB Infinity Cache).  Printed
// numbers are back-to-back hipEvent averages with the stream parked behind a
// spin kernel while the host enqueues (so they time the GPU, not submission); run under rocprofv3
// --kernel-trace --stats for kernel-only durations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <functional>
#include <string>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

__global__ void k_empty(uint32_t *sink) {
  if (threadIdx.x == 1023) sink[0] = 1;  // never true (blockDim <= 256)
}

// KIND 0: non-temporal, 1: plain, 2: glc|slc (streaming) via builtin
template <int T, int L, int KIND>
__global__ __launch_bounds__(T) void k_floor(const unsigned char *__restrict__ p, long long nchunk, uint32_t *sink) {
  uint32_t acc = 0;
  v4 v[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const long long c = ((long long)blockIdx.x * L + i) * T + threadIdx.x;
    const v4 *q = reinterpret_cast<const v4 *>(p) + (c < nchunk ? c : 0);
    if constexpr (KIND == 0) v[i] = __builtin_nontemporal_load(q);
    else v[i] = *q;
  }
#pragma unroll
  for (int i = 0; i < L; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  if (acc == 0x12345678u) sink[0] = acc;
}

// the same, with the block's results written at the end: SK 0 = no store,
// 1 = 2 plain dword stores per wave (the GEMV's y pattern at R = 2), 2 = same with nt stores
template <int T, int L, int SK>
__global__ __launch_bounds__(T) void k_floor_st(const unsigned char *__restrict__ p, long long nchunk, uint32_t *out) {
  uint32_t acc = 0;
  v4 v[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const long long c = ((long long)blockIdx.x * L + i) * T + threadIdx.x;
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p) + (c < nchunk ? c : 0));
  }
#pragma unroll
  for (int i = 0; i < L; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  const int lane = threadIdx.x & 63;
  const long long o = ((long long)blockIdx.x * T + threadIdx.x) / 32;
  if constexpr (SK == 1) { if (lane >= 62) out[o] = acc; }
  if constexpr (SK == 2) { if (lane >= 62) __builtin_nontemporal_store(acc, out + o); }
}

// park the stream (~20 ms) so the host has enqueued a whole round before the GPU reaches it
__global__ void k_spin(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

__global__ void k_fill(uint32_t *p, long long n, uint32_t seed) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i * 0x9E3779B1u ^ seed;
}

int main(int argc, char **argv) {
  const long long bytes = argc > 1 ? atoll(argv[1]) : 8388608LL;
  const int ROUNDS = argc > 2 ? atoi(argv[2]) : 9;
  const int NC = 64, ITERS = 100;
  std::vector<unsigned char *> P(NC);
  for (int i = 0; i < NC; ++i) {
    CK(hipMalloc(&P[i], bytes));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(P[i]), bytes / 4, 77u + i);
  }
  uint32_t *sink, *out;
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&out, 1 << 24));
  const long long nchunk = bytes / 16;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V { std::string n; std::function<void(int)> f; std::vector<double> us; };
  std::vector<V> vs;
  auto add = [&](std::string n, std::function<void(int)> f) { vs.push_back({n, f, {}}); };
  add("empty grid=1 x64", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, sink); });
  add("empty grid=2048 x256", [&](int) { hipLaunchKernelGGL(k_empty, dim3(2048), dim3(256), 0, 0, sink); });
  add("empty grid=8192 x256", [&](int) { hipLaunchKernelGGL(k_empty, dim3(8192), dim3(256), 0, 0, sink); });
#define FL(T, L, KIND) add("floor T=" #T " L=" #L " kind=" #KIND, [&](int i) { \
    const unsigned g = (unsigned)((nchunk + (long long)T * L - 1) / ((long long)T * L)); \
    hipLaunchKernelGGL((k_floor<T, L, KIND>), dim3(g), dim3(T), 0, 0, P[i % NC], nchunk, sink); })
  FL(256, 1, 0); FL(256, 2, 0); FL(256, 4, 0); FL(256, 8, 0); FL(256, 16, 0);
  FL(512, 2, 0); FL(512, 4, 0); FL(1024, 1, 0); FL(1024, 2, 0); FL(1024, 4, 0);
  FL(64, 1, 0); FL(64, 4, 0); FL(128, 2, 0); FL(128, 4, 0);
  FL(256, 1, 1); FL(256, 2, 1); FL(256, 4, 1);
#define FS(T, L, SK) add("floor+store T=" #T " L=" #L " sk=" #SK, [&](int i) { \
    const unsigned g = (unsigned)((nchunk + (long long)T * L - 1) / ((long long)T * L)); \
    hipLaunchKernelGGL((k_floor_st<T, L, SK>), dim3(g), dim3(T), 0, 0, P[i % NC], nchunk, out); })
  FS(256, 2, 0); FS(256, 2, 1); FS(256, 2, 2); FS(256, 4, 1); FS(256, 4, 2);
  for (auto &v : vs) for (int i = 0; i < NC; ++i) v.f(i);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < ROUNDS; ++r)
    for (auto &v : vs) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 2000000LL);  // 20 ms at the 100 MHz wall clock
      CK(hipEventRecord(e0));
      for (int i = 0; i < ITERS; ++i) v.f(i);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / ITERS);
    }
  printf("buffer %lld B\n", bytes);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-36s median %7.3f  min %7.3f us/launch (b2b)  %7.1f GB/s @median\n", v.n.c_str(), med, v.us[0],
           bytes / med / 1e3);
  }
  return 0;
}

// prefetch.hip -- warming the die-level Infinity Cache (256 MiB) with a decode step's NEXT weights.
//
// A batch-1 decode step reads every weight byte once, launch after launch, and each launch spends
// its ramp, prologue and drain with HBM partly idle (the four Linear4bit
// launches of a Llama-3-8B layer average 0.37 of peak).  The weights do not depend on the
// activations, so a second stream can stream layer L + 1's bytes from HBM while layer L computes:
// a line stays in the Infinity Cache while the bytes moved between its two uses fit in about
// 256 MiB (MI355X_MICROARCH.md, Infinity Cache), i.e. one Llama-3-8B layer ahead (2 x 113 MB).
// k_prefetch loads every 16-B piece of up to kPrefetchMaxSeg byte ranges once, with the default
// cache policy, and discards it (a data-dependent store that never fires keeps the loads alive).
// Nothing is written: running it or not changes no result, only where the consumers' loads hit.
#include <atomic>

#include "common.h"

namespace qz {
namespace {

constexpr int kPrefetchMaxSeg = 16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct PrefetchArgs {
  const unsigned char *p[kPrefetchMaxSeg];
  unsigned long long end[kPrefetchMaxSeg];   // prefix sums of the segments' 16-B pieces
  unsigned long long total;
  int nseg;
  uint32_t magic;
  uint32_t *sink;
};

// U pieces in flight per lane (16 U bytes), one wave per workgroup, grid-stride over the pieces
template <int U>
__global__ __launch_bounds__(64) void k_prefetch(PrefetchArgs a) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 64ull * U;
  uint32_t acc = 0;
  for (unsigned long long base = (unsigned long long)blockIdx.x * 64ull * U + threadIdx.x; base < a.total;
       base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned long long idx = base + 64ull * u;
      v[u] = u32x4{0u, 0u, 0u, 0u};
      if (idx < a.total) {
        int s = 0;
        unsigned long long start = 0;
#pragma unroll
        for (int j = 0; j < kPrefetchMaxSeg - 1; ++j)
          if (j < a.nseg - 1 && idx >= a.end[j]) { s = j + 1; start = a.end[j]; }
        v[u] = reinterpret_cast<const u32x4 *>(a.p[s])[idx - start];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == a.magic) a.sink[threadIdx.x] = acc;   // a 2^-32 event per lane; the sink is the caller's scratch
}

int cus_of_current_device() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int c = cache[dev].load(std::memory_order_relaxed);
  if (c <= 0) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cache[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

}  // namespace
}  // namespace qz

using namespace qz;

extern "C" int qz_prefetch_l3(int nseg, const void *const *ptrs, const long long *bytes, int workgroups, int depth,
                              unsigned int *sink, void *stream) {
  if (nseg < 0 || nseg > kPrefetchMaxSeg || workgroups < 0 || (depth != 0 && depth != 4 && depth != 8 && depth != 16))
    return QZ_ERR_ARG;
  if (nseg == 0) return QZ_OK;
  if (!ptrs || !bytes || !sink) return QZ_ERR_ARG;
  PrefetchArgs a{};
  unsigned long long tot = 0;
  int n = 0;
  for (int i = 0; i < nseg; ++i) {
    if (!ptrs[i] || bytes[i] < 0) return QZ_ERR_ARG;
    // whole aligned 16-B pieces inside the range (a ragged head or tail is not worth a load)
    const uintptr_t b0 = ((uintptr_t)ptrs[i] + 15u) & ~(uintptr_t)15u;
    const uintptr_t b1 = ((uintptr_t)ptrs[i] + (uintptr_t)bytes[i]) & ~(uintptr_t)15u;
    if (b1 <= b0) continue;
    a.p[n] = reinterpret_cast<const unsigned char *>(b0);
    tot += (unsigned long long)((b1 - b0) >> 4);
    a.end[n] = tot;
    ++n;
  }
  if (n == 0) return QZ_OK;
  a.nseg = n;
  a.total = tot;
  a.magic = 0x9E3779B9u;
  a.sink = sink;
  const int wgs = workgroups > 0 ? workgroups : 2 * cus_of_current_device();
  hipStream_t st = (hipStream_t)stream;
  if (depth == 4) hipLaunchKernelGGL((k_prefetch<4>), dim3((unsigned)wgs), dim3(64), 0, st, a);
  else if (depth == 16) hipLaunchKernelGGL((k_prefetch<16>), dim3((unsigned)wgs), dim3(64), 0, st, a);
  else hipLaunchKernelGGL((k_prefetch<8>), dim3((unsigned)wgs), dim3(64), 0, st, a);
  return (int)hipGetLastError();
}

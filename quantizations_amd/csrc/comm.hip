// comm.hip -- one-shot all-gather of the row-split decode outputs over xGMI (SURVEY.md 8(e),
// DESIGN.md section 6): the exchange step of RowShardedLinear4bit without a collective library.
//
// Every rank owns one exchange buffer in UNCACHED device memory (hipDeviceMallocUncached: no
// cache of any GPU holds its lines, so a peer's store over xGMI is what the owner's next load
// sees) and maps its peers' buffers through hipIpc handles.  One launch of k_allgather_oneshot
// (one workgroup) per all-gather:
//   1. push: the rank's shard (the GEMV output) is stored into slot [parity][rank] of EVERY
//      rank's buffer, its own included -- remote stores go straight over xGMI;
//   2. signal: after its stores have completed (vmcnt(0), workgroup barrier), one lane per peer
//      stores the call's epoch into flag [parity][rank] of that peer's buffer (system scope);
//      every byte a peer reads lives in uncached memory, so no cache write-back (release
//      fence) is needed -- only the stores' completion;
//   3. wait: one lane per peer polls flag [parity][peer] of the OWN buffer (system-scope loads,
//      bounded spin: a peer that never arrives sets the status word instead of hanging the GPU),
//      then the uncached slots are read (no cache to invalidate);
//   4. unpack: the world x nbytes slots are copied into the output tensor (ordinary memory, so
//      the consumers of the gathered activation read it through the caches as usual).
// The epoch is a device-side counter (read at entry, advanced at exit by the same launch), so
// the launch is HIP-graph capturable with fixed arguments.  Slots alternate by epoch parity: a
// peer can be at most one call ahead (it cannot finish call e+1 before this rank has signalled
// e+1, i.e. finished call e), so call e+1's pushes never land in the slots call e still reads.
#include <cstring>

#include "common.h"

namespace qz {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kAgThreads = 1024;
constexpr int kAgMaxWorld = 8;
constexpr int kAgFlagBytes = 256;   // flags [2][32] u32 (one 128-B line per parity) at the buffer's head

struct AllGatherParams {
  const void *src;                    // this rank's shard, nbytes (16-B aligned)
  void *dst;                          // world * nbytes, rank-major (all_gather_into_tensor order)
  unsigned char *peer[kAgMaxWorld];   // every rank's exchange buffer, mapped here (own included)
  unsigned char *own;                 // this rank's exchange buffer
  unsigned int *epoch;                // device counter (ordinary memory)
  unsigned int *status;               // 0 = ok; 1 = a peer's flag never arrived
  long long slot_bytes;               // bytes per (parity, rank) slot
  int nbytes, rank, world;
};

__device__ __forceinline__ unsigned int *ag_flag(unsigned char *buf, int par, int r) {
  return reinterpret_cast<unsigned int *>(buf) + par * 32 + r;
}

__global__ __launch_bounds__(kAgThreads) void k_allgather_oneshot(AllGatherParams p) {
  const int tid = threadIdx.x;
  const unsigned int epoch = *p.epoch + 1u;
  const int par = (int)(epoch & 1u);
  const int n16 = p.nbytes >> 4;
  const long long slot0 = kAgFlagBytes + (long long)par * p.world * p.slot_bytes;
  // 1. push the shard into every rank's slot [par][rank]
  const v4u *src = reinterpret_cast<const v4u *>(p.src);
  for (int i = tid; i < n16; i += kAgThreads) {
    const v4u v = src[i];
#pragma unroll
    for (int r = 0; r < kAgMaxWorld; ++r) {
      if (r < p.world)
        reinterpret_cast<v4u *>(p.peer[r] + slot0 + (long long)p.rank * p.slot_bytes)[i] = v;
    }
  }
  // 2. every store of this workgroup has completed, then the epoch goes to each peer
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // (no release fence: the shard went to UNCACHED memory, so no cache holds anything a peer
  // must see -- a fence's L2 write-back would only flush unrelated dirty lines, ~2 us)
  if (tid < p.world)
    __hip_atomic_store(ag_flag(p.peer[tid], par, p.rank), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every peer's epoch in the own buffer (bounded: ~1 s, then report and go on)
  if (tid < p.world) {
    unsigned int *f = ag_flag(p.own, par, tid);
    long long spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1LL << 24)) {
        __hip_atomic_store(p.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  // 4. unpack the world slots (uncached) into the output
  v4u *dst = reinterpret_cast<v4u *>(p.dst);
  const int total = n16 * p.world;
  for (int i = tid; i < total; i += kAgThreads) {
    const int r = i / n16, j = i - r * n16;
    dst[i] = reinterpret_cast<const v4u *>(p.own + slot0 + (long long)r * p.slot_bytes)[j];
  }
  // 5. the next call's epoch (every thread has read this one: the barrier above)
  if (tid == 0) *p.epoch = epoch;
}

}  // namespace qz

using namespace qz;

extern "C" int qz_ipc_handle_size(void) { return (int)sizeof(hipIpcMemHandle_t); }

extern "C" int qz_exchange_alloc(long long bytes, void **ptr) {
  if (!ptr || bytes <= 0) return QZ_ERR_ARG;
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}

extern "C" int qz_exchange_free(void *ptr) { return (int)hipFree(ptr); }

extern "C" int qz_ipc_get_handle(const void *ptr, void *handle) {
  if (!ptr || !handle) return QZ_ERR_ARG;
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t *>(handle), const_cast<void *>(ptr));
}

extern "C" int qz_ipc_open_handle(const void *handle, void **ptr) {
  if (!handle || !ptr) return QZ_ERR_ARG;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int qz_ipc_close_handle(void *ptr) { return (int)hipIpcCloseMemHandle(ptr); }

extern "C" int qz_enable_peer_access(int peer_device) {
  int dev = 0, can = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  if (peer_device == dev) return QZ_OK;
  e = hipDeviceCanAccessPeer(&can, dev, peer_device);
  if (e != hipSuccess) return (int)e;
  if (!can) return QZ_ERR_ARG;
  e = hipDeviceEnablePeerAccess(peer_device, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return QZ_OK;
  }
  return (int)e;
}

extern "C" int qz_allgather_oneshot(const void *src, int nbytes, void *dst, int rank, int world,
                                    void *const *peer_bufs, void *own_buf, long long slot_bytes, unsigned int *epoch,
                                    unsigned int *status, void *stream) {
  if (!src || !dst || !peer_bufs || !own_buf || !epoch || !status || nbytes < 0) return QZ_ERR_ARG;
  if (world < 1 || world > kAgMaxWorld || rank < 0 || rank >= world) return QZ_ERR_ARG;
  if (nbytes % 16 != 0 || nbytes > slot_bytes || slot_bytes % 16 != 0 ||
      (reinterpret_cast<uintptr_t>(src) % 16) != 0 || (reinterpret_cast<uintptr_t>(dst) % 16) != 0)
    return QZ_ERR_SHAPE;
  AllGatherParams p{};
  p.src = src;
  p.dst = dst;
  for (int r = 0; r < world; ++r) {
    if (!peer_bufs[r]) return QZ_ERR_ARG;
    p.peer[r] = reinterpret_cast<unsigned char *>(peer_bufs[r]);
  }
  p.own = reinterpret_cast<unsigned char *>(own_buf);
  p.epoch = epoch;
  p.status = status;
  p.slot_bytes = slot_bytes;
  p.nbytes = nbytes;
  p.rank = rank;
  p.world = world;
  hipLaunchKernelGGL(k_allgather_oneshot, dim3(1), dim3(kAgThreads), 0, (hipStream_t)stream, p);
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" long long qz_exchange_bytes(int world, long long slot_bytes) {
  return kAgFlagBytes + 2LL * world * slot_bytes;
}

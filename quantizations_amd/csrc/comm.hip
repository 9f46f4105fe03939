// comm.hip -- one-shot all-gather of the row-split decode outputs over xGMI (SURVEY.md 8(e),
// DESIGN.md section 6): the exchange step of RowShardedLinear4bit without a collective library.
//
// Every rank owns one exchange buffer in UNCACHED device memory (hipDeviceMallocUncached: no
// cache of any GPU holds its lines, so a peer's store over xGMI is what the owner's next load
// sees) and maps its peers' buffers through hipIpc handles.  The payload travels as TAGGED
// GRANULES: every 4-byte word of a shard is stored as one 8-byte {word, epoch} granule by a
// single 8-byte system-scope store, so a reader knows a word has arrived when its tag equals
// the call's epoch -- no separate flag, no store-completion wait, no cache fence, one xGMI
// trip per word (the guide's granule hand-off, MI355X_MICROARCH.md price list).
// Payloads up to QZ_AG_GRANULE_MAX_BYTES: one launch of k_allgather_granules, one 1024-thread
// workgroup per rank (larger payloads: k_allgather_flags below):
//   1. push: workgroup b stores granules of words [b, b + 1) * nwords / world of this rank's
//      shard into region [parity][rank] of EVERY rank's buffer (its own included);
//   2. pull: workgroup b polls the granules of rank b's region in the OWN buffer (all of a
//      thread's loads in flight at once, re-polling the ones not yet tagged; bounded, 5 s: a
//      peer that never arrives sets the status word instead of hanging the GPU) and writes the
//      words into the output (ordinary memory), rank-major.
// The epoch is a device-side counter: every workgroup reads it at entry and the last one to
// finish (an agent-scope ticket) advances it, so the launch is HIP-graph capturable with fixed
// arguments.  Regions alternate by epoch parity: a peer can be at most one call ahead (it cannot
// finish call e+1 before this rank has pushed e+1, i.e. finished call e), so call e+1's granules
// never land in the region call e still reads; a stale granule there carries epoch e-1 or e-2.
#include <cstring>

#include "common.h"

#ifndef QZ_AG_GRANULE_MAX_BYTES
#define QZ_AG_GRANULE_MAX_BYTES 2048
#endif

namespace qz {

constexpr int kAgThreads = 1024;
constexpr int kAgMaxWorld = 8;
constexpr int kAgHeadBytes = 256;   // buffer head: the flags [2][32] u32 of the flag protocol
constexpr int kAgPoll = 8;          // granules per thread per polling round
// a peer that never arrives: give up after 5 s of the 100 MHz s_memrealtime clock (the status
// word reports it) -- long enough for any rank skew of a healthy job, bounded so a dead peer
// cannot hang the GPU
constexpr unsigned long long kAgWaitTicks = 500000000ull;

struct AllGatherParams {
  const void *src;                    // this rank's shard, nbytes (16-B aligned)
  void *dst;                          // world * nbytes, rank-major (all_gather_into_tensor order)
  unsigned char *peer[kAgMaxWorld];   // every rank's exchange buffer, mapped here (own included)
  unsigned char *own;                 // this rank's exchange buffer
  unsigned int *epoch;                // device counter (ordinary memory) + ticket at epoch[1]
  unsigned int *status;               // 0 = ok; 1 = a peer's granules never arrived
  long long slot_bytes;               // payload bytes per (parity, rank) region (granules: 2x)
  int nbytes, rank, world;
};

// granule i of rank q's region, parity par, in buffer buf
__device__ __forceinline__ unsigned long long *ag_granule(unsigned char *buf, int par, int q, int world,
                                                         long long slot_bytes) {
  return reinterpret_cast<unsigned long long *>(buf + kAgHeadBytes + ((long long)par * world + q) * 2 * slot_bytes);
}
// flag protocol: rank q's plain slot (after all granule regions) and its flag, parity par
__device__ __forceinline__ unsigned char *ag_slot(unsigned char *buf, int par, int q, int world, long long slot_bytes) {
  return buf + kAgHeadBytes + 4LL * world * slot_bytes + ((long long)par * world + q) * slot_bytes;
}
__device__ __forceinline__ unsigned int *ag_flag(unsigned char *buf, int par, int q) {
  return reinterpret_cast<unsigned int *>(buf) + par * 32 + q;
}
// the last workgroup of a launch to finish advances the epoch (all have read it by then)
__device__ __forceinline__ void ag_advance_epoch(unsigned int *ep, unsigned int epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int t = __hip_atomic_fetch_add(ep + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned int)(gridDim.x - 1)) {
      __hip_atomic_store(ep + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ep, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Flag protocol (large payloads: 16-B stores, half the bytes of the granules, but one more
// xGMI trip): one workgroup stores the shard into slot [parity][rank] of every rank, waits for
// the stores' completion, stores the epoch into each rank's flag [parity][rank] (system scope),
// polls its own flags, then copies the world slots out.  No cache fence: all of it is uncached.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(kAgThreads) void k_allgather_flags(AllGatherParams p) {
  const int tid = threadIdx.x;
  const unsigned int epoch = p.epoch[0] + 1u;
  const int par = (int)(epoch & 1u);
  const int n16 = p.nbytes >> 4;
  const v4u *src = reinterpret_cast<const v4u *>(p.src);
  for (int i = tid; i < n16; i += kAgThreads) {
    const v4u v = src[i];
#pragma unroll
    for (int r = 0; r < kAgMaxWorld; ++r) {
      if (r < p.world) reinterpret_cast<v4u *>(ag_slot(p.peer[r], par, p.rank, p.world, p.slot_bytes))[i] = v;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < p.world)
    __hip_atomic_store(ag_flag(p.peer[tid], par, p.rank), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < p.world) {
    unsigned int *f = ag_flag(p.own, par, tid);
    const unsigned long long t_give_up = __builtin_amdgcn_s_memrealtime() + kAgWaitTicks;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() > t_give_up) {
        __hip_atomic_store(p.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  v4u *dst = reinterpret_cast<v4u *>(p.dst);
  for (int i = tid; i < n16 * p.world; i += kAgThreads) {
    const int r = i / n16, j = i - r * n16;
    dst[i] = reinterpret_cast<const v4u *>(ag_slot(p.own, par, r, p.world, p.slot_bytes))[j];
  }
  ag_advance_epoch(p.epoch, epoch);
}

__global__ __launch_bounds__(kAgThreads) void k_allgather_granules(AllGatherParams p) {
  const int tid = threadIdx.x, b = blockIdx.x;
  const unsigned int epoch = p.epoch[0] + 1u;
  const int par = (int)(epoch & 1u);
  const int nw = p.nbytes >> 2;
  const unsigned long long tag = (unsigned long long)epoch << 32;
  // 1. push words [w0, w1) of the shard to every rank, one 8-byte {word, epoch} store each
  const unsigned int *src = reinterpret_cast<const unsigned int *>(p.src);
  const int w0 = (int)((long long)nw * b / p.world), w1 = (int)((long long)nw * (b + 1) / p.world);
  for (int i = w0 + tid; i < w1; i += kAgThreads) {
    const unsigned long long g = tag | src[i];
#pragma unroll
    for (int r = 0; r < kAgMaxWorld; ++r) {
      if (r < p.world)
        __hip_atomic_store(ag_granule(p.peer[r], par, p.rank, p.world, p.slot_bytes) + i, g, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // 2. pull rank b's words from the own buffer once their tags say this epoch
  unsigned long long *in = ag_granule(p.own, par, b, p.world, p.slot_bytes);
  unsigned int *dst = reinterpret_cast<unsigned int *>(p.dst) + (long long)b * nw;
  for (int base = tid; base < nw; base += kAgPoll * kAgThreads) {
    unsigned long long g[kAgPoll];
#pragma unroll
    for (int k = 0; k < kAgPoll; ++k) {
      const int i = base + k * kAgThreads;
      g[k] = i < nw ? __hip_atomic_load(in + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : tag;
    }
    const unsigned long long t_give_up = __builtin_amdgcn_s_memrealtime() + kAgWaitTicks;
    for (;;) {
      bool all = true;
#pragma unroll
      for (int k = 0; k < kAgPoll; ++k) {
        const int i = base + k * kAgThreads;
        if ((g[k] >> 32) != epoch) {
          all = false;
          g[k] = __hip_atomic_load(in + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      if (all) break;
      if (__builtin_amdgcn_s_memrealtime() > t_give_up) {
        __hip_atomic_store(p.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int k = 0; k < kAgPoll; ++k) {
      const int i = base + k * kAgThreads;
      if (i < nw) dst[i] = (unsigned int)g[k];
    }
  }
  // 3. the last workgroup to finish advances the epoch (every workgroup has read it by then)
  ag_advance_epoch(p.epoch, epoch);
}

}  // namespace qz

using namespace qz;

extern "C" int qz_allgather_oneshot_mode(const void *src, int nbytes, void *dst, int rank, int world,
                                         void *const *peer_bufs, void *own_buf, long long slot_bytes,
                                         unsigned int *epoch, unsigned int *status, int mode, void *stream);

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

// Payloads up to this size travel as tagged granules (one xGMI trip, 2x the bytes), larger ones
// by the flag protocol (16-B stores + one flag trip); measured: DESIGN.md section 6.
constexpr int kAgGranuleMaxBytes = QZ_AG_GRANULE_MAX_BYTES;

extern "C" int qz_allgather_oneshot(const void *src, int nbytes, void *dst, int rank, int world,
                                    void *const *peer_bufs, void *own_buf, long long slot_bytes, unsigned int *epoch,
                                    unsigned int *status, void *stream) {
  return qz_allgather_oneshot_mode(src, nbytes, dst, rank, world, peer_bufs, own_buf, slot_bytes, epoch, status,
                                   nbytes <= kAgGranuleMaxBytes ? 2 : 1, stream);
}

extern "C" int qz_allgather_oneshot_mode(const void *src, int nbytes, void *dst, int rank, int world,
                                         void *const *peer_bufs, void *own_buf, long long slot_bytes,
                                         unsigned int *epoch, unsigned int *status, int mode, void *stream) {
  if (mode != 1 && mode != 2) return QZ_ERR_ARG;
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
  if (mode == 2)
    hipLaunchKernelGGL(k_allgather_granules, dim3(world), dim3(kAgThreads), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(k_allgather_flags, dim3(1), dim3(kAgThreads), 0, (hipStream_t)stream, p);
  QZ_LAUNCH_CHECK();
  return QZ_OK;
}

extern "C" long long qz_exchange_bytes(int world, long long slot_bytes) {
  // flags head + [parity][rank] regions of 8-B granules (2x the payload) + [parity][rank] plain slots
  return kAgHeadBytes + 2LL * world * 2 * slot_bytes + 2LL * world * slot_bytes;
}

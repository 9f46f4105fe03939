// common.h -- shared device helpers for the gfx950 4-bit kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <atomic>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/quantizations.h"

namespace qz {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// Codebooks
// ---------------------------------------------------------------------------

// NF4 codebook q_data (reference kernels.cu:851), fp32.
__device__ __constant__ static const float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
    0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};

// NF4 quantiser thresholds: fp32 midpoints of adjacent q_data entries
// (bitsandbytes' dQuantizeNF4 tree; see oracle/oracle.c).
__device__ __forceinline__ uint32_t quantize_nf4(float x) {
  if (x > 0.03979014977812767f) {
    if (x > 0.3893125355243683f) {
      if (x > 0.6427869200706482f) return x > 0.8614784181118011f ? 15u : 14u;
      return x > 0.5016634166240692f ? 13u : 12u;
    }
    if (x > 0.2035212516784668f) return x > 0.2920137718319893f ? 11u : 10u;
    return x > 0.1202552504837513f ? 9u : 8u;
  }
  if (x > -0.33967943489551544f) {
    if (x > -0.13791173323988914f) return x > -0.045525018125772476f ? 7u : 6u;
    return x > -0.23460740596055984f ? 5u : 4u;
  }
  if (x > -0.6106329262256622f) return x > -0.4599952697753906f ? 3u : 2u;
  return x > -0.8480964004993439f ? 1u : 0u;
}

// FP4 quantiser: the fp32 decision tree of reference kernels.cu:113-163.
__device__ __forceinline__ uint32_t quantize_fp4(float x) {
  const uint32_t sign = x < 0.0f ? 8u : 0u;
  x = fabsf(x);
  uint32_t c;
  if (x > 0.29166667f) {
    if (x > 0.583333f) c = x > 0.8333333f ? 3u : 2u;
    else c = x > 0.4166667f ? 5u : 4u;
  } else {
    if (x > 0.0859375f) c = x > 0.20833333f ? 7u : 6u;
    else c = x > 0.00260417f ? 1u : 0u;
  }
  return c + sign;
}

// FP4 dequantisation (reference kernels.cu:70-111): (c * absmax) * sign.
__device__ __forceinline__ float dequant_fp4_tree(uint32_t nib, float absmax) {
  float c;
  switch (nib & 7u) {
    case 0: c = 0.00000000f; break;
    case 1: c = 5.208333333e-03f; break;
    case 2: c = 0.66666667f; break;
    case 3: c = 1.00000000f; break;
    case 4: c = 0.33333333f; break;
    case 5: c = 0.50000000f; break;
    case 6: c = 0.16666667f; break;
    default: c = 0.25000000f; break;
  }
  const float sign = (nib & 8u) ? -1.0f : 1.0f;
  return __fmul_rn(__fmul_rn(c, absmax), sign);
}

// ---------------------------------------------------------------------------
// Element load/store helpers
// ---------------------------------------------------------------------------

template <int DT> struct Elem;
template <> struct Elem<QZ_DT_F16> { typedef __half T; };
template <> struct Elem<QZ_DT_BF16> { typedef __hip_bfloat16 T; };
template <> struct Elem<QZ_DT_F32> { typedef float T; };

template <int DT> __device__ __forceinline__ float load_f32(const void *p, long long i) {
  if constexpr (DT == QZ_DT_F16) {
    return __half2float(reinterpret_cast<const __half *>(p)[i]);
  } else if constexpr (DT == QZ_DT_BF16) {
    const uint32_t u = (uint32_t)reinterpret_cast<const uint16_t *>(p)[i] << 16;
    return __uint_as_float(u);
  } else {
    return reinterpret_cast<const float *>(p)[i];
  }
}

// fp32 -> 2 x fp16, round-to-nearest-even.  Measured on gfx950 (ROCm 7.2):
// the packed v_cvt_pk_f16_f32 rounds exact ties to even, while the scalar
// v_cvt_f16_f32 that __float2half_rn can lower to rounded the tie 0x3c8d1000
// UP (0x2469 instead of 0x2468; tests/test_gpu_rounding.py).  Every fp16 store
// that must be bit-exact goes through the packed instruction.
__device__ __forceinline__ uint32_t cvt_pk_f16_rne(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ uint16_t f32_to_f16_bits(float v) { return (uint16_t)cvt_pk_f16_rne(v, 0.0f); }

template <int DT> __device__ __forceinline__ void store_f32(void *p, long long i, float v) {
  if constexpr (DT == QZ_DT_F16) {
    reinterpret_cast<uint16_t *>(p)[i] = f32_to_f16_bits(v);
  } else if constexpr (DT == QZ_DT_BF16) {
    reinterpret_cast<__hip_bfloat16 *>(p)[i] = __float2bfloat16(v);
  } else {
    reinterpret_cast<float *>(p)[i] = v;
  }
}

// Per-block scale as the consumer sees it (reference core.py:467-468):
// DQ: code2[q] * absmax2[b / bs2] then + offset, each separately rounded.
struct ScaleSrc {
  const float *absmax;           // fp32[nb] or nullptr
  const unsigned char *qabsmax;  // u8[nb] or nullptr (double quant)
  const float *absmax2;
  const float *code2;
  const float *offset;
  int bs2;
};

__device__ __forceinline__ float dq_scale(const ScaleSrc &s, long long b, float offset) {
  const float c = s.code2[s.qabsmax[b]];
  return __fadd_rn(__fmul_rn(c, s.absmax2[b / s.bs2]), offset);
}

inline bool valid_blocksize(int bs) {
  return bs == 64 || bs == 128 || bs == 256 || bs == 512 || bs == 1024 || bs == 2048 || bs == 4096;
}

// Compute units of the current device (hipDeviceGetAttribute), cached per device: the persistent
// grids are sized in workgroups per CU.
static int device_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int v = cache[dev].load(std::memory_order_relaxed);
  if (v <= 0) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

}  // namespace qz

#define QZ_LAUNCH_CHECK()                      \
  do {                                         \
    hipError_t _e = hipGetLastError();         \
    if (_e != hipSuccess) return (int)_e;      \
  } while (0)

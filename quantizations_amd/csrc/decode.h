// decode.h -- shared 4-bit decode helpers for the fused GEMM (gemm.hip) and
// the full-weight dequantiser (dequantize.hip): the per-(row, block) table of
// exact 16-bit weights fp16/bf16(code[i] * absmax) and the AND-combined
// v_perm nibble lookup through it (see decode_lut16 in gemv.hip).
#pragma once
#include "common.h"

namespace qz {

__device__ __forceinline__ uint32_t gperm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// fp32 pair -> packed 16-bit pair, round-to-nearest-even (bit-exact with the
// dequant kernel's stores; see common.h on the scalar-convert tie bug)
template <int DT> __device__ __forceinline__ uint32_t cvt_pk16(float lo, float hi) {
  if constexpr (DT == QZ_DT_F16) {
    return cvt_pk_f16_rne(lo, hi);
  } else {
    uint32_t r;
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
    return r;
  }
}

// fp32 FP4 dequant-tree magnitudes (kernels.cu:70-111; sign = bit 3); NF4 uses
// kNF4 (kernels.cu:851) from common.h
__device__ __constant__ static const float kFP4Mag[8] = {0.00000000f, 5.208333333e-03f, 0.66666667f, 1.00000000f,
                                                         0.33333333f, 0.50000000f,      0.16666667f, 0.25000000f};

// 16-entry table of one (row, block): entries fp16/bf16(code[i] * am) as byte
// planes t[0..3] = low bytes of entries 0-3, 4-7, 8-11, 12-15 and t[4..7] =
// high bytes (the layout decode_codes expects).
template <int QT, int DT>
__device__ __forceinline__ void block_table(float am, uint32_t (&t)[8]) {
  uint32_t p[8];  // p[k] = (entry 2k, entry 2k+1)
  if constexpr (QT == QZ_NF4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = cvt_pk16<DT>(__fmul_rn(kNF4[2 * k], am), __fmul_rn(kNF4[2 * k + 1], am));
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p[k] = cvt_pk16<DT>(__fmul_rn(kFP4Mag[2 * k], am), __fmul_rn(kFP4Mag[2 * k + 1], am));
      p[4 + k] = p[k] ^ 0x80008000u;  // (c * am) * -1: exact sign flip, code 8 -> -0.0
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[j] = gperm(p[2 * j + 1], p[2 * j], 0x06040200u);
    t[4 + j] = gperm(p[2 * j + 1], p[2 * j], 0x07050301u);
  }
}

// 8 nibbles (one dword, high nibble = even element) -> 4 packed 16-bit pairs in
// the order (e0,e2),(e4,e6),(e1,e3),(e5,e7): AND-combined 8-entry v_perm
// lookups (see decode_lut16 in gemv.hip).
__device__ __forceinline__ void decode_codes(uint32_t w, const uint32_t (&t)[8], uint32_t (&P)[4]) {
  uint32_t ah = ((w >> 4) & 0x0F0F0F0Fu) | (w & 0x80808080u);
  asm("" : "+v"(ah));
  const uint32_t bh = ah ^ 0x88888888u;
  const uint32_t lh = gperm(t[1], t[0], ah) & gperm(t[3], t[2], bh);
  const uint32_t hh = gperm(t[5], t[4], ah) & gperm(t[7], t[6], bh);
  uint32_t al = (w & 0x0F0F0F0Fu) | ((w << 4) & 0x80808080u);
  asm("" : "+v"(al));
  const uint32_t bl = al ^ 0x88888888u;
  const uint32_t ll = gperm(t[1], t[0], al) & gperm(t[3], t[2], bl);
  const uint32_t hl = gperm(t[5], t[4], al) & gperm(t[7], t[6], bl);
  P[0] = gperm(hh, lh, 0x05010400u);
  P[1] = gperm(hh, lh, 0x07030602u);
  P[2] = gperm(hl, ll, 0x05010400u);
  P[3] = gperm(hl, ll, 0x07030602u);
}

// 8 nibbles -> 4 packed 16-bit pairs in NATURAL order (e0,e1),(e2,e3),(e4,e5),(e6,e7)
__device__ __forceinline__ void decode_codes_natural(uint32_t w, const uint32_t (&t)[8], uint32_t (&N)[4]) {
  uint32_t P[4];
  decode_codes(w, t, P);  // (e0,e2),(e4,e6),(e1,e3),(e5,e7)
  N[0] = gperm(P[2], P[0], 0x05040100u);
  N[1] = gperm(P[2], P[0], 0x07060302u);
  N[2] = gperm(P[3], P[1], 0x05040100u);
  N[3] = gperm(P[3], P[1], 0x07060302u);
}

}  // namespace qz

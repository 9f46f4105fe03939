// Dev tool: VALU throughput of the decode instructions on gfx950 (cycles per
// wave-instruction per SIMD), with W waves per SIMD.  Each wave runs N
// iterations of 8 independent chains of one instruction kind.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(1024) void k_rate(uint32_t *out, int n, uint32_t seed, unsigned long long *cyc) {
  uint32_t a[8], b = seed * 0x9E3779B9u + threadIdx.x, c = seed ^ 0x01020304u;
  float f[8];
  f2 F[8], B2 = {1.0001f, 0.999f}, C2 = {0.5f, 0.25f};
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = b + i * 0x01010101u; f[i] = (float)i; F[i] = f2{(float)i, 1.0f}; }
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) a[i] = __builtin_amdgcn_perm(a[i], b, c);
      else if constexpr (OP == 1) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      else if constexpr (OP == 2) a[i] = (a[i] >> 4) & 0x07070707u;          // shift+and (2 ops)
      else if constexpr (OP == 3) f[i] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, a[i]), __builtin_bit_cast(h2, b), f[i], false);
      else if constexpr (OP == 4) f[i] = __builtin_fmaf(f[i], 1.0001f, 0.5f);
      else if constexpr (OP == 5) a[i] = a[i] ^ b;
      else if constexpr (OP == 6) { h2 r = __builtin_bit_cast(h2, a[i]) * __builtin_bit_cast(h2, b) + __builtin_bit_cast(h2, c); a[i] = __builtin_bit_cast(uint32_t, r); }
      else if constexpr (OP == 7) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(f[i]) : "v"(b), "v"(c));
      else if constexpr (OP == 8) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a[i]) : "v"(b));
      else if constexpr (OP == 9) asm volatile("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(a[i]) : "v"(a[i]), "v"(c));
      else if constexpr (OP == 10) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(F[i]) : "v"(B2), "v"(C2));
      else if constexpr (OP == 11) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(f[i]) : "v"(a[i]));
      else if constexpr (OP == 12) asm volatile("v_cvt_f32_f16_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "=v"(f[i]) : "v"(a[i]));
      else if constexpr (OP == 13) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      else if constexpr (OP == 14) asm volatile("v_lshrrev_b32 %0, 9, %0" : "+v"(a[i]));
      else if constexpr (OP == 15) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[i]));
      else if constexpr (OP == 16) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(F[i]) : "v"(B2));
      else if constexpr (OP == 17) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[i]) : "v"(b), "v"(c));
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc ^= a[i] ^ __float_as_uint(f[i]) ^ __float_as_uint(F[i].x) ^ __float_as_uint(F[i].y);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  uint32_t *out; unsigned long long *cyc;
  CK(hipMalloc(&out, 256 * 1024 * 4 * 8)); CK(hipMalloc(&cyc, 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char *names[] = {"v_perm_b32", "v_bfi_b32", "lshr+and (2 ops)", "v_dot2c_f32_f16", "v_fma_f32", "v_xor_b32", "v_pk_fma_f16", "v_fma_mix_f32", "v_mov_b32_sdwa", "v_lshl_or_b32",
                         "v_pk_fma_f32", "v_cvt_f32_f16", "v_cvt_f32_f16_sdwa w1", "v_and_or_b32", "v_lshrrev_b32",
                         "v_bfe_u32", "v_pk_mul_f32", "v_fma_f32 (asm)"};
  const int n = 4096;
  for (int wps : {1, 2, 4}) {
    for (int op = 0; op < 18; ++op) {
      const int threads = 256 * wps;  // one block per CU: 4 SIMDs x wps waves
      auto launch = [&]() {
        switch (op) {
          case 0: hipLaunchKernelGGL(k_rate<0>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 1: hipLaunchKernelGGL(k_rate<1>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 2: hipLaunchKernelGGL(k_rate<2>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 3: hipLaunchKernelGGL(k_rate<3>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 4: hipLaunchKernelGGL(k_rate<4>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 5: hipLaunchKernelGGL(k_rate<5>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 6: hipLaunchKernelGGL(k_rate<6>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 7: hipLaunchKernelGGL(k_rate<7>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 8: hipLaunchKernelGGL(k_rate<8>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 9: hipLaunchKernelGGL(k_rate<9>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 10: hipLaunchKernelGGL(k_rate<10>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 11: hipLaunchKernelGGL(k_rate<11>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 12: hipLaunchKernelGGL(k_rate<12>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 13: hipLaunchKernelGGL(k_rate<13>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 14: hipLaunchKernelGGL(k_rate<14>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 15: hipLaunchKernelGGL(k_rate<15>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 16: hipLaunchKernelGGL(k_rate<16>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
          case 17: hipLaunchKernelGGL(k_rate<17>, dim3(256), dim3(threads), 0, 0, out, n, 1u, cyc); break;
        }
      };
      launch(); CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
      const double insts = (double)n * 8 * wps;  // per SIMD
      printf("waves/SIMD %d %-20s %8.3f us  wave0 cycles/inst/SIMD(cyc-ctr) %6.2f  wall-based(2.4GHz) %6.2f\n", wps,
             names[op], ms * 1e3, (double)c * wps / insts, ms * 1e-3 * 2.4e9 / insts);
    }
  }
  return 0;
}

// capi.hip -- the reference-compatible C-ABI (pythonInterface.cpp:34-46 names,
// argument order and meaning), routed onto the MI355X-native kernels.
//
// The reference binds five C++ functions into the CPython module kbkim_lib
// (pythonInterface.cpp:154-178) and launches on the legacy default stream with
// no error checking.  Here they are plain extern "C" symbols returning a status;
// the *_stream variants take the HIP stream explicitly.
#include "common.h"

extern "C" int cgemm_4bit_inference_naive_fp32_stream(int m, int n, int k, float *A, unsigned char *B,
                                                      float *absmax, float *datatype, float *out, int lda, int ldb,
                                                      int ldc, int blocksize, void *stream) {
  (void)lda;
  (void)ldc;
  if (n != 1) return QZ_ERR_SHAPE;  // gemv only (core.py:477, n = 1)
  if (!datatype) return QZ_ERR_ARG;
  // core.py:482 passes ldb = (k+1)//2; the packed layout is flat (row stride
  // k/2 bytes for even k), which is what the kernels address.
  if (ldb != (k + 1) / 2) return QZ_ERR_SHAPE;
  return qz_gemv_4bit(m, k, A, QZ_DT_F32, B, QZ_FP4, blocksize, absmax, nullptr, nullptr, nullptr, nullptr, 0, 0,
                      datatype, nullptr, out, stream);
}

extern "C" int cquantize_blockwise_fp16_fp4_stream(float *code, void *A, float *absmax, unsigned char *out,
                                                   int blocksize, int n, void *stream) {
  (void)code;  // unused by the FP4 path (core.py:553 passes NULL)
  return qz_quantize_4bit(A, QZ_DT_F16, n, blocksize, QZ_FP4, absmax, out, stream);
}

extern "C" int cdequantize_blockwise_fp16_fp4_stream(float *code, unsigned char *A, float *absmax, void *out,
                                                     int blocksize, int n, void *stream) {
  (void)code;
  if (!absmax) return QZ_ERR_ARG;
  return qz_dequantize_4bit(A, n, QZ_FP4, blocksize, absmax, nullptr, nullptr, nullptr, nullptr, 0, out, QZ_DT_F16,
                            stream);
}

extern "C" int cquantize_blockwise_fp32_stream(float *code, float *A, float *absmax, unsigned char *out,
                                               int blocksize, int n, void *stream) {
  return qz_quantize_blockwise_8bit(code, A, n, blocksize, nullptr, absmax, out, stream);
}

extern "C" int cdequantize_blockwise_fp32_stream(float *code, unsigned char *A, float *absmax, float *out,
                                                 int blocksize, int n, void *stream) {
  return qz_dequantize_blockwise_8bit(code, A, absmax, n, blocksize, nullptr, out, stream);
}

// Legacy-default-stream forms: exactly the reference's five symbols.
extern "C" int cgemm_4bit_inference_naive_fp32(int m, int n, int k, float *A, unsigned char *B, float *absmax,
                                               float *datatype, float *out, int lda, int ldb, int ldc,
                                               int blocksize) {
  return cgemm_4bit_inference_naive_fp32_stream(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize,
                                                nullptr);
}

extern "C" int cquantize_blockwise_fp16_fp4(float *code, void *A, float *absmax, unsigned char *out, int blocksize,
                                            int n) {
  return cquantize_blockwise_fp16_fp4_stream(code, A, absmax, out, blocksize, n, nullptr);
}

extern "C" int cdequantize_blockwise_fp16_fp4(float *code, unsigned char *A, float *absmax, void *out, int blocksize,
                                              int n) {
  return cdequantize_blockwise_fp16_fp4_stream(code, A, absmax, out, blocksize, n, nullptr);
}

extern "C" int cquantize_blockwise_fp32(float *code, float *A, float *absmax, unsigned char *out, int blocksize,
                                        int n) {
  return cquantize_blockwise_fp32_stream(code, A, absmax, out, blocksize, n, nullptr);
}

extern "C" int cdequantize_blockwise_fp32(float *code, unsigned char *A, float *absmax, float *out, int blocksize,
                                          int n) {
  return cdequantize_blockwise_fp32_stream(code, A, absmax, out, blocksize, n, nullptr);
}

extern "C" int qz_version(void) { return 100; }  // 0.1.0

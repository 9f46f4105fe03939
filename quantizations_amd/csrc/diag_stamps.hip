// diag_stamps.hip -- measurement-only library (libqz_diag.so, NOT the product): the product
// decode GEMV instantiation with in-kernel timeline stamps (s_memrealtime, 100 MHz chip-wide
// clock) at wave start and after the wave's last store (gemv.hip, QZ_STAMP / STAMP = 2).
// bench.py times the kernel's own duration with it -- first wave start to last wave end --
// which the rocprofv3 tracer cannot resolve at a few microseconds.
// Built with hidden visibility: only the qz_diag_* entry points are exported, so the
// included product entry points of gemv.hip never clash with libquantizations.so.
#define QZ_STAMPS 1
#include "gemv.hip"

#define QZ_DIAG_API extern "C" __attribute__((visibility("default")))

// Stamp buffer: 8 u64 per wave (wave id = block * 4 + wave in block): [0] start, [4] after the
// wave's stores were issued (the "light" stamps, STAMP 2: nothing in between is timed, so
// the schedule between them is the product's).  Every launch overwrites it.
QZ_DIAG_API int qz_diag_set_stamp_buffer(unsigned long long *buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_qz_stamp), &buf, sizeof(buf));
}

// The product qz_gemv_4bit launch for fp16 x, NF4 + double quant, full-step rows (K % 2048 == 0)
// at the geometry choose_geometry picks, with stamps.  exact != 0: the exact-code table (CL).
// *nwaves = the number of waves launched (stamp records written).  Returns QZ_OK or a status.
QZ_DIAG_API int qz_diag_gemv_stamped(int M, int K, const void *x, const unsigned char *B, int exact,
                                     const unsigned char *qabsmax, const float *absmax2, const float *code2,
                                     const float *offset, void *y, int *nwaves, void *stream) {
  GemvParams p;
  bool vec_ok;
  const int st = make_params(M, K, x, QZ_DT_F16, B, QZ_NF4, 64, nullptr, qabsmax, absmax2, code2, offset, 256, 0,
                             nullptr, nullptr, y, &p, &vec_ok);
  if (st != QZ_OK) return st;
  if (!vec_ok || !full_steps(K, 64, 256, true, 0) || !nwaves) return QZ_ERR_SHAPE;
  int R, WK;
  choose_geometry(M, K, QZ_DT_F16, &R, &WK);
  if (WK != 1 || (R != 2 && R != 4)) return QZ_ERR_SHAPE;
  set_tables(QZ_NF4, nullptr, exact != 0, QZ_DT_F16, &p);
  const unsigned grid = (unsigned)((M + R * 4 - 1) / (R * 4));
  hipStream_t s = (hipStream_t)stream;
  // the product's instantiation for this shape (launch_vec): the straight-line two-step form at
  // K = 4096, the loop form otherwise; STAMP 2 = start / end stamps only
  const bool two = two_steps(K, 1, true);
#define QZ_DG(RR, CL_, TWO_) \
  hipLaunchKernelGGL((k_gemv_4bit<true, QZ_DT_F16, RR, 1, 4, true, CL_, false, TWO_, 2>), dim3(grid), dim3(256), 0, s, p)
#define QZ_DG2(RR, CL_) do { if (two) QZ_DG(RR, CL_, true); else QZ_DG(RR, CL_, false); } while (0)
  if (R == 2) { if (exact) QZ_DG2(2, true); else QZ_DG2(2, false); }
  else { if (exact) QZ_DG2(4, true); else QZ_DG2(4, false); }
#undef QZ_DG2
#undef QZ_DG
  QZ_LAUNCH_CHECK();
  *nwaves = (int)grid * 4;
  return QZ_OK;
}


/*
 * oracle.c -- CPU restatement of the reference 4-bit Linear4bit path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in quantizations_amd/ links, loads or
 * calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker.
 *
 * Every function cites the reference file:line it restates
 * (reference = kkbwilldo/quantizations @ 2024_10_08).  The reference CUDA
 * sources need nvcc, CUB and WMMA (CMakeLists.txt:2,9,26; kernels.cu:2-3) and
 * are therefore unbuildable in this image; the codebooks, the dynamic 8-bit
 * map and the host orchestration are pinned against the importable reference
 * Python (tests/golden/make_golden.py).  See DESIGN.md "Oracle".
 *
 * Conventions: all arithmetic is IEEE fp32 (x86-64 SSE, FLT_EVAL_METHOD 0,
 * built with -ffp-contract=off so that no product is fused into an FMA,
 * matching the separately rounded operations of the reference kernels).
 * fp16/bf16 <-> fp32 conversions are done by the caller (numpy / torch, RNE).
 */
#include <stdint.h>
#include <math.h>
#include <float.h>
#include <string.h>

#define ORC_FP4 0
#define ORC_NF4 1

/* ------------------------------------------------------------------------ */
/* Codebooks                                                                */
/* ------------------------------------------------------------------------ */

/* FP4 dequantisation tree constants, kernels.cu:70-111 (dDequantizeFP4Tree),
 * indexed by the 3 magnitude bits (nibble & 7). */
static const float FP4_TREE[8] = {
    0.00000000f, 5.208333333e-03f, 0.66666667f, 1.00000000f,
    0.33333333f, 0.50000000f,      0.16666667f, 0.25000000f};

/* NF4 codebook q_data, kernels.cu:851 (data only; the kernel that reads it is
 * dead code).  Double literals rounded to fp32 exactly as the CUDA array. */
static const float NF4_LUT[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
    0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};

/* NF4 decision thresholds: the double-precision midpoints of adjacent
 * q_data entries rounded to fp32 (bitsandbytes' published dQuantizeNF4 tree;
 * bitsandbytes is not vendored by the reference -- see DESIGN.md). */
static const float NF4_MID[15] = {
    -0.8480964004993439f, -0.6106329262256622f, -0.4599952697753906f,
    -0.33967943489551544f, -0.23460740596055984f, -0.13791173323988914f,
    -0.045525018125772476f, 0.03979014977812767f, 0.1202552504837513f,
    0.2035212516784668f, 0.2920137718319893f, 0.3893125355243683f,
    0.5016634166240692f, 0.6427869200706482f, 0.8614784181118011f};

/* The 15 NF4 thresholds as the compiler rounds the decimal literals (directly
 * to fp32, as nvcc/hipcc do; NOT decimal -> double -> fp32, which differs by
 * one ulp for 3 of them). */
void orc_nf4_thresholds(float *out15)
{
    for (int i = 0; i < 15; ++i) out15[i] = NF4_MID[i];
}

void orc_codebook(int quant_type, float *out16)
{
    /* FP4 as the GEMV consumes it: get_4bit_type("fp4"), core.py:208-229:
     * [0, .0625, 8, 12, 4, 6, 2, 3, -0, ...]/12.  Index 8 is +0.0 because
     * the Python literal -0 is an int. */
    static const float fp4_raw[16] = {0.0f, 0.0625f, 8.0f, 12.0f, 4.0f, 6.0f, 2.0f, 3.0f,
                                      0.0f, -0.0625f, -8.0f, -12.0f, -4.0f, -6.0f, -2.0f, -3.0f};
    for (int i = 0; i < 16; ++i)
        out16[i] = quant_type == ORC_NF4 ? NF4_LUT[i] : fp4_raw[i] / 12.0f;
}

/* ------------------------------------------------------------------------ */
/* Scalar codecs                                                            */
/* ------------------------------------------------------------------------ */

/* kernels.cu:113-163 dQuantizeFP4: fp32 decision tree with strict '>'. */
uint8_t orc_quantize_fp4(float x)
{
    int sign = x < 0 ? 8 : 0;
    x = fabsf(x);
    if (x > 0.29166667f) {
        if (x > 0.583333f)
            return (uint8_t)((x > 0.8333333f ? 3 : 2) + sign);
        return (uint8_t)((x > 0.4166667f ? 5 : 4) + sign);
    }
    if (x > 0.0859375f)
        return (uint8_t)((x > 0.20833333f ? 7 : 6) + sign);
    return (uint8_t)((x > 0.00260417f ? 1 : 0) + sign);
}

/* NF4 quantiser (build-defined, bitsandbytes dQuantizeNF4 restated): a
 * balanced tree over the 15 midpoints with strict '>'.  For every non-NaN x
 * this equals the number of midpoints below x; NaN falls to code 0. */
uint8_t orc_quantize_nf4(float x)
{
    if (x > NF4_MID[7]) {
        if (x > NF4_MID[11]) {
            if (x > NF4_MID[13]) return x > NF4_MID[14] ? 15 : 14;
            return x > NF4_MID[12] ? 13 : 12;
        }
        if (x > NF4_MID[9]) return x > NF4_MID[10] ? 11 : 10;
        return x > NF4_MID[8] ? 9 : 8;
    }
    if (x > NF4_MID[3]) {
        if (x > NF4_MID[5]) return x > NF4_MID[6] ? 7 : 6;
        return x > NF4_MID[4] ? 5 : 4;
    }
    if (x > NF4_MID[1]) return x > NF4_MID[2] ? 3 : 2;
    return x > NF4_MID[0] ? 1 : 0;
}

/* kernels.cu:70-111 dDequantizeFP4Tree: (c * absmax) * sign, fp32.
 * Code 8 yields -0.0 (unlike the GEMV LUT, whose index 8 is +0.0). */
float orc_dequantize_fp4_tree(uint8_t nib, float absmax)
{
    float sign = (nib & 8) ? -1.0f : 1.0f;
    return FP4_TREE[nib & 7] * absmax * sign;
}

/* kernels.cu:166-237 dQuantize<0>: 7-step binary search over the sorted
 * 256-entry code, then round to nearest by midpoint. */
uint8_t orc_quantize_8bit(const float *code, float x)
{
    int pivot = 127, upper_pivot = 255, lower_pivot = 0;
    float lower = -1.0f, upper = 1.0f;
    float val = code[pivot];
    for (int i = 64; i > 0; i >>= 1) {
        if (x > val) {
            lower_pivot = pivot;
            lower = val;
            pivot += i;
        } else {
            upper_pivot = pivot;
            upper = val;
            pivot -= i;
        }
        val = code[pivot];
    }
    if (upper_pivot == 255) upper = code[upper_pivot];
    if (lower_pivot == 0) lower = code[lower_pivot];
    if (x > val) {
        float midpoint = (upper + val) * 0.5f;
        return (uint8_t)(x > midpoint ? upper_pivot : pivot);
    }
    float midpoint = (lower + val) * 0.5f;
    return (uint8_t)(x < midpoint ? lower_pivot : pivot);
}

/* ------------------------------------------------------------------------ */
/* Blockwise quantisation                                                   */
/* ------------------------------------------------------------------------ */

/* Block absmax as kQuantizeBlockwise computes it (kernels.cu:406-431):
 * fmaxf over |x| (NaN-ignoring), seeded with -FLT_MAX; padding lanes of a
 * partial block contribute 0 (BlockLoad default, kernels.cu:410). */
static float block_absmax(const float *A, int64_t start, int64_t valid, int bs)
{
    float m = -FLT_MAX;
    for (int64_t j = 0; j < valid; ++j) m = fmaxf(m, fabsf(A[start + j]));
    if (valid < bs) m = fmaxf(m, 0.0f);
    return m;
}

/* quantize_4bit's kernel, kernels.cu:340-478 with DATA_TYPE=FP4 (and NF4 as
 * the build's extension): byte j of the output holds q(A[2j]) in its HIGH
 * nibble and q(A[2j+1]) in its low nibble (kernels.cu:467-468).  The input is
 * the exact fp32 image of the fp16/bf16/fp32 weight.
 * Note: reference blocksizes >= 1024 (NUM_PER_TH=4) OR-accumulate
 * packed_4bit across the two bytes of a thread (kernels.cu:450,465-470); this
 * restatement (and the HIP path) packs every byte independently -- the
 * Linear4bit path only ever uses blocksize 64 (core.py:102). */
void orc_quantize_4bit(const float *A, int64_t n, int blocksize, int quant_type,
                       uint8_t *out, float *absmax)
{
    int64_t nblocks = (n + blocksize - 1) / blocksize;
    for (int64_t b = 0; b < nblocks; ++b) {
        int64_t start = b * blocksize;
        int64_t valid = n - start < blocksize ? n - start : blocksize;
        float amax = block_absmax(A, start, valid, blocksize);
        absmax[b] = amax;
        float s = 1.0f / amax;
        for (int64_t j = 0; j < valid; j += 2) {
            float x0 = A[start + j] * s;
            float x1 = (j + 1 < valid ? A[start + j + 1] : 0.0f) * s;
            uint8_t q0, q1;
            if (quant_type == ORC_NF4) {
                q0 = orc_quantize_nf4(x0);
                q1 = orc_quantize_nf4(x1);
            } else {
                q0 = orc_quantize_fp4(x0);
                q1 = orc_quantize_fp4(x1);
            }
            out[(start + j) >> 1] = (uint8_t)((q0 << 4) | q1);
        }
    }
}

/* quantize_blockwise's kernel, kernels.cu:340-478 with General8bit, fed by
 * core.py:563-565 (absmax -= offset).  If `subtract` is non-NULL the input is
 * A[i] - *subtract (fp32), which is exactly the in-place torch subtraction. */
void orc_quantize_8bit_blockwise(const float *code, const float *A, int64_t n, int blocksize,
                                 const float *subtract, uint8_t *out, float *absmax)
{
    int64_t nblocks = (n + blocksize - 1) / blocksize;
    float off = subtract ? *subtract : 0.0f;
    for (int64_t b = 0; b < nblocks; ++b) {
        int64_t start = b * blocksize;
        int64_t valid = n - start < blocksize ? n - start : blocksize;
        float m = -FLT_MAX;
        for (int64_t j = 0; j < valid; ++j) {
            float a = subtract ? A[start + j] - off : A[start + j];
            m = fmaxf(m, fabsf(a));
        }
        if (valid < blocksize) m = fmaxf(m, 0.0f);
        absmax[b] = m;
        float s = 1.0f / m;
        for (int64_t j = 0; j < valid; ++j) {
            float a = subtract ? A[start + j] - off : A[start + j];
            out[start + j] = orc_quantize_8bit(code, a * s);
        }
    }
}

/* Deterministic mean of the fp32 absmax vector (the build's fixed-order
 * replacement for core.py:563 `absmax.mean()`, whose CUDA reduction order is
 * unspecified).  fp64 accumulation; chunks of 1024 summed by 256 lanes
 * (4 sequential adds per lane, then a halving tree), chunk sums reduced the
 * same way; offset = (float)(sum / n).  The HIP kernel uses this exact tree. */
#define MEAN_LANES 256
#define MEAN_PER_LANE 4
static double tree256(double *s)
{
    for (int stride = MEAN_LANES / 2; stride > 0; stride >>= 1)
        for (int t = 0; t < stride; ++t) s[t] += s[t + stride];
    return s[0];
}

double orc_mean_chunk(const float *a, int64_t n, int64_t c)
{
    double s[MEAN_LANES];
    for (int t = 0; t < MEAN_LANES; ++t) {
        s[t] = 0.0;
        for (int j = 0; j < MEAN_PER_LANE; ++j) {
            int64_t idx = c * (MEAN_LANES * MEAN_PER_LANE) + (int64_t)j * MEAN_LANES + t;
            if (idx < n) s[t] += (double)a[idx];
        }
    }
    return tree256(s);
}

float orc_absmax_mean(const float *a, int64_t n)
{
    int64_t nc = (n + MEAN_LANES * MEAN_PER_LANE - 1) / (MEAN_LANES * MEAN_PER_LANE);
    double s[MEAN_LANES];
    for (int t = 0; t < MEAN_LANES; ++t) {
        s[t] = 0.0;
        for (int64_t idx = t; idx < nc; idx += MEAN_LANES) s[t] += orc_mean_chunk(a, n, idx);
    }
    return (float)(tree256(s) / (double)n);
}

/* ------------------------------------------------------------------------ */
/* Dequantisation                                                           */
/* ------------------------------------------------------------------------ */

/* dequantize_blockwise's kernel, kernels.cu:549-553 (General8bit):
 * out[i] = code[q[i]] * absmax[i / blocksize], followed (when `offset` is
 * non-NULL) by core.py:468 `absmax += offset` -- two separate fp32 roundings. */
void orc_dequantize_8bit_blockwise(const float *code, const uint8_t *q, const float *absmax,
                                   int64_t n, int blocksize, const float *offset, float *out)
{
    for (int64_t i = 0; i < n; ++i) {
        float v = code[q[i]] * absmax[i / blocksize];
        if (offset) v = v + *offset;
        out[i] = v;
    }
}

/* dequantize_4bit's kernel, kernels.cu:554-560 (FP4 via the tree) and the
 * NF4 extension (LUT * absmax).  Output is fp32; the caller rounds to fp16
 * (RNE), as the kernel's half store does. */
void orc_dequantize_4bit(const uint8_t *packed, const float *absmax, int64_t n, int blocksize,
                         int quant_type, float *out)
{
    for (int64_t e = 0; e < n; ++e) {
        uint8_t byte = packed[e >> 1];
        uint8_t nib = (e & 1) ? (byte & 0x0F) : (byte >> 4);
        float am = absmax[e / blocksize];
        out[e] = quant_type == ORC_NF4 ? NF4_LUT[nib] * am : orc_dequantize_fp4_tree(nib, am);
    }
}

/* ------------------------------------------------------------------------ */
/* GEMV                                                                     */
/* ------------------------------------------------------------------------ */

/* kgemm_4bit_inference_naive, kernels.cu:1061-1219, as a numerical
 * reference: y[r] = sum_k x[k] * (lut[nib(r,k)] * absmax[(r*K+k)/bs]).
 * The weight product is formed in fp32 exactly as kernels.cu:1169-1170 do;
 * the sum is accumulated in fp64 (the reference's lane/warp order is not
 * reproduced -- parity on y is by tolerance, see tests). */
void orc_gemv_4bit(const float *x, const uint8_t *packed, const float *absmax, const float *lut,
                   int64_t M, int64_t K, int blocksize, double *y)
{
    for (int64_t r = 0; r < M; ++r) {
        double acc = 0.0;
        for (int64_t k = 0; k < K; ++k) {
            int64_t e = r * K + k;
            uint8_t byte = packed[e >> 1];
            uint8_t nib = (e & 1) ? (byte & 0x0F) : (byte >> 4);
            float w = lut[nib] * absmax[e / blocksize];
            acc += (double)x[k] * (double)w;
        }
        y[r] = acc;
    }
}

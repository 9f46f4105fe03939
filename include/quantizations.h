/*
 * quantizations.h -- C-ABI of libquantizations.so, the MI355X (gfx950) native
 * 4-bit Linear4bit library.
 *
 * Drop-in boundary.  The reference exposes its kernels as the CPython module
 * `kbkim_lib` (pythonInterface.cpp:154-178) whose five functions take raw
 * device pointers as Python ints and integer sizes.  This header exports the
 * SAME five names with the SAME argument order and meaning as plain
 * `extern "C"` symbols, so any FFI (ctypes -- quantizations_amd/kbkim_lib.py --,
 * cgo, JNI, N-API) can bind them.  Differences, all additive:
 *   - every function returns an int status (0 = success, <0 = argument error,
 *     >0 = hipError_t) instead of silently ignoring errors;
 *   - `*_stream` variants take the HIP stream to launch on (the reference
 *     launches on the legacy default stream, ops.cu:170);
 *   - qz_* entry points expose the MI355X-native fused path (in-kernel double
 *     quant, NF4, fp16/bf16/fp32 activations, fused bias, row-shard views).
 *
 * Ownership: every buffer is owned by the caller (torch in Python); the
 * library never allocates, frees or synchronises.  Any workspace is passed in.
 * All pointers are device pointers unless stated otherwise.
 */
#ifndef QUANTIZATIONS_H
#define QUANTIZATIONS_H

#ifdef __cplusplus
extern "C" {
#endif

/* element dtypes */
#define QZ_DT_F16 0
#define QZ_DT_BF16 1
#define QZ_DT_F32 2

/* 4-bit codebooks */
#define QZ_FP4 0 /* bnb FP4 (get_4bit_type("fp4"), core.py:208-229)         */
#define QZ_NF4 1 /* NF4 codebook q_data (kernels.cu:851)                     */
/* Flag OR-ed into qz_gemv_4bit(_grouped)'s quant_type for fp16 activations:
 * decode with the fp32 codes (each split into two fp16 parts, ~2^-23
 * relative) instead of the fp16-rounded codes of the default byte table.  A
 * runtime `lut` is always decoded this way; the built-in FP4 book (x12) is
 * exact either way.  fp32 activations always multiply by the fp32 codes (a
 * runtime lut verbatim: the reference GEMV's quant_map, kernels.cu:1115-1120)
 * and bf16 activations by bf16 hi + lo codes (~2^-16); the flag does not
 * change them. */
#define QZ_EXACT_CODES 0x100

/* status codes (>0 values are hipError_t) */
#define QZ_OK 0
#define QZ_ERR_ARG (-1)       /* null pointer / negative size                 */
#define QZ_ERR_BLOCKSIZE (-2) /* blocksize not in {64,...,4096} (core.py:549) */
#define QZ_ERR_SHAPE (-3)     /* unsupported M/K/n combination               */
#define QZ_ERR_DTYPE (-4)     /* unknown dtype / quant type                  */

/* ------------------------------------------------------------------------ */
/* Reference-compatible entry points (pythonInterface.cpp:34-46)            */
/* ------------------------------------------------------------------------ */

/* Replaces gemm_4bit_inference_naive_fp32 (pythonInterface.cpp:34, kernel
 * kernels.cu:1061-1219, launcher ops.cu:167-171).  out[m] = B[m,k] . A[k]
 * with fp32 A/out, fp32 per-block absmax (already double-dequantised by the
 * caller, core.py:467-468) and a 16-float device codebook `datatype`.
 * n must be 1; lda/ldc are ignored (=m); ldb is the row stride in bytes
 * ((k+1)/2, core.py:482). */
int cgemm_4bit_inference_naive_fp32(int m, int n, int k, float *A, unsigned char *B, float *absmax,
                                    float *datatype, float *out, int lda, int ldb, int ldc, int blocksize);

/* Replaces quantizeBlockwise_fp16_fp4 (pythonInterface.cpp:37, kernels.cu:340-478
 * with FP4): fp16 A[n] -> packed out[(n+1)/2] (high nibble = even element) and
 * fp32 absmax[ceil(n/blocksize)].  `code` is unused (NULL in core.py:553). */
int cquantize_blockwise_fp16_fp4(float *code, void *A, float *absmax, unsigned char *out, int blocksize, int n);

/* Replaces dequantizeBlockwise_fp16_fp4 (pythonInterface.cpp:40, kernels.cu:554-560):
 * packed A -> fp16 out[n] via the FP4 tree (code 8 -> -0.0). */
int cdequantize_blockwise_fp16_fp4(float *code, unsigned char *A, float *absmax, void *out, int blocksize, int n);

/* Replaces quantizeBlockwise_fp32 (pythonInterface.cpp:43, kernels.cu:340-478
 * General8bit): fp32 A[n] -> u8 out[n] + fp32 absmax via the 256-entry code. */
int cquantize_blockwise_fp32(float *code, float *A, float *absmax, unsigned char *out, int blocksize, int n);

/* Replaces dequantizeBlockwise_fp32 (pythonInterface.cpp:46, kernels.cu:549-553):
 * out[i] = code[A[i]] * absmax[i / blocksize]. */
int cdequantize_blockwise_fp32(float *code, unsigned char *A, float *absmax, float *out, int blocksize, int n);

/* Same five, launched on an explicit HIP stream (hipStream_t passed as void*). */
int cgemm_4bit_inference_naive_fp32_stream(int m, int n, int k, float *A, unsigned char *B, float *absmax,
                                           float *datatype, float *out, int lda, int ldb, int ldc, int blocksize,
                                           void *stream);
int cquantize_blockwise_fp16_fp4_stream(float *code, void *A, float *absmax, unsigned char *out, int blocksize, int n,
                                        void *stream);
int cdequantize_blockwise_fp16_fp4_stream(float *code, unsigned char *A, float *absmax, void *out, int blocksize,
                                          int n, void *stream);
int cquantize_blockwise_fp32_stream(float *code, float *A, float *absmax, unsigned char *out, int blocksize, int n,
                                    void *stream);
int cdequantize_blockwise_fp32_stream(float *code, unsigned char *A, float *absmax, float *out, int blocksize, int n,
                                      void *stream);

/* ------------------------------------------------------------------------ */
/* MI355X-native entry points                                               */
/* ------------------------------------------------------------------------ */

/* Per-block scale source shared by the 4-bit consumers (GEMV, GEMM, dequant).
 * Exactly one of `absmax` (fp32[nb], no double quant) or `qabsmax` (u8[nb],
 * double quant) is non-NULL.  With double quant the consumer computes, in
 * kernel, absmax[b] = code2[qabsmax[b]] * absmax2[b / blocksize2] + *offset
 * (two separately rounded fp32 ops, = core.py:467-468).  Block indices are
 * global: b = block_base + (local flat element) / blocksize, so a row shard
 * can pass the unsliced scale arrays with block_base = row0 * K / blocksize. */

/* Fused 4-bit GEMV (decode, modules.py:56-61 -> core.py:426-504):
 *   y[r] = sum_k x[k] * lut[nib(r,k)] * absmax[blk(r,k)]  (+ bias[r]),
 * r in [0,M), B = packed rows (K/2 bytes each, high nibble first).
 * x/bias/y share `dtype` (QZ_DT_*); accumulation is fp32.  `lut` (16 fp32,
 * device) is optional: NULL selects the built-in codebook of `quant_type`
 * (| QZ_EXACT_CODES: the exact fp32 codes for fp16 x).  fp32 and bf16 x of
 * any finite magnitude are multiplied raw (fp32 FMAs / bf16 dot2 into fp32). */
int qz_gemv_4bit(int M, int K, const void *x, int dtype, const unsigned char *B, int quant_type, int blocksize,
                 const float *absmax, const unsigned char *qabsmax, const float *absmax2, const float *code2,
                 const float *offset, int blocksize2, long long block_base, const float *lut, const void *bias,
                 void *y, void *stream);

/* qz_gemv_4bit with a residual add in the epilogue -- LlamaDecoderLayer.forward's
 * `residual + h` (modeling_llama.py:316,322) on the o_proj / down_proj output:
 *   y[r] = round(residual[r] + round(gemv[r]))   (both roundings to `dtype`, as torch stores h
 * and then the sum), residual [M] of `dtype`.  One launch instead of two. */
int qz_gemv_4bit_residual(int M, int K, const void *x, int dtype, const unsigned char *B, int quant_type,
                          int blocksize, const float *absmax, const unsigned char *qabsmax, const float *absmax2,
                          const float *code2, const float *offset, int blocksize2, long long block_base,
                          const float *lut, const void *bias, const void *residual, void *y, void *stream);

/* Grouped decode GEMV: several Linear4bit layers that
 * read the SAME x (q/k/v, or gate/up, of one decoder layer) in ONE launch,
 * replacing nseg separate modules.py:56-61 calls.  Each segment keeps its own
 * packed weights, statistics, offset, bias and output y (length M);
 * K, x, dtype, quant_type, blocksize(2) and lut are shared, and every segment
 * must use the same scale format (all double-quant or all fp32 absmax).
 * 1 <= nseg <= QZ_GEMV_MAX_SEGMENTS. */
#define QZ_GEMV_MAX_SEGMENTS 4
typedef struct qz_gemv_segment {
  int M;
  const unsigned char *B;
  const float *absmax;          /* fp32 absmax, or NULL with double quant */
  const unsigned char *qabsmax; /* double quant: u8 codes */
  const float *absmax2;
  const float *code2;
  const float *offset;
  long long block_base;
  const void *bias; /* or NULL */
  void *y;
} qz_gemv_segment;

int qz_gemv_4bit_grouped(int nseg, const qz_gemv_segment *segs, int K, const void *x, int dtype, int quant_type,
                         int blocksize, int blocksize2, const float *lut, void *stream);

/* The same launch with the layer's RMSNorm in front (extension; no reference
 * counterpart): every segment multiplies x' = norm_weight * rmsnorm(x, eps)
 * (LlamaRMSNorm, modeling_llama.py:62-67), computed once per workgroup in its
 * prologue and bit-identical to qz_rmsnorm's output, so the outputs equal
 * qz_rmsnorm followed by qz_gemv_4bit_grouped.  Takes one token of F16/BF16
 * activations, K % 2048 == 0, K <= 16384, 16-B-aligned x and norm_weight and
 * full-step scale layouts, and launches of at most 4096 workgroups (each one
 * repeats the norm; beyond that the two calls are faster); anything else
 * returns QZ_ERR_SHAPE (nothing is launched: run the two calls). */
int qz_gemv_4bit_grouped_rmsnorm(int nseg, const qz_gemv_segment *segs, int K, const void *x, int dtype,
                                 int quant_type, int blocksize, int blocksize2, const float *lut,
                                 const void *norm_weight, float eps, void *stream);

/* Fused 4-bit GEMM (prefill, modules.py:62-64): Y[T,M] = X[T,K] . W[M,K]^T
 * (+ bias).  W is decoded tile-by-tile into LDS as exactly the values
 * qz_dequantize_4bit would store (fp16/bf16 of code * absmax) and multiplied
 * on MFMA with fp32 accumulation.  X/Y/bias share `dtype` (F16 or BF16);
 * ldx/ldy are row strides in elements.  Requires K % 64 == 0, M % 4 == 0,
 * blocksize >= 64 (else QZ_ERR_SHAPE / QZ_ERR_BLOCKSIZE).  For small T the K
 * range is split across workgroups: pass a workspace of
 * qz_gemm_4bit_workspace_size(T, M, K) bytes (fp32 partials) to enable it;
 * with less (or none) the split is reduced accordingly. */
int qz_gemm_4bit(int T, int M, int K, const void *X, int ldx, int dtype, const unsigned char *B, int quant_type,
                 int blocksize, const float *absmax, const unsigned char *qabsmax, const float *absmax2,
                 const float *code2, const float *offset, int blocksize2, const void *bias, void *Y, int ldy,
                 float *workspace, long long workspace_bytes, void *stream);

/* Grouped multi-token GEMM (2 <= T <= 16 tokens, K % 256 == 0): the batched-
 * decode counterpart of qz_gemv_4bit_grouped -- segments that share X (e.g.
 * q/k/v or gate/up of one layer over a small batch) in ONE launch.  Segment
 * i writes y_i[T, M_i] (row stride M_i); every output is bit-identical to
 * qz_gemm_4bit on that segment alone (block_base as in qz_gemv_4bit).
 * Other T / K return QZ_ERR_SHAPE (run the segments one by one). */
int qz_gemm_4bit_grouped(int nseg, const qz_gemv_segment *segs, int T, int K, const void *X, int ldx, int dtype,
                         int quant_type, int blocksize, int blocksize2, void *stream);

/* Dense 16-bit GEMM Y[T,M] = X[T,K] . W[M,K]^T (+ bias), fp32 accumulation
 * (v_mfma_f32_16x16x32_{f16,bf16}), on the same staggered 8-phase 256x256 schedule as the
 * fused kernel.  The large-T prefill route: qz_dequantize_4bit (bit-exact 16-bit weight,
 * kernels.cu:554-560) then this GEMM -- modules.py:62-64's "dequantise, then F.linear",
 * both halves hand-written.  X/W/Y/bias share `dtype` (F16 or BF16); W is contiguous
 * [M][K]; row strides in elements.  Requires qz_gemm_16bit_ok(...) (K % 64 == 0, M % 8 == 0,
 * 16-B aligned X/W/Y, row strides % 8 == 0, 32-bit byte offsets), else QZ_ERR_SHAPE. */
int qz_gemm_16bit(int T, int M, int K, const void *X, int ldx, int dtype, const void *W, const void *bias, void *Y,
                  int ldy, void *stream);
int qz_gemm_16bit_ok(int T, int M, int K, const void *X, int ldx, const void *W, const void *Y, int ldy);

/* Workspace bytes qz_gemm_4bit uses for (T, M, K) at its preferred K split
 * (0 = no split). */
long long qz_gemm_4bit_workspace_size(int T, int M, int K);

/* 4-bit blockwise quantisation (quantize_4bit, core.py:507-559): A[n] of
 * `a_dtype` -> packed out[(n+1)/2] + fp32 absmax[ceil(n/blocksize)]. */
int qz_quantize_4bit(const void *A, int a_dtype, long long n, int blocksize, int quant_type, float *absmax,
                     unsigned char *out, void *stream);

/* Deterministic mean of absmax[n] (core.py:563), fixed fp64 reduction tree
 * (see DESIGN.md).  `workspace` must hold qz_absmax_mean_workspace(n) doubles. */
long long qz_absmax_mean_workspace(long long n);
int qz_absmax_mean(const float *absmax, long long n, double *workspace, float *offset, void *stream);

/* 8-bit blockwise quantisation with the 256-entry code (quantize_blockwise,
 * core.py:317-366).  If `subtract` (device fp32 scalar) is non-NULL the input
 * is A[i] - *subtract, fusing core.py:564. */
int qz_quantize_blockwise_8bit(const float *code, const float *A, long long n, int blocksize, const float *subtract,
                               float *absmax, unsigned char *out, void *stream);

/* 8-bit blockwise dequantisation (dequantize_blockwise, core.py:369-423);
 * optional `offset` fuses core.py:468. */
int qz_dequantize_blockwise_8bit(const float *code, const unsigned char *A, const float *absmax, long long n,
                                 int blocksize, const float *offset, float *out, void *stream);

/* 4-bit dequantisation to `out_dtype` (dequantize_4bit, core.py:581-631):
 * FP4 through the dDequantizeFP4Tree semantics (code 8 -> -0.0), NF4 via its
 * codebook; scale source as for qz_gemv_4bit (block_base = 0). */
int qz_dequantize_4bit(const unsigned char *A, long long n, int quant_type, int blocksize, const float *absmax,
                       const unsigned char *qabsmax, const float *absmax2, const float *code2, const float *offset,
                       int blocksize2, void *out, int out_dtype, void *stream);

/* Measurement helper (bench.py's roofline context, not on the product path):
 * one non-temporal 16-B read per thread over `bytes` of device memory -- the
 * one-shot HBM read floor of a buffer the GEMV's size. */
int qz_bench_read_floor(const void *p, long long bytes, unsigned int *sink, void *stream);

/* Measurement helper: one empty 64-thread launch -- the fixed back-to-back
 * period every dependent launch on a stream pays (dispatch + end of kernel). */
int qz_bench_empty(unsigned int *sink, void *stream);

/* ---- one-shot all-gather over xGMI (the row-split output exchange) ----
 * Replaces the RCCL all_gather_into_tensor behind parallel.RowShardedLinear4bit (no reference
 * counterpart: the reference is single-GPU).  Each rank allocates one exchange buffer of
 * qz_exchange_bytes(world, slot_bytes) bytes with qz_exchange_alloc (uncached device memory),
 * exports it with qz_ipc_get_handle (qz_ipc_handle_size() bytes), and maps the peers' buffers
 * with qz_ipc_open_handle (after qz_enable_peer_access to every peer device).  One
 * qz_allgather_oneshot launch then writes the world x nbytes shards of every rank, rank-major,
 * into dst (the layout all_gather_into_tensor produces); the shard words travel as 8-byte
 * {word, epoch} granules (one system-scope store each, read once tagged with the call's epoch).
 * epoch: a zeroed device u32[2] per buffer (epoch, ticket), advanced by every launch
 * (graph-capturable); status: a zeroed device u32 set to 1 if a peer's granules never arrived
 * (bounded wait, 5 s).  nbytes % 16 == 0, nbytes <= slot_bytes, 16-B aligned src/dst, world <= 8. */
int qz_ipc_handle_size(void);
long long qz_exchange_bytes(int world, long long slot_bytes);
int qz_exchange_alloc(long long bytes, void **ptr);
int qz_exchange_free(void *ptr);
int qz_ipc_get_handle(const void *ptr, void *handle);
int qz_ipc_open_handle(const void *handle, void **ptr);
int qz_ipc_close_handle(void *ptr);
int qz_enable_peer_access(int peer_device);
int qz_allgather_oneshot(const void *src, int nbytes, void *dst, int rank, int world, void *const *peer_bufs,
                         void *own_buf, long long slot_bytes, unsigned int *epoch, unsigned int *status,
                         void *stream);
/* The same with the protocol forced: mode 1 = flag protocol (16-B stores into plain slots,
 * a store-completion wait, one epoch flag per peer), 2 = tagged granules.  qz_allgather_oneshot
 * takes granules up to 2 KiB per rank and flags above (measured). */
int qz_allgather_oneshot_mode(const void *src, int nbytes, void *dst, int rank, int world, void *const *peer_bufs,
                              void *own_buf, long long slot_bytes, unsigned int *epoch, unsigned int *status,
                              int mode, void *stream);

/* ---- the Linear4bit's callers in a Llama decoder layer (integration.fuse_layer_ops) ----
 * Neither op is in the reference (it leaves them to transformers); they are
 * one-launch restatements of the torch code around the 4-bit projections, with
 * torch's fp32 opmath and its per-op rounding, so that a decode step is not
 * dominated by ~8 small launches per norm and ~10 per rotary application. */

/* LlamaRMSNorm.forward (transformers modeling_llama.py:62-67) over `rows` rows
 * of K elements: h = fp32(x); var = sum(h*h) * (1/K); h *= rsqrt(var + eps);
 * y = weight * round_to_dtype(h) (fp32 product, rounded to `dtype`).  x, weight
 * and y share `dtype`; row strides ldx/ldy are in elements. */
int qz_rmsnorm(const void *x, int dtype, long long rows, int K, long long ldx, const void *weight, float eps, void *y,
               long long ldy, void *stream);

/* `residual + x` followed by the RMSNorm above (LlamaDecoderLayer.forward:317-321)
 * in one launch: sum = round_to_dtype(residual + x) is stored (the new residual
 * stream) and y = rmsnorm(sum).  residual shares x's row stride ldx; sum and y
 * use ldy. */
int qz_add_rmsnorm(const void *x, const void *residual, int dtype, long long rows, int K, long long ldx,
                   const void *weight, float eps, void *sum, void *y, long long ldy, void *stream);

/* apply_rotary_pos_emb (modeling_llama.py:130-160) for q AND k in one launch:
 * out = x*cos + rotate_half(x)*sin, each product and the sum rounded to `dtype`
 * as torch does.  q/k are [B, H, S, D] with element strides (b, h, s) given in
 * q_str/k_str (d contiguous); outputs use qo_str/ko_str; cos/sin are [B, S, D]
 * with strides cs_str (b, s) (stride 0 broadcasts).  D must be even. */
int qz_rope_qk(int dtype, int B, int S, int D, const void *q, int Hq, const long long *q_str, void *q_out,
               const long long *qo_str, const void *k, int Hk, const long long *k_str, void *k_out,
               const long long *ko_str, const void *cos, const void *sin, const long long *cs_str, void *stream);

/* LlamaMLP's act_fn(gate_proj(x)) * up_proj(x) for hidden_act "silu"
 * (modeling_llama.py:175): y = round(round(g / (1 + exp(-g))) * u) over n
 * contiguous elements of `dtype` (torch's two rounded elementwise ops). */
int qz_silu_mul(const void *gate, const void *up, int dtype, long long n, void *y, void *stream);


/* One new token of LlamaAttention.forward (modeling_llama.py:243-281) against a static KV
 * cache, from the q/k/v projection outputs to the o_proj input, in one launch (two when
 * L > 128): rotary of q and k (qz_rope_qk's arithmetic; the cache receives the same bits),
 * StaticLayer.update (cache_utils.py:455-487: k_cache/v_cache[b, :, p] = k, v with
 * p = *pos, then *pos = p + 1) and sdpa_attention_forward's masked GQA attention
 *   out[b, hq] = softmax_j(mask[b, j] ? (q[b, hq] . k_cache[b, hq / (Hq / Hkv), j]) * scale : -inf) v
 * in fp32 (scores, probabilities, accumulation), rounded once to `dtype`.
 *   q [B, Hq*D], k/v [B, Hkv*D]: row strides q_row/k_row/v_row elements, head-major;
 *   cos/sin [B or 1, D]: row stride cs_row (0: one row for every b);
 *   k_cache/v_cache [B, Hkv, L, D] contiguous, 16-B aligned; mask bool, (b, j) at
 *   b*mask_b + j*mask_j; pos int64 (device); arrive: a device uint32 that is 0 before the
 *   call and is left 0; out [B, Hq*D] with row stride out_row;
 *   work: L > 128 only, B*Hkv*ceil(L/128)*(Hq/Hkv)*(D+2) floats.
 * F16/BF16, D in {64, 128}, Hq/Hkv <= 8; otherwise QZ_ERR_SHAPE / QZ_ERR_DTYPE, nothing launched. */
int qz_decode_attention(int dtype, int B, int Hq, int Hkv, int D, int L, const void *q, long long q_row,
                        const void *k, long long k_row, const void *v, long long v_row, const void *cos,
                        const void *sin, long long cs_row, void *k_cache, void *v_cache, const void *mask,
                        long long mask_b, long long mask_j, long long *pos, unsigned int *arrive, void *out,
                        long long out_row, float *work, float scale, void *stream);

/* Decode-step glue of the host model (transformers' LlamaModel.forward), one launch each in place
 * of the small torch kernels it issues per step.  Not part of the Linear4bit path; the
 * integration (integration.fuse_decode_glue) takes them only where they give the same values.
 * qz_decode_mask: masking_utils.create_causal_mask for one new token against a static cache
 *   (sdpa, causal, no padding mask, kv_offset 0): mask[b*L + j] = (j <= *q_offset), bool bytes,
 *   q_offset = StaticLayer.cumulative_length (device int64, read in-kernel).
 * qz_rope_table: LlamaRotaryEmbedding.forward for positions pos[b*pos_b + s*pos_s]: cos/sin
 *   [B, S, D] contiguous copied from the [T, D] tables that module computed for positions 0..T-1;
 *   a position outside [0, T) is computed from inv_freq [D/2] (fp32 product, cosf/sinf, * scale,
 *   rounded to dtype).  D even; F16/BF16/F32. */
/* qz_greedy_step: the greedy pick and its feedback (two launches: 2048 logits per workgroup, then
 *   one workgroup over the partials): for b < B, next = argmax_v logits[b*row + v] (v < V;
 *   torch.argmax's order: NaN above every number, the first index among equals),
 *   hist[b*hist_row + *pos] = next (skipped when *pos is outside [0, hist_len)), tok[b] = next; then
 *   *pos += 1.  int64 hist/pos/tok on the
 *   device (graph-capturable); F16/BF16/F32 logits; work: qz_greedy_step_work_bytes(B, V) bytes. */
long long qz_greedy_step_work_bytes(int B, long long V);
int qz_greedy_step(const void *logits, int dtype, int B, long long V, long long row, long long *hist,
                   long long hist_row, long long hist_len, long long *pos, long long *tok, void *work, void *stream);
/* qz_gemv_dense: the model's fp16/bf16 lm_head for one decode token (transformers keeps it
 *   unquantised): y[m] = sum_k W[m*K + k] x[k] for m < M, fp32 accumulation, rounded once to
 *   dtype; K in {4096, 8192}, W and x 16-B aligned (else QZ_ERR_SHAPE, nothing launched). */
int qz_gemv_dense(int M, int K, const void *x, int dtype, const void *W, void *y, void *stream);
int qz_decode_mask(const long long *q_offset, int B, int L, void *mask, void *stream);
int qz_rope_table(int dtype, int B, int S, int D, const long long *pos, long long pos_b, long long pos_s,
                  const void *cos_table, const void *sin_table, long long T, const float *inv_freq, float scale,
                  void *cos, void *sin, void *stream);

/* LlamaMLP's act_fn(gate_proj(x)) * up_proj(x) for hidden_act "silu" (modeling_llama.py:175) as
 * ONE launch: segs[0] = gate_proj, segs[1] = up_proj (equal M; their `y` are ignored), both
 * GEMVs as qz_gemv_4bit_grouped computes them, then h[r] = round(round(g / (1 + exp(-g))) * u)
 * on the rounded g[r], u[r] (qz_silu_mul's arithmetic) -- bit-identical to the grouped launch +
 * qz_silu_mul.  norm_weight (nullable): x is first RMSNorm'd as qz_gemv_4bit_grouped_rmsnorm does.
 * Where the grouped geometry splits K over waves (K = 8192: Llama-3-70B) the pair keeps whole rows
 * per wave -- another fp32 summation order, within fp16 rounding of the grouped launch, not its
 * bits; the QZ_PAIR_WK1 knob (qz_gemv_set_knob) = 1 declines a fused norm there (QZ_ERR_SHAPE: run
 * qz_rmsnorm, then this without the norm), 0 declines those geometries.
 * F16/BF16, full K-steps (K % 2048 == 0); otherwise QZ_ERR_SHAPE and nothing launched. */
int qz_gemv_4bit_pair_silu(const qz_gemv_segment *segs, int K, const void *x, int dtype, int quant_type,
                           int blocksize, int blocksize2, const float *lut, const void *norm_weight, float eps,
                           void *h, void *stream);

/* The launch-geometry measurement knobs in effect (QZ_GEMV_WIDE8, QZ_GROUPED_NORM_R, QZ_PAIR_R,
 * QZ_PAIR_WT, QZ_PAIR_PS, QZ_PAIR_WK1, and QZ_GEMM16_SCHED -- the schedule qz_gemm_16bit (default 971, persistent)
 * launches: environment variables read ONCE when the library is loaded) and the
 * device's CU count, as a JSON object written to buf (NUL-terminated when n > the length).
 * Returns the length of the JSON text.  No reference counterpart (measurement bookkeeping). */
int qz_gemv_knobs(char *buf, int n);
/* Sets one of those knobs explicitly (name as above; QZ_PAIR_PS -1 = the default grid), for
 * measurements and tests comparing launch forms.  QZ_OK, or QZ_ERR_ARG for an unknown name. */
int qz_gemv_set_knob(const char *name, int value);

/* Library/ABI version (major*10000 + minor*100 + patch). */
int qz_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QUANTIZATIONS_H */

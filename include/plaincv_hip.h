/* include/plaincv_hip.h -- C ABI of libplaincv_hip.so (gfx950 / MI355X).
 *
 * The drop-in boundary for plainCV's transformer training hot path.  The
 * reference (GeorgTirp/plainCV) is JAX/Flax/Optax: every op below replaces an
 * XLA-emitted kernel behind one of its Python call sites (cited per entry).
 *
 * Conventions
 *   - plain pointers + sizes; bf16 tensors are raw 16-bit words; "ld" = row
 *     stride in elements (bf16 operands of GEMM/attention need ld % 8 == 0 and
 *     16-byte aligned bases);
 *   - every function returns int: 0 ok, <0 invalid argument (-1 EINVAL,
 *     -2 alignment, -3 shape), >0 hipError_t;  pcv_last_error_string(code);
 *   - every launch goes on the caller's `stream` (hipStream_t), with no host
 *     synchronisation and no allocation, so a train step is hipGraph-capturable;
 *   - the caller owns every buffer (kernels never allocate); accumulating
 *     outputs ("+=") expect the caller to zero grads once per optimizer step.
 */
#ifndef PLAINCV_HIP_H
#define PLAINCV_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- GEMM ----
 * C = epi(alpha * op(A) . op(B)); A [M,K] (trans_a=0) or [K,M]; B [K,N]
 * (trans_b=0) or [N,K].  Epilogue: +bias[N] -> act (1 GELU-tanh, writes the
 * pre-activation to aux; 2 multiplies by gelu'(aux)) -> dropout -> +res_scale*res
 * -> store (bf16, or fp32 with C = v + beta*C; split_k>1 = fp32 atomic accumulate).
 * colsum (optional, fp32) += column sums of the stored tile.  col_reps > 1: colsum (and
 * pcv_gemm_ln's ln_dscale / ln_dbias) is a [col_reps][N] block and workgroup b adds into row
 * b % col_reps (spreads the float atomics of hundreds of workgroups over several rows); the
 * caller folds the rows, e.g. with a zero_after column-sum job of pcv_gemm_grouped.
 * attn_delta (optional; bf16 C whose N columns are attn_H heads of 32 or 64, rows b*attn_T + t):
 * attn_delta[(b*attn_H + h)*attn_T + t] = <bf16 C row head h, attn_o row head h> -- the
 * attention-backward row constant computed where dO is produced (see pcv_attn_bwd delta_ready).
 * Replaces every flax nn.Dense / DenseGeneral / Conv(patch) contraction:
 * models/vit_small.py:13-16,41-45,78-88,126; models/LM/transformer.py:194-201,
 * 246-253,110-134,393-405 and their autodiff transposes. */
int pcv_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K,
                  int64_t lda, int64_t ldb, int64_t ldc, int trans_a, int trans_b,
                  int64_t batch, int64_t stride_a, int64_t stride_b, int64_t stride_c,
                  float alpha, float beta, int out_f32,
                  const float* bias, const void* res, int64_t ldr, int64_t stride_r, int res_f32, float res_scale,
                  void* aux, int64_t ldaux, int act,
                  float dropout_rate, const uint32_t* seed, uint32_t site, float* colsum, int col_reps,
                  const void* attn_o, int64_t ld_attn_o, const void* attn_o_lo, float* attn_delta, int attn_T,
                  int attn_H, int split_k, void* stream);

/* 256x256 8-wave ping-pong GEMM (csrc/gemm_big.hip) for large products with BOTH operands
 * K-contiguous: C[M,N] (bf16) = alpha * A[M,K] . B[N,K]^T (+ res_scale * res (bf16)).  pcv_gemm_bf16
 * dispatches to it by itself when pcv_gemm_big_ok() (eligible shape, >= 512 tiles, enabled);
 * pcv_gemm_big_enable(on) toggles that dispatch (on < 0: query) and returns the previous state.
 * Replaces the same flax Dense contractions as pcv_gemm_bf16 (the LM forward and dgrad GEMMs). */
int pcv_gemm_big_enable(int on);
int pcv_gemm_big_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb);
int pcv_gemm_big(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                 int64_t ldc, float alpha, const void* res, int64_t ldr, float res_scale, void* stream);
/* C[M,N] (bf16) = A[M,K] . B[N,K]^T and delta[(b H + h) T + t] = <C[row, head h], attn_o[row, head h]>
 * (head width N / H in {32, 64}, row = b T + t): pcv_gemm_bf16's attn_delta epilogue on the 256-wide
 * kernel, which pcv_gemm_bf16 takes by itself for eligible shapes (PCV_EINVAL otherwise).  Replaces the
 * LM's out-projection data gradient and the attention VJP's row constant (transformer.py:246-253,
 * 228-240). */
int pcv_gemm_big_attn_delta(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, const void* attn_o, int64_t ld_o, float* delta, int T, int H,
                            void* stream);
/* C[M,N] (bf16) = A[M,K] . B[N,K]^T with the forward RoPE on columns [0, rope_cols) (heads of head_dim,
 * row r at position r % T, cos/sin fp32 [T][head_dim/2]): the LM's qkv Dense product and the rotation
 * of its q | k heads (models/LM/transformer.py:194-201, embedding.py:29-66) -- pcv_gemm_bf16 + pcv_rope in
 * one pass (the rotation on the bf16-rounded product in the 256-wide kernel's epilogue; otherwise the
 * two launches). */
int pcv_gemm_rope(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                  int64_t ldc, int rope_cols, int T, int head_dim, const float* cos_tab, const float* sin_tab,
                  void* stream);
/* gu = A[M,K] . W_gu^T ([gate | up] halves Fp = F rounded to 8 apart, pads 0) and h = silu(gate) * up
 * ([M][ldh >= Fp], pads 0) in one pass: the LM's fc_gate / fc_up products and the GLU
 * (models/LM/transformer.py:110-134).  Bi = the weight rows K-contiguous, interleaved in 128-row blocks
 * ([gate rows 128j..128j+127 | up rows 128j..] per block j, zero rows past F; 256 ceil(F/128) rows).
 * pcv_gemm_swiglu_fwd_ok(): whether the 256-wide kernel takes the product (otherwise run pcv_gemm_bf16 on
 * the plain layout + pcv_swiglu_fwd). */
int pcv_gemm_swiglu_fwd_ok(int64_t M, int64_t F, int64_t K, const void* A, int64_t lda, const void* Bi, int64_t ldb);
int pcv_gemm_swiglu_fwd(const void* A, const void* Bi, int64_t M, int64_t F, int64_t K, int64_t lda, int64_t ldb,
                        void* gu, int64_t ldgu, void* h, int64_t ldh, void* stream);
/* dgu = SwiGLU VJP of dh = A[M,K] . B[F,K]^T against gu = [gate | up] (halves Fp = F rounded to 8
 * apart; pad columns of dgu written 0): the LM's fc2 data gradient and the GLU backward
 * (models/LM/transformer.py:110-134) in one pass, dh never stored; products the 256-wide kernel does
 * not take run as pcv_gemm_bf16 into the caller's dh [M][lddh >= Fp] + pcv_swiglu_bwd. */
int pcv_gemm_swiglu_bwd(const void* A, const void* B, int64_t M, int64_t F, int64_t K, int64_t lda, int64_t ldb,
                        const void* gu, int64_t ldgu, void* dgu, int64_t lddgu, void* dh, int64_t lddh, void* stream);
/* Persistent form (csrc/gemm_stream.hip): one workgroup per CU, the 32-deep K steps of all its
 * 256x256 / 256x192 output tiles in one continuous LDS-DMA ring, epilogue stored straight from the
 * accumulators (operand-swapped MFMAs, 16-B column chunks).  Same product and operand rules as
 * pcv_gemm_big (K % 32 != 0 allowed: the tail goes through registers).  pcv_gemm_bf16 prefers it when
 * pcv_gemm_stream_ok(); pcv_gemm_stream_enable(on) toggles that (on < 0: query).  Replaces the LM's
 * forward / data-gradient Dense products incl. the vocabulary-wide lm_head (transformer.py:393-405). */
int pcv_gemm_stream_enable(int on);
int pcv_gemm_stream_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb);
int pcv_gemm_stream(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                    int64_t ldb, int64_t ldc, float alpha, const void* res, int64_t ldr, float res_scale,
                    void* stream);
/* Grouped deterministic split-K weight gradients (csrc/gemm_wgrad.hip): for j < njobs (<= 8),
 * C_j[M,N] (fp32) = beta * C_j + alpha * A_j[K,M]^T . B_j[K,N], A_j [K][lda >= M] and B_j [K][ldb >= N]
 * bf16 (K-major: the Dense layer's inputs and output gradients), dims[6 j ..] = {M, N, K, lda, ldb,
 * ldc}, K % 32 == 0.  256 x 256 tiles, K split `splits` ways (0: automatic); the splits' fp32
 * partials go to workspace slabs and the last split of each tile sums them in split order, so the
 * result is run-to-run identical.  ws: pcv_gemm_wgrad_ws_bytes() bytes (0 when the plan has one
 * split), zero-filled once before first use (tile tickets the kernel leaves at zero).  Replaces the
 * kernel cotangents X^T dY of the LM's Dense layers and lm_head (transformer.py:194-201, 246-253,
 * 110-134, 393-405 VJPs; accumulated over micro-steps with beta = 1, train_lm.py:189-241). */
int64_t pcv_gemm_wgrad_ws_bytes(int njobs, const int64_t* dims, int splits);
int pcv_gemm_wgrad_grouped(int njobs, const void* const* A, const void* const* B, float* const* C,
                           const int64_t* dims, float alpha, float beta, int splits, void* ws, int64_t ws_bytes,
                           void* stream);
/* Weight-gradient form of the same kernel: C[M,N] (fp32) += alpha * A[K,M]^T . B[K,N] with A and B
 * K-major (M-/N-contiguous rows), K split over the grid and added with fp32 atomics (K % 32 == 0).
 * pcv_gemm_bf16 dispatches trans_a, !trans_b, fp32-out, beta == 1 products without epilogue here.
 * Replaces the kernel cotangents X^T dY of the LM's flax Dense layers (transformer.py:194-201,
 * 246-253, 110-134, 393-405 VJPs). */
int pcv_gemm_big_wgrad_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb);
int pcv_gemm_big_wgrad(const void* A, const void* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                       int64_t ldb, int64_t ldc, float alpha, void* stream);

/* GEMM + LayerNorm over each complete output row (N <= 128, N % 8 == 0; ViT residual stream).
 * ln_mode 1: C = x1 = alpha*op(A)op(B) + bias (+dropout) + res (fp32); ln_y = bf16 LN(x1),
 *            ln_mean / ln_rstd written (flax LayerNorm fwd, models/vit_small.py:38,52).
 * ln_mode 2: dy = alpha*op(A)op(B); C = dx = res + LN_bwd(dy; ln_x, ln_mean, ln_rstd, ln_scale);
 *            y = dropout_bwd(dx) (site/seed/rate of the sublayer below; rate 0: y = dx):
 *            ln_y = bf16(y) (optional), colsum += sum y; ln_dscale += sum dy*xhat, ln_dbias += sum dy;
 *            requires trans_b (B stored [N][K]: the dgrad against the weight rows).
 * col_reps = -1: ln_dscale / ln_dbias / colsum are [ceil(M/64)][N] blocks, each 64-row output tile
 * storing its partial to its own row (plain stores, deterministic; a column-sum job adds them). */
int pcv_gemm_ln(const void* A, const void* B, float* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, int trans_a, int trans_b, float alpha, const float* bias, const float* res, int64_t ldr,
                float dropout_rate, const uint32_t* seed, uint32_t site, int ln_mode, const float* ln_scale,
                const float* ln_bias, float ln_eps, void* ln_y, int64_t ld_lny, float* ln_mean, float* ln_rstd,
                const float* ln_x, int64_t ld_lnx, float* ln_dscale, float* ln_dbias, float* colsum, int col_reps,
                void* stream);

/* Grouped weight-gradient GEMM: n independent C_i[M,N] (fp32) += alpha_i * A_i^T B_i with
 * A_i [K][M], B_i [K][N] bf16 (row strides lda/ldb % 8 == 0, 16-B aligned bases), each split
 * split_k_i ways over K (fp32 atomics), ONE launch for all of them -- the flax autodiff
 * kernel gradients of every Dense in a backward pass (models/vit_small.py:41-45,78-88).
 * Descriptor (pcv_gemm_desc_size() bytes): {A, B, C, M, N, K, lda, ldb, ldc, alpha, split_k, kind, a_f32,
 * zero_after, pad}.
 * kind 1 = column-sum job in the same launch (bias gradients): C[c] += sum_r A[r, c] over A
 * [M][N] (bf16, or fp32 if a_f32; N % 8 == 0), rows split split_k ways; zero_after (fp32 only)
 * resets A after reading it (the fold of col_reps replica rows, below).
 * plan: host descriptors -> device plan buffer (pcv_gemm_grouped_plan_size(n) bytes, caller
 * owned, synchronous copy); run: stream-ordered, graph-capturable.  No two descriptors of a
 * plan may share a C.  sk_ws (optional, pcv_gemm_grouped_ws_floats(...) floats, 16-B aligned):
 * split-K slices write their partial tiles there with plain stores instead of fp32 atomics into C,
 * and pcv_gemm_grouped_fold (after run, fold_blocks from the plan) adds them to C in slice order --
 * deterministic and free of contended atomics. */
int64_t pcv_gemm_grouped_plan_size(int n);
int pcv_gemm_desc_size(void);
int64_t pcv_gemm_grouped_ws_floats(const void* descs, int n, int tile);
int pcv_gemm_grouped_plan(const void* descs, int n, int tile /* 64 | 128 */, void* plan_dev, int64_t* total_blocks,
                          float* sk_ws, int64_t ws_floats, int64_t* fold_blocks);
int pcv_gemm_grouped_run(const void* plan_dev, int n, int tile /* as planned */, int64_t total_blocks, void* stream);
int pcv_gemm_grouped_fold(const void* plan_dev, int n, int tile, int64_t fold_blocks, void* stream);

/* ----------------------------------------------------------- attention ----
 * Flash attention on the packed QKV activation (q/k/v = column blocks, head h
 * at column h*head_dim); lse2[B,H,T] is log2-domain.  head_dim in {32,64,128}.
 * Replaces flax SelfAttention's dot_product_attention (models/vit_small.py:41-45,
 * broadcast dropout over batch/heads) and jax.nn.dot_product_attention(is_causal)
 * (models/LM/transformer.py:233-240). */
int pcv_attn_fwd(const void* q, const void* k, const void* v, int64_t ldq, void* out, int64_t ldo,
                 float* lse2, int B, int T, int H, int head_dim, int causal,
                 float dropout_rate, const uint16_t* drop_mask, const int* doc_start, const int* doc_end,
                 void* out_lo, void* stream);
int pcv_attn_bwd(const void* q, const void* k, const void* v, int64_t ldq,
                 const void* o, int64_t ldo, const void* dout, int64_t lddo,
                 const float* lse2, float* delta_ws /* [B,H,T] */,
                 void* dq, void* dk, void* dv, int64_t lddq,
                 int B, int T, int H, int head_dim, int causal,
                 float dropout_rate, const uint16_t* drop_mask, int delta_ready, const int* doc_start,
                 const int* doc_end, const void* o_lo, void* stream);
/* pcv_attn_bwd followed by the inverse RoPE of the q and k heads of dq / dk (pcv_rope backward on both):
 * the attention VJP through apply_rotary_emb (models/LM/transformer.py:228-240, embedding.py:29-66).
 * cos/sin fp32 [T][head_dim/2]; no o_lo.  The tiled kernels rotate the bf16-rounded values in their
 * stores; the short-sequence path runs the two rope launches after it. */
int pcv_attn_bwd_rope(const void* q, const void* k, const void* v, int64_t ldq,
                      const void* o, int64_t ldo, const void* dout, int64_t lddo,
                      const float* lse2, float* delta_ws, void* dq, void* dk, void* dv, int64_t lddq,
                      int B, int T, int H, int head_dim, int causal, float dropout_rate,
                      const uint16_t* drop_mask, int delta_ready, const int* doc_start, const int* doc_end,
                      const float* cos_tab, const float* sin_tab, void* stream);
/* out_lo / o_lo (optional, short-sequence path only -- pcv_attn_short_ok): the forward also
 * writes O's bf16 rounding residual O - bf16(O) (row stride ldo, P.V accumulated with P split
 * into bf16 hi + lo), and the backward forms delta = <dO, O_hi + O_lo> from it, so delta
 * matches the backward's own fp32 softmax P.  Required for deep-layer dQ accuracy when keys
 * share a large common component (DESIGN.md §3).  PCV_EINVAL elsewhere, or with delta_ready. */
int pcv_attn_short_ok(int T, int head_dim, int causal);
/* (delta_ready: delta_ws already holds rowsum(dO * O) per (b, h, t) -- pcv_gemm_bf16's
 * attention-delta epilogue on the GEMM that produced dO -- so its kernel is skipped.)
 * doc_start/doc_end (optional, causal only): int32 [B*T], the intra-document causal mask of
 * train_lm.py:107-131 / data_prep_utils.py:14-43 -- key k is visible to query t iff
 * doc_start[t] <= k <= t; doc_end[t] = end (exclusive) of t's document.  Key/query tiles outside
 * a block's documents are skipped, so short documents cost proportionally less. */
 * Attention-weight dropout mask: flax draws ONE [T,T] keep mask per layer and
 * broadcasts it over batch and heads (models/vit_small.py:41-45, nn.Dropout with
 * broadcast_dims (0,1) inside dot_product_attention).  Drawn once per step for
 * `layers` consecutive layers (site = site + l*site_stride) into packed bits,
 * pcv_attn_mask_words(T) uint16 words per layer; read by pcv_attn_fwd/bwd. */
int64_t pcv_attn_mask_words(int T);
int pcv_attn_drop_mask(const uint32_t* seed, uint32_t site, uint32_t site_stride, int layers, int T,
                       float dropout_rate, uint16_t* mask, void* stream);

/* --------------------------------------------------------------- norms ----
 * flax LayerNorm (models/vit_small.py:38,52,124) on the fp32 residual stream,
 * bf16 output; backward adds into dres (may alias dx) and accumulates dscale/dbias.
 * flax RMSNorm (models/LM/transformer.py:41-47) on the bf16 residual stream. */
int pcv_layernorm_fwd(const float* x, int64_t ldx, const float* scale, const float* bias, void* y,
                      int64_t ldy, float* mean, float* rstd, int64_t R, int D, float eps, void* stream);
int pcv_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* scale,
                      const float* mean, const float* rstd, const float* dres, int64_t ldres,
                      float* dx, int64_t lddx, void* dx_bf16, int64_t lddxb, float* dscale, float* dbias,
                      int64_t R, int D, void* stream);
int pcv_rmsnorm_fwd(const void* x, int64_t ldx, const float* scale, void* y, int64_t ldy, float* rstd,
                    int64_t R, int D, float eps, void* stream);
int pcv_rmsnorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* scale,
                    const float* rstd, const void* dres, int64_t ldres, void* dx, int64_t lddx,
                    float* dscale, int64_t R, int D, void* stream);
/* Parameter gradients alone (the *_bwd entries skip them when dscale is NULL), so a
 * caller can run them on a side stream beside the data-gradient chain. */
int pcv_layernorm_param_grad(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* mean,
                             const float* rstd, float* dscale, float* dbias, int64_t R, int D, void* stream);
int pcv_rmsnorm_param_grad(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* rstd,
                           float* dscale, int64_t R, int D, void* stream);

/* flax BatchNorm (models/vit_small.py:35-36,49-50,121-122; use_batchnorm=True): momentum 0.99,
 * eps 1e-5, column statistics over all R rows.  stats: train -> batch mean/rstd (fast variance) and
 * the running averages updated in place (flax_engine.py:74-85 mutable batch_stats); eval -> mean /
 * rstd from the running averages (ws unused).  apply: y = (x-mean)*rstd*scale+bias (bf16), any rows
 * of the same columns (the final norm normalises only the cls rows with the full-batch stats).
 * bwd (train mode): dx = dres + scale*rstd*(dy - mean(dy) - xhat*mean(dy*xhat)); dscale/dbias +=.
 * Deterministic (fixed-order partial reduction, no float atomics).  ws: workspace_size(R, D) bytes. */
size_t pcv_batchnorm_workspace_size(int64_t R, int D);
int pcv_batchnorm_stats(const float* x, int64_t ldx, int64_t R, int D, int train, float momentum, float eps,
                        float* ra_mean, float* ra_var, float* mean, float* rstd, void* ws, size_t ws_bytes,
                        void* stream);
int pcv_batchnorm_apply(const float* x, int64_t ldx, int64_t R, int D, const float* mean, const float* rstd,
                        const float* scale, const float* bias, void* y, int64_t ldy, void* stream);
/* the fp32 ViT runner's BatchNorm (models/vit_f32.py): the same normalisation, fp32 output
   (the reference BatchNorm ViT computes in fp32, vit_small.py:95) */
int pcv_batchnorm_apply_f32(const float* x, int64_t ldx, int64_t R, int D, const float* mean, const float* rstd,
                            const float* scale, const float* bias, float* y, int64_t ldy, void* stream);
int pcv_batchnorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t R, int D,
                      const float* mean, const float* rstd, const float* scale, const float* dres, int64_t ldres,
                      float* dx, int64_t lddx, void* dx_bf16, int64_t lddxb, float* dscale, float* dbias,
                      void* ws, size_t ws_bytes, void* stream);

/* --------------------------------------------------------- elementwise ----
 * RoPE, in place on the q|k column blocks (models/LM/embedding.py:28-66; backward = rotation by -theta). */
int pcv_rope(void* qk, int64_t ld, int64_t R, int ncols, int T, int head_dim, const float* cos_tab,
             const float* sin_tab, int backward, void* stream);
/* SwiGLU h = silu(gate)*up on the packed [gate|up] activation (models/LM/transformer.py:110-134):
 * gate at columns [0,F), up at [Fp, Fp+F) with Fp = F padded to 8; pad columns are written as 0. */
int pcv_swiglu_fwd(const void* gu, int64_t ldgu, void* h, int64_t ldh, int64_t R, int F, int Fp, void* stream);
int pcv_swiglu_bwd(const void* dh, int64_t lddh, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu,
                   int64_t R, int F, int Fp, void* stream);
/* Non-gated LM MLPs: h = act(a) on the fc1 output a [R][Fp] (kind 1 silu: MLP,
 * models/LM/transformer.py:70-97; kind 2 relu^2: MLPReluSquared, 138-165); backward da = dh * act'(a)
 * (da may alias dh).  Pad columns [F, Fp) are written as 0. */
int pcv_mlp_act_fwd(const void* a, int64_t lda, void* h, int64_t ldh, int64_t R, int F, int Fp, int kind,
                    void* stream);
int pcv_mlp_act_bwd(const void* dh, int64_t lddh, const void* a, int64_t lda, void* da, int64_t ldda, int64_t R,
                    int F, int Fp, int kind, void* stream);
/* out = bf16(x * dropout_mask) (backward of an output dropout, models/vit_small.py:17). */
int pcv_dropout_bwd_cast(const float* x, int64_t ldx, void* out, int64_t ldo, int64_t R, int N,
                         float rate, const uint32_t* seed, uint32_t site, void* stream);
int pcv_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
/* Advance the device-resident dropout seed (one per train step; hipGraph-replay safe). */
int pcv_seed_next(uint32_t* seed, void* stream);
/* Step prologue: x[0:n) = 0 (the flat gradient buffer, 16-B aligned) and, if seed is given,
 * the dropout seed advanced as pcv_seed_next -- one launch (flax_engine.py:95-123's fresh
 * gradients and per-step dropout rng). */
int pcv_zero_seed(float* x, int64_t n, uint32_t* seed, void* stream);
/* out[c] += sum_r x[r,c]  (Dense bias gradients). */
/* out[c] += sum_r x[r][c]; ws (optional, pcv_colsum_ws_floats(R, N) floats): the row groups' partials
 * are stored there and added in order by a second launch (deterministic); ws null: fp32 atomics. */
int64_t pcv_colsum_ws_floats(int64_t R, int N);
int pcv_colsum(const void* x, int64_t ld, int64_t R, int N, int x_f32, float* out, float* ws, void* stream);
/* ViT patch embedding input (models/vit_small.py:78-88, (kh,kw,c) flatten, /255) and token
 * assembly cls|patches + pos_embedding + dropout (models/vit_small.py:95-109). */
int pcv_vit_patchify(const uint8_t* img, void* out, int B, int H, int W, int C, int patch, void* stream);
int pcv_vit_embed_fwd(const float* patch, const float* cls, const float* pos, float* x, void* x_bf16,
                      int B, int T, int D, float rate, const uint32_t* seed, uint32_t site, void* stream);
/* pcv_vit_embed_fwd followed by the first block's LayerNorm_0 in one launch (D <= 256, D % 4 == 0,
 * 16-B aligned x / patch / cls / pos / LN parameters): x as pcv_vit_embed_fwd, y = bf16(LN(x)) with row
 * stride ldy, mean / rstd per row -- bit-identical to the two-launch form (vit_small.py:110-116, 38). */
int pcv_vit_embed_ln_fwd(const float* patch, const float* cls, const float* pos, float* x, int B, int T, int D,
                         float rate, const uint32_t* seed, uint32_t site, const float* ln_scale, const float* ln_bias,
                         void* y, int64_t ldy, float* mean, float* rstd, float eps, void* stream);
/* The embedding VJP: g = dropout_vjp(dx); dpatch rows = bf16(g[b, 1:]); dpos += sum_b g; dcls += sum_b g[b, 0]
 * (fixed-order sums: run-to-run identical). */
int pcv_vit_embed_bwd(const float* dx, void* dpatch, float* dcls, float* dpos, int B, int T, int D, float rate,
                      const uint32_t* seed, uint32_t site, void* stream);
/* nn.Embed gather / scatter-add (models/LM/transformer.py:361-369). */
int pcv_embed_fwd(const int* ids, const void* table, int64_t ldt, void* out, int64_t ldo, int64_t R,
                  int D, int V, int* oob_flag, void* stream);
int pcv_embed_bwd(const int* ids, const void* dx, int64_t lddx, float* dtable, int64_t ldt, int64_t R,
                  int D, int V, void* stream);

/* fp32 ViT path (VisionTransformer(dtype="float32"): the reference ViT's own precision; every
 * contraction on the exact-fp32 MFMA via pcv_gemm_f32_grouped).  patchify: uint8 NHWC -> fp32/255
 * patches (models/vit_small.py:78-95); LayerNorm with fp32 output; the Dense epilogue out =
 * dropout(act(x + bias)) + res_scale * res (act 1 = tanh-GELU, aux = pre-activation) and its VJP;
 * attention softmax over materialised scores S [rows = B*H*T][T] -> P and the weight-dropped Pd
 * (packed keep bits of pcv_attn_drop_mask), its VJP dS = P o (dP - rowsum(dP o P)) in place of dPd;
 * the embedding VJP with an fp32 patch gradient.  Dropout index = flat output index, as everywhere. */
int pcv_vit_patchify_f32(const uint8_t* img, float* out, int B, int H, int W, int C, int patch, void* stream);
int pcv_layernorm_fwd_f32(const float* x, int64_t ldx, const float* scale, const float* bias, float* y, int64_t ldy,
                          float* mean, float* rstd, int64_t R, int D, float eps, void* stream);
/* LayerNorm VJP with dscale/dbias (+=) computed in the same pass over dy and x (per-block partials
 * in ws, pcv_layernorm_bwd_f32_ws(R, D) floats, then one small reduction launch); D in
 * {64, 128, 256, 384, 512}, rows 16-B aligned (pcv_layernorm_bwd_f32_ok -> 0); dres may be NULL and
 * may alias dx.  dxd (optional): also dxd = dropout_vjp(dx) with keep = hash3(*seed, site, row*D+col)
 * (the next sublayer's dropout VJP, pcv_f32_epilogue_bwd's indexing).  Replaces pcv_layernorm_bwd + its parameter-gradient launch for the fp32 ViT
 * (models/vit_small.py:39-41 nn.LayerNorm under value_and_grad, flax_engine.py:95). */
int pcv_layernorm_bwd_f32_ok(int D, int64_t lddy, int64_t ldx, int64_t ldres, int64_t lddx);
int64_t pcv_layernorm_bwd_f32_ws(int64_t R, int D);
int pcv_layernorm_bwd_f32(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* scale,
                          const float* mean, const float* rstd, const float* dres, int64_t ldres, float* dx,
                          int64_t lddx, float* dscale, float* dbias, float* ws, int64_t ws_floats, int64_t R, int D,
                          float* dxd, int64_t lddxd, float rate, const uint32_t* seed, uint32_t site, void* stream);
/* dscale == dbias == NULL: the partials stay in ws and a later pcv_layernorm_part_reduce adds the
 * partials of several LayerNorms in one launch (device table of {part, dscale, dbias, nblk, D}). */
int pcv_layernorm_part_job_size(void);
int pcv_layernorm_part_reduce(const void* jobs, int njobs, int max_D, int64_t max_nblk, void* stream);
/* pcv_layernorm_part_reduce + the step's metrics (pcv_mean2 of loss / correct: metrics = [mean loss, mean
 * accuracy] * n * scale) in the same launch -- the training step's metrics taken off a launch of their own */
int pcv_layernorm_part_reduce_metrics(const void* jobs, int njobs, int max_D, int64_t max_nblk, const float* loss,
                                      const float* correct, int64_t n, float scale, float* metrics, void* stream);
int pcv_f32_epilogue(const float* x, int64_t ldx, const float* bias, const float* res, int64_t ldr, float res_scale,
                     float* aux, int64_t ldaux, float* out, int64_t ldo, int64_t R, int N, int act, float rate,
                     const uint32_t* seed, uint32_t site, void* stream);
int pcv_f32_epilogue_bwd(const float* dy, int64_t lddy, const float* aux, int64_t ldaux, float* dx, int64_t lddx,
                         int64_t R, int N, int act, float rate, const uint32_t* seed, uint32_t site, void* stream);
int pcv_attn_softmax_f32(const float* S, float* P, float* Pd, int64_t rows, int T, const uint16_t* mask, float rate,
                         void* stream);
int pcv_attn_softmax_bwd_f32(const float* P, float* dPd, int64_t rows, int T, const uint16_t* mask, float rate,
                             void* stream);
/* x[b,t] = dropout((t == 0 ? cls : patch[b,t-1] + bias) + pos[t]) in fp32 (the patch-conv bias
 * epilogue and flax's cls concat + pos add + Dropout, models/vit_small.py:95-109, in one pass; D % 4 == 0) */
int pcv_vit_embed_fwd_f32(const float* patch, const float* bias, const float* cls, const float* pos, float* x, int B,
                          int T, int D, float rate, const uint32_t* seed, uint32_t site, void* stream);
int pcv_vit_embed_bwd_f32(const float* dx, float* dpatch, float* dcls, float* dpos, int B, int T, int D, float rate,
                          const uint32_t* seed, uint32_t site, void* stream);
/* The cls-row chain of a cls-token ViT's last encoder block (after its cls-query attention), one launch
 * per direction, block = cls row b (rows b ldrow of the D-wide and b ldrowm of the M-wide tensors; the
 * dropout index uses the token row b T): forward x1 = o wo + bo + x, y1 = LayerNorm(x1; s1, c1, eps) (+
 * mean / rstd at b), pre = y1 w0 + b0, a = dropout(gelu(pre)) (site_h), xo = x1 + dropout(a w1 + b1)
 * (site_o); VJP da = dropout_vjp(dmo w1^T) gelu'(pre), dy1 = da w0^T, dx1 = dres + LayerNorm VJP(dy1),
 * dO = dx1 wo^T and the LayerNorm parameter partials part[b] = [dy1 xhat | dy1] (B partial rows for
 * pcv_layernorm_part_reduce).  The row GEMM epilogue's GELU / dropout conventions.  ok: D <= 256,
 * M <= 1024, D % 32 == 0, M % 32 == 0. */
int pcv_vit_cls_chain_f32_ok(int D, int M);
int pcv_vit_cls_chain_fwd_f32(const float* o, const float* x, const float* wo, int64_t ldwo, const float* bo,
                              const float* s1, const float* c1, const float* w0, int64_t ldw0, const float* b0,
                              const float* w1, int64_t ldw1, const float* b1, float* x1, float* y1, float* mean,
                              float* rstd, float* pre, float* a, float* xo, int64_t ldrow, int64_t ldrowm, int B, int T,
                              int D, int M, float eps, float rate, const uint32_t* seed, uint32_t site_h,
                              uint32_t site_o, void* stream);
int pcv_vit_cls_chain_bwd_f32(const float* dmo, const float* w1, int64_t ldw1, const float* pre, const float* w0,
                              int64_t ldw0, const float* x1, const float* s1, const float* mean, const float* rstd,
                              const float* dres, const float* wo, int64_t ldwo, float* da, float* dx1, float* dO,
                              float* part, int64_t ldrow, int64_t ldrowm, int B, int T, int D, int M, float rate,
                              const uint32_t* seed, uint32_t site_h, void* stream);
/* Fused fp32 classifier head (models/vit_small.py:111-127 + the softmax cross-entropy of
 * flax_engine.py:38-44): per cls row b (x + b ldx), yf = LayerNorm(x; scale, bias, eps) (+ mean / rstd),
 * logits = yf wh + bh (wh [D][Kc]), row_loss = lse - logits[label], row_correct = argmax == label (lowest
 * index on ties), dlogits = (softmax - onehot) grad_scale (NULL: none).  Its VJP: dyf = dlogits wh^T, the
 * LayerNorm VJP into dx's cls rows (dx + b lddx), the LayerNorm parameter partials part [B][2 D] =
 * [dyf xhat | dyf] (for pcv_layernorm_part_reduce with B partial rows), gwh += yf^T dlogits, gbh +=
 * column sums of dlogits -- fixed summation orders.  wh / gwh rows ldw / ldgw apart (the ParamStore pads
 * rows to 8).  dxd (optional): also the next consumer's dropout VJP of the dx cls rows, dxd[b] =
 * dropout_vjp(dx[b]) with index (b drow) D + d (the MLP-out dropout of the last block).  ok: D <= 256,
 * D % 16 == 0, Kc <= 1024 (and B <= 1024 for the VJP). */
int pcv_vit_head_f32_ok(int D, int Kc);
int pcv_vit_head_fwd_f32(const float* x, int64_t ldx, const float* scale, const float* bias, const float* wh,
                         int64_t ldw, const float* bh, const int* labels, float* yf, float* mean, float* rstd,
                         float* logits, float* row_loss, float* row_correct, float* dlogits, int B, int D, int Kc,
                         float eps, float grad_scale, void* stream);
int pcv_vit_head_bwd_f32(const float* dlogits, const float* wh, int64_t ldw, const float* x, int64_t ldx,
                         const float* scale, const float* mean, const float* rstd, const float* yf, float* dx,
                         int64_t lddx, float* part, float* gwh, int64_t ldgw, float* gbh, int B, int D, int Kc,
                         float* dxd, int64_t lddxd, int64_t drow, float rate, const uint32_t* seed, uint32_t site,
                         void* stream);
/* Fused fp32 patch embedding (models/vit_small.py:78-109): x[b, t] = dropout(t == 0 ? cls + pos[0] :
 * pos[t] + (patch(b, t - 1) . w + bias)) straight from the uint8 images (patch = the (kh, kw, c) flatten
 * / 255, w = Conv_0/kernel as [patch*patch*C][D]) -- pcv_vit_patchify_f32 + the patch GEMM +
 * pcv_vit_embed_fwd_f32 in one launch, same element order and dropout index.  Its VJP: dpos += sum_b g,
 * dcls += sum_b g[b, 0], gw += patches^T g[:, 1:], gbias += column sums of g[:, 1:] (g =
 * dropout_vjp(dx)), through ws (pcv_vit_patch_embed_bwd_f32_ws floats) in a fixed order.  ok: patch *
 * patch * C <= 48, D % 4 == 0, the LDS images fit (B <= ~200 at C = 3). */
int pcv_vit_patch_embed_f32_ok(int B, int H, int W, int C, int patch, int D);
int64_t pcv_vit_patch_embed_bwd_f32_ws(int B, int H, int W, int C, int patch, int D);
int pcv_vit_patch_embed_fwd_f32(const uint8_t* img, const float* w, const float* bias, const float* cls,
                                const float* pos, float* x, int B, int H, int W, int C, int patch, int D, float rate,
                                const uint32_t* seed, uint32_t site, void* stream);
/* pcv_vit_patch_embed_fwd_f32 + the first encoder block's LayerNorm_0 of every row (vit_small.py:38) in the same
 * pass: y [B*T][D] (flax LayerNorm, fast variance clipped at 0, ln_eps), mean / rstd [B*T] */
int pcv_vit_patch_embed_ln_fwd_f32(const uint8_t* img, const float* w, const float* bias, const float* cls,
                                   const float* pos, float* x, int B, int H, int W, int C, int patch, int D, float rate,
                                   const uint32_t* seed, uint32_t site, const float* ln_s, const float* ln_c, float* y,
                                   float* ln_mean, float* ln_rstd, float ln_eps, void* stream);
int pcv_vit_patch_embed_bwd_f32(const float* dx, const uint8_t* img, float* dcls, float* dpos, float* ws, float* gw,
                                float* gbias, int B, int H, int W, int C, int patch, int D, float rate,
                                const uint32_t* seed, uint32_t site, void* stream);
/* Exact-fp32 row-panel GEMM with the Dense epilogue fused (csrc/gemm_f32.hip): C[M][N] =
 * dropout(act(A[M][K] op(B) + bias)) + res_scale * res, op(B) = B [K][N] (tb = 0) or B^T with B
 * stored [N][K] (tb = 1); aux = the pre-activation when act = 1 (GELU tanh); act = 2 is the backward of
 * that MLP activation: C = dropout_vjp(A op(B)) * gelu'(aux) (aux read; no bias / res); dropout index row * N +
 * col (as pcv_f32_epilogue).  ok: N % 128 == 0, K % 64 == 0, 16-B aligned A / B, lda / ldb % 4 == 0. */
int pcv_gemm_f32_rows_ok(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb,
                         int tb);
int pcv_gemm_f32_rows(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C, int64_t ldc,
                      int64_t M, int64_t N, int64_t K, const float* bias, float* aux, int64_t ldaux, const float* res,
                      int64_t ldr, float res_scale, int act, float rate, const uint32_t* seed, uint32_t site,
                      void* stream);
/* The same product in the tiled form only (32 x 64 / 64 x 64 / 64 x 128 tiles; what pcv_gemm_f32_rows
 * runs for shapes outside the panel form).  pcv_gemm_f32_rows takes the panel form -- a persistent grid of
 * one workgroup per CU owning 64-row panels, the A strip in registers, op(B) streamed through LDS in
 * column blocks -- when pcv_gemm_f32_rows_form(M, N, K) is 1: K in {128, 256, 384}, M >= 64 and the rows
 * past the persistent panels fit one tail unit per workgroup. */
int pcv_gemm_f32_rows_tiled(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C, int64_t ldc,
                            int64_t M, int64_t N, int64_t K, const float* bias, float* aux, int64_t ldaux,
                            const float* res, int64_t ldr, float res_scale, int act, float rate, const uint32_t* seed,
                            uint32_t site, void* stream);
int pcv_gemm_f32_rows_form(int64_t M, int64_t N, int64_t K);
/* C = A B + bias, dropout, + res_scale res (pcv_gemm_f32_rows with tb = 0, act = 0) for N = 128, then the
 * LayerNorm of every C row -> ln_y (row stride ldy), ln_mean / ln_rstd [M] (flax LayerNorm, fast variance
 * clipped at 0, ln_eps): the ViT's attention residual -> LayerNorm_1 (models/vit_small.py:46, :52) and
 * MLP residual -> the next block's LayerNorm_0 (:56, :38) in one launch.  PCV_EINVAL for N != 128, K % 64.
 * ws (optional, pcv_gemm_f32_rows_lnout_ws_floats): the split tail, as pcv_gemm_f32_rows_ws. */
int pcv_gemm_f32_rows_lnout(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                            int64_t N, int64_t K, const float* bias, const float* res, int64_t ldr, float res_scale,
                            float rate, const uint32_t* seed, uint32_t site, const float* ln_s, const float* ln_c,
                            float* ln_y, int64_t ldy, float* ln_mean, float* ln_rstd, float ln_eps, float* ws,
                            int64_t ws_floats, void* stream);
/* floats of pcv_gemm_f32_rows_lnout's split-tail workspace at (M, K) (0: none; zeroed, one launch at a time) */
int64_t pcv_gemm_f32_rows_lnout_ws_floats(int64_t M, int64_t K);
/* dy = A B^T (B stored [N][K], N = 128; dy is not stored), then the LayerNorm VJP of every dy row: dx = dres +
 * rstd (g - mean(g) - xhat mean(g xhat)), g = dy scale, xhat = (x - mean) rstd (pcv_layernorm_bwd_f32's
 * arithmetic); dxd (optional) = dropout_vjp(dx) (rate, seed, site, index row * N + col); the column sums of
 * dy xhat / dy of each 32-row tile -> part[tile][0, N) / [N, 2 N) for pcv_layernorm_part_reduce (nblk =
 * ceil(M / 32); part_floats >= pcv_gemm_f32_rows_lnbwd_part_floats).  The ViT's MLP Dense_0 data gradient ->
 * LayerNorm_1 VJP and qkv data gradient -> LayerNorm_0 VJP (models/vit_small.py:46-56, :38) in one launch.
 * B2 / C2 (optional, both or neither): C2 = dx B2^T (B2 stored [N][N]) from the same rows in the same launch
 * (the attention out projection's data gradient after LayerNorm_1's VJP).
 * ws (optional, pcv_gemm_f32_rows_lnout_ws_floats(M, K)): the split tail, as pcv_gemm_f32_rows_lnout. */
int pcv_gemm_f32_rows_lnbwd(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                            const float* x, int64_t ldx, const float* scale, const float* mean, const float* rstd,
                            const float* dres, int64_t ldres, float* dx, int64_t lddx, float* part,
                            int64_t part_floats, float* dxd, int64_t lddxd, float rate, const uint32_t* seed,
                            uint32_t site, const float* B2, int64_t ldb2, float* C2, int64_t ldc2, float* ws,
                            int64_t ws_floats, void* stream);
int64_t pcv_gemm_f32_rows_lnbwd_part_floats(int64_t M, int64_t N);
/* pcv_gemm_f32_rows with a workspace for the split tail of its tiled form (data-gradient products, no
 * epilogue: the few tiles past a whole number of 4-per-CU rounds run as K slices beside the first round, the
 * tile's last slice adding the slabs in order); pcv_gemm_f32_rows_ws_floats gives the floats needed (0: no
 * split at this shape).  The workspace starts zeroed and is used by one launch at a time (stream order). */
int64_t pcv_gemm_f32_rows_ws_floats(int64_t M, int64_t N, int64_t K, int tb, int epi);
int pcv_gemm_f32_rows_ws(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C, int64_t ldc,
                         int64_t M, int64_t N, int64_t K, const float* bias, float* aux, int64_t ldaux, const float* res,
                         int64_t ldr, float res_scale, int act, float rate, const uint32_t* seed, uint32_t site,
                         float* ws, int64_t ws_floats, void* stream);
/* pcv_gemm_f32_rows whose dropout index of output row r is r * drop_row_step * N + col: the product of a
 * strided subset of the token rows (every drop_row_step-th, e.g. the cls rows b * T) with the dropout bits
 * those rows have in the full [rows][N] product. */
int pcv_gemm_f32_rows_rs(const float* A, int64_t lda, const float* B, int64_t ldb, int tb, float* C, int64_t ldc,
                         int64_t M, int64_t N, int64_t K, const float* bias, float* aux, int64_t ldaux,
                         const float* res, int64_t ldr, float res_scale, int act, float rate, const uint32_t* seed,
                         uint32_t site, int64_t drop_row_step, void* stream);
/* Attention of the cls query only (query 0 of each (b, h); head_dim 32, T <= 512): O row 0 and its row
 * statistics (mrow = max of the scaled scores, linv = 1 / sum at slot b H T + h T), the same numerics and
 * dropout keep bits as pcv_attn_fwd_f32's row 0; the VJP with dO nonzero only at query 0: dK / dV of
 * every key and dQ of query 0 (the other dQ rows are not written). */
int pcv_attn_cls_f32_ok(int T, int head_dim);
int pcv_attn_cls_fwd_f32(const float* qkv, int64_t ldqkv, float* out, int64_t ldo, float* mrow, float* linv, int B,
                         int T, int H, int D, const uint16_t* mask, float rate, void* stream);
int pcv_attn_cls_bwd_f32(const float* qkv, int64_t ldqkv, const float* dout, int64_t lddo, const float* mrow,
                         const float* linv, float* dqkv, int64_t lddqkv, int B, int T, int H, int D,
                         const uint16_t* mask, float rate, void* stream);
/* Every fp32 weight gradient of a step in one launch (csrc/gemm_f32.hip): jobs_dev holds njobs
 * records (pcv_gemm_f32_wgrad_job_size() bytes) {A, B, C, colsum, ws, lda, ldb, ldc, M, N, K, tiles_n,
 * tiles, ksplit, kchunk, first, ffirst, pad} (colsum optional: += the column sums of B -- the Dense's
 * bias gradient):  C[M][N] += A^T B with A [K][M], B [K][N] (K-major token rows), 64 x bn
 * panels x ksplit K slices; first = prefix sum of tiles * ksplit.  ws == NULL: the slices are added
 * with fp32 atomics; ws (tiles * ksplit * 64 * bn floats): each slice stores its partial tile there and
 * pcv_gemm_f32_wgrad_fold (fold_tiles = sum of tiles over the ws jobs; ffirst = their prefix) adds
 * the slices to C in order -- deterministic.  With colsum and ws, the first 64-row panel's column
 * partials go to ws + tiles * ksplit * 64 * bn ([N / bn][ksplit][bn] floats) and the fold adds them
 * to colsum in slice order too.
 * Requires M % 64, N % bn, K % 64, kchunk % 64 == 0, 16-B aligned operands, ld % 4 == 0. */
int pcv_gemm_f32_wgrad_job_size(void);
int pcv_gemm_f32_wgrad(const void* jobs_dev, int njobs, int64_t total_blocks, int bn, void* stream);
int pcv_gemm_f32_wgrad_fold(const void* jobs_dev, int njobs, int64_t fold_tiles, int bn, void* stream);
/* Blocked Householder QR (csrc/qr_blocked.hip; jnp.linalg.qr of SOAP's refresh, soap.py:108-133):
 * jobs {A, perm, Q, Wt, Qt, V, T, lda, ldq, n} (pcv_qrb_job_size() bytes; workspaces Wt, Qt, V
 * n x n and T n x nb, fp32).  init: Wt = A[:, perm]^T, Qt = I; panel(j0, nb): factorise columns
 * [j0, j0 + nb) of every matrix in LDS, write the reflector vectors into V and the block factor
 * into T (the caller then applies the trailing update and, backwards, the Q accumulation as GEMMs);
 * out: Q = Qt^T.  LAPACK sgeqrf / sorgqr conventions (same reflectors as pcv_householder_qr). */
int pcv_qrb_job_size(void);
size_t pcv_qrb_panel_lds(int max_n, int nb);
int pcv_qrb_init(const void* jobs, int njobs, int max_n, void* stream);
int pcv_qrb_panel(const void* jobs, int njobs, int max_n, int j0, int nb, void* stream);
int pcv_qrb_out(const void* jobs, int njobs, int max_n, void* stream);
/* Fused fp32 self-attention of one layer (flax MultiHeadDotProductAttention at
 * models/vit_small.py:41-45, fp32): qkv [B*T][ldqkv] holds q | k | v column blocks of width D = H * 32;
 * out [B*T][ldo] = softmax(q k^T / sqrt(32)) (weight dropout: packed keep words `mask`, rate) v;
 * mrow / linv [B*H*T] = each query's row max and 1/sum.  The backward writes dq | dk | dv into
 * dqkv's column blocks from qkv, out, dout and those stats.  ok: head_dim 32, 1 <= T <= 272. */
int pcv_attn_fused_f32_ok(int T, int head_dim);
int pcv_attn_fwd_f32(const float* qkv, int64_t ldqkv, float* out, int64_t ldo, float* mrow, float* linv, int B, int T,
                     int H, int D, const uint16_t* mask, float rate, void* stream);
int pcv_attn_bwd_f32(const float* qkv, int64_t ldqkv, const float* o, int64_t ldo, const float* dout, int64_t lddo,
                     const float* mrow, const float* linv, float* dqkv, int64_t lddqkv, int B, int T, int H, int D,
                     const uint16_t* mask, float rate, void* stream);

/* The ViT classifier head in ONE workgroup (models/vit_small.py:123-127, flax_engine.py:13-22):
 * y = LayerNorm(x cls rows) -> yf (bf16), logits = y W + bias (fp32, [B][ldl]), metrics = [mean CE,
 * mean accuracy]; with dlogits != NULL also dlogits = (softmax - onehot) * grad_scale (fp32 + bf16),
 * dx (cls rows) = LayerNorm VJP of dlogits W^T, dscale / dbias += its parameter gradients, dhead_bias
 * (optional) += the column sums of dlogits, and dym
 * (cls rows) = bf16 dropout VJP of dx (index (b * row_stride) * D + c, the top block's MLP-out site).
 * x / dx / dym rows: stride ldx / lddx / lddym (T * D for the cls rows).  pcv_vit_head_ok(B, D, K):
 * B <= 64, D <= 128 multiple of 32, K <= 256.  work (optional, 16-B aligned, zero-filled once before
 * first use, pcv_vit_head_work_floats(B, D, K) floats): one workgroup per 16 rows with a
 * deterministic last-workgroup reduction of the cross-row sums; NULL: one workgroup.
 * defer != 0 (split form with dlogits, B > 16, K and D multiples of 8): no last-workgroup reduction;
 * each workgroup leaves its partial row at work + 4 + j * (8 + K + 2D) -- [loss/B, accuracy/B, 0 x 6 |
 * dhead_bias K | dscale D | dbias D] -- metrics[0..8) are zeroed (metrics must hold 8 floats), and a
 * later launch adds the rows into metrics / dhead_bias / dscale / dbias (the grouped weight-gradient
 * launch's fold jobs, pcv_gemm_grouped_run). */
int pcv_vit_head_ok(int B, int D, int K);
int64_t pcv_vit_head_work_floats(int B, int D, int K);
int pcv_vit_head(const float* x, int64_t ldx, const float* ln_scale, const float* ln_bias, float eps, const void* W,
                 int64_t ldw, const float* bias, const int* labels, int B, int D, int K, void* yf, int64_t ldy,
                 float* logits, int64_t ldl, float* metrics, float grad_scale, float* dlogits, void* dlogits_b,
                 int64_t ldd, float* dx, int64_t lddx, float* dscale, float* dbias, float* dhead_bias, void* dym,
                 int64_t lddym, float drop_rate, const uint32_t* seed, uint32_t site, int64_t row_stride,
                 float* work, int defer, void* stream);
/* ---------------------------------------------------------------- loss ----
 * Softmax cross-entropy + argmax accuracy per row, gradient (softmax-onehot)*grad_scale
 * (engine/flax_engine.py:13-22; train_lm.py:181-186).  pcv_mean2: deterministic means. */
int pcv_xent_fwd_bwd(const void* logits, int64_t ld, int logits_f32, const int* labels, int64_t R, int V,
                     float* row_loss, float* row_correct, void* dlogits, int64_t ldd, float grad_scale,
                     void* stream);
int pcv_mean2(const float* x, const float* y, int64_t n, float scale, float* out, void* stream);

/* ----------------------------------------------------------- optimizer ----
 * Multi-tensor AdamW over chunk tables {int64 start, int64 len} of the flat fp32
 * buffers (optax.adamw at optim/factory.py:199-205; nesterov = the adam branch of
 * optax.contrib.muon, factory.py:464-484).  step/gscale are device scalars. */
int pcv_adamw_step(float* p, const float* g, float* m, float* v, void* p_bf16, float* upd,
                   const void* chunks, int nchunks, float lr, float b1, float b2, float eps,
                   float eps_root, float wd, int nesterov, int apply, const int* step,
                   const float* gscale, void* stream);
/* Signum (optim/signum.py:14-66): m = mom*m + (1-mom)*g*gscale; d = nesterov ? (1-mom)*g + mom*m : m;
 * u = -lr*(sign(d) + wd*p) (sign(0) = 0, wd term only when wd > 0).  apply: p += u and the bf16
 * shadow; else u -> upd (the functional update() facade / a schedule-free base). */
int pcv_signum_step(float* p, const float* g, float* m, void* p_bf16, float* upd, const void* chunks, int nchunks,
                    float lr, float momentum, float wd, int nesterov, int apply, const float* gscale, void* stream);
/* Schedule-free wrapper (optim/factory.py:82-99 -> optax.contrib.schedule_free): given the base
 * optimizer's update u (base_upd) at y = params, z <- z + u, x = (1-ck)(y-(1-b1)z_old)/b1 + ck z,
 * y' = b1 x + (1-b1) z; apply: y += (y' - y) (+ bf16 shadow), else y' - y -> upd_out.
 * sf_scalars = device [weight_sum, max_lr, ck] (zeros at init), step_count device int (1 at init):
 * ck = max_lr^p / (weight_sum + max_lr^p) is formed on the device, so the step replays from a graph. */
int pcv_schedule_free_step(float* y, float* z, const float* base_upd, void* y_bf16, float* upd_out,
                           const void* chunks, int nchunks, float b1, float lr, float weight_lr_power,
                           float* sf_scalars, int* step_count, int apply, void* stream);
/* gscale = min(1, clip/(||g/accum||+1e-6))/accum  (train_lm.py:173-178, 664). */
int pcv_grad_scale(const float* g, const void* chunks, int nchunks, float* partial_ws, float inv_accum,
                   float clip, float* gscale, float* gnorm, void* stream);
int pcv_step_bump(int* step, void* stream);
/* Muon (optax.contrib.muon scale_by_muon): momentum + nesterov + Frobenius normalisation
 * into NS workspaces, and the shape-scaled weight-decayed update; descriptors are
 * pcv_muon_mat_size()-byte records (see optim_types.h MuonMat; norm2 points to MUON_NSLOT = 256
 * zeroed doubles: prep block b stores its partial sum of squares in slot b, the NS / norm kernels add
 * the slots in slot order, so the norm does not depend on block order -- by construction). */
int pcv_muon_norm_slots(void);
int pcv_muon_prep(const void* mats, int nmats, int nnorm, int64_t max_elems, float beta, int nesterov, float eps,
                  const int* step, const float* gscale, void* stream);
int pcv_muon_apply(const void* mats, int nmats, int64_t max_elems, float lr, float wd, int shape_scale,
                   int apply, void* stream);
/* muon_adaptive (factory.py:457,475 -> optax.contrib.muon adaptive=True): dual[m] += <mu_hat, O>_F per
 * record (dual: nmats zeroed doubles; mu_hat re-formed from mu, g, *step, *gscale as pcv_muon_prep did),
 * then pcv_muon_apply_dual scales each record's orthogonalised update by dual[m] before the shape scale. */
/* Muon's gradient phase in one launch: pcv_muon_prep of every record (all normalised by the NS kernel)
 * and the Adam branch's chunks (as pcv_adamw_step, applied, optax.contrib.muon's Nesterov flag) --
 * the first half of the overlapped step (engine.GraphedTrainStep overlap_opt); *step is not bumped. */
int pcv_muon_grad_phase(const void* mats, int nmats, int64_t max_elems, float beta, int nesterov, const void* chunks,
                        int nchunks, float* p, const float* g, float* mu, float* nu, void* p_bf16, float lr, float b1,
                        float b2, float eps, float eps_root, float wd, const int* step, const float* gscale,
                        void* stream);
int pcv_muon_dual_dot(const void* mats, int nmats, int64_t max_elems, float beta, int nesterov, const int* step,
                      const float* gscale, double* dual, void* stream);
int pcv_muon_apply_dual(const void* mats, int nmats, int64_t max_elems, float lr, float wd, int shape_scale,
                        int apply, const double* dual, void* stream);
int pcv_muon_mat_size(void);
/* Batched bf16 transpose (64x64 tiles, many matrices per launch): records
 * {src, dst, rows, cols, ld_src, ld_dst, first_tile} (pcv_transpose_rec_size() bytes),
 * dst[c][r] = src[r][c].  Keeps K-contiguous copies of the forward-GEMM weights. */
int pcv_transpose_bf16_batch(const void* recs, int nrec, int64_t total_tiles, void* stream);
int pcv_transpose_rec_size(void);
/* Newton-Schulz of matrices whose NS operand is at most 128 x 256, entirely in one
 * workgroup's LDS (csrc/muon_fused.hip): reads each record's x32 (un-normalised, from
 * pcv_muon_prep) and norm2, writes xo.  pcv_muon_fused_ok(rows, cols) says which shapes qualify. */
int pcv_muon_fused_ok(int64_t rows, int64_t cols);
/* The Muon step's middle launch when every routed matrix fits pcv_muon_ns_fused (ViT-small), between
 * pcv_muon_prep and pcv_muon_apply: nmats workgroups run the NS of one matrix each (x32 / norm slots
 * from pcv_muon_prep, xo for pcv_muon_apply: the streaming parts stay wide launches), nchunks more run
 * the Adam branch (chunk table as pcv_adamw_step) over the flat p, g, mu, nu; the last block to finish
 * bumps *step (ticket: a zeroed device int the call leaves zeroed).  apply = 0: updates to the flat upd
 * (functional update()).  nchunks = 0: the NS phase of the overlapped step (pcv_muon_grad_phase ran
 * the prep and the Adam branch). */
int pcv_muon_step_fused(const void* mats, int nmats, const void* chunks, int nchunks, float* p, const float* g,
                        float* mu, float* nu, void* p_bf16, float* upd, float lr, float wd, float beta, int nesterov,
                        float eps, int shape_scale, float ns_a, float ns_b, float ns_c, int ns_steps, float adam_b1,
                        float adam_b2, float adam_eps_root, float adam_wd, int apply, int* step, const float* gscale,
                        int* ticket, void* stream);
int pcv_muon_ns_fused(const void* mats, int nmats, float eps, float ns_a, float ns_b, float ns_c, int ns_steps,
                      void* stream);
int pcv_chunk_size(void);

/* ------------------------------------------------- matrix preconditioners ----
 * SOAP (optim/soap.py:136-368) and Shampoo (optim/shampoo.py:81-296): the per-leaf
 * jnp matmuls, jnp.linalg.eigh (soap.py:100-105, shampoo.py:205-206) and jnp.linalg.qr
 * (soap.py:125,131) of the reference, batched over every routed matrix (csrc/precond.hip).
 * Job records are plain 8-byte fields (pointers, int64, double), sizes from pcv_*_job_size().
 *
 * Grouped fp32 GEMM (v_mfma_f32_16x16x4_f32, exact fp32), one launch for all jobs:
 *   C = alpha * (*alpha_dev)^apow * op(A) diag(kscale) op(B) + beta * C + rscale * R; Cb = bf16(C),
 *   op(A) = a_mul * A + a_diag * I (likewise B) -- the Newton iteration's T = aI + bM unmaterialised;
 *   conv_in: the job is skipped when *conv_in <= conv_tol; conv_out: atomic max of |C - I|.
 *   record {A, B, C, kscale, R, Cb, alpha_dev, conv_in, conv_out, M, N, K, lda, ldb, ldc, ldr, ldcb,
 *           ta, tb, apow, tiles_n, first_tile, ksplit, kchunk, alpha, beta, rscale, a_diag, a_mul, b_diag, b_mul,
 *           conv_tol} (64x64 tiles, first_tile = prefix sum; apow bit 4 marks a float4-aligned job,
 *           bit 5 a symmetric result: upper-triangle tiles only, mirrored).
 * vec = 1: every job is float4-aligned (16-B bases, ld % 4, M, N, K % 4) -> vector staging.
 * vec = 2: small jobs (M, N, K <= 512, ta = 0, tb = 1, float4-aligned, no kscale / split-K) on
 *          32x32 tiles with K split over the workgroup's waves (tiles_n / first_tile in 32-tiles).
 * Split-K jobs (ksplit > 1; C += alpha op(A) op(B) only): R null -> the slices are added to C with fp32
 * atomics; R = a workspace of ksplit * ntile * 4096 floats (ntile = the job's 64x64 C tiles) -> each
 * slice stores its partial tile there and pcv_gemm_f32_split_fold adds them to C in slice order
 * (deterministic): fold records {ws, C, M, N, ldc, tiles_n, ntile, ksplit, first} (pcv_f32_fold_size()
 * bytes; first = prefix sum of ntile), one block per C tile. */
int pcv_f32_job_size(void);
int pcv_gemm_f32_grouped(const void* jobs, int njobs, int64_t total_tiles, int vec, const int64_t* firsts_host,
                         void* stream);   /* firsts_host (optional): the jobs' first_tile values, host copy */
int pcv_f32_fold_size(void);
int pcv_gemm_f32_split_fold(const void* folds_dev, int nfolds, int64_t total_tiles, void* stream);
/* Shampoo inverse p-th root (shampoo.py:195-215) by the coupled Newton iteration on the grouped
 * GEMM above: pcv_newton_init (record {L, M0, X0, conv[iters], X1, P, ldl, n, shift}; M0 = zA,
 * X0 = z^(1/p) I with A = L + shift I, z = (1+p)/(2||A||_F)), the per-iteration GEMM jobs, and
 * pcv_newton_select (P = X of the first iteration whose max|M - I| <= tol; record field status =
 * 0 converged / 1 not, read by the exact-eigh fallback jobs' skip field).  Record {L, M0, X0, conv,
 * X1, P, status, ldl, n, shift}. */
int pcv_newton_job_size(void);
/* conv[iters + 1]: conv[0] = 1 if ||A||_F / shift <= kappa_max (else the chain is skipped and status = 1). */
int pcv_newton_init(const void* jobs, int njobs, float p, int iters, float kappa_max, void* stream);
int pcv_newton_select(const void* jobs, int njobs, int iters, float tol, int64_t max_n, void* stream);
/* Symmetric eigendecomposition, n <= 256, one workgroup per matrix (cyclic Jacobi, packed upper
 * triangle in LDS, round-robin parallel rotations, rotation log for the vectors pass):
 *   record {A, w, wpow, perm, log, nrounds, skip, lda, n, shift}: eigenvalues of A + shift*I into w
 *   (descending if sort_desc, else in Jacobi order), wpow = max(w, pow_floor)^(-pow_expo) (optional),
 *   perm = source column of each output; log holds pcv_eigh_log_floats(n, max_sweeps) floats.
 * pcv_eigh_vectors replays the log: Vout = V0 (identity if NULL) x rotations, columns in w's order;
 *   record {V0, Vout, perm, log, nrounds, skip, ld0, ldo, n}; Vout may alias V0.  skip (optional
 *   device float): the job is skipped when *skip <= 0.5. */
int pcv_eigh_job_size(void);
int pcv_vec_job_size(void);
int64_t pcv_eigh_log_floats(int64_t n, int max_sweeps);
int pcv_eigh_jacobi(const void* jobs, int njobs, int max_n, int max_sweeps, float tol_rel, float tol_abs_rel,
                    int sort_desc, float pow_floor, float pow_expo, void* stream);
int pcv_eigh_vectors(const void* jobs, int njobs, int max_n, void* stream);
/* Householder QR (LAPACK geqrf/orgqr sign convention), Q of A[:, perm] (perm optional), n <= 4096:
 *   record {A, perm, Q, W, Qt, lda, ldq, n}; W and Qt are n*n fp32 workspaces. */
int pcv_qr_job_size(void);
int pcv_householder_qr(const void* jobs, int njobs, int max_n, void* stream);
int pcv_soap_sort_max_n(void);   /* largest n of pcv_householder_qr / pcv_soap_est_sort (4096) */
/* Batched symmetric eigendecomposition for 256 < n <= 4096 (LM-sized SOAP / Shampoo factors;
 * jnp.linalg.eigh at optim/soap.py:100-105, shampoo.py:205-206): one-sided (Hestenes) Jacobi on
 * the rows of A + shift I in HBM, one workgroup per rotation, a round of np/2 disjoint rotations per
 * launch (round-robin schedule), rotation flags per sweep [64] for the host's convergence test.
 * Jobs: pcv_eigh_big_job_size() bytes each {A, At, Vt, w, wpow, perm, flags, skip, vout, lda, ldv,
 * ldo, n, shift}; finish writes w (descending when sort_desc), wpow = max(w, floor)^-expo, perm and
 * the eigenvectors as the columns of vout. */
int pcv_eigh_big_job_size(void);
int pcv_eigh_big_init(const void* jobs_dev, int njobs, int max_n, int64_t max_ldv, void* stream);
int pcv_eigh_big_round(const void* jobs_dev, int njobs, int max_n, int round, int sweep, float tol, float tiny,
                       void* stream);
int pcv_eigh_big_finish(const void* jobs_dev, int njobs, int max_n, int sort_desc, float pow_floor, float pow_expo,
                        void* stream);
/* SOAP Adam in the rotated basis over flat arenas (soap.py:249-268), step = device int from 1. */
int pcv_soap_adam(const float* g_rot, float* m, float* v, float* n_rot, int64_t n, float b1, float b2, float eps,
                  const int* step, int correct_bias, void* stream);
/* SOAP refresh order (soap.py:115-126): perm = stable argsort(-diag(Q^T T)), T = M Q;
 * record {Q, T, perm, ldq, ldt, n}.  Re-index: dst[i][j] = src[pl[i]][pr[j]];
 * record {src, dst, pl, pr, rows, cols, first_block} (256-element blocks). */
int pcv_sort_job_size(void);
int pcv_soap_est_sort(const void* jobs, int njobs, void* stream);
int pcv_perm_job_size(void);
int pcv_permute_rc(const void* jobs, int njobs, int64_t total_blocks, void* stream);
const char* pcv_last_error_string(int code);

#ifdef __cplusplus
}
#endif
#endif /* PLAINCV_HIP_H */

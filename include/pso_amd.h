/*
 * pso_amd.h -- C-ABI of the MI355X-native PSO hot path (libpso_amd.so, gfx950).
 *
 * The reference (yaramohamadi/Pairwise_Sample_Optimization) is 100% Python; it has no FFI.  Every entry point below
 * replaces an IMPLICIT kernel the reference runs through PyTorch/diffusers/peft on CUDA, and is bound from Python with
 * ctypes by pairwise_sample_optimization_amd/_lib.py.  The `Replaces:` line of each function cites the reference call
 * site (file:line) whose arithmetic it performs.
 *
 * Conventions
 *   - Plain pointers and sizes only; no framework types.  Every device buffer (weights, activations, workspace) is
 *     owned by the caller; the library never allocates on the hot path.
 *   - bf16 tensors are raw uint16 bit patterns; activations are channels-last (NHWC / [tokens][channels]).
 *   - Every function returns 0 (PSO_OK) or an error code; pso_last_error() gives a thread-local message.
 *   - Work is enqueued on the caller's hipStream_t (pass the stream handle as void*); nothing synchronises, so every
 *     call is capturable into a hipGraph.
 */
#ifndef PSO_AMD_H
#define PSO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSO_ABI_VERSION 1

#define PSO_OK 0
#define PSO_ERR_ARG 1
#define PSO_ERR_HIP 2
#define PSO_ERR_UNSUPPORTED 3

/* dtype codes */
#define PSO_F32 0
#define PSO_BF16 1
#define PSO_U8 2 /* uint8 images (pso_clip_preprocess only) */

/* step modes */
#define PSO_MODE_TURBO 0 /* Euler-ancestral (SDXL-Turbo)   DP/turbo_inference_with_logprob.py:24-116 */
#define PSO_MODE_DMD 1   /* DDPM re-noise (SDXL-DMD2)      DP/distilled_inference_with_logprob.py:45-137 */
/* DMD2 "replay" modes: the reference computes x0, the mean and the log-prob in the LATENT dtype when the latents are
 * fp16 / bf16 (DP/distilled_inference_with_logprob.py:84-86 `.to(sample.dtype)`, :98-112 the table cast to the latent
 * dtype, :129-135 the log-density in that dtype).  These modes round every intermediate to that
 * dtype in the reference's operation order (values stay fp32 in memory, holding fp16 / bf16-representable numbers),
 * and the loss stage rounds Δ, exp, the clipped ratio, its log and beta*log to it (T:844-850 on latent-dtype
 * log-probs).  The coefficients of these modes are the latent-dtype values of the reference (pso_core.dmd_coef). */
#define PSO_MODE_DMD_F16 2
#define PSO_MODE_DMD_BF16 3

/* Per-sample step coefficients, PSO_COEF_STRIDE floats each (host-computed in float32 from the scheduler tables):
 *   TURBO: [sigma, sigma_up, dt = sigma_down - sigma, 2*sigma_up^2, log(sigma_up), log(sqrt(2*pi)), 0, 0]
 *   DMD:   [sqrt(abar_t), sqrt(1-abar_t), sqrt(abar_prev), sqrt(1-abar_prev), 2*(1-abar_prev),
 *           log(sqrt(1-abar_prev)), log(sqrt(2*pi)), 0]                                                        */
#define PSO_COEF_STRIDE 8

/* DreamBooth PSO loss types (DB:1924-1929) */
#define PSO_DB_SIGMOID 0 /* "pso":    -log sigmoid(beta * (ref_diff - model_diff)), reference eps required */
#define PSO_DB_HINGE 1   /* "pso_db": relu(1 - beta * (-model_diff)) (the personalization/scripts recipe)    */

const char* pso_last_error(void);
int pso_abi_version(void);

/* ------------------------------------------------------------------------------------------------------------------
 * PSO step log-prob (one scheduler step for a batch of B latents of n elements each).
 * Replaces: turbo_step_with_logprob  DP/turbo_inference_with_logprob.py:24-116  (mode TURBO)
 *           distilled_step_with_logprob DP/distilled_inference_with_logprob.py:45-137 (mode DMD)
 * sample, prev_in, noise, prev_out are fp32 [B][n]; eps is [B][n] in eps_dtype.
 * If prev_in is NULL the sampling branch runs: prev_out = mean + std * noise (noise [B][n], or [1][n] shared when
 * noise_shared != 0 -- the DMD2 batch-shared draw, DP/distilled_inference_with_logprob.py:123-126).
 * log_prob [B] fp32.  ws must hold pso_step_logprob_ws_bytes(B, n) bytes.
 * ---------------------------------------------------------------------------------------------------------------- */
size_t pso_step_logprob_ws_bytes(int B, int n);
int pso_step_logprob(int mode, int B, int n, const float* sample, const void* eps, int eps_dtype,
                     const float* prev_in, const float* noise, int noise_shared, const float* coef,
                     float* prev_out, float* log_prob, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * Fused PSO pairwise loss, forward and backward to the policy epsilon.
 * Replaces: the 4 step log-probs + clipped log-ratio loss of one micro-step, T:810-850 / D:812-854 (forward), and
 *           the autograd backward of that loss down to the UNet output (part of accelerator.backward, T:857).
 * Layout: image i = 2*p + k (pair p, member k).  x, x_prev fp32 [2P][n]; eps_pol/eps_ref [2P][n] in eps_dtype;
 * coef [2P][PSO_COEF_STRIDE]; pref [P][2] (+-1 or 0).
 * fwd outputs: lp_out [2P][2] = (lp_theta, lp_ref) per image; loss_out [1] = mean over pairs; ws keeps the fp64
 *   partial sums that bwd re-reads (keep it alive between the two calls).
 * bwd output: deps_pol [2P][n] (deps_dtype) = (*grad_out or 1) * grad_scale * dL/d eps_pol; grad_out is a DEVICE
 *   pointer to the upstream scalar gradient (may be NULL), so the call never synchronises.
 * ---------------------------------------------------------------------------------------------------------------- */
size_t pso_pair_loss_ws_bytes(int P, int n);
int pso_pair_loss_fwd(int mode, int P, int n, const float* x, const float* x_prev, const void* eps_pol,
                      const void* eps_ref, int eps_dtype, const float* coef, const float* pref, float beta,
                      float clip_eps, float* lp_out, float* loss_out, void* ws, size_t ws_bytes, void* stream);
int pso_pair_loss_bwd(int mode, int P, int n, const float* x, const float* x_prev, const void* eps_pol,
                      int eps_dtype, const float* coef, const float* pref, float beta, float clip_eps,
                      const float* grad_out, float grad_scale, void* deps_pol, int deps_dtype, const void* ws,
                      size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * The scalar stage of the pairwise loss on given log-probs (the part of pso_pair_loss_fwd/bwd after the reductions).
 * Replaces: T:844-850 / D:848-854 (clamp(exp(lp_theta - lp_ref), 1-eps, 1+eps), -log sigmoid(beta * sum log ratio *
 *           pref)).mean() and its autograd gradient w.r.t. lp_theta.  torch.clamp passes the gradient AT the bounds
 *           (mask lo <= r <= hi), which this reproduces.
 * lp_pol, lp_ref, pref, dlp_out: [P][2] fp32 (member k of pair p at [p][k]); loss_out [1].  Same device function as
 * the fused kernels, exposed so the clamp-boundary / tie cases can be driven with exact log-prob values.
 * ---------------------------------------------------------------------------------------------------------------- */
int pso_pair_loss_from_lp(int mode, int P, const float* lp_pol, const float* lp_ref, const float* pref, float beta,
                          float clip_eps, float* loss_out, float* dlp_out, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * bf16 MFMA GEMM, fp32 accumulate.
 *   out[M][N] = alpha*(A1[M][K1].B1[N][K1]^T + A2[M][K2].B2[N][K2]^T) + bias[N] + rowbias[m/rows_per_group][N]
 *               + resid[M][N]    (out bf16, f32, or f32 accumulate: out += ...)
 * Replaces: every nn.Linear of the SDXL UNet/VAE (diffusers, run by cuBLAS) and the peft LoRA adapter
 *           (peft 0.11.1 lora.Linear: base(x) + lora_B(lora_A(x)) * scaling), called from T:775-805, D:777-806,
 *           DP/sdxl_turbo_with_logprob.py:126-132, DP/sdxl_dmd_with_logprob.py:117-122.  The (A2, B2) pair is the
 *           LoRA up-projection fused as a K-tail; the same entry point computes the backward GEMMs (dX with W^T, dW).
 * All A/B operands are bf16 with K contiguous; K1, K2 multiples of 8; rows 16-B aligned.
 * tail_group_n > 0 (multiple of 64): output columns [j*tail_group_n, (j+1)*tail_group_n) take their K2-tail from A2
 * columns [j*K2, (j+1)*K2) -- three LoRA adapters (q, k, v) fused into one QKV projection with B2 = [3C][r].
 * tail_rows > 0: only rows m < tail_rows take the K2-tail (A2 then has tail_rows rows) -- the policy (LoRA on) and
 * reference (adapters disabled, T:790-805) images of one micro-step ride in one pass, policy rows first.
 * ---------------------------------------------------------------------------------------------------------------- */
int pso_gemm(int M, int N, const void* a1, long lda1, int K1, const void* b1, long ldb1, const void* a2, long lda2,
             int K2, const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
             int rows_per_group, const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate,
             int tail_group_n, int tail_rows, void* stream);
/* pso_gemm with a caller-owned fp32 workspace: dense products whose output tiles leave most CUs idle while the
 * reduction is long (M x N <= 128 tiles of 128 x 160, K >= 2048: the bs = 1 backward at M = 2048) split K over
 * workgroups; every split STORES its partial into ws and a second kernel adds them in split order and applies the
 * epilogue (deterministic, no atomics).  pso_gemm_ws_bytes(M, N, K1, K2) = the workspace that needs (0: no split);
 * any other shape or a smaller workspace runs as pso_gemm. */
size_t pso_gemm_ws_bytes(int M, int N, int K1, int K2);
int pso_gemm_ws(int M, int N, const void* a1, long lda1, int K1, const void* b1, long ldb1, const void* a2, long lda2,
                int K2, const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
                int rows_per_group, const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate,
                int tail_group_n, int tail_rows, void* ws, size_t ws_bytes, void* stream);

/* Batched dense product out_z[M][N] = alpha * A_z[M][K] . B_z[N][K]^T for z < batch, operand z at z * stride_* elements
 * (bf16 A/B, bf16 or f32 out).  Replaces the per-image loop of the VAE mid-block attention (diffusers Attention with
 * one 512-wide head over the H*W tokens, AutoencoderKL decode at DP/sdxl_turbo_with_logprob.py:154-155): scores
 * S_z = Q_z K_z^T and O_z = P_z V_z for every image of the batch in one launch each. */
int pso_gemm_batched(int batch, int M, int N, int K, const void* a, long lda, long stride_a, const void* b, long ldb,
                     long stride_b, float alpha, void* out, long ldo, long stride_o, int out_dtype, void* stream);

/* Name of the last GEMM-family kernel this thread launched, as rocprofv3 prints it (e.g.
 * "gemm_bf16_kernel<128, 160, 0, 2, 2, 2, false, 0>"): lets the bench attribute its HIP-event timings per kernel. */
const char* pso_last_kernel(void);

/* (The benchmark knobs -- forced tile shapes, A/B variants -- are not part of this library: they live in the tools
 * build libpso_amd_knobs.so, declared in include/pso_amd_knobs.h.  This library holds no mutable global state.) */

/* TN GEMM, f32 accumulate: out[I][J] += alpha * sum_m A[m][I] * B[m][J] (A [M][I], B [M][J] row-major, row strides
 * lda/ldb; I, J multiples of 8).  Replaces the peft LoRA weight-gradient GEMMs of the backward (dA = v^T x,
 * dB = s dy^T u, reduction over tokens) without materialising transposes; split-K with f32 atomics. */
int pso_gemm_tn(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                long ldo, void* stream);
/* Deterministic pso_gemm_tn with a caller-owned fp32 workspace (the training path for every TN product): wherever the
 * product splits its reduction rows (rank-16/32/64/96 side: the streaming rank kernel's row ranges; both sides >= 128:
 * 128 x 128 tiles over slices, e.g. the 640^2 / 1280^2 weights; otherwise 64 x 64 tiles over slices), every split
 * STORES its partial product into ws and a second kernel adds them into out in split order -- no f32 atomics, so two
 * runs give the same bits.  pso_gemm_tn_ws_bytes(M, I, J) = the workspace that plan needs (0: no split, out += A^T B
 * directly).  A smaller workspace falls back to pso_gemm_tn (atomic split). */
size_t pso_gemm_tn_ws_bytes(int M, int I, int J);
int pso_gemm_tn_ws(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                   long ldo, void* ws, size_t ws_bytes, void* stream);
/* Grouped (block-diagonal) form of pso_gemm_tn for the fused q/k/v LoRA adapters: with A = [M][I] the big side and
 * B = [M][J] the rank side (J = r * I / group), out[i][j] += alpha * sum_m A[m][i] B[m][(i / group) * r + j % r]
 * restricted to j in that group's r columns (out is [I][r]).  group = 0: plain pso_gemm_tn. */
int pso_gemm_tn_grouped(int M, int I, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                        long ldo, int group, void* stream);
/* The GEGLU proj weight gradient straight into the natural row order: out[F2][J] (f32, accumulated) += alpha *
 * A^T B where A [M][F2] is the interleaved pre-activation gradient (per 32 outputs [h 32 | gate 32], the layout
 * pso_gemm_geglu_bwd writes) and row i of the product lands in row (i / 64) * 32 + i % 32 (+ F2 / 2 for the gate
 * half).  128 | F2, J >= 128, 8 | J.  One pass over the reduction rows, no atomics.  Replaces the full-UNet
 * `ff.net.0.proj` weight gradient of torch autograd under `T:857` (C3 / C4 only). */
int pso_gemm_tn_geglu(int M, int F2, int J, const void* A, long lda, const void* B, long ldb, float alpha, float* out,
                      long ldo, void* stream);
/* Batched rank-r TN products (the LoRA weight gradients of one gradient unit, deferred to the unit's end and issued
 * as ONE launch per rank / orientation instead of one launch each; same arithmetic as pso_gemm_tn).  Problem i:
 *   out_jc = 0 (dB = s dY^T u):  out[c][j]  += alpha * sum_m x[m][c] * u[m][(c / group_c) * R + j]   (out [C][R])
 *   out_jc = 1 (dA = v^T x):     out[j][c]  += alpha * sum_m x[m][c] * u[m][j]                       (out [R][C])
 * with x [M][C] (C % 128 == 0) the activation / output-gradient stream and u [M][*] the rank-R projection
 * (R = 16, 32, 64 or 96), group_c = 0 or a multiple of 128 dividing C (the fused q/k/v adapters).  f32 atomics into
 * out; probs is HOST memory, copied into the launch arguments (capturable in a hipGraph). */
typedef struct {
  const void* x; long ldx;
  const void* u; long ldu;
  float* out; long ldo;
  int M, C, group_c;
  float alpha;
} PsoTnRankProblem;
int pso_gemm_tn_rank_batch(int R, int out_jc, int count, const PsoTnRankProblem* probs, void* stream);
/* Deterministic form of pso_gemm_tn_rank_batch (the training path, TnRankQueue): no f32 atomics -- every workgroup
 * STORES its 128 x R partial into the caller-owned device workspace ws and a second kernel adds the partials of each
 * output block in row-range order, then out += alpha * sum.  Two runs, and a hipGraph replay, give the same bits (the
 * reference's LoRA dW are cuBLAS GEMMs under autograd, T:857: a fixed reduction order).  Products whose outputs
 * overlap go to separate launches.  pso_gemm_tn_rank_batch_ws_bytes = the workspace the call needs (0 on bad args). */
size_t pso_gemm_tn_rank_batch_ws_bytes(int R, int out_jc, int count, const PsoTnRankProblem* probs);
int pso_gemm_tn_rank_batch_ws(int R, int out_jc, int count, const PsoTnRankProblem* probs, void* ws, size_t ws_bytes,
                              void* stream);
/* Grouped (block-diagonal) skinny product for the fused q/k/v LoRA adapters of the backward (v = dy sB per adapter):
 * out[m][g*N + n] = alpha * sum_k A[m][g*K + k] * W[n][g*K + k] for g < groups (bf16 out, N <= 128, N % 4 == 0). */
int pso_gemm_skinny_grouped(int M, int N, int K, const void* A, long lda, const void* W, long ldw, float alpha,
                            void* out, long ldo, int groups, void* stream);

/* GEGLU feed-forward projection with the activation fused into the GEMM epilogue (diffusers GEGLU, `net.0`):
 * w is the proj weight [N][K] with its rows INTERLEAVED per 64 as [h rows 32 | gate rows 32] (bias likewise), N =
 * 2F, N % 256 == 0.  out [M][F] = h * gelu(gate) (exact erf GELU, h / gate rounded to bf16 first, as the unfused
 * path does); out_pre (optional) receives the interleaved pre-activation the backward needs, rows < pre_rows only
 * (pre_rows = 0: all M rows). */
int pso_gemm_geglu(int M, int N, const void* a, long lda, int K, const void* w, long ldw, const void* bias, void* out,
                   long ldo, void* out_pre, long ld_pre, int pre_rows, void* stream);
/* Backward of the GEGLU fused into the GEMM producing its output gradient: dout = a . w^T ([M][N], N = F, rounded to
 * bf16), pre = the interleaved pre-activation [M][2F]; out [M][2F] = interleaved [dout*gelu(g) | dout*h*gelu'(g)]. */
int pso_gemm_geglu_bwd(int M, int N, const void* a, long lda, int K, const void* w, long ldw, const void* pre,
                       long ld_pre, void* out, long ldo, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * FP8 forward GEMMs (BASELINE config 5: "fp8 MFMA UNet fwd + bf16 bwd").  The reference runs this forward in its
 * mixed-precision dtype (DB:1815-1825 under accelerate autocast); here the projections fed by a LayerNorm (attention
 * q/k/v, cross-attention q, the GEGLU ff.net.0.proj) can run on OCP e4m3 operands with one power-of-two scale per
 * row, stored as an E8M0 byte (127 + exponent; value = e4m3 * 2^exponent).
 *
 * pso_quant_rows_fp8: q[m][k] = e4m3(x[m][k] * 2^-e[m]) (round to nearest even, |.| <= 448), e[m] = the smallest
 *   exponent with rowmax|x| * 2^-e <= 448 (0 for an all-zero row); x bf16 [M][K] (row stride ldx), q [M][K] bytes
 *   (ldq), e8m0[m] = 127 + e[m].  Used for activations (per token) and weights (per output channel) alike.
 * pso_gemm_fp8: acc[m][n] = sum_k (a[m][k] 2^ea[m]) (w[n][k] 2^ew[n]) (+ the LoRA K-tail a2 . w2^T on rows < tail_m,
 *   a2 / w2 fp8 with their own row / column scales, tail_group_n as pso_gemm), fp32 accumulate; epi 0:
 *   out = bf16(alpha*acc + bias) (+ resid); epi 1: the GEGLU epilogue of pso_gemm_geglu (interleaved weight rows,
 *   out [M][N/2], out_pre rows < pre_rows).  N % 256 == 0, K % 128 == 0, K2 % 16 == 0, 16-B aligned rows.
 * ---------------------------------------------------------------------------------------------------------------- */
int pso_quant_rows_fp8(int M, int K, const void* x, long ldx, void* q, long ldq, void* e8m0, void* stream);
int pso_gemm_fp8(int epi, int M, int N, int K, const void* a, long lda, const void* sa, const void* w, long ldw,
                 const void* sw, const void* a2, long lda2, int K2, const void* sa2, const void* w2, long ldw2,
                 const void* sw2, int tail_m, int tail_group_n, float alpha, const void* bias, const void* resid,
                 long ldr, void* out, long ldo, void* out_pre, long ld_pre, int pre_rows, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * DreamBooth PSO loss (config 5), forward and backward to the UNet eps.
 * Replaces: DB = personalization/train_pso_sdxl_turbo_dreambooth.py:1847-1935 -- EDM-style x0 = eps*(-sigma) + noisy,
 *           per-image sigma^-2-weighted MSE vs the clean latent, instance/negative split, pso / pso_db loss, prior
 *           loss -- and the autograd backward of it down to the UNet output (DB:1953).
 * Layout: 2B images, instance b at row b, its negative at row B + b.  eps [2B][n] (eps_dtype), eps_ref the same
 * (adapters disabled, loss_type PSO_DB_SIGMOID only), noisy / x0 fp32 [2B][n], sigma fp32 [2B].
 * fwd outputs: losses_out [2B] (+ [2B] reference) per-image MSE, logits_out [B], loss_out [1]; ws (keep it for the
 * bwd) holds the fp64 partials.  bwd: deps [2B][n] = (*grad_out or 1) * grad_scale * dL/d eps.
 * ---------------------------------------------------------------------------------------------------------------- */
size_t pso_db_loss_ws_bytes(int B, int n);
int pso_db_loss_fwd(int loss_type, int B, int n, const void* eps, const void* eps_ref, int eps_dtype,
                    const float* noisy, const float* x0, const float* sigma, float beta, float neg_defactor,
                    float prior_w, float* losses_out, float* logits_out, float* loss_out, void* ws, size_t ws_bytes,
                    void* stream);
int pso_db_loss_bwd(int loss_type, int B, int n, const void* eps, int eps_dtype, const float* noisy, const float* x0,
                    const float* sigma, float beta, float neg_defactor, float prior_w, const float* grad_out,
                    float grad_scale, void* deps, int deps_dtype, const void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * Implicit-GEMM 2-D convolution on NHWC bf16 images (fp32 accumulate).  weight is [Cout][ks][ks][C1+C2] (bf16).
 * Input = channel concat of src1 [B][H][W][C1] and src2 [B][H][W][C2] (C2 may be 0); output [B][Ho][Wo][Cout] (ldo).
 * Gather modes: PSO_CONV_NORMAL (stride/pad), PSO_CONV_UP2 (nearest 2x upsample fused, Ho=2H), PSO_CONV_T2
 * (transposed stride-2: input-gradient of a stride-2 conv; weight = W^T per tap, unflipped).
 * Epilogue as pso_gemm; rowbias is per image ([B][Cout], the ResnetBlock2D time-embedding add).
 * Replaces: cuDNN conv2d of every diffusers ResnetBlock2D / Downsample2D / Upsample2D / conv_in / conv_out (UNet and
 *           VAE decoder), plus the torch.cat of skip connections in the up blocks.
 * ---------------------------------------------------------------------------------------------------------------- */
#define PSO_CONV_NORMAL 1
#define PSO_CONV_UP2 2
#define PSO_CONV_T2 3
int pso_conv2d(int mode, int B, const void* src1, int C1, const void* src2, int C2, int H, int W, int Ho, int Wo,
               int ks, int stride, int pad, const void* weight, int Cout, const void* a2, long lda2, int K2,
               const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
               const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate, void* stream);
/* Deterministic split-K form of pso_conv2d for small outputs with a long reduction (the bs = 1 / GPU backward's
 * input-gradient convolutions at 2 images: 2048 x 1280 x 11520): same arguments plus a caller-owned fp32 workspace of
 * pso_conv2d_ws_bytes(B, Ho, Wo, Cout, ks*ks*(C1+C2), K2) bytes (0: no split applies, pso_conv2d is used); every
 * K-split stores its partial product and they are added in split order with the epilogue (bias, row bias,
 * residual) applied once.  No atomics. */
size_t pso_conv2d_ws_bytes(int B, int Ho, int Wo, int Cout, int K1, int K2);
int pso_conv2d_ws(int mode, int B, const void* src1, int C1, const void* src2, int C2, int H, int W, int Ho, int Wo,
                  int ks, int stride, int pad, const void* weight, int Cout, const void* a2, long lda2, int K2,
                  const void* b2, long ldb2, float alpha, const void* bias, const void* rowbias, long ld_rowbias,
                  const void* resid, long ldr, void* out, long ldo, int out_dtype, int accumulate, void* ws,
                  size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * GroupNorm (+ fused SiLU) on NHWC bf16, fp32 statistics.  stats [B][G][2] = (mean, rstd).
 * Replaces: torch.nn.GroupNorm(32) + SiLU of diffusers ResnetBlock2D (norm1/norm2), Transformer2DModel.norm,
 *           conv_norm_out (UNet, VAE decoder); its autograd backward (dx, optional dgamma/dbeta).
 * ws: pso_group_norm_ws_bytes(B,HW,C) bytes (fwd and bwd).  dadd (optional) is added to dx.
 * ---------------------------------------------------------------------------------------------------------------- */
size_t pso_group_norm_ws_bytes(int B, int HW, int C);
int pso_group_norm_fwd(int B, int HW, int C, int G, float eps, const void* x, const void* gamma, const void* beta,
                       int silu, void* y, float* stats, void* ws, size_t ws_bytes, void* stream);
int pso_group_norm_bwd(int B, int HW, int C, int G, const void* x, const void* dy, const float* stats,
                       const void* gamma, const void* beta, int silu, const void* dadd, void* dx, float* dgamma,
                       float* dbeta, int accumulate_dparams, void* ws, size_t ws_bytes, void* stream);

/* LayerNorm over the last dim (C <= 2048), bf16 I/O, stats [M][2] fp32.
 * Replaces: torch.nn.LayerNorm norm1/norm2/norm3 of diffusers BasicTransformerBlock (and its backward). */
int pso_layer_norm_fwd(int M, int C, float eps, const void* x, long ldx, const void* gamma, const void* beta, void* y,
                       long ldy, float* stats, void* stream);
int pso_layer_norm_bwd(int M, int C, const void* x, long ldx, const void* dy, long lddy, const float* stats,
                       const void* gamma, const void* dadd, long ldadd, void* dx, long lddx, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * Flash attention, head dim 64, bf16 in/out (fp32 softmax).  Q [B][Sq][H*64] (row stride ldq, batch stride sq_b),
 * K/V [B][Sk][H*64], O like Q; lse [B][H][Sq] (natural log of the scaled-score normaliser) for the backward.
 * Replaces: F.scaled_dot_product_attention in diffusers AttnProcessor2_0 (attn1 self / attn2 cross attention of the
 *           140 SDXL BasicTransformerBlocks) and its autograd backward.
 * bwd: ws of pso_attention_bwd_ws_bytes(); for Sk <= 256 (cross-attention) dk/dv must be dense [B*Sk][.] with row
 *      stride lddk/lddv and batch stride Sk*ld.  Sk <= 96 (the 77 text tokens) runs ONE pass over the query tiles
 *      for dQ, dK and dV (attn_bwd_x_kernel, query splits reduced in order: deterministic); longer key sequences run
 *      the dQ and the dK/dV kernels.
 * ---------------------------------------------------------------------------------------------------------------- */
int pso_attention_fwd(int B, int H, int Sq, int Sk, const void* q, long ldq, long sq_b, const void* k, long ldk,
                      long sk_b, const void* v, long ldv, long sv_b, float scale, void* o, long ldo, long so_b,
                      float* lse, void* stream);
size_t pso_attention_bwd_ws_bytes(int B, int H, int Sq, int Sk);
int pso_attention_bwd(int B, int H, int Sq, int Sk, const void* q, long ldq, long sq_b, const void* k, long ldk,
                      long sk_b, const void* v, long ldv, long sv_b, const void* o, long ldo, long so_b,
                      const float* lse, const void* dO, long lddo, long sdo_b, float scale, void* dq, long lddq,
                      long sdq_b, void* dk, long lddk, long sdk_b, void* dv, long lddv, long sdv_b, void* ws,
                      size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * Element-wise / data movement (bf16 unless noted).
 *   geglu: in [M][ldi] = [h | gate] (F each) -> out = h * gelu_erf(gate)     (diffusers GEGLU, FeedForward.net[0])
 *   silu: y = x * sigmoid(x)                                                 (time-embedding nonlinearity)
 *   timestep_embedding: t fp32 [n] -> out[:, out_col:out_col+dim] = [cos | sin](t * 10000^(-i/(dim/2)))
 *                                                       (diffusers Timesteps, flip_sin_to_cos=True, shift=0)
 *   transpose [R][C] -> [C][Rp] (rows >= R read as 0: zero-padded GEMM reduction dims); im2col3 (3x3 pad 1, small C, zero padded to Kp columns); sumpool2 (2x2 sum, the
 *   input-gradient of nearest-2x upsample); axpby y = a*x + b*z; casts; conv_weight_t ([Co][k][k][Ci] ->
 *   [Ci][k][k][Co], flip=1 rotates the taps: the input-gradient weight of a stride-1 conv).
 * ---------------------------------------------------------------------------------------------------------------- */
int pso_geglu_fwd(long M, int F, const void* in, long ldi, void* out, long ldo, void* stream);
int pso_geglu_bwd(long M, int F, const void* in, long ldi, const void* dout, long lddo, void* din, long lddi,
                  void* stream);
int pso_silu(long n, const void* x, void* y, void* stream);
int pso_timestep_embedding(int n, int dim, const float* t, void* out, long ldo, int out_col, void* stream);
int pso_transpose(int R, int Rp, int C, const void* in, long ldi, void* out, long ldo, void* stream);
int pso_im2col3(int B, int H, int W, int C, const void* in, void* out, int Kp, void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * Full-UNet weight gradients (BASELINE C3 / C4, SURVEY §8a a6 "full dW in C3 (build-only)"; the reference trains LoRA
 * only, App. A #4).  The dW products run on pso_gemm_tn; these supply the rest:
 * pso_colsum_acc: out[g][n] += sum over rows m in [g*rows_per_group, (g+1)*rows_per_group) of x[m][n] (bf16 in, f32
 *   out; bias gradients with rows_per_group = M, per-image time-embedding row-bias gradients with rows_per_group = HW).
 * pso_layer_norm_dparam: dgamma[c] += sum_m dy[m][c] (x[m][c] - mean_m) rstd_m; dbeta[c] += sum_m dy[m][c] (stats
 *   from pso_layer_norm_fwd).  torch LayerNorm weight / bias grads.
 * pso_im2col_conv: 3x3 patch matrix [B*Ho*Wo][9*(C1+C2)] in the NHWC weight order (tap-major, channel-minor) for mode
 *   PSO_CONV_NORMAL (stride 1 / 2) or PSO_CONV_UP2 (nearest 2x upsample), sources concatenated on channels; zero
 *   padding.  dW[Cout][3][3][Cin] = dY^T . cols (torch conv2d weight grad).
 * ------------------------------------------------------------------------------------------------------------------ */
int pso_colsum_acc(long M, int N, const void* x, long ldx, long rows_per_group, float* out, long ldo, void* stream);
int pso_layer_norm_dparam(int M, int C, const void* x, long ldx, const void* dy, long lddy, const float* stats,
                          float* dgamma, float* dbeta, void* stream);
/* Ordered forms of the two sums above (no float atomics: per-row-block partials in a caller-owned workspace, added in
 * row-block order -- bit-reproducible full-UNet gradients).  The workspace sizes are *_ws_bytes. */
size_t pso_colsum_acc_ws_bytes(long M, int N, long rows_per_group);
int pso_colsum_acc_ws(long M, int N, const void* x, long ldx, long rows_per_group, float* out, long ldo, void* ws,
                      size_t ws_bytes, void* stream);
size_t pso_layer_norm_dparam_ws_bytes(int M, int C);
int pso_layer_norm_dparam_ws(int M, int C, const void* x, long ldx, const void* dy, long lddy, const float* stats,
                             float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);
int pso_im2col_conv(int mode, int B, const void* src1, int C1, const void* src2, int C2, int H, int W, int Ho, int Wo,
                    int stride, int pad, void* out, long ldo, void* stream);
int pso_sumpool2(int B, int H, int W, int C, const void* in, const void* dadd, void* out, void* stream);
int pso_axpby(long n, float a, const void* x, float b, const void* z, void* y, void* stream);
int pso_cast_f32_bf16(long n, const float* x, float scale, void* y, void* stream);
int pso_cast_bf16_f32(long n, const void* x, float* y, void* stream);
int pso_conv_weight_t(int Co, int ks, int Ci, int flip, const void* w, void* wt, void* stream);
/* channel concat of NHWC rows (torch.cat([h, skip], dim=1) of the up blocks) and its inverse; the split can add a
 * second gradient into the skip part (the skip tensor also feeds the next down layer). */
/* batched transpose: descs = device array of n {const bf16* src; bf16* dst; int R, C; long ldi, ldo;} (src [R][C]
 * -> dst [C][R]); one launch for all LoRA working-copy transposes after an optimizer step. */
int pso_transpose_batched(int n, const void* descs, int max_r, int max_c, void* stream);
/* many transposes in one launch over a flat grid of 64 x 64 tiles: descs = device array of n 48-B records
 * {const bf16* src; bf16* dst; long ldi, ldo; int R, C, tiles_c, tile0;} (src [R][C] -> dst [C][R], tiles_c =
 * ceil(C / 64), tile0 = the record's first tile, ascending from 0), total_tiles = sum of ceil(R/64) * tiles_c. */
int pso_transpose_multi(int n, const void* descs, int total_tiles, void* stream);
/* dst row i = src row idx[i] (row_bytes % 4 == 0): the pair/time shuffles of the trajectory buffer (T:733-745) */
int pso_gather_rows(long n, long row_bytes, const void* src, const int64_t* idx, void* dst, void* stream);
/* layout conversion of the (small) latent tensors at the diffusers NCHW API boundary */
int pso_nchw_to_nhwc(int B, int C, int Cp, long HW, const void* src, int src_dtype, float scale, void* dst,
                     void* stream);  /* channels zero-padded to Cp, values scaled */
/* in-place row softmax of a bf16 [M][N] score matrix (fp32 math): the single-head 16384-token attention of the SDXL
 * VAE decoder mid-block (diffusers Attention, head dim 512) runs as GEMM -> softmax -> GEMM */
int pso_softmax_rows(int M, int N, void* x, long ld, void* stream);
int pso_nhwc_to_nchw(int B, int C, long HW, const void* src, void* dst, int dst_dtype, void* stream);
int pso_concat_channels(long npix, int C1, const void* x1, int C2, const void* x2, void* out, void* stream);
int pso_split_channels(long npix, int C1, int C2, const void* in, void* y1, void* y2, const void* add2,
                       void* stream);

/* ------------------------------------------------------------------------------------------------------------------
 * Optimizer / clipping / preference (fp32, on device, no host synchronisation).
 * pso_grad_clip_coef: out[0] = ||grad||_2 * grad_scale, out[1] = min(1, max_norm / (norm + 1e-6))
 *   Replaces: accelerator.clip_grad_norm_(params_to_optimize, max_grad_norm)   T:858-859
 * pso_adamw_step: torch.optim.AdamW semantics on (param, grad * grad_scale * clip_coef[1]); step counts from 1.
 *   Replaces: optimizer.step() T:860 (AdamW; bitsandbytes AdamW8bit has no ROCm build here)
 * pso_preference: rewards [P][2][m] -> pref [P][2]; mode 0 = sample_compare (T:401-416, reward column reward_idx[p]
 *   or 0, ties -> member 0 loses), mode 1 = compare (D:420-434, strict Pareto, ties -> (0,0)).
 * ---------------------------------------------------------------------------------------------------------------- */
size_t pso_grad_clip_ws_bytes(long n);
int pso_grad_clip_coef(long n, const float* grad, float grad_scale, float max_norm, float* out_norm_coef, void* ws,
                       size_t ws_bytes, void* stream);
int pso_adamw_step(long n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float lr, float beta1,
                   float beta2, float eps, float weight_decay, int step, float grad_scale, const float* clip_coef,
                   void* stream);
/* Blockwise 8-bit AdamW (bitsandbytes AdamW8bit, the reference's default optimizer: config_sdxl_turbo_dpo.py:86
 * `use_8bit_adam = True`, T:427-435).  exp_avg_q / exp_avg_sq_q are uint8 codes [n] into the signed / unsigned dynamic
 * quantisation maps (pso_adamw8bit_maps), absmax_m / absmax_v one fp32 scale per 2048-element block
 * (pso_adamw8bit_blocks(n) of each); all zero-initialised.  Per element: dequantise with the block's previous absmax,
 * m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2, p += -lr c2/c1 * m / (sqrt(v) + c2 eps), p *= 1 - lr wd (c1 = 1-b1^t,
 * c2 = sqrt(1-b2^t)), then requantise to the nearest code against the block's new absmax.  g = grad * grad_scale *
 * clip_coef[1] (clip_coef may be NULL).  Parity unpinned (bitsandbytes is not in this image; oracle/adam8bit.py). */
size_t pso_adamw8bit_blocks(long n);
void pso_adamw8bit_maps(float* signed_map, float* unsigned_map);
int pso_adamw8bit_step(long n, float* param, const float* grad, uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q,
                       float* absmax_m, float* absmax_v, float lr, float beta1, float beta2, float eps,
                       float weight_decay, int step, float grad_scale, const float* clip_coef, void* stream);
/* The same step that also writes the updated parameters rounded to bf16 (RNE) into param_bf16 [n] (16-B aligned; NULL
 * = pso_adamw8bit_step): the bf16 working copy the UNet kernels read, without a separate cast pass. */
int pso_adamw8bit_step_bf16(long n, float* param, void* param_bf16, const float* grad, uint8_t* exp_avg_q,
                            uint8_t* exp_avg_sq_q, float* absmax_m, float* absmax_v, float lr, float beta1, float beta2,
                            float eps, float weight_decay, int step, float grad_scale, const float* clip_coef,
                            void* stream);
/* Per-tensor form (what bitsandbytes does with a list of parameter tensors, T:428-448): nblk blocks described by the
 * device table desc [nblk][4] (int64: start element, length <= 2048, 32-bit state offset or -1, unused).  The blocks
 * restart at every tensor, so one absmax never spans two tensors; a tensor under bitsandbytes' min_8bit_size (4096
 * elements) keeps 32-bit state (no quantisation: m / v fp32 at exp_avg_32 / exp_avg_sq_32 + offset, same update),
 * absmax_m / absmax_v hold one entry per table block.  Elements no block covers (alignment pads) are not touched.
 * Non-finite gradient elements leave the parameter and its state unchanged.  param_bf16 may be NULL. */
int pso_adamw8bit_step_blocks(long n, int nblk, const long* desc, float* param, void* param_bf16, const float* grad,
                              uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q, float* absmax_m, float* absmax_v,
                              float* exp_avg_32, float* exp_avg_sq_32, float lr, float beta1, float beta2, float eps,
                              float weight_decay, int step, float grad_scale, const float* clip_coef, void* stream);
/* = pso_adamw8bit_step_blocks, and every gradient element a block covers is zeroed once it has been read
 * (optimizer.zero_grad, T:861, folded into the step: no separate pass over the gradient).  Pads are not touched. */
int pso_adamw8bit_step_blocks_zero_grad(long n, int nblk, const long* desc, float* param, void* param_bf16,
                                        float* grad, uint8_t* exp_avg_q, uint8_t* exp_avg_sq_q, float* absmax_m,
                                        float* absmax_v, float* exp_avg_32, float* exp_avg_sq_32, float lr,
                                        float beta1, float beta2, float eps, float weight_decay, int step,
                                        float grad_scale, const float* clip_coef, void* stream);
int pso_zero_f32(long n, float* x, void* stream);
int pso_preference(int P, int m, const float* rewards, const int64_t* reward_idx, int mode, float* pref,
                   void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * CLIP towers and the reward image path (clip.hip): the SDXL prompt encoders (CLIP ViT-L/14 text
 * + OpenCLIP ViT-bigG/14 text, `encode_prompt` T:81-118) and the PickScore reward (CLIP ViT-H/14,
 * pso_pytorch/pickscore_utils.py:12-62) run their projections on pso_gemm and their norms on pso_layer_norm_fwd;
 * these are the remaining pieces.
 * ------------------------------------------------------------------------------------------------------------- */
#define PSO_ACT_GELU 0       /* exact (erf) GELU: OpenCLIP bigG / ViT-H towers                                    */
#define PSO_ACT_QUICK_GELU 1 /* x * sigmoid(1.702 x): OpenAI CLIP ViT-L/14 text encoder                          */

/* Softmax attention over short sequences (S <= a few hundred; head dim D <= 128), fp32 online softmax.  Token rows
 * of q / k / v / o are strided (ld*) inside a batch (stride s*_b); head h occupies columns [h*D, (h+1)*D).  causal:
 * key j > query i masked (the CLIP text encoders' causal mask). */
int pso_attention_small(int B, int H, int S, int D, const void* q, long ldq, long sq_b, const void* k, long ldk,
                        long sk_b, const void* v, long ldv, long sv_b, int causal, float scale, void* o, long ldo,
                        long so_b, void* stream);
/* In-place activation of n bf16 values (mode PSO_ACT_*). */
int pso_activation(long n, void* x, int mode, void* stream);
/* out[b*S + t][:] = tok[ids[b*S + t]][:] + pos[t][:] (bf16 tables, int64 ids). */
int pso_embed_tokens(int B, int S, int C, const int64_t* ids, const void* tok, const void* pos, void* out,
                     void* stream);
/* Vision embeddings: row 0 of image b = cls + pos[0], row 1 + p = patch[b*P + p] + pos[1 + p]  -> [B*(P+1)][C]. */
int pso_embed_vision(int B, int P, int C, const void* patch, const void* cls, const void* pos, void* out,
                     void* stream);
/* out[i] = cos(a_i, b_i) for fp32 rows (PickScore: diag(text_n @ image_n^T), pickscore_utils.py:50-58). */
int pso_cosine_rows(int n, int C, const float* a, long lda, const float* b, long ldb, float* out, void* stream);
/* out[r] = mean of row r (n bf16 values, 16-B aligned rows, n % 8 == 0): light_reward (pso_pytorch/rewards.py:5-9). */
int pso_row_mean(int rows, long n, const void* x, float* out, void* stream);
/* Reward-image preprocessing, GPU-resident replacement of T:632-640 + the CLIPImageProcessor: image NHWC bf16
 * [B,H,W,3] in [-1,1] -> uint8 as ((x + 1) * 127.5).clamp(0, 255).to(uint8) in bf16 arithmetic -> PIL bicubic resize
 * of the shortest edge to `size` (8-bit fixed point, horizontal then vertical pass, bit-exact) -> centre crop
 * size x size -> x / 255 -> (x - mean) / std (float32) -> patch rows [B * (size/patch)^2][kpad] bf16 in
 * (channel, ky, kx) order (zero columns past 3 * patch^2): the A operand of the patch-embedding GEMM. */
/* Patch rows of an already processed NCHW fp32 image [B, C, S, S] (same layout as pso_clip_preprocess's output). */
int pso_patchify(int B, int C, int S, int P, int kpad, const float* x, void* out, void* stream);
size_t pso_clip_preprocess_ws_bytes(int B, int H, int W, int size);
int pso_clip_preprocess(int B, int H, int W, const void* img, int img_dtype, int size, int patch, int kpad,
                        const float* mean, const float* stdv, void* out, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PSO_AMD_H */

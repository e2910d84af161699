// Host-side launch entry points of the gfx950 kernels (implemented in *.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "attention.h"

namespace dlion {

// ---- optimizer (lion_kernels.hip)
hipError_t launch_lion_local(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks, float decay,
                             float neg_lr, float b1, float omb1, float b2, float omb2, const float* gscale,
                             hipStream_t st);
hipError_t launch_lion_encode(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks, uint8_t* bits,
                              float b1, float omb1, float b2, float omb2, int update_m, int stochastic, float rr,
                              uint64_t seed, uint32_t step, const float* gscale, hipStream_t st);
// fused clip_grad_norm_: per-chunk sum of squares, then norm + clip coefficient on device
hipError_t launch_grad_sumsq(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks, float* partial,
                             hipStream_t st);
hipError_t launch_clip_coef(const float* partial, int64_t n, float max_norm, float* out, hipStream_t st);
hipError_t launch_lion_vote_apply(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks,
                                  const uint8_t* planes, int64_t plane_stride, const uint8_t* alive, int world,
                                  int mode, int tie, const uint8_t* neg, float decay, float neg_lr, const uint8_t* own,
                                  unsigned long long* agree, hipStream_t st);
hipError_t launch_vote_reduce(const uint8_t* recv, int64_t nbytes, const uint8_t* alive, int world, int tie,
                              uint8_t* out, uint8_t* neg_out, unsigned long long* ties, hipStream_t st);

// ---- flash attention (attention.hip)
hipError_t launch_attn_fwd(const AttnArgs& a, int D, bool drop, hipStream_t st);
hipError_t launch_attn_bwd(const AttnArgs& a, int D, bool drop, hipStream_t st);

// ---- fused residual + dropout + LayerNorm/RMSNorm (norm_kernels.hip)
// backward: `parts` blocks (4 rows of C <= 1024, or one wide row, per block
// iteration); part is [parts][3][C]
hipError_t launch_add_norm_fwd(const void* x, const void* y, const void* bias, const void* gamma, const void* beta,
                               void* xo, void* h, float* mean, float* rstd, int64_t rows, int C, float eps, bool rms,
                               uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st);
hipError_t launch_add_norm_bwd(const void* dh, const void* dxo_in, const void* xo, const void* gamma, const float* mean,
                               const float* rstd, void* dx, void* dy, float* part, int parts, int64_t rows, int C,
                               bool rms, uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st);

// ---- bias + GELU, SwiGLU, RoPE, partial sums (elementwise_kernels.hip)
hipError_t launch_bias_gelu_fwd(const void* z, const void* b, void* h, int64_t rows, int N, bool exact,
                                hipStream_t st);
hipError_t launch_bias_gelu_bwd(const void* dh, const void* z, const void* b, void* dz, float* dbpart, int parts,
                                int64_t rows, int N, bool exact, hipStream_t st);
hipError_t launch_swiglu_fwd(const void* g, const void* u, void* h, int64_t rows, int64_t F, int64_t ld_in,
                             hipStream_t st);
hipError_t launch_swiglu_fwd_t(const void* g, const void* u, void* h, void* ht, int64_t rows, int64_t F,
                               int64_t ld_in, hipStream_t st);
hipError_t launch_swiglu_bwd_t(const void* dh, const void* g, const void* u, void* dgu, void* dgut, int64_t rows,
                               int64_t F, int64_t ld_in, hipStream_t st);
hipError_t launch_swiglu_bwd(const void* dh, const void* g, const void* u, void* dg, void* du, int64_t rows,
                             int64_t F, int64_t ld_in, int64_t ld_out, hipStream_t st);
hipError_t launch_rope(const void* x, const void* cos, const void* sin, void* y, int64_t rows, int T, int H, int D,
                       bool inverse, int64_t x_ld, int64_t y_ld, hipStream_t st);
// out (+)= bf16(scale[0] * sum_s part[s]) (scale: optional device scalar)
hipError_t launch_sum_partials(const float* part, int S, int64_t n, int64_t ld, void* out, bool accumulate,
                               hipStream_t st, const float* scale = nullptr);
hipError_t launch_colsum(const void* x, float* part, int parts, int64_t rows, int N, hipStream_t st);
// out (+)= bf16(sum over every row of up to 16 fp32 stacks [rows_k, >= n] (row stride lds_k))
hipError_t launch_sum_partials_multi(const float* const* ptrs, const int64_t* rows, const int64_t* lds, int nseg,
                                     int64_t n, void* out, bool accumulate, hipStream_t st);
// the same over Y row groups: pass 1 into scratch fp32 [Y, n], pass 2 out (+)= bf16(scale * sum) --
// for narrow tall stacks (few column blocks); Y from sum_partials_split_factor (1 = not worth it)
int sum_partials_split_factor(int64_t n, int64_t total_rows);
// out [C, Rp] (16-bit elements) = x [R, C]^T (row stride ldx), output columns R..Rp-1 zero; Rp % 8 == 0
hipError_t launch_transpose_pad(const void* x, int64_t R, int64_t C, int64_t ldx, void* out, int64_t Rp,
                                hipStream_t st);
hipError_t launch_sum_partials_split(const float* const* ptrs, const int64_t* rows, const int64_t* lds, int nseg,
                                     int64_t n, int Y, float* scratch, void* out, bool accumulate, const float* scale,
                                     hipStream_t st);

// ---- bf16 GEMM C[M,N] = A[M,K] . B[N,K]^T with fused epilogue (gemm.hip)
// epi: 0 plain, 1 + bias, 2 aux = z, C = gelu_tanh(z + bias), 3 the same with erf GELU,
// 4 C = bf16(A.B^T) * gelu_tanh'(aux + bias) with aux an input and part [2 * ceil(M/256)][N]
// fp32 column sums of C (bias gradient partials), 5 the same with erf GELU; 6 / 7 as 2 / 3 but
// aux = bf16(gelu'(z + bias)) (output); 8 C = bf16(A.B^T) * aux with aux that derivative (input)
// and the part column sums of 4 (no bias).
// Needs K % 128 == 0, N % 8 == 0, leading dims % 8 == 0.
hipError_t launch_gemm_nt(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                          void* aux, int ldaux, int M, int N, int K, int epi, float* part, hipStream_t st);

// ---- token + position embedding with dropout, scaled gradient accumulation (embedding.hip)
hipError_t launch_embed_fwd(const int64_t* ids, const void* wte, const void* wpe, void* out, int64_t n, int C, int T,
                            int64_t V, uint32_t seed, uint32_t thresh16, float inv_keep, int32_t* err, hipStream_t st);
// error-flag bits (index_check / embed_fwd): OR-ed into err[0]
constexpr int kIndexErrEmbed = 1, kIndexErrLabel = 2;
hipError_t launch_index_check(const int64_t* ids, int64_t n, int64_t hi, int64_t ignore, int32_t* err, int code,
                              hipStream_t st);
// dwte / dwpe nullable; sid / perm = stably sorted ids and their positions (needed with dwte)
hipError_t launch_embed_bwd(const void* dx, const int64_t* sid, const int64_t* perm, void* dwte, void* dwpe, int64_t n,
                            int C, int T, int64_t V, int pos_accumulate, uint32_t seed, uint32_t thresh16,
                            float inv_keep, hipStream_t st);
// y (+)= bf16(x * bf16(s[0])), s a device fp32 scalar
hipError_t launch_scale_acc(const void* x, const float* s, void* y, int64_t n, int accumulate, hipStream_t st);

// ---- weight-gradient GEMM (gemm_tn.hip): C[z][M,N] fp32 (+)= P^T Q over split z's rows of the
// nseg segments (P_i [seg_rows, >= M] ld ldp, Q_i [seg_rows, >= N] ld ldq; bf16, 16-byte aligned).
// Needs seg_rows % 128 == 0, M % 8 == N % 8 == 0, 1 <= splits <= nseg * seg_rows / 128, nseg <= 16.
// Cb non-null (splits == 1): C ignored, Cb [M, N] bf16 (+)= bf16(P^T Q) instead (the gradient itself).
hipError_t launch_gemm_tn(const void* const* P, const void* const* Q, int nseg, int64_t seg_rows, int ldp, int ldq,
                          float* C, int M, int N, int splits, bool accumulate, hipStream_t st, void* Cb = nullptr);

// diagnostic build of the plain GEMM with per-block timestamps (tools/gemm_stamps.py)
hipError_t launch_gemm_nt_stamped(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                                  unsigned long long* stamps, hipStream_t st);

// ---- LoRA adapter streams (lora.hip), bf16, r in {8, 16}, widths % 8 == 0
// out[t, :r] = scale * drop(in)[t, :] . w^T, w [r, K]; dropout when thresh16 > 0
hipError_t launch_lora_rows(const void* in, int64_t ldin, const void* w, void* out, int64_t rows, int K, int r,
                            float scale, uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st);
// out [rows, N] = o + bf16(s * u . b^T), u [rows, r], b [N, r]
hipError_t launch_lora_up(const void* o, int64_t ldo, const void* u, const void* b, void* out, int64_t rows, int N, int r,
                          float s, hipStream_t st);
// part fp32 = yscale * per-row-range y^T g'; mode 0: g' = g, part [parts, N, r]; mode 1:
// g' = drop(g), part [parts, r, N], also dx = drop'(y . a) with a [r, N]; lora_cols_parts picks
// the range count
int lora_cols_parts(int64_t rows, int N);
hipError_t launch_lora_cols(const void* g, int64_t ldg, const void* y, const void* a, void* dx, float* part, int64_t rows,
                            int N, int r, int parts, int mode, float yscale, uint32_t seed, uint32_t thresh16,
                            float inv_keep, hipStream_t st);

// ---- 4-bit blockwise quantization of frozen weights (quant.hip); n % 64 == 0, 16-byte aligned
// q [n / 2] uint8 (first element of a pair in the high nibble), absmax [n / 64] fp32, code [16] fp32
hipError_t launch_quant4(int dt, const void* w, const float* code, uint8_t* q, float* absmax, int64_t n,
                         hipStream_t st);
hipError_t launch_dequant4(int dt, const uint8_t* q, const float* absmax, const float* code, void* out, int64_t n,
                           hipStream_t st);
// transposed: out [K, >= N] (row stride ldo, 16-bit dtypes) = W^T for W [N, K]; N % 64 == 0, K % 128 == 0
hipError_t launch_dequant4_t(int dt, const uint8_t* q, const float* absmax, const float* code, void* out, int N, int K,
                             int64_t ldo, hipStream_t st);

// ---- LM head cross-entropy (xent_kernels.hip)
// variant 0 = auto (DLION_XENT env override), 1 fp32-row, 2 streaming, 3/4/5 packed 16-bit row (256/512/1024 thr)
hipError_t launch_softmax_xent(int dt, void* logits, const int64_t* labels, int64_t n, int64_t vp, int v, float* loss,
                               int variant, hipStream_t st);

}  // namespace dlion

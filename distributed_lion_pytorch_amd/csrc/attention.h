// Argument block of the gfx950 flash-attention kernels (attention.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dlion {

struct AttnArgs {
  const __bf16* q;
  const __bf16* k;
  const __bf16* v;
  const __bf16* o;
  const __bf16* dout;
  __bf16* out;        // fwd O
  __bf16* dq;
  __bf16* dk;
  __bf16* dv;
  float* lse;          // [B][H][T] base-2 log-sum-exp of scaled scores
  const float* delta;  // [B][H][T] rowsum(dO * O)
  float* colsum;       // nullable, [B * T/32][3 * H * D]: per-32-row column sums of dq | dk | dv (packed
                       // qkv bias gradient partials; needs H == Hkv)
  int64_t q_sb, q_st, q_sh;
  int64_t k_sb, k_st, k_sh;
  int64_t v_sb, v_st, v_sh;
  int64_t o_sb, o_st, o_sh;    // O and dO share this layout
  int64_t dq_sb, dq_st, dq_sh;
  int64_t dk_sb, dk_st, dk_sh;  // dK and dV share this layout
  int B, T, H, Hkv;
  float scale;       // softmax scale (1/sqrt(D))
  float scale_log2;  // scale * log2(e)
  uint32_t thresh16; // dropout threshold (keep if u16 >= thresh16), 0 = no dropout
  float inv_keep;
  uint32_t seed;
  // nullable [T][D] bf16 rotary tables: the backward stores dq / dk through the
  // inverse rotation (the gradient of rope(q), rope(k) w.r.t. q, k)
  const __bf16* rope_cos;
  const __bf16* rope_sin;
  // sliding window (Mistral, Qwen2 sliding layers): query q attends keys
  // q - window < k <= q; 0 = plain causal.  Key / query tiles wholly outside
  // the window are skipped, the boundary tiles masked per element.
  int window;
};

}  // namespace dlion

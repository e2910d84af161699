// Token + position embedding with dropout (the GPT-2 input layer) for gfx950.
//
// Reference path (HF GPT-2 on ATen, /root/reference/run_clm.py:442): two
// gathers, an add, a dropout kernel forward; backward a dropout-backward
// pass, ATen's sort-based embedding backward writing a DENSE [V, C] gradient
// (zero fill + scatter), then AccumulateGrad adding it into the tied
// wte/lm_head gradient -- ~300 us per GPT-2 micro-batch of mostly 77 MB
// passes over a gradient that receives 20480 rows.
//
// Here: one forward kernel (gather + add + hashed dropout), and two backward
// kernels that read the incoming gradient once each and touch only the rows
// that received tokens: the token gradient is a deterministic segmented sum
// over the stably sorted ids (one wave per distinct id, fixed order), added
// in place into the existing wte gradient; the position gradient sums the
// batch for each position.  The dropout keep-mask is keep4() of the flat
// element index (common.h), regenerated in the backward.
#include "common.h"
#include "kernels.h"

namespace dlion {

// 8 consecutive bf16 of one row, dropout-scaled (keep bits kp for elements 0..7)
__device__ __forceinline__ void drop8(float (&v)[8], uint32_t kp, float inv_keep) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = ((kp >> j) & 1u) ? v[j] * inv_keep : 0.f;
}

__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ ids, const uint16_t* __restrict__ wte,
                                                        const uint16_t* __restrict__ wpe, uint16_t* __restrict__ out,
                                                        int64_t n, int C, int T, int64_t V, uint32_t seed,
                                                        uint32_t thresh16, float inv_keep, int32_t* __restrict__ err) {
  const int cpr = C / 8;
  const int64_t total = n * cpr;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t row = i / cpr;
    const int c = static_cast<int>(i - row * cpr) * 8;
    int64_t id = ids[row];
    if (id < 0 || id >= V) {  // an error (flag checked once per step, ops/fused.py), never an out-of-bounds read
      if (err != nullptr) atomicOr(err, kIndexErrEmbed);
      id = id < 0 ? 0 : V - 1;
    }
    float a[8], b[8];
    Elem<kBF16>::load8(wte + id * C + c, a);
    Elem<kBF16>::load8(wpe + static_cast<int64_t>(row % T) * C + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = bf16_to_f32(f32_to_bf16(a[j] + b[j]));  // the bf16 sum ATen stores
    if (thresh16) drop8(a, keep8(seed, static_cast<uint64_t>(row) * C + c, thresh16), inv_keep);
    Elem<kBF16>::store8(out + row * C + c, a);
  }
}

// dropout-backward of 8 incoming gradient values, rounded like ATen's bf16 pass
__device__ __forceinline__ void dx8(const uint16_t* dx, int64_t row, int C, int c, uint32_t seed, uint32_t thresh16,
                                    float inv_keep, float (&v)[8]) {
  Elem<kBF16>::load8(dx + row * C + c, v);
  if (thresh16) {
    drop8(v, keep8(seed, static_cast<uint64_t>(row) * C + c, thresh16), inv_keep);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(f32_to_bf16(v[j]));
  }
}

// dwte[id] += sum of the (dropout-backward) gradient rows of the tokens with
// that id.  sid = ids sorted stably, perm = their positions.  One wave per
// sorted position; only the first position of each run of equal ids works,
// summing the run in sorted (= original) order: deterministic.
__global__ void __launch_bounds__(256) embed_bwd_tok_kernel(const uint16_t* __restrict__ dx,
                                                            const int64_t* __restrict__ sid,
                                                            const int64_t* __restrict__ perm,
                                                            uint16_t* __restrict__ dwte, int64_t n, int C, int64_t V,
                                                            uint32_t seed, uint32_t thresh16, float inv_keep) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * 4;
  const int cpr = C / 8;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); i < n; i += waves) {
    const int64_t id = sid[i];
    if ((i > 0 && sid[i - 1] == id) || id < 0 || id >= V) continue;  // wave-uniform
    for (int ch = lane; ch < cpr; ch += 64) {
      const int c = ch * 8;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int64_t j = i; j < n && sid[j] == id; ++j) {
        float v[8];
        dx8(dx, perm[j], C, c, seed, thresh16, inv_keep, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[k];
      }
      float g[8];
      uint16_t* dst = dwte + id * C + c;
      Elem<kBF16>::load8(dst, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] += bf16_to_f32(f32_to_bf16(acc[k]));  // + bf16(embedding grad)
      Elem<kBF16>::store8(dst, g);
    }
  }
}

// dwpe[t] (+)= sum over the batch of the gradient rows at position t
__global__ void __launch_bounds__(256) embed_bwd_pos_kernel(const uint16_t* __restrict__ dx, uint16_t* __restrict__ dwpe,
                                                            int64_t n, int C, int T, int accumulate, uint32_t seed,
                                                            uint32_t thresh16, float inv_keep) {
  const int cpr = C / 8;
  const int64_t total = static_cast<int64_t>(T) * cpr;
  const int64_t nb = n / T;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int t = static_cast<int>(i / cpr);
    const int c = static_cast<int>(i - static_cast<int64_t>(t) * cpr) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t b = 0; b < nb; ++b) {
      float v[8];
      dx8(dx, b * T + t, C, c, seed, thresh16, inv_keep, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    uint16_t* dst = dwpe + static_cast<int64_t>(t) * C + c;
    float g[8];
    if (accumulate) {
      Elem<kBF16>::load8(dst, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] += bf16_to_f32(f32_to_bf16(acc[k]));
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = acc[k];
    }
    Elem<kBF16>::store8(dst, g);
  }
}

// y (+)= bf16(x * bf16(s[0])) with s a device scalar (no host sync); bf16, n % 8 == 0
__global__ void __launch_bounds__(256) scale_acc_kernel(const uint16_t* __restrict__ x, const float* __restrict__ s,
                                                        uint16_t* __restrict__ y, int64_t n8, int accumulate) {
  const float sc = bf16_to_f32(f32_to_bf16(s[0]));
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n8;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    float a[8], g[8];
    Elem<kBF16>::load8(x + i * 8, a);
    if (accumulate) Elem<kBF16>::load8(y + i * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float t = bf16_to_f32(f32_to_bf16(a[k] * sc));
      g[k] = accumulate ? g[k] + t : t;
    }
    Elem<kBF16>::store8(y + i * 8, g);
  }
}

static inline unsigned grid_for(int64_t work, int64_t cap = 4096) {
  const int64_t g = (work + 255) / 256;
  return static_cast<unsigned>(g < 1 ? 1 : (g > cap ? cap : g));
}

// err[0] |= code for every id outside [0, hi) other than `ignore` (labels: -100)
__global__ void __launch_bounds__(256) index_check_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t hi,
                                                          int64_t ignore, int32_t* __restrict__ err, int code) {
  bool bad = false;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t v = ids[i];
    bad |= (v < 0 || v >= hi) && v != ignore;
  }
  if (bad) atomicOr(err, code);
}

hipError_t launch_index_check(const int64_t* ids, int64_t n, int64_t hi, int64_t ignore, int32_t* err, int code,
                              hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(index_check_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, ids, n, hi, ignore, err, code);
  return hipGetLastError();
}

hipError_t launch_embed_fwd(const int64_t* ids, const void* wte, const void* wpe, void* out, int64_t n, int C, int T,
                            int64_t V, uint32_t seed, uint32_t thresh16, float inv_keep, int32_t* err,
                            hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (C % 8 != 0 || T <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(n * (C / 8))), dim3(256), 0, st, ids,
                     static_cast<const uint16_t*>(wte), static_cast<const uint16_t*>(wpe), static_cast<uint16_t*>(out),
                     n, C, T, V, seed, thresh16, inv_keep, err);
  return hipGetLastError();
}

hipError_t launch_embed_bwd(const void* dx, const int64_t* sid, const int64_t* perm, void* dwte, void* dwpe, int64_t n,
                            int C, int T, int64_t V, int pos_accumulate, uint32_t seed, uint32_t thresh16,
                            float inv_keep, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (C % 8 != 0 || T <= 0 || n % T != 0) return hipErrorInvalidValue;
  const uint16_t* g = static_cast<const uint16_t*>(dx);
  if (dwte != nullptr) {
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(embed_bwd_tok_kernel, dim3(static_cast<unsigned>(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                       st, g, sid, perm, static_cast<uint16_t*>(dwte), n, C, V, seed, thresh16, inv_keep);
  }
  if (dwpe != nullptr) {
    hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(grid_for(static_cast<int64_t>(T) * (C / 8))), dim3(256), 0, st, g,
                       static_cast<uint16_t*>(dwpe), n, C, T, pos_accumulate, seed, thresh16, inv_keep);
  }
  return hipGetLastError();
}

hipError_t launch_scale_acc(const void* x, const float* s, void* y, int64_t n, int accumulate, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n % 8 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scale_acc_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, static_cast<const uint16_t*>(x), s,
                     static_cast<uint16_t*>(y), n / 8, accumulate);
  return hipGetLastError();
}

}  // namespace dlion

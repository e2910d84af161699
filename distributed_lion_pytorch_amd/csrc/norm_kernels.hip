// Fused residual + bias + dropout + LayerNorm / RMSNorm (forward and backward) for gfx950.
//
// One transformer sub-block boundary in the reference model (HF GPT-2 /
// Llama via ATen) is: bias add (GEMM epilogue) -> dropout(branch) ->
// residual add -> LayerNorm, i.e. 3-4 kernels forward and 7-8 backward
// (dropout mask + scale, add, LN grad-input, gamma/beta partial reductions,
// bias-grad reduction, grad accumulation adds).  Here it is one kernel each way:
//
//   fwd:  xo = x + keep * (y + bias) / (1-p)           (bf16 residual stream)
//         h  = (xo - mean) * rstd * gamma + beta         [RMS: xo * rstd * gamma]
//   bwd:  dxo = dxo_in + Norm_bwd(dh) -> dx (residual) and dy = keep * dxo / (1-p)
//         dgamma / dbeta / dbias: register accumulation over each wave's rows,
//         the block's 4 waves folded through LDS once at the end -> one fp32
//         partial row triple per block, summed by the caller.  Each wave
//         prefetches its next row while reducing the current one.
//
// One wave per row, 4 consecutive bf16 (8 bytes) per lane per step, C a
// multiple of 256 (<= 5120).  The dropout keep-mask is a stateless hash of
// (seed, row * C + col) at 16-bit resolution -- regenerated, never stored.
#include "common.h"
#include "kernels.h"

namespace dlion {

constexpr int kFwdWaves = 4;
constexpr int kBwdWaves = kNormBwdWaves;

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// keep bits for 4 consecutive elements starting at flat index idx (idx % 4 == 0):
// two 32-bit hashes, 16 bits per element
__device__ __forceinline__ uint32_t keep4(uint32_t seed, uint64_t idx, uint32_t thresh16) {
  const uint32_t hi = static_cast<uint32_t>(idx >> 33);
  const uint32_t h0 = mix32(seed ^ static_cast<uint32_t>(idx >> 1) * 0x9E3779B1u ^ hi);
  const uint32_t h1 = mix32(seed ^ static_cast<uint32_t>((idx >> 1) + 1) * 0x9E3779B1u ^ hi);
  uint32_t k = 0;
  k |= ((h0 & 0xffffu) >= thresh16) << 0;
  k |= ((h0 >> 16) >= thresh16) << 1;
  k |= ((h1 & 0xffffu) >= thresh16) << 2;
  k |= ((h1 >> 16) >= thresh16) << 3;
  return k;
}

__device__ __forceinline__ void ld4(const uint16_t* p, float (&o)[4]) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  o[0] = bf16_to_f32(v.x & 0xffffu);
  o[1] = bf16_to_f32(v.x >> 16);
  o[2] = bf16_to_f32(v.y & 0xffffu);
  o[3] = bf16_to_f32(v.y >> 16);
}
__device__ __forceinline__ void st4(uint16_t* p, const float (&o)[4]) {
  uint2 v;
  v.x = static_cast<uint32_t>(f32_to_bf16(o[0])) | (static_cast<uint32_t>(f32_to_bf16(o[1])) << 16);
  v.y = static_cast<uint32_t>(f32_to_bf16(o[2])) | (static_cast<uint32_t>(f32_to_bf16(o[3])) << 16);
  *reinterpret_cast<uint2*>(p) = v;
}

// --------------------------------------------------------------------- forward
// y may be null (plain norm of x), bias may be null.  NS = C / 256.
template <int NS, bool RMS>
__global__ void __launch_bounds__(64 * kFwdWaves)
add_norm_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ y, const uint16_t* __restrict__ bias,
                    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta, uint16_t* __restrict__ xo,
                    uint16_t* __restrict__ h, float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t rows,
                    float eps, uint32_t seed, uint32_t thresh16, float inv_keep) {
  constexpr int C = NS * 256;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kFwdWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t base = row * C;
  float v[NS][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int c = k * 256 + lane * 4;
    ld4(x + base + c, v[k]);
    if (y != nullptr) {
      float yv[4], bv[4] = {0.f, 0.f, 0.f, 0.f};
      ld4(y + base + c, yv);
      if (bias != nullptr) ld4(bias + c, bv);
      const uint32_t kp = thresh16 ? keep4(seed, static_cast<uint64_t>(base + c), thresh16) : 0xfu;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float add = ((kp >> j) & 1u) ? (yv[j] + bv[j]) * inv_keep : 0.f;
        v[k][j] = bf16_to_f32(f32_to_bf16(v[k][j] + add));  // residual stream is stored in bf16
      }
      st4(xo + base + c, v[k]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[k][j];
  }
  float mean = 0.f;
  if constexpr (!RMS) mean = wsum(s) * (1.f / C);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[k][j] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wsum(q) * (1.f / C) + eps);
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int c = k * 256 + lane * 4;
    float g[4], b[4] = {0.f, 0.f, 0.f, 0.f}, o[4];
    ld4(gamma + c, g);
    if constexpr (!RMS) ld4(beta + c, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + b[j];
    st4(h + base + c, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// -------------------------------------------------------------------- backward
// xo: the normalised input (the residual stream after the add); dxo_in: the
// residual-stream gradient from later layers (nullable).  Outputs: dx (residual
// grad), dy (branch grad, nullable for a plain norm).  part: [gridDim.x][3][C]
// fp32 partial sums of dgamma, dbeta, dbias (= sum dy) for this block's rows.
template <int NS, bool RMS>
__global__ void __launch_bounds__(64 * kBwdWaves)
add_norm_bwd_kernel(const uint16_t* __restrict__ dh, const uint16_t* __restrict__ dxo_in,
                    const uint16_t* __restrict__ xo, const uint16_t* __restrict__ gamma,
                    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, uint16_t* __restrict__ dx,
                    uint16_t* __restrict__ dy, float* __restrict__ part, int64_t rows, uint32_t seed,
                    uint32_t thresh16, float inv_keep) {
  constexpr int C = NS * 256;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float gacc[NS][4], bacc[NS][4], yacc[NS][4], g[NS][4];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    ld4(gamma + k * 256 + lane * 4, g[k]);
#pragma unroll
    for (int j = 0; j < 4; ++j) gacc[k][j] = bacc[k][j] = yacc[k][j] = 0.f;
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBwdWaves;
  int64_t row = static_cast<int64_t>(blockIdx.x) * kBwdWaves + w;
  // the row loop is a short dependent chain (two wave reductions per row), so
  // the next row's inputs are loaded before the current row is processed
  float nxo[NS][4], ndh[NS][4], ndx[NS][4];
  float nmean = 0.f, nrstd = 0.f;
  auto load_row = [&](int64_t r) {
    const int64_t b = r * C;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int c = k * 256 + lane * 4;
      ld4(xo + b + c, nxo[k]);
      ld4(dh + b + c, ndh[k]);
      if (dxo_in != nullptr) ld4(dxo_in + b + c, ndx[k]);
    }
    nmean = RMS ? 0.f : mean_in[r];
    nrstd = rstd_in[r];
  };
  if (row < rows) load_row(row);
  for (; row < rows; row += stride) {
    const int64_t base = row * C;
    const float mean = nmean, rstd = nrstd;
    float cxo[NS][4], cdh[NS][4], cdx[NS][4];
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cxo[k][j] = nxo[k][j];
        cdh[k][j] = ndh[k][j];
        cdx[k][j] = dxo_in != nullptr ? ndx[k][j] : 0.f;
      }
    if (row + stride < rows) load_row(row + stride);
    float xh[NS][4], gd[NS][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const float* xv = cxo[k];
      const float* dv = cdh[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[k][j] = (xv[j] - mean) * rstd;
        gd[k][j] = dv[j] * g[k][j];
        s1 += gd[k][j];
        s2 += gd[k][j] * xh[k][j];
        gacc[k][j] += dv[j] * xh[k][j];
        bacc[k][j] += dv[j];
      }
    }
    const float m1 = RMS ? 0.f : wsum(s1) * (1.f / C);
    const float m2 = wsum(s2) * (1.f / C);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int c = k * 256 + lane * 4;
      float t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = cdx[k][j] + rstd * (gd[k][j] - m1 - xh[k][j] * m2);
      st4(dx + base + c, t);
      if (dy != nullptr) {
        const uint32_t kp = thresh16 ? keep4(seed, static_cast<uint64_t>(base + c), thresh16) : 0xfu;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = ((kp >> j) & 1u) ? t[j] * inv_keep : 0.f;
          yacc[k][j] += bf16_to_f32(f32_to_bf16(o[j]));  // bias grad of exactly what is stored
        }
        st4(dy + base + c, o);
      }
    }
  }
  // fold the block's waves into one fp32 partial row triple part[block][3][C]:
  // waves kBwdWaves-1 .. 1 accumulate into one LDS row triple in turn (every
  // lane touches only its own columns), wave 0 adds it and stores
  __shared__ float4 red[3 * C / 4];
  for (int src = kBwdWaves - 1; src >= 1; --src) {
    if (w == src) {
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const int c4 = k * 64 + lane;
        float4 a = make_float4(gacc[k][0], gacc[k][1], gacc[k][2], gacc[k][3]);
        float4 b = make_float4(bacc[k][0], bacc[k][1], bacc[k][2], bacc[k][3]);
        float4 d = make_float4(yacc[k][0], yacc[k][1], yacc[k][2], yacc[k][3]);
        if (src != kBwdWaves - 1) {
          const float4 a0 = red[c4], b0 = red[C / 4 + c4], d0 = red[C / 2 + c4];
          a.x += a0.x; a.y += a0.y; a.z += a0.z; a.w += a0.w;
          b.x += b0.x; b.y += b0.y; b.z += b0.z; b.w += b0.w;
          d.x += d0.x; d.y += d0.y; d.z += d0.z; d.w += d0.w;
        }
        red[c4] = a;
        red[C / 4 + c4] = b;
        red[C / 2 + c4] = d;
      }
    }
    __syncthreads();
  }
  if (w == 0) {
    float4* out = reinterpret_cast<float4*>(part + static_cast<int64_t>(blockIdx.x) * 3 * C);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int c4 = k * 64 + lane;
      const float4 a0 = red[c4], b0 = red[C / 4 + c4], d0 = red[C / 2 + c4];
      out[c4] = make_float4(gacc[k][0] + a0.x, gacc[k][1] + a0.y, gacc[k][2] + a0.z, gacc[k][3] + a0.w);
      out[C / 4 + c4] = make_float4(bacc[k][0] + b0.x, bacc[k][1] + b0.y, bacc[k][2] + b0.z, bacc[k][3] + b0.w);
      out[C / 2 + c4] = make_float4(yacc[k][0] + d0.x, yacc[k][1] + d0.y, yacc[k][2] + d0.z, yacc[k][3] + d0.w);
    }
  }
}

// ------------------------------------------------------------------ launchers
#define NORM_DISPATCH(NS_VAL, ...)                                 \
  switch (NS_VAL) {                                                \
    case 1: { constexpr int NS = 1; __VA_ARGS__; break; }          \
    case 2: { constexpr int NS = 2; __VA_ARGS__; break; }          \
    case 3: { constexpr int NS = 3; __VA_ARGS__; break; }          \
    case 4: { constexpr int NS = 4; __VA_ARGS__; break; }          \
    case 5: { constexpr int NS = 5; __VA_ARGS__; break; }          \
    case 8: { constexpr int NS = 8; __VA_ARGS__; break; }          \
    case 16: { constexpr int NS = 16; __VA_ARGS__; break; }        \
    case 20: { constexpr int NS = 20; __VA_ARGS__; break; }        \
    default: return hipErrorInvalidValue;                          \
  }

hipError_t launch_add_norm_fwd(const void* x, const void* y, const void* bias, const void* gamma, const void* beta,
                               void* xo, void* h, float* mean, float* rstd, int64_t rows, int C, float eps, bool rms,
                               uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st) {
  if (C % 256 != 0) return hipErrorInvalidValue;
  const dim3 grid((rows + kFwdWaves - 1) / kFwdWaves), block(64 * kFwdWaves);
  auto X = static_cast<const uint16_t*>(x);
  auto Y = static_cast<const uint16_t*>(y);
  auto Bi = static_cast<const uint16_t*>(bias);
  auto G = static_cast<const uint16_t*>(gamma);
  auto Bt = static_cast<const uint16_t*>(beta);
  auto XO = static_cast<uint16_t*>(xo);
  auto H = static_cast<uint16_t*>(h);
  if (rms) {
    NORM_DISPATCH(C / 256, hipLaunchKernelGGL((add_norm_fwd_kernel<NS, true>), grid, block, 0, st, X, Y, Bi, G, Bt,
                                              XO, H, mean, rstd, rows, eps, seed, thresh16, inv_keep));
  } else {
    NORM_DISPATCH(C / 256, hipLaunchKernelGGL((add_norm_fwd_kernel<NS, false>), grid, block, 0, st, X, Y, Bi, G, Bt,
                                              XO, H, mean, rstd, rows, eps, seed, thresh16, inv_keep));
  }
  return hipGetLastError();
}

hipError_t launch_add_norm_bwd(const void* dh, const void* dxo_in, const void* xo, const void* gamma, const float* mean,
                               const float* rstd, void* dx, void* dy, float* part, int parts, int64_t rows, int C,
                               bool rms, uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st) {
  if (C % 256 != 0) return hipErrorInvalidValue;
  const dim3 grid(parts), block(64 * kBwdWaves);
  auto DH = static_cast<const uint16_t*>(dh);
  auto DXI = static_cast<const uint16_t*>(dxo_in);
  auto XO = static_cast<const uint16_t*>(xo);
  auto G = static_cast<const uint16_t*>(gamma);
  auto DX = static_cast<uint16_t*>(dx);
  auto DY = static_cast<uint16_t*>(dy);
  if (rms) {
    NORM_DISPATCH(C / 256, hipLaunchKernelGGL((add_norm_bwd_kernel<NS, true>), grid, block, 0, st, DH, DXI, XO, G,
                                              mean, rstd, DX, DY, part, rows, seed, thresh16, inv_keep));
  } else {
    NORM_DISPATCH(C / 256, hipLaunchKernelGGL((add_norm_bwd_kernel<NS, false>), grid, block, 0, st, DH, DXI, XO, G,
                                              mean, rstd, DX, DY, part, rows, seed, thresh16, inv_keep));
  }
  return hipGetLastError();
}

}  // namespace dlion

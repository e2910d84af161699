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
// One wave per row for C <= 1024 (GPT-2), one WPR-wave block per row for the
// wide Llama rows (C = 2048..8192); 4 consecutive bf16 (8 bytes) per lane per
// step, the whole row held in registers.  The dropout keep-mask is a stateless hash of
// (seed, row * C + col) at 16-bit resolution -- regenerated, never stored.
#include "common.h"
#include "kernels.h"

namespace dlion {


// full-wave sum without LDS (common.h wave_sum_dpp): __shfl_xor lowered to six
// dependent ds_bpermute round trips per reduction, two reductions per row
__device__ __forceinline__ float wsum(float v) { return wave_sum_dpp(v); }

__device__ __forceinline__ void unpack4(const uint2 v, float (&o)[4]) {
  o[0] = bf16_to_f32(v.x & 0xffffu);
  o[1] = bf16_to_f32(v.x >> 16);
  o[2] = bf16_to_f32(v.y & 0xffffu);
  o[3] = bf16_to_f32(v.y >> 16);
}
__device__ __forceinline__ void ld4(const uint16_t* p, float (&o)[4]) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  o[0] = bf16_to_f32(v.x & 0xffffu);
  o[1] = bf16_to_f32(v.x >> 16);
  o[2] = bf16_to_f32(v.y & 0xffffu);
  o[3] = bf16_to_f32(v.y >> 16);
}
// row loads / stores use the default cache policy: non-temporal hints on the
// row streams (as on the MLP GEMM epilogues) measured neutral here
typedef unsigned int norm_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 ldrow(const uint16_t* p) {
  const norm_u32x2 v = *reinterpret_cast<const norm_u32x2*>(p);
  return make_uint2(v[0], v[1]);
}
__device__ __forceinline__ void st4(uint16_t* p, const float (&o)[4]) {
  norm_u32x2 v;
  v[0] = static_cast<uint32_t>(f32_to_bf16(o[0])) | (static_cast<uint32_t>(f32_to_bf16(o[1])) << 16);
  v[1] = static_cast<uint32_t>(f32_to_bf16(o[2])) | (static_cast<uint32_t>(f32_to_bf16(o[3])) << 16);
  *reinterpret_cast<norm_u32x2*>(p) = v;
}

// Row groups: WPR waves cooperate on one row (WPR = 1 for C <= 1024; 2..8 for
// the wide Llama rows, C = 2048 .. 8192), so a lane holds NS*4 <= 16 values of
// a row in registers.  C = NS * 4 * 64 * WPR; column of chunk k for group
// thread tg: k * 256 * WPR + tg * 4.  Blocks are 4 waves of 4 rows when
// WPR = 1, else WPR waves of one row.
template <int WPR>
struct RowGroup {
  static constexpr int kWaves = WPR == 1 ? 4 : WPR;  // waves per block
  static constexpr int kRows = kWaves / WPR;         // rows per block
};
template <int WPR>
__device__ __forceinline__ float2 gsum2(float a, float b, float2* scratch) {
  a = wsum(a);
  b = wsum(b);
  if constexpr (WPR == 1) {
    return make_float2(a, b);
  } else {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) scratch[w] = make_float2(a, b);
    __syncthreads();
    float2 t = scratch[0];
#pragma unroll
    for (int i = 1; i < WPR; ++i) {
      t.x += scratch[i].x;
      t.y += scratch[i].y;
    }
    __syncthreads();  // scratch is reused by the next reduction
    return t;
  }
}

// --------------------------------------------------------------------- forward
// y may be null (plain norm of x), bias may be null.
template <int NS, int WPR, bool RMS>
__global__ void __launch_bounds__(64 * RowGroup<WPR>::kWaves)
add_norm_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ y, const uint16_t* __restrict__ bias,
                    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta, uint16_t* __restrict__ xo,
                    uint16_t* __restrict__ h, float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t rows,
                    float eps, uint32_t seed, uint32_t thresh16, float inv_keep) {
  constexpr int G = 64 * WPR, C = NS * 4 * G;
  __shared__ float2 scratch[WPR];
  const int tg = threadIdx.x % G;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * RowGroup<WPR>::kRows + threadIdx.x / G;
  if (row >= rows) return;  // uniform per row group (the whole block when WPR > 1)
  const int64_t base = row * C;
  // every load of the row is issued before any use (with the null checks
  // inside the k loop, hipcc waited vmcnt(0) per chunk: six serial round
  // trips per row); gamma / beta too, ahead of the reductions
  uint2 rx[NS], ry[NS], rb[NS], rg[NS], re[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) rx[k] = ldrow(x + base + k * 4 * G + tg * 4);
  const bool has_y = y != nullptr, has_b = has_y && bias != nullptr;
  if (has_y) {
#pragma unroll
    for (int k = 0; k < NS; ++k) ry[k] = ldrow(y + base + k * 4 * G + tg * 4);
  }
  if (has_b) {
#pragma unroll
    for (int k = 0; k < NS; ++k) rb[k] = *reinterpret_cast<const uint2*>(bias + k * 4 * G + tg * 4);
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    rg[k] = *reinterpret_cast<const uint2*>(gamma + k * 4 * G + tg * 4);
    if constexpr (!RMS) re[k] = *reinterpret_cast<const uint2*>(beta + k * 4 * G + tg * 4);
  }
  float v[NS][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int c = k * 4 * G + tg * 4;
    unpack4(rx[k], v[k]);
    if (has_y) {
      float yv[4], bv[4] = {0.f, 0.f, 0.f, 0.f};
      unpack4(ry[k], yv);
      if (has_b) unpack4(rb[k], bv);
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
  if constexpr (!RMS) mean = gsum2<WPR>(s, 0.f, scratch).x * (1.f / C);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[k][j] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(gsum2<WPR>(q, 0.f, scratch).x * (1.f / C) + eps);
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int c = k * 4 * G + tg * 4;
    float g[4], b[4] = {0.f, 0.f, 0.f, 0.f}, o[4];
    unpack4(rg[k], g);
    if constexpr (!RMS) unpack4(re[k], b);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + b[j];
    st4(h + base + c, o);
  }
  if (tg == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// -------------------------------------------------------------------- backward
// xo: the normalised input (the residual stream after the add); dxo_in: the
// residual-stream gradient from later layers (nullable).  Outputs: dx (residual
// grad), dy (branch grad, nullable for a plain norm).  part: [gridDim.x][3][C]
// fp32 partial sums of dgamma, dbeta, dbias (= sum dy) for this block's rows.
template <int NS, int WPR, bool RMS>
__global__ void __launch_bounds__(64 * RowGroup<WPR>::kWaves)
add_norm_bwd_kernel(const uint16_t* __restrict__ dh, const uint16_t* __restrict__ dxo_in,
                    const uint16_t* __restrict__ xo, const uint16_t* __restrict__ gamma,
                    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, uint16_t* __restrict__ dx,
                    uint16_t* __restrict__ dy, float* __restrict__ part, int64_t rows, uint32_t seed,
                    uint32_t thresh16, float inv_keep) {
  constexpr int G = 64 * WPR, C = NS * 4 * G, RPB = RowGroup<WPR>::kRows;
  __shared__ float2 scratch[WPR];
  const int tg = threadIdx.x % G, grp = threadIdx.x / G;
  float gacc[NS][4], bacc[NS][4], yacc[NS][4], g[NS][4];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    ld4(gamma + k * 4 * G + tg * 4, g[k]);
#pragma unroll
    for (int j = 0; j < 4; ++j) gacc[k][j] = bacc[k][j] = yacc[k][j] = 0.f;
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * RPB;
  int64_t row = static_cast<int64_t>(blockIdx.x) * RPB + grp;
  // the row loop is a short dependent chain (two group reductions per row), so
  // the next row's inputs are loaded before the current row is processed
  // (kept as packed bf16 until use: half the registers of fp32)
  uint2 nxo[NS], ndh[NS], ndx[NS];
  float nmean = 0.f, nrstd = 0.f;
  auto load_row = [&](int64_t r) {
    const int64_t b = r * C;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int c = k * 4 * G + tg * 4;
      nxo[k] = ldrow(xo + b + c);
      ndh[k] = ldrow(dh + b + c);
      if (dxo_in != nullptr) ndx[k] = ldrow(dxo_in + b + c);
    }
    nmean = RMS ? 0.f : mean_in[r];
    nrstd = rstd_in[r];
  };
  if (row < rows) load_row(row);
  for (; row < rows; row += stride) {  // uniform trip count per row group
    const int64_t base = row * C;
    const float mean = nmean, rstd = nrstd;
    float cxo[NS][4], cdh[NS][4], cdx[NS][4];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      unpack4(nxo[k], cxo[k]);
      unpack4(ndh[k], cdh[k]);
      if (dxo_in != nullptr) unpack4(ndx[k], cdx[k]);
      else cdx[k][0] = cdx[k][1] = cdx[k][2] = cdx[k][3] = 0.f;
    }
    if (row + stride < rows) load_row(row + stride);
    float xh[NS][4], gd[NS][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[k][j] = (cxo[k][j] - mean) * rstd;
        gd[k][j] = cdh[k][j] * g[k][j];
        s1 += gd[k][j];
        s2 += gd[k][j] * xh[k][j];
        gacc[k][j] += cdh[k][j] * xh[k][j];
        bacc[k][j] += cdh[k][j];
      }
    }
    const float2 ms = gsum2<WPR>(RMS ? 0.f : s1, s2, scratch);
    const float m1 = ms.x * (1.f / C), m2 = ms.y * (1.f / C);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int c = k * 4 * G + tg * 4;
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
  float4* out = reinterpret_cast<float4*>(part + static_cast<int64_t>(blockIdx.x) * 3 * C);
  if constexpr (RPB == 1) {
    // one row group per block: every thread owns distinct columns
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int c4 = k * G + tg;
      out[c4] = make_float4(gacc[k][0], gacc[k][1], gacc[k][2], gacc[k][3]);
      out[C / 4 + c4] = make_float4(bacc[k][0], bacc[k][1], bacc[k][2], bacc[k][3]);
      out[C / 2 + c4] = make_float4(yacc[k][0], yacc[k][1], yacc[k][2], yacc[k][3]);
    }
  } else {
    // fold the block's RPB row groups into one partial row triple: groups
    // RPB-1 .. 1 accumulate into one LDS row triple in turn (each thread
    // touches only its own columns), group 0 adds it and stores
    __shared__ float4 red[3 * C / 4];
    for (int src = RPB - 1; src >= 1; --src) {
      if (grp == src) {
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          const int c4 = k * G + tg;
          float4 a = make_float4(gacc[k][0], gacc[k][1], gacc[k][2], gacc[k][3]);
          float4 b = make_float4(bacc[k][0], bacc[k][1], bacc[k][2], bacc[k][3]);
          float4 d = make_float4(yacc[k][0], yacc[k][1], yacc[k][2], yacc[k][3]);
          if (src != RPB - 1) {
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
    if (grp == 0) {
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const int c4 = k * G + tg;
        const float4 a0 = red[c4], b0 = red[C / 4 + c4], d0 = red[C / 2 + c4];
        out[c4] = make_float4(gacc[k][0] + a0.x, gacc[k][1] + a0.y, gacc[k][2] + a0.z, gacc[k][3] + a0.w);
        out[C / 4 + c4] = make_float4(bacc[k][0] + b0.x, bacc[k][1] + b0.y, bacc[k][2] + b0.z, bacc[k][3] + b0.w);
        out[C / 2 + c4] = make_float4(yacc[k][0] + d0.x, yacc[k][1] + d0.y, yacc[k][2] + d0.z, yacc[k][3] + d0.w);
      }
    }
  }
}

// ------------------------------------------------------------------ launchers
// (WPR, NS) shapes: C = 256..1024 one wave per row; C = 2048..8192 (multiples
// of 1024) one WPR-wave block per row.  Anything else -> hipErrorInvalidValue
// (the Python side checks norm_supported() first and uses ATen otherwise).
#define NORM_DISPATCH(C_VAL, ...)                                                 \
  switch (C_VAL) {                                                                \
    case 256: { constexpr int NS = 1, WPR = 1; __VA_ARGS__; break; }             \
    case 512: { constexpr int NS = 2, WPR = 1; __VA_ARGS__; break; }             \
    case 768: { constexpr int NS = 3, WPR = 1; __VA_ARGS__; break; }             \
    case 1024: { constexpr int NS = 4, WPR = 1; __VA_ARGS__; break; }            \
    case 2048: { constexpr int NS = 4, WPR = 2; __VA_ARGS__; break; }            \
    case 3072: { constexpr int NS = 4, WPR = 3; __VA_ARGS__; break; }            \
    case 4096: { constexpr int NS = 4, WPR = 4; __VA_ARGS__; break; }            \
    case 5120: { constexpr int NS = 4, WPR = 5; __VA_ARGS__; break; }            \
    case 6144: { constexpr int NS = 4, WPR = 6; __VA_ARGS__; break; }            \
    case 8192: { constexpr int NS = 4, WPR = 8; __VA_ARGS__; break; }            \
    default: return hipErrorInvalidValue;                                         \
  }

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

hipError_t launch_add_norm_fwd(const void* x, const void* y, const void* bias, const void* gamma, const void* beta,
                               void* xo, void* h, float* mean, float* rstd, int64_t rows, int C, float eps, bool rms,
                               uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st) {
  auto X = static_cast<const uint16_t*>(x);
  auto Y = static_cast<const uint16_t*>(y);
  auto Bi = static_cast<const uint16_t*>(bias);
  auto G = static_cast<const uint16_t*>(gamma);
  auto Bt = static_cast<const uint16_t*>(beta);
  auto XO = static_cast<uint16_t*>(xo);
  auto H = static_cast<uint16_t*>(h);
  if (rms) {
    NORM_DISPATCH(C, hipLaunchKernelGGL((add_norm_fwd_kernel<NS, WPR, true>), dim3(ceil_div(rows, RowGroup<WPR>::kRows)),
                                        dim3(64 * RowGroup<WPR>::kWaves), 0, st, X, Y, Bi, G, Bt, XO, H, mean, rstd, rows, eps, seed, thresh16,
                                        inv_keep));
  } else {
    NORM_DISPATCH(C, hipLaunchKernelGGL((add_norm_fwd_kernel<NS, WPR, false>), dim3(ceil_div(rows, RowGroup<WPR>::kRows)),
                                        dim3(64 * RowGroup<WPR>::kWaves), 0, st, X, Y, Bi, G, Bt, XO, H, mean, rstd, rows, eps, seed, thresh16,
                                        inv_keep));
  }
  return hipGetLastError();
}

hipError_t launch_add_norm_bwd(const void* dh, const void* dxo_in, const void* xo, const void* gamma, const float* mean,
                               const float* rstd, void* dx, void* dy, float* part, int parts, int64_t rows, int C,
                               bool rms, uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st) {
  const dim3 grid(parts);
  auto DH = static_cast<const uint16_t*>(dh);
  auto DXI = static_cast<const uint16_t*>(dxo_in);
  auto XO = static_cast<const uint16_t*>(xo);
  auto G = static_cast<const uint16_t*>(gamma);
  auto DX = static_cast<uint16_t*>(dx);
  auto DY = static_cast<uint16_t*>(dy);
  if (rms) {
    NORM_DISPATCH(C, hipLaunchKernelGGL((add_norm_bwd_kernel<NS, WPR, true>), grid, dim3(64 * RowGroup<WPR>::kWaves), 0, st, DH, DXI, XO, G,
                                        mean, rstd, DX, DY, part, rows, seed, thresh16, inv_keep));
  } else {
    NORM_DISPATCH(C, hipLaunchKernelGGL((add_norm_bwd_kernel<NS, WPR, false>), grid, dim3(64 * RowGroup<WPR>::kWaves), 0, st, DH, DXI, XO, G,
                                        mean, rstd, DX, DY, part, rows, seed, thresh16, inv_keep));
  }
  return hipGetLastError();
}

}  // namespace dlion

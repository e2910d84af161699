// Elementwise epilogues for gfx950: bias + GELU (forward / backward with fused
// bias gradient), SwiGLU, rotary embedding, and fp32 partial-sum reduction to bf16.
//
// MLP up-projection in the reference (HF GPT-2 NewGELU on ATen): GEMM with
// bias epilogue -> GELU kernel; backward: GELU-backward kernel -> separate
// column-sum kernel for the bias gradient.  Here the GEMM runs without bias
// and one kernel does bias + GELU; the backward kernel emits dZ and the bias
// gradient's per-block partial sums in the same pass.
// sum_partials reduces split-K / per-block fp32 partials [S][n] straight to
// bf16 (one pass instead of ATen sum + dtype copy).
#include "common.h"

namespace dlion {

// rows x N, 8 columns per thread per step; EXACT selects erf-GELU
template <bool EXACT>
__global__ void __launch_bounds__(256) bias_gelu_fwd_kernel(const uint16_t* __restrict__ z,
                                                           const uint16_t* __restrict__ b, uint16_t* __restrict__ h,
                                                           int64_t rows, int N) {
  const int64_t n8 = static_cast<int64_t>(rows) * (N / 8);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n8;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t e = i * 8;
    const int col = static_cast<int>(e % N);
    float zv[8], bv[8], o[8];
    Elem<kBF16>::load8(z + e, zv);
    Elem<kBF16>::load8(b + col, bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gelu_f(zv[j] + bv[j], EXACT);
    Elem<kBF16>::store8(h + e, o);
  }
}

// grid = parts blocks; block walks rows blockIdx.x, += gridDim.x; each thread
// owns NC groups of 8 columns; writes dz and one fp32 partial row of db.
template <bool EXACT, int NC>
__global__ void __launch_bounds__(1024) bias_gelu_bwd_kernel(const uint16_t* __restrict__ dh,
                                                            const uint16_t* __restrict__ z,
                                                            const uint16_t* __restrict__ b, uint16_t* __restrict__ dz,
                                                            float* __restrict__ dbpart, int64_t rows, int N) {
  const int groups = N / 8;
  const int bd = blockDim.x;
  float bv[NC][8], acc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int g = c * bd + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
    if (g < groups) Elem<kBF16>::load8(b + g * 8, bv[c]);
  }
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t base = r * N;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int g = c * bd + threadIdx.x;
      if (g >= groups) continue;
      float dv[8], zv[8], o[8];
      Elem<kBF16>::load8(dh + base + g * 8, dv);
      Elem<kBF16>::load8(z + base + g * 8, zv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = dv[j] * gelu_grad(zv[j] + bv[c][j], EXACT);
        acc[c][j] += bf16_to_f32(f32_to_bf16(o[j]));
      }
      Elem<kBF16>::store8(dz + base + g * 8, o);
    }
  }
  float* out = dbpart + static_cast<int64_t>(blockIdx.x) * N;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int g = c * bd + threadIdx.x;
    if (g < groups) {
      *reinterpret_cast<float4*>(out + g * 8) = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
      *reinterpret_cast<float4*>(out + g * 8 + 4) = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
    }
  }
}

// out[i] = bf16(sum_s part[s][i] (+ out[i] when ACC: gradient accumulation
// fused into the split-K reduction)), 4 elements per thread
template <bool ACC>
__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ part, int S, int64_t n,
                                                          int64_t ld, uint16_t* __restrict__ out,
                                                          const float* __restrict__ scale) {
  const int64_t n4 = n / 4;
  const float sc = scale ? scale[0] : 1.f;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n4;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    float4 acc = reinterpret_cast<const float4*>(part)[i];
    for (int s = 1; s < S; ++s) {
      const float4 v = reinterpret_cast<const float4*>(part + static_cast<int64_t>(s) * ld)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    acc.x *= sc; acc.y *= sc; acc.z *= sc; acc.w *= sc;
    if constexpr (ACC) {
      const uint2 o = reinterpret_cast<const uint2*>(out)[i];
      acc.x += bf16_to_f32(o.x & 0xffffu);
      acc.y += bf16_to_f32(o.x >> 16);
      acc.z += bf16_to_f32(o.y & 0xffffu);
      acc.w += bf16_to_f32(o.y >> 16);
    }
    uint2 w;
    w.x = static_cast<uint32_t>(f32_to_bf16(acc.x)) | (static_cast<uint32_t>(f32_to_bf16(acc.y)) << 16);
    w.y = static_cast<uint32_t>(f32_to_bf16(acc.z)) | (static_cast<uint32_t>(f32_to_bf16(acc.w)) << 16);
    reinterpret_cast<uint2*>(out)[i] = w;
  }
}

// Column sums of a bf16 [rows, N] matrix as fp32 per-block partial rows (the
// bias gradient of a linear layer whose output gradient has no other consumer
// to fuse into); same thread layout as bias_gelu_bwd.
template <int NC>
__global__ void __launch_bounds__(1024) colsum_kernel(const uint16_t* __restrict__ x, float* __restrict__ part,
                                                     int64_t rows, int N) {
  const int groups = N / 8, bd = blockDim.x;
  float acc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int g = c * bd + threadIdx.x;
      if (g >= groups) continue;
      float v[8];
      Elem<kBF16>::load8(x + r * N + g * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[c][j] += v[j];
    }
  }
  float* out = part + static_cast<int64_t>(blockIdx.x) * N;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int g = c * bd + threadIdx.x;
    if (g < groups) {
      *reinterpret_cast<float4*>(out + g * 8) = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
      *reinterpret_cast<float4*>(out + g * 8 + 4) = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
    }
  }
}

// ------------------------------------------------------------------ SwiGLU
// Llama MLP activation h = silu(g) * u (HF LlamaMLP: act_fn(gate_proj(x)) *
// up_proj(x)), one pass each way: ATen needs silu + mul forward and
// mul / silu_backward / mul backward with fp32 -> bf16 round trips between.
__device__ __forceinline__ float sigmoid_f(float a) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-a * 1.4426950408889634f));
}

// Row geometry: rows x F, inputs g / u at row stride ld_in (the two halves of a
// fused [gate | up] projection output, ld_in = 2F, need no copy), h / dh
// contiguous, dg / du at row stride ld_out (2F: straight into the fused
// projection's input-gradient buffer).
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u,
                                                        uint16_t* __restrict__ h, int64_t n8, int64_t f8,
                                                        int64_t ld_in) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n8;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t src = (i / f8) * ld_in + (i % f8) * 8;
    float gv[8], uv[8], o[8];
    Elem<kBF16>::load8(g + src, gv);
    Elem<kBF16>::load8(u + src, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gv[j] * sigmoid_f(gv[j]) * uv[j];
    Elem<kBF16>::store8(h + i * 8, o);
  }
}

__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const uint16_t* __restrict__ dh,
                                                        const uint16_t* __restrict__ g,
                                                        const uint16_t* __restrict__ u, uint16_t* __restrict__ dg,
                                                        uint16_t* __restrict__ du, int64_t n8, int64_t f8,
                                                        int64_t ld_in, int64_t ld_out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n8;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t row = i / f8, c = (i % f8) * 8;
    const int64_t src = row * ld_in + c, dst = row * ld_out + c;
    float dv[8], gv[8], uv[8], og[8], ou[8];
    Elem<kBF16>::load8(dh + i * 8, dv);
    Elem<kBF16>::load8(g + src, gv);
    Elem<kBF16>::load8(u + src, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = sigmoid_f(gv[j]);
      ou[j] = dv[j] * gv[j] * sg;
      og[j] = dv[j] * uv[j] * sg * (1.f + gv[j] * (1.f - sg));
    }
    Elem<kBF16>::store8(dg + dst, og);
    Elem<kBF16>::store8(du + dst, ou);
  }
}

// The forward on 64-token x 64-feature tiles that also writes hT [F, rows],
// the token-contiguous copy of h the down projection's weight gradient uses
// in its NT form (written once here instead of transposed in the backward).
__global__ void __launch_bounds__(256) swiglu_fwd_t_kernel(const uint16_t* __restrict__ g,
                                                          const uint16_t* __restrict__ u, uint16_t* __restrict__ h,
                                                          uint16_t* __restrict__ ht, int64_t F, int64_t ld_in,
                                                          int64_t rows) {
  __shared__ uint16_t th[64][66];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * 64, c0 = static_cast<int64_t>(blockIdx.x) * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = threadIdx.x + k * 256, tr = idx >> 3, tc = (idx & 7) * 8;
    const int64_t row = r0 + tr, c = c0 + tc;
    float gv[8], uv[8], o[8];
    Elem<kBF16>::load8(g + row * ld_in + c, gv);
    Elem<kBF16>::load8(u + row * ld_in + c, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = gv[j] * sigmoid_f(gv[j]) * uv[j];
      th[tr][tc + j] = f32_to_bf16(o[j]);
    }
    Elem<kBF16>::store8(h + row * F + c, o);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = threadIdx.x + k * 256, oc = idx >> 3, orr = (idx & 7) * 8;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = static_cast<uint32_t>(th[orr + 2 * j][oc]) | (static_cast<uint32_t>(th[orr + 2 * j + 1][oc]) << 16);
    *reinterpret_cast<uint4*>(ht + (c0 + oc) * rows + r0 + orr) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// The same backward on 64-token x 64-feature tiles that also writes the
// token-contiguous copy dguT [2F, rows] of dgu = [dg | du] (the operand the
// gate/up weight gradient's NT form wants, ops/linear.py _wgrad_via_transposes):
// the tile's results go out row-major as above and, staged through LDS,
// transposed -- one extra write of dgu instead of a transpose pass that reads
// and writes it again.  rows % 64 == 0, F % 64 == 0 (the launcher checks).
__global__ void __launch_bounds__(256) swiglu_bwd_t_kernel(const uint16_t* __restrict__ dh,
                                                          const uint16_t* __restrict__ g,
                                                          const uint16_t* __restrict__ u,
                                                          uint16_t* __restrict__ dgu, uint16_t* __restrict__ dgut,
                                                          int64_t F, int64_t ld_in, int64_t rows) {
  __shared__ uint16_t tg[64][66], tu[64][66];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * 64, c0 = static_cast<int64_t>(blockIdx.x) * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + h * 256, tr = idx >> 3, tc = (idx & 7) * 8;
    const int64_t row = r0 + tr, c = c0 + tc;
    float dv[8], gv[8], uv[8], og[8], ou[8];
    Elem<kBF16>::load8(dh + row * F + c, dv);
    Elem<kBF16>::load8(g + row * ld_in + c, gv);
    Elem<kBF16>::load8(u + row * ld_in + c, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = sigmoid_f(gv[j]);
      ou[j] = dv[j] * gv[j] * sg;
      og[j] = dv[j] * uv[j] * sg * (1.f + gv[j] * (1.f - sg));
      tg[tr][tc + j] = f32_to_bf16(og[j]);
      tu[tr][tc + j] = f32_to_bf16(ou[j]);
    }
    Elem<kBF16>::store8(dgu + row * 2 * F + c, og);
    Elem<kBF16>::store8(dgu + row * 2 * F + F + c, ou);
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + h * 256, oc = idx >> 3, orr = (idx & 7) * 8;
    uint32_t wg[4], wu[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wg[j] = static_cast<uint32_t>(tg[orr + 2 * j][oc]) | (static_cast<uint32_t>(tg[orr + 2 * j + 1][oc]) << 16);
      wu[j] = static_cast<uint32_t>(tu[orr + 2 * j][oc]) | (static_cast<uint32_t>(tu[orr + 2 * j + 1][oc]) << 16);
    }
    *reinterpret_cast<uint4*>(dgut + (c0 + oc) * rows + r0 + orr) = make_uint4(wg[0], wg[1], wg[2], wg[3]);
    *reinterpret_cast<uint4*>(dgut + (F + c0 + oc) * rows + r0 + orr) = make_uint4(wu[0], wu[1], wu[2], wu[3]);
  }
}

// 4 bf16 <-> fp32 (one 8-byte access)
__device__ __forceinline__ void load4(const uint16_t* p, float (&o)[4]) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  o[0] = bf16_to_f32(v.x & 0xffffu);
  o[1] = bf16_to_f32(v.x >> 16);
  o[2] = bf16_to_f32(v.y & 0xffffu);
  o[3] = bf16_to_f32(v.y >> 16);
}
__device__ __forceinline__ void store4(uint16_t* p, const float (&o)[4]) {
  uint2 v;
  v.x = static_cast<uint32_t>(f32_to_bf16(o[0])) | (static_cast<uint32_t>(f32_to_bf16(o[1])) << 16);
  v.y = static_cast<uint32_t>(f32_to_bf16(o[2])) | (static_cast<uint32_t>(f32_to_bf16(o[3])) << 16);
  *reinterpret_cast<uint2*>(p) = v;
}

// ------------------------------------------------------------------- RoPE
// HF rotate-half rotary embedding on x [rows = B*T, H, D] (row r is position
// r % T) with cos/sin tables [T, D]; one rounding per output instead of
// ATen's slice / neg / cat / 2 mul / add chain.  inverse = the transpose
// rotation (the backward).  Thread = 4 consecutive dims of the first half and
// their partners in the second half.
// x and y may be the same buffer (rope_ in place): each thread reads its
// rotate-half pair before writing it, so x / y are not __restrict__
__global__ void __launch_bounds__(256) rope_kernel(const uint16_t* x, const uint16_t* __restrict__ cs,
                                                  const uint16_t* __restrict__ sn, uint16_t* y,
                                                  int64_t rows, int T, int H, int D, bool inverse, int64_t x_ld,
                                                  int64_t y_ld) {
  const int hd = D / 2, q = hd / 4;  // quads per half
  const int64_t n = rows * H * q;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int d0 = static_cast<int>(i % q) * 4;
    const int64_t rh = i / q;  // row * H + head
    const int64_t row = rh / H;
    const int t = static_cast<int>(row % T);
    const int64_t o = row * x_ld + (rh % H) * D;   // token rows may be strided (slices of a fused
    const int64_t oy = row * y_ld + (rh % H) * D;  // q|k|v projection output / input gradient)
    float a[4], b[4], ca[4], cb[4], sa[4], sb[4], oa[4], ob[4];
    load4(x + o + d0, a);
    load4(x + o + hd + d0, b);
    load4(cs + static_cast<int64_t>(t) * D + d0, ca);
    load4(cs + static_cast<int64_t>(t) * D + hd + d0, cb);
    load4(sn + static_cast<int64_t>(t) * D + d0, sa);
    load4(sn + static_cast<int64_t>(t) * D + hd + d0, sb);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!inverse) {
        oa[j] = a[j] * ca[j] - b[j] * sa[j];
        ob[j] = b[j] * cb[j] + a[j] * sb[j];
      } else {
        oa[j] = a[j] * ca[j] + b[j] * sb[j];
        ob[j] = b[j] * cb[j] - a[j] * sa[j];
      }
    }
    store4(y + oy + d0, oa);
    store4(y + oy + hd + d0, ob);
  }
}

// Tall stacks (S in the hundreds/thousands, n a few thousand: the per-block /
// per-wave partials of the norm and bias-GELU backward kernels).  Block = 8
// float4 column quads x 32 row lanes; each thread strides the rows by 32 and
// the 32 row lanes are folded through LDS.  128-byte row segments per load.
constexpr int kTallQ = 8, kTallR = 32;
template <bool ACC>
__global__ void __launch_bounds__(kTallQ * kTallR) sum_partials_tall_kernel(const float* __restrict__ part, int S,
                                                                           int64_t n, int64_t ld,
                                                                           uint16_t* __restrict__ out,
                                                                           const float* __restrict__ scale) {
  __shared__ float4 red[kTallR][kTallQ];
  const int q = threadIdx.x % kTallQ, r = threadIdx.x / kTallQ;
  const int64_t col4 = static_cast<int64_t>(blockIdx.x) * kTallQ + q;  // float4 column index
  const int64_t n4 = n / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col4 < n4) {
    const float4* p = reinterpret_cast<const float4*>(part) + col4;
    for (int s = r; s < S; s += kTallR) {
      const float4 v = p[static_cast<int64_t>(s) * (ld / 4)];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[r][q] = acc;
  __syncthreads();
  if (r == 0 && col4 < n4) {
#pragma unroll 8
    for (int i = 1; i < kTallR; ++i) {
      const float4 v = red[i][q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (scale) {
      const float sc = scale[0];
      acc.x *= sc; acc.y *= sc; acc.z *= sc; acc.w *= sc;
    }
    if constexpr (ACC) {
      const uint2 o = reinterpret_cast<const uint2*>(out)[col4];
      acc.x += bf16_to_f32(o.x & 0xffffu);
      acc.y += bf16_to_f32(o.x >> 16);
      acc.z += bf16_to_f32(o.y & 0xffffu);
      acc.w += bf16_to_f32(o.y >> 16);
    }
    uint2 w;
    w.x = static_cast<uint32_t>(f32_to_bf16(acc.x)) | (static_cast<uint32_t>(f32_to_bf16(acc.y)) << 16);
    w.y = static_cast<uint32_t>(f32_to_bf16(acc.z)) | (static_cast<uint32_t>(f32_to_bf16(acc.w)) << 16);
    reinterpret_cast<uint2*>(out)[col4] = w;
  }
}

// The tall reduction over up to kMaxPartSeg separately allocated stacks (the
// per-micro-batch partials a fusion window keeps): no concatenation copy.
constexpr int kMaxPartSeg = 16;
struct PartSegs {
  const float* ptr[kMaxPartSeg];
  int64_t rows[kMaxPartSeg];
  int64_t ld4[kMaxPartSeg];  // row stride in float4 units
  int nseg;
};
template <bool ACC>
__global__ void __launch_bounds__(kTallQ * kTallR) sum_partials_multi_kernel(const PartSegs sg, int64_t n,
                                                                            uint16_t* __restrict__ out) {
  __shared__ float4 red[kTallR][kTallQ];
  const int q = threadIdx.x % kTallQ, r = threadIdx.x / kTallQ;
  const int64_t col4 = static_cast<int64_t>(blockIdx.x) * kTallQ + q;
  const int64_t n4 = n / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col4 < n4) {
    for (int k = 0; k < sg.nseg; ++k) {
      const float4* p = reinterpret_cast<const float4*>(sg.ptr[k]) + col4;
      for (int64_t s = r; s < sg.rows[k]; s += kTallR) {
        const float4 v = p[s * sg.ld4[k]];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
  }
  red[r][q] = acc;
  __syncthreads();
  if (r == 0 && col4 < n4) {
#pragma unroll 8
    for (int i = 1; i < kTallR; ++i) {
      const float4 v = red[i][q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if constexpr (ACC) {
      const uint2 o = reinterpret_cast<const uint2*>(out)[col4];
      acc.x += bf16_to_f32(o.x & 0xffffu);
      acc.y += bf16_to_f32(o.x >> 16);
      acc.z += bf16_to_f32(o.y & 0xffffu);
      acc.w += bf16_to_f32(o.y >> 16);
    }
    uint2 w;
    w.x = static_cast<uint32_t>(f32_to_bf16(acc.x)) | (static_cast<uint32_t>(f32_to_bf16(acc.y)) << 16);
    w.y = static_cast<uint32_t>(f32_to_bf16(acc.z)) | (static_cast<uint32_t>(f32_to_bf16(acc.w)) << 16);
    reinterpret_cast<uint2*>(out)[col4] = w;
  }
}

// Pass 1 of the row-split tall reduction: with only n/32 column blocks (GPT-2's
// 768..3072-wide bias / norm partial stacks: 24-96 blocks, one CU each, 0.4-1.3
// TB/s) the rows are also split over gridDim.y: block (x, y) sums the kTallR-row
// groups y, y + Y, ... of every segment into scratch[y] (fp32); pass 2 is the
// plain sum_partials kernel over those Y rows (fixed order: deterministic).
__global__ void __launch_bounds__(kTallQ * kTallR) sum_partials_split_kernel(const PartSegs sg, int64_t n,
                                                                            float* __restrict__ scratch) {
  __shared__ float4 red[kTallR][kTallQ];
  const int q = threadIdx.x % kTallQ, r = threadIdx.x / kTallQ;
  const int64_t col4 = static_cast<int64_t>(blockIdx.x) * kTallQ + q;
  const int64_t n4 = n / 4;
  const int64_t step = static_cast<int64_t>(kTallR) * gridDim.y;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col4 < n4) {
    for (int k = 0; k < sg.nseg; ++k) {
      const float4* p = reinterpret_cast<const float4*>(sg.ptr[k]) + col4;
      for (int64_t s = static_cast<int64_t>(blockIdx.y) * kTallR + r; s < sg.rows[k]; s += step) {
        const float4 v = p[s * sg.ld4[k]];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
  }
  red[r][q] = acc;
  __syncthreads();
  if (r == 0 && col4 < n4) {
#pragma unroll 8
    for (int i = 1; i < kTallR; ++i) {
      const float4 v = red[i][q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(scratch + static_cast<int64_t>(blockIdx.y) * n)[col4] = acc;
  }
}

// out [C, Rp] = x[R, C]^T, columns R..Rp-1 zero (the per-step transposed / vocab-padded weight
// copies of the GPT-2 step: ATen's strided copy ran them at 0.2-0.6 TB/s).  64 x 64 tile per
// 256-thread block through LDS: 16-byte row loads, 2-byte LDS column reads (row pitch 66
// elements = 33 dwords: the 8 rows a lane gathers fall in distinct banks), 16-byte stores.
__global__ void __launch_bounds__(256) transpose_pad_kernel(const uint16_t* __restrict__ x, int64_t R, int64_t C,
                                                            int64_t ldx, uint16_t* __restrict__ out, int64_t Rp) {
  __shared__ uint16_t tile[64][66];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * 64, c0 = static_cast<int64_t>(blockIdx.x) * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + h * 256;  // 512 chunks of 8 elements: 64 rows x 8 chunks
    const int tr = idx >> 3, tc = (idx & 7) * 8;
    const int64_t r = r0 + tr, c = c0 + tc;
    uint16_t v[8];
    if (r < R && c + 8 <= C) {
      const uint4 w = *reinterpret_cast<const uint4*>(x + r * ldx + c);
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = static_cast<uint16_t>(ws[j] & 0xffffu);
        v[2 * j + 1] = static_cast<uint16_t>(ws[j] >> 16);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (r < R && c + j < C) ? x[r * ldx + c + j] : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[tr][tc + j] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + h * 256;  // out tile: 64 rows (x columns) x 8 chunks (x rows)
    const int oc = idx >> 3, orr = (idx & 7) * 8;
    const int64_t row = c0 + oc, col = r0 + orr;
    if (row >= C || col >= Rp) continue;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = static_cast<uint32_t>(tile[orr + 2 * j][oc]) | (static_cast<uint32_t>(tile[orr + 2 * j + 1][oc]) << 16);
    *reinterpret_cast<uint4*>(out + row * Rp + col) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

static inline int grid_for(int64_t work, int64_t per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g > 2048) g = 2048;
  return static_cast<int>(g < 1 ? 1 : g);
}

hipError_t launch_bias_gelu_fwd(const void* z, const void* b, void* h, int64_t rows, int N, bool exact,
                                hipStream_t st) {
  if (N % 8 != 0) return hipErrorInvalidValue;
  const int g = grid_for(rows * (N / 8), 256);
  auto Z = static_cast<const uint16_t*>(z);
  auto B = static_cast<const uint16_t*>(b);
  auto H = static_cast<uint16_t*>(h);
  if (exact) hipLaunchKernelGGL((bias_gelu_fwd_kernel<true>), dim3(g), dim3(256), 0, st, Z, B, H, rows, N);
  else hipLaunchKernelGGL((bias_gelu_fwd_kernel<false>), dim3(g), dim3(256), 0, st, Z, B, H, rows, N);
  return hipGetLastError();
}

hipError_t launch_bias_gelu_bwd(const void* dh, const void* z, const void* b, void* dz, float* dbpart, int parts,
                                int64_t rows, int N, bool exact, hipStream_t st) {
  if (N % 8 != 0) return hipErrorInvalidValue;
  // one thread per 8-column group of a row (block up to 1024 threads), NC
  // groups per thread beyond that; each block walks rows with stride `parts`
  const int groups = N / 8;
  const int bd = groups <= 1024 ? (groups + 63) / 64 * 64 : 1024;
  const int nc = (groups + bd - 1) / bd;
  auto DH = static_cast<const uint16_t*>(dh);
  auto Z = static_cast<const uint16_t*>(z);
  auto B = static_cast<const uint16_t*>(b);
  auto DZ = static_cast<uint16_t*>(dz);
#define GELU_BWD(NCV)                                                                                        \
  if (exact) hipLaunchKernelGGL((bias_gelu_bwd_kernel<true, NCV>), dim3(parts), dim3(bd), 0, st, DH, Z, B, DZ, \
                                dbpart, rows, N);                                                            \
  else hipLaunchKernelGGL((bias_gelu_bwd_kernel<false, NCV>), dim3(parts), dim3(bd), 0, st, DH, Z, B, DZ,    \
                          dbpart, rows, N);
  switch (nc) {
    case 1: GELU_BWD(1) break;
    case 2: GELU_BWD(2) break;
    default: return hipErrorInvalidValue;  // N <= 16384
  }
#undef GELU_BWD
  return hipGetLastError();
}

hipError_t launch_colsum(const void* x, float* part, int parts, int64_t rows, int N, hipStream_t st) {
  if (N % 8 != 0) return hipErrorInvalidValue;
  const int groups = N / 8;
  const int bd = groups <= 1024 ? (groups + 63) / 64 * 64 : 1024;
  const int nc = (groups + bd - 1) / bd;
  auto X = static_cast<const uint16_t*>(x);
  switch (nc) {
    case 1: hipLaunchKernelGGL(colsum_kernel<1>, dim3(parts), dim3(bd), 0, st, X, part, rows, N); break;
    case 2: hipLaunchKernelGGL(colsum_kernel<2>, dim3(parts), dim3(bd), 0, st, X, part, rows, N); break;
    default: return hipErrorInvalidValue;  // N <= 16384
  }
  return hipGetLastError();
}

hipError_t launch_swiglu_fwd(const void* g, const void* u, void* h, int64_t rows, int64_t F, int64_t ld_in,
                             hipStream_t st) {
  if (F % 8 != 0 || ld_in % 8 != 0) return hipErrorInvalidValue;
  const int64_t n8 = rows * F / 8;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(n8, 256)), dim3(256), 0, st, static_cast<const uint16_t*>(g),
                     static_cast<const uint16_t*>(u), static_cast<uint16_t*>(h), n8, F / 8, ld_in);
  return hipGetLastError();
}

hipError_t launch_swiglu_fwd_t(const void* g, const void* u, void* h, void* ht, int64_t rows, int64_t F,
                               int64_t ld_in, hipStream_t st) {
  if (rows % 64 != 0 || F % 64 != 0 || ld_in % 8 != 0 || rows / 64 > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_fwd_t_kernel, dim3(static_cast<unsigned>(F / 64), static_cast<unsigned>(rows / 64)),
                     dim3(256), 0, st, static_cast<const uint16_t*>(g), static_cast<const uint16_t*>(u),
                     static_cast<uint16_t*>(h), static_cast<uint16_t*>(ht), F, ld_in, rows);
  return hipGetLastError();
}

hipError_t launch_swiglu_bwd_t(const void* dh, const void* g, const void* u, void* dgu, void* dgut, int64_t rows,
                               int64_t F, int64_t ld_in, hipStream_t st) {
  if (rows % 64 != 0 || F % 64 != 0 || ld_in % 8 != 0 || rows / 64 > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_bwd_t_kernel, dim3(static_cast<unsigned>(F / 64), static_cast<unsigned>(rows / 64)),
                     dim3(256), 0, st, static_cast<const uint16_t*>(dh), static_cast<const uint16_t*>(g),
                     static_cast<const uint16_t*>(u), static_cast<uint16_t*>(dgu), static_cast<uint16_t*>(dgut), F,
                     ld_in, rows);
  return hipGetLastError();
}

hipError_t launch_swiglu_bwd(const void* dh, const void* g, const void* u, void* dg, void* du, int64_t rows,
                             int64_t F, int64_t ld_in, int64_t ld_out, hipStream_t st) {
  if (F % 8 != 0 || ld_in % 8 != 0 || ld_out % 8 != 0) return hipErrorInvalidValue;
  const int64_t n8 = rows * F / 8;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(n8, 256)), dim3(256), 0, st, static_cast<const uint16_t*>(dh),
                     static_cast<const uint16_t*>(g), static_cast<const uint16_t*>(u), static_cast<uint16_t*>(dg),
                     static_cast<uint16_t*>(du), n8, F / 8, ld_in, ld_out);
  return hipGetLastError();
}

hipError_t launch_rope(const void* x, const void* cos, const void* sin, void* y, int64_t rows, int T, int H, int D,
                       bool inverse, int64_t x_ld, int64_t y_ld, hipStream_t st) {
  if (D % 8 != 0 || T <= 0 || x_ld % 4 != 0 || y_ld % 4 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(rows * H * (D / 8), 256)), dim3(256), 0, st,
                     static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(cos),
                     static_cast<const uint16_t*>(sin), static_cast<uint16_t*>(y), rows, T, H, D, inverse, x_ld, y_ld);
  return hipGetLastError();
}

hipError_t launch_sum_partials(const float* part, int S, int64_t n, int64_t ld, void* out, bool accumulate,
                               hipStream_t st, const float* scale) {
  if (n % 4 != 0 || ld % 4 != 0 || ld < n) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  auto O = static_cast<uint16_t*>(out);
  if (S > 64 || n4 < 256 * static_cast<int64_t>(S)) {
    // tall / narrow stack: parallelise over rows too
    const int64_t blocks = (n4 + kTallQ - 1) / kTallQ;
    if (blocks > 0x7fffffff) return hipErrorInvalidValue;
    const dim3 g(static_cast<unsigned>(blocks)), blk(kTallQ * kTallR);
    if (accumulate) hipLaunchKernelGGL(sum_partials_tall_kernel<true>, g, blk, 0, st, part, S, n, ld, O, scale);
    else hipLaunchKernelGGL(sum_partials_tall_kernel<false>, g, blk, 0, st, part, S, n, ld, O, scale);
    return hipGetLastError();
  }
  const dim3 g(grid_for(n / 4, 256)), blk(256);
  if (accumulate) hipLaunchKernelGGL(sum_partials_kernel<true>, g, blk, 0, st, part, S, n, ld, O, scale);
  else hipLaunchKernelGGL(sum_partials_kernel<false>, g, blk, 0, st, part, S, n, ld, O, scale);
  return hipGetLastError();
}

hipError_t launch_sum_partials_multi(const float* const* ptrs, const int64_t* rows, const int64_t* lds, int nseg,
                                     int64_t n, void* out, bool accumulate, hipStream_t st) {
  if (nseg < 1 || nseg > kMaxPartSeg || n % 4 != 0) return hipErrorInvalidValue;
  PartSegs sg{};
  for (int k = 0; k < nseg; ++k) {
    if (lds[k] % 4 != 0 || lds[k] < n || reinterpret_cast<uintptr_t>(ptrs[k]) % 16 != 0) return hipErrorInvalidValue;
    sg.ptr[k] = ptrs[k];
    sg.rows[k] = rows[k];
    sg.ld4[k] = lds[k] / 4;
  }
  sg.nseg = nseg;
  const int64_t blocks = (n / 4 + kTallQ - 1) / kTallQ;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 g(static_cast<unsigned>(blocks)), blk(kTallQ * kTallR);
  auto O = static_cast<uint16_t*>(out);
  if (accumulate) hipLaunchKernelGGL(sum_partials_multi_kernel<true>, g, blk, 0, st, sg, n, O);
  else hipLaunchKernelGGL(sum_partials_multi_kernel<false>, g, blk, 0, st, sg, n, O);
  return hipGetLastError();
}

hipError_t launch_transpose_pad(const void* x, int64_t R, int64_t C, int64_t ldx, void* out, int64_t Rp,
                                hipStream_t st) {
  if (R <= 0 || C <= 0) return hipSuccess;
  if (Rp < R || Rp % 8 != 0 || ldx % 8 != 0 || ldx < C || reinterpret_cast<uintptr_t>(x) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(out) % 16 != 0)
    return hipErrorInvalidValue;
  const int64_t gx = (C + 63) / 64, gy = (Rp + 63) / 64;
  if (gx > 0x7fffffff || gy > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_pad_kernel, dim3(static_cast<unsigned>(gx), static_cast<unsigned>(gy)), dim3(256), 0, st,
                     static_cast<const uint16_t*>(x), R, C, ldx, static_cast<uint16_t*>(out), Rp);
  return hipGetLastError();
}

int sum_partials_split_factor(int64_t n, int64_t total_rows) {
  const int64_t col_blocks = (n / 4 + kTallQ - 1) / kTallQ;
  if (col_blocks >= 256 || total_rows < 4 * kTallR) return 1;
  int64_t y = (512 + col_blocks - 1) / col_blocks;  // ~2 blocks per CU
  y = y < total_rows / (2 * kTallR) ? y : total_rows / (2 * kTallR);
  y = y < 64 ? y : 64;
  return static_cast<int>(y < 1 ? 1 : y);
}

hipError_t launch_sum_partials_split(const float* const* ptrs, const int64_t* rows, const int64_t* lds, int nseg,
                                     int64_t n, int Y, float* scratch, void* out, bool accumulate, const float* scale,
                                     hipStream_t st) {
  if (nseg < 1 || nseg > kMaxPartSeg || n % 4 != 0 || Y < 1 || reinterpret_cast<uintptr_t>(scratch) % 16 != 0)
    return hipErrorInvalidValue;
  PartSegs sg{};
  for (int k = 0; k < nseg; ++k) {
    if (lds[k] % 4 != 0 || lds[k] < n || reinterpret_cast<uintptr_t>(ptrs[k]) % 16 != 0) return hipErrorInvalidValue;
    sg.ptr[k] = ptrs[k];
    sg.rows[k] = rows[k];
    sg.ld4[k] = lds[k] / 4;
  }
  sg.nseg = nseg;
  const int64_t blocks = (n / 4 + kTallQ - 1) / kTallQ;
  if (blocks > 0x7fffffff || Y > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sum_partials_split_kernel, dim3(static_cast<unsigned>(blocks), static_cast<unsigned>(Y)),
                     dim3(kTallQ * kTallR), 0, st, sg, n, scratch);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  auto O = static_cast<uint16_t*>(out);
  const dim3 g(grid_for(n / 4, 256)), blk(256);
  if (accumulate) hipLaunchKernelGGL(sum_partials_kernel<true>, g, blk, 0, st, scratch, Y, n, n, O, scale);
  else hipLaunchKernelGGL(sum_partials_kernel<false>, g, blk, 0, st, scratch, Y, n, n, O, scale);
  return hipGetLastError();
}

}  // namespace dlion

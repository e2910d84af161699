// Shared device helpers for the gfx950 (CDNA4) kernels of distributed_lion_pytorch_amd.
//
// Everything here is written for a 64-lane wavefront and 16-byte-per-lane
// vector memory access (cdna_hip_programming.md Guideline 13): bf16/fp16 are
// moved as uint4 (8 elements), fp32 as two float4.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dlion {

// dtype codes shared with the Python side (ops/hip.py::DTYPE_CODE)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

// ---------------------------------------------------------------- conversions
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

// round-to-nearest-even, NaN preserved (quietened) -- identical to ATen's
// c10::BFloat16 round_to_nearest_even so that bf16 results are bit-exact with
// the PyTorch reference path.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  return static_cast<float>(__builtin_bit_cast(_Float16, h));
}
// Integer round-to-nearest-even f32 -> f16.  Deliberately not
// static_cast<_Float16>: hipcc is free to fold a (float)(half)x round trip
// into mixed-precision FMAs, which broke bit-parity with ATen (measured:
// tools/probe_fp16.py, 476 / 300k momentum mismatches).
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  const uint32_t x = __float_as_uint(f);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7fffffffu;
  if (ax > 0x7f800000u) return static_cast<uint16_t>(sign | 0x7e00u);  // NaN
  if (ax >= 0x47800000u) return static_cast<uint16_t>(sign | 0x7c00u);  // >= 2^16 (and inf) -> inf
  if (ax < 0x33000000u) return static_cast<uint16_t>(sign);             // < 2^-25 -> 0
  const uint32_t e = ax >> 23;
  uint32_t h, rem, halfway;
  if (e >= 113) {  // normal half
    h = ((e - 112) << 10) | ((ax & 0x7fffffu) >> 13);
    rem = ax & 0x1fffu;
    halfway = 0x1000u;
  } else {  // subnormal half: round(mant24 * 2^(e - 126))
    const uint32_t mant = (ax & 0x7fffffu) | 0x800000u;
    const uint32_t shift = 126 - e;  // 14..24
    h = mant >> shift;
    rem = mant & ((1u << shift) - 1u);
    halfway = 1u << (shift - 1u);
  }
  if (rem > halfway || (rem == halfway && (h & 1u))) ++h;  // carry into the exponent is correct
  return static_cast<uint16_t>(sign | h);
}

// Element traits: storage type, load/store of 8 consecutive elements.
template <int DT> struct Elem;

template <> struct Elem<kF32> {
  using S = float;
  __device__ __forceinline__ static float to_f(S v) { return v; }
  __device__ __forceinline__ static S from_f(float v) { return v; }
  __device__ __forceinline__ static void load8(const S* p, float (&o)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  __device__ __forceinline__ static void store8(S* p, const float (&o)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
  // round-trip through storage precision (identity for f32)
  __device__ __forceinline__ static float rnd(float v) { return v; }
};

template <int DT> struct Elem16 {
  using S = uint16_t;
  __device__ __forceinline__ static float to_f(S v) {
    return DT == kBF16 ? bf16_to_f32(v) : f16_to_f32(v);
  }
  __device__ __forceinline__ static S from_f(float v) {
    return DT == kBF16 ? f32_to_bf16(v) : f32_to_f16(v);
  }
  __device__ __forceinline__ static void load8(const S* p, float (&o)[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = to_f(static_cast<S>(w[i] & 0xffffu));
      o[2 * i + 1] = to_f(static_cast<S>(w[i] >> 16));
    }
  }
  __device__ __forceinline__ static void store8(S* p, const float (&o)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = static_cast<uint32_t>(from_f(o[2 * i])) |
             (static_cast<uint32_t>(from_f(o[2 * i + 1])) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ __forceinline__ static float rnd(float v) { return to_f(from_f(v)); }
};
template <> struct Elem<kBF16> : Elem16<kBF16> {};
template <> struct Elem<kF16> : Elem16<kF16> {};

// Load / store 8 elements starting at element e of a tensor with n elements.
// `vec` says the tensor base is 16-B aligned and n % 8 == 0, so the fast path
// is one (bf16) or two (f32) dwordx4 per lane; otherwise a guarded scalar path.
template <int DT>
__device__ __forceinline__ void load8g(const typename Elem<DT>::S* base, int64_t e, int64_t n,
                                       bool vec, float (&o)[8]) {
  if (vec) {
    Elem<DT>::load8(base + e, o);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (e + j < n) ? Elem<DT>::to_f(base[e + j]) : 0.f;
  }
}
template <int DT>
__device__ __forceinline__ void store8g(typename Elem<DT>::S* base, int64_t e, int64_t n, bool vec,
                                        const float (&o)[8]) {
  if (vec) {
    Elem<DT>::store8(base + e, o);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (e + j < n) base[e + j] = Elem<DT>::from_f(o[j]);
  }
}

// ------------------------------------------------------- wave reductions
// Full-wave fp32 sum / max, the result in every lane, without LDS: two
// quad_perm DPP ops and two row_ror DPP ops leave each 16-lane row's result in
// its lanes; the four row results are read with v_readlane and combined
// (wave-uniform).  __shfl_xor lowers to six dependent ds_bpermute round trips.
// (Recombining rows with the permlane16/32 swap builtins on identical operands
// came out of hipcc as r[0] op r[0] in one kernel -- wrong -- so no swaps.)
template <bool MAX>
__device__ __forceinline__ float dpp_step(float v, int sel) {
  const int x = __builtin_bit_cast(int, v);
  int y;
  switch (sel) {  // the DPP control must be an immediate
    case 0: y = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false); break;   // quad_perm [1,0,3,2]
    case 1: y = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false); break;   // quad_perm [2,3,0,1]
    case 2: y = __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false); break;  // row_ror:4
    default: y = __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false); break; // row_ror:8
  }
  const float o = __builtin_bit_cast(float, y);
  return MAX ? fmaxf(v, o) : v + o;
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce_dpp(float v) {
  v = dpp_step<MAX>(v, 0);
  v = dpp_step<MAX>(v, 1);
  v = dpp_step<MAX>(v, 2);
  v = dpp_step<MAX>(v, 3);
  const int x = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 48));
  return MAX ? fmaxf(fmaxf(r0, r1), fmaxf(r2, r3)) : (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ float wave_sum_dpp(float v) { return wave_reduce_dpp<false>(v); }
__device__ __forceinline__ float wave_max_dpp(float v) { return wave_reduce_dpp<true>(v); }

// ------------------------------------------------------------------- GELU
// tanh via one v_exp_f32 + one v_rcp_f32 (libm tanhf is a ~30-instruction
// polynomial path and made the memory-bound bias+GELU kernels VALU-bound);
// |err| ~1e-7, far below the bf16 output rounding.  Saturates correctly.
__device__ __forceinline__ float fast_tanh(float a) {
  const float e = __builtin_amdgcn_exp2f(a * 2.8853900817779268f);  // exp(2a)
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}
constexpr float kSqrt2OverPi = 0.7978845608028654f;
constexpr float kKappa = 0.044715f;
constexpr float kInvSqrt2 = 0.7071067811865476f;
constexpr float kInvSqrt2Pi = 0.3989422804014327f;
constexpr float kLog2e = 1.4426950408889634f;
// tanh-approximate GELU in its sigmoid form: 0.5 u (1 + tanh y) = u s with
// s = 1 / (1 + exp(-2y)), y = sqrt(2/pi) (u + kappa u^3); the exponent's
// constants fold into one FMA on u^2.  Saturates correctly (exp2 -> inf: s = 0).
__device__ __forceinline__ float gelu_sig(float u, float u2) {
  const float a = u * __builtin_fmaf(u2, -2.f * kSqrt2OverPi * kKappa * kLog2e, -2.f * kSqrt2OverPi * kLog2e);
  return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(a) + 1.f);
}
// GELU: exact = erf form (nn.GELU()), else the tanh approximation (gelu_new).
// Shared by the bias+GELU kernels and the GEMM epilogues (bitwise-identical).
__device__ __forceinline__ float gelu_f(float u, bool exact) {
  if (exact) return 0.5f * u * (1.f + erff(u * 0.7071067811865476f));
  return u * gelu_sig(u, u * u);
}

// d gelu(u) / du, matching gelu_f (shared by the bias+GELU backward kernel and
// the GEMM's DGELU epilogue): s + 2k u s (1 - s) (1 + 3 kappa u^2)
__device__ __forceinline__ float gelu_grad(float u, bool exact) {
  if (exact) return 0.5f * (1.f + erff(u * kInvSqrt2)) + u * kInvSqrt2Pi * __expf(-0.5f * u * u);
  const float u2 = u * u;
  const float s = gelu_sig(u, u2);
  const float q = u * __builtin_fmaf(u2, 6.f * kSqrt2OverPi * kKappa, 2.f * kSqrt2OverPi);
  return __builtin_fmaf(q, __builtin_fmaf(-s, s, s), s);
}

// gelu(u) and gelu'(u) from one exp / rcp (or erf): the GEMM's GELU epilogue
// that stores the derivative for the backward instead of the pre-activation
// (8 VALU + 2 transcendental per element; the tanh form took ~17 + 2)
__device__ __forceinline__ void gelu_and_grad(float u, bool exact, float& g, float& dg) {
  if (exact) {
    const float e = erff(u * kInvSqrt2);
    g = 0.5f * u * (1.f + e);
    dg = 0.5f * (1.f + e) + u * kInvSqrt2Pi * __expf(-0.5f * u * u);
    return;
  }
  const float u2 = u * u;
  const float s = gelu_sig(u, u2);
  g = u * s;
  const float q = u * __builtin_fmaf(u2, 6.f * kSqrt2OverPi * kKappa, 2.f * kSqrt2OverPi);
  dg = __builtin_fmaf(q, __builtin_fmaf(-s, s, s), s);
}

// ------------------------------------------------------------ vote counting
// Spread the 8 bits of a byte into the 8 bytes of a u64 (bit j -> bit 8j), so
// that summing spread bytes over W <= 255 ranks counts 8 votes in parallel.
__device__ __forceinline__ uint64_t spread8(uint32_t b) {
  uint64_t x = b & 0xffu;
  x = (x | (x << 28)) & 0x0000000F0000000FULL;
  x = (x | (x << 14)) & 0x0003000300030003ULL;
  x = (x | (x << 7)) & 0x0101010101010101ULL;
  return x;
}

// ------------------------------------------------------- dropout keep hash
// Stateless dropout mask shared by the norm and embedding kernels (and
// ops/fused.norm_dropout_keep on the host): element e of a flat index space
// keeps iff 16 bits of mix32(seed ^ (e >> 1) * golden ^ (e >> 33)) >= thresh16.
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
// keep bits for 8 consecutive elements (idx % 8 == 0); all kept when thresh16 == 0
__device__ __forceinline__ uint32_t keep8(uint32_t seed, uint64_t idx, uint32_t thresh16) {
  if (!thresh16) return 0xffu;
  return keep4(seed, idx, thresh16) | (keep4(seed, idx + 4, thresh16) << 4);
}

// ------------------------------------------------------------- Philox4x32-10
// Counter-based RNG for the stochastic-binarization encoder: every
// (seed, element, step) triple gets an independent, reproducible draw.
__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}
__device__ __forceinline__ float u32_to_unit(uint32_t x) {
  return static_cast<float>(x >> 8) * (1.0f / 16777216.0f);  // [0, 1)
}

}  // namespace dlion

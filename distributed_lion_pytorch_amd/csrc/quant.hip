// 4-bit blockwise weight quantization for frozen base models (gfx950).
//
// The reference loads its Llama-2-7B SFT / DPO base models through
// bitsandbytes 4-bit NF4 (/root/reference/sft_llama2.py:141-149:
// load_in_4bit, bnb_4bit_quant_type="nf4", compute dtype bf16;
// dpo_llama2.py:133-152, policy + reference model, fp16).  Format kept here:
// the weight is flattened row-major, cut into 64-element blocks, each block
// stores its fp32 absmax and 64 4-bit indices into a 16-entry codebook
// (NF4 or FP4, ops/quant.py), two indices per byte with the FIRST element in
// the HIGH nibble.  w ~= code[idx] * absmax.
//
// The frozen weight is only ever read by GEMMs, so the 4-bit copy is expanded
// right before use into a transient compute-dtype buffer (forward GEMM, and
// again for the input-gradient GEMM in backward) and dropped after: the
// replica keeps 0.5 B/param (+ 1/16 B/param of absmax) resident instead of
// 2 B/param.  The expansion is a pure HBM stream -- 0.5 B in, 2 B out per
// element -- so the kernel is shaped for bandwidth: lane-contiguous dword
// loads and 16-byte stores (dequant4_kernel), and the per-nibble codebook
// lookup is one ds_read_b64 per byte from a 256-entry LDS table of
// (code[hi], code[lo]) pairs.
#include "common.h"

namespace dlion {

namespace {

constexpr int kQBlock = 64;  // elements per absmax block
constexpr int kThreads = 256;

// 8 consecutive outputs (one packed dword) as the compute dtype: one 16-byte store
// (two for fp32)
template <int DT>
__device__ __forceinline__ void store8q(typename Elem<DT>::S* p, const float (&o)[8]);

template <>
__device__ __forceinline__ void store8q<kBF16>(uint16_t* p, const float (&o)[8]) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = static_cast<__bf16>(o[j]);  // v_cvt_pk_bf16_f32 (RNE)
  *reinterpret_cast<bf16x8*>(p) = b;
}

template <>
__device__ __forceinline__ void store8q<kF16>(uint16_t* p, const float (&o)[8]) {
  Elem<kF16>::store8(p, o);
}

template <>
__device__ __forceinline__ void store8q<kF32>(float* p, const float (&o)[8]) {
  Elem<kF32>::store8(p, o);
}

// A lane expands one packed dword (8 elements) per unrolled step; the block's
// 256 lanes take 256 consecutive dwords per step, so every load instruction
// reads 256 contiguous bytes per wave and every store writes 1 KB contiguous
// (bf16) -- full cache lines, no partial-line write merging.  kU steps are
// issued load-first so each lane has kU dword loads in flight.
constexpr int kU = 4;

template <int DT>
__global__ __launch_bounds__(kThreads) void dequant4_kernel(const uint32_t* __restrict__ q,
                                                            const float* __restrict__ absmax,
                                                            const float* __restrict__ code,
                                                            typename Elem<DT>::S* __restrict__ out, int64_t words) {
  __shared__ float2 tab[256];
  tab[threadIdx.x] = make_float2(code[threadIdx.x >> 4], code[threadIdx.x & 15]);
  __syncthreads();
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads * kU;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kThreads * kU + threadIdx.x; base < words; base += step) {
    uint32_t w[kU];
    float s[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = base + u * kThreads;
      if (i < words) {
        w[u] = q[i];
        s[u] = absmax[i >> 3];  // 8 dwords = 64 elements per absmax block
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = base + u * kThreads;
      if (i < words) {
        float o[8];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const float2 c = tab[(w[u] >> (8 * b)) & 0xffu];
          o[2 * b] = c.x * s[u];
          o[2 * b + 1] = c.y * s[u];
        }
        store8q<DT>(out + i * 8, o);
      }
    }
  }
}

// Transposed expansion for the input-gradient GEMM (dX = dY . W as the NT
// product against W^T): out[k, n] (row stride ldo) = code[q(n, k)] * absmax,
// for W [N, K] stored as above.  64 (n) x 128 (k) tile per 256-thread block:
// each thread expands one 16-byte load (32 elements of a row; 64 contiguous
// packed bytes per row and tile -- a 64 x 64 tile fetched 32-byte row pieces,
// measured 4.4x the ideal packed-weight traffic) into an LDS tile of 16-bit
// values, then gathers tile columns into 16-byte stores of the transposed rows.
// N % 64 == 0, K % 128 == 0.
template <int DT>
__global__ __launch_bounds__(kThreads) void dequant4_t_kernel(const uint4* __restrict__ q,
                                                              const float* __restrict__ absmax,
                                                              const float* __restrict__ code,
                                                              uint16_t* __restrict__ out, int N, int K, int64_t ldo) {
  __shared__ float2 tab[256];
  __shared__ uint16_t tile[64][130];
  tab[threadIdx.x] = make_float2(code[threadIdx.x >> 4], code[threadIdx.x & 15]);
  __syncthreads();
  const int n0 = blockIdx.y * 64, k0 = blockIdx.x * 128;
  {
    const int nl = threadIdx.x >> 2, part = threadIdx.x & 3;
    const int64_t e = static_cast<int64_t>(n0 + nl) * K + k0 + part * 32;  // first element of the 32
    const uint4 w = q[e / 32];
    const float s = absmax[e / kQBlock];
    const uint32_t words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float2 c = tab[(words[k] >> (8 * b)) & 0xffu];
        const int col = part * 32 + k * 8 + b * 2;
        if constexpr (DT == kBF16) {
          tile[nl][col] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(c.x * s));
          tile[nl][col + 1] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(c.y * s));
        } else {
          tile[nl][col] = f32_to_f16(c.x * s);
          tile[nl][col + 1] = f32_to_f16(c.y * s);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int idx = threadIdx.x + h * kThreads;  // 128 output rows (k) x 8 chunks of 8 n
    const int kl = idx >> 3, nb = (idx & 7) * 8;
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = static_cast<uint32_t>(tile[nb + 2 * j][kl]) | (static_cast<uint32_t>(tile[nb + 2 * j + 1][kl]) << 16);
    *reinterpret_cast<uint4*>(out + static_cast<int64_t>(k0 + kl) * ldo + n0 + nb) = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// One thread per 64-element block: absmax, then the nearest codebook entry
// per element (first minimum on ties, the torch.argmin rule of the oracle).
template <int DT>
__global__ __launch_bounds__(kThreads) void quant4_kernel(const typename Elem<DT>::S* __restrict__ w,
                                                          const float* __restrict__ code, uint4* __restrict__ q,
                                                          float* __restrict__ absmax, int64_t nblocks) {
  __shared__ float cb[16];
  if (threadIdx.x < 16) cb[threadIdx.x] = code[threadIdx.x];
  __syncthreads();
  const int64_t b = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (b >= nblocks) return;
  float v[kQBlock];
#pragma unroll
  for (int j = 0; j < kQBlock / 8; ++j) {
    float t[8];
    Elem<DT>::load8(w + b * kQBlock + j * 8, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[j * 8 + e] = t[e];
  }
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < kQBlock; ++j) m = fmaxf(m, fabsf(v[j]));
  absmax[b] = m;
  uint32_t words[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t word = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = m > 0.f ? v[k * 8 + e] / m : 0.f;
      float best = fabsf(x - cb[0]);
      uint32_t bi = 0;
#pragma unroll
      for (int c = 1; c < 16; ++c) {
        const float d = fabsf(x - cb[c]);
        if (d < best) {
          best = d;
          bi = c;
        }
      }
      // byte (e / 2) of the word: element e even -> high nibble
      word |= bi << (8 * (e >> 1) + ((e & 1) ? 0 : 4));
    }
    words[k] = word;
  }
  q[b * 2] = make_uint4(words[0], words[1], words[2], words[3]);
  q[b * 2 + 1] = make_uint4(words[4], words[5], words[6], words[7]);
}

}  // namespace

hipError_t launch_dequant4(int dt, const uint8_t* q, const float* absmax, const float* code, void* out, int64_t n,
                           hipStream_t st) {
  if (n % kQBlock) return hipErrorInvalidValue;
  const int64_t words = n / 8;
  if (words == 0) return hipSuccess;
  const int64_t want = (words + kThreads * kU - 1) / (kThreads * kU);
  const int grid = static_cast<int>(want < 4096 ? want : 4096);
  const uint32_t* qv = reinterpret_cast<const uint32_t*>(q);
  switch (dt) {
    case kBF16:
      dequant4_kernel<kBF16><<<grid, kThreads, 0, st>>>(qv, absmax, code, static_cast<uint16_t*>(out), words);
      break;
    case kF16:
      dequant4_kernel<kF16><<<grid, kThreads, 0, st>>>(qv, absmax, code, static_cast<uint16_t*>(out), words);
      break;
    case kF32:
      dequant4_kernel<kF32><<<grid, kThreads, 0, st>>>(qv, absmax, code, static_cast<float*>(out), words);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_dequant4_t(int dt, const uint8_t* q, const float* absmax, const float* code, void* out, int N, int K,
                             int64_t ldo, hipStream_t st) {
  if (N <= 0 || K <= 0) return hipSuccess;
  if (N % 64 || K % 128 || ldo < N || ldo % 8 || reinterpret_cast<uintptr_t>(out) % 16 ||
      reinterpret_cast<uintptr_t>(q) % 16)
    return hipErrorInvalidValue;
  const dim3 grid(K / 128, N / 64);
  if (grid.y > 65535) return hipErrorInvalidValue;
  const uint4* qv = reinterpret_cast<const uint4*>(q);
  switch (dt) {
    case kBF16:
      dequant4_t_kernel<kBF16><<<grid, kThreads, 0, st>>>(qv, absmax, code, static_cast<uint16_t*>(out), N, K, ldo);
      break;
    case kF16:
      dequant4_t_kernel<kF16><<<grid, kThreads, 0, st>>>(qv, absmax, code, static_cast<uint16_t*>(out), N, K, ldo);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_quant4(int dt, const void* w, const float* code, uint8_t* q, float* absmax, int64_t n,
                         hipStream_t st) {
  if (n % kQBlock) return hipErrorInvalidValue;
  const int64_t nblocks = n / kQBlock;
  if (nblocks == 0) return hipSuccess;
  const int grid = static_cast<int>((nblocks + kThreads - 1) / kThreads);
  uint4* qv = reinterpret_cast<uint4*>(q);
  switch (dt) {
    case kBF16:
      quant4_kernel<kBF16><<<grid, kThreads, 0, st>>>(static_cast<const uint16_t*>(w), code, qv, absmax, nblocks);
      break;
    case kF16:
      quant4_kernel<kF16><<<grid, kThreads, 0, st>>>(static_cast<const uint16_t*>(w), code, qv, absmax, nblocks);
      break;
    case kF32:
      quant4_kernel<kF32><<<grid, kThreads, 0, st>>>(static_cast<const float*>(w), code, qv, absmax, nblocks);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dlion

// LoRA adapter path for gfx950:  out = o + s * (drop(x) A^T) B^T   (rank r in {8, 16}).
//
// The reference (peft on ATen; /root/reference/sft_llama2.py:44-51) runs the
// adapter as dropout -> Linear(K, r) -> Linear(r, N) -> scale -> add, and the
// same chain backward: a dropout pass that materialises drop(x), two skinny
// hipBLASLt GEMMs each way, full [tokens, N] elementwise passes for the scale
// and the add, then the dropout backward -- ~200 us per adapter per
// Llama-2-7B micro-batch, ~10 % of the LoRA SFT step.  With r = 8 output
// columns the adapter GEMMs are memory-bound streams over x / dout, not MFMA
// work, so here every kernel reads its big operand once, and the dropout mask
// is regenerated from the stateless hash (keep8 of the flat element index,
// common.h) instead of being stored:
//
//   rows (down):    u[t, :]  = drop(x)[t, :] . A^T               reads x
//   up:             out      = o + s * u . B^T                   reads o, writes out
//   rows (bwd u):   du[t, :] = s * dout[t, :] . B                reads dout
//   cols mode 0:    dB       = dout^T u     (fp32 partials)      reads dout
//   cols mode 1:    dA       = du^T drop(x) (fp32 partials),
//                   dx       = drop'(du . A)                    reads x, writes dx
//
// Row kernels: a skinny MFMA GEMM, 16 tokens per 8-wave block, split-K over
// the waves.  Up kernel: a lane owns 8 columns (their B rows in registers)
// over a chunk of rows.  Column kernels: a 4-wave block owns 512 columns over
// a range of rows; the waves split the rows, batch 4 rows of loads at a time,
// and reduce through LDS into one partial per block.  (tools/bench_lora.py
// times each kernel.)
#include <cstdlib>

#include "common.h"

namespace dlion {

__device__ __forceinline__ float lora_wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

typedef __bf16 lora_bf16x8 __attribute__((ext_vector_type(8)));
typedef float lora_f32x4 __attribute__((ext_vector_type(4)));

// out[t, j] = scale * sum_k in'[t, k] * w[j, k], in' = drop(in) when DROP; w [R, K], K % 32 == 0.
// A skinny GEMM on the matrix cores: a block of 8 waves owns 16 rows (tokens);
// wave v takes the 32-wide k-steps v, v + 8, ... and runs one
// v_mfma_f32_16x16x32_bf16 per step with W as the 16-row A operand (rows >= R
// zero) and the 16 tokens as the B operand, so one 16-byte W load per lane
// serves 16 tokens (a VALU dot per token re-reads all of W per row: the
// L2 traffic of that version was 4x the x stream and bounded it at ~1.7 TB/s).
// A lane's 16-byte x load is its operand fragment as is (after the dropout
// scaling, rounded to bf16 like ATen's dropout output); 16 steps of loads (all
// of a wave's share at K = 4096) are issued before the first MFMA.  The 8 per-wave partial tiles meet in LDS.
template <int R, bool DROP>
__global__ void __launch_bounds__(512) lora_rows_kernel(const uint16_t* __restrict__ in, int64_t ldin,
                                                        const uint16_t* __restrict__ w, uint16_t* __restrict__ out,
                                                        int64_t rows, int K, float scale, uint32_t seed,
                                                        uint32_t thresh16, float inv_keep) {
  constexpr int NW = 8, NB = 16;
  __shared__ lora_f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = lane & 15, grp = lane >> 4;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * 16;
  const int64_t row = row0 + j;
  const bool rok = row < rows;
  const bool wok = j < R;
  const uint16_t* xr = in + (rok ? row : 0) * ldin + grp * 8;
  const uint16_t* wr = w + static_cast<int64_t>(wok ? j : 0) * K + grp * 8;
  const int steps = K / 32;
  lora_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s0 = wv; s0 < steps; s0 += NW * NB) {
    uint4 xv[NB], wf[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int st = s0 + b * NW;
      xv[b] = (st < steps && rok) ? *reinterpret_cast<const uint4*>(xr + st * 32) : make_uint4(0u, 0u, 0u, 0u);
      wf[b] = (st < steps && wok) ? *reinterpret_cast<const uint4*>(wr + st * 32) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int st = s0 + b * NW;
      if (st < steps) {  // wave-uniform
        uint4 xx = xv[b];
        if constexpr (DROP) {
          const uint32_t kp = keep8(seed, static_cast<uint64_t>(row) * K + st * 32 + grp * 8, thresh16);
          float f[8];
          Elem<kBF16>::load8(reinterpret_cast<const uint16_t*>(&xx), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = ((kp >> e) & 1u) ? f[e] * inv_keep : 0.f;
          Elem<kBF16>::store8(reinterpret_cast<uint16_t*>(&xx), f);
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(lora_bf16x8, wf[b]),
                                                       __builtin_bit_cast(lora_bf16x8, xx), acc, 0, 0, 0);
      }
    }
  }
  // acc[q] = partial out[row0 + (lane & 15)][(lane >> 4) * 4 + q]
  red[wv][lane] = acc;
  __syncthreads();
  if (threadIdx.x < 256) {
    const int l = threadIdx.x >> 2, q = threadIdx.x & 3;
    float sum = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) sum += red[v][l][q];
    const int tok = l & 15, r = (l >> 4) * 4 + q;
    if (r < R && row0 + tok < rows) out[(row0 + tok) * R + r] = f32_to_bf16(sum * scale);
  }
}

typedef __bf16 lora_bf16x2 __attribute__((ext_vector_type(2)));

// sum_i a.pair[i] * b.pair[i] over R bf16 held as R/2 packed pairs (v_dot2c_f32_bf16)
template <int R>
__device__ __forceinline__ float lora_dot(const uint32_t* a, const uint32_t* b) {
  float d = 0.f;
#pragma unroll
  for (int i = 0; i < R / 2; ++i)
    d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(lora_bf16x2, a[i]), __builtin_bit_cast(lora_bf16x2, b[i]), d,
                                        false);
  return d;
}

__device__ __forceinline__ void lora_ld16(const uint16_t* p, uint32_t* w) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
}

// out[t, n] = o[t, n] + bf16(s * sum_j u[t, j] * b[n, j]); b [N, R]; a thread
// owns 8 columns over `rpt` rows, RB rows per load batch.  B's rows stay
// packed bf16 in registers and the rank-R dot is R/2 v_dot2c_f32_bf16 (109
// VGPRs against 212 with fp32 rows; the time did not move: ~21 us for the
// 64 MB at the SFT shape, where an ATen strided copy takes 12 us -- open).
template <int R, int RB>
__global__ void __launch_bounds__(256) lora_up_kernel(const uint16_t* __restrict__ o, int64_t ldo,
                                                      const uint16_t* __restrict__ u, const uint16_t* __restrict__ b,
                                                      uint16_t* __restrict__ out, int64_t rows, int N, int rpt,
                                                      float s) {
  const int cpr = N / 8;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t chunk = i / cpr;
  const int c = static_cast<int>(i - chunk * cpr) * 8;
  const int64_t t0 = chunk * rpt;
  if (t0 >= rows) return;
  const int64_t t1 = t0 + rpt < rows ? t0 + rpt : rows;
  uint32_t bp[8][R / 2];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int j = 0; j < R; j += 8) lora_ld16(b + static_cast<int64_t>(c + e) * R + j, &bp[e][j / 2]);
  for (int64_t tb = t0; tb < t1; tb += RB) {
    // the batch's o rows stay packed bf16 (4 VGPRs a row) so that all RB
    // 16-byte loads are in flight at once (the kernel is latency-bound: 4 rows
    // per batch ran at 2.4 TB/s)
    uint4 raw[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q)
      if (tb + q < t1) raw[q] = *reinterpret_cast<const uint4*>(o + (tb + q) * ldo + c);
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int64_t t = tb + q;
      if (t < t1) {
        float ov[8];
        Elem<kBF16>::load8(reinterpret_cast<const uint16_t*>(&raw[q]), ov);
        uint32_t up[R / 2];
#pragma unroll
        for (int j = 0; j < R; j += 8) lora_ld16(u + t * R + j, &up[j / 2]);
        lora_bf16x8 ob;
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // + the bf16 adapter output, as the unfused add sees it
          const float a = static_cast<float>(static_cast<__bf16>(lora_dot<R>(bp[e], up) * s));
          ob[e] = static_cast<__bf16>(ov[e] + a);  // v_cvt_pk_bf16_f32 (RNE)
        }
        *reinterpret_cast<lora_bf16x8*>(out + t * N + c) = ob;
      }
    }
  }
}

// part = yscale * (sum over the rows t of range p of y[t, j] * g'(t, n)), written
// [P][N][R] in mode 0 and [P][R][N] in mode 1 -- the layouts of B and A:
//   MODE 0 (dB):  g' = g = dout
//   MODE 1 (dA):  g' = drop(x), and dx[t, n] = drop'(sum_j y[t, j] * a[j, n]) is written on the way
// A lane owns 8 columns (16-byte loads: 8-byte lanes measured 1.6x slower); a
// 4-wave block owns 512 columns, its waves take alternate batches of RB rows,
// and the four partial sums meet in LDS.
template <int R, int MODE, int RB = 4>
__global__ void __launch_bounds__(256) lora_cols_kernel(const uint16_t* __restrict__ g, int64_t ldg,
                                                        const uint16_t* __restrict__ y, const uint16_t* __restrict__ a,
                                                        uint16_t* __restrict__ dx, float* __restrict__ part,
                                                        int64_t rows, int N, int rpp, float yscale, uint32_t seed,
                                                        uint32_t thresh16, float inv_keep) {
  // RB rows per load batch per wave (packed bf16 until used)
  __shared__ float red[3][32][64];
  const int cblocks = (N + 511) / 512;
  const int p = blockIdx.x / cblocks;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = ((blockIdx.x % cblocks) * 64 + lane) * 8;
  const bool active = c < N;
  const int64_t t0 = static_cast<int64_t>(p) * rpp;
  const int64_t t1 = t0 + rpp < rows ? t0 + rpp : rows;
  float acc[R][8];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
  uint32_t ap[MODE == 1 ? 8 : 1][R / 2];  // ap[e][i] = (a[2i][c+e], a[2i+1][c+e]) packed
  if constexpr (MODE == 1) {
    if (active) {
#pragma unroll
      for (int i = 0; i < R / 2; ++i) {
        uint32_t lo[4], hi[4];
        lora_ld16(a + static_cast<int64_t>(2 * i) * N + c, lo);
        lora_ld16(a + static_cast<int64_t>(2 * i + 1) * N + c, hi);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t l = (e & 1) ? (lo[e / 2] >> 16) : (lo[e / 2] & 0xffffu);
          const uint32_t h = (e & 1) ? (hi[e / 2] & 0xffff0000u) : (hi[e / 2] << 16);
          ap[e][i] = l | h;
        }
      }
    }
  }
  if (active) {
    for (int64_t tb = t0 + wv * RB; tb < t1; tb += 4 * RB) {
      uint32_t gp[RB][4], yp[RB][R / 2];  // packed bf16 until used
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int64_t t = tb + q;
        if (t < t1) {
          lora_ld16(g + t * ldg + c, gp[q]);
#pragma unroll
          for (int j = 0; j < R; j += 8) lora_ld16(y + t * R + j, &yp[q][j / 2]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) gp[q][e] = 0u;
#pragma unroll
          for (int j = 0; j < R / 2; ++j) yp[q][j] = 0u;
        }
      }
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        float gv[8], yv[R];
#pragma unroll
        for (int e = 0; e < 8; ++e) gv[e] = bf16_to_f32((e & 1) ? (gp[q][e / 2] >> 16) : (gp[q][e / 2] & 0xffffu));
#pragma unroll
        for (int j = 0; j < R; ++j) yv[j] = bf16_to_f32((j & 1) ? (yp[q][j / 2] >> 16) : (yp[q][j / 2] & 0xffffu));
        if constexpr (MODE == 1) {
          const int64_t t = tb + q;
          if (t < t1) {
            const uint32_t kp = keep8(seed, static_cast<uint64_t>(t) * N + c, thresh16);
            float d[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const bool keep = (kp >> e) & 1u;
              d[e] = keep ? lora_dot<R>(yp[q], ap[e]) * inv_keep : 0.f;
              gv[e] = keep ? gv[e] * inv_keep : 0.f;
            }
            lora_bf16x8 db;
#pragma unroll
            for (int e = 0; e < 8; ++e) db[e] = static_cast<__bf16>(d[e]);  // v_cvt_pk_bf16_f32 (RNE)
            *reinterpret_cast<lora_bf16x8*>(dx + t * N + c) = db;
          }
        }
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[j][e] += yv[j] * gv[e];
      }
    }
  }
  // the four waves' partial sums -> wave 0, 4 r-columns (32 floats per lane) at a time
#pragma unroll
  for (int jg = 0; jg < R; jg += 4) {
    if (wv > 0) {
#pragma unroll
      for (int q = 0; q < 32; ++q) red[wv - 1][q][lane] = acc[jg + q / 8][q % 8];
    }
    __syncthreads();
    if (wv == 0) {
#pragma unroll
      for (int q = 0; q < 32; ++q) acc[jg + q / 8][q % 8] += red[0][q][lane] + red[1][q][lane] + red[2][q][lane];
    }
    __syncthreads();
  }
  if (wv == 0 && active) {
    if constexpr (MODE == 0) {  // [P][N][R]: the layout of B [N, r]
      float* dst = part + (static_cast<int64_t>(p) * N + c) * R;
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int j = 0; j < R; j += 4)
          *reinterpret_cast<float4*>(dst + e * R + j) = make_float4(acc[j][e] * yscale, acc[j + 1][e] * yscale,
                                                                    acc[j + 2][e] * yscale, acc[j + 3][e] * yscale);
    } else {  // [P][R][N]: the layout of A [r, K]
      float* dst = part + static_cast<int64_t>(p) * R * N + c;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        *reinterpret_cast<float4*>(dst + static_cast<int64_t>(j) * N) =
            make_float4(acc[j][0] * yscale, acc[j][1] * yscale, acc[j][2] * yscale, acc[j][3] * yscale);
        *reinterpret_cast<float4*>(dst + static_cast<int64_t>(j) * N + 4) =
            make_float4(acc[j][4] * yscale, acc[j][5] * yscale, acc[j][6] * yscale, acc[j][7] * yscale);
      }
    }
  }
}

#define LORA_R_DISPATCH(R_VAL, ...)                          \
  switch (R_VAL) {                                           \
    case 8: { constexpr int R = 8; __VA_ARGS__; break; }     \
    case 16: { constexpr int R = 16; __VA_ARGS__; break; }   \
    default: return hipErrorInvalidValue;                    \
  }

hipError_t launch_lora_rows(const void* in, int64_t ldin, const void* w, void* out, int64_t rows, int K, int r,
                            float scale, uint32_t seed, uint32_t thresh16, float inv_keep, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (K % 32 != 0 || ldin % 8 != 0) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>((rows + 15) / 16)), block(512);
  auto I = static_cast<const uint16_t*>(in);
  auto W = static_cast<const uint16_t*>(w);
  auto O = static_cast<uint16_t*>(out);
  if (thresh16) {
    LORA_R_DISPATCH(r, hipLaunchKernelGGL((lora_rows_kernel<R, true>), grid, block, 0, st, I, ldin, W, O, rows, K, scale,
                                          seed, thresh16, inv_keep));
  } else {
    LORA_R_DISPATCH(r, hipLaunchKernelGGL((lora_rows_kernel<R, false>), grid, block, 0, st, I, ldin, W, O, rows, K,
                                          scale, seed, thresh16, inv_keep));
  }
  return hipGetLastError();
}

hipError_t launch_lora_up(const void* o, int64_t ldo, const void* u, const void* b, void* out, int64_t rows, int N, int r,
                          float s, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (N % 8 != 0 || ldo % 8 != 0) return hipErrorInvalidValue;
  const int rpt = 16;
  const int64_t threads = ((rows + rpt - 1) / rpt) * (N / 8);
  const dim3 grid(static_cast<unsigned>((threads + 255) / 256)), block(256);
  LORA_R_DISPATCH(r, hipLaunchKernelGGL((lora_up_kernel<R, 8>), grid, block, 0, st, static_cast<const uint16_t*>(o),
                                        ldo, static_cast<const uint16_t*>(u), static_cast<const uint16_t*>(b),
                                        static_cast<uint16_t*>(out), rows, N, rpt, s));
  return hipGetLastError();
}

int lora_cols_parts(int64_t rows, int N) {
  const int cblocks = (N + 511) / 512;
  int64_t p = 512 / cblocks;  // ~512 blocks of 4 waves
  const int64_t pmax = (rows + 15) / 16;
  if (p > pmax) p = pmax;
  return static_cast<int>(p < 1 ? 1 : p);
}

hipError_t launch_lora_cols(const void* g, int64_t ldg, const void* y, const void* a, void* dx, float* part, int64_t rows,
                            int N, int r, int parts, int mode, float yscale, uint32_t seed, uint32_t thresh16,
                            float inv_keep, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (N % 8 != 0 || ldg % 8 != 0 || parts < 1) return hipErrorInvalidValue;
  const int rpp = static_cast<int>((rows + parts - 1) / parts);
  const dim3 grid(static_cast<unsigned>(parts * ((N + 511) / 512))), block(256);
  auto G = static_cast<const uint16_t*>(g);
  auto Y = static_cast<const uint16_t*>(y);
  auto A = static_cast<const uint16_t*>(a);
  auto DX = static_cast<uint16_t*>(dx);
  if (mode == 0) {  // 8-row batches measured neutral at the SFT shape (profiles/r2/lora_up_rb_ab.txt)
    LORA_R_DISPATCH(r, hipLaunchKernelGGL((lora_cols_kernel<R, 0>), grid, block, 0, st, G, ldg, Y, A, DX, part, rows, N,
                                          rpp, yscale, seed, thresh16, inv_keep));
  } else {
    LORA_R_DISPATCH(r, hipLaunchKernelGGL((lora_cols_kernel<R, 1>), grid, block, 0, st, G, ldg, Y, A, DX, part, rows, N,
                                          rpp, yscale, seed, thresh16, inv_keep));
  }
  return hipGetLastError();
}

}  // namespace dlion

// Fused softmax cross-entropy for the LM head (gfx950).
//
// One 1024-thread workgroup per row.  The whole row (vocab padded to a multiple
// of 64) is held in registers -- each lane owns VPT 16-byte vectors -- so the
// logits are read from HBM exactly once and the gradient (softmax - onehot) is
// written back in place exactly once: 4 B/logit of traffic for bf16, against
// ~20 B/logit for the upcast + log_softmax + nll + backward chain of the HF
// reference path (HF GPT2LMHeadModel loss, /root/reference/run_clm.py:442).
#include "common.h"

#include <cstdlib>
#include <cstring>

namespace dlion {

constexpr int kXentThreads = 1024;
constexpr int kXentWaves = kXentThreads / 64;

// DPP / readlane wave reductions (common.h), no ds_bpermute chains
__device__ __forceinline__ float wave_max(float v) { return wave_max_dpp(v); }
__device__ __forceinline__ float wave_sum(float v) { return wave_sum_dpp(v); }

template <int DT, int VPT>
__global__ void __launch_bounds__(kXentThreads)
softmax_xent_kernel(typename Elem<DT>::S* __restrict__ logits, const int64_t* __restrict__ labels, int64_t vp,
                    int v, float* __restrict__ row_loss) {
  using E = Elem<DT>;
  using S = typename E::S;
  __shared__ float red[kXentWaves];
  __shared__ float tgt_logit;
  const int64_t row = blockIdx.x;
  S* x = logits + row * vp;
  const int64_t label = labels[row];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  float val[VPT][8];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int64_t e = (static_cast<int64_t>(i) * kXentThreads + tid) * 8;
    if (e < vp) {
      E::load8(x + e, val[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (e + j >= v) val[i][j] = -INFINITY;  // padded vocab columns
        if (e + j == label) tgt_logit = val[i][j];
        mx = fmaxf(mx, val[i][j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) val[i][j] = -INFINITY;
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int w = 1; w < kXentWaves; ++w) mx = fmaxf(mx, red[w]);
  __syncthreads();

  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      val[i][j] = __expf(val[i][j] - mx);  // exp(-inf) = 0 for padding
      sum += val[i][j];
    }
  sum = wave_sum(sum);
  if (lane == 0) red[wid] = sum;
  __syncthreads();
  sum = 0.f;
#pragma unroll
  for (int w = 0; w < kXentWaves; ++w) sum += red[w];

  const bool valid = label >= 0 && label < v;
  const float inv = 1.f / sum;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int64_t e = (static_cast<int64_t>(i) * kXentThreads + tid) * 8;
    if (e < vp) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = valid ? val[i][j] * inv - (e + j == label ? 1.f : 0.f) : 0.f;
      E::store8(x + e, o);
    }
  }
  if (tid == 0) row_loss[row] = valid ? (mx + __logf(sum)) - tgt_logit : 0.f;
}

// Wide vocabularies (> 8 vectors per thread of the register-resident kernel,
// e.g. Llama-3's 128k, which spilled there: 1.3 TB/s): two streaming passes
// over the row -- online max / sum-of-exp per thread, one block combine, then
// the gradient pass (the second read mostly hits L2).  3.2 TB/s at 8192 x 128256.
constexpr int kStreamThreads = 512;
template <int DT>
__global__ void __launch_bounds__(kStreamThreads)
softmax_xent_stream_kernel(typename Elem<DT>::S* __restrict__ logits, const int64_t* __restrict__ labels, int64_t n,
                           int64_t vp, int v, float* __restrict__ row_loss) {
  using E = Elem<DT>;
  using S = typename E::S;
  constexpr int W = kStreamThreads / 64;
  __shared__ float redm[2][W], reds[2][W];
  __shared__ float tgt_logit[2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int par = 0;
  for (int64_t row = blockIdx.x; row < n; row += gridDim.x, par ^= 1) {
    S* x = logits + row * vp;
    const int64_t label = labels[row];
    const int lab = (label >= 0 && label < v) ? static_cast<int>(label) : -1;
    float m = -INFINITY, sm = 0.f;
    for (int e = tid * 8; e < vp; e += kStreamThreads * 8) {
      float val[8];
      E::load8(x + e, val);
      float cm = m;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (e + j >= v) val[j] = -INFINITY;
        if (e + j == lab) tgt_logit[par] = val[j];
        cm = fmaxf(cm, val[j]);
      }
      if (cm > -INFINITY) {
        sm *= __expf(m - cm);
#pragma unroll
        for (int j = 0; j < 8; ++j) sm += __expf(val[j] - cm);
        m = cm;
      }
    }
    const float wm = wave_max(m);
    const float ws = wave_sum(m > -INFINITY ? sm * __expf(m - wm) : 0.f);
    if (lane == 0) {
      redm[par][wid] = wm;
      reds[par][wid] = ws;
    }
    __syncthreads();
    float mx = redm[par][0];
#pragma unroll
    for (int w = 1; w < W; ++w) mx = fmaxf(mx, redm[par][w]);
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) sum += redm[par][w] > -INFINITY ? reds[par][w] * __expf(redm[par][w] - mx) : 0.f;
    const bool valid = lab >= 0;
    const float inv = valid ? 1.f / sum : 0.f;
    for (int e = tid * 8; e < vp; e += kStreamThreads * 8) {
      float val[8], o[8];
      E::load8(x + e, val);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = (e + j < v ? __expf(val[j] - mx) * inv : 0.f) - (e + j == lab ? 1.f : 0.f);
      E::store8(x + e, o);
    }
    if (tid == 0) row_loss[row] = valid ? (mx + __logf(sum)) - tgt_logit[par] : 0.f;
  }
}


// an empty asm that "modifies" the packed row: values unpacked before it
// cannot be reused after it, so hipcc keeps 4 VGPRs per chunk live, not 8 floats
template <int CH>
__device__ __forceinline__ void opaque(uint4 (&raw)[CH]) {
#pragma unroll
  for (int i = 0; i < CH; ++i) asm volatile("" : "+v"(raw[i].x), "+v"(raw[i].y), "+v"(raw[i].z), "+v"(raw[i].w));
}

// Packed variant for 16-bit logits: the row stays in registers as raw 16-bit
// pairs (CH 16-byte chunks per lane, 4 VGPRs each) instead of fp32 (8 VGPRs
// per chunk), so a row needs half the registers and THREADS-thread blocks run
// several rows per CU at once: every chunk load is issued up front, and one
// row's reductions / write-back overlap the next row's loads.  Each pass
// (max, sum of exp, gradient) unpacks on the fly -- two exps per logit, which
// is noise next to the memory traffic.
template <int DT, int THREADS, int CH>
__global__ void __launch_bounds__(THREADS)
softmax_xent_packed_kernel(uint16_t* __restrict__ logits, const int64_t* __restrict__ labels, int64_t vp, int v,
                           float* __restrict__ row_loss) {
  using E = Elem<DT>;
  constexpr int W = THREADS / 64;
  __shared__ float red[2][W];
  const int64_t row = blockIdx.x;
  uint16_t* x = logits + row * vp;
  const int64_t label = labels[row];
  const int lab = (label >= 0 && label < v) ? static_cast<int>(label) : -1;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // the target logit comes straight from memory (one scalar load per row)
  const float tgt = lab >= 0 ? E::to_f(x[lab]) : 0.f;
  constexpr uint32_t kNegInf2 = DT == kBF16 ? 0xff80ff80u : 0xfc00fc00u;
  uint4 raw[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int e = (i * THREADS + tid) * 8;
    raw[i] = e < vp ? *reinterpret_cast<const uint4*>(x + e) : make_uint4(kNegInf2, kNegInf2, kNegInf2, kNegInf2);
  }
  // padded vocab columns (v <= e+j < vp) become -inf in the packed row itself,
  // so no pass needs a per-element bound check
  {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int e = (i * THREADS + tid) * 8;
      if (e + 8 > v && e < vp) {
        uint32_t wv[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (e + j >= v) wv[j >> 1] = (j & 1) ? ((wv[j >> 1] & 0xffffu) | (kNegInf2 & 0xffff0000u))
                                               : ((wv[j >> 1] & 0xffff0000u) | (kNegInf2 & 0xffffu));
        raw[i] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    }
  }
  auto unpack = [&](const uint4& r4, float (&f)[8]) {
    const uint32_t wv[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = E::to_f(static_cast<uint16_t>(j & 1 ? wv[j >> 1] >> 16 : wv[j >> 1] & 0xffffu));
  };
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    float f[8];
    unpack(raw[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, f[j]);
  }
  opaque(raw);  // keep the row packed: the next pass re-unpacks instead of holding fp32 copies live
  mx = wave_max(mx);
  if (lane == 0) red[0][wid] = mx;
  __syncthreads();
  mx = red[0][0];
#pragma unroll
  for (int w = 1; w < W; ++w) mx = fmaxf(mx, red[0][w]);

  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    float f[8];
    unpack(raw[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += __expf(f[j] - mx);  // exp(-inf) = 0: padding and past-the-row
  }
  opaque(raw);
  sum = wave_sum(sum);
  if (lane == 0) red[1][wid] = sum;
  __syncthreads();
  sum = 0.f;
#pragma unroll
  for (int w = 0; w < W; ++w) sum += red[1][w];

  const float inv = lab >= 0 ? 1.f / sum : 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int e = (i * THREADS + tid) * 8;
    if (e < vp) {
      float f[8], o[8];
      unpack(raw[i], f);
      const int rel = lab - e;  // the one-hot column, if it is in this chunk
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = __expf(f[j] - mx) * inv - (rel == j ? 1.f : 0.f);
      E::store8(x + e, o);
    }
  }
  if (tid == 0) row_loss[row] = lab >= 0 ? (mx + __logf(sum)) - tgt : 0.f;
}

template <int DT, int THREADS, int CH>
static void launch_packed(uint16_t* lp, const int64_t* labels, int64_t n, int64_t vp, int v, float* loss,
                          hipStream_t st) {
  hipLaunchKernelGGL((softmax_xent_packed_kernel<DT, THREADS, CH>), dim3(n), dim3(THREADS), 0, st, lp, labels, vp, v,
                     loss);
}

// packed 16-bit row kernel when the row fits: returns false otherwise
template <int DT>
static bool launch_packed_dt(int threads, void* logits, const int64_t* labels, int64_t n, int64_t vp, int v,
                             float* loss, hipStream_t st) {
  uint16_t* lp = static_cast<uint16_t*>(logits);
  const int64_t ch = (vp + threads * 8 - 1) / (threads * 8);
  if (threads == 1024) {
    if (ch <= 4) launch_packed<DT, 1024, 4>(lp, labels, n, vp, v, loss, st);
    else if (ch <= 7) launch_packed<DT, 1024, 7>(lp, labels, n, vp, v, loss, st);
    else return false;
  } else if (threads == 256) {
    if (ch <= 16) launch_packed<DT, 256, 16>(lp, labels, n, vp, v, loss, st);
    else if (ch <= 25) launch_packed<DT, 256, 25>(lp, labels, n, vp, v, loss, st);
    else return false;
  } else {
    if (ch <= 8) launch_packed<DT, 512, 8>(lp, labels, n, vp, v, loss, st);
    else if (ch <= 13) launch_packed<DT, 512, 13>(lp, labels, n, vp, v, loss, st);
    else if (ch <= 16) launch_packed<DT, 512, 16>(lp, labels, n, vp, v, loss, st);
    else return false;
  }
  return true;
}

// Measured at the GPT-2 shape (20480 x 50304 bf16, tools/bench_xent.py): fp32-row
// 1194 us, streaming 1224 us, packed 512 thr 966 us, packed 1024 thr 874 us
// (4.7 TB/s); Llama-2 vocab (8192 x 32000): 280 / - / 204 / 210 us.
template <int DT>
static hipError_t launch_xent_dt(void* logits, const int64_t* labels, int64_t n, int64_t vp, int v, float* loss,
                                 int var, hipStream_t st) {
  using S = typename Elem<DT>::S;
  const int64_t per = kXentThreads * 8;
  const int vpt = static_cast<int>((vp + per - 1) / per);
  S* lp = static_cast<S*>(logits);
  if constexpr (DT != kF32) {
    if (var == 0) var = (vp + 8191) / 8192 <= 7 ? 5 : (vp + 4095) / 4096 <= 16 ? 4 : 0;
    if (var >= 3 && launch_packed_dt<DT>(var == 3 ? 256 : var == 4 ? 512 : 1024, logits, labels, n, vp, v, loss, st))
      return hipGetLastError();
  }
#define XENT_CASE(K)                                                                                   \
  case K:                                                                                              \
    hipLaunchKernelGGL((softmax_xent_kernel<DT, K>), dim3(n), dim3(kXentThreads), 0, st, lp, labels, vp, v, loss); \
    break;
  if (vpt > 8 || var == 2) {
    const int64_t grid = n < 1024 ? n : 1024;  // persistent
    hipLaunchKernelGGL((softmax_xent_stream_kernel<DT>), dim3(grid), dim3(kStreamThreads), 0, st, lp, labels, n, vp,
                       v, loss);
    return hipGetLastError();
  }
  switch (vpt) {
    XENT_CASE(1)
    XENT_CASE(2)
    XENT_CASE(4)
    XENT_CASE(7)
    XENT_CASE(8)
    default:
      if (vpt <= 4) { hipLaunchKernelGGL((softmax_xent_kernel<DT, 4>), dim3(n), dim3(kXentThreads), 0, st, lp, labels, vp, v, loss); }
      else { hipLaunchKernelGGL((softmax_xent_kernel<DT, 8>), dim3(n), dim3(kXentThreads), 0, st, lp, labels, vp, v, loss); }
  }
#undef XENT_CASE
  return hipGetLastError();
}

hipError_t launch_softmax_xent(int dt, void* logits, const int64_t* labels, int64_t n, int64_t vp, int v, float* loss,
                               int variant, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(logits) % 16 != 0) return hipErrorInvalidValue;
  switch (dt) {
    case kF32: return launch_xent_dt<kF32>(logits, labels, n, vp, v, loss, variant, st);
    case kBF16: return launch_xent_dt<kBF16>(logits, labels, n, vp, v, loss, variant, st);
    case kF16: return launch_xent_dt<kF16>(logits, labels, n, vp, v, loss, variant, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlion

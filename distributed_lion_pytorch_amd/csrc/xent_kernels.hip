// Fused softmax cross-entropy for the LM head (gfx950).
//
// One 1024-thread workgroup per row.  The whole row (vocab padded to a multiple
// of 64) is held in registers -- each lane owns VPT 16-byte vectors -- so the
// logits are read from HBM exactly once and the gradient (softmax - onehot) is
// written back in place exactly once: 4 B/logit of traffic for bf16, against
// ~20 B/logit for the upcast + log_softmax + nll + backward chain of the HF
// reference path (HF GPT2LMHeadModel loss, /root/reference/run_clm.py:442).
#include "common.h"

namespace dlion {

constexpr int kXentThreads = 1024;
constexpr int kXentWaves = kXentThreads / 64;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

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

template <int DT>
static hipError_t launch_xent_dt(void* logits, const int64_t* labels, int64_t n, int64_t vp, int v, float* loss,
                                 hipStream_t st) {
  using S = typename Elem<DT>::S;
  const int64_t per = kXentThreads * 8;
  const int vpt = static_cast<int>((vp + per - 1) / per);
  S* lp = static_cast<S*>(logits);
#define XENT_CASE(K)                                                                                   \
  case K:                                                                                              \
    hipLaunchKernelGGL((softmax_xent_kernel<DT, K>), dim3(n), dim3(kXentThreads), 0, st, lp, labels, vp, v, loss); \
    break;
  if (vpt > 8) {
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
                               hipStream_t st) {
  if (n == 0) return hipSuccess;
  switch (dt) {
    case kF32: return launch_xent_dt<kF32>(logits, labels, n, vp, v, loss, st);
    case kBF16: return launch_xent_dt<kBF16>(logits, labels, n, vp, v, loss, st);
    case kF16: return launch_xent_dt<kF16>(logits, labels, n, vp, v, loss, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlion

// Distributed Lion optimizer kernels for gfx950 (MI355X / CDNA4).
//
// Replaces the per-parameter ATen chains of the reference optimizer
// (/root/reference/distributed_lion.py:47-96, ~20 + 6*W launches and one
// collective PER TENSOR) with multi-tensor kernels that touch every byte once:
//
//   K0 lion_local      p,g,m -> p,m           local Lion          (ref :47-59)
//   K1 lion_encode     g,m   -> m, sign bits  WD-free interp+sign+1-bit pack
//                                             + momentum EMA       (ref :64-77, :96)
//   K3 (K1 with stochastic=1)                 stochastic binarization, Philox
//                                                                  (ref :98-108)
//   K2 lion_vote_apply p, W bit planes -> p   popcount majority / average vote
//                                             + decoupled WD + step (ref :84-92)
//   K4 vote_reduce     W shards -> voted bits  (all-to-all "vote-RS" scheme)
//
// Multi-tensor layout (built once per parameter set by parallel/plan.py):
//   seg   [T][8] int64 : p_ptr, g_ptr, m_ptr, numel, bit_off, flags, 0, 0
//   chunk [C][2] int64 : segment index, first element
// A chunk is CHUNK=8192 elements (one 256-thread block, 4 iterations of 2048);
// each tensor owns ceil(numel/2048)*2048 bits of the bucket's bit space, so the
// packed bits of tensor t start at byte bit_off/8 and never straddle tensors.
// Bit layout is little-endian "packbits": element e <-> byte e/8, bit e%8, i.e.
// exactly the reference's wire encoding (ref :75-77) but 1 bit/param (the
// reference promotes to int64, 8 bytes per 8 params).
#include "common.h"

namespace dlion {

// Launch shape, fixed by A/B measurement (tools/bench_lion.py, profiles/r3/):
// * the pre-voted and majority applies run two chunks per block (one metadata
//   chain per 16k params): GPT-2 122 -> 113 us, W=8 majority 170 -> 155 us,
//   Llama-3-8B majority 9.3 -> 8.5 ms (profiles/r3/lion_pair_ab.txt,
//   lion_pair_maj_ab.txt); four chunks per block and non-temporal p stores
//   measured neutral and were removed;
// * the sliced K4 vote loads two words per thread per grid-stride step
//   (GPT-2 shard 8.1 -> 7.4 us) on a grid capped at 2048 blocks.
constexpr int kPairChunks = 2;
constexpr int kK4Unroll = 2;
constexpr int kK4MaxBlocks = 2048;

constexpr int kThreads = 256;
constexpr int kIters = 4;
constexpr int kSpan = kThreads * 8;        // 2048 elements per block iteration
constexpr int64_t kChunk = kSpan * kIters;  // 8192 elements per block

struct SegRow {
  const void* p;
  const void* g;
  const void* m;
  int64_t n;
  int64_t bit_off;
  bool vec;
};

__device__ __forceinline__ SegRow load_seg(const int64_t* __restrict__ seg, int64_t s) {
  const int64_t* r = seg + 8 * s;
  SegRow o;
  o.p = reinterpret_cast<const void*>(r[0]);
  o.g = reinterpret_cast<const void*>(r[1]);
  o.m = reinterpret_cast<const void*>(r[2]);
  o.n = r[3];
  o.bit_off = r[4];
  o.vec = (r[5] & 1) != 0;
  return o;
}

__device__ __forceinline__ float sgn(float x) {  // ATen sign: NaN -> 0, +-0 -> 0
  return static_cast<float>((x > 0.f) - (x < 0.f));
}

// Raw 8-element vectors for the full-chunk fast paths: every load of a
// block's 4 iterations is issued before the first use (a chunk that lies
// wholly inside a 16-byte-aligned tensor -- all but the last chunk of a
// tensor).  In the general loop below the per-iteration bounds test keeps
// hipcc from hoisting iteration i+1's loads above iteration i's stores, so
// each lane had one load in flight at a time: K2 reached 68 % of HBM against
// K0's 89 % (profiles/lion/bench_lion_roofline.txt).
template <int DT>
struct Raw8 {
  static constexpr int N = DT == kF32 ? 2 : 1;  // uint4 per 8 elements
  uint4 v[N];
  __device__ __forceinline__ void load(const typename Elem<DT>::S* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = reinterpret_cast<const uint4*>(p)[i];
  }
  __device__ __forceinline__ void unpack(float (&o)[8]) const {
    if constexpr (DT == kF32) {
      const uint32_t w[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = __uint_as_float(w[j]);
    } else {
      const uint32_t w[4] = {v[0].x, v[0].y, v[0].z, v[0].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[2 * i] = Elem<DT>::to_f(static_cast<uint16_t>(w[i] & 0xffffu));
        o[2 * i + 1] = Elem<DT>::to_f(static_cast<uint16_t>(w[i] >> 16));
      }
    }
  }
};

// Fused gradient clipping: g <- round(g * coef) in the parameter dtype, i.e.
// what clip_grad_norm_'s in-place _foreach_mul_ would have stored, applied on
// load instead of as a separate read+write pass over every gradient.
template <int DT>
__device__ __forceinline__ void clip8(float (&gv)[8], float cs) {
#pragma unroll
  for (int j = 0; j < 8; ++j) gv[j] = Elem<DT>::rnd(gv[j] * cs);
}

// ----------------------------------------------------------------------- K0
template <int DT>
__global__ void __launch_bounds__(kThreads)
lion_local_kernel(const int64_t* __restrict__ seg, const int64_t* __restrict__ chunks,
                  float decay, float neg_lr, float b1, float omb1, float b2, float omb2,
                  const float* __restrict__ gscale) {
  using E = Elem<DT>;
  using S = typename E::S;
  const int64_t s = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const float cs = gscale != nullptr ? gscale[1] : 1.f;
  const SegRow r = load_seg(seg, s);
  S* p = const_cast<S*>(static_cast<const S*>(r.p));
  const S* g = static_cast<const S*>(r.g);
  S* m = const_cast<S*>(static_cast<const S*>(r.m));
  if (r.vec && start + kChunk <= r.n) {  // block-uniform: all loads first
    Raw8<DT> rp[kIters], rg[kIters], rm[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t e = start + it * kSpan + threadIdx.x * 8;
      rp[it].load(p + e);
      rg[it].load(g + e);
      rm[it].load(m + e);
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t e = start + it * kSpan + threadIdx.x * 8;
      float pv[8], gv[8], mv[8];
      rp[it].unpack(pv);
      rg[it].unpack(gv);
      rm[it].unpack(mv);
      if (gscale != nullptr) clip8<DT>(gv, cs);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pw = E::rnd(pv[j] * decay);
        const float u = E::rnd(__fmaf_rn(gv[j], omb1, E::rnd(mv[j] * b1)));
        pv[j] = __fmaf_rn(neg_lr, sgn(u), pw);
        mv[j] = __fmaf_rn(gv[j], omb2, E::rnd(mv[j] * b2));
      }
      E::store8(p + e, pv);
      E::store8(m + e, mv);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t e = start + it * kSpan + threadIdx.x * 8;
    if (e >= r.n) break;
    float pv[8], gv[8], mv[8];
    load8g<DT>(p, e, r.n, r.vec, pv);
    load8g<DT>(g, e, r.n, r.vec, gv);
    load8g<DT>(m, e, r.n, r.vec, mv);
    if (gscale != nullptr) clip8<DT>(gv, cs);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float pw = E::rnd(pv[j] * decay);                       // p *= 1 - lr*wd
      const float u = E::rnd(__fmaf_rn(gv[j], omb1, E::rnd(mv[j] * b1)));  // b1*m + (1-b1)*g
      pv[j] = __fmaf_rn(neg_lr, sgn(u), pw);                         // p -= lr*sign(u)
      mv[j] = __fmaf_rn(gv[j], omb2, E::rnd(mv[j] * b2));            // m = b2*m + (1-b2)*g
    }
    store8g<DT>(p, e, r.n, r.vec, pv);
    store8g<DT>(m, e, r.n, r.vec, mv);
  }
}

// ----------------------------------------------------------------- K1 / K3
// The 4 lanes of a quad own 32 consecutive coordinates (bit_off % 2048 == 0,
// lane stride 8): their sign bytes are gathered with DPP quad broadcasts (VALU,
// no LDS) and the quad's first lane stores the dword -- 16 dword stores per
// wave instead of 64 byte stores.  Every lane of the wave must be active.
__device__ __forceinline__ uint32_t quad_pack(uint32_t b) {
  const int v = static_cast<int>(b);
  const uint32_t b1 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(v, 0x55, 0xf, 0xf, false));
  const uint32_t b2 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(v, 0xaa, 0xf, 0xf, false));
  const uint32_t b3 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(v, 0xff, 0xf, 0xf, false));
  const uint32_t b0 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(v, 0x00, 0xf, 0xf, false));
  return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}

__device__ __forceinline__ void store_quad_bits(uint8_t* bits, int64_t bit, uint32_t byte) {
  const uint32_t w = quad_pack(byte);
  if ((threadIdx.x & 3) == 0) reinterpret_cast<uint32_t*>(bits)[bit >> 5] = w;
}

// bits: this rank's packed sign plane for the bucket (bucket-relative bit_off).
// stochastic: bit = Bernoulli(clamp((u + rr) / (2 rr), 0, 1)) with
//   rr = (1 + 1/b1) * max_grad_norm  (ref :106-108, clamped: SURVEY D4).
template <int DT, bool STOC>
__global__ void __launch_bounds__(kThreads)
lion_encode_kernel(const int64_t* __restrict__ seg, const int64_t* __restrict__ chunks,
                   uint8_t* __restrict__ bits, float b1, float omb1, float b2, float omb2,
                   int update_m, float rr, uint32_t seed_lo, uint32_t seed_hi, uint32_t step,
                   const float* __restrict__ gscale) {
  using E = Elem<DT>;
  using S = typename E::S;
  const int64_t s = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const float cs = gscale != nullptr ? gscale[1] : 1.f;
  const SegRow r = load_seg(seg, s);
  const S* g = static_cast<const S*>(r.g);
  S* m = const_cast<S*>(static_cast<const S*>(r.m));
  const int64_t region = (r.n + kSpan - 1) / kSpan * kSpan;
  if (!STOC && r.vec && start + kChunk <= r.n) {  // block-uniform: all loads first
    Raw8<DT> rg[kIters], rm[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t e = start + it * kSpan + threadIdx.x * 8;
      rg[it].load(g + e);
      rm[it].load(m + e);
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t e = start + it * kSpan + threadIdx.x * 8;
      float gv[8], mv[8];
      rg[it].unpack(gv);
      rm[it].unpack(mv);
      if (gscale != nullptr) clip8<DT>(gv, cs);
      uint32_t byte = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        byte |= static_cast<uint32_t>(E::rnd(__fmaf_rn(gv[j], omb1, E::rnd(mv[j] * b1))) > 0.f) << j;
      if (update_m) {
#pragma unroll
        for (int j = 0; j < 8; ++j) mv[j] = __fmaf_rn(gv[j], omb2, E::rnd(mv[j] * b2));
        E::store8(m + e, mv);
      }
      store_quad_bits(bits, r.bit_off + e, byte);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t e = start + it * kSpan + threadIdx.x * 8;
    if (e >= region) break;  // uniform per block iteration (region % 2048 == 0)
    uint32_t byte = 0;
    if (e < r.n) {
      float gv[8], mv[8];
      load8g<DT>(g, e, r.n, r.vec, gv);
      load8g<DT>(m, e, r.n, r.vec, mv);
      if (gscale != nullptr) clip8<DT>(gv, cs);
      float u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = E::rnd(__fmaf_rn(gv[j], omb1, E::rnd(mv[j] * b1)));
      if constexpr (STOC) {
        const uint64_t gi = static_cast<uint64_t>(r.bit_off + e);  // unique per element
        const uint4 c0 = philox4x32_10(
            make_uint4(static_cast<uint32_t>(gi), static_cast<uint32_t>(gi >> 32), step, 0u),
            make_uint2(seed_lo, seed_hi));
        const uint4 c1 = philox4x32_10(
            make_uint4(static_cast<uint32_t>(gi), static_cast<uint32_t>(gi >> 32), step, 1u),
            make_uint2(seed_lo, seed_hi));
        const uint32_t rnd[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float inv = 0.5f / rr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (e + j < r.n) {
            const float pr = fminf(fmaxf((u[j] + rr) * inv, 0.f), 1.f);
            byte |= static_cast<uint32_t>(u32_to_unit(rnd[j]) < pr) << j;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (e + j < r.n) byte |= static_cast<uint32_t>(u[j] > 0.f) << j;  // sign 0/NaN -> 0
      }
      if (update_m) {
#pragma unroll
        for (int j = 0; j < 8; ++j) mv[j] = __fmaf_rn(gv[j], omb2, E::rnd(mv[j] * b2));
        store8g<DT>(m, e, r.n, r.vec, mv);
      }
    }
    store_quad_bits(bits, r.bit_off + e, byte);  // all lanes reach here (the break above is block-uniform)
  }
}

// ----------------------------------------------------------------------- K2
// mode 0: majority vote over the alive planes  delta = +1 / -1 / tie rule
// mode 1: average (paper's server "Averaging")  delta = (2c - n) / n
// mode 2: pre-voted bitmap (vote-RS/AG path)    delta = pos ? +1 : (neg ? -1 : 0)
//         planes = pos bitmap, neg = optional neg bitmap (nullptr -> ~pos)
// tie: 0 -> -1 (reference parity: torch.mode tie -> False), 1 -> 0, 2 -> +1
// p <- round(round(p * decay) - lr * delta)   (ref :64 then :92)
// agree (optional): count of coordinates where this rank's own bits (`own`,
// its send plane) agree with the voted direction (vote-agreement telemetry).
template <int DT>
__global__ void __launch_bounds__(kThreads)
lion_vote_apply_kernel(const int64_t* __restrict__ seg, const int64_t* __restrict__ chunks,
                       const uint8_t* __restrict__ planes, int64_t plane_stride,
                       const uint8_t* __restrict__ alive, int world, int mode, int tie,
                       const uint8_t* __restrict__ neg, float decay, float neg_lr,
                       const uint8_t* __restrict__ own, unsigned long long* __restrict__ agree) {
  using E = Elem<DT>;
  using S = typename E::S;
  const int64_t s = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const SegRow r = load_seg(seg, s);
  S* p = const_cast<S*>(static_cast<const S*>(r.p));
  const float tie_delta = tie == 0 ? -1.f : (tie == 1 ? 0.f : 1.f);
  int n_live = 0;  // liveness is a device vector: no host sync to learn who voted
  for (int k = 0; k < world; ++k) n_live += alive[k] != 0;
  const float inv_n = n_live > 0 ? 1.f / static_cast<float>(n_live) : 0.f;
  uint32_t n_agree = 0, n_tie = 0;
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t e = start + it * kSpan + threadIdx.x * 8;
    if (e >= r.n) break;
    const int64_t byte_idx = (r.bit_off + e) >> 3;
    float delta[8];
    if (mode == 2) {
      const uint32_t pos = planes[byte_idx];
      const uint32_t ng = neg ? neg[byte_idx] : (~pos & 0xffu);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        delta[j] = ((pos >> j) & 1) ? 1.f : (((ng >> j) & 1) ? -1.f : 0.f);
    } else {
      uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int r0 = 0; r0 < world; r0 += 255) {
        const int r1 = min(world, r0 + 255);
        uint64_t acc = 0;
        for (int k = r0; k < r1; ++k)
          if (alive[k]) acc += spread8(planes[k * plane_stride + byte_idx]);
#pragma unroll
        for (int j = 0; j < 8; ++j) cnt[j] += static_cast<uint32_t>((acc >> (8 * j)) & 0xffu);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int twice = 2 * static_cast<int>(cnt[j]);
        if (agree != nullptr && n_live > 0 && twice == n_live && e + j < r.n) ++n_tie;
        if (n_live == 0)
          delta[j] = 0.f;  // nobody voted: weight decay only
        else if (mode == 1)
          delta[j] = static_cast<float>(twice - n_live) * inv_n;
        else
          delta[j] = twice > n_live ? 1.f : (twice < n_live ? -1.f : tie_delta);
      }
    }
    if (agree != nullptr) {
      const uint32_t mine = own[byte_idx];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (e + j < r.n) n_agree += (((mine >> j) & 1) ? 1.f : -1.f) * delta[j] > 0.f;
    }
    float pv[8];
    load8g<DT>(p, e, r.n, r.vec, pv);
#pragma unroll
    for (int j = 0; j < 8; ++j) pv[j] = __fmaf_rn(neg_lr, delta[j], E::rnd(pv[j] * decay));
    store8g<DT>(p, e, r.n, r.vec, pv);
  }
  if (agree != nullptr) {
    // wave reduce then one atomic per wave (Guideline 12)
    for (int off = 32; off > 0; off >>= 1) {
      n_agree += __shfl_xor(n_agree, off);
      n_tie += __shfl_xor(n_tie, off);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(agree, static_cast<unsigned long long>(n_agree));
      if (n_tie) atomicAdd(agree + 1, static_cast<unsigned long long>(n_tie));
    }
  }
}

// K2, word-sliced: one dword per live plane per 32 coordinates, the vote as
// bit-sliced counters.  The byte version above is latency-bound at W > 1 (a runtime loop
// of dependent byte loads per plane, 64-bit spreads): 2.0 TB/s effective at
// W = 8.  Here every plane word is loaded up front, each plane costs 7 bitwise
// ops per 32 coordinates (a 4-bit vertical counter), and the majority is a
// bit-sliced compare with floor(n_live / 2).  Majority (mode 0) for W <= 15
// and pre-voted bitmaps (mode 2); mode 1 and wider worlds use the byte kernel.
constexpr int kMaxSliced = 15;

// Majority over up to 15 planes for 32 coordinates at once: a 4-bit vertical
// counter per bit position (7 bitwise ops per plane), then count vs
// K = floor(n_live / 2) compared bit-sliced from the MSB.  pos / neg follow the
// byte kernels' rules (ties by `tie`, nobody alive -> neither).
__device__ __forceinline__ void sliced_vote(const uint32_t (&w)[kMaxSliced], int world, int n_live, int tie,
                                            uint32_t& pos, uint32_t& neg, uint32_t& ties) {
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
  for (int k = 0; k < kMaxSliced; ++k) {
    if (k >= world) break;  // uniform
    const uint32_t x = w[k];
    const uint32_t t0 = c0 & x;
    c0 ^= x;
    const uint32_t t1 = c1 & t0;
    c1 ^= t0;
    const uint32_t t2 = c2 & t1;
    c2 ^= t1;
    c3 ^= t2;
  }
  const int K = n_live >> 1;
  uint32_t gt = 0, eq = 0xffffffffu;
  const uint32_t cb[4] = {c0, c1, c2, c3};
#pragma unroll
  for (int b = 3; b >= 0; --b) {
    if ((K >> b) & 1) {
      eq &= cb[b];
    } else {
      gt |= eq & cb[b];
      eq &= ~cb[b];
    }
  }
  ties = 0;
  if (n_live == 0) {
    pos = neg = 0;  // nobody voted: weight decay only
  } else if (n_live & 1) {
    pos = gt;  // count > K  <=>  2*count > n_live
    neg = ~gt;
  } else {
    const uint32_t lt = ~(gt | eq);
    pos = gt | (tie == 2 ? eq : 0u);
    neg = lt | (tie == 0 ? eq : 0u);
    ties = eq;  // count == n_live / 2: resolved by the tie rule
  }
}

template <int DT>
__global__ void __launch_bounds__(kThreads)
lion_vote_apply32_kernel(const int64_t* __restrict__ seg, const int64_t* __restrict__ chunks,
                         const uint8_t* __restrict__ planes, int64_t plane_stride,
                         const uint8_t* __restrict__ alive, int world, int mode, int tie,
                         const uint8_t* __restrict__ neg_plane, float decay, float neg_lr,
                         const uint8_t* __restrict__ own, unsigned long long* __restrict__ agree) {
  using E = Elem<DT>;
  using S = typename E::S;
  const int64_t s = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const SegRow r = load_seg(seg, s);
  S* p = const_cast<S*>(static_cast<const S*>(r.p));
  int n_live = 0;
  uint32_t live_mask = 0;
  for (int k = 0; k < world && k < kMaxSliced; ++k)
    if (alive[k]) {
      live_mask |= 1u << k;
      ++n_live;
    }
  uint32_t n_agree = 0, n_tie = 0;
  // Each lane owns 8 consecutive coordinates (coalesced 16-byte p accesses,
  // as in K0); the 4 lanes of a 32-coordinate group load the same plane dword
  // and vote on all of it, then keep their byte.
  const int sub = threadIdx.x & 3;  // bit_off % 2048 == 0, start % 8192 == 0
  if (r.vec && start + kChunk <= r.n && agree == nullptr) {  // block-uniform: all loads first
    Raw8<DT> rp[kIters];
    uint32_t pw[kIters], nw[kIters];
    if (mode == 2) {
#pragma unroll
      for (int it = 0; it < kIters; ++it) {
        const int64_t e = start + it * kSpan + threadIdx.x * 8;
        const int64_t word = (r.bit_off + e) >> 5;
        rp[it].load(p + e);
        pw[it] = reinterpret_cast<const uint32_t*>(planes)[word];
        nw[it] = neg_plane ? reinterpret_cast<const uint32_t*>(neg_plane)[word] : ~pw[it];
      }
    } else {
      // majority over W planes: hoisting every plane word of all 4 iterations
      // (4 x 15 registers behind a runtime live mask) spilled and ran at 21 %
      // of HBM; only the p loads are hoisted here, the plane words of each
      // iteration are loaded and voted on per iteration (the byte-light part)
#pragma unroll
      for (int it = 0; it < kIters; ++it) rp[it].load(p + start + it * kSpan + threadIdx.x * 8);
#pragma unroll
      for (int it = 0; it < kIters; ++it) {
        const int64_t word = (r.bit_off + start + it * kSpan + threadIdx.x * 8) >> 5;
        uint32_t w[kMaxSliced], tb;
#pragma unroll
        for (int k = 0; k < kMaxSliced; ++k)
          w[k] = (live_mask >> k) & 1 ? reinterpret_cast<const uint32_t*>(planes + k * plane_stride)[word] : 0u;
        sliced_vote(w, world, n_live, tie, pw[it], nw[it], tb);
      }
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t e = start + it * kSpan + threadIdx.x * 8;
      const uint32_t pos = (pw[it] >> (8 * sub)) & 0xffu, neg = (nw[it] >> (8 * sub)) & 0xffu;
      float pv[8];
      rp[it].unpack(pv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float delta = static_cast<float>(static_cast<int>((pos >> j) & 1) - static_cast<int>((neg >> j) & 1));
        pv[j] = __fmaf_rn(neg_lr, delta, E::rnd(pv[j] * decay));
      }
      E::store8(p + e, pv);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t e = start + it * kSpan + threadIdx.x * 8;
    if (e >= r.n) break;
    const int64_t word = (r.bit_off + e) >> 5;
    uint32_t pos, neg, tb = 0;
    if (mode == 2) {
      pos = reinterpret_cast<const uint32_t*>(planes)[word];
      neg = neg_plane ? reinterpret_cast<const uint32_t*>(neg_plane)[word] : ~pos;
    } else {
      uint32_t w[kMaxSliced];
#pragma unroll
      for (int k = 0; k < kMaxSliced; ++k)  // every live plane's load first
        w[k] = (live_mask >> k) & 1 ? reinterpret_cast<const uint32_t*>(planes + k * plane_stride)[word] : 0u;
      sliced_vote(w, world, n_live, tie, pos, neg, tb);
    }
    pos = (pos >> (8 * sub)) & 0xffu;
    neg = (neg >> (8 * sub)) & 0xffu;
    if (agree != nullptr) {
      const uint32_t mine = own[(r.bit_off + e) >> 3];
      const int64_t left = r.n - e;
      const uint32_t valid = left >= 8 ? 0xffu : ((1u << left) - 1u);
      n_agree += __popc(((mine & pos) | (~mine & neg)) & valid);
      n_tie += __popc((tb >> (8 * sub)) & valid);  // (pre-voted planes: the ties were counted by K4)
    }
    float pv[8];
    load8g<DT>(p, e, r.n, r.vec, pv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float delta = static_cast<float>(static_cast<int>((pos >> j) & 1) - static_cast<int>((neg >> j) & 1));
      pv[j] = __fmaf_rn(neg_lr, delta, E::rnd(pv[j] * decay));
    }
    store8g<DT>(p, e, r.n, r.vec, pv);
  }
  if (agree != nullptr) {
    for (int off = 32; off > 0; off >>= 1) {
      n_agree += __shfl_xor(n_agree, off);
      n_tie += __shfl_xor(n_tie, off);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(agree, static_cast<unsigned long long>(n_agree));
      if (n_tie) atomicAdd(agree + 1, static_cast<unsigned long long>(n_tie));
    }
  }
}

// K2 without telemetry, two chunks per block: pre-voted (mode 2, the a2a
// path) and majority over W <= 15 planes (mode 0, the all-gather path).
// Every block of the one-chunk kernel starts with two dependent metadata
// loads (chunk row -> segment row) before its first data load, and a
// pre-voted chunk moves only 4.125 B per parameter, so that chain is a large
// share of a block's life (GPT-2: 67 % of HBM against the copy reference's
// 86 %, profiles/r3/lion_ab_nt_k4cap.txt).  Here both chunks' metadata loads
// are in flight together and, when both chunks are full, all 8 p vectors of
// the pair (and the pre-voted plane words) are loaded before the first use.
struct VoteCtx {
  const uint8_t* planes;
  int64_t plane_stride;
  const uint8_t* neg_plane;
  uint32_t live_mask;
  int world, n_live, tie;
};

template <bool MAJ>
__device__ __forceinline__ void vote_word(const VoteCtx& v, int64_t word, uint32_t& pos, uint32_t& neg) {
  if constexpr (MAJ) {
    uint32_t w[kMaxSliced], tb;
#pragma unroll
    for (int k = 0; k < kMaxSliced; ++k)
      w[k] = (v.live_mask >> k) & 1 ? reinterpret_cast<const uint32_t*>(v.planes + k * v.plane_stride)[word] : 0u;
    sliced_vote(w, v.world, v.n_live, v.tie, pos, neg, tb);
  } else {
    pos = reinterpret_cast<const uint32_t*>(v.planes)[word];
    neg = v.neg_plane ? reinterpret_cast<const uint32_t*>(v.neg_plane)[word] : ~pos;
  }
}

template <int DT>
__device__ __forceinline__ void apply8(float (&pv)[8], uint32_t pos, uint32_t neg, float decay, float neg_lr) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float delta = static_cast<float>(static_cast<int>((pos >> j) & 1) - static_cast<int>((neg >> j) & 1));
    pv[j] = __fmaf_rn(neg_lr, delta, Elem<DT>::rnd(pv[j] * decay));
  }
}

template <int DT, bool MAJ>
__device__ __forceinline__ void apply_chunk(const SegRow& r, int64_t start, const VoteCtx& v, float decay,
                                            float neg_lr) {
  using S = typename Elem<DT>::S;
  S* p = const_cast<S*>(static_cast<const S*>(r.p));
  const int sub = threadIdx.x & 3;
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t e = start + it * kSpan + threadIdx.x * 8;
    if (e >= r.n) break;
    uint32_t pos, neg;
    vote_word<MAJ>(v, (r.bit_off + e) >> 5, pos, neg);
    float pv[8];
    load8g<DT>(p, e, r.n, r.vec, pv);
    apply8<DT>(pv, (pos >> (8 * sub)) & 0xffu, (neg >> (8 * sub)) & 0xffu, decay, neg_lr);
    store8g<DT>(p, e, r.n, r.vec, pv);
  }
}

template <int DT, bool MAJ, int CPB>
__global__ void __launch_bounds__(kThreads)
lion_apply_pair_kernel(const int64_t* __restrict__ seg, const int64_t* __restrict__ chunks, int64_t n_chunks,
                       const uint8_t* __restrict__ planes, int64_t plane_stride, const uint8_t* __restrict__ alive,
                       int world, int tie, const uint8_t* __restrict__ neg_plane, float decay, float neg_lr) {
  using E = Elem<DT>;
  using S = typename E::S;
  // CPB chunks per block (kPairChunks): every chunk's metadata chain is in
  // flight together, and when all are full every p vector (and pre-voted
  // plane word) is loaded before the first use
  const int64_t c0 = CPB * static_cast<int64_t>(blockIdx.x);
  int64_t sidx[CPB], st[CPB];
  bool has[CPB];
#pragma unroll
  for (int c = 0; c < CPB; ++c) {
    has[c] = c0 + c < n_chunks;  // chunk 0 always exists
    const int64_t ci = has[c] ? c0 + c : c0;
    sidx[c] = chunks[2 * ci];
    st[c] = chunks[2 * ci + 1];
  }
  SegRow rs[CPB];
#pragma unroll
  for (int c = 0; c < CPB; ++c) rs[c] = load_seg(seg, sidx[c]);
  VoteCtx v{planes, plane_stride, neg_plane, 0u, world, 0, tie};
  if constexpr (MAJ) {
    for (int k = 0; k < world && k < kMaxSliced; ++k)
      if (alive[k]) {
        v.live_mask |= 1u << k;
        ++v.n_live;
      }
  }
  bool full = true;
#pragma unroll
  for (int c = 0; c < CPB; ++c) full = full && has[c] && rs[c].vec && st[c] + kChunk <= rs[c].n;
  if (full) {  // block-uniform
    const int sub = threadIdx.x & 3;
    Raw8<DT> rp[CPB * kIters];
    uint32_t pw[CPB * kIters], nw[CPB * kIters];
#pragma unroll
    for (int q = 0; q < CPB * kIters; ++q) {
      const int c = q / kIters;
      const int64_t e = st[c] + (q % kIters) * kSpan + threadIdx.x * 8;
      rp[q].load(static_cast<const S*>(rs[c].p) + e);
      // pre-voted: the plane words join the hoisted loads; majority: voted
      // below, one iteration's W words at a time (hoisting all of them spilled)
      if constexpr (!MAJ) vote_word<false>(v, (rs[c].bit_off + e) >> 5, pw[q], nw[q]);
    }
#pragma unroll
    for (int q = 0; q < CPB * kIters; ++q) {
      const int c = q / kIters;
      const int64_t e = st[c] + (q % kIters) * kSpan + threadIdx.x * 8;
      if constexpr (MAJ) vote_word<true>(v, (rs[c].bit_off + e) >> 5, pw[q], nw[q]);
      float pv[8];
      rp[q].unpack(pv);
      apply8<DT>(pv, (pw[q] >> (8 * sub)) & 0xffu, (nw[q] >> (8 * sub)) & 0xffu, decay, neg_lr);
      E::store8(const_cast<S*>(static_cast<const S*>(rs[c].p)) + e, pv);
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < CPB; ++c)
    if (has[c]) apply_chunk<DT, MAJ>(rs[c], st[c], v, decay, neg_lr);
}

// ----------------------------------------------------------------------- K4
// recv: [W][nbytes] shards gathered by all_to_all; out: voted positive bits;
// neg_out (optional): voted negative bits (only needed when ties map to 0).
// 4 bytes (32 coordinates) per thread, grid-stride.
// SLICED (W <= 15) and the byte-spread path are separate instantiations: the
// byte path's 32 counters would otherwise set the register budget of both
template <bool SLICED>
__global__ void __launch_bounds__(kThreads)
vote_reduce_kernel(const uint8_t* __restrict__ recv, int64_t nbytes, const uint8_t* __restrict__ alive,
                   int world, int tie, uint8_t* __restrict__ out, uint8_t* __restrict__ neg_out,
                   unsigned long long* __restrict__ ties) {
  const int64_t nwords = nbytes >> 2;  // nbytes % 4 == 0 guaranteed by the planner
  int n_live = 0;
  for (int k = 0; k < world; ++k) n_live += alive[k] != 0;
  uint32_t n_tie = 0;  // tie-rate telemetry (ties != nullptr)
  if constexpr (SLICED) {  // bit-sliced counters, every plane word loaded up front
    uint32_t live_mask = 0;
    for (int k = 0; k < world; ++k) live_mask |= static_cast<uint32_t>(alive[k] != 0) << k;
    // (a 16-byte-per-plane variant measured slower: 31 vs 40 % of HBM at Llama-3-8B)
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    int64_t w = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    {
      // two words per iteration, every plane load of both issued first
      // (one word per lane keeps only W dwords in flight per wave)
      for (; w + stride < nwords; w += 2 * stride) {
        uint32_t v[kMaxSliced], u[kMaxSliced];
#pragma unroll
        for (int k = 0; k < kMaxSliced; ++k) {
          const bool on = (live_mask >> k) & 1;
          v[k] = on ? reinterpret_cast<const uint32_t*>(recv + k * nbytes)[w] : 0u;
          u[k] = on ? reinterpret_cast<const uint32_t*>(recv + k * nbytes)[w + stride] : 0u;
        }
        uint32_t pos, ng, tb, pos2, ng2, tb2;
        sliced_vote(v, world, n_live, tie, pos, ng, tb);
        sliced_vote(u, world, n_live, tie, pos2, ng2, tb2);
        n_tie += __popc(tb) + __popc(tb2);
        reinterpret_cast<uint32_t*>(out)[w] = pos;
        reinterpret_cast<uint32_t*>(out)[w + stride] = pos2;
        if (neg_out != nullptr) {
          reinterpret_cast<uint32_t*>(neg_out)[w] = ng;
          reinterpret_cast<uint32_t*>(neg_out)[w + stride] = ng2;
        }
      }
    }
    for (; w < nwords; w += stride) {
      uint32_t v[kMaxSliced];
#pragma unroll
      for (int k = 0; k < kMaxSliced; ++k)
        v[k] = (live_mask >> k) & 1 ? reinterpret_cast<const uint32_t*>(recv + k * nbytes)[w] : 0u;
      uint32_t pos, ng, tb;
      sliced_vote(v, world, n_live, tie, pos, ng, tb);
      n_tie += __popc(tb);
      reinterpret_cast<uint32_t*>(out)[w] = pos;
      if (neg_out != nullptr) reinterpret_cast<uint32_t*>(neg_out)[w] = ng;
    }
  } else {  // wider worlds: byte-spread counters
    for (int64_t w = blockIdx.x * (int64_t)kThreads + threadIdx.x; w < nwords;
         w += (int64_t)gridDim.x * kThreads) {
      uint32_t cnt[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) cnt[j] = 0;
      for (int r0 = 0; r0 < world; r0 += 255) {
        const int r1 = min(world, r0 + 255);
        uint64_t acc[4] = {0, 0, 0, 0};
        for (int k = r0; k < r1; ++k) {
          if (!alive[k]) continue;
          const uint32_t v = reinterpret_cast<const uint32_t*>(recv + k * nbytes)[w];
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[b] += spread8(v >> (8 * b));
        }
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int j = 0; j < 8; ++j) cnt[8 * b + j] += static_cast<uint32_t>((acc[b] >> (8 * j)) & 0xffu);
      }
      uint32_t pos = 0, ng = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int twice = 2 * static_cast<int>(cnt[j]);
        const bool is_pos = n_live > 0 && (twice > n_live || (twice == n_live && tie == 2));
        const bool is_neg = n_live > 0 && (twice < n_live || (twice == n_live && tie == 0));
        n_tie += n_live > 0 && twice == n_live;
        pos |= static_cast<uint32_t>(is_pos) << j;
        ng |= static_cast<uint32_t>(is_neg) << j;
      }
      reinterpret_cast<uint32_t*>(out)[w] = pos;
      if (neg_out != nullptr) reinterpret_cast<uint32_t*>(neg_out)[w] = ng;
    }
  }
  if (ties != nullptr) {
    for (int off = 32; off > 0; off >>= 1) n_tie += __shfl_xor(n_tie, off);
    if ((threadIdx.x & 63) == 0 && n_tie) atomicAdd(ties, static_cast<unsigned long long>(n_tie));
  }
}

// ------------------------------------------------------------ gradient norm
// partial[chunk] = sum of g^2 (fp32) over the chunk's elements, one block per
// chunk of the same pointer table the update kernels walk; clip_coef_kernel
// then reduces the partials in a fixed order (deterministic) and stores
// out[0] = ||g||_2, out[1] = min(1, max_norm / (||g|| + 1e-6)) (NaN -> NaN,
// as clip_grad_norm_ without error_if_nonfinite).  No host sync: the update
// kernels read out[1] on the device.
template <int DT>
__global__ void __launch_bounds__(kThreads)
grad_sumsq_kernel(const int64_t* __restrict__ seg, const int64_t* __restrict__ chunks, float* __restrict__ partial) {
  const int64_t s = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const SegRow r = load_seg(seg, s);
  const typename Elem<DT>::S* g = static_cast<const typename Elem<DT>::S*>(r.g);
  float acc = 0.f;
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t e = start + it * kSpan + threadIdx.x * 8;
    if (e >= r.n) break;
    float gv[8];
    load8g<DT>(g, e, r.n, r.vec, gv);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __fmaf_rn(gv[j], gv[j], acc);
  }
  __shared__ float red[kThreads / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) t += red[i];
    partial[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(1024) clip_coef_kernel(const float* __restrict__ partial, int64_t n, float max_norm,
                                                         float* __restrict__ out) {
  // fp64 across up to ~10^6 chunk partials; four independent accumulators per
  // thread over 4-partial strides (one 1024-thread block: the single chain of
  // dependent fp64 adds took 415 us at Llama-3-8B's 1M partials)
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int64_t i = static_cast<int64_t>(threadIdx.x) * 4;
  for (; i + 3 < n; i += 4096) {
    a0 += partial[i];
    a1 += partial[i + 1];
    a2 += partial[i + 2];
    a3 += partial[i + 3];
  }
  for (; i < n; ++i) a0 += partial[i];  // the tail (< 4 partials) of the last thread's group
  double acc = (a0 + a1) + (a2 + a3);
  __shared__ double red[1024 / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 1024 / 64; ++i) t += red[i];
    const float norm = static_cast<float>(sqrt(t));
    const float coef = max_norm / (norm + 1e-6f);
    out[0] = norm;
    out[1] = (coef != coef) ? coef : fminf(coef, 1.f);
  }
}

// ------------------------------------------------------------ host launchers
#define DLION_DISPATCH(dt, ...)                         \
  switch (dt) {                                         \
    case kF32: { constexpr int DT = kF32; __VA_ARGS__; break; } \
    case kBF16: { constexpr int DT = kBF16; __VA_ARGS__; break; } \
    case kF16: { constexpr int DT = kF16; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;               \
  }

hipError_t launch_lion_local(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks,
                             float decay, float neg_lr, float b1, float omb1, float b2, float omb2,
                             const float* gscale, hipStream_t st) {
  if (n_chunks == 0) return hipSuccess;
  DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_local_kernel<DT>), dim3(n_chunks), dim3(kThreads), 0, st,
                                        seg, chunks, decay, neg_lr, b1, omb1, b2, omb2, gscale));
  return hipGetLastError();
}

hipError_t launch_lion_encode(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks,
                              uint8_t* bits, float b1, float omb1, float b2, float omb2, int update_m,
                              int stochastic, float rr, uint64_t seed, uint32_t step, const float* gscale,
                              hipStream_t st) {
  if (n_chunks == 0) return hipSuccess;
  const uint32_t lo = static_cast<uint32_t>(seed), hi = static_cast<uint32_t>(seed >> 32);
  if (stochastic) {
    DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_encode_kernel<DT, true>), dim3(n_chunks), dim3(kThreads), 0,
                                          st, seg, chunks, bits, b1, omb1, b2, omb2, update_m, rr, lo, hi, step, gscale));
  } else {
    DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_encode_kernel<DT, false>), dim3(n_chunks), dim3(kThreads), 0,
                                          st, seg, chunks, bits, b1, omb1, b2, omb2, update_m, rr, lo, hi, step, gscale));
  }
  return hipGetLastError();
}

hipError_t launch_lion_vote_apply(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks,
                                  const uint8_t* planes, int64_t plane_stride, const uint8_t* alive, int world,
                                  int mode, int tie, const uint8_t* neg, float decay, float neg_lr,
                                  const uint8_t* own, unsigned long long* agree, hipStream_t st) {
  if (n_chunks == 0) return hipSuccess;
  if (mode == 2 && agree == nullptr) {
    DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_apply_pair_kernel<DT, false, kPairChunks>), dim3((n_chunks + kPairChunks - 1) / kPairChunks),
                                          dim3(kThreads), 0, st, seg, chunks, n_chunks, planes, plane_stride, alive,
                                          world, tie, neg, decay, neg_lr));
    return hipGetLastError();
  }
  if (mode == 0 && world <= kMaxSliced && agree == nullptr) {
    DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_apply_pair_kernel<DT, true, kPairChunks>), dim3((n_chunks + kPairChunks - 1) / kPairChunks),
                                          dim3(kThreads), 0, st, seg, chunks, n_chunks, planes, plane_stride, alive,
                                          world, tie, neg, decay, neg_lr));
    return hipGetLastError();
  }
  if (mode == 2 || (mode == 0 && world <= kMaxSliced)) {
    DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_vote_apply32_kernel<DT>), dim3(n_chunks), dim3(kThreads), 0, st,
                                          seg, chunks, planes, plane_stride, alive, world, mode, tie, neg, decay,
                                          neg_lr, own, agree));
    return hipGetLastError();
  }
  DLION_DISPATCH(dt, hipLaunchKernelGGL((lion_vote_apply_kernel<DT>), dim3(n_chunks), dim3(kThreads), 0, st,
                                        seg, chunks, planes, plane_stride, alive, world, mode, tie, neg, decay,
                                        neg_lr, own, agree));
  return hipGetLastError();
}

hipError_t launch_grad_sumsq(int dt, const int64_t* seg, const int64_t* chunks, int64_t n_chunks, float* partial,
                             hipStream_t st) {
  if (n_chunks == 0) return hipSuccess;
  DLION_DISPATCH(dt, hipLaunchKernelGGL((grad_sumsq_kernel<DT>), dim3(n_chunks), dim3(kThreads), 0, st, seg, chunks,
                                        partial));
  return hipGetLastError();
}

hipError_t launch_clip_coef(const float* partial, int64_t n, float max_norm, float* out, hipStream_t st) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1024), 0, st, partial, n, max_norm, out);
  return hipGetLastError();
}

hipError_t launch_vote_reduce(const uint8_t* recv, int64_t nbytes, const uint8_t* alive, int world, int tie,
                              uint8_t* out, uint8_t* neg_out, unsigned long long* ties, hipStream_t st) {
  const int64_t nwords = nbytes >> 2;
  if (nwords == 0) return hipSuccess;
  const int64_t per_block = static_cast<int64_t>(kThreads) * (world <= kMaxSliced ? kK4Unroll : 1);
  int64_t blocks = (nwords + per_block - 1) / per_block;
  if (blocks > kK4MaxBlocks) blocks = kK4MaxBlocks;
  if (world <= kMaxSliced)
    hipLaunchKernelGGL(vote_reduce_kernel<true>, dim3(blocks), dim3(kThreads), 0, st, recv, nbytes, alive, world, tie,
                       out, neg_out, ties);
  else
    hipLaunchKernelGGL(vote_reduce_kernel<false>, dim3(blocks), dim3(kThreads), 0, st, recv, nbytes, alive, world,
                       tie, out, neg_out, ties);
  return hipGetLastError();
}

}  // namespace dlion

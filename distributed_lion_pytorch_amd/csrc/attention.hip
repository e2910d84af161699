// Causal flash attention (forward + backward, optional dropout) for gfx950.
//
// Replaces PyTorch SDPA (aotriton on ROCm) plus the layout copies around it
// (q/k/v unbind + stack in backward, output transpose) in the GPT-2/Llama
// blocks.  Inputs are read in their native strided layout ([B,T,3,H,D] packed
// qkv for GPT-2, separate [B,T,H,D] / [B,T,Hkv,D] for Llama GQA) and the
// gradients are written straight into the packed dqkv layout.
//
// Design (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's
// operand"): every wave owns one 32x32 tile pair and uses
// v_mfma_f32_32x32x16_bf16 only.  Scores are computed TRANSPOSED,
// S^T = K Q^T, so the accumulator has the query on the lane and 16 keys in
// registers: the softmax row-reduction is 15 in-register ops + one
// cross-half shuffle, and P^T feeds O^T += V^T P^T with no lane movement.
// The permuted-k operand (V^T rows) comes from a V^T copy in HBM (two 8-byte
// loads per fragment).  Backward uses two kernels without atomics:
//   dKV: per 32-key tile, S = Q K^T orientation (key on the lane), loops over
//        query tiles accumulating dV += Pd^T dO and dK += dS^T Q in registers;
//   dQ : per 32-query tile, forward orientation, dQ += dS K.
// Dropout: keep(q, key) is a stateless hash of (seed, b*H+h, q, key) with
// 16-bit resolution, so forward and both backward kernels regenerate the
// identical mask in any register layout.
#include <cstdlib>

#include "common.h"
#include "attention.h"

namespace dlion {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));



__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// 32 random bits shared by keys (2i, 2i+1) of query q; key & 1 picks the half
// (low 16 bits: even key).  Keep tests run in the high half so the low half
// needs one shift and the high half none: with thr_hi = thresh16 << 16,
//   keep(even) = (hash << 16) >= thr_hi,  keep(odd) = hash >= thr_hi.
__device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint32_t bh, uint32_t q, uint32_t key) {
  return lowbias32(seed ^ (bh * 0x9E3779B9u) ^ (q * 0x85EBCA6Bu) ^ ((key >> 1) * 0xC2B2AE35u));
}

// x op x(lane ^ 32) via v_permlane32_swap (guide T12): no LDS round trip,
// and max / sum are symmetric so the swapped pair needs no lane select
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float a = __uint_as_float(r[0]), b = __uint_as_float(r[1]);
  return a > b ? a : b;
}
__device__ __forceinline__ float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// forward online softmax: rescale O only when a row max grew by more than this (log2 units)
constexpr float kDeferLog2 = 8.f;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 ld8(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
// permuted-k fragment: elements 0..3 from p[0..3], 4..7 from p[8..11]
__device__ __forceinline__ bf16x8 ld4x2(const __bf16* p) {
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 8);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// accumulator registers 8s..8s+7 as a bf16 operand fragment (k-step s)
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(x[8 * s + j]);
  return r;
}
__device__ __forceinline__ int acc_row(int reg, int hf) { return (reg & 3) + 8 * (reg >> 2) + 4 * hf; }

// (blockIdx, wave) -> (bh, tile): the 4 waves of a block take 4 consecutive
// 32-row tiles of ONE head (their K/V or Q/dO fragment loads coincide and hit
// the CU's L1), all blocks of a head share an XCD (bijective remap, guide §5)
// so a head's K/V stay in that XCD's L2, heads are walked one after the other
// (few heads in flight -> the working set fits L2), heavy tiles first.
// Returns false for waves past the last tile.
__device__ __forceinline__ bool tile_map(int order, int nbh, int ntiles, bool heavy_high, int& bh, int& tile) {
  if (order == 0) {  // waves walk heads fastest; globally heaviest tiles first
    const int64_t gw = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (gw >= static_cast<int64_t>(nbh) * ntiles) return false;
    const int t = static_cast<int>(gw / nbh);
    tile = heavy_high ? ntiles - 1 - t : t;
    bh = static_cast<int>(gw % nbh);
    return true;
  }
  const int bpb = (ntiles + 3) >> 2;  // blocks per head
  const int nblocks = nbh * bpb;
  const int i = blockIdx.x, xcd = i & 7, q = nblocks >> 3, rr = nblocks & 7;
  const int L = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (i >> 3);
  bh = L / bpb;
  int blk = L - bh * bpb;
  if (heavy_high) blk = bpb - 1 - blk;
  tile = blk * 4 + (threadIdx.x >> 6);
  return bh < nbh && tile < ntiles;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ------------------------------------------------------------------ forward
template <int D, bool DROP>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5;
  int bh, qtile;
  if (!tile_map(a.order, a.B * a.H, a.T >> 5, true, bh, qtile)) return;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int q = qtile * 32 + r;

  bf16x8 qf[D / 16];
  const __bf16* qp = a.q + b * a.q_sb + static_cast<int64_t>(q) * a.q_st + h * a.q_sh + 8 * hf;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) qf[s] = ld8(qp + 16 * s);

  f32x16 oacc[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) oacc[t] = zero16();
  float m = -INFINITY, l = 0.f;
  const __bf16* kbase = a.k + b * a.k_sb + hk * a.k_sh + 8 * hf;
  const __bf16* vtb = a.vt + static_cast<int64_t>(b * a.Hkv + hk) * D * a.ldt + 4 * hf;

  // register double-buffering with two NAMED fragment sets (A, B) and a 2x
  // unrolled loop: tile kt+1 loads into one set while tile kt computes from the
  // other -- no per-iteration register copies (a runtime-indexed or copied
  // buffer costs ~64 v_mov per tile)
  bf16x8 ka[D / 16], va[2][D / 32], kb_[D / 16], vb[2][D / 32];
  auto load_kv = [&](int kt, bf16x8(&kf)[D / 16], bf16x8(&vf)[2][D / 32]) {
    const __bf16* kp = kbase + static_cast<int64_t>(kt * 32 + r) * a.k_st;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) kf[ks] = ld8(kp + 16 * ks);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int t = 0; t < D / 32; ++t)
        vf[s2][t] = ld4x2(vtb + static_cast<int64_t>(32 * t + r) * a.ldt + kt * 32 + 16 * s2);
  };
  const uint32_t hbase = a.seed ^ (static_cast<uint32_t>(bh) * 0x9E3779B9u) ^ (static_cast<uint32_t>(q) * 0x85EBCA6Bu);
  const uint32_t thr_hi = a.thresh16 << 16;
  auto tile = [&](int kt, const bf16x8(&kc)[D / 16], const bf16x8(&vc)[2][D / 32]) {
    const int kb = kt * 32;
    f32x16 s = zero16();
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) s = mfma32(kc[ks], qf[ks], s);
    if (kt == qtile) {  // causal mask only on the diagonal tile (wave-uniform branch)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg)
        if (kb + acc_row(reg, hf) > q) s[reg] = -INFINITY;
    }
    // row max on the raw scores (scale > 0); the scale is folded into the
    // exponent's FMA below instead of a separate multiply pass
    float tmax = s[0];
#pragma unroll
    for (int reg = 1; reg < 16; ++reg) tmax = fmaxf(tmax, s[reg]);
    tmax = xmax32(tmax) * a.scale_log2;
    // deferred rescale (guide T13): keep the running max while no row of the
    // wave grew by more than kDeferLog2 -- P stays <= 2^kDeferLog2, exact in
    // fp32 l / O, and the O-wide rescale pass is skipped on most tiles
    float alpha = 1.f;
    if (!__all(tmax - m <= kDeferLog2)) {
      const float mn = fmaxf(m, tmax);
      alpha = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
#pragma unroll
      for (int t = 0; t < D / 32; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[t][i] *= alpha;
    }
    float rs = 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[reg], a.scale_log2, -m));
      rs += p;
      s[reg] = p;
    }
    l = l * alpha + xsum32(rs);
    if constexpr (DROP) {  // 1/(1-p) is applied once to O at the end
#pragma unroll
      for (int reg = 0; reg < 16; reg += 2) {  // regs (2i, 2i+1) hold keys (2j, 2j+1)
        const uint32_t key = kb + acc_row(reg, hf);
        const uint32_t hsh = lowbias32(hbase ^ ((key >> 1) * 0xC2B2AE35u));
        // 16-bit halves compared in the high half: (h & 0xffff) < t <=> (h << 16) < (t << 16)
        if ((hsh << 16) < thr_hi) s[reg] = 0.f;
        if (hsh < thr_hi) s[reg + 1] = 0.f;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = acc_frag(s, s2);
#pragma unroll
      for (int t = 0; t < D / 32; ++t) oacc[t] = mfma32(vc[s2][t], pf, oacc[t]);
    }
  };
  load_kv(0, ka, va);
  int kt = 0;
  for (; kt < qtile; kt += 2) {  // pairs (kt, kt+1), both <= qtile
    load_kv(kt + 1, kb_, vb);
    tile(kt, ka, va);
    if (kt + 2 <= qtile) load_kv(kt + 2, ka, va);
    tile(kt + 1, kb_, vb);
  }
  if (kt == qtile) tile(kt, ka, va);  // odd tile count: the last tile sits in set A
  const float inv_l = (DROP ? a.inv_keep : 1.f) / l;
  __bf16* op = a.out + b * a.o_sb + static_cast<int64_t>(q) * a.o_st + h * a.o_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 w;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = static_cast<__bf16>(oacc[t][4 * g + i] * inv_l);
      *reinterpret_cast<bf16x4*>(op + 32 * t + 8 * g + 4 * hf) = w;
    }
  if (hf == 0) a.lse[static_cast<int64_t>(bh) * a.T + q] = m + log2f(l);
}

// ------------------------------------------------- forward, LDS-shared K / V
// Same math as attn_fwd_kernel, but the 4 waves of a block own 4 consecutive
// query tiles of ONE head and share every K / V^T tile through LDS: one
// cooperative 16-byte load per thread per operand instead of 4 private copies
// per wave (the private-copy kernel streams ~1 GB of L2/MALL traffic per
// GPT-2 layer and is cache-bandwidth bound).  Global loads for tile kt+1 are
// issued before tile kt's math and written to the other LDS buffer after it
// (guide T14).  Waves whose causal range ended idle through the block's
// remaining tiles (the last <= 3) but keep the barriers.
constexpr int kKPad = 8;   // K tile rows: 64 + 8 bf16 (144 B) -- breaks the 128-B bank period
constexpr int kVPad = 8;   // V^T tile rows: 32 + 8 bf16 (80 B)

template <int D, bool DROP>
__global__ void __launch_bounds__(256) attn_fwd_lds_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 ks_[2][32][D + kKPad];
  __shared__ __attribute__((aligned(16))) __bf16 vs_[2][D][32 + kVPad];
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5, w = threadIdx.x >> 6;
  const int ntiles = a.T >> 5, ngroups = (ntiles + 3) >> 2, nbh = a.B * a.H;
  // heads fastest, heavy (late) query groups first
  const int bh = static_cast<int>(blockIdx.x % nbh);
  const int grp = ngroups - 1 - static_cast<int>(blockIdx.x / nbh);
  const int qtile = grp * 4 + w;
  const int last = min(grp * 4 + 3, ntiles - 1);  // block-uniform loop bound
  const bool active = qtile < ntiles;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int q = qtile * 32 + r;

  bf16x8 qf[D / 16];
  if (active) {
    const __bf16* qp = a.q + b * a.q_sb + static_cast<int64_t>(q) * a.q_st + h * a.q_sh + 8 * hf;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) qf[s] = ld8(qp + 16 * s);
  }
  f32x16 oacc[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) oacc[t] = zero16();
  float m = -INFINITY, l = 0.f;

  // cooperative tile load: K [32 keys][D] and V^T [D][32 keys], 16 B per thread-chunk
  constexpr int KCH = 32 * D / 8, VCH = D * 32 / 8;  // 16-byte chunks per tile
  constexpr int KPT = (KCH + 255) / 256, VPT = (VCH + 255) / 256;
  const __bf16* kg = a.k + b * a.k_sb + hk * a.k_sh;
  const __bf16* vg = a.vt + static_cast<int64_t>(b * a.Hkv + hk) * D * a.ldt;
  uint4 kreg[KPT], vreg[VPT];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / (D / 8), col = (c % (D / 8)) * 8;
      if (c < KCH) kreg[i] = *reinterpret_cast<const uint4*>(kg + static_cast<int64_t>(kt * 32 + row) * a.k_st + col);
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / 4, col = (c % 4) * 8;
      if (c < VCH) vreg[i] = *reinterpret_cast<const uint4*>(vg + static_cast<int64_t>(row) * a.ldt + kt * 32 + col);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / (D / 8), col = (c % (D / 8)) * 8;
      if (c < KCH) *reinterpret_cast<uint4*>(&ks_[buf][row][col]) = kreg[i];
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / 4, col = (c % 4) * 8;
      if (c < VCH) *reinterpret_cast<uint4*>(&vs_[buf][row][col]) = vreg[i];
    }
  };

  const uint32_t hbase = a.seed ^ (static_cast<uint32_t>(bh) * 0x9E3779B9u) ^ (static_cast<uint32_t>(q) * 0x85EBCA6Bu);
  const uint32_t thr_hi = a.thresh16 << 16;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt <= last; ++kt) {
    const int buf = kt & 1;
    if (kt < last) gload(kt + 1);
    if (active && kt <= qtile) {  // wave-uniform
      const int kb = kt * 32;
      f32x16 s = zero16();
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) s = mfma32(*reinterpret_cast<const bf16x8*>(&ks_[buf][r][16 * ks + 8 * hf]),
                                                     qf[ks], s);
      if (kt == qtile) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          if (kb + acc_row(reg, hf) > q) s[reg] = -INFINITY;
      }
      float tmax = s[0];
#pragma unroll
      for (int reg = 1; reg < 16; ++reg) tmax = fmaxf(tmax, s[reg]);
      tmax = xmax32(tmax) * a.scale_log2;
      float alpha = 1.f;
      if (!__all(tmax - m <= kDeferLog2)) {
        const float mn = fmaxf(m, tmax);
        alpha = __builtin_amdgcn_exp2f(m - mn);
        m = mn;
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) oacc[t][i] *= alpha;
      }
      float rs = 0.f;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[reg], a.scale_log2, -m));
        rs += p;
        s[reg] = p;
      }
      l = l * alpha + xsum32(rs);
      if constexpr (DROP) {
#pragma unroll
        for (int reg = 0; reg < 16; reg += 2) {
          const uint32_t key = kb + acc_row(reg, hf);
          const uint32_t hsh = lowbias32(hbase ^ ((key >> 1) * 0xC2B2AE35u));
          if ((hsh << 16) < thr_hi) s[reg] = 0.f;
          if (hsh < thr_hi) s[reg + 1] = 0.f;
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = acc_frag(s, s2);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          const __bf16* vp = &vs_[buf][32 * t + r][16 * s2 + 4 * hf];
          oacc[t] = mfma32(ld4x2(vp), pf, oacc[t]);
        }
      }
    }
    if (kt < last) swrite(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  const float inv_l = (DROP ? a.inv_keep : 1.f) / l;
  __bf16* op = a.out + b * a.o_sb + static_cast<int64_t>(q) * a.o_st + h * a.o_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 wv;
#pragma unroll
      for (int i = 0; i < 4; ++i) wv[i] = static_cast<__bf16>(oacc[t][4 * g + i] * inv_l);
      *reinterpret_cast<bf16x4*>(op + 32 * t + 8 * g + 4 * hf) = wv;
    }
  if (hf == 0) a.lse[static_cast<int64_t>(bh) * a.T + q] = m + log2f(l);
}

// --------------------------------------------------------------- backward dQ
template <int D, bool DROP>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5;
  int bh, qtile;
  if (!tile_map(a.order, a.B * a.H, a.T >> 5, true, bh, qtile)) return;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int q = qtile * 32 + r;

  bf16x8 qf[D / 16], dof[D / 16];
  const __bf16* qp = a.q + b * a.q_sb + static_cast<int64_t>(q) * a.q_st + h * a.q_sh + 8 * hf;
  const __bf16* dop = a.dout + b * a.o_sb + static_cast<int64_t>(q) * a.o_st + h * a.o_sh + 8 * hf;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    qf[s] = ld8(qp + 16 * s);
    dof[s] = ld8(dop + 16 * s);
  }
  const float lse2 = a.lse[static_cast<int64_t>(bh) * a.T + q];
  const float dlt = a.delta[static_cast<int64_t>(bh) * a.T + q];
  const uint32_t thr_hi = a.thresh16 << 16;
  f32x16 dq[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dq[t] = zero16();
  const __bf16* kbase = a.k + b * a.k_sb + hk * a.k_sh + 8 * hf;
  const __bf16* vbase = a.v + b * a.v_sb + hk * a.v_sh + 8 * hf;
  const __bf16* ktb = a.kt + static_cast<int64_t>(b * a.Hkv + hk) * D * a.ldt + 4 * hf;

  // K / V rows and K^T fragments of tile kt+1 are prefetched during tile kt
  // into the other of two named fragment sets (2x unrolled, no copies)
  bf16x8 ka[D / 16], va[D / 16], ta[2][D / 32], kb2[D / 16], vb2[D / 16], tb2[2][D / 32];
  auto load_kv = [&](int kt, bf16x8(&kf)[D / 16], bf16x8(&vf)[D / 16], bf16x8(&tf)[2][D / 32]) {
    const __bf16* kp = kbase + static_cast<int64_t>(kt * 32 + r) * a.k_st;
    const __bf16* vp = vbase + static_cast<int64_t>(kt * 32 + r) * a.v_st;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      kf[ks] = ld8(kp + 16 * ks);
      vf[ks] = ld8(vp + 16 * ks);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int t = 0; t < D / 32; ++t)
        tf[s2][t] = ld4x2(ktb + static_cast<int64_t>(32 * t + r) * a.ldt + kt * 32 + 16 * s2);
  };
  const uint32_t hq = a.seed ^ (static_cast<uint32_t>(bh) * 0x9E3779B9u) ^ (static_cast<uint32_t>(q) * 0x85EBCA6Bu);
  auto tile = [&](int kt, const bf16x8(&kc)[D / 16], const bf16x8(&vc)[D / 16], const bf16x8(&tc)[2][D / 32]) {
    const int kb = kt * 32;
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      s = mfma32(kc[ks], qf[ks], s);
      dp = mfma32(vc[ks], dof[ks], dp);
    }
#pragma unroll
    for (int reg = 0; reg < 16; reg += 2) {
      const int key = kb + acc_row(reg, hf);  // even: regs (reg, reg+1) = keys (key, key+1)
      uint32_t hsh = 0;
      if constexpr (DROP) hsh = lowbias32(hq ^ ((static_cast<uint32_t>(key) >> 1) * 0xC2B2AE35u));
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int kk = key + e;
        float p = (kt == qtile && kk > q) ? 0.f : __builtin_amdgcn_exp2f(__builtin_fmaf(s[reg + e], a.scale_log2, -lse2));
        float dpv = dp[reg + e];
        if constexpr (DROP) dpv = ((e == 0 ? hsh << 16 : hsh) >= thr_hi) ? dpv * a.inv_keep : 0.f;
        s[reg + e] = p * (dpv - dlt);  // dS^T
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 dsf = acc_frag(s, s2);
#pragma unroll
      for (int t = 0; t < D / 32; ++t) dq[t] = mfma32(dsf, tc[s2][t], dq[t]);
    }
  };
  load_kv(0, ka, va, ta);
  int kt = 0;
  for (; kt < qtile; kt += 2) {
    load_kv(kt + 1, kb2, vb2, tb2);
    tile(kt, ka, va, ta);
    if (kt + 2 <= qtile) load_kv(kt + 2, ka, va, ta);
    tile(kt + 1, kb2, vb2, tb2);
  }
  if (kt == qtile) tile(kt, ka, va, ta);
  // dq[t]: rows = q (registers), cols = d (lane)
  __bf16* base = a.dq + b * a.dq_sb + h * a.dq_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int qq = qtile * 32 + acc_row(reg, hf);
      base[static_cast<int64_t>(qq) * a.dq_st + 32 * t + r] = static_cast<__bf16>(dq[t][reg] * a.scale);
    }
}

// ---------------------------------------------- cooperative LDS tile staging
// A 32-row x D tile (rows at `stride` elements) and a D-row x 32-column tile
// of a [.., D, T] transposed operand, moved 16 B per thread-chunk by a
// 256-thread block: global -> registers (issued early) -> LDS (written late).
template <int D>
struct RowTile {  // [32][D + kKPad]
  static constexpr int CH = 32 * D / 8, PT = (CH + 255) / 256;
  uint4 reg[PT];
  __device__ __forceinline__ void load(const __bf16* base, int64_t stride) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / (D / 8), col = (c % (D / 8)) * 8;
      if (c < CH) reg[i] = *reinterpret_cast<const uint4*>(base + static_cast<int64_t>(row) * stride + col);
    }
  }
  __device__ __forceinline__ void store(__bf16 (*dst)[D + kKPad]) const {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / (D / 8), col = (c % (D / 8)) * 8;
      if (c < CH) *reinterpret_cast<uint4*>(&dst[row][col]) = reg[i];
    }
  }
};
template <int D>
struct ColTile {  // [D][32 + kVPad]
  static constexpr int CH = D * 32 / 8, PT = (CH + 255) / 256;
  uint4 reg[PT];
  __device__ __forceinline__ void load(const __bf16* base, int64_t ldt) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / 4, col = (c % 4) * 8;
      if (c < CH) reg[i] = *reinterpret_cast<const uint4*>(base + static_cast<int64_t>(row) * ldt + col);
    }
  }
  __device__ __forceinline__ void store(__bf16 (*dst)[32 + kVPad]) const {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / 4, col = (c % 4) * 8;
      if (c < CH) *reinterpret_cast<uint4*>(&dst[row][col]) = reg[i];
    }
  }
};

// --------------------------------------------------- backward dQ, LDS-shared
// 4 waves = 4 consecutive query tiles of one head; K, V (rows) and K^T tiles
// staged once per block per key tile.
template <int D, bool DROP>
__global__ void __launch_bounds__(256) attn_bwd_dq_lds_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 ks_[2][32][D + kKPad];
  __shared__ __attribute__((aligned(16))) __bf16 vs_[2][32][D + kKPad];
  __shared__ __attribute__((aligned(16))) __bf16 ts_[2][D][32 + kVPad];
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5, w = threadIdx.x >> 6;
  const int ntiles = a.T >> 5, ngroups = (ntiles + 3) >> 2, nbh = a.B * a.H;
  const int bh = static_cast<int>(blockIdx.x % nbh);
  const int grp = ngroups - 1 - static_cast<int>(blockIdx.x / nbh);
  const int qtile = grp * 4 + w;
  const int last = min(grp * 4 + 3, ntiles - 1);
  const bool active = qtile < ntiles;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int q = qtile * 32 + r;

  bf16x8 qf[D / 16], dof[D / 16];
  float lse2 = 0.f, dlt = 0.f;
  if (active) {
    const __bf16* qp = a.q + b * a.q_sb + static_cast<int64_t>(q) * a.q_st + h * a.q_sh + 8 * hf;
    const __bf16* dop = a.dout + b * a.o_sb + static_cast<int64_t>(q) * a.o_st + h * a.o_sh + 8 * hf;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      qf[s] = ld8(qp + 16 * s);
      dof[s] = ld8(dop + 16 * s);
    }
    lse2 = a.lse[static_cast<int64_t>(bh) * a.T + q];
    dlt = a.delta[static_cast<int64_t>(bh) * a.T + q];
  }
  const uint32_t thr_hi = a.thresh16 << 16;
  const uint32_t hq = a.seed ^ (static_cast<uint32_t>(bh) * 0x9E3779B9u) ^ (static_cast<uint32_t>(q) * 0x85EBCA6Bu);
  f32x16 dq[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dq[t] = zero16();
  const __bf16* kg = a.k + b * a.k_sb + hk * a.k_sh;
  const __bf16* vg = a.v + b * a.v_sb + hk * a.v_sh;
  const __bf16* tg = a.kt + static_cast<int64_t>(b * a.Hkv + hk) * D * a.ldt;
  RowTile<D> kr, vr;
  ColTile<D> tr;
  auto gload = [&](int kt) {
    kr.load(kg + static_cast<int64_t>(kt * 32) * a.k_st, a.k_st);
    vr.load(vg + static_cast<int64_t>(kt * 32) * a.v_st, a.v_st);
    tr.load(tg + kt * 32, a.ldt);
  };
  auto swrite = [&](int buf) {
    kr.store(ks_[buf]);
    vr.store(vs_[buf]);
    tr.store(ts_[buf]);
  };
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt <= last; ++kt) {
    const int buf = kt & 1;
    if (kt < last) gload(kt + 1);
    if (active && kt <= qtile) {
      const int kb = kt * 32;
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        s = mfma32(*reinterpret_cast<const bf16x8*>(&ks_[buf][r][16 * ks + 8 * hf]), qf[ks], s);
        dp = mfma32(*reinterpret_cast<const bf16x8*>(&vs_[buf][r][16 * ks + 8 * hf]), dof[ks], dp);
      }
#pragma unroll
      for (int reg = 0; reg < 16; reg += 2) {
        const int key = kb + acc_row(reg, hf);
        uint32_t hsh = 0;
        if constexpr (DROP) hsh = lowbias32(hq ^ ((static_cast<uint32_t>(key) >> 1) * 0xC2B2AE35u));
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int kk = key + e;
          float p = (kt == qtile && kk > q) ? 0.f
                                            : __builtin_amdgcn_exp2f(__builtin_fmaf(s[reg + e], a.scale_log2, -lse2));
          float dpv = dp[reg + e];
          if constexpr (DROP) dpv = ((e == 0 ? hsh << 16 : hsh) >= thr_hi) ? dpv * a.inv_keep : 0.f;
          s[reg + e] = p * (dpv - dlt);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 dsf = acc_frag(s, s2);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) dq[t] = mfma32(dsf, ld4x2(&ts_[buf][32 * t + r][16 * s2 + 4 * hf]), dq[t]);
      }
    }
    if (kt < last) swrite(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  __bf16* base = a.dq + b * a.dq_sb + h * a.dq_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int qq = qtile * 32 + acc_row(reg, hf);
      base[static_cast<int64_t>(qq) * a.dq_st + 32 * t + r] = static_cast<__bf16>(dq[t][reg] * a.scale);
    }
}

// -------------------------------------------------- backward dKV, LDS-shared
// 4 waves = 4 consecutive key tiles of one (b, kv-head); every query tile of
// every head in the GQA group is staged once per block: Q, dO (rows), Q^T,
// dO^T (columns) and the 32 lse / delta values.
template <int D, bool DROP>
__global__ void __launch_bounds__(256) attn_bwd_dkv_lds_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 qs_[2][32][D + kKPad];
  __shared__ __attribute__((aligned(16))) __bf16 ds_[2][32][D + kKPad];
  __shared__ __attribute__((aligned(16))) __bf16 qts_[2][D][32 + kVPad];
  __shared__ __attribute__((aligned(16))) __bf16 dts_[2][D][32 + kVPad];
  __shared__ __attribute__((aligned(16))) float ls_[2][2][32];  // [buf][lse | delta][q]
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5, w = threadIdx.x >> 6;
  const int ntiles = a.T >> 5, ngroups = (ntiles + 3) >> 2, nbhk = a.B * a.Hkv;
  // heads fastest; low key groups (most query tiles) first
  const int bhk = static_cast<int>(blockIdx.x % nbhk);
  const int grp = static_cast<int>(blockIdx.x / nbhk);
  const int ktile = grp * 4 + w;
  const bool active = ktile < ntiles;
  const int first = grp * 4;  // block's first query tile = its lowest key tile
  const int b = bhk / a.Hkv, hk = bhk % a.Hkv, group = a.H / a.Hkv;
  const int kb = ktile * 32, key = kb + r;

  bf16x8 kf[D / 16], vf[D / 16];
  if (active) {
    const __bf16* kp = a.k + b * a.k_sb + static_cast<int64_t>(key) * a.k_st + hk * a.k_sh + 8 * hf;
    const __bf16* vp = a.v + b * a.v_sb + static_cast<int64_t>(key) * a.v_st + hk * a.v_sh + 8 * hf;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      kf[s] = ld8(kp + 16 * s);
      vf[s] = ld8(vp + 16 * s);
    }
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) {
    dk[t] = zero16();
    dv[t] = zero16();
  }
  const uint32_t thr_hi = a.thresh16 << 16, kshift = (key & 1) ? 0u : 16u;
  RowTile<D> qr, dr;
  ColTile<D> qtr, dtr;
  float lsr = 0.f;  // threads 0..63: lse (0..31) / delta (32..63) of the staged tile
  const int nq = ntiles - first;  // query tiles per head
  const int total = group * nq;   // (head, query tile) steps, head-major
  auto gload = [&](int i) {
    const int gh = i / nq, qt = first + i % nq;
    const int h = hk * group + gh, bh = b * a.H + h;
    const int64_t qrow = static_cast<int64_t>(qt * 32);
    qr.load(a.q + b * a.q_sb + h * a.q_sh + qrow * a.q_st, a.q_st);
    dr.load(a.dout + b * a.o_sb + h * a.o_sh + qrow * a.o_st, a.o_st);
    qtr.load(a.qt + static_cast<int64_t>(bh) * D * a.ldt + qt * 32, a.ldt);
    dtr.load(a.dot + static_cast<int64_t>(bh) * D * a.ldt + qt * 32, a.ldt);
    if (threadIdx.x < 64) {
      const float* src = (threadIdx.x < 32 ? a.lse : a.delta) + static_cast<int64_t>(bh) * a.T + qt * 32;
      lsr = src[threadIdx.x & 31];
    }
  };
  auto swrite = [&](int buf) {
    qr.store(qs_[buf]);
    dr.store(ds_[buf]);
    qtr.store(qts_[buf]);
    dtr.store(dts_[buf]);
    if (threadIdx.x < 64) ls_[buf][threadIdx.x >> 5][threadIdx.x & 31] = lsr;
  };
  gload(0);
  swrite(0);
  __syncthreads();
  for (int i = 0; i < total; ++i) {
    const int buf = i & 1;
    if (i + 1 < total) gload(i + 1);
    const int gh = i / nq, qt = first + i % nq;
    if (active && qt >= ktile) {
      const int bh = b * a.H + hk * group + gh;
      const int qb = qt * 32;
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        s = mfma32(*reinterpret_cast<const bf16x8*>(&qs_[buf][r][16 * ks + 8 * hf]), kf[ks], s);
        dp = mfma32(*reinterpret_cast<const bf16x8*>(&ds_[buf][r][16 * ks + 8 * hf]), vf[ks], dp);
      }
      const uint32_t hkey = a.seed ^ (static_cast<uint32_t>(bh) * 0x9E3779B9u) ^
                            ((static_cast<uint32_t>(key) >> 1) * 0xC2B2AE35u);
      const uint32_t hq = static_cast<uint32_t>(qb + 4 * hf) * 0x85EBCA6Bu;
      f32x16 pd;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = acc_row(reg, hf), qq = qb + row;
        const float p = (qt == ktile && key > qq)
                            ? 0.f
                            : __builtin_amdgcn_exp2f(__builtin_fmaf(s[reg], a.scale_log2, -ls_[buf][0][row]));
        float dpv = dp[reg];
        float pdv = p;
        if constexpr (DROP) {
          const uint32_t rowc = static_cast<uint32_t>((reg & 3) + 8 * (reg >> 2)) * 0x85EBCA6Bu;
          const uint32_t hsh = lowbias32(hkey ^ (hq + rowc));
          const bool kp_ = (hsh << kshift) >= thr_hi;
          dpv = kp_ ? dpv * a.inv_keep : 0.f;
          pdv = kp_ ? p * a.inv_keep : 0.f;
        }
        pd[reg] = pdv;
        s[reg] = p * (dpv - ls_[buf][1][row]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = acc_frag(pd, s2);
        const bf16x8 dsf = acc_frag(s, s2);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          dv[t] = mfma32(pf, ld4x2(&dts_[buf][32 * t + r][16 * s2 + 4 * hf]), dv[t]);
          dk[t] = mfma32(dsf, ld4x2(&qts_[buf][32 * t + r][16 * s2 + 4 * hf]), dk[t]);
        }
      }
    }
    if (i + 1 < total) swrite(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  __bf16* dkb = a.dk + b * a.dk_sb + hk * a.dk_sh;
  __bf16* dvb = a.dv + b * a.dk_sb + hk * a.dk_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int64_t off = static_cast<int64_t>(kb + acc_row(reg, hf)) * a.dk_st + 32 * t + r;
      dkb[off] = static_cast<__bf16>(dk[t][reg] * a.scale);
      dvb[off] = static_cast<__bf16>(dv[t][reg]);
    }
}

// -------------------------------------------------------------- backward dKV
template <int D, bool DROP>
__global__ void __launch_bounds__(256) attn_bwd_dkv_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5;
  int bhk, ktile;  // low key tiles see the most queries: first
  if (!tile_map(a.order, a.B * a.Hkv, a.T >> 5, false, bhk, ktile)) return;
  const int b = bhk / a.Hkv, hk = bhk % a.Hkv;
  const int group = a.H / a.Hkv;
  const int kb = ktile * 32;
  const int key = kb + r;
  const uint32_t thr_hi = a.thresh16 << 16, kshift = (key & 1) ? 0u : 16u;

  bf16x8 kf[D / 16], vf[D / 16];
  const __bf16* kp = a.k + b * a.k_sb + static_cast<int64_t>(key) * a.k_st + hk * a.k_sh + 8 * hf;
  const __bf16* vp = a.v + b * a.v_sb + static_cast<int64_t>(key) * a.v_st + hk * a.v_sh + 8 * hf;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    kf[s] = ld8(kp + 16 * s);
    vf[s] = ld8(vp + 16 * s);
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) {
    dk[t] = zero16();
    dv[t] = zero16();
  }
  for (int gh = 0; gh < group; ++gh) {
    const int h = hk * group + gh;
    const int bh = b * a.H + h;
    const __bf16* qbase = a.q + b * a.q_sb + h * a.q_sh + 8 * hf;
    const __bf16* dobase = a.dout + b * a.o_sb + h * a.o_sh + 8 * hf;
    const __bf16* qtb = a.qt + static_cast<int64_t>(bh) * D * a.ldt + 4 * hf;
    const __bf16* dotb = a.dot + static_cast<int64_t>(bh) * D * a.ldt + 4 * hf;
    const float* lseb = a.lse + static_cast<int64_t>(bh) * a.T;
    const float* dlb = a.delta + static_cast<int64_t>(bh) * a.T;
    // loop-invariant part of drop_hash(seed, bh, q, key) for this lane's key
    const uint32_t hkey = a.seed ^ (static_cast<uint32_t>(bh) * 0x9E3779B9u) ^
                          ((static_cast<uint32_t>(key) >> 1) * 0xC2B2AE35u);
    // Q / dO rows of tile qt+1 are prefetched while tile qt is computed (two
    // named fragment sets, 2x unrolled); the transposed fragments and row
    // statistics of tile qt are issued at the top of the tile so their latency
    // hides under the S / dP MFMAs.
    bf16x8 qa[D / 16], da[D / 16], qb2[D / 16], db2[D / 16];
    auto load_qd = [&](int qt, bf16x8(&qf)[D / 16], bf16x8(&df)[D / 16]) {
      const __bf16* qp = qbase + static_cast<int64_t>(qt * 32 + r) * a.q_st;
      const __bf16* dop = dobase + static_cast<int64_t>(qt * 32 + r) * a.o_st;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        qf[ks] = ld8(qp + 16 * ks);
        df[ks] = ld8(dop + 16 * ks);
      }
    };
    auto tile = [&](int qt, const bf16x8(&qc)[D / 16], const bf16x8(&dc)[D / 16]) {
      const int qb = qt * 32;
      float lse4[16], dl4[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 lv = *reinterpret_cast<const float4*>(lseb + qb + 8 * g + 4 * hf);
        const float4 dv4 = *reinterpret_cast<const float4*>(dlb + qb + 8 * g + 4 * hf);
        lse4[4 * g] = lv.x; lse4[4 * g + 1] = lv.y; lse4[4 * g + 2] = lv.z; lse4[4 * g + 3] = lv.w;
        dl4[4 * g] = dv4.x; dl4[4 * g + 1] = dv4.y; dl4[4 * g + 2] = dv4.z; dl4[4 * g + 3] = dv4.w;
      }
      bf16x8 qtf[2][D / 32], dtf[2][D / 32];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          const int64_t row = static_cast<int64_t>(32 * t + r) * a.ldt + qb + 16 * s2;
          qtf[s2][t] = ld4x2(qtb + row);
          dtf[s2][t] = ld4x2(dotb + row);
        }
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        s = mfma32(qc[ks], kf[ks], s);   // S  = Q K^T : rows q, cols key
        dp = mfma32(dc[ks], vf[ks], dp);  // dP = dO V^T
      }
      f32x16 pd;
      const uint32_t hq = static_cast<uint32_t>(qb + 4 * hf) * 0x85EBCA6Bu;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int qq = qb + acc_row(reg, hf);
        const float p = (qt == ktile && key > qq)
                            ? 0.f
                            : __builtin_amdgcn_exp2f(__builtin_fmaf(s[reg], a.scale_log2, -lse4[reg]));
        float dpv = dp[reg];
        float pdv = p;
        if constexpr (DROP) {
          // one hash per element here (the lane is the key): q * C2 = (qb + 4hf) * C2 + row * C2
          const uint32_t rowc = static_cast<uint32_t>((reg & 3) + 8 * (reg >> 2)) * 0x85EBCA6Bu;
          const uint32_t hsh = lowbias32(hkey ^ (hq + rowc));
          const bool kp_ = (hsh << kshift) >= thr_hi;
          dpv = kp_ ? dpv * a.inv_keep : 0.f;
          pdv = kp_ ? p * a.inv_keep : 0.f;
        }
        pd[reg] = pdv;
        s[reg] = p * (dpv - dl4[reg]);  // dS
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = acc_frag(pd, s2);
        const bf16x8 dsf = acc_frag(s, s2);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          dv[t] = mfma32(pf, dtf[s2][t], dv[t]);   // dV += Pd^T dO
          dk[t] = mfma32(dsf, qtf[s2][t], dk[t]);  // dK += dS^T Q
        }
      }
    };
    const int nq = a.T >> 5;
    load_qd(ktile, qa, da);
    int qt = ktile;
    for (; qt + 1 < nq; qt += 2) {
      load_qd(qt + 1, qb2, db2);
      tile(qt, qa, da);
      if (qt + 2 < nq) load_qd(qt + 2, qa, da);
      tile(qt + 1, qb2, db2);
    }
    if (qt < nq) tile(qt, qa, da);
  }
  // dk/dv[t]: rows = key (registers), cols = d (lane)
  __bf16* dkb = a.dk + b * a.dk_sb + hk * a.dk_sh;
  __bf16* dvb = a.dv + b * a.dk_sb + hk * a.dk_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int64_t off = static_cast<int64_t>(kb + acc_row(reg, hf)) * a.dk_st + 32 * t + r;
      dkb[off] = static_cast<__bf16>(dk[t][reg] * a.scale);
      dvb[off] = static_cast<__bf16>(dv[t][reg]);
    }
}

// ------------------------------------------------- transpose [B,T,X,D] -> [B,X,D,T]
// 64 tokens x D tile per 256-thread block through LDS (padded rows).
template <int D>
__global__ void __launch_bounds__(256) transpose_btxd_kernel(const __bf16* __restrict__ in, int64_t sb, int64_t st,
                                                            int64_t sx, __bf16* __restrict__ out, int ldt, int X) {
  __shared__ __bf16 tile[D][64 + 2];
  const int tt = blockIdx.x, bx = blockIdx.y;
  const int b = bx / X, x = bx % X;
  const __bf16* src = in + b * sb + x * sx + static_cast<int64_t>(tt * 64) * st;
  // load: 64 tokens x D, 8 elements per thread per step
  for (int i = threadIdx.x; i < 64 * (D / 8); i += 256) {
    const int tok = i / (D / 8), c8 = (i % (D / 8)) * 8;
    const bf16x8 v = ld8(src + static_cast<int64_t>(tok) * st + c8);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[c8 + j][tok] = v[j];
  }
  __syncthreads();
  __bf16* dst = out + (static_cast<int64_t>(bx) * D) * ldt + tt * 64;
  for (int i = threadIdx.x; i < D * 32; i += 256) {  // 2 tokens per thread
    const int d = i / 32, t2 = (i % 32) * 2;
    const uint32_t lo = __builtin_bit_cast(uint16_t, tile[d][t2]);
    const uint32_t hi = __builtin_bit_cast(uint16_t, tile[d][t2 + 1]);
    *reinterpret_cast<uint32_t*>(dst + static_cast<int64_t>(d) * ldt + t2) = lo | (hi << 16);
  }
}

// ------------------------------------------------------------- delta = rowsum(dO*O)
template <int D>
__global__ void __launch_bounds__(256) attn_delta_kernel(AttnArgs a) {
  // one wave-quarter (16 lanes) per row: D/16 elements per lane
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 16 + (threadIdx.x >> 4);
  const int64_t nrows = static_cast<int64_t>(a.B) * a.H * a.T;
  if (row >= nrows) return;
  const int sub = threadIdx.x & 15;
  const int bh = static_cast<int>(row / a.T), q = static_cast<int>(row % a.T);
  const int b = bh / a.H, h = bh % a.H;
  const int64_t off = b * a.o_sb + static_cast<int64_t>(q) * a.o_st + h * a.o_sh;
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < D / 16; ++j) {
    const int d = sub * (D / 16) + j;
    acc += static_cast<float>(a.o[off + d]) * static_cast<float>(a.dout[off + d]);
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
  if (sub == 0) const_cast<float*>(a.delta)[row] = acc;
}

// ------------------------------------------------------------------ launchers
// grid of tile_map(): ceil(tiles / 4) blocks of 4 waves per head
static inline int64_t tile_blocks(int64_t nbh, int T) { return nbh * (((T >> 5) + 3) >> 2); }

static int fwd_impl() {
  static const int v = [] {
    const char* e = std::getenv("DLION_ATTN_FWD");
    return e ? std::atoi(e) : 1;  // 1: LDS-shared K/V (default), 0: per-wave private loads
  }();
  return v;
}

hipError_t launch_attn_fwd(const AttnArgs& a, int D, bool drop, hipStream_t st) {
  const int64_t blocks = tile_blocks(static_cast<int64_t>(a.B) * a.H, a.T);
  if (fwd_impl() == 1) {
#define FWD_LDS(DD)                                                                              \
  if (drop) hipLaunchKernelGGL((attn_fwd_lds_kernel<DD, true>), dim3(blocks), dim3(256), 0, st, a); \
  else hipLaunchKernelGGL((attn_fwd_lds_kernel<DD, false>), dim3(blocks), dim3(256), 0, st, a);
    if (D == 64) {
      FWD_LDS(64)
    } else if (D == 128) {
      FWD_LDS(128)
    } else {
      return hipErrorInvalidValue;
    }
#undef FWD_LDS
    return hipGetLastError();
  }
  if (D == 64) {
    if (drop) hipLaunchKernelGGL((attn_fwd_kernel<64, true>), dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<64, false>), dim3(blocks), dim3(256), 0, st, a);
  } else if (D == 128) {
    if (drop) hipLaunchKernelGGL((attn_fwd_kernel<128, true>), dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<128, false>), dim3(blocks), dim3(256), 0, st, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_attn_bwd(const AttnArgs& a, int D, bool drop, hipStream_t st) {
  const int64_t rows = static_cast<int64_t>(a.B) * a.H * a.T;
  const int64_t bq = tile_blocks(static_cast<int64_t>(a.B) * a.H, a.T);
  const int64_t bkv = tile_blocks(static_cast<int64_t>(a.B) * a.Hkv, a.T);
#define BWD(DD)                                                                                         \
  hipLaunchKernelGGL((attn_delta_kernel<DD>), dim3((rows + 15) / 16), dim3(256), 0, st, a);             \
  if (fwd_impl() == 1) {                                                                                \
    if (drop) {                                                                                         \
      hipLaunchKernelGGL((attn_bwd_dkv_lds_kernel<DD, true>), dim3(bkv), dim3(256), 0, st, a);         \
      hipLaunchKernelGGL((attn_bwd_dq_lds_kernel<DD, true>), dim3(bq), dim3(256), 0, st, a);           \
    } else {                                                                                            \
      hipLaunchKernelGGL((attn_bwd_dkv_lds_kernel<DD, false>), dim3(bkv), dim3(256), 0, st, a);        \
      hipLaunchKernelGGL((attn_bwd_dq_lds_kernel<DD, false>), dim3(bq), dim3(256), 0, st, a);          \
    }                                                                                                   \
  } else if (drop) {                                                                                    \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, true>), dim3(bkv), dim3(256), 0, st, a);               \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, true>), dim3(bq), dim3(256), 0, st, a);                 \
  } else {                                                                                              \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, false>), dim3(bkv), dim3(256), 0, st, a);              \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, false>), dim3(bq), dim3(256), 0, st, a);                \
  }
  if (D == 64) {
    BWD(64)
  } else if (D == 128) {
    BWD(128)
  } else {
    return hipErrorInvalidValue;
  }
#undef BWD
  return hipGetLastError();
}

hipError_t launch_transpose_btxd(const void* in, int64_t sb, int64_t st, int64_t sx, void* out, int B, int T, int X,
                                 int D, int ldt, hipStream_t stream) {
  const dim3 grid(T / 64, B * X);
  const __bf16* i = static_cast<const __bf16*>(in);
  __bf16* o = static_cast<__bf16*>(out);
  if (D == 64) hipLaunchKernelGGL((transpose_btxd_kernel<64>), grid, dim3(256), 0, stream, i, sb, st, sx, o, ldt, X);
  else if (D == 128) hipLaunchKernelGGL((transpose_btxd_kernel<128>), grid, dim3(256), 0, stream, i, sb, st, sx, o, ldt, X);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace dlion

// Weight-gradient GEMM for gfx950:  C[z][M,N] (fp32) = sum over split z's rows k of P[k,M]^T . Q[k,N]
//
// Both operands are token-major ("TN": the contraction runs over their ROWS),
// which is how a linear's weight gradient sees its input and output gradient
// (dW = dY^T X over the tokens).  hipBLASLt's TN kernels reach 0.78-0.90 PF/s
// at the GPT-2 shapes (tools/bench_wgrad.py); this kernel is the NT kernel of
// gemm.hip with the operand images transposed:
//
//   * LDS image of a K-tile half: 64 k-rows x 128 columns (256-byte rows),
//     filled by LDS-DMA (global_load_lds_dwordx4) straight from the token-major
//     rows -- the 16-byte chunks of a row are coalesced along M / N.
//   * MFMA fragments (16 columns x 8 consecutive k per lane) come out of the
//     [k][col] image with two ds_read_b64_tr_b16 each (4 k-rows x 16 columns
//     per 16-lane group, delivered column-major).  Chunk swizzle: physical
//     chunk = logical ^ 2 * ((row & 3) | ((row >> 3) & 1) << 2) -- the 8 rows
//     a 32-lane half reads in one transposed read (two groups, 8 rows apart)
//     land on 8 distinct 32-byte bank ranges: conflict-free.
//   * Everything else -- 256x256 tile per 8-wave block, BK = 64, the 8-phase
//     stage order with counted vmcnt waits, the wave-group stagger, the
//     XCD-aware tile order -- is gemm.hip's.
//   * K is split S ways (z = split index, output slice z) and may span up to
//     kMaxSeg separate operand buffers of seg_rows rows each (e.g. the
//     micro-batches of one optimizer step); k-tiles never straddle a segment.
//   * Epilogue: fp32 float4 stores (or read-add-stores into a running
//     accumulator) straight from the accumulators (a lane owns 4 consecutive
//     columns of a row), no LDS round trip.  Unsplit (S = 1) the result can
//     instead go out as bf16 (optionally added onto a bf16 gradient): the
//     weight gradient itself, with no fp32 [M, N] round trip through HBM and no
//     separate reduction pass (Llama-3-8B full-parameter: 7 B weights x 10 B of
//     fp32-partial traffic, ~11 ms per step).
#include "common.h"


namespace dlion {

namespace {

typedef __bf16 tn_bf16x8 __attribute__((ext_vector_type(8)));
typedef float tn_f32x4 __attribute__((ext_vector_type(4)));
typedef short tn_v4i16 __attribute__((ext_vector_type(4)));
typedef short tn_v8i16 __attribute__((ext_vector_type(8)));

constexpr int kTBM = 256, kTBN = 256, kTBK = 64;
constexpr int kTHalf = 64 * 256;      // one half-tile: 64 k-rows x 128 columns bf16 = 16 KiB
constexpr int kTLds = 8 * kTHalf;     // 128 KiB
constexpr int kMaxSeg = 16;

struct TnArgs {
  const uint16_t* P[kMaxSeg];
  const uint16_t* Q[kMaxSeg];
  float* C;
  uint16_t* Cb;  // non-null (splits == 1): bf16 output instead of C
  int ldp, ldq;
  int M, N;
  int seg_kt;  // k-tiles (of 64 rows) per segment
  int kpairs;  // total k-tile pairs over all segments
  int splits;
  int tiles_m, tiles_n;
  int accumulate;  // C += result (the fp32 split-K accumulators of a fusion window)
};

__device__ __forceinline__ constexpr int tslot(int dbuf, int ab, int half) { return ((dbuf * 2 + ab) * 2 + half) * kTHalf; }

__device__ __forceinline__ void tn_wait6() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }
__device__ __forceinline__ void tn_wait8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
__device__ __forceinline__ void tn_wait2() { asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); }
__device__ __forceinline__ void tn_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// scalar operand base + 32-bit lane byte offset: the saddr form of the load
// (no per-load 64-bit address add); dst is wave-uniform (m0)
__device__ __forceinline__ void tn_glds16(const uint16_t* base, uint32_t boff, uint8_t* dst) {
  const uint8_t* src = reinterpret_cast<const uint8_t*>(base) + boff;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

__device__ __forceinline__ tn_f32x4 tn_mfma(const tn_bf16x8& a, const tn_bf16x8& b, const tn_f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// One 16-column x 8-k fragment: two transposed reads, 4 k-rows apart.  Inline
// asm, not __builtin_amdgcn_ds_read_tr16_b64: the compiler treats the builtin
// as possibly aliasing the in-flight LDS-DMA writes and put an
// "s_waitcnt vmcnt(0)" in front of every read phase, draining the staging
// pipeline (the kernel ran at 58 % of the NT kernel's per-CU rate).  The asm
// reads are covered by the explicit lgkmcnt(0) each phase issues before its
// MFMAs (DLION_TN_PHASE_MATH); the results are consumed only there.  The
// constant part of the address (the second read's 4 rows, the second k-step's
// 32 rows) rides in the instruction's offset field: as a register operand
// hipcc materialised it with a v_add / v_or per read (57 VALU per pair).
template <int OFF>
__device__ __forceinline__ tn_v4i16 tn_tr_read(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
  tn_v4i16 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ tn_bf16x8 tn_frag(uint32_t addr) {
  const tn_v4i16 lo = tn_tr_read<OFF>(addr);
  const tn_v4i16 hi = tn_tr_read<OFF + 4 * 256>(addr);
  // a concatenation, not a copy: lets the register allocator place both reads
  // in the fragment's 4 VGPRs
  return __builtin_bit_cast(tn_bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__global__ void __launch_bounds__(512, 1) gemm_tn_kernel(const TnArgs g) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kTLds];

  const int tid = threadIdx.x;
  // wave index as a scalar: the LDS-DMA destinations (m0) need no readfirstlane
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wr = w >> 2, wc = w & 3;

  // ---- XCD-aware order over (split, tile); tiles grouped 8 M-tiles deep
  const int tiles = g.tiles_m * g.tiles_n;
  const int nwg = tiles * g.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg_all = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int z = wg_all / tiles;
  const int wg = wg_all - z * tiles;
  constexpr int GM = 8;
  const int per_group = GM * g.tiles_n;
  const int grp = wg / per_group;
  const int first_m = grp * GM;
  const int gsz = min(g.tiles_m - first_m, GM);
  const int in_g = wg - grp * per_group;
  const int tm = first_m + in_g % gsz;
  const int tn = in_g / gsz;
  const int m0 = tm * kTBM, n0 = tn * kTBN;
  // this split's k-tile pairs
  const int p0 = static_cast<int>((static_cast<int64_t>(z) * g.kpairs) / g.splits);
  const int p1 = static_cast<int>((static_cast<int64_t>(z + 1) * g.kpairs) / g.splits);
  const int nit = p1 - p0;  // >= 1 (splits <= kpairs)

  // ---- staging offsets (elements, relative to the k-tile's first row).  Lane ->
  // LDS row lr = 4q + lane/16 of half-tile piece q, physical chunk pc = lane%16,
  // logical chunk c = pc ^ swz(lr).  Columns past the edge are clamped (loaded,
  // never stored).
  uint32_t off[2][2][2];  // [ab][half][piece], bytes
  {
    const int pc = lane & 15;
#pragma unroll
    for (int pi = 0; pi < 2; ++pi) {
      const int q = 2 * w + pi;
      const int lr = 4 * q + (lane >> 4);
      const int c = pc ^ (((lr & 3) | (((lr >> 3) & 1) << 2)) << 1);
      const int col = c * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // P half h: column col -> tile m (col/64)*128 + 64h + col%64
        const int ma = min(m0 + (col >> 6) * 128 + 64 * h + (col & 63), g.M - 8);
        off[0][h][pi] = static_cast<uint32_t>(lr * g.ldp + ma) * 2u;
        // Q half h: column col -> tile n 128h + col
        const int nb = min(n0 + 128 * h + col, g.N - 8);
        off[1][h][pi] = static_cast<uint32_t>(lr * g.ldq + nb) * 2u;
      }
    }
  }

  // K-tile pair bases, walked incrementally: the current pair's and the next
  // pair's operand pointers are scalars known one iteration ahead, advanced by
  // one pair stride; the segment pointer table is read only when the walk
  // crosses into the next segment (a table read per pair put a scalar load and
  // its lgkmcnt(0) wait in every iteration).
  const int seg_pairs = g.seg_kt / 2;
  const int64_t kstepP = static_cast<int64_t>(kTBK) * g.ldp, kstepQ = static_cast<int64_t>(kTBK) * g.ldq;
  int sg = p0 / seg_pairs, lc = p0 - sg * seg_pairs;
  const uint16_t* cP = g.P[sg] + lc * (2 * kstepP);
  const uint16_t* cQ = g.Q[sg] + lc * (2 * kstepQ);
  const uint16_t* nP = cP;
  const uint16_t* nQ = cQ;
  // nP / nQ <- the pair after the current next one
  auto advance = [&]() {
    if (++lc == seg_pairs) {
      ++sg;
      lc = 0;
      nP = g.P[sg];
      nQ = g.Q[sg];
    } else {
      nP += 2 * kstepP;
      nQ += 2 * kstepQ;
    }
  };
  if (nit > 1) advance();
  // stage half `half` of operand ab (0 = P, 1 = Q) of the K-tile at `base` into buffer dbuf
  auto stage = [&](int ab, int half, int dbuf, const uint16_t* base) {
    uint8_t* dst = lds + tslot(dbuf, ab, half) + (2 * w) * 1024;
    // opaque in-place "update": the offsets stay 32-bit lane registers next to
    // the loads (hoisted, they became 64-bit pairs and a v_lshl_add_u64 per load)
    asm volatile("" : "+v"(off[ab][half][0]), "+v"(off[ab][half][1]));
    tn_glds16(base, off[ab][half][0], dst);
    tn_glds16(base, off[ab][half][1], dst + 1024);
  };

  // ---- fragment read offsets.  Group gq = lane/16, in-group lane 4q+p: rows
  // 8gq + q (+4 for the second read) of the 32-k step, columns c0 + 4p..+3.
  // The swizzle of those rows is the lane constant 2 * (q | (gq & 1) << 2).
  const int gq = lane >> 4, fq = (lane & 15) >> 2, fp = lane & 3;
  const int swz16 = fq | ((gq & 1) << 2);  // swizzle in units of 32-byte chunk pairs
  const int row_off = (8 * gq + fq) * 256 + (fp & 1) * 8;
  // byte offset of the fragment of 16-column block cb (0..7) at k-step s: one
  // lane register per block, the k-step and the image slot are immediates
  auto fcol = [&](int cb) { return row_off + (((cb ^ swz16) * 2 + (fp >> 1)) << 4); };
  int fb[4], fa[4];  // this wave's B column blocks 4(wc & 1) + nt and A column blocks 4wr + j
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    fb[j] = fcol(4 * (wc & 1) + j);
    fa[j] = fcol(4 * wr + j);
  }

  tn_f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = tn_f32x4{0.f, 0.f, 0.f, 0.f};

  tn_bf16x8 bfr[4][2];
  tn_bf16x8 afr[2][2];

  // B (Q): this wave's 64 columns are column blocks 4(wc & 1) .. +3 of half (wc >> 1)
  // 32-bit LDS address of the image
  const uint32_t lds32 =
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds));
  auto read_b = [&](int dbuf) {
    const uint32_t base = lds32 + tslot(dbuf, 1, wc >> 1);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      bfr[nt][0] = tn_frag<0>(base + fb[nt]);
      bfr[nt][1] = tn_frag<32 * 256>(base + fb[nt]);
    }
  };
  // A (P): block p (0..3) = m-tiles 2p, 2p+1: half p >> 1, column block 4wr + 2(p & 1) + mt
  auto read_a = [&](int dbuf, int p) {
    const uint32_t base = lds32 + tslot(dbuf, 0, p >> 1);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      afr[mt][0] = tn_frag<0>(base + fa[2 * (p & 1) + mt]);
      afr[mt][1] = tn_frag<32 * 256>(base + fa[2 * (p & 1) + mt]);
    }
  };

#define DLION_TN_MFMA(P)                                                         \
  do {                                                                           \
    __builtin_amdgcn_s_setprio(1);                                               \
    _Pragma("unroll") for (int mt = 0; mt < 2; ++mt)                             \
    _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                             \
    _Pragma("unroll") for (int s = 0; s < 2; ++s)                                \
      acc[2 * (P) + mt][nt] = tn_mfma(bfr[nt][s], afr[mt][s], acc[2 * (P) + mt][nt]); \
    __builtin_amdgcn_s_setprio(0);                                               \
  } while (0)

#define DLION_TN_PHASE_MATH(P)                       \
  __builtin_amdgcn_s_barrier();                      \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  __builtin_amdgcn_sched_barrier(0);                 \
  DLION_TN_MFMA(P);                                  \
  __builtin_amdgcn_sched_barrier(0);                 \
  __builtin_amdgcn_s_barrier();

  // ---- prologue: T0.{B0,B1,A0,A1}, T1.{B0,B1}; retire T0.{B0,B1,A0}
  stage(1, 0, 0, cQ);
  stage(1, 1, 0, cQ);
  stage(0, 0, 0, cP);
  stage(0, 1, 0, cP);
  stage(1, 0, 1, cQ + kstepQ);
  stage(1, 1, 1, cQ + kstepQ);
  tn_wait6();
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // wave-group stagger (gemm.hip)

  // Branch-free body: the last pair also stages (its "next" pointers still
  // point at the current pair -- valid memory, buffers past their last read,
  // the same restage order as every other pair), so the wait counts never
  // change and hipcc emits one straight-line block instead of ~15 blocks of
  // scalar branches on a runtime `more` (SALU per pair 116 -> 90); the extra
  // 64 KiB of DMA per block is drained before the epilogue.
  for (int it = 0; it < nit; ++it) {
    // P1
    read_b(0);
    read_a(0, 0);
    stage(0, 0, 1, cP + kstepP);
    DLION_TN_PHASE_MATH(0)
    // P2
    read_a(0, 1);
    stage(0, 1, 1, cP + kstepP);
    tn_wait8();  // T(kt).A1
    DLION_TN_PHASE_MATH(1)
    // P3
    read_a(0, 2);
    stage(1, 0, 0, nQ);
    DLION_TN_PHASE_MATH(2)
    // P4
    read_a(0, 3);
    stage(1, 1, 0, nQ);
    tn_wait6();  // T(kt+1).{B0,B1,A0}
    DLION_TN_PHASE_MATH(3)
    // P5
    read_b(1);
    read_a(1, 0);
    stage(0, 0, 0, nP);
    DLION_TN_PHASE_MATH(0)
    // P6
    read_a(1, 1);
    stage(0, 1, 0, nP);
    tn_wait8();  // T(kt+1).A1
    DLION_TN_PHASE_MATH(1)
    // P7
    read_a(1, 2);
    stage(1, 0, 1, nQ + kstepQ);
    DLION_TN_PHASE_MATH(2)
    // P8
    read_a(1, 3);
    stage(1, 1, 1, nQ + kstepQ);
    tn_wait6();  // T(kt+2).{B0,B1,A0}
    DLION_TN_PHASE_MATH(3)
    cP = nP;
    cQ = nQ;
    if (it + 2 < nit) advance();
  }
#undef DLION_TN_PHASE_MATH
#undef DLION_TN_MFMA
  tn_wait0();  // the last pair's (unused) stages have landed: no DMA outlives the block
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the wave groups

  // ---- epilogue: acc[mt][nt][j] = C[wr*128 + 16mt + (lane&15)][wc*64 + 16nt + 4(lane>>4) + j]
  if (g.Cb != nullptr) {  // unsplit: bf16(acc (+ old bf16)), the sum_partials rounding
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int gm = m0 + wr * 128 + 16 * mt + (lane & 15);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int gn = n0 + wc * 64 + 16 * nt + 4 * (lane >> 4);
        if (gm < g.M && gn < g.N) {
          uint2* dst = reinterpret_cast<uint2*>(g.Cb + static_cast<int64_t>(gm) * g.N + gn);
          float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
          if (g.accumulate) {
            const uint2 o = *dst;
            v[0] += bf16_to_f32(o.x & 0xffffu);
            v[1] += bf16_to_f32(o.x >> 16);
            v[2] += bf16_to_f32(o.y & 0xffffu);
            v[3] += bf16_to_f32(o.y >> 16);
          }
          const uint32_t lo = static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(v[0]))) |
                              (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(v[1]))) << 16);
          const uint32_t hi = static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(v[2]))) |
                              (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(v[3]))) << 16);
          *dst = make_uint2(lo, hi);
        }
      }
    }
    return;
  }
  float* Cz = g.C + static_cast<int64_t>(z) * g.M * g.N;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int gm = m0 + wr * 128 + 16 * mt + (lane & 15);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int gn = n0 + wc * 64 + 16 * nt + 4 * (lane >> 4);
      if (gm < g.M && gn < g.N) {
        float4* dst = reinterpret_cast<float4*>(Cz + static_cast<int64_t>(gm) * g.N + gn);
        float4 v = make_float4(acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]);
        if (g.accumulate) {
          const float4 o = *dst;
          v.x += o.x;
          v.y += o.y;
          v.z += o.z;
          v.w += o.w;
        }
        *dst = v;
      }
    }
  }
}

}  // namespace

hipError_t launch_gemm_tn(const void* const* P, const void* const* Q, int nseg, int64_t seg_rows, int ldp, int ldq,
                          float* C, int M, int N, int splits, bool accumulate, hipStream_t st, void* Cb) {
  if (Cb != nullptr && (splits != 1 || reinterpret_cast<uintptr_t>(Cb) % 8 != 0)) return hipErrorInvalidValue;
  if (M <= 0 || N <= 0) return hipSuccess;
  if (nseg < 1 || nseg > kMaxSeg || seg_rows <= 0 || seg_rows % (2 * kTBK) != 0) return hipErrorInvalidValue;
  if (M % 8 != 0 || N % 8 != 0 || ldp % 8 != 0 || ldq % 8 != 0 || ldp < M || ldq < N) return hipErrorInvalidValue;
  if (seg_rows * ldp >= (1ll << 31) || seg_rows * ldq >= (1ll << 31)) return hipErrorInvalidValue;
  TnArgs g{};
  for (int i = 0; i < nseg; ++i) {
    g.P[i] = static_cast<const uint16_t*>(P[i]);
    g.Q[i] = static_cast<const uint16_t*>(Q[i]);
    if (g.P[i] == nullptr || g.Q[i] == nullptr || reinterpret_cast<uintptr_t>(P[i]) % 16 != 0 ||
        reinterpret_cast<uintptr_t>(Q[i]) % 16 != 0)
      return hipErrorInvalidValue;
  }
  g.C = C;
  g.Cb = static_cast<uint16_t*>(Cb);
  g.ldp = ldp;
  g.ldq = ldq;
  g.M = M;
  g.N = N;
  g.seg_kt = static_cast<int>(seg_rows / kTBK);
  g.kpairs = g.seg_kt / 2 * nseg;
  g.splits = splits;
  g.accumulate = accumulate ? 1 : 0;
  if (splits < 1 || splits > g.kpairs) return hipErrorInvalidValue;
  g.tiles_m = (M + kTBM - 1) / kTBM;
  g.tiles_n = (N + kTBN - 1) / kTBN;
  const int64_t blocks = static_cast<int64_t>(g.tiles_m) * g.tiles_n * splits;
  if (blocks >= (1ll << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gemm_tn_kernel, dim3(static_cast<unsigned>(blocks)), dim3(512), 0, st, g);
  return hipGetLastError();
}

}  // namespace dlion

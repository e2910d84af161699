// bf16 GEMM with fused epilogues for gfx950:  C[M,N] = A[M,K] . B[N,K]^T  (+ bias, GELU, DGELU)
//
// Both operands K-contiguous ("NT"), fp32 accumulation in MFMA, bf16 output;
// the bias / bias+GELU of a linear can ride in the epilogue instead of a
// separate HBM pass (ops/gemm.py).
//
// Structure (cdna_hip_programming.md §5 "256² 8-phase template", with its
// stage order re-derived for this kernel):
//   * 256x256 output tile per 512-thread block (8 waves as 2(M) x 4(N), each
//     wave 128x64 = 8x4 tiles of v_mfma_f32_16x16x32_bf16), BK = 64, one
//     block per CU (128 KiB LDS).
//   * LDS = 2 K-tile buffers x {A, B} x 2 half-tiles of 128 rows x 64 k
//     (16 KiB each), filled ONLY by global_load_lds_dwordx4 (LDS-DMA: no
//     staging registers, no ds_write).  The LDS image is lane-linear, so the
//     bank swizzle is applied to the per-lane SOURCE address and undone on
//     the read (guide rule 21): physical 16-byte chunk = k-chunk ^ ((row >> 1) & 7),
//     which makes every ds_read_b128 fragment read conflict-free.
//   * A K-tile is consumed in 4 phases (one 32-row block of the wave's 128
//     rows each, 16 MFMAs); every phase also stages one half-tile of a LATER
//     K-tile, so 3-4 half-tiles are always in flight across the barriers
//     (counted s_waitcnt vmcnt(6|8), never 0 while more K-tiles follow, raw
//     s_barrier).  Stage order per 2-K-tile iteration (kt = 2i):
//        P1 T(kt+1).A0  P2 T(kt+1).A1  P3 T(kt+2).B0  P4 T(kt+2).B1
//        P5 T(kt+2).A0  P6 T(kt+2).A1  P7 T(kt+3).B0  P8 T(kt+3).B1
//     reads: P1 B(all)+A0 blk0, P2 A0 blk1, P3 A1 blk2, P4 A1 blk3 (dbuf 0),
//     P5..P8 the same on dbuf 1.  Every restage is >= 2 phases after the last
//     read of its buffer; every read is one phase after the wait that retired
//     it (vmcnt(6) in P4/P8, vmcnt(8) in P2/P6).
//   * Wave-group stagger: waves 4-7 run one barrier behind waves 0-3, so on
//     each SIMD one wave's MFMA segment overlaps its partner's ds_read /
//     LDS-DMA segment (measured +12-25 % over lock-step phases).
//   * XCD-aware block order: the blocks of one XCD get a contiguous range of
//     tiles, grouped 8 M-tiles deep, so neighbouring tiles share A / B panels
//     in that XCD's L2.
//   * Epilogue through LDS: each wave parks its 128x64 bf16 tile (16-byte
//     chunks swizzled by row) and writes whole 128-byte row segments.
//
// Measured on MI355X against hipBLASLt (tools/bench_gemm_nt.py, random data,
// M = 20480): 0.84-0.95 PF/s at K = 768 (hipBLASLt 0.99-1.15), 1.25-1.33 PF/s
// at K = 2304-3072 (hipBLASLt 1.41-1.51).  A persistent variant that streams
// the next tile's first K-tiles during the current tile's tail and stores
// straight from the accumulators (8-byte stores, operands swapped so a lane
// owns 4 consecutive columns) measured 4-10 % SLOWER: the scattered 8-byte
// epilogue stores cost more than the hidden prologue saved; a second one that
// parked through spare LDS and overlapped the next tile's prologue with the
// epilogue measured neutral (profiles/r4/gemm_epi_persist.txt) and was removed.
#include "common.h"

#include <algorithm>

namespace dlion {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kHalf = 128 * kBK * 2;  // one half-tile: 128 rows x 64 k bf16 = 16 KiB
constexpr int kLds = 8 * kHalf;       // 128 KiB

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  uint16_t* C;
  const uint16_t* bias;
  uint16_t* aux;
  float* part;  // EPI 4/5: [2 * tiles_m][N] fp32 column partial sums of C
  unsigned long long* stamps;  // diagnostic build only (STAMP): [blocks][8] timestamps
  int lda, ldb, ldc, ldaux;
  int M, N, K;
  int tiles_m, tiles_n;
};

__device__ __forceinline__ constexpr int slot(int dbuf, int ab, int half) { return ((dbuf * 2 + ab) * 2 + half) * kHalf; }

__device__ __forceinline__ void vm_wait6() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }
__device__ __forceinline__ void vm_wait8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
__device__ __forceinline__ void vm_wait2() { asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); }
__device__ __forceinline__ void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// scalar operand base + 32-bit lane byte offset: the saddr form of the load
// (no per-load 64-bit address add); dst is wave-uniform (m0)
__device__ __forceinline__ void glds16(const uint16_t* base, uint32_t boff, uint8_t* dst) {
  const uint8_t* src = reinterpret_cast<const uint8_t*>(base) + boff;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// Epilogue store / aux-load flavour: the MLP epilogues write / read the aux
// tensor (gelu'(z): written here, read once by the backward) and their C with
// non-temporal hints (plain / bias outputs keep normal stores).  Same-box GPT-2
// A/B: 1.019M (both off) -> 1.024M (aux) -> 1.035M tok/s (both)
// (profiles/r3/nt_stores_ab.txt); in isolation the MLP GEMMs gain only 1-5 us,
// the rest is what the other kernels of the step no longer lose to the
// 126 MB outputs streaming through L2 / MALL.  Non-temporal operand loads and
// non-temporal plain-C stores measured neutral and were removed.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT, typename V>
__device__ __forceinline__ void st16(uint16_t* p, const V& v) {
  const u32x4 x = __builtin_bit_cast(u32x4, v);
  if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = x;
}
template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint16_t* p) {
  u32x4 x;
  if constexpr (NT) x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else x = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(x[0], x[1], x[2], x[3]);
}
constexpr bool kNtAux = true, kNtC = true;

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Per-thread staging state: the element offsets (relative to the operand
// base, k = 0) of the 2 pieces this wave fills in each of the 4 half-tiles
// {A0, A1, B0, B1}.  Piece q of a half-tile = LDS rows 8q..8q+7 (1 KiB).
struct Stage {
  uint32_t off[2][2][2];  // [ab][half][piece], bytes
};

// Diagnostic stamps (STAMP builds only, tools/gemm_stamps.py): s_memtime at
// fixed points plus s_memrealtime at entry / exit, written by vector stores.
#define DLION_STAMP(dst)                                                            \
  if constexpr (STAMP) {                                                            \
    __builtin_amdgcn_sched_barrier(0);                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(dst) :: "memory");    \
    __builtin_amdgcn_sched_barrier(0);                                              \
  }
#define DLION_RSTAMP(dst)                                                           \
  if constexpr (STAMP) {                                                            \
    __builtin_amdgcn_sched_barrier(0);                                              \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(dst) :: "memory"); \
    __builtin_amdgcn_sched_barrier(0);                                              \
  }

template <int EPI, bool STAMP = false>
__global__ void __launch_bounds__(512, 1) gemm_nt_kernel(const GemmArgs g) {
  unsigned long long st_[7] = {0, 0, 0, 0, 0, 0, 0};
  DLION_RSTAMP(st_[5])
  DLION_STAMP(st_[0])
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];

  const int tid = threadIdx.x;
  // wave index as a scalar: the LDS-DMA destinations (m0) need no readfirstlane
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wr = w >> 2, wc = w & 3;

  // ---- XCD-aware tile order (bijective for any grid size)
  const int nwg = g.tiles_m * g.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int per_group = GM * g.tiles_n;
  const int grp = wg / per_group;
  const int first_m = grp * GM;
  const int gsz = min(g.tiles_m - first_m, GM);
  const int in_g = wg - grp * per_group;
  const int tm = first_m + in_g % gsz;
  const int tn = in_g / gsz;
  const int m0 = tm * kBM, n0 = tn * kBN;

  // ---- staging offsets.  Lane -> LDS row lr = 8q + lane/8, physical chunk
  // pc = lane%8, logical k-chunk c = pc ^ ((lr >> 1) & 7).  Rows past the
  // matrix edge are clamped (loaded, never stored).
  Stage st;
  {
    const int pc = lane & 7;
#pragma unroll
    for (int pi = 0; pi < 2; ++pi) {
      const int q = 2 * w + pi;
      const int lr = 8 * q + (lane >> 3);
      const int c = pc ^ ((lr >> 1) & 7);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // A half h: LDS row lr -> tile row (lr/64)*128 + 64h + lr%64
        const int ra = min(m0 + (lr >> 6) * 128 + 64 * h + (lr & 63), g.M - 1);
        st.off[0][h][pi] = static_cast<uint32_t>(ra * g.lda + c * 8) * 2u;
        // B half h: LDS row lr -> tile col 128h + lr
        const int rb = min(n0 + 128 * h + lr, g.N - 1);
        st.off[1][h][pi] = static_cast<uint32_t>(rb * g.ldb + c * 8) * 2u;
      }
    }
  }
  const uint16_t* __restrict__ Ag = g.A;
  const uint16_t* __restrict__ Bg = g.B;

  auto stage = [&](int ab, int half, int dbuf, int kt) {
    const uint16_t* base = (ab == 0 ? Ag : Bg) + kt * kBK;
    asm volatile("" : "+s"(base));  // a scalar base, not re-associated into the lane offsets
    uint8_t* dst = lds + slot(dbuf, ab, half) + (2 * w) * 1024;
    // opaque in-place "update": the offsets stay 32-bit lane registers next to
    // the loads (hoisted, they became 64-bit pairs and a v_lshl_add_u64 per load)
    asm volatile("" : "+v"(st.off[ab][half][0]), "+v"(st.off[ab][half][1]));
    glds16(base, st.off[ab][half][0], dst);
    glds16(base, st.off[ab][half][1], dst + 1024);
  };

  // ---- fragment read offsets (bytes within a half-tile)
  // lane reads row (lane & 15) of a 16-row tile, k-chunk 4s + (lane >> 4)
  const int lr16 = lane & 15;
  const int swz = (lr16 >> 1) & 7;
  const int foff0 = lr16 * 128 + (((lane >> 4) ^ swz) << 4);
  const int foff1 = lr16 * 128 + (((4 + (lane >> 4)) ^ swz) << 4);
  // A rows of this wave: LDS row wr*64 + 16*(m-tile & 3) within half (m-tile >> 2)
  const int a_row_base = wr * 64 * 128;
  // B: this wave's 64 columns are rows (wc & 1)*64 .. +63 of half (wc >> 1)
  const int b_base_off = ((wc >> 1) * kHalf) + (wc & 1) * 64 * 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 bfr[4][2];
  bf16x8 afr[2][2];

  auto read_b = [&](int dbuf) {
    const uint8_t* base = lds + slot(dbuf, 1, 0) + b_base_off;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      bfr[nt][0] = *reinterpret_cast<const bf16x8*>(base + nt * 16 * 128 + foff0);
      bfr[nt][1] = *reinterpret_cast<const bf16x8*>(base + nt * 16 * 128 + foff1);
    }
  };
  // block p (0..3) = m-tiles 2p, 2p+1: half p >> 1, tile-in-half 2(p&1) + mt
  auto read_a = [&](int dbuf, int p) {
    const uint8_t* base = lds + slot(dbuf, 0, p >> 1) + a_row_base + (2 * (p & 1)) * 16 * 128;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      afr[mt][0] = *reinterpret_cast<const bf16x8*>(base + mt * 16 * 128 + foff0);
      afr[mt][1] = *reinterpret_cast<const bf16x8*>(base + mt * 16 * 128 + foff1);
    }
  };

#define DLION_GEMM_MFMA(P)                                                       \
  do {                                                                           \
    __builtin_amdgcn_s_setprio(1);                                               \
    _Pragma("unroll") for (int mt = 0; mt < 2; ++mt)                             \
    _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                             \
    _Pragma("unroll") for (int s = 0; s < 2; ++s)                                \
      acc[2 * (P) + mt][nt] = mfma16(bfr[nt][s], afr[mt][s], acc[2 * (P) + mt][nt]); \
    __builtin_amdgcn_s_setprio(0);                                               \
  } while (0)

  // phase math: barrier, wait for this wave's LDS reads, MFMAs, barrier
#define DLION_GEMM_PHASE_MATH(P)                     \
  __builtin_amdgcn_s_barrier();                      \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  __builtin_amdgcn_sched_barrier(0);                 \
  DLION_GEMM_MFMA(P);                                \
  __builtin_amdgcn_sched_barrier(0);                 \
  __builtin_amdgcn_s_barrier();

  const int nk = g.K / kBK;  // even, >= 2
  const int nit = nk / 2;

  // ---- prologue: T0.{B0,B1,A0,A1}, T1.{B0,B1}; retire T0.{B0,B1,A0}
  stage(1, 0, 0, 0);
  stage(1, 1, 0, 0);
  stage(0, 0, 0, 0);
  stage(0, 1, 0, 0);
  stage(1, 0, 1, 1);
  stage(1, 1, 1, 1);
  vm_wait6();
  __builtin_amdgcn_s_barrier();
  // Stagger: waves 4-7 (wr = 1) run one barrier behind waves 0-3, so on every
  // SIMD (waves w and w+4) one wave's MFMA segment overlaps its partner's
  // ds_read / LDS-DMA segment.  Legal for this stage order: a read follows the
  // retiring wait by >= 1 phase and a restage follows the last read by >= 2
  // phases in both group orders (re-derived with the half-phase offset).
  if (wr == 1) __builtin_amdgcn_s_barrier();
  DLION_STAMP(st_[1])

  for (int it = 0; it < nit; ++it) {
    const int kt = 2 * it;
    const bool more = it + 1 < nit;
    // P1
    read_b(0);
    read_a(0, 0);
    stage(0, 0, 1, kt + 1);
    DLION_GEMM_PHASE_MATH(0)
    // P2
    read_a(0, 1);
    stage(0, 1, 1, kt + 1);
    vm_wait8();  // T(kt).A1
    DLION_GEMM_PHASE_MATH(1)
    // P3
    read_a(0, 2);
    if (more) stage(1, 0, 0, kt + 2);
    DLION_GEMM_PHASE_MATH(2)
    // P4
    read_a(0, 3);
    if (more) {
      stage(1, 1, 0, kt + 2);
      vm_wait6();  // T(kt+1).{B0,B1,A0}
    } else {
      vm_wait2();
    }
    DLION_GEMM_PHASE_MATH(3)
    // P5
    read_b(1);
    read_a(1, 0);
    if (more) stage(0, 0, 0, kt + 2);
    DLION_GEMM_PHASE_MATH(0)
    // P6
    read_a(1, 1);
    if (more) {
      stage(0, 1, 0, kt + 2);
      vm_wait8();  // T(kt+1).A1
    } else {
      vm_wait0();
    }
    DLION_GEMM_PHASE_MATH(1)
    // P7
    read_a(1, 2);
    if (more) stage(1, 0, 1, kt + 3);
    DLION_GEMM_PHASE_MATH(2)
    // P8
    read_a(1, 3);
    if (more) {
      stage(1, 1, 1, kt + 3);
      vm_wait6();  // T(kt+2).{B0,B1,A0}
    }
    DLION_GEMM_PHASE_MATH(3)
  }
#undef DLION_GEMM_PHASE_MATH
#undef DLION_GEMM_MFMA
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups: every MFMA and LDS read is done
  DLION_STAMP(st_[2])

  // ---- epilogue.  The MFMA operands are swapped (B fragment first), so each
  // 16x16 accumulator block is transposed: acc[mt][nt][j] =
  // C[wr*128 + 16mt + (lane&15)][wc*64 + 16nt + 4(lane>>4) + j] -- a lane owns
  // 4 consecutive columns of one row, parked with one 8-byte LDS write instead
  // of four 2-byte ones (32 instead of 128 park writes per lane).
  uint8_t* reg = lds + w * (128 * 128);
  float bv[4][4] = {};
  if constexpr (EPI == 1) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + nt * 16 + 4 * (lane >> 4) + j;
        bv[nt][j] = n < g.N ? bf16_to_f32(g.bias[n]) : 0.f;
      }
  }
  const int row_base = m0 + wr * 128;
  const int col_base = n0 + wc * 64;

  // park 4 bf16 per (mt, nt) at [row][col..col+3] with 16-byte chunk ^= row & 7
  auto park = [&](auto fn) {
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int row = mt * 16 + (lane & 15);
        const int col = nt * 16 + 4 * (lane >> 4);
        const int chunk = (col >> 3) ^ (row & 7);
        const uint32_t lo = static_cast<uint32_t>(fn(acc[mt][nt][0], nt, 0)) |
                            (static_cast<uint32_t>(fn(acc[mt][nt][1], nt, 1)) << 16);
        const uint32_t hi = static_cast<uint32_t>(fn(acc[mt][nt][2], nt, 2)) |
                            (static_cast<uint32_t>(fn(acc[mt][nt][3], nt, 3)) << 16);
        *reinterpret_cast<uint2*>(reg + row * 128 + chunk * 16 + (col & 7) * 2) = make_uint2(lo, hi);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };
  const int ch = lane & 7;
  const int gn = col_base + ch * 8;

  if constexpr (EPI <= 1) {
    park([&](float v, int nt, int j) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(v + bv[nt][j])); });
    DLION_STAMP(st_[3])
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = i * 8 + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4*>(reg + row * 128 + ((ch ^ (row & 7)) << 4));
      const int gm = row_base + row;
      // plain / bias outputs (input gradients, projections: read at once by the
      // next kernel) keep normal stores; only the MLP epilogues' streams go non-temporal
      if (gm < g.M && gn < g.N) st16<false>(g.C + (int64_t)gm * g.ldc + gn, v);
    }
    if constexpr (STAMP) {
      DLION_STAMP(st_[4])
      DLION_RSTAMP(st_[6])
      // per-lane value -> a vector store; lane i of wave 0 writes stamp i
      if (tid < 8) g.stamps[static_cast<int64_t>(blockIdx.x) * 8 + tid] = tid < 7 ? st_[tid < 7 ? tid : 0] : 0ull;
    }
  } else if constexpr (EPI <= 3 || EPI == 6 || EPI == 7) {
    // EPI 2/3: aux = z (bf16, no bias); C = gelu(z + b) evaluated on the ROUNDED z
    // exactly like the unfused GEMM -> bias_gelu path (3: erf GELU).  The GELU
    // runs in the drain, 8 columns per lane (one bias chunk per lane).
    // EPI 6/7: the same C, but aux = bf16(gelu'(z + b)) -- the derivative the
    // backward needs, from the same tanh/erf -- so the backward's drain is one
    // multiply instead of a GELU derivative per element (EPI 8).
    park([&](float v, int, int) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(v)); });
    float b8[8];
    if (gn < g.N) {
      Elem<kBF16>::load8(g.bias + gn, b8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b8[j] = 0.f;
    }
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int row = i * 8 + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4*>(reg + row * 128 + ((ch ^ (row & 7)) << 4));
      const int gm = row_base + row;
      if (gm < g.M && gn < g.N) {
        float z[8];
        Elem<kBF16>::load8(reinterpret_cast<const uint16_t*>(&v), z);
        bf16x8 hb;
        if constexpr (EPI <= 3) {
          st16<kNtAux>(g.aux + (int64_t)gm * g.ldaux + gn, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) hb[j] = static_cast<__bf16>(gelu_f(z[j] + b8[j], EPI == 3));
        } else {
          bf16x8 db;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float gv, dgv;
            gelu_and_grad(z[j] + b8[j], EPI == 7, gv, dgv);
            hb[j] = static_cast<__bf16>(gv);
            db[j] = static_cast<__bf16>(dgv);
          }
          st16<kNtAux>(g.aux + (int64_t)gm * g.ldaux + gn, db);
        }
        st16<kNtC>(g.C + (int64_t)gm * g.ldc + gn, hb);
      }
    }
  } else {
    // EPI 4/5 (DGELU, the MLP down-projection's input gradient): g = A.B^T is
    // rounded to bf16 (what the unfused GEMM stores), then C = g * gelu'(z + b)
    // with z = aux (the up-projection's pre-activation, an INPUT here) -- the
    // bias+GELU backward kernel's pass over [tokens, 4C] rides in the drain.
    // Each wave also sums its 128 rows of C (bf16-rounded, as that kernel does)
    // per column: one fp32 partial row per wave, part[2 * tm + wr][n], for the
    // up-projection's bias gradient.
    // the lane's 16 rows x 8 columns of z are loaded up front -- in flight
    // while the accumulators are parked, and held in the registers the parked
    // accumulators free -- instead of one dependent load per drain row
    uint4 zr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int gm = min(row_base + i * 8 + (lane >> 3), g.M - 1);
      zr[i] = gn < g.N ? ld16<kNtAux>(g.aux + (int64_t)gm * g.ldaux + gn) : make_uint4(0, 0, 0, 0);
    }
    park([&](float v, int, int) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(v)); });
    float b8[8], cs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cs[j] = 0.f;
    if (EPI != 8 && gn < g.N) {
      Elem<kBF16>::load8(g.bias + gn, b8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b8[j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = i * 8 + (lane >> 3);
      const uint4 v = *reinterpret_cast<const uint4*>(reg + row * 128 + ((ch ^ (row & 7)) << 4));
      const int gm = row_base + row;
      if (gm < g.M && gn < g.N) {
        float gv[8], z[8], o[8];
        Elem<kBF16>::load8(reinterpret_cast<const uint16_t*>(&v), gv);
        Elem<kBF16>::load8(reinterpret_cast<const uint16_t*>(&zr[i]), z);
        bf16x8 ob;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if constexpr (EPI == 8) {
            o[j] = gv[j] * z[j];  // aux holds gelu'(z + b) already (EPI 6/7 forward)
          } else {
            o[j] = gv[j] * gelu_grad(z[j] + b8[j], EPI == 5);
          }
          ob[j] = static_cast<__bf16>(o[j]);  // v_cvt_pk_bf16_f32 (RNE)
          cs[j] += static_cast<float>(ob[j]);  // the bias gradient sums the stored bf16 values
        }
        st16<kNtC>(g.C + (int64_t)gm * g.ldc + gn, ob);
      }
    }
    // fold the 8 lanes that share this lane's 8 columns (lane bits 3..5)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      cs[j] += __shfl_xor(cs[j], 8);
      cs[j] += __shfl_xor(cs[j], 16);
      cs[j] += __shfl_xor(cs[j], 32);
    }
    if (lane < 8 && gn < g.N) {
      float* dst = g.part + (int64_t)(2 * tm + wr) * g.N + gn;
      *reinterpret_cast<float4*>(dst) = make_float4(cs[0], cs[1], cs[2], cs[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
    }
  }
}

}  // namespace

// diagnostic: plain GEMM (EPI 0) with per-block timestamps into stamps[grid][8]
hipError_t launch_gemm_nt_stamped(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                                  unsigned long long* stamps, hipStream_t st) {
  if (K % 128 != 0 || N % 8 != 0) return hipErrorInvalidValue;
  GemmArgs g{};
  g.A = static_cast<const uint16_t*>(A);
  g.B = static_cast<const uint16_t*>(B);
  g.C = static_cast<uint16_t*>(C);
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.tiles_m = (M + kBM - 1) / kBM;
  g.tiles_n = (N + kBN - 1) / kBN;
  g.stamps = stamps;
  hipLaunchKernelGGL((gemm_nt_kernel<0, true>), dim3(g.tiles_m * g.tiles_n), dim3(512), 0, st, g);
  return hipGetLastError();
}


hipError_t launch_gemm_nt(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                          void* aux, int ldaux, int M, int N, int K, int epi, float* part, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K % 128 != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || ldc % 8 != 0) return hipErrorInvalidValue;
  if ((int64_t)M * lda >= (1ll << 31) || (int64_t)N * ldb >= (1ll << 31)) return hipErrorInvalidValue;
  if (epi >= 2 && (aux == nullptr || ldaux % 8 != 0)) return hipErrorInvalidValue;
  if (epi >= 1 && epi != 8 && (bias == nullptr || reinterpret_cast<uintptr_t>(bias) % 16 != 0))
    return hipErrorInvalidValue;
  if ((epi == 4 || epi == 5 || epi == 8) && (part == nullptr || reinterpret_cast<uintptr_t>(part) % 16 != 0))
    return hipErrorInvalidValue;
  GemmArgs g;
  g.A = static_cast<const uint16_t*>(A);
  g.B = static_cast<const uint16_t*>(B);
  g.C = static_cast<uint16_t*>(C);
  g.bias = static_cast<const uint16_t*>(bias);
  g.aux = static_cast<uint16_t*>(aux);
  g.part = part;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.ldaux = ldaux;
  g.M = M;
  g.N = N;
  g.K = K;
  g.tiles_m = (M + kBM - 1) / kBM;
  g.tiles_n = (N + kBN - 1) / kBN;
  const dim3 grid(g.tiles_m * g.tiles_n), block(512);
  switch (epi) {
    case 0: hipLaunchKernelGGL(gemm_nt_kernel<0>, grid, block, 0, st, g); break;
    case 1: hipLaunchKernelGGL(gemm_nt_kernel<1>, grid, block, 0, st, g); break;
    case 2: hipLaunchKernelGGL(gemm_nt_kernel<2>, grid, block, 0, st, g); break;
    case 3: hipLaunchKernelGGL(gemm_nt_kernel<3>, grid, block, 0, st, g); break;
    case 4: hipLaunchKernelGGL(gemm_nt_kernel<4>, grid, block, 0, st, g); break;
    case 5: hipLaunchKernelGGL(gemm_nt_kernel<5>, grid, block, 0, st, g); break;
    case 6: hipLaunchKernelGGL(gemm_nt_kernel<6>, grid, block, 0, st, g); break;
    case 7: hipLaunchKernelGGL(gemm_nt_kernel<7>, grid, block, 0, st, g); break;
    case 8: hipLaunchKernelGGL(gemm_nt_kernel<8>, grid, block, 0, st, g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dlion

// Causal flash attention (forward + backward, optional dropout) for gfx950.
//
// Replaces PyTorch SDPA (aotriton on ROCm) plus the layout copies around it
// (q/k/v unbind + stack in backward, output transpose) in the GPT-2/Llama
// blocks.  Inputs are read in their native strided layout ([B,T,3,H,D] packed
// qkv for GPT-2, separate [B,T,H,D] / [B,T,Hkv,D] for Llama GQA) and the
// gradients are written straight into the packed dqkv layout.
//
// Structure (all three kernels): a 256-thread block = 4 waves, each wave owns
// one 32-row tile (queries for fwd / dQ, keys for dKV) of ONE head, and the
// block streams the other side's 32-row tiles through LDS: one cooperative
// 16-byte load per thread-chunk per tile, issued before the current tile's
// math and written to the other LDS buffer after it (guide T14), so every
// K/V (or Q/dO) tile leaves L2 once per block instead of once per wave.
//
// Math (guide §3 "accumulator tile as the next MFMA's operand"): only
// v_mfma_f32_32x32x16_bf16.  Scores are computed TRANSPOSED, S^T = K Q^T, so
// the accumulator has the query on the lane and 16 keys in registers: the
// softmax row reduction is in-register plus one v_permlane32_swap, and P^T
// feeds O^T += V^T P^T with no lane movement.  The V^T / K^T / Q^T / dO^T
// operand fragments are read straight from the row-major LDS tiles with
// ds_read_b64_tr_b16 (hardware transpose, guide T10) -- no transposed copies
// in HBM.  Backward uses two kernels without atomics:
//   dKV: per 32-key tile, S = Q K^T orientation (key on the lane), loops over
//        query tiles accumulating dV += Pd^T dO and dK += dS^T Q in registers;
//   dQ : per 32-query tile, forward orientation, dQ += dS K.
// Dropout: keep(q, key) is a stateless hash of (seed, b*H+h, q, key) with
// 16-bit resolution, so forward and both backward kernels regenerate the
// identical mask in any register layout.
#include "common.h"
#include "attention.h"

#include <cstdlib>

// Occupancy floors (waves per SIMD), A/B-measured (profiles/r3/attn_occupancy_ab.txt):
// dK/dV D=64 at 3 waves fits 168 VGPRs without spills and is ~4 % faster over
// fwd+bwd; dK/dV D=128 at 2 waves (~30 dwords of spill) does not pay.  dQ D=64
// at 4 waves: 12 dwords of spill in round 3 (slower); since the round-4/5
// kernel changes it fits 128 VGPRs with 3 dwords spilled outside the key loop
// (its epilogue addresses) and runs the GPT-2 bench 1.070-1.071M -> 1.075-1.077M
// (profiles/r5/attn_dq4_c14.txt).
#ifndef DLION_DKV_WAVES64
#define DLION_DKV_WAVES64 3
#endif
#ifndef DLION_DQ_WAVES64
#define DLION_DQ_WAVES64 4
#endif
// key tiles per barrier in the D = 64 forward
#ifndef DLION_FWD_NT64
#define DLION_FWD_NT64 2
#endif
#ifndef DLION_DKV_WAVES128
#define DLION_DKV_WAVES128 1
#endif
// dK/dV at D = 128 without dropout: the wave's K tile in registers (32 VGPRs)
// instead of LDS, which takes the block's LDS from 97.5 to 65.5 KiB -- two
// blocks per CU, two waves per SIMD (the kernel fits 256 VGPRs there).
// Interleaved (tools/r5/bench_dkv_kreg.py, profiles/r5/dkv_kreg_c38.txt):
// Llama-2-7B SFT shape (no GQA) fwd + bwd 0.309 -> 0.283 ms, SFT preset
// +0.5-1.4 %; at Llama-3-8B's GQA shape (4 heads per K/V head) 0.777 ->
// 0.806 ms, so the launcher takes it only when H == Hkv.
#ifndef DLION_DKV_KREG128
#define DLION_DKV_KREG128 1
#endif
// LDS ring depth of the 4-wave backward kernels' streamed tiles: tile i+NB-1
// is staged while tile i is consumed (NB = 2: classic double buffering).
// NB = 3 spills 34 dwords in dK/dV under the 3-wave floor (168 VGPRs) and
// lifts dQ from 133 to 162 VGPRs: GPT-2 bench 977k (NB 3) vs 1007k (NB 2)
// same box (profiles/r3/attn_stages_ab.txt)
#ifndef DLION_ATTN_STAGES
#define DLION_ATTN_STAGES 2
#endif
// Variants measured neutral or slower and removed in round 5 (numbers in
// docs/DESIGN.md and profiles/r4/): dQ's Q / dO rows read from LDS per tile,
// a start stagger between co-resident blocks, dK/dV's K fragments held in
// registers or loaded straight from global memory, two key tiles per barrier
// in dQ, non-temporal O / dQ / dK / dV stores, per-kernel ring depths, LDS
// fragment prefetch before the VALU section, and the dQ cycle-stamp build.
//
// s_setprio 1 around the first (1) / second (2) MFMA phase of each tile, per
// kernel.  At the GPT-2 shape (interleaved, 2 rounds) the second phase at
// priority 1 took fwd 69.3-69.9 -> 67.9-68.2 us and dK/dV 117-119 -> 115 us,
// but dQ 85-86 -> 92 us (its dS VALU then waits behind the other waves' MFMAs)
constexpr int kFwdPrio = 2, kDqPrio = 0, kDkvPrio = 2;
#define DLION_PRIO_ON(mask, bit) if constexpr (((mask) & (bit)) != 0) __builtin_amdgcn_s_setprio(1)
#define DLION_PRIO_OFF(mask, bit) if constexpr (((mask) & (bit)) != 0) __builtin_amdgcn_s_setprio(0)

namespace dlion {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// drop hash (v2): 32 random bits shared by keys (2i, 2i+1) of query q, in two
// stages so the per-pair cost is one full-rate 24-bit multiply:
//   arow(bh, q)  = lowbias32(seed ^ bh*0x9E3779B9 ^ q*0x85EBCA6B)   (per row)
//   hash(q, key) = mix1(arow + (key>>1)*kKeyMul),
//   mix1(x) = y ^ (y >> 16),  y = (x mod 2^24) * 0x9E3779  (v_mul_u32_u24)
// The key enters by ADDITION (v1 xored it in): per tile the row constant and
// the tile's pair base fold into one register, and each pair costs one
// v_add with a literal + v_mul_u32_u24 + v_xor_b32_sdwa.
// Keep test, two keys at once on the packed halves (low = even key): the
// halves are read as SIGNED 16-bit values s and a key is kept iff
// s >= thresh16 - 32768 (same keep probability 1 - thresh16/65536 as an
// unsigned compare).  keep_mask2 gives 0xFFFF per kept half with a saturating
// v_pk_sub_i16 and a v_pk_ashrrev_i16 -- no v_cmp / VCC / v_cndmask (v1's
// per-element compare + select, with the VCC-hazard s_nops between them, was
// ~45 % of the forward's VALU work) -- and is applied to the packed bf16
// operand dword with one v_and (P) or v_bfi_b32 (dS).
constexpr uint32_t kKeyMul = 0xC2B2AE35u;
__device__ __forceinline__ uint32_t drop_row(uint32_t seed, uint32_t bh, uint32_t q) {
  return lowbias32(seed ^ (bh * 0x9E3779B9u) ^ (q * 0x85EBCA6Bu));
}
__device__ __forceinline__ uint32_t mix1(uint32_t x) {
  x = __umul24(x, 0x9E3779u);
  return x ^ (x >> 16);
}
// drop hash v3: the pair hash of tile kt starts from a per-(row, tile) base,
// each tile reading a different 24-bit view (rotation by 8 (kt mod 4)) of the
// 32-bit row key: v2's base arow + 16 kt kKeyMul was linear in the tile, so
// every row's mask was a window of one fixed sequence (rows a small multiple
// of kKeyMul apart had shifted copies of each other's masks) and rows sharing
// arow's low 24 bits had identical masks (CPU statistics in
// tests/test_attention_gpu.py).  4 VALU per tile and lane.
constexpr uint32_t kTileMul = 0x27D4EB2Fu;
__device__ __forceinline__ uint32_t tile_base(uint32_t arow, int kt) {
  return mix1(__builtin_amdgcn_alignbit(arow, arow, 8u * static_cast<uint32_t>(kt & 3)) ^
              (static_cast<uint32_t>(kt) * kTileMul));
}
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// tm1 = (thresh16 - 32769) mod 2^16 in both halves (thresh16 >= 1)
__device__ __forceinline__ uint32_t drop_tm1(uint32_t thresh16) {
  const uint32_t t = (thresh16 - 32769u) & 0xFFFFu;
  return t | (t << 16);
}
// 0xFFFF per half whose signed random u16 is >= tm1 + 1 (kept), else 0
__device__ __forceinline__ uint32_t keep_mask2(uint32_t u, uint32_t tm1) {
  const s16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2, tm1), __builtin_bit_cast(s16x2, u));
  const s16x2 m = d >> (s16x2){15, 15};
  return __builtin_bit_cast(uint32_t, m);
}
// (m & a) | (~m & b) as one v_bfi_b32 (written as C, hipcc turns it back
// into per-half compares and selects)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
// two floats -> packed bf16 (v_cvt_pk_bf16_f32, RNE), low half = a
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const bf16x2 v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, v);
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
__device__ __forceinline__ void st_bf16(__bf16* p, float v) { *p = static_cast<__bf16>(v); }
// accumulator registers 8s..8s+7 as a bf16 operand fragment (k-step s).  The
// k order this gives -- rows {0..3, 8..11} + 4hf (+16s) -- is the "permuted k"
// every partner operand below is read in.
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(x[8 * s + j]);
  return r;
}
__device__ __forceinline__ int acc_row(int reg, int hf) { return (reg & 3) + 8 * (reg >> 2) + 4 * hf; }
// key-pair index, relative to the tile's pair base (key >> 1 of the lane's
// first key: kt*16 + 2hf), of the two keys in dword i (regs 8s+2i, 8s+2i+1)
// of acc_frag(x, s)
__device__ __forceinline__ constexpr int frag_pair(int s, int i) { return (i & 1) + 4 * (i >> 1) + 8 * s; }

// P^T operand (query on the lane, keys in registers) with the dropout mask
// applied to the packed bf16 pairs.  pbase = arow + (kt*16 + 2hf) * kKeyMul.
template <bool DROP>
__device__ __forceinline__ bf16x8 p_frag(const f32x16& x, int s, uint32_t pbase, uint32_t tm1) {
  bf16x8 f = acc_frag(x, s);
  if constexpr (DROP) {
    i32x4 d = __builtin_bit_cast(i32x4, f);
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] &= keep_mask2(mix1(pbase + frag_pair(s, i) * kKeyMul), tm1);
    f = __builtin_bit_cast(bf16x8, d);
  }
  return f;
}
// dS^T operand of the dQ kernel: dS = P (keep ? dP : 0) - P delta, built as
// both packed candidates and merged per half by the keep mask (one v_bfi_b32)
template <bool DROP>
__device__ __forceinline__ bf16x8 ds_frag(const f32x16& p, const f32x16& dp, float dlt, int s, uint32_t pbase,
                                          uint32_t tm1) {
  i32x4 d;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = 8 * s + 2 * i;
    if constexpr (DROP) {
      const float a0 = p[r0] * dlt, a1 = p[r0 + 1] * dlt;
      const uint32_t kv = pk2(__builtin_fmaf(p[r0], dp[r0], -a0), __builtin_fmaf(p[r0 + 1], dp[r0 + 1], -a1));
      d[i] = bfi(keep_mask2(mix1(pbase + frag_pair(s, i) * kKeyMul), tm1), kv, pk2(-a0, -a1));
    } else {
      d[i] = pk2(p[r0] * (dp[r0] - dlt), p[r0 + 1] * (dp[r0 + 1] - dlt));
    }
  }
  return __builtin_bit_cast(bf16x8, d);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ------------------------------------------------------------- LDS tiles
// A 32-row x D tile, unpadded rows, 16-byte chunks XOR-swizzled per row so
// that all three access patterns are bank-conflict-free (guide T2/T10; model
// and check: tools/lds_bank_sim.py): the ds_read_b128 row reads of the
// 32x32x16 operand (16 lanes = 16 rows, one chunk), the ds_read_b64_tr_b16
// transposed reads (a 32-lane half = 4 rows x 4 chunks) and the ds_write_b128
// staging stores.  The first layout (rows padded by 8 bf16) left the
// transposed reads 2-way (D=64) / 4-way (D=128): SQ_LDS_BANK_CONFLICT was 50%
// of the LDS-active cycles at D=128.
template <int D>
using LdsTile = __bf16[32 * D];

template <int D>
__device__ __forceinline__ int swz_chunk(int row, int ch) {
  if constexpr (D == 128) return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  else return ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
}
// element offset of 16-byte chunk `ch` of row `row`
template <int D>
__device__ __forceinline__ int lds_off(int row, int ch) { return row * D + 8 * swz_chunk<D>(row, ch); }

// row fragment: row `r` of the tile, columns 16ks + 8hf .. +7 (an operand whose
// m / n index is the lane's row, k = the D axis)
template <int D>
__device__ __forceinline__ bf16x8 row_frag(const LdsTile<D>& t, int r, int ks, int hf) {
  return *reinterpret_cast<const bf16x8*>(&t[lds_off<D>(r, 2 * ks + hf)]);
}
// transposed fragment: column d = 32tt + (lane & 31) of the tile, rows in the
// permuted-k order of acc_frag(s2): {0..3, 8..11} + 4hf + 16s2.  Two
// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, columns
// 4p..4p+3 of a 4x16 block and lane i receives column i of the 4 rows
// (verified on gfx950 with tools/probes/tr_read.hip).
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const LdsTile<D>& t, int s2, int tt, int lane) {
  const int j = lane & 15, hf = lane >> 5, gh = (lane >> 4) & 1;
  const int row = 16 * s2 + 4 * hf + (j >> 2), ch = 4 * tt + 2 * gh + ((j & 3) >> 1), sub = 4 * (j & 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&t[lds_off<D>(row, ch) + sub]));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&t[lds_off<D>(row + 8, ch) + sub]));
  // assemble as whole dwords: per-element bf16 inserts of the builtin's result
  // miscompile (only dword 0 of each read survived, replicated by v_perm)
  const i32x2 l2 = __builtin_bit_cast(i32x2, lo), h2 = __builtin_bit_cast(i32x2, hi);
  const i32x4 r = {l2[0], l2[1], h2[0], h2[1]};
  return __builtin_bit_cast(bf16x8, r);
}

// LDS-DMA staging of one 32 x D tile (global_load_lds_dwordx4, guide §5 /
// T3): each wave moves 1 KiB pieces (64 lanes x 16 B) straight into LDS, so
// the tile costs no staging VGPRs, no ds_write and -- the point -- the fetch
// is issued where it is written, a whole tile ahead of its use.  (The
// register-staged version had its global loads sunk past the branchy compute
// block to just before their ds_write, and for D=128 the staging registers
// were even kept in scratch: every tile paid the full fetch latency.)  A
// piece lands lane-linear at base + 16*lane, so the swizzle of lds_off goes on
// the SOURCE side: LDS chunk slot p = row*CPR + pos holds source chunk
// swz_chunk(row, pos) (the XOR is an involution).
//
// Issued through inline asm, not __builtin_amdgcn_global_load_lds: for the
// builtin hipcc cannot tell the DMA's LDS buffer (buf^1) from the one the
// math reads (buf) and puts an s_waitcnt vmcnt(0) before the first ds_read,
// serialising the prefetch again.  The asm is invisible to its waitcnt pass,
// so every consumer goes through vm_wait0() + barrier; the compiler's own
// counted vmcnt waits stay correct (ops issued later only make a vmcnt(N)
// stricter).  M0 = the wave-uniform LDS destination.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p)));
}
__device__ __forceinline__ void glds16(const __bf16* src, const void* dst) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr(dst)));
}
// scalar-base form: SGPR-pair tile base + per-lane 32-bit byte offset -- the
// address costs no VALU (the 64-bit form paid a v_mul_lo_u32 + two
// v_lshl_add_u64 per piece on a tile row that is wave-uniform anyway)
__device__ __forceinline__ void glds16s(const __bf16* base, uint32_t boff, const void* dst) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(boff), "s"(base),
               "s"(lds_addr(dst)));
}
__device__ __forceinline__ void glds4(const float* src, const void* dst) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds_addr(dst)));
}
// the same three with the destination as a 32-bit LDS byte address computed
// once per kernel (lds_addr of the generic pointer costs a shared-aperture
// null check -- s_mov src_shared_base, s_cmp, s_cselect -- per piece)
__device__ __forceinline__ void glds16_a(const __bf16* src, uint32_t dst) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst));
}
__device__ __forceinline__ void glds16s_a(const __bf16* base, uint32_t boff, uint32_t dst) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(boff), "s"(base), "s"(dst));
}
__device__ __forceinline__ void glds4_a(const float* src, uint32_t dst) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(dst));
}
// vmcnt(0) through the builtin (gfx9 encoding: lgkmcnt 15, expcnt 7, vmcnt 0),
// not asm: the waitcnt pass then knows the Q/K/V register loads issued
// before it are complete, instead of re-waiting for them with counted vmcnt
// inside the loop -- which, counting the asm DMAs too, drained the prefetch
__device__ __forceinline__ void vm_wait0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// vmcnt(n) for a wave-uniform n < 16 (scalar branch over the immediates)
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(0x0F70); break;
    case 1: __builtin_amdgcn_s_waitcnt(0x0F71); break;
    case 2: __builtin_amdgcn_s_waitcnt(0x0F72); break;
    case 3: __builtin_amdgcn_s_waitcnt(0x0F73); break;
    case 4: __builtin_amdgcn_s_waitcnt(0x0F74); break;
    case 5: __builtin_amdgcn_s_waitcnt(0x0F75); break;
    case 6: __builtin_amdgcn_s_waitcnt(0x0F76); break;
    case 7: __builtin_amdgcn_s_waitcnt(0x0F77); break;
    case 8: __builtin_amdgcn_s_waitcnt(0x0F78); break;
    case 9: __builtin_amdgcn_s_waitcnt(0x0F79); break;
    case 10: __builtin_amdgcn_s_waitcnt(0x0F7A); break;
    default: __builtin_amdgcn_s_waitcnt(0x0F7B); break;
  }
}

template <int D>
struct DmaTile {
  static constexpr int CPR = D / 8, PPW = D / 64;  // 16-byte chunks per row, 1 KiB pieces per wave
  static_assert(D == 64 || D == 128, "head dim");
  int off0, off1, lds;  // source element offsets (tile-relative) of the lane's chunks; wave's LDS byte offset
  uint32_t boff0, boff1;  // the same as byte offsets (scalar-base DMA)
  int r0, r1, c0, c1, st;  // the lane's tile rows / swizzled chunk offsets, for partial (tail) tiles
  __device__ __forceinline__ DmaTile(int64_t stride) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int p0 = 64 * PPW * w + lane, p1 = p0 + 64;
    r0 = p0 / CPR;
    r1 = p1 / CPR;
    c0 = 8 * swz_chunk<D>(r0, p0 % CPR);
    c1 = 8 * swz_chunk<D>(r1, p1 % CPR);
    st = static_cast<int>(stride);
    off0 = r0 * st + c0;
    off1 = r1 * st + c1;
    boff0 = 2u * static_cast<uint32_t>(off0);
    boff1 = 2u * static_cast<uint32_t>(off1);
    lds = 1024 * PPW * w;
  }
  // `valid` = rows of the sequence left from this tile's first row: a tail
  // tile (valid < 32) re-reads row valid-1 for its missing rows -- memory
  // that exists; those rows are masked or dropped by every consumer.
  // `tile` is wave-uniform (the full-tile form passes it in SGPRs).
  __device__ __forceinline__ void issue(const __bf16* tile, LdsTile<D>& t, int valid = 32) const {
    char* dst = reinterpret_cast<char*>(&t[0]) + lds;
    if (valid >= 32) {  // block-uniform
      glds16s(tile, boff0, dst);
      if constexpr (PPW == 2) glds16s(tile, boff1, dst + 1024);
    } else {
      glds16(tile + min(r0, valid - 1) * st + c0, dst);
      if constexpr (PPW == 2) glds16(tile + min(r1, valid - 1) * st + c1, dst + 1024);
    }
  }
  // issue() into the tile at LDS byte address `ldsb` (lds_addr of the tile,
  // hoisted out of the loop by the caller)
  __device__ __forceinline__ void issue_at(const __bf16* tile, uint32_t ldsb, int valid = 32) const {
    const uint32_t dst = ldsb + static_cast<uint32_t>(lds);
    if (valid >= 32) {  // block-uniform
      glds16s_a(tile, boff0, dst);
      if constexpr (PPW == 2) glds16s_a(tile, boff1, dst + 1024);
    } else {
      glds16_a(tile + min(r0, valid - 1) * st + c0, dst);
      if constexpr (PPW == 2) glds16_a(tile + min(r1, valid - 1) * st + c1, dst + 1024);
    }
  }
};

// 32-row tiles covering T (the last one may be partial)
__device__ __forceinline__ int ntiles32(int T) { return (T + 31) >> 5; }

// query-side blocks (fwd, dQ): heads fastest, heavy (late) query groups first
struct QBlock {
  int bh, qtile, last;
  bool active;
  __device__ __forceinline__ QBlock(int nbh, int ntiles) {
    const int ngroups = (ntiles + 3) >> 2, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branches
    bh = static_cast<int>(blockIdx.x % nbh);
    const int grp = ngroups - 1 - static_cast<int>(blockIdx.x / nbh);
    qtile = grp * 4 + w;
    last = min(grp * 4 + 3, ntiles - 1);  // block-uniform loop bound
    active = qtile < ntiles;
  }
};

// The sliding window is compiled for D = 128 only (Mistral-7B; the D = 64
// GPT-2 / Qwen2-0.5B kernels stay as they were -- the window's registers put
// dQ D = 64 past its 4-wave budget: 12-19 dwords of spill); the host refuses a
// window at D = 64 (ops/fused.py then takes the masked SDPA path).
template <int D>
__device__ __forceinline__ int window_of(const AttnArgs& a) { return D == 128 ? a.window : 0; }

// Sliding-window key range of a query-side wave (fwd, dQ): its first key tile
// wlo (row qtile*32's lowest key, q - window + 1) and the block's first
// NT-aligned key tile kstart (its first wave's wlo); window 0 = from key 0.
struct SlideRange {
  int wlo, kstart, lim;
  __device__ __forceinline__ SlideRange(int window, int qtile, int w, int nt) {
    if (window > 0) {
      wlo = max(0, qtile * 32 - window + 1) >> 5;
      kstart = ((max(0, (qtile - w) * 32 - window + 1) >> 5) / nt) * nt;
      lim = qtile * 32 + 31 - window;  // keys <= lim are outside some row's window
    } else {
      wlo = kstart = 0;
      lim = -1;
    }
  }
  // a key-tile group starting at tile kt holds keys outside some row's window
  __device__ __forceinline__ bool cut(int kt, int) const { return kt * 32 <= lim; }
};

// scores with the query on the lane (fwd / dQ orientation): -inf where key <= q - window
template <int NT>
__device__ __forceinline__ void window_mask_qlane(f32x16 (&s)[NT], int kt, int q, int window, int hf) {
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg)
      if ((kt + j) * 32 + acc_row(reg, hf) <= q - window) s[j][reg] = -INFINITY;
}

// ------------------------------------------------------------------ forward
// NT key tiles (32 keys each) per barrier: with NT = 2 every wave has two
// independent QK^T chains and two PV chains per iteration, so hipcc can put one
// tile's MFMAs beside the other's softmax VALU work; with NT = 1 each step of
// the QK -> max -> exp -> PV chain waits for the previous one.  (Software-
// pipelined variants -- QK^T of the next tile issued before this tile's
// softmax -- measured neutral to -1 % in round 3 and were removed.)
template <int D, bool DROP, int NT>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) LdsTile<D> ks_[2][NT];
  __shared__ __attribute__((aligned(16))) LdsTile<D> vs_[2][NT];
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5;
  const QBlock blk(a.B * a.H, ntiles32(a.T));
  const int bh = blk.bh, qtile = blk.qtile, last = blk.last;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int q = qtile * 32 + r;
  // rows past T (tail tile): computed on a copy of row T-1, never stored; keys
  // past T are behind every valid query, so the causal mask already drops them
  const int qc = min(q, a.T - 1);
  const int win = window_of<D>(a);
  const SlideRange sw(win, qtile, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), NT);

  bf16x8 qf[D / 16];
  if (blk.active) {
    const __bf16* qp = a.q + b * a.q_sb + static_cast<int64_t>(qc) * a.q_st + h * a.q_sh + 8 * hf;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) qf[s] = ld8(qp + 16 * s);
  }
  f32x16 oacc[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) oacc[t] = zero16();
  // a finite start under a sliding window: a row whose keys in the wave's first
  // tile are all masked then gets p = 0 there instead of exp2(-inf + inf)
  float m = win > 0 ? -1e30f : -INFINITY, l = 0.f;

  const __bf16* kg = a.k + b * a.k_sb + hk * a.k_sh;
  const __bf16* vg = a.v + b * a.v_sb + hk * a.v_sh;
  // dropout: the row key; per key tile the pair base tile_base(arow, kt) + 2hf kKeyMul
  const uint32_t arow = drop_row(a.seed, bh, q), hoff = static_cast<uint32_t>(2 * hf) * kKeyMul;
  const uint32_t tm1 = drop_tm1(a.thresh16);
  const DmaTile<D> kd(a.k_st), vd(a.v_st);
  const uint32_t ks_lds = lds_addr(&ks_[0][0]), vs_lds = lds_addr(&vs_[0][0]);
  constexpr uint32_t kTileB = sizeof(LdsTile<D>);
  // tiles past `last` re-read tile `last` (valid memory); the causal mask
  // zeroes them, since they lie beyond every query of the block.  stage() is
  // called for kstart, kstart + NT, ... in order: the tile pointers advance by
  // adds (the dQ / dK/dV kernels' strength reduction)
  const int64_t kstep = 32 * a.k_st, vstep = 32 * a.v_st;
  const __bf16* kn = kg + static_cast<int64_t>(sw.kstart) * kstep;
  const __bf16* vn = vg + static_cast<int64_t>(sw.kstart) * vstep;
  const __bf16* kl = kg + static_cast<int64_t>(last) * kstep;
  const __bf16* vl = vg + static_cast<int64_t>(last) * vstep;
  auto stage = [&](int first, int buf) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int row = __builtin_amdgcn_readfirstlane(min(first + j, last) * 32);
      const bool in = NT == 1 || first + j <= last;
      const uint32_t slot = static_cast<uint32_t>(buf * NT + j) * kTileB;
      kd.issue_at(in ? kn + j * kstep : kl, ks_lds + slot, a.T - row);
      vd.issue_at(in ? vn + j * vstep : vl, vs_lds + slot, a.T - row);
    }
    kn += NT * kstep;
    vn += NT * vstep;
  };
  stage(sw.kstart, (sw.kstart / NT) & 1);
  vm_wait0();
  __syncthreads();
  for (int kt = sw.kstart; kt <= last; kt += NT) {
    const int buf = (kt / NT) & 1;
    if (kt + NT <= last) stage(kt + NT, buf ^ 1);  // the other buffer was last read before the previous barrier
    if (blk.active && kt <= qtile && kt + NT - 1 >= sw.wlo) {  // wave-uniform
      f32x16 s[NT];
      DLION_PRIO_ON(kFwdPrio, 1);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        s[j] = zero16();
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) s[j] = mfma32(row_frag<D>(ks_[buf][j], r, ks, hf), qf[ks], s[j]);
      }
      DLION_PRIO_OFF(kFwdPrio, 1);
      if (kt + NT - 1 >= qtile) {  // the diagonal (or tiles past it) in this group: causal mask
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int reg = 0; reg < 16; ++reg)
            if ((kt + j) * 32 + acc_row(reg, hf) > q) s[j][reg] = -INFINITY;
      }
      if (sw.cut(kt, qtile)) window_mask_qlane<NT>(s, kt, q, win, hf);
      // row max on the raw scores (scale > 0); the scale is folded into the
      // exponent's FMA instead of a separate multiply pass
      float tmax = s[0][0];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) tmax = fmaxf(tmax, s[j][reg]);
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
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j][reg], a.scale_log2, -m));
          rs += p;
          s[j][reg] = p;
        }
      l = l * alpha + xsum32(rs);
      // PV with the dropout mask on the packed bf16 P pairs (1/(1-p) is
      // applied once to O at the end)
      DLION_PRIO_ON(kFwdPrio, 2);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint32_t pb = DROP ? tile_base(arow, kt + j) + hoff : 0u;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 pf = p_frag<DROP>(s[j], s2, pb, tm1);
#pragma unroll
          for (int t = 0; t < D / 32; ++t)
            oacc[t] = mfma32(tr_frag<D>(vs_[buf][j], s2, t, lane), pf, oacc[t]);
        }
      }
      DLION_PRIO_OFF(kFwdPrio, 2);
    }
    vm_wait0();  // this wave's pieces of the next tiles have landed
    __syncthreads();
  }
  if (!blk.active || q >= a.T) return;
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
  // under dropout the stored row constant is lse + log2(1-p): the backward's
  // exp2(s*scale - lse') is then P/(1-p) directly, and with delta' = delta*(1-p)
  // (computed in the dQ kernel) both backward kernels drop their per-element 1/(1-p)
  // multiplies: dS = P'*(keep ? dP : 0) - P'*delta', Pd = keep ? P' : 0
  if (hf == 0) a.lse[static_cast<int64_t>(bh) * a.T + q] = m + log2f(l) + (DROP ? -log2f(a.inv_keep) : 0.f);
}

// --------------------------------------------------------------- backward dQ
// One 32-query tile per wave, key tiles streamed through a DLION_ATTN_STAGES
// ring; NT key tiles per barrier (see the forward; dQ runs NT = 1: NT = 2 was
// 4 % slower, profiles/r4/attn_dq_nt2_ab.txt).  (Round 3's software-pipelined
// and sequential-NT variants measured neutral and were removed.)
// Inverse rotary embedding of a [32 rows (registers)] x [D (lane + 32 t)]
// accumulator set, in place, before the store: with x = (x1 | x2) halves,
// dx1 = g1 cos1 + g2 sin2, dx2 = g2 cos2 - g1 sin1 (the gradient of
// rope(x) = x cos + rotate_half(x) sin; csrc/elementwise_kernels.hip
// rope_kernel, inverse) -- column d and d + D/2 sit in the same lane and
// register of tiles t and t + D/64.  Rows past T read row T-1's tables.
template <int D>
__device__ __forceinline__ void unrope(f32x16 (&x)[D / 32], const AttnArgs& a, int row0, int hf, int r) {
  constexpr int TH = D / 64;  // tiles per half
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int64_t pos = min(row0 + acc_row(reg, hf), a.T - 1);
    const __bf16* cr = a.rope_cos + pos * D;
    const __bf16* sr = a.rope_sin + pos * D;
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      const int d = 32 * t + r;
      const float c1 = static_cast<float>(cr[d]), c2 = static_cast<float>(cr[d + D / 2]);
      const float s1 = static_cast<float>(sr[d]), s2 = static_cast<float>(sr[d + D / 2]);
      const float g1 = x[t][reg], g2 = x[t + TH][reg];
      x[t][reg] = g1 * c1 + g2 * s2;
      x[t + TH][reg] = g2 * c2 - g1 * s1;
    }
  }
}

template <int D, bool DROP, int NT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D == 64 ? DLION_DQ_WAVES64 : 1)))
attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int NB = DLION_ATTN_STAGES;
  __shared__ __attribute__((aligned(16))) LdsTile<D> ks_[NB][NT];
  __shared__ __attribute__((aligned(16))) LdsTile<D> vs_[NB][NT];
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5;
  const int nt = ntiles32(a.T);
  const QBlock blk(a.B * a.H, nt);
  const int bh = blk.bh, qtile = blk.qtile, last = blk.last;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int q = qtile * 32 + r;
  const int qc = min(q, a.T - 1);  // tail rows: a copy of row T-1, never stored (see the forward)
  const int win = window_of<D>(a);
  const SlideRange sw(win, qtile, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), NT);

  bf16x8 qf[D / 16], dof[D / 16];
  float lse2 = 0.f, dlt = 0.f;
  if (blk.active) {
    const __bf16* qp = a.q + b * a.q_sb + static_cast<int64_t>(qc) * a.q_st + h * a.q_sh + 8 * hf;
    const __bf16* dop = a.dout + b * a.o_sb + static_cast<int64_t>(qc) * a.o_st + h * a.o_sh + 8 * hf;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      qf[s] = ld8(qp + 16 * s);
      dof[s] = ld8(dop + 16 * s);
    }
    lse2 = a.lse[static_cast<int64_t>(bh) * a.T + qc];
    // delta = rowsum(dO * O) for this wave's 32 rows, computed here (the dQ
    // kernel already holds the dO rows) and published for the dKV kernel that
    // runs next -- instead of a separate pass over O and dO.  Lanes r and r+32
    // hold the two halves of row q.
    const __bf16* op = a.o + b * a.o_sb + static_cast<int64_t>(qc) * a.o_st + h * a.o_sh + 8 * hf;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 of = ld8(op + 16 * s);
#pragma unroll
      for (int j = 0; j < 8; ++j) part += static_cast<float>(of[j]) * static_cast<float>(dof[s][j]);
    }
    dlt = xsum32(part);
    if (a.thresh16) dlt /= a.inv_keep;  // delta * (1-p), see the forward's lse note
    if (hf == 0 && q < a.T) const_cast<float*>(a.delta)[static_cast<int64_t>(bh) * a.T + q] = dlt;
  }
  const uint32_t arow = drop_row(a.seed, bh, q), hoff = static_cast<uint32_t>(2 * hf) * kKeyMul;
  const uint32_t tm1 = drop_tm1(a.thresh16);
  f32x16 dq[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dq[t] = zero16();
  const __bf16* kg = a.k + b * a.k_sb + hk * a.k_sh;
  const __bf16* vg = a.v + b * a.v_sb + hk * a.v_sh;
  const DmaTile<D> kd(a.k_st), vd(a.v_st);
  const uint32_t ks_lds = lds_addr(&ks_[0][0]), vs_lds = lds_addr(&vs_[0][0]);
  constexpr uint32_t kTileB = sizeof(LdsTile<D>);
  const int ns = last / NT + 1, st0 = sw.kstart / NT;
  // super-tile st = key tiles st*NT .. st*NT+NT-1, one LDS slot each; tiles
  // past `last` re-read tile `last` (valid memory) and are masked below.
  // stage() is called for st0, st0+1, ... in order: the K / V tile pointers
  // run one super-tile ahead by an add, not a 64-bit row * stride product
  const int64_t kstep = 32 * a.k_st, vstep = 32 * a.v_st;
  const __bf16* kn = kg + static_cast<int64_t>(st0 * NT) * kstep;
  const __bf16* vn = vg + static_cast<int64_t>(st0 * NT) * vstep;
  auto stage = [&](int st, int buf) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int row = __builtin_amdgcn_readfirstlane(min(st * NT + j, last) * 32);
      const uint32_t slot = static_cast<uint32_t>(buf * NT + j) * kTileB;
      if (NT == 1 || st * NT + j <= last) {
        kd.issue_at(kn + j * kstep, ks_lds + slot, a.T - row);
        vd.issue_at(vn + j * vstep, vs_lds + slot, a.T - row);
      } else {
        kd.issue_at(kg + static_cast<int64_t>(row) * a.k_st, ks_lds + slot, a.T - row);
        vd.issue_at(vg + static_cast<int64_t>(row) * a.v_st, vs_lds + slot, a.T - row);
      }
    }
    kn += NT * kstep;
    vn += NT * vstep;
  };
  for (int j = st0; j < st0 + NB - 1 && j < ns; ++j) stage(j, j % NB);
  for (int st = st0; st < ns; ++st) {
    const int buf = st % NB;
    // super-tile st has landed once only the later ones' pieces (NT * 2 PPW each) are in flight
    vm_wait_n(min(ns - 1 - st, NB - 2) * NT * 2 * DmaTile<D>::PPW);
    __syncthreads();  // ... for every wave; and every wave is done with the buffer restaged next
    if (st + NB - 1 < ns) stage(st + NB - 1, (st + NB - 1) % NB);
    const int kt0 = st * NT;
    if (blk.active && kt0 <= qtile && kt0 + NT - 1 >= sw.wlo) {
      // NT independent S / dP chains: one tile's exp / hash VALU work can sit
      // beside the other's MFMAs
      f32x16 s[NT], dp[NT];
      DLION_PRIO_ON(kDqPrio, 1);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        s[j] = zero16();
        dp[j] = zero16();
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
          s[j] = mfma32(row_frag<D>(ks_[buf][j], r, ks, hf), qf[ks], s[j]);    // S^T  = K Q^T
          dp[j] = mfma32(row_frag<D>(vs_[buf][j], r, ks, hf), dof[ks], dp[j]);  // dP^T = V dO^T
        }
      }
      DLION_PRIO_OFF(kDqPrio, 1);
      if (kt0 + NT - 1 >= qtile) {  // the diagonal (or tiles past it) in this group: exp2(-inf) = 0
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int reg = 0; reg < 16; ++reg)
            if ((kt0 + j) * 32 + acc_row(reg, hf) > q) s[j][reg] = -INFINITY;
      }
      if (sw.cut(kt0, qtile)) window_mask_qlane<NT>(s, kt0, q, win, hf);
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          s[j][reg] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j][reg], a.scale_log2, -lse2));  // p, carries 1/(1-p)
      DLION_PRIO_ON(kDqPrio, 2);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint32_t pb = DROP ? tile_base(arow, kt0 + j) + hoff : 0u;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 dsf = ds_frag<DROP>(s[j], dp[j], dlt, s2, pb, tm1);  // dS^T
#pragma unroll
          for (int t = 0; t < D / 32; ++t) dq[t] = mfma32(dsf, tr_frag<D>(ks_[buf][j], s2, t, lane), dq[t]);  // dQ += dS K
        }
      }
      DLION_PRIO_OFF(kDqPrio, 2);
    }
  }
  if (!blk.active) return;
  // dq[t]: rows = q (registers), cols = d (lane)
  __bf16* base = a.dq + b * a.dq_sb + h * a.dq_sh;
  if (a.rope_cos != nullptr) unrope<D>(dq, a, qtile * 32, hf, r);
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int qq = qtile * 32 + acc_row(reg, hf);
      if (qq < a.T) st_bf16(base + static_cast<int64_t>(qq) * a.dq_st + 32 * t + r, dq[t][reg] * a.scale);
    }
  if (a.colsum != nullptr) {
    // the c_attn bias gradient's partials: column sums of the stored (bf16) dq
    // over this wave's 32 rows (valid ones); lanes r and r+32 hold the two row halves
    float* cs = a.colsum + static_cast<int64_t>(b * nt + qtile) * (3 * a.H * D) + h * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) {
      float sum = 0.f;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg)
        if (qtile * 32 + acc_row(reg, hf) < a.T) sum += static_cast<float>(static_cast<__bf16>(dq[t][reg] * a.scale));
      sum = xsum32(sum);
      if (hf == 0) cs[32 * t + r] = sum;
    }
  }
}

// -------------------------------------------------------------- backward dKV
// 4 waves = 4 consecutive key tiles of one (b, kv-head); every query tile of
// every head in the GQA group is staged once per block (Q, dO and the 32
// lse / delta values).  Low key groups (most query tiles) go first.  (Round
// 3's software-pipelined variant measured -1 % and was removed.)
template <int D, bool DROP, bool KREG = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    D == 64 ? DLION_DKV_WAVES64 : (KREG ? 2 : DLION_DKV_WAVES128))))
attn_bwd_dkv_kernel(AttnArgs a) {
  constexpr int NB = DLION_ATTN_STAGES;
  __shared__ __attribute__((aligned(16))) LdsTile<D> qs_[NB];
  __shared__ __attribute__((aligned(16))) LdsTile<D> ds_[NB];
  static_assert(!KREG || (D == 128 && !DROP), "K in registers: D = 128 without dropout");  // (see above)
  constexpr int KV = KREG ? 0 : 1;  // V's slot in kvs_
  __shared__ __attribute__((aligned(16))) LdsTile<D> kvs_[KREG ? 1 : 2][4];  // [K | V][wave's key tile]
  __shared__ __attribute__((aligned(16))) float ls_[NB][6][32];  // [buf][lse | delta | hash base of key tile 0..3][row]
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = ntiles32(a.T), nbhk = a.B * a.Hkv;
  const int bhk = static_cast<int>(blockIdx.x % nbhk);
  const int grp = static_cast<int>(blockIdx.x / nbhk);
  const int ktile = grp * 4 + w;
  const bool active = ktile < ntiles;
  const int first = grp * 4;  // the block's first query tile = its lowest key tile
  const int b = bhk / a.Hkv, hk = bhk % a.Hkv, group = a.H / a.Hkv;
  const int kb = ktile * 32, key = kb + r;

  // the block's 4 key tiles of K and V go to LDS once (LDS-DMA, issued before
  // the first Q / dO stage, so the first step's wait covers them): the
  // B operands of S = Q K^T and dP = dO V^T are read from there per step
  // instead of living in 16 * D / 32 VGPRs for the whole kernel (round 3 held
  // them in registers: 168 VGPRs at the 3-wave floor, no room left)
  {
    const DmaTile<D> kd(a.k_st), vd(a.v_st);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = __builtin_amdgcn_readfirstlane((first + j) * 32);
      if (row < a.T) {  // block-uniform
        if constexpr (!KREG)
          kd.issue(a.k + b * a.k_sb + hk * a.k_sh + static_cast<int64_t>(row) * a.k_st, kvs_[0][j], a.T - row);
        vd.issue(a.v + b * a.v_sb + hk * a.v_sh + static_cast<int64_t>(row) * a.v_st, kvs_[KV][j], a.T - row);
      }
    }
  }
  // KREG: row r of the wave's K tile, columns 16 ks + 8 hf .. +7 (row_frag's layout);
  // rows past T read row T-1 (their keys are masked out of every product)
  bf16x8 kf[KREG ? D / 16 : 1];
  if constexpr (KREG) {
    const __bf16* kp = a.k + b * a.k_sb + hk * a.k_sh + static_cast<int64_t>(min(key, a.T - 1)) * a.k_st + 8 * hf;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) kf[ks] = ld8(kp + 16 * ks);
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) {
    dk[t] = zero16();
    dv[t] = zero16();
  }
  // dropout: the lane is the key.  The hash of (row q, key pair) covers both
  // keys of the pair, which sit in neighbouring lanes: for a row pair (q0, q1)
  // the even lane hashes q0 and the odd lane q1, the two swap their words with
  // one DPP quad_perm, and v_perm_b32 gathers the lane's 16-bit halves (low
  // half for an even key, high half for an odd one) -- one hash per lane and
  // row pair instead of two.  perm(other, own, sel): even lane [own.lo, other.lo],
  // odd lane [other.hi, own.hi]; the row keys sit in LDS parity-interleaved.
  const uint32_t tm1 = drop_tm1(a.thresh16), sel = (key & 1) ? 0x03020706u : 0x05040100u;
  const int par2 = 2 * (key & 1);
  const uint32_t kmix = (static_cast<uint32_t>(key & 31) >> 1) * kKeyMul;  // pair within the key tile
  const DmaTile<D> qd(a.q_st), dd(a.o_st);
  // query tiles per head: first .. qhi (a sliding window ends the block's range
  // at the last query its highest key reaches)
  const int win = window_of<D>(a);
  const int qhi = win > 0 ? min(ntiles - 1, (first * 32 + 127 + win - 1) >> 5) : ntiles - 1;
  // this wave's last in-window query tile, and the first query tile holding a
  // query at or past (lowest key) + window: only those need the element mask
  const int wq_last = win > 0 ? (kb + 30 + win) >> 5 : ntiles;
  const int wq_cut = win > 0 ? kb + win - 31 : 1 << 30;
  const int nq = qhi - first + 1;
  const int total = group * nq;    // (head, query tile) steps, head-major
  // step i -> buffer i&1: Q and dO tiles by LDS-DMA; wave 0 also DMAs the 32
  // lse (lanes 0..31) and delta (lanes 32..63) values into ls_[buf][0..1];
  // with dropout, wave 1 writes the 32 per-row hash keys into ls_[buf][2]
  // (head in the group, query tile) of the next step to stage: advanced by
  // counters, not i / nq and i % nq (a runtime division is ~40 SALU per step)
  // (The forward and dQ kernels advance running stage pointers; here the
  // per-step (head, row) address products stay: running pointers, row steps
  // and LDS byte addresses pushed the D = 128 variants, already at ~100 of
  // their ~106 SGPRs, into SGPR spills.)
  int sg = 0, sq = first;
  auto stage_next = [&](int buf) {
    const int h = hk * group + sg, bh = b * a.H + h;
    const int qrow = __builtin_amdgcn_readfirstlane(sq * 32);
    qd.issue(a.q + b * a.q_sb + h * a.q_sh + static_cast<int64_t>(qrow) * a.q_st, qs_[buf], a.T - qrow);
    dd.issue(a.dout + b * a.o_sb + h * a.o_sh + static_cast<int64_t>(qrow) * a.o_st, ds_[buf], a.T - qrow);
    if (w == 0) {
      const float* src = (lane < 32 ? a.lse : a.delta) + static_cast<int64_t>(bh) * a.T +
                         min(qrow + (lane & 31), a.T - 1);
      glds4(src, &ls_[buf][0][0]);
    } else if (DROP && w == 1) {
      // the hash bases of the 32 rows for the block's 4 key tiles (lane: row
      // lane & 31, tiles 2 (lane >> 5) + {0, 1}); rows 4i..4i+3 stored as
      // [4i, 4i+2, 4i+1, 4i+3]: an even lane reads the pair heads, an odd lane
      // the pair tails, as one 8-byte read
      const int row = lane & 31, slot = (row & ~3) | ((row & 1) << 1) | ((row >> 1) & 1);
      const uint32_t ar = drop_row(a.seed, bh, qrow + row);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int tt = 2 * (lane >> 5) + u;
        ls_[buf][2 + tt][slot] = __uint_as_float(tile_base(ar, first + tt));
      }
    }
    if (++sq > qhi) {
      sq = first;
      ++sg;
    }
  };
  for (int j = 0; j < NB - 1 && j < total; ++j) stage_next(j);
  // LDS-DMA pieces per stage: Q + dO tiles, and wave 0's lse / delta row values
  const int per_stage = 2 * DmaTile<D>::PPW + (w == 0 ? 1 : 0);
  int qt = first;  // query tile of step i
  for (int i = 0; i < total; ++i, qt = (qt + 1 > qhi ? first : qt + 1)) {
    const int buf = i % NB;
    vm_wait_n(min(total - 1 - i, NB - 2) * per_stage);  // step i landed (later steps may be in flight)
    __syncthreads();  // for every wave; and every wave is done with the buffer restaged next
    if (i + NB - 1 < total) stage_next((i + NB - 1) % NB);
    if (active && qt >= ktile && (D != 128 || qt <= wq_last)) {  // wave-uniform
      const int qb = qt * 32;
      f32x16 s = zero16(), dp = zero16();
      DLION_PRIO_ON(kDkvPrio, 1);
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        if constexpr (KREG)
          s = mfma32(row_frag<D>(qs_[buf], r, ks, hf), kf[ks], s);                            // S = Q K^T
        else
          s = mfma32(row_frag<D>(qs_[buf], r, ks, hf), row_frag<D>(kvs_[0][w], r, ks, hf), s);   // S = Q K^T
        dp = mfma32(row_frag<D>(ds_[buf], r, ks, hf), row_frag<D>(kvs_[KV][w], r, ks, hf), dp);  // dP = dO V^T
      }
      DLION_PRIO_OFF(kDkvPrio, 1);
      if (qt == ktile) {  // causal mask on the diagonal tile only (scalar branch): exp2(-inf) = 0
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          if (key > qb + acc_row(reg, hf)) s[reg] = -INFINITY;
      }
      if (qb + 32 > a.T) {  // tail query tile: rows past T contribute nothing (p = 0, dS = 0)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          if (qb + acc_row(reg, hf) >= a.T) s[reg] = -INFINITY;
      }
      if (D == 128 && qb >= wq_cut) {  // sliding window: queries at or past key + window (window_of<D> reloaded here)
        const int kw = key + window_of<D>(a);
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          if (qb + acc_row(reg, hf) >= kw) s[reg] = -INFINITY;
      }
      // row statistics of the lane's 16 query rows: rows (reg&3) + 8(reg>>2) + 4hf
      // come in 4 runs of 4 consecutive rows -> 16-byte LDS reads (broadcast),
      // consumed run by run (not all 48 values staged up front: that held the
      // kernel at 212 VGPRs, two waves per SIMD).  Runs 2s2, 2s2+1 = operand
      // fragment s2 (two row pairs each); each fragment's MFMAs are issued as
      // soon as it is built, so only one fragment pair is live at a time.
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        i32x4 pw, dw;
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int g = 2 * s2 + gg;
          const float4 lv = *reinterpret_cast<const float4*>(&ls_[buf][0][8 * g + 4 * hf]);
          const float4 dv4 = *reinterpret_cast<const float4*>(&ls_[buf][1][8 * g + 4 * hf]);
          uint2 av = make_uint2(0, 0);
          if constexpr (DROP) av = *reinterpret_cast<const uint2*>(&ls_[buf][2 + w][8 * g + 4 * hf + par2]);
          const float lse_g[4] = {lv.x, lv.y, lv.z, lv.w};
          const float dl_g[4] = {dv4.x, dv4.y, dv4.z, dv4.w};
          // this lane's hash word of row pair pi, and the neighbour's (both
          // hashes before either swap: no DPP read-after-write stall)
          uint32_t own[2], other[2];
          if constexpr (DROP) {
            own[0] = mix1(av.x + kmix);
            own[1] = mix1(av.y + kmix);
#pragma unroll
            for (int pi = 0; pi < 2; ++pi)  // lanes 0<->1, 2<->3
              other[pi] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(own[pi]), 0xB1, 0xF, 0xF, false));
          }
#pragma unroll
          for (int pi = 0; pi < 2; ++pi) {
            const int e0 = 2 * pi, r0 = 4 * g + e0;
            // p and the delta row values already carry 1/(1-p)
            const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r0], a.scale_log2, -lse_g[e0]));
            const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r0 + 1], a.scale_log2, -lse_g[e0 + 1]));
            uint32_t pv, dsv;
            if constexpr (DROP) {
              const uint32_t mk = keep_mask2(__builtin_amdgcn_perm(other[pi], own[pi], sel), tm1);
              pv = pk2(p0, p1) & mk;  // Pd
              const float a0 = p0 * dl_g[e0], a1 = p1 * dl_g[e0 + 1];
              dsv = bfi(mk, pk2(__builtin_fmaf(p0, dp[r0], -a0), __builtin_fmaf(p1, dp[r0 + 1], -a1)),
                        pk2(-a0, -a1));
            } else {
              pv = pk2(p0, p1);
              dsv = pk2(p0 * (dp[r0] - dl_g[e0]), p1 * (dp[r0 + 1] - dl_g[e0 + 1]));
            }
            pw[2 * gg + pi] = static_cast<int>(pv);
            dw[2 * gg + pi] = static_cast<int>(dsv);
          }
        }
        const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
        const bf16x8 dsf = __builtin_bit_cast(bf16x8, dw);
        DLION_PRIO_ON(kDkvPrio, 2);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          dv[t] = mfma32(pf, tr_frag<D>(ds_[buf], s2, t, lane), dv[t]);   // dV += Pd^T dO
          dk[t] = mfma32(dsf, tr_frag<D>(qs_[buf], s2, t, lane), dk[t]);  // dK += dS^T Q
        }
        DLION_PRIO_OFF(kDkvPrio, 2);
        // keep the second fragment's LDS reads from being hoisted above this
        // point (their registers pushed the kernel past 168 VGPRs: spills)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if (!active) return;
  // dk/dv[t]: rows = key (registers), cols = d (lane)
  __bf16* dkb = a.dk + b * a.dk_sb + hk * a.dk_sh;
  if (a.rope_cos != nullptr) unrope<D>(dk, a, kb, hf, r);
  __bf16* dvb = a.dv + b * a.dk_sb + hk * a.dk_sh;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      if (kb + acc_row(reg, hf) >= a.T) continue;
      const int64_t off = static_cast<int64_t>(kb + acc_row(reg, hf)) * a.dk_st + 32 * t + r;
      st_bf16(dkb + off, dk[t][reg] * a.scale);
      st_bf16(dvb + off, dv[t][reg]);
    }
  if (a.colsum != nullptr) {  // bias-gradient partials of the k and v columns (H == Hkv)
    float* cs = a.colsum + static_cast<int64_t>(b * ntiles + ktile) * (3 * a.H * D) + hk * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) {
      float sk = 0.f, sv = 0.f;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        if (kb + acc_row(reg, hf) >= a.T) continue;
        sk += static_cast<float>(static_cast<__bf16>(dk[t][reg] * a.scale));
        sv += static_cast<float>(static_cast<__bf16>(dv[t][reg]));
      }
      sk = xsum32(sk);
      sv = xsum32(sv);
      if (hf == 0) {
        cs[a.H * D + 32 * t + r] = sk;
        cs[2 * a.H * D + 32 * t + r] = sv;
      }
    }
  }
}

// ------------------------------------------------------------------ launchers
// ceil(tiles / 4) blocks of 4 waves per head
static inline int64_t tile_blocks(int64_t nbh, int T) { return nbh * ((((T + 31) >> 5) + 3) >> 2); }

hipError_t launch_attn_fwd(const AttnArgs& a, int D, bool drop, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>(tile_blocks(static_cast<int64_t>(a.B) * a.H, a.T))), block(256);
  // NT = 2 key tiles per barrier at D=64 (GPT-2 shape fwd 0.067 -> 0.065 ms);
  // at D=128 the extra 64 VGPRs cost a wave of occupancy and it was neutral
#define FWD(DD, NT)                                                                        \
  if (drop) hipLaunchKernelGGL((attn_fwd_kernel<DD, true, NT>), grid, block, 0, st, a); \
  else hipLaunchKernelGGL((attn_fwd_kernel<DD, false, NT>), grid, block, 0, st, a);
  if (D == 64) {
    FWD(64, DLION_FWD_NT64)
  } else if (D == 128) {
    FWD(128, 1)
  } else {
    return hipErrorInvalidValue;
  }
#undef FWD
  return hipGetLastError();
}

// the D = 128 K-in-registers dK/dV variant (build macro DLION_DKV_KREG128=0 takes the K-in-LDS kernel)
static constexpr bool dkv_kreg() { return DLION_DKV_KREG128 != 0; }

hipError_t launch_attn_bwd(const AttnArgs& a, int D, bool drop, hipStream_t st) {
  const dim3 bq(static_cast<unsigned>(tile_blocks(static_cast<int64_t>(a.B) * a.H, a.T)));
  const dim3 bkv(static_cast<unsigned>(tile_blocks(static_cast<int64_t>(a.B) * a.Hkv, a.T)));
  // dQ first: it also computes delta = rowsum(dO * O), which dKV reads
#define BWD(DD)                                                                         \
  if (drop) {                                                                           \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, true, 1>), bq, dim3(256), 0, st, a);    \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, true>), bkv, dim3(256), 0, st, a);     \
  } else {                                                                              \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, false, 1>), bq, dim3(256), 0, st, a);   \
    if (DD == 128 && a.H == a.Hkv && dkv_kreg())                                        \
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<128, false, true>), bkv, dim3(256), 0, st, a); \
    else                                                                                \
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, false>), bkv, dim3(256), 0, st, a);  \
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

}  // namespace dlion

// Weight-gradient GEMM for gfx950: C[M, N] (+)= alpha * A^T B with A = dY [K, M] and B = X [K, N]
// both row-major (the reduction dimension K = tokens is the ROW index of both operands), fp32 C.
//
// Why a hand-written kernel: this is the one training GEMM shape class whose operands are both
// k-strided, and with an fp32 accumulate-in-place output (the ZeRO gradient accumulator) the vendor
// library runs it 20-35 % below its forward-layout GEMMs on MI355X (measured: 850-1110 TF vs
// 1260-1610 TF, tools/tune_gemms.py). Here both operands stream row-wise through LDS (global_load_lds,
// lane-linear image with a source-side XOR swizzle) and are read back TRANSPOSED with
// ds_read_b64_tr_b16, so no operand ever needs a transposed copy in HBM, and the fp32
// read-add-write of C happens once per tile in the epilogue.
//
// Geometry: 256 x 256 tile, 8 waves (2 along M x 4 along N), 128 x 64 per wave as 4 x 2
// v_mfma_f32_32x32x16_bf16 accumulators. K streams through an LDS ring of R slabs of 16 k rows
// (A and B, two [16][128] halves each: 16 KiB per slab). Phase s:
//   (a) issues slab s+D (2 LDS-DMA per thread) into the slot of a slab every wave has consumed,
//   (b) s_waitcnt vmcnt(N) + s_barrier: the slab the NEXT phase reads has landed in every wave's
//       DMA (D-1 or D-2 slabs stay in flight across each barrier; never vmcnt(0) in the loop),
//   (c) reads the next phase's fragments (ds_read_b64_tr_b16) into the other register set,
//   (d) runs its 8 MFMAs on the fragments read one phase earlier.
// STAGGER: the two wave groups (A rows 0-127 / 128-255: one wave of each per SIMD) run one barrier
// apart with two barriers per phase, so each SIMD alternates between the groups' MFMA clusters and
// one group's barrier/wait/read latency hides under the other's MFMAs.
// Block order: XCD-aware remap + GROUP_M super-rows so blocks on one XCD share A/B tiles in L2.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace wg {

constexpr int BM = 256, BN = 256, SLAB = 16;
constexpr int NWAVE = 8, NTHR = NWAVE * 64;
constexpr int ROWB = 256;                   // bytes per LDS row (128 bf16)
constexpr int HALF = SLAB * ROWB;           // one [16][128] half slab = 4 KiB
constexpr int SLOT = 4 * HALF;              // A (2 halves) + B (2 halves) = 16 KiB
constexpr int GROUP_M = 8;  // default super-row height (runtime argument of the kernels)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// LDS image of a [k][128] half tile: 16-byte chunk ch of row r sits at chunk position ch ^ swz(r).
// Only transposed reads touch it: one ds_read_b64_tr_b16 covers rows r0+q (q = 0..3) x 64 bytes per
// 32-lane half, and the XOR by (q << 2) puts those four rows on four different 64-byte bank
// groups (conflict-free); the DMA writes whole 256-byte rows and cannot conflict.
__device__ __forceinline__ int swz(int row) { return (row & 3) << 2; }

__device__ __forceinline__ i16x4 lds_tr(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(const_cast<char*>(base) + byte_off));
}

// MFMA operand (A or B of 32x32x16) from a row-major [k][128] LDS half tile, transposed: lane gets
// column 32*dt + (lane&31); element j of lane half h <- k row row0 + 8*(j>>2) + 4h + (j&3).
// A and B use the same k permutation, so it cancels in the product.
// frag_off(dt, lane): the lane's byte offset for row0 = 0; row0 (a multiple of 4) only adds
// row0 * ROWB, because the swizzle depends on row & 3 alone -- so a phase's reads are one base
// VGPR per column block + compile-time immediates.
__device__ __forceinline__ int frag_off(int dt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const int row = 4 * h + q;
  return row * ROWB + 16 * (ch ^ swz(row)) + 8 * (p & 1);
}

__device__ __forceinline__ bf16x8 frag_at(const char* lane_base, int row0) {
  i16x4 lo = lds_tr(lane_base, row0 * ROWB);
  i16x4 hi = lds_tr(lane_base, (row0 + 8) * ROWB);
  const i16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

// LDS-DMA issued from inline asm: hipcc's waitcnt pass cannot see it, so it does not put a
// conservative `s_waitcnt vmcnt(0)` in front of every ds_read of the ring (it did with the
// builtin: the whole prefetch drained each K-step). Completion is tracked by the explicit counted
// vmcnt + barrier in the main loop. `lds` is the wave-uniform LDS byte address (M0).
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(gsrc) : "memory", "m0");
}

// Per-thread DMA source/destination of one slab. Wave w moves 4 k rows x 256 bytes of A-half
// (w>>2)&1 (first instruction) and of B-half (w>>2)&1 (second): rows 4*(w&3) + (lane>>4) of the
// slab, 16-byte chunk (lane&15) ^ swz(row). Slab j is the same pattern shifted by 16j rows (a
// scalar offset) into its ring slot.
struct DmaPlan {
  const unsigned short* a;  // A source at k row = row-in-slab
  const unsigned short* b;
  unsigned lds_a, lds_b;    // LDS byte address of this wave's 1 KiB pieces in slot 0
};

__device__ __forceinline__ DmaPlan dma_plan(const unsigned short* A, int64_t lda, const unsigned short* B,
                                            int64_t ldb, int m0, int n0, unsigned lds_base) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int half = (w >> 2) & 1, rq = w & 3;
  const int row = 4 * rq + (lane >> 4);
  const int ch = (lane & 15) ^ swz(row);
  DmaPlan d;
  d.a = A + (int64_t)row * lda + m0 + half * 128 + ch * 8;
  d.b = B + (int64_t)row * ldb + n0 + half * 128 + ch * 8;
  d.lds_a = __builtin_amdgcn_readfirstlane(lds_base + half * HALF + 4 * rq * ROWB);
  d.lds_b = __builtin_amdgcn_readfirstlane(lds_base + (2 + half) * HALF + 4 * rq * ROWB);
  return d;
}

__device__ __forceinline__ void load_slab(const DmaPlan& d, int64_t lda, int64_t ldb, int slab, int slot) {
  const int r = SLAB * slab;
  glds16(d.a + (int64_t)r * lda, d.lds_a + slot * SLOT);
  glds16(d.b + (int64_t)r * ldb, d.lds_b + slot * SLOT);
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Two K segments (A, B) rows [0, 16 ns1) then (A2, B2) rows [0, K - 16 ns1), same leading dims: the
// product over the concatenated token axis without materialising the concatenation (the deferred
// expert weight gradients of moe/experts.py: the stashed micro-step, then the boundary one).
// ns1 = K / 16 (and A2 = A, B2 = B) for one segment.
template <bool ACCUM, int R, bool STAGGER, bool NODMA = false, bool SEG2 = false>
__global__ void __launch_bounds__(NTHR, 1) wgrad_kernel(const unsigned short* __restrict__ A, int64_t lda,
                                                        const unsigned short* __restrict__ B, int64_t ldb,
                                                        float* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        float alpha, int group_m, const unsigned short* A2,
                                                        const unsigned short* B2, int ns1) {
  static_assert(R == 8, "fragment bases assume slots 0-3 / 4-7");
  constexpr int D = STAGGER ? R - 3 : R - 2;              // prefetch distance in slabs
  constexpr int WAIT = STAGGER ? 2 * (D - 2) : 2 * (D - 1);  // DMA left in flight at each wait
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  // ---- block -> tile (XCD-aware, grouped along M) ------------------------------------------
  const int tm = M / BM, tn = N / BN, nwg = tm * tn;
  const int orig = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int per_group = group_m * tn;
  const int grp = wgid / per_group;
  const int first_m = grp * group_m;
  const int gsz = min(tm - first_m, group_m);
  const int bm = first_m + (wgid % per_group) % gsz;
  const int bn = (wgid % per_group) / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int ns = K / SLAB;  // a multiple of R (host check)
  bf16x8 fa[2][4], fb[2][2];
  // per-lane fragment bases: A columns wr*128 .. +128 (4 blocks of 32), B columns
  // (wc>>1)*128 + (wc&1)*64 .. +64 (2 blocks); slots 0-3 from base 0, slots 4-7 from base 1 (the
  // ds_read immediate offset field is 16 bits)
  const char* fbase[2][6];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fbase[h][i] = smem + 4 * h * SLOT + wr * HALF + frag_off(i, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fbase[h][4 + j] = smem + 4 * h * SLOT + (2 + (wc >> 1)) * HALF + frag_off((wc & 1) * 2 + j, lane);
  }
  auto read_frags = [&](int slot, bf16x8 (&a)[4], bf16x8 (&b)[2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag_at(fbase[slot >> 2][i] + (slot & 3) * SLOT, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = frag_at(fbase[slot >> 2][4 + j] + (slot & 3) * SLOT, 0);
  };
  auto mma = [&](const bf16x8 (&a)[4], const bf16x8 (&b)[2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  const unsigned lds_base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const DmaPlan dp = dma_plan(A, lda, B, ldb, m0, n0, lds_base);
  // one-segment instantiations keep the original single DMA plan (SEG2 = false: no second plan's
  // registers, no per-slab segment test)
  const DmaPlan dp2 = SEG2 ? dma_plan(A2, lda, B2, ldb, m0, n0, lds_base) : dp;
  auto load_any = [&](int slab, int slot) {  // slab in the first or the second K segment (wave-uniform)
    if (!SEG2 || slab < ns1)
      load_slab(dp, lda, ldb, slab, slot);
    else
      load_slab(dp2, lda, ldb, slab - ns1, slot);
  };
  // prologue: slabs 0 .. D-1, then the first phase's fragments
#pragma unroll
  for (int j = 0; j < D; ++j) load_any(j, j);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT) : "memory");
  __builtin_amdgcn_s_barrier();
  read_frags(0, fa[0], fb[0]);
  if (STAGGER && __builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();
  for (int s0 = 0; s0 < ns; s0 += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {  // phase s = s0 + j, slab s in slot j
      // the surplus DMA of the last D phases (clamped to the last slab) lands in consumed slots
      if (!NODMA) load_any(min(s0 + j + D, ns - 1), (j + D) % R);
      if (NODMA)  // ablation (variant 3): the ring is never refilled -- MFMA + LDS + barrier ceiling
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT) : "memory");
      __builtin_amdgcn_s_barrier();
      read_frags((j + 1) % R, fa[(j + 1) & 1], fb[(j + 1) & 1]);
      mma(fa[j & 1], fb[j & 1]);
      if (STAGGER) __builtin_amdgcn_s_barrier();
    }
  }
  if (STAGGER && __builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();
  // ---- epilogue: C (+)= alpha * acc, two accumulator tiles (32 values / lane) per batch so the
  // C reads are in flight together instead of one dependent round trip per value
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* rowp[2];
    float old[2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      rowp[j] = C + (int64_t)(m0 + wr * 128 + i * 32) * ldc + n0 + wc * 64 + j * 32 + col;
      if (ACCUM) {
#pragma unroll
        for (int e = 0; e < 16; ++e) old[j][e] = __builtin_nontemporal_load(rowp[j] + (int64_t)acc_row(e, h) * ldc);
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float v = alpha * acc[i][j][e];
        rowp[j][(int64_t)acc_row(e, h) * ldc] = ACCUM ? old[j][e] + v : v;
      }
  }
}


// ---------------------------------------------------------------------------------------------
// Variant 2: 4 waves (one per SIMD), 2 x 2 waves of 128 x 128 (4 x 4 accumulators = 256 fp32 per
// lane, in AGPRs), slabs of 32 k rows (32 KiB: A and B, two [32][128] halves each) in a ring of 4.
// Per phase a wave runs 32 MFMAs between barriers (twice the MFMA work per barrier of the 8-wave
// form) and reads 1 ds_read_b64_tr_b16 per MFMA. Every wave drains its LDS reads (lgkmcnt(0),
// already complete: they fed this phase) before the barrier, so the slot of the slab consumed in
// the previous phase can be refilled right after it: prefetch distance 3 slabs.
namespace w4 {
constexpr int SLAB = 32, R = 4, D = 3;
constexpr int NTHR = 256;
constexpr int HALF = SLAB * ROWB;           // [32][128] bf16 = 8 KiB
constexpr int SLOT = 4 * HALF;              // 32 KiB
constexpr int WAIT = 8 * (D - 1);           // DMA per slab per thread = 8

struct Plan {
  const unsigned short* a;  // A at (k row lane>>4, this lane's swizzled chunk)
  const unsigned short* b;
  unsigned lds;             // LDS byte address of slot 0
};

template <bool ACCUM>
__global__ void __launch_bounds__(NTHR, 1) kernel(const unsigned short* __restrict__ A, int64_t lda,
                                                  const unsigned short* __restrict__ B, int64_t ldb,
                                                  float* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                  float alpha, int group_m, const unsigned short* A2,
                                                  const unsigned short* B2, int ns1) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int tm = M / BM, tn = N / BN, nwg = tm * tn;
  const int orig = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int per_group = group_m * tn;
  const int grp = wgid / per_group;
  const int first_m = grp * group_m;
  const int gsz = min(tm - first_m, group_m);
  const int bm = first_m + (wgid % per_group) % gsz;
  const int bn = (wgid % per_group) / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // DMA: slab rows 4*rq + (lane>>4), rq = 0..7; the 32 wave-instructions of a slab are
  // (op, half, rq) = (it>>2, (it>>1)&1, (it&1)*4 + w) for it = 0..7
  Plan pl, pl2;
  {
    const int row = lane >> 4;  // row & 3 == (lane >> 4) & 3 for every rq
    const int ch = (lane & 15) ^ swz(row);
    pl.a = A + (int64_t)row * lda + m0 + ch * 8;
    pl.b = B + (int64_t)row * ldb + n0 + ch * 8;
    pl.lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    pl2 = pl;
    pl2.a = A2 + (int64_t)row * lda + m0 + ch * 8;
    pl2.b = B2 + (int64_t)row * ldb + n0 + ch * 8;
  }
  const int ns1_32 = ns1 / 2;  // 16-row slabs of the first segment -> 32-row slabs (host: ns1 even)
  auto load_slab = [&](int slab_any, int slot) {
    const bool second = slab_any >= ns1_32;
    const Plan& P = second ? pl2 : pl;
    const int slab = second ? slab_any - ns1_32 : slab_any;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int op = it >> 2, half = (it >> 1) & 1, rq = (it & 1) * 4 + w;
      const int64_t rows = (int64_t)SLAB * slab + 4 * rq;
      const unsigned short* src = op == 0 ? P.a + rows * lda + half * 128 : P.b + rows * ldb + half * 128;
      const unsigned dst = __builtin_amdgcn_readfirstlane(pl.lds + slot * SLOT + (op * 2 + half) * HALF + 4 * rq * ROWB);
      glds16(src, dst);
    }
  };
  // fragment bases: A half wr (columns wr*128 + 32i), B half wc (columns wc*128 + 32j); slots
  // 0-1 from base 0, slots 2-3 from base 1 (16-bit ds_read immediate offsets)
  const char* fa_base[2][4];
  const char* fb_base[2][4];
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa_base[hb][i] = smem + 2 * hb * SLOT + wr * HALF + frag_off(i, lane);
      fb_base[hb][i] = smem + 2 * hb * SLOT + (2 + wc) * HALF + frag_off(i, lane);
    }
  bf16x8 fa[2][2][4], fb[2][2][4];  // [register set][k16 step][block]
  auto read_frags = [&](int slot, bf16x8 (&a)[2][4], bf16x8 (&b)[2][4]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[kk][i] = frag_at(fa_base[slot >> 1][i] + (slot & 1) * SLOT, 16 * kk);
        b[kk][i] = frag_at(fb_base[slot >> 1][i] + (slot & 1) * SLOT, 16 * kk);
      }
  };
  auto mma = [&](const bf16x8 (&a)[2][4], const bf16x8 (&b)[2][4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  const int ns = K / SLAB;  // a multiple of R (host check)
#pragma unroll
  for (int j = 0; j < D; ++j) load_slab(j, j);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT) : "memory");
  __builtin_amdgcn_s_barrier();
  read_frags(0, fa[0], fb[0]);
  for (int s0 = 0; s0 < ns; s0 += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {  // phase s = s0 + j: slab s in slot j
      load_slab(min(s0 + j + D, ns - 1), (j + D) % R);  // surplus DMA at the end lands in consumed slots
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(WAIT) : "memory");
      __builtin_amdgcn_s_barrier();
      read_frags((j + 1) % R, fa[(j + 1) & 1], fb[(j + 1) & 1]);
      mma(fa[j & 1], fb[j & 1]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* rowp[4];
    float old[4][16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      rowp[j] = C + (int64_t)(m0 + wr * 128 + i * 32) * ldc + n0 + wc * 128 + j * 32 + col;
      if (ACCUM) {
#pragma unroll
        for (int e = 0; e < 16; ++e) old[j][e] = __builtin_nontemporal_load(rowp[j] + (int64_t)acc_row(e, h) * ldc);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float v = alpha * acc[i][j][e];
        rowp[j][(int64_t)acc_row(e, h) * ldc] = ACCUM ? old[j][e] + v : v;
      }
  }
}
}  // namespace w4

}  // namespace wg

bool wgrad_supported(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c) {
  return a.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
         c.scalar_type() == at::kFloat && a.dim() == 2 && b.dim() == 2 && c.dim() == 2 && a.stride(1) == 1 &&
         b.stride(1) == 1 && c.stride(1) == 1 && a.size(0) == b.size(0) && c.size(0) == a.size(1) &&
         c.size(1) == b.size(1) && a.size(1) % wg::BM == 0 && b.size(1) % wg::BN == 0 && a.size(0) % (8 * wg::SLAB) == 0 &&
         (reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0) && (reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0) &&
         a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0;
}

// c (+)= alpha * a^T @ b ; a: [K, M] bf16, b: [K, N] bf16, c: [M, N] fp32.
// variant: 0 = 8 lock-step waves, 1 = 8 staggered waves, 2 = 4 waves of 128 x 128, for in-process A/B.
static void wgrad_launch(const at::Tensor& a, const at::Tensor& b, const at::Tensor& a2, const at::Tensor& b2, int K,
                         int ns1, at::Tensor c, double alpha, bool accumulate, int64_t variant, bool seg2 = false) {
  c10::DeviceGuard g(a.device());
  const int M = a.size(1), N = b.size(1);
  const int nwg = (M / wg::BM) * (N / wg::BN);
  const size_t lds = 8 * wg::SLOT;
  using Kern = void (*)(const unsigned short*, int64_t, const unsigned short*, int64_t, float*, int64_t, int, int,
                        int, float, int, const unsigned short*, const unsigned short*, int);
  const int group_m = variant >= 16 ? (int)(variant >> 4) : wg::GROUP_M;  // A/B knob: variant + 16 * group_m
  variant &= 15;
  static const Kern kerns[5][2] = {{wg::wgrad_kernel<false, 8, false>, wg::wgrad_kernel<true, 8, false>},
                                   {wg::wgrad_kernel<false, 8, true>, wg::wgrad_kernel<true, 8, true>},
                                   {wg::w4::kernel<false>, wg::w4::kernel<true>},
                                   {wg::wgrad_kernel<false, 8, false, true>, wg::wgrad_kernel<true, 8, false, true>},
                                   {wg::wgrad_kernel<false, 8, false, false, true>,
                                    wg::wgrad_kernel<true, 8, false, false, true>}};
  static bool attr_set = [&] {
    for (auto& row : kerns)
      for (Kern k : row)
        SXE_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return true;
  }();
  (void)attr_set;
  SXE_CHECK(variant >= 0 && variant <= 3, "wgrad_gemm_: variant must be 0..3");
  SXE_CHECK(!seg2 || variant == 0, "wgrad_gemm2_: the 8-wave lock-step schedule only");
  const int nthr = variant == 2 ? wg::w4::NTHR : wg::NTHR;
  hipLaunchKernelGGL(kerns[seg2 ? 4 : variant][accumulate ? 1 : 0], dim3(nwg), dim3(nthr), lds, cur_stream(),
                     reinterpret_cast<const unsigned short*>(a.data_ptr()), a.stride(0),
                     reinterpret_cast<const unsigned short*>(b.data_ptr()), b.stride(0), c.data_ptr<float>(),
                     c.stride(0), M, N, K, (float)alpha, group_m, reinterpret_cast<const unsigned short*>(a2.data_ptr()),
                     reinterpret_cast<const unsigned short*>(b2.data_ptr()), ns1);
  SXE_LAUNCH_CHECK();
}

void wgrad_gemm_variant_(const at::Tensor& a, const at::Tensor& b, at::Tensor c, double alpha, bool accumulate,
                         int64_t variant) {
  SXE_CHECK(wgrad_supported(a, b, c), "wgrad_gemm_: unsupported shapes/dtypes/strides");
  const int K = a.size(0);
  wgrad_launch(a, b, a, b, K, K / wg::SLAB, c, alpha, accumulate, variant);
}

static int64_t default_variant(const at::Tensor& a, const at::Tensor& b) {
  // 8 lock-step waves; super-rows of 4 M-tiles for tall outputs, 8 otherwise (tools/wgrad_exp.py)
  const int64_t tm = a.size(1) / wg::BM, tn = b.size(1) / wg::BN;
  return 0 + 16 * (tm >= 4 * tn ? 4 : 8);
}

void wgrad_gemm_(const at::Tensor& a, const at::Tensor& b, at::Tensor c, double alpha, bool accumulate) {
  wgrad_gemm_variant_(a, b, c, alpha, accumulate, default_variant(a, b));
}

// c (+)= alpha * [a; a2]^T @ [b; b2] (concatenated along K = rows) without the concatenation:
// a, a2 [K1 | K2, M], b, b2 [K1 | K2, N], equal leading dims, K1 % 32 == 0, (K1 + K2) % 128 == 0
bool wgrad2_supported(const at::Tensor& a, const at::Tensor& b, const at::Tensor& a2, const at::Tensor& b2,
                      const at::Tensor& c) {
  if (a2.dim() != 2 || b2.dim() != 2 || a2.scalar_type() != a.scalar_type() || b2.scalar_type() != b.scalar_type() ||
      a2.size(1) != a.size(1) || b2.size(1) != b.size(1) || a2.size(0) != b2.size(0) || a2.stride(1) != 1 ||
      b2.stride(1) != 1 || a2.stride(0) != a.stride(0) || b2.stride(0) != b.stride(0) || a.size(0) % 32 != 0 ||
      (reinterpret_cast<uintptr_t>(a2.data_ptr()) % 16) != 0 || (reinterpret_cast<uintptr_t>(b2.data_ptr()) % 16) != 0)
    return false;
  const int64_t K = a.size(0) + a2.size(0);
  if (K % (8 * wg::SLAB) != 0) return false;
  // the one-segment shape checks, with K = K1 + K2
  return a.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
         c.scalar_type() == at::kFloat && a.dim() == 2 && b.dim() == 2 && c.dim() == 2 && a.stride(1) == 1 &&
         b.stride(1) == 1 && c.stride(1) == 1 && a.size(0) == b.size(0) && c.size(0) == a.size(1) &&
         c.size(1) == b.size(1) && a.size(1) % wg::BM == 0 && b.size(1) % wg::BN == 0 &&
         (reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0) && (reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0) &&
         a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0;
}

void wgrad_gemm2_(const at::Tensor& a, const at::Tensor& b, const at::Tensor& a2, const at::Tensor& b2, at::Tensor c,
                  double alpha, bool accumulate) {
  SXE_CHECK(wgrad2_supported(a, b, a2, b2, c), "wgrad_gemm2_: unsupported shapes/dtypes/strides");
  const int K = (int)(a.size(0) + a2.size(0));
  wgrad_launch(a, b, a2, b2, K, (int)(a.size(0) / wg::SLAB), c, alpha, accumulate, default_variant(a, b), true);
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("wgrad_gemm_(Tensor a, Tensor b, Tensor(a!) c, float alpha, bool accumulate) -> ()");
  m.def("wgrad_gemm_variant_(Tensor a, Tensor b, Tensor(a!) c, float alpha, bool accumulate, int variant) -> ()");
  m.def("wgrad_gemm2_(Tensor a, Tensor b, Tensor a2, Tensor b2, Tensor(a!) c, float alpha, bool accumulate) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("wgrad_gemm_", &sxe::wgrad_gemm_);
  m.impl("wgrad_gemm_variant_", &sxe::wgrad_gemm_variant_);
  m.impl("wgrad_gemm2_", &sxe::wgrad_gemm2_);
}

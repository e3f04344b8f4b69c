// OCP-MX block-scaled GEMM on gfx950's scaled matrix cores (v_mfma_scale_f32_32x32x64_f8f6f4):
//   Y[M, N] = dequant(Xq, Xs) @ dequant(Wq, Ws)^T  (+ bias[N]) (* col_scale[N])
// with X quantized per 32-element K block to MXFP8 (e4m3 + one E8M0 exponent) by mx_quant_fp8 and
// W stored as MXFP8 (e4m3), MXFP6 (e3m2 or e2m3) or MXFP4 (e2m1) codes with one E8M0 exponent per
// 32 K elements. The dequantisation is done by the MFMA itself: each lane hands the instruction its
// 32 K-contiguous codes plus the block's exponent byte, so the weight never exists in bf16 -- in HBM,
// LDS or registers (the FP6-LLM counterpart, reference inference/v2/kernels/core_ops/cuda_linear/
// linear_kernels_cuda.cu:70,216, decodes FP6 to fp16 in registers and runs fp16 tensor cores).
//
// Operand maps (measured by tools/probes/mx_mfma_layout.hip + mx_layout_check.py on MI355X,
// profiles/mx_mfma_layout.log): in a 32x32x64 MFMA lane l feeds row / column (l & 31), half
// h = l >> 5, 32 codes (element j at bits [w j, w j + w) of the 8-dword operand, w = 8 / 6 / 4):
//   * 6- and 4-bit operands: K = 32 h + j -- the lane's codes are exactly K block h;
//   * 8-bit operands: K = 16 h + j for j < 16 and K = 32 + 16 h + (j - 16) for j >= 16 -- the
//     two 16-byte halves of the operand cover the two K blocks;
//   * the lane's E8M0 byte scales K block h of its row / column, wherever those codes sit (so an
//     fp8 lane's codes use its own exponent and its partner half's).
// Both operands are K-contiguous rows -- X as [M, K], W in nn.Linear's [N, K] layout -- so the
// layouts only decide which bytes of an LDS row a lane reads; no data is ever permuted.
//
// Geometry: BM x BN output tile (256x256 / 256x128 / 128x128), WM x WN waves, each wave
// (BM/WM) x (BN/WN) as 32x32 accumulators; K in stages of 128 (two MFMA k-steps). Operand tiles are
// staged global -> registers -> LDS with rows padded by 16 B (row strides of 144 / 112 / 80 B put
// the 16 lanes of a ds_read_b128 phase on distinct banks); the next stage's loads (tiles + the
// lanes' scale words) are in flight while the current stage's MFMAs run. Workgroups are mapped
// XCD-major: the 8 XCDs each take a contiguous range of output tiles (M fastest), so the weight
// column tiles a workgroup streams are shared through its XCD's L2.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace mx {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 128;
constexpr int SA = 128 + 16;  // padded LDS row stride of the fp8 activation tile

// MFMA format codes (cbsz / blgp): 0 e4m3, 1 e5m2, 2 e2m3, 3 e3m2, 4 e2m1
__host__ __device__ constexpr int fmt_bits(int f) { return f <= 1 ? 8 : (f <= 3 || f == 16) ? 6 : 4; }
// 16 / 17: FPxWeight's bit-plane FP6 (e3m2) / FP4 (e2m1) layout (ops/fp_quantizer.py): transcoded
// exactly to e4m3 in registers and multiplied as fp8 (both formats embed in e4m3)
__host__ __device__ constexpr bool is_planes(int f) { return f >= 16; }
__host__ __device__ constexpr int mfma_fmt(int f) { return is_planes(f) ? 0 : f; }

template <int FB>
struct BLayout {
  static constexpr int BITS = fmt_bits(FB);
  static constexpr int RB = 16 * BITS;  // bytes per row per 128-element K stage
  static constexpr int SB = RB + 16;    // padded LDS stride
  static constexpr int CPR = RB / 16;   // 16-byte chunks per row
  static constexpr int LB = 4 * BITS;   // bytes one lane feeds per MFMA (32 elements)
};

template <int ROWS, int CPR, int STRIDE, int NTHR>
struct Stager {
  static constexpr int N = (ROWS * CPR + NTHR - 1) / NTHR;
  u32x4 r[N];
  __device__ __forceinline__ void load(const uint8_t* base, int64_t row_bytes, int row0, int valid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHR;
      const int row = c / CPR, ch = c % CPR;
      r[i] = (c < ROWS * CPR && row0 + row < valid)
                 ? *reinterpret_cast<const u32x4*>(base + (int64_t)(row0 + row) * row_bytes + ch * 16)
                 : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(char* lds) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHR;
      if (c < ROWS * CPR) *reinterpret_cast<u32x4*>(lds + (c / CPR) * STRIDE + (c % CPR) * 16) = r[i];
    }
  }
};

// The 32 codes a lane feeds to one 64-K MFMA step, from the step's bytes of an LDS row (`p` points
// at the step's first byte): fp8 = bytes [16 h, 16 h + 16) and [32 + 16 h, 32 + 16 h + 16); fp6 /
// fp4 = the LB contiguous bytes of block h.
template <int LB>
__device__ __forceinline__ i32x8 lds_operand(const char* p, int h) {
  i32x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (LB == 32) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(p + 16 * h), b = *reinterpret_cast<const u32x4*>(p + 32 + 16 * h);
    v = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
    return v;
  }
  p += LB * h;
  if constexpr (LB == 24) {
    const u32x2 a = *reinterpret_cast<const u32x2*>(p), b = *reinterpret_cast<const u32x2*>(p + 8),
                c = *reinterpret_cast<const u32x2*>(p + 16);
    v = i32x8{(int)a[0], (int)a[1], (int)b[0], (int)b[1], (int)c[0], (int)c[1], 0, 0};
  } else {
    const u32x4 a = *reinterpret_cast<const u32x4*>(p);
    v = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], 0, 0, 0, 0};
  }
  return v;
}

// Epilogue of transposed accumulators acc[i][j] (the weight was the MFMA's A operand, so each 32x32
// tile is Y^T): lane (l32, h) owns token row m0w + 32 i + l32 and, per j, the 4 runs of 4 consecutive
// columns n0w + 32 j + 8 g + 4 h + 0..3 -- one 8-byte store per run, column scale / bias loaded once
// per run before the stores, no per-element branch (a per-element `if` around a store makes hipcc
// wait for the previous store before each element).
template <int MI, int NJ>
__device__ __forceinline__ void store_t(const f32x16 (&acc)[MI][NJ], unsigned short* __restrict__ Y,
                                        const float* __restrict__ col_scale, const unsigned short* __restrict__ bias,
                                        int m0w, int n0w, int M, int N, int h, int l32) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {  // per column block: its scales / biases, then every row's stores
    float4 cs[4];
    float bv[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = n0w + j * 32 + 8 * g + 4 * h;
      cs[g] = col_scale ? *reinterpret_cast<const float4*>(col_scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
      if (bias) {
        const u32x2 bb = *reinterpret_cast<const u32x2*>(bias + n);
        bv[g][0] = __uint_as_float(bb[0] << 16);
        bv[g][1] = __uint_as_float(bb[0] & 0xffff0000u);
        bv[g][2] = __uint_as_float(bb[1] << 16);
        bv[g][3] = __uint_as_float(bb[1] & 0xffff0000u);
      } else {
        bv[g][0] = bv[g][1] = bv[g][2] = bv[g][3] = 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0w + i * 32 + l32;
      if (m >= M) continue;
      unsigned short* yr = Y + (int64_t)m * N + n0w + j * 32 + 4 * h;
      const f32x16& c = acc[i][j];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float v0 = c[4 * g + 0] * cs[g].x + bv[g][0], v1 = c[4 * g + 1] * cs[g].y + bv[g][1];
        const float v2 = c[4 * g + 2] * cs[g].z + bv[g][2], v3 = c[4 * g + 3] * cs[g].w + bv[g][3];
        const unsigned lo = (unsigned)f32_to_bf16(v0) | ((unsigned)f32_to_bf16(v1) << 16);
        const unsigned hi = (unsigned)f32_to_bf16(v2) | ((unsigned)f32_to_bf16(v3) << 16);
        *reinterpret_cast<u32x2*>(yr + 8 * g) = u32x2{lo, hi};
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int FB>
__global__ void __launch_bounds__(64 * WM * WN, 1)
    mx_gemm_kernel(const uint8_t* __restrict__ Xq, const uint8_t* __restrict__ Xs, const uint8_t* __restrict__ Wq,
                   const uint8_t* __restrict__ Ws, const unsigned short* __restrict__ bias,
                   const float* __restrict__ col_scale, unsigned short* __restrict__ Y, int M, int N, int K) {
  using L = BLayout<FB>;
  constexpr int NTHR = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, MI = TM / 32, NJ = TN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* lA = smem;
  char* lB = smem + BM * SA;

  // ---- XCD-major tile order: XCD x (= blockIdx % 8) owns tiles [x G/8, (x+1) G/8), M fastest -----
  const int tm = (M + BM - 1) / BM, tn = N / BN, G = tm * tn;
  int pid = blockIdx.x;
  if ((G & 7) == 0) pid = (pid & 7) * (G >> 3) + (pid >> 3);
  const int m0 = (pid % tm) * BM, n0 = (pid / tm) * BN;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w / WN, wn = w % WN, h = lane >> 5, l32 = lane & 31;
  const int KS = K / 32;          // scale bytes per row
  const int64_t WRB = (int64_t)K * L::BITS / 8;  // weight bytes per row

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // scale words (4 E8M0 bytes = one 128-K stage) of the rows / columns this lane feeds
  unsigned sa[MI], sb[NJ];
  auto load_scales = [&](int kb) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * TM + i * 32 + l32;
      sa[i] = m < M ? *reinterpret_cast<const unsigned*>(Xs + (int64_t)m * KS + 4 * kb) : 0x7f7f7f7fu;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * TN + j * 32 + l32;
      sb[j] = *reinterpret_cast<const unsigned*>(Ws + (int64_t)n * KS + 4 * kb);
    }
  };

  Stager<BM, 8, SA, NTHR> stA;
  Stager<BN, L::CPR, L::SB, NTHR> stB;
  stA.load(Xq, K, m0, M);
  stB.load(Wq, WRB, n0, N);
  load_scales(0);
  const int nk = K / BK;
  for (int kb = 0; kb < nk; ++kb) {
    if (kb) __syncthreads();
    stA.store(lA);
    stB.store(lB);
    unsigned csa[MI], csb[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) csa[i] = sa[i];
#pragma unroll
    for (int j = 0; j < NJ; ++j) csb[j] = sb[j];
    __syncthreads();
    if (kb + 1 < nk) {  // the next stage's loads overlap this stage's MFMAs
      stA.load(Xq + (int64_t)(kb + 1) * BK, K, m0, M);
      stB.load(Wq + (int64_t)(kb + 1) * L::RB, WRB, n0, N);
      load_scales(kb + 1);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      i32x8 a[MI], b[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = lds_operand<32>(lA + (wm * TM + i * 32 + l32) * SA + 64 * s, h);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        b[j] = lds_operand<L::LB>(lB + (wn * TN + j * 32 + l32) * L::SB + 2 * L::LB * s, h);
      const int sh = 8 * (2 * s + h);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(  // Y^T tile: see store_t
              b[j], a[i], acc[i][j], FB, 0, 0, (int)((csb[j] >> sh) & 0xff), 0, (int)((csa[i] >> sh) & 0xff));
      __builtin_amdgcn_s_setprio(0);
    }
  }
  store_t<MI, NJ>(acc, Y, col_scale, bias, m0 + wm * TM, n0 + wn * TN, M, N, h, l32);
}

// X [M, K] bf16 -> e4m3 codes [M, K] + E8M0 exponents [M, K/32]; one thread per 32-element block.
// The block exponent is ceil(log2(amax / 448)), so every scaled element is within e4m3's range and
// the hardware converter (round to nearest even) never saturates.
__global__ void mx_quant_fp8_kernel(const unsigned short* __restrict__ x, uint8_t* __restrict__ q,
                                    uint8_t* __restrict__ s, int64_t nblocks) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const u16x8* p = reinterpret_cast<const u16x8*>(x + b * 32);
  u16x8 v[4];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = p[c];
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(bf16_to_f32(v[c][e])));
  }
  int ex = -127;
  if (amax > 0.f) {
    int fe;
    const float f = frexpf(amax * (1.f / 448.f), &fe);
    ex = (f == 0.5f) ? fe - 1 : fe;
    if (ldexpf(amax, -ex) > 448.f) ++ex;
    ex = max(-127, min(127, ex));
  }
  s[b] = (uint8_t)(ex + 127);
  const float inv = ldexpf(1.f, -ex);
  unsigned out[8];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int e = 0; e < 8; e += 4) {
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[c][e]) * inv, bf16_to_f32(v[c][e + 1]) * inv, 0, false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[c][e + 2]) * inv, bf16_to_f32(v[c][e + 3]) * inv, pk, true);
      out[2 * c + e / 4] = (unsigned)pk;
    }
  u32x4* o = reinterpret_cast<u32x4*>(q + b * 32);
  o[0] = u32x4{out[0], out[1], out[2], out[3]};
  o[1] = u32x4{out[4], out[5], out[6], out[7]};
}


// ---------------------------------------------------------------------------------------------------
// Deep-pipelined variant: 256 x 256 output tile, 4 waves (2 x 2, 128 x 128 each: 16 accumulators in
// AGPRs), every operand byte -- codes AND the lanes' exponent words -- staged by LDS-DMA
// (global_load_lds, 16 B per lane for codes, 4 B for exponents) into NBUF stage buffers, waited with
// a counted vmcnt and a raw s_barrier so the next stage's DMA stays in flight across the barrier
// (cdna_hip_programming.md "Pipelining across barriers"). A glds writes lane i's bytes at the
// wave-uniform base + i * size, so the LDS image is lane-linear; the bank-conflict swizzle is applied
// to the SOURCE address instead: 16-byte slot s of row r holds chunk s ^ f(r), with f(r) = (r >> 1) & 7
// for 128-byte rows (fp8 / padded fp6) and (r >> 2) & 3 for 64-byte rows (fp4), which puts the 16
// rows a ds_read_b128 phase touches on distinct banks. fp6 rows (96 data bytes) are padded to 128 B.
namespace dp {
constexpr int BM = 256, NT = 256;
template <int FB, int BN, int NWV = 4> struct L {
  static constexpr bool PL = is_planes(FB);
  static constexpr int BITS = fmt_bits(FB);
  static constexpr int RB = 16 * BITS;                // data bytes per row per 128-K stage
  static constexpr int RP = (BITS == 4 || PL) ? 64 : 128;  // LDS row pitch (planes: the nibble plane)
  static constexpr int CH = PL ? 4 : RB / 16;         // data chunks per row
  static constexpr int SL = RP / 16;                  // slots per row
  static constexpr int ROWS_PER_INSTR = 64 / SL;      // rows one wave instruction fills
  static constexpr int A_INSTR = BM / 8 / NWV;        // A: 8 rows x 128 B per instruction
  static constexpr int NI = BN / ROWS_PER_INSTR / NWV; // B codes (planes: the nibble plane)
  static constexpr int CR_INSTR = (PL && BITS == 6) ? BN / 32 / NWV : 0;  // crumb-plane (32 B rows) instructions
  static constexpr int B_INSTR = NI + CR_INSTR;        // per wave per stage
  static constexpr int SI = ((BM + BN) / 64 + NWV - 1) / NWV;  // exponent instructions per wave (64 rows each)
  static constexpr int A_BYTES = BM * 128, B_BYTES = BN * RP + (CR_INSTR ? BN * 32 : 0), S_BYTES = NWV * SI * 64 * 4;
  static constexpr int STAGE = A_BYTES + B_BYTES + S_BYTES;
  static constexpr int LOADS = A_INSTR + B_INSTR + SI;  // glds per wave per stage (A, B, exponents)
};
__device__ __forceinline__ int fA(int r) { return (r >> 1) & 7; }
template <int RP> __device__ __forceinline__ int fB(int r) { return RP == 64 ? ((r >> 2) & 3) : ((r >> 1) & 7); }

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 4, 0, 0);
}

template <int FB, int BN, int NWV>
__device__ __forceinline__ void issue_stage(char* buf, const uint8_t* Xq, const uint8_t* Xs, const uint8_t* Wq,
                                            const uint8_t* Wq2, const uint8_t* Ws, int wks, int m0, int n0, int M,
                                            int K, int64_t WRB, int KS, int kb, int w, int lane) {
  using G = L<FB, BN, NWV>;
  // A: BM / 8 instructions of 8 rows x 128 B
#pragma unroll
  for (int j = 0; j < G::A_INSTR; ++j) {
    const int g = w * G::A_INSTR + j, row = 8 * g + (lane >> 3), slot = lane & 7;
    const int gr = min(m0 + row, M - 1);
    glds16(Xq + (int64_t)gr * K + (int64_t)kb * 128 + 16 * (slot ^ fA(row)), buf + 8 * g * 128);
  }
  // B
  if constexpr (G::PL) {
    constexpr int NI = G::NI;  // nibble plane: 64 B rows, 16 rows per instruction
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int g = w * NI + j, row = 16 * g + (lane >> 2), ch = (lane & 3) ^ ((row >> 2) & 3);
      glds16(Wq + (int64_t)(n0 + row) * (K / 2) + (int64_t)kb * 64 + 16 * ch, buf + G::A_BYTES + 16 * g * 64);
    }
#pragma unroll
    for (int j = 0; j < G::CR_INSTR; ++j) {  // crumb plane: 32 B rows, 32 rows per instruction
      const int g = w * G::CR_INSTR + j, row = 32 * g + (lane >> 1), ch = (lane & 1) ^ ((row >> 3) & 1);
      glds16(Wq2 + (int64_t)(n0 + row) * (K / 4) + (int64_t)kb * 32 + 16 * ch, buf + G::A_BYTES + BN * 64 + 32 * g * 32);
    }
  } else {
#pragma unroll
    for (int j = 0; j < G::NI; ++j) {
      const int g = w * G::NI + j, row = G::ROWS_PER_INSTR * g + lane / G::SL, slot = lane % G::SL;
      int ch = slot ^ fB<G::RP>(row);
      if (ch >= G::CH) ch = 0;  // fp6 padding slots: any in-row chunk, never read
      glds16(Wq + (int64_t)(n0 + row) * WRB + (int64_t)kb * G::RB + 16 * ch,
             buf + G::A_BYTES + G::ROWS_PER_INSTR * g * G::RP);
    }
  }
  // exponent words (4 E8M0 bytes per row per stage): waves 0-1 the A rows, waves 2-3 the B rows
  char* sb = buf + G::A_BYTES + G::B_BYTES;
  // exponent instructions per wave (64 rows each); every wave issues the same count (so one vmcnt
  // constant fits all), the slots past the A and B rows re-load A rows into a spare area
#pragma unroll
  for (int j = 0; j < G::SI; ++j) {
    const int g = w * G::SI + j;  // A rows 0..BM-1 first, then B rows 0..BN-1, then spares
    if (g < BM / 64 || g >= (BM + BN) / 64) {
      const int ga = g < BM / 64 ? g : 0;
      const int row = 64 * ga + lane, gr = min(m0 + row, M - 1);
      glds4(Xs + (int64_t)gr * KS + 4 * kb, sb + 64 * g * 4);
    } else {
      const int row = 64 * (g - BM / 64) + lane;
      glds4(Ws + (int64_t)(n0 + row) * wks + 4 * kb, sb + BM * 4 + 64 * (g - BM / 64) * 4);
    }
  }
}

// 0xFF in each byte whose (small) value is zero
__device__ __forceinline__ unsigned zero_bytes(unsigned e) {
  const unsigned nz = (e | (e >> 1) | (e >> 2)) & 0x01010101u;
  const unsigned z = nz ^ 0x01010101u;
  return (z << 8) - z;
}
// 4 e3m2 codes (sign|exp nibble per byte, 2 mantissa bits per byte) -> 4 e4m3 bytes, exact. Pure
// bytewise arithmetic (no carries cross a byte): hipcc 7.2's instcombine crashes on v_perm table
// lookups in this kernel.
__device__ __forceinline__ unsigned e3m2x4_to_e4m3(unsigned se, unsigned m) {
  const unsigned e = se & 0x07070707u, sg = (se & 0x08080808u) << 4;
  const unsigned nrm = ((e + 0x04040404u) << 3) | (m << 1);
  const unsigned z = zero_bytes(e);  // subnormal / zero codes: m * 2^-4 = e4m3 00 / 18 / 20 / 24
  const unsigned b1 = m & 0x01010101u, b2 = (m >> 1) & 0x01010101u;
  const unsigned sub = ((b1 | b2) << 4) + (m << 3) - ((b1 & b2) << 2);
  return sg | (z & sub) | (~z & nrm);
}
// 4 e2m1 codes (one per byte) -> 4 e4m3 bytes, exact
__device__ __forceinline__ unsigned e2m1x4_to_e4m3(unsigned x) {
  const unsigned sg = (x & 0x08080808u) << 4, e = (x >> 1) & 0x03030303u, m = x & 0x01010101u;
  const unsigned nrm = ((e + 0x06060606u) << 3) | (m << 2);
  const unsigned z = zero_bytes(e);
  return sg | (z & ((m << 5) | (m << 4))) | (~z & nrm);
}

template <int FB, int BN>
__device__ __forceinline__ i32x8 read_b(const char* bb, int row, int s, int h) {
  using G = L<FB, BN>;
  const char* rp = bb + row * G::RP;
  if constexpr (G::PL) {
    // two 16-value pieces at K = 64 s + 32 p + 16 h of the stage (the fp8 operand's halves)
    unsigned d[8];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int k0 = 64 * s + 32 * p + 16 * h;
      const int no = k0 >> 1;  // nibble-plane byte offset (8 B = 16 values)
      const u32x2 n = *reinterpret_cast<const u32x2*>(rp + 16 * ((no >> 4) ^ ((row >> 2) & 3)) + (no & 15));
      if constexpr (G::BITS == 6) {
        const int co = k0 >> 2;  // crumb-plane byte offset (4 B = 16 values)
        const unsigned c = *reinterpret_cast<const unsigned*>(bb + BN * 64 + row * 32 + 16 * ((co >> 4) ^ ((row >> 3) & 1)) +
                                                              (co & 15));
        d[4 * p + 0] = e3m2x4_to_e4m3(n[0] & 0x0F0F0F0Fu, c & 0x03030303u);
        d[4 * p + 1] = e3m2x4_to_e4m3((n[0] >> 4) & 0x0F0F0F0Fu, (c >> 2) & 0x03030303u);
        d[4 * p + 2] = e3m2x4_to_e4m3(n[1] & 0x0F0F0F0Fu, (c >> 4) & 0x03030303u);
        d[4 * p + 3] = e3m2x4_to_e4m3((n[1] >> 4) & 0x0F0F0F0Fu, (c >> 6) & 0x03030303u);
      } else {
        d[4 * p + 0] = e2m1x4_to_e4m3(n[0] & 0x0F0F0F0Fu);
        d[4 * p + 1] = e2m1x4_to_e4m3((n[0] >> 4) & 0x0F0F0F0Fu);
        d[4 * p + 2] = e2m1x4_to_e4m3(n[1] & 0x0F0F0F0Fu);
        d[4 * p + 3] = e2m1x4_to_e4m3((n[1] >> 4) & 0x0F0F0F0Fu);
      }
    }
    return i32x8{(int)d[0], (int)d[1], (int)d[2], (int)d[3], (int)d[4], (int)d[5], (int)d[6], (int)d[7]};
  } else if constexpr (G::BITS == 8) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(rp + 16 * ((4 * s + h) ^ fB<G::RP>(row)));
    const u32x4 b = *reinterpret_cast<const u32x4*>(rp + 16 * ((4 * s + 2 + h) ^ fB<G::RP>(row)));
    return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
  } else if constexpr (G::BITS == 4) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(rp + 16 * ((2 * s + h) ^ fB<G::RP>(row)));
    return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], 0, 0, 0, 0};
  } else {
    const int o = 48 * s + 24 * h;
    u32x2 p[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int oq = o + 8 * q;
      p[q] = *reinterpret_cast<const u32x2*>(rp + 16 * ((oq >> 4) ^ fB<G::RP>(row)) + (oq & 15));
    }
    return i32x8{(int)p[0][0], (int)p[0][1], (int)p[1][0], (int)p[1][1], (int)p[2][0], (int)p[2][1], 0, 0};
  }
}

template <int FB, int NBUF, int BN, int NWV>
__global__ void __launch_bounds__(64 * NWV, 1)
    mx_gemm_dp_kernel(const uint8_t* __restrict__ Xq, const uint8_t* __restrict__ Xs, const uint8_t* __restrict__ Wq,
                      const uint8_t* __restrict__ Wq2, const uint8_t* __restrict__ Ws, int wks,
                      const unsigned short* __restrict__ bias, const float* __restrict__ col_scale,
                      unsigned short* __restrict__ Y, int M, int N, int K) {
  using G = L<FB, BN, NWV>;
  constexpr int WNW = NWV / 2;   // waves along N (2 along M)
  constexpr int TNW = BN / WNW;  // wave tile 128 x TNW
  constexpr int NJ = TNW / 32;   // 32-column accumulators per wave
  constexpr int MF = mfma_fmt(FB);  // an immediate operand of the MFMA
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // bijective XCD-major remap (8 XCDs, round-robin dispatch)
  const int tm = (M + BM - 1) / BM, tn = N / BN, nwg = tm * tn;
  const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int m0 = (pid % tm) * BM, n0 = (pid / tm) * BN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w / WNW, wn = w % WNW, h = lane >> 5, l32 = lane & 31;
  const int KS = K / 32;
  const int64_t WRB = (int64_t)K * G::BITS / 8;
  const int nk = K / BK;

  f32x16 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  issue_stage<FB, BN, NWV>(smem, Xq, Xs, Wq, Wq2, Ws, wks, m0, n0, M, K, WRB, KS, 0, w, lane);
  if (NBUF == 3 && nk > 1) issue_stage<FB, BN, NWV>(smem + G::STAGE, Xq, Xs, Wq, Wq2, Ws, wks, m0, n0, M, K, WRB, KS, 1, w, lane);
  for (int kb = 0; kb < nk; ++kb) {
    if (NBUF == 3 && kb + 1 < nk) vm_wait<G::LOADS>(); else vm_wait<0>();
    raw_barrier();  // stage kb landed for every wave; every wave is done reading stage kb - 1
    const int ahead = NBUF - 1;
    if (kb + ahead < nk)
      issue_stage<FB, BN, NWV>(smem + ((kb + ahead) % NBUF) * G::STAGE, Xq, Xs, Wq, Wq2, Ws, wks, m0, n0, M, K, WRB, KS,
                          kb + ahead, w, lane);
    const char* buf = smem + (kb % NBUF) * G::STAGE;
    const char* ba = buf;
    const char* bb = buf + G::A_BYTES;
    const unsigned* sc = reinterpret_cast<const unsigned*>(buf + G::A_BYTES + G::B_BYTES);
    unsigned sa[4], sbw[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) sa[i] = sc[wm * 128 + i * 32 + l32];
#pragma unroll
    for (int j = 0; j < NJ; ++j) sbw[j] = sc[BM + wn * TNW + j * 32 + l32];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      i32x8 a[4], b[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 128 + i * 32 + l32;
        const char* rp = ba + row * 128;
        const u32x4 x0 = *reinterpret_cast<const u32x4*>(rp + 16 * ((4 * s + h) ^ fA(row)));
        const u32x4 x1 = *reinterpret_cast<const u32x4*>(rp + 16 * ((4 * s + 2 + h) ^ fA(row)));
        a[i] = i32x8{(int)x0[0], (int)x0[1], (int)x0[2], (int)x0[3], (int)x1[0], (int)x1[1], (int)x1[2], (int)x1[3]};
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = read_b<FB, BN>(bb, wn * TNW + j * 32 + l32, s, h);
      const int sh = 8 * (2 * s + h);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(  // Y^T tile: see store_t
              b[j], a[i], acc[i][j], MF, 0, 0, (int)((sbw[j] >> sh) & 0xff), 0, (int)((sa[i] >> sh) & 0xff));
      __builtin_amdgcn_s_setprio(0);
    }
  }
  store_t<4, NJ>(acc, Y, col_scale, bias, m0 + wm * 128, n0 + wn * TNW, M, N, h, l32);
}
}  // namespace dp



template <int BM, int BN, int WM, int WN, int FB>
void launch(const at::Tensor& xq, const at::Tensor& xs, const at::Tensor& wq, const at::Tensor& ws,
            const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& col_scale, at::Tensor& y, int M,
            int N, int K) {
  const size_t lds = (size_t)BM * SA + (size_t)BN * BLayout<FB>::SB;
  static bool attr = [&] {
    SXE_HIP_CHECK(hipFuncSetAttribute((const void*)mx_gemm_kernel<BM, BN, WM, WN, FB>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return true;
  }();
  (void)attr;
  const int G = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((mx_gemm_kernel<BM, BN, WM, WN, FB>), dim3(G), dim3(64 * WM * WN), lds, cur_stream(),
                     xq.data_ptr<uint8_t>(), xs.data_ptr<uint8_t>(), wq.data_ptr<uint8_t>(), ws.data_ptr<uint8_t>(),
                     bias ? reinterpret_cast<const unsigned short*>(bias->data_ptr()) : nullptr,
                     col_scale ? col_scale->data_ptr<float>() : nullptr,
                     reinterpret_cast<unsigned short*>(y.data_ptr()), M, N, K);
}

// tile variants: 0 auto, 1 = 128x128 / 4 waves, 2 = 256x128 / 4 waves, 3 = 256x256 / 4 waves
// (128x128 per wave, accumulators in AGPRs), 4 = 256x256 / 8 waves, 5 = 256x128 / 8 waves,
// 6 = 256x256 / 8 waves LDS-DMA pipelined (namespace dp), 7 = the same at 256x128 / 4 waves,
// 8 = 256x256 / 4 waves (a phased 64-deep-stage form of 6 measured slower on every shape:
// profiles/r05/mx_gemm_phased_tile_ab.log; 6 with 64-deep half stages, four in LDS, was slower
// too: profiles/r05/mx_half_stage_tile_ab.log), 9 = 64x128 / 4 waves (32x64 per wave) and
// 10 = 64x64 / 4 waves (32x32 per wave) for problems whose 128x128 grid leaves CUs idle
static int tile_override() {  // read per call: the kernel tests sweep every variant in one process
  const char* e = getenv("SXE_MX_TILE");
  return e ? atoi(e) : 0;
}

template <int FB, int BN, int NWV = (BN == 256 ? 8 : 4)>
void launch_dp(const at::Tensor& xq, const at::Tensor& xs, const at::Tensor& wq, const at::Tensor& ws,
               const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& cs, at::Tensor& y, int M, int N,
               int K, const uint8_t* wq2 = nullptr) {
  using G = dp::L<FB, BN, NWV>;
  constexpr int NBUF = G::STAGE * 3 <= 160 * 1024 ? 3 : 2;
  const size_t lds = (size_t)NBUF * G::STAGE;
  static bool attr = [&] {
    SXE_HIP_CHECK(hipFuncSetAttribute((const void*)dp::mx_gemm_dp_kernel<FB, NBUF, BN, NWV>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return true;
  }();
  (void)attr;
  const int G_ = ((M + dp::BM - 1) / dp::BM) * (N / BN);
  const int wks = ws.size(0) == 1 ? 0 : (int)ws.size(1);  // one exponent row shared by all columns
  hipLaunchKernelGGL((dp::mx_gemm_dp_kernel<FB, NBUF, BN, NWV>), dim3(G_), dim3(64 * NWV), lds, cur_stream(),
                     xq.data_ptr<uint8_t>(), xs.data_ptr<uint8_t>(), wq.data_ptr<uint8_t>(), wq2,
                     ws.data_ptr<uint8_t>(), wks, bias ? reinterpret_cast<const unsigned short*>(bias->data_ptr()) : nullptr,
                     cs ? cs->data_ptr<float>() : nullptr, reinterpret_cast<unsigned short*>(y.data_ptr()), M, N, K);
}

template <int FB>
void dispatch_tile(const at::Tensor& xq, const at::Tensor& xs, const at::Tensor& wq, const at::Tensor& ws,
                   const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& cs, at::Tensor& y, int M,
                   int N, int K) {
  int v = tile_override();
  if (v == 0) {
    // measured on MI355X (profiles/mx_gemm_bench.log, profiles/r06/mx/mx_small_tiles.log): the LDS-DMA
    // pipelined 256 x 256 tile once it fills the chip, its 256 x 128 form when that still gives >= half
    // a workgroup per CU, the 64 x 64 tile while a 128 x 128 grid would leave CUs idle (M <= 512 at
    // N 4096 / 6144, M 128 at N 14336: 1.2-1.7x faster than 128 x 128 there), else 128 x 128
    const int64_t g256 = (int64_t)((M + 255) / 256) * (N / 256), g2561 = (int64_t)((M + 255) / 256) * (N / 128);
    const int64_t g128 = (int64_t)((M + 127) / 128) * (N / 128);
    v = (N % 256 == 0 && M > 256 && g256 >= kNumCUs) ? 6
        : (M > 256 && g2561 >= kNumCUs / 2)          ? 7
        : g128 < kNumCUs                             ? 10
                                                     : 1;
  }
  if ((v == 3 || v == 4 || v == 6 || v == 8) && N % 256 != 0) v = 2;
  switch (v) {
    case 6: launch_dp<FB, 256>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 8: launch_dp<FB, 256, 4>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 7: launch_dp<FB, 128>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 2: launch<256, 128, 2, 2, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 3: launch<256, 256, 2, 2, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 4: launch<256, 256, 2, 4, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 5: launch<256, 128, 2, 4, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 9: launch<64, 128, 2, 2, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    case 10: launch<64, 64, 2, 2, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
    default: launch<128, 128, 2, 2, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K); break;
  }
}

}  // namespace mx

// x [M, K] bf16 (K % 32 == 0) -> (e4m3 codes uint8 [M, K], E8M0 exponents uint8 [M, K / 32])
std::vector<at::Tensor> mx_quant_fp8(at::Tensor x) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.dim() == 2 && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "mx_quant_fp8: x [M, K] bf16");
  SXE_CHECK(x.size(1) % 32 == 0, "mx_quant_fp8: K must be a multiple of 32");
  c10::DeviceGuard guard(x.device());
  auto q = at::empty({x.size(0), x.size(1)}, x.options().dtype(at::kByte));
  auto s = at::empty({x.size(0), x.size(1) / 32}, x.options().dtype(at::kByte));
  const int64_t nb = x.numel() / 32;
  if (nb)
    hipLaunchKernelGGL(mx::mx_quant_fp8_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const unsigned short*>(x.data_ptr()), q.data_ptr<uint8_t>(),
                       s.data_ptr<uint8_t>(), nb);
  SXE_LAUNCH_CHECK();
  return {q, s};
}

// y [M, N] bf16 = MX(xq, xs) @ MX(wq, ws)^T (+ bias) (* col_scale); fmt: 0 e4m3, 2 e2m3, 3 e3m2, 4 e2m1
// fmt 16 / 17: FPxWeight bit planes -- wq = nibble plane [N, K / 2], wq2 = 2-bit plane [N, K / 4] (FP6),
// ws = E8M0 127s [1, K / 32] (per-row scales go in col_scale)
at::Tensor mx_gemm(at::Tensor xq, at::Tensor xs, at::Tensor wq, at::Tensor ws, int64_t fmt,
                   c10::optional<at::Tensor> bias, c10::optional<at::Tensor> col_scale, c10::optional<at::Tensor> wq2) {
  SXE_CHECK_CUDA(xq);
  SXE_CHECK(fmt == 0 || fmt == 2 || fmt == 3 || fmt == 4 || fmt == 16 || fmt == 17,
            "mx_gemm: weight format 0 (e4m3) / 2 (e2m3) / 3 (e3m2) / 4 (e2m1) / 16, 17 (FP6 / FP4 bit planes)");
  SXE_CHECK(xq.dim() == 2 && xq.is_contiguous() && xq.scalar_type() == at::kByte, "mx_gemm: xq uint8 [M, K]");
  SXE_CHECK(wq.dim() == 2, "mx_gemm: wq [N, bytes per row]");
  const int64_t M = xq.size(0), K = xq.size(1), N = wq.size(0);
  const bool planes = mx::is_planes((int)fmt);
  const int bits = mx::fmt_bits((int)fmt);
  SXE_CHECK(K % mx::BK == 0, "mx_gemm: K must be a multiple of 128");
  SXE_CHECK(N % 128 == 0, "mx_gemm: N must be a multiple of 128");
  SXE_CHECK(xs.is_contiguous() && xs.scalar_type() == at::kByte && xs.numel() == M * (K / 32), "mx_gemm: xs uint8 [M, K/32]");
  SXE_CHECK(wq.is_contiguous() && wq.scalar_type() == at::kByte && wq.numel() == N * K * (planes ? 4 : bits) / 8,
            "mx_gemm: wq packed codes [N, K * bits / 8] (planes: nibble plane [N, K / 2])");
  if (planes && bits == 6) {
    SXE_CHECK(wq2.has_value() && wq2->defined() && wq2->is_cuda() && wq2->is_contiguous() &&
                  wq2->scalar_type() == at::kByte && wq2->numel() == N * K / 4,
              "mx_gemm: FP6 planes need the 2-bit plane [N, K / 4]");
  }
  SXE_CHECK(ws.dim() == 2 && ws.is_contiguous() && ws.scalar_type() == at::kByte && ws.size(1) == K / 32 &&
                (ws.size(0) == N || (planes && ws.size(0) == 1)),
            "mx_gemm: ws uint8 [N, K/32] (planes: [1, K/32])");
  SXE_CHECK(xs.is_cuda() && wq.is_cuda() && ws.is_cuda(), "mx_gemm: operands on the GPU");
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N,
              "mx_gemm: bias bf16 [N]");
  } else {
    bias = c10::nullopt;
  }
  if (col_scale.has_value() && col_scale->defined()) {
    SXE_CHECK(col_scale->is_cuda() && col_scale->is_contiguous() && col_scale->scalar_type() == at::kFloat &&
                  col_scale->numel() == N,
              "mx_gemm: col_scale fp32 [N]");
  } else {
    col_scale = c10::nullopt;
  }
  SXE_CHECK(M * N < (1ll << 31) && N * K < (1ll << 31), "mx_gemm: problem too large");
  c10::DeviceGuard guard(xq.device());
  auto y = at::empty({M, N}, xq.options().dtype(at::kBFloat16));
  if (M == 0) return y;
  if (planes) {  // the LDS-DMA pipelined tiles (the planes are staged as two sub-tiles)
    const uint8_t* w2 = bits == 6 ? wq2->data_ptr<uint8_t>() : nullptr;
    const bool wide = N % 256 == 0 && ((M + 255) / 256) * (N / 256) >= sxe::kNumCUs;
    if (bits == 6) {
      wide ? mx::launch_dp<16, 256>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K, w2)
           : mx::launch_dp<16, 128>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K, w2);
    } else {
      wide ? mx::launch_dp<17, 256>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K)
           : mx::launch_dp<17, 128>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K);
    }
    SXE_LAUNCH_CHECK();
    return y;
  }
  switch (fmt) {
    case 0: mx::dispatch_tile<0>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
    case 2: mx::dispatch_tile<2>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
    case 3: mx::dispatch_tile<3>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
    default: mx::dispatch_tile<4>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
  }
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("mx_quant_fp8(Tensor x) -> Tensor[]");
  m.def("mx_gemm(Tensor xq, Tensor xs, Tensor wq, Tensor ws, int fmt, Tensor? bias=None, Tensor? col_scale=None, "
        "Tensor? wq2=None) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("mx_quant_fp8", &sxe::mx_quant_fp8);
  m.impl("mx_gemm", &sxe::mx_gemm);
}

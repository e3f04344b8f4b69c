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
// Geometry: 256 x 256 tile, BK = 32, 8 waves (2 along M x 4 along N), 128 x 64 per wave as 4 x 2
// v_mfma_f32_32x32x16_bf16 accumulators (128 AGPR-able fp32 / lane); LDS ring of NSTAGE K-slabs.
// Block order: XCD-aware remap + GROUP_M super-rows so blocks on one XCD share A/B tiles in L2.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace wg {

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int NWAVE = 8, NTHR = NWAVE * 64;
constexpr int ROWB = 256;                   // bytes per LDS row (128 bf16)
constexpr int HALF = BK * ROWB;             // one [BK][128] half tile
constexpr int STAGE = 4 * HALF;             // A (2 halves) + B (2 halves) = 32 KiB
constexpr int NSTAGE = 4;               // 128 KiB ring: slabs issued 3 ahead
constexpr int GROUP_M = 8;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int soff(int row, int ch) { return row * ROWB + 16 * (ch ^ swz(row)); }

__device__ __forceinline__ i16x4 lds_tr(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(const_cast<char*>(base) + byte_off));
}

// MFMA operand (A or B of 32x32x16) from a row-major [k][128] LDS half tile, transposed: lane gets
// column 32*dt + (lane&31); element j of lane half h <- k row row0 + 8*(j>>2) + 4h + (j&3).
// A and B use the same k permutation, so it cancels in the product.
__device__ __forceinline__ bf16x8 frag(const char* base, int row0, int dt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const int row = row0 + 4 * h + q;
  i16x4 lo = lds_tr(base, soff(row, ch) + 8 * (p & 1));
  i16x4 hi = lds_tr(base, soff(row + 8, ch) + 8 * (p & 1));
  const i16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

// LDS-DMA issued from inline asm: hipcc's waitcnt pass cannot see it, so it does not put a
// conservative `s_waitcnt vmcnt(0)` in front of every ds_read of the ring (it did with the
// builtin: the whole prefetch drained each K-step). Completion is tracked by the explicit counted
// vmcnt + barrier in the main loop.
__device__ __forceinline__ void glds16(const void* gsrc, char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(gsrc) : "memory", "m0");
}

// One K-slab: rows k0..k0+BK of A[:, m0:m0+256] and B[:, n0:n0+256] into stage `st`.
// 32 wave-instructions of 1 KiB (4 rows x 16 chunks of one half tile); 4 per wave.
__device__ __forceinline__ void load_stage(const unsigned short* A, int64_t lda, const unsigned short* B,
                                           int64_t ldb, int k0, int m0, int n0, char* st) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int n = it * NWAVE + w;          // 0..31
    const int op = n >> 4;                 // 0 = A, 1 = B
    const int half = (n >> 3) & 1;
    const int rq = n & 7;                  // row quad within the half
    const int row = 4 * rq + (lane >> 4);
    const int ch = (lane & 15) ^ swz(row);
    const unsigned short* src = op == 0 ? A + (int64_t)(k0 + row) * lda + m0 + half * 128 + ch * 8
                                        : B + (int64_t)(k0 + row) * ldb + n0 + half * 128 + ch * 8;
    glds16(src, st + (op * 2 + half) * HALF + rq * 1024);
  }
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

template <bool ACCUM>
__global__ void __launch_bounds__(NTHR, 1) wgrad_kernel(const unsigned short* __restrict__ A, int64_t lda,
                                                        const unsigned short* __restrict__ B, int64_t ldb,
                                                        float* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        float alpha) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  // ---- block -> tile (XCD-aware, grouped along M) ------------------------------------------
  const int tm = M / BM, tn = N / BN, nwg = tm * tn;
  const int orig = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int per_group = GROUP_M * tn;
  const int grp = wgid / per_group;
  const int first_m = grp * GROUP_M;
  const int gsz = min(tm - first_m, GROUP_M);
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

  const int nk = K / BK;
  // prologue: slabs 0..NSTAGE-2 in flight
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) load_stage(A, lda, B, ldb, s * BK, m0, n0, smem + s * STAGE);
  for (int kt = 0; kt < nk; ++kt) {
    // slab kt must have landed; slabs issued after it (up to NSTAGE-2 of them, 4 loads each) may
    // still be in flight -- counted wait, never vmcnt(0) in steady state
    const int after = min(nk - 1 - kt, NSTAGE - 2);
    if (after >= 2)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // WAR-safe: stage (kt-1)%NSTAGE was last read in iteration kt-1, which every wave has left
    if (kt + NSTAGE - 1 < nk)
      load_stage(A, lda, B, ldb, (kt + NSTAGE - 1) * BK, m0, n0, smem + ((kt + NSTAGE - 1) % NSTAGE) * STAGE);
    const char* cur = smem + (kt % NSTAGE) * STAGE;
    const char* Ah = cur + wr * HALF;                         // A columns wr*128 .. +128
    const char* Bh = cur + (2 + (wc >> 1)) * HALF;            // B columns (wc>>1)*128 .. +128
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(Ah, ks * 16, i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = frag(Bh, ks * 16, (wc & 1) * 2 + j, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
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

}  // namespace wg

bool wgrad_supported(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c) {
  return a.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
         c.scalar_type() == at::kFloat && a.dim() == 2 && b.dim() == 2 && c.dim() == 2 && a.stride(1) == 1 &&
         b.stride(1) == 1 && c.stride(1) == 1 && a.size(0) == b.size(0) && c.size(0) == a.size(1) &&
         c.size(1) == b.size(1) && a.size(1) % wg::BM == 0 && b.size(1) % wg::BN == 0 && a.size(0) % wg::BK == 0 &&
         (reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0) && (reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0) &&
         a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0;
}

// c (+)= alpha * a^T @ b ; a: [K, M] bf16, b: [K, N] bf16, c: [M, N] fp32
void wgrad_gemm_(const at::Tensor& a, const at::Tensor& b, at::Tensor c, double alpha, bool accumulate) {
  SXE_CHECK(wgrad_supported(a, b, c), "wgrad_gemm_: unsupported shapes/dtypes/strides");
  c10::DeviceGuard g(a.device());
  const int K = a.size(0), M = a.size(1), N = b.size(1);
  const int nwg = (M / wg::BM) * (N / wg::BN);
  const size_t lds = wg::NSTAGE * wg::STAGE;
  auto launch = [&](auto kern) {
    static bool attr_set = false;
    if (!attr_set) {
      SXE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr_set = true;
    }
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(wg::NTHR), lds, cur_stream(),
                       reinterpret_cast<const unsigned short*>(a.data_ptr()), a.stride(0),
                       reinterpret_cast<const unsigned short*>(b.data_ptr()), b.stride(0), c.data_ptr<float>(),
                       c.stride(0), M, N, K, (float)alpha);
  };
  if (accumulate)
    launch(wg::wgrad_kernel<true>);
  else
    launch(wg::wgrad_kernel<false>);
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("wgrad_gemm_(Tensor a, Tensor b, Tensor(a!) c, float alpha, bool accumulate) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("wgrad_gemm_", &sxe::wgrad_gemm_); }

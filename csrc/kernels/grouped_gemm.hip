// Ragged grouped GEMM for MoE experts on gfx950: Y[r, :] = s[r] * X[r, :] @ W[e(r)]^T for rows
// sorted by expert, ONE launch for all experts, row counts read on the device.
//
// Reference semantics: inference/v2/kernels/cutlass_ops/moe_gemm/moe_gemm.cu (CUTLASS grouped
// GEMM over expert-sorted rows with per-expert cumulative row offsets). Differences,
// MI355X-first: the row offsets stay on the GPU -- each workgroup finds its (expert, row tile) by
// scanning the E+1 offsets itself, and the grid is launched for the upper bound ceil(R/128) + E
// row tiles (surplus workgroups exit at once) -- so a MoE layer needs no host synchronisation and
// can be captured in a HIP graph (the per-expert hipBLASLt loop needs the counts on the host).
// The optional per-row scale fuses the top-k routing weight into the down-projection epilogue.
//
// Mixed-precision experts (reference cutlass_ops/mixed_gemm/mixed_gemm.cu, mixed_moe_gemm: int8 /
// int4 weights x 16-bit activations): the same kernel with W[e] stored as int8 or packed int4
// (two's complement, low nibble first) plus one fp32 scale per (expert, output row, K group of
// gs = 128 x 2^j elements). The weight bytes are what HBM streams (1/2 and 1/4 of bf16); each
// workgroup widens its staged K block to bf16 (q * scale, exact for int8 up to the bf16 rounding of
// the product) on the way into LDS, so the conversion is paid once per 128-row output tile, and
// the MFMA loop is the bf16 one.
//
// Geometry: 128 x 128 output tile, 4 waves (2 x 2, 64 x 64 each as 2 x 2 v_mfma_f32_32x32x16_bf16
// accumulators), K in blocks of 128: both operands are K-contiguous (X rows; W[e] as [N, K], the
// nn.Linear layout), staged through registers into XOR-swizzled LDS tiles (sxe_mfma.h RowStager)
// and read back with ds_read_b128 -- the next K block's global loads are in flight while the
// current block's 32 MFMAs per wave run. Rows past the expert's range read as zeros and are not
// stored.
#include "sxe_common.h"
#include "sxe_mfma.h"
#include <torch/library.h>

namespace sxe {
namespace gg {
using namespace mf;

constexpr int BM = 128, BN = 128, BK = 128, NTHR = 256;
constexpr int TILE_BYTES = BM * ROWB;  // 32 KiB per operand tile

// K block of ROWS weight rows stored as int8 (BITS 8) or packed int4 (BITS 4), widened to bf16
// (times the row's group scale) into the same swizzled LDS tile RowStager<ROWS, BK> would write.
template <int ROWS, int BITS>
struct QStager {
  static constexpr int CPR = BK * BITS / 128;           // 16-byte chunks per row per K block
  static constexpr int EPC = 128 / BITS;                // elements per chunk
  static constexpr int N = ROWS * CPR / NTHR;
  u32x4 r[N];
  float sc[N];
  __device__ __forceinline__ void load(const uint8_t* base, int64_t row_bytes, const float* scale, int64_t srow,
                                       int sg, int row0, int valid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHR;
      const int row = c / CPR, ch = c % CPR;
      const bool ok = row0 + row < valid;
      r[i] = ok ? *reinterpret_cast<const u32x4*>(base + (int64_t)(row0 + row) * row_bytes + ch * 16)
                : u32x4{0u, 0u, 0u, 0u};
      sc[i] = ok ? scale[(int64_t)(row0 + row) * srow + sg] : 0.f;
    }
  }
  __device__ __forceinline__ void store(char* lds) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHR;
      const int row = c / CPR, ch = c % CPR;
#pragma unroll
      for (int o = 0; o < EPC / 8; ++o) {  // one 8-element bf16 chunk of LDS per step
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int idx = 8 * o + e;  // element within the 16-byte chunk
          int q;
          if constexpr (BITS == 8) {
            q = (int)(signed char)((r[i][idx >> 2] >> (8 * (idx & 3))) & 0xff);
          } else {
            q = (int)((r[i][idx >> 3] >> (4 * (idx & 7))) & 0xf);
            q = q >= 8 ? q - 16 : q;
          }
          v[e] = (__bf16)((float)q * sc[i]);
        }
        *reinterpret_cast<bf16x8*>(lds + soff(row, ch * (EPC / 8) + o)) = v;
      }
    }
  }
};

template <typename ScaleT>
__global__ void __launch_bounds__(NTHR, 2) grouped_gemm_kernel(const unsigned short* __restrict__ X,
                                                               const unsigned short* __restrict__ W,
                                                               const int* __restrict__ offs, int E,
                                                               const ScaleT* __restrict__ scale,
                                                               unsigned short* __restrict__ Y, int R, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* lA = smem;
  char* lB = smem + TILE_BYTES;
  // ---- (expert, row tile) of this workgroup: wave-uniform scan of the offsets --------------------
  int idx = blockIdx.x, e = 0, lo = 0, hi = 0;
  for (; e < E; ++e) {
    const int a = offs[e], b = offs[e + 1];
    const int nt = (b - a + BM - 1) / BM;
    if (idx < nt) {
      lo = a + idx * BM;
      hi = min(min(b, lo + BM), R);  // offsets past R (malformed input) never address outside X / Y
      break;
    }
    idx -= nt;
  }
  if (e == E || lo < 0 || lo >= hi) return;  // surplus workgroup of the upper-bound grid (uniform)
  const int n0 = blockIdx.y * BN;
  const unsigned short* We = W + (int64_t)e * N * K;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1, h = lane >> 5, l32 = lane & 31;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  RowStager<BM, BK, NTHR> sa;
  RowStager<BN, BK, NTHR> sb;
  sa.load(X, K, lo, hi);  // rows lo .. lo+127 of X (zeros past hi), columns 0 .. 127
  sb.load(We, K, n0, N);
  const int nk = K / BK;
  for (int kb = 0; kb < nk; ++kb) {
    if (kb) __syncthreads();  // every wave is done reading the previous block
    sa.store(lA);
    sb.store(lB);
    __syncthreads();
    if (kb + 1 < nk) {  // next block's global loads overlap this block's MFMAs
      sa.load(X + (kb + 1) * BK, K, lo, hi);
      sb.load(We + (kb + 1) * BK, K, n0, N);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = lds_row16(lA, wm * 64 + i * 32 + l32, 2 * ks + h);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = lds_row16(lB, wn * 64 + j * 32 + l32, 2 * ks + h);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // Y^T tile: see store_acc_t
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // ---- epilogue: lane holds token row m, 4 runs of 4 columns per accumulator ---------------------
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = lo + wm * 64 + i * 32 + l32;  // lane's token row (transposed accumulators)
    if (m >= hi) continue;
    const float sm = scale ? (float)scale[m] : 1.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) store_acc_t(acc[i][j], Y + (int64_t)m * N + n0 + wn * 64 + j * 32 + 4 * h, sm);
  }
}



// ---------------------------------------------------------------------------------------------------
// Large-expert form (bf16): 256 x 256 output tile, 4 waves (2 x 2, 128 x 128 each = 16 accumulators
// in AGPRs), K in stages of 64 staged by LDS-DMA (global_load_lds) into two stage buffers with a raw
// s_barrier, so the next stage's DMA overlaps the current stage's 64 MFMAs per wave -- the same
// pipeline as the MX GEMM (mx_gemm.hip namespace dp). A glds writes lane-linear LDS, so the
// bank-conflict swizzle goes on the source address: 16-byte slot s of a 128-byte row r holds chunk
// s ^ ((r >> 1) & 7). Rows past the expert's range load the range's last row and are not stored.
namespace dp {
constexpr int BM = 256, BN = 256, BKD = 64;
constexpr int TILE = BM * BKD * 2;           // 32 KiB per operand per stage
constexpr int STAGE = 2 * TILE;
__device__ __forceinline__ int sw(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// WN = waves along N (2 -> 4 waves of 128 x 128; 4 -> 8 waves of 128 x 64, two per SIMD -- the
// default: 800-903 TF/s vs 713-853 for 4 waves and 472-600 for the 128 x 128 kernel at 1024-4096
// rows per expert, profiles/grouped_gemm_bench.log)
template <typename ScaleT, int WN>
__global__ void __launch_bounds__(128 * WN, 1) grouped_gemm_dp_kernel(const unsigned short* __restrict__ X,
                                                                const unsigned short* __restrict__ W,
                                                                const int* __restrict__ offs, int E,
                                                                const ScaleT* __restrict__ scale,
                                                                unsigned short* __restrict__ Y, int R, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int idx = blockIdx.x, e = 0, lo = 0, hi = 0;
  for (; e < E; ++e) {
    const int a = offs[e], b = offs[e + 1];
    const int nt = (b - a + BM - 1) / BM;
    if (idx < nt) {
      lo = a + idx * BM;
      hi = min(min(b, lo + BM), R);
      break;
    }
    idx -= nt;
  }
  if (e == E || lo < 0 || lo >= hi) return;  // surplus workgroup of the upper-bound grid (uniform)
  const int n0 = blockIdx.y * BN;
  const unsigned short* We = W + (int64_t)e * N * K;
  constexpr int NW = 2 * WN, NJ = 4 * 2 / WN, PI = 32 / NW;  // waves, 32-col tiles per wave, glds per operand
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w / WN, wn = w % WN, h = lane >> 5, l32 = lane & 31;

  auto issue = [&](char* buf, int kb) {
#pragma unroll
    for (int j = 0; j < PI; ++j) {  // A: 32 instructions of 8 rows x 128 B
      const int g = w * PI + j, row = 8 * g + (lane >> 3), slot = lane & 7;
      const int gr = min(lo + row, hi - 1);
      glds16(X + (int64_t)gr * K + (int64_t)kb * BKD + 8 * (slot ^ sw(row)), buf + 8 * g * 128);
    }
#pragma unroll
    for (int j = 0; j < PI; ++j) {  // B: the expert's weight rows n0 .. n0 + 255
      const int g = w * PI + j, row = 8 * g + (lane >> 3), slot = lane & 7;
      glds16(We + (int64_t)(n0 + row) * K + (int64_t)kb * BKD + 8 * (slot ^ sw(row)), buf + TILE + 8 * g * 128);
    }
  };

  f32x16 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = zero16();

  const int nk = K / BKD;
  issue(smem, 0);
  for (int kb = 0; kb < nk; ++kb) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // stage kb landed for every wave; every wave is done with stage kb - 1
    if (kb + 1 < nk) issue(smem + ((kb + 1) & 1) * STAGE, kb + 1);
    const char* ba = smem + (kb & 1) * STAGE;
    const char* bb = ba + TILE;
#pragma unroll
    for (int ks = 0; ks < BKD / 16; ++ks) {
      bf16x8 a[4], b[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 128 + i * 32 + l32;
        a[i] = *reinterpret_cast<const bf16x8*>(ba + row * 128 + 16 * ((2 * ks + h) ^ sw(row)));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * (BN / WN) + j * 32 + l32;
        b[j] = *reinterpret_cast<const bf16x8*>(bb + row * 128 + 16 * ((2 * ks + h) ^ sw(row)));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // Y^T tile
      __builtin_amdgcn_s_setprio(0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = lo + wm * 128 + i * 32 + l32;
    if (m >= hi) continue;
    const float sm = scale ? (float)scale[m] : 1.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      store_acc_t(acc[i][j], Y + (int64_t)m * N + n0 + wn * (BN / WN) + j * 32 + 4 * h, sm);
  }
}
}  // namespace dp

// Mixed-precision variant: W[e] as int8 / int4 codes [E, N, K * BITS / 8] with fp32 group scales
// [E, N, K / gs]; everything else as grouped_gemm_kernel.
template <typename ScaleT, int BITS>
__global__ void __launch_bounds__(NTHR, 2) grouped_gemm_q_kernel(const unsigned short* __restrict__ X,
                                                                 const uint8_t* __restrict__ Wq,
                                                                 const float* __restrict__ Ws, int gs_blocks,
                                                                 const int* __restrict__ offs, int E,
                                                                 const ScaleT* __restrict__ scale,
                                                                 unsigned short* __restrict__ Y, int R, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* lA = smem;
  char* lB = smem + TILE_BYTES;
  int idx = blockIdx.x, e = 0, lo = 0, hi = 0;
  for (; e < E; ++e) {
    const int a = offs[e], b = offs[e + 1];
    const int nt = (b - a + BM - 1) / BM;
    if (idx < nt) {
      lo = a + idx * BM;
      hi = min(min(b, lo + BM), R);
      break;
    }
    idx -= nt;
  }
  if (e == E || lo < 0 || lo >= hi) return;
  const int n0 = blockIdx.y * BN;
  const int64_t WRB = (int64_t)K * BITS / 8;
  const int G = K / (BK * gs_blocks);  // scale groups per row
  const uint8_t* We = Wq + (int64_t)e * N * WRB;
  const float* Se = Ws + (int64_t)e * N * G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1, h = lane >> 5, l32 = lane & 31;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  RowStager<BM, BK, NTHR> sa;
  QStager<BN, BITS> sb;
  sa.load(X, K, lo, hi);
  sb.load(We, WRB, Se, G, 0, n0, N);
  const int nk = K / BK;
  for (int kb = 0; kb < nk; ++kb) {
    if (kb) __syncthreads();
    sa.store(lA);
    sb.store(lB);
    __syncthreads();
    if (kb + 1 < nk) {
      sa.load(X + (kb + 1) * BK, K, lo, hi);
      sb.load(We + (int64_t)(kb + 1) * BK * BITS / 8, WRB, Se, G, (kb + 1) / gs_blocks, n0, N);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = lds_row16(lA, wm * 64 + i * 32 + l32, 2 * ks + h);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = lds_row16(lB, wn * 64 + j * 32 + l32, 2 * ks + h);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // Y^T tile: see store_acc_t
      __builtin_amdgcn_s_setprio(0);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = lo + wm * 64 + i * 32 + l32;  // lane's token row (transposed accumulators)
    if (m >= hi) continue;
    const float sm = scale ? (float)scale[m] : 1.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) store_acc_t(acc[i][j], Y + (int64_t)m * N + n0 + wn * 64 + j * 32 + 4 * h, sm);
  }
}

}  // namespace gg

// y[R, N] = row_scale * x[R, K] @ w[e]^T per expert segment offsets[e] .. offsets[e+1]
at::Tensor grouped_gemm(at::Tensor x, at::Tensor w, at::Tensor offsets, c10::optional<at::Tensor> row_scale) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.dim() == 2 && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "grouped_gemm: x [R, K] bf16");
  SXE_CHECK(w.dim() == 3 && w.is_contiguous() && w.scalar_type() == at::kBFloat16, "grouped_gemm: w [E, N, K] bf16");
  const int64_t R = x.size(0), K = x.size(1), E = w.size(0), N = w.size(1);
  SXE_CHECK(w.size(2) == K, "grouped_gemm: K mismatch");
  SXE_CHECK(K % gg::BK == 0 && N % gg::BN == 0, "grouped_gemm: K and N must be multiples of 128");
  SXE_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.is_contiguous() &&
                offsets.numel() == E + 1,
            "grouped_gemm: offsets int32 [E + 1] on the device");
  SXE_CHECK(R + E * gg::BM < (1ll << 31), "grouped_gemm: too many rows");
  const bool hs = row_scale.has_value() && row_scale->defined();
  if (hs)
    SXE_CHECK(row_scale->is_cuda() && row_scale->is_contiguous() && row_scale->numel() == R &&
                  (row_scale->scalar_type() == at::kFloat || row_scale->scalar_type() == at::kBFloat16),
              "grouped_gemm: row_scale fp32/bf16 [R]");
  c10::DeviceGuard guard(x.device());
  auto y = at::empty({R, N}, x.options());
  if (R == 0 || N == 0) return y;
  auto X = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto Wp = reinterpret_cast<const unsigned short*>(w.data_ptr());
  auto Yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  const int* off = offsets.data_ptr<int>();
  // many rows per expert: the LDS-DMA pipelined 256 x 256 tiles (decided from the shapes only --
  // the row counts stay on the device; measured crossover in profiles/grouped_gemm_bench.log)
  const char* force = getenv("SXE_GG_TILE");
  const bool big = force ? atoi(force) == 256 : (R >= 256 * E && N % gg::dp::BN == 0 && K % gg::dp::BKD == 0);
  if (big && N % gg::dp::BN == 0 && K % gg::dp::BKD == 0) {
    const size_t lds_dp = 2 * gg::dp::STAGE;
    const dim3 grid_dp((unsigned)((R + gg::dp::BM - 1) / gg::dp::BM + E), (unsigned)(N / gg::dp::BN));
    const char* wne = getenv("SXE_GG_WN");
    const int wn = wne ? atoi(wne) : 4;
    auto go = [&](auto kern, int nthr) {
      SXE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_dp));
      return nthr;
    };
    if (hs && row_scale->scalar_type() == at::kBFloat16) {
      const __bf16* rs = reinterpret_cast<const __bf16*>(row_scale->data_ptr());
      if (wn == 2) {
        go(gg::dp::grouped_gemm_dp_kernel<__bf16, 2>, 256);
        hipLaunchKernelGGL((gg::dp::grouped_gemm_dp_kernel<__bf16, 2>), grid_dp, dim3(256), lds_dp, cur_stream(), X, Wp,
                           off, (int)E, rs, Yp, (int)R, (int)N, (int)K);
      } else {
        go(gg::dp::grouped_gemm_dp_kernel<__bf16, 4>, 512);
        hipLaunchKernelGGL((gg::dp::grouped_gemm_dp_kernel<__bf16, 4>), grid_dp, dim3(512), lds_dp, cur_stream(), X, Wp,
                           off, (int)E, rs, Yp, (int)R, (int)N, (int)K);
      }
    } else {
      const float* rs = hs ? row_scale->data_ptr<float>() : nullptr;
      if (wn == 2) {
        go(gg::dp::grouped_gemm_dp_kernel<float, 2>, 256);
        hipLaunchKernelGGL((gg::dp::grouped_gemm_dp_kernel<float, 2>), grid_dp, dim3(256), lds_dp, cur_stream(), X, Wp,
                           off, (int)E, rs, Yp, (int)R, (int)N, (int)K);
      } else {
        go(gg::dp::grouped_gemm_dp_kernel<float, 4>, 512);
        hipLaunchKernelGGL((gg::dp::grouped_gemm_dp_kernel<float, 4>), grid_dp, dim3(512), lds_dp, cur_stream(), X, Wp,
                           off, (int)E, rs, Yp, (int)R, (int)N, (int)K);
      }
    }
    SXE_LAUNCH_CHECK();
    return y;
  }
  const size_t lds = 2 * gg::TILE_BYTES;
  const dim3 grid((unsigned)((R + gg::BM - 1) / gg::BM + E), (unsigned)(N / gg::BN));
  if (hs && row_scale->scalar_type() == at::kBFloat16) {
    static bool a = [&] {
      SXE_HIP_CHECK(hipFuncSetAttribute((const void*)gg::grouped_gemm_kernel<__bf16>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      return true;
    }();
    (void)a;
    hipLaunchKernelGGL(gg::grouped_gemm_kernel<__bf16>, grid, dim3(gg::NTHR), lds, cur_stream(), X, Wp, off, (int)E,
                       reinterpret_cast<const __bf16*>(row_scale->data_ptr()), Yp, (int)R, (int)N, (int)K);
  } else {
    static bool a = [&] {
      SXE_HIP_CHECK(hipFuncSetAttribute((const void*)gg::grouped_gemm_kernel<float>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      return true;
    }();
    (void)a;
    hipLaunchKernelGGL(gg::grouped_gemm_kernel<float>, grid, dim3(gg::NTHR), lds, cur_stream(), X, Wp, off, (int)E,
                       hs ? row_scale->data_ptr<float>() : nullptr, Yp, (int)R, (int)N, (int)K);
  }
  SXE_LAUNCH_CHECK();
  return y;
}

// Mixed-precision experts: wq int8 [E, N, K] or packed int4 [E, N, K / 2] (uint8 storage), ws fp32
// [E, N, K / gs] with gs a multiple of 128 dividing K.
at::Tensor grouped_gemm_q(at::Tensor x, at::Tensor wq, at::Tensor ws, int64_t bits, at::Tensor offsets,
                          c10::optional<at::Tensor> row_scale) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(bits == 8 || bits == 4, "grouped_gemm_q: bits 8 or 4");
  SXE_CHECK(x.dim() == 2 && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "grouped_gemm_q: x [R, K] bf16");
  SXE_CHECK(wq.dim() == 3 && wq.is_contiguous() && (wq.scalar_type() == at::kByte || wq.scalar_type() == at::kChar),
            "grouped_gemm_q: wq [E, N, K * bits / 8] int8 / uint8");
  const int64_t R = x.size(0), K = x.size(1), E = wq.size(0), N = wq.size(1);
  SXE_CHECK(wq.size(2) * 8 == K * bits, "grouped_gemm_q: K mismatch");
  SXE_CHECK(K % gg::BK == 0 && N % gg::BN == 0, "grouped_gemm_q: K and N must be multiples of 128");
  SXE_CHECK(ws.dim() == 3 && ws.is_contiguous() && ws.scalar_type() == at::kFloat && ws.size(0) == E &&
                ws.size(1) == N && ws.size(2) >= 1 && K % ws.size(2) == 0 && (K / ws.size(2)) % gg::BK == 0,
            "grouped_gemm_q: ws fp32 [E, N, K / gs], gs a multiple of 128");
  SXE_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.is_contiguous() &&
                offsets.numel() == E + 1,
            "grouped_gemm_q: offsets int32 [E + 1] on the device");
  SXE_CHECK(wq.is_cuda() && ws.is_cuda(), "grouped_gemm_q: weights on the GPU");
  SXE_CHECK(R + E * gg::BM < (1ll << 31), "grouped_gemm_q: too many rows");
  const bool hs = row_scale.has_value() && row_scale->defined();
  if (hs) {
    SXE_CHECK(row_scale->is_cuda() && row_scale->is_contiguous() && row_scale->numel() == R &&
                  row_scale->scalar_type() == at::kFloat,
              "grouped_gemm_q: row_scale fp32 [R]");
  }
  c10::DeviceGuard guard(x.device());
  auto y = at::empty({R, N}, x.options());
  if (R == 0 || N == 0) return y;
  const int gsb = (int)(K / ws.size(2) / gg::BK);
  const size_t lds = 2 * gg::TILE_BYTES;
  const dim3 grid((unsigned)((R + gg::BM - 1) / gg::BM + E), (unsigned)(N / gg::BN));
  auto X = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto Wp = reinterpret_cast<const uint8_t*>(wq.data_ptr());
  auto Yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  const float* rs = hs ? row_scale->data_ptr<float>() : nullptr;
  auto go = [&](auto kern) {
    SXE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, grid, dim3(gg::NTHR), lds, cur_stream(), X, Wp, ws.data_ptr<float>(), gsb,
                       offsets.data_ptr<int>(), (int)E, rs, Yp, (int)R, (int)N, (int)K);
  };
  if (bits == 8)
    go(gg::grouped_gemm_q_kernel<float, 8>);
  else
    go(gg::grouped_gemm_q_kernel<float, 4>);
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("grouped_gemm(Tensor x, Tensor w, Tensor offsets, Tensor? row_scale=None) -> Tensor");
  m.def("grouped_gemm_q(Tensor x, Tensor wq, Tensor ws, int bits, Tensor offsets, Tensor? row_scale=None) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("grouped_gemm", &sxe::grouped_gemm);
  m.impl("grouped_gemm_q", &sxe::grouped_gemm_q);
}

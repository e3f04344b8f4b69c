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
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // ---- epilogue: lane holds column n of 16 rows per accumulator --------------------------------
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = lo + wm * 64 + i * 32 + acc_row(r, h);
        if (m < hi) {
          float v = acc[i][j][r];
          if (scale) v *= (float)scale[m];
          Y[(int64_t)m * N + n] = f32_to_bf16(v);
        }
      }
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
  const size_t lds = 2 * gg::TILE_BYTES;
  const dim3 grid((unsigned)((R + gg::BM - 1) / gg::BM + E), (unsigned)(N / gg::BN));
  auto X = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto Wp = reinterpret_cast<const unsigned short*>(w.data_ptr());
  auto Yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  const int* off = offsets.data_ptr<int>();
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

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("grouped_gemm(Tensor x, Tensor w, Tensor offsets, Tensor? row_scale=None) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("grouped_gemm", &sxe::grouped_gemm); }

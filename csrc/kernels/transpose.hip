// 16-bit 2-D transpose for gfx950: y[C, R] = x[R, C]^T.
//
// Why: hipBLASLt runs the weight-gradient GEMM dW = dY^T X (both operands token-major, i.e. the
// reduction index is the ROW of both) in its "NT" layout at 1.06-1.19 PF on MI355X, while the same
// product with K-contiguous operands ("TN", the forward layout) runs at 1.47-1.61 PF
// (tools/wgrad_layout_exp.py). Transposing both operands at HBM speed first is cheaper than the
// slow layout for the large MLP projections (ops/linear.py picks per shape).
//
// Geometry: one 256-thread workgroup per 64x64 tile. Load: each thread moves two 16-byte vectors
// (row r = t/4, 16 columns) into an LDS tile with a 66-element (33-dword) row stride, which puts
// the four row groups a wave reads together on distinct banks; store: each thread gathers 16
// elements of one input column and writes two 16-byte vectors of the output row. Grid is
// XCD-agnostic (no inter-tile reuse), ~3x the CU count of tiles for the shapes that matter.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {

constexpr int TT = 64;       // tile edge
constexpr int TLD = TT + 2;  // LDS row stride (elements)

__global__ void __launch_bounds__(256) transpose16_kernel(const unsigned short* __restrict__ x,
                                                          unsigned short* __restrict__ y, int64_t R, int64_t C) {
  __shared__ unsigned short tile[TT * TLD];
  const int64_t tiles_c = C / TT;
  const int64_t tr = blockIdx.x / tiles_c, tc = blockIdx.x - tr * tiles_c;
  const int t = threadIdx.x;
  const int r = t >> 2, c0 = (t & 3) * 16;
  const unsigned short* src = x + (tr * TT + r) * C + tc * TT + c0;
  const u16x8 a = *reinterpret_cast<const u16x8*>(src);
  const u16x8 b = *reinterpret_cast<const u16x8*>(src + 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    tile[r * TLD + c0 + j] = a[j];
    tile[r * TLD + c0 + 8 + j] = b[j];
  }
  __syncthreads();
  // output row = input column (t/4), output columns = input rows (t%4)*16 .. +16
  const int oc = t >> 2, r0 = (t & 3) * 16;
  u16x8 o0, o1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o0[j] = tile[(r0 + j) * TLD + oc];
    o1[j] = tile[(r0 + 8 + j) * TLD + oc];
  }
  unsigned short* dst = y + (tc * TT + oc) * R + tr * TT + r0;
  *reinterpret_cast<u16x8*>(dst) = o0;
  *reinterpret_cast<u16x8*>(dst + 8) = o1;
}

at::Tensor transpose16(at::Tensor x) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.dim() == 2 && x.is_contiguous(), "transpose16: contiguous 2-D input");
  SXE_CHECK(x.element_size() == 2, "transpose16: 16-bit dtype");
  const int64_t R = x.size(0), C = x.size(1);
  SXE_CHECK(R % TT == 0 && C % TT == 0, "transpose16: dims must be multiples of 64");
  c10::DeviceGuard guard(x.device());
  auto y = at::empty({C, R}, x.options());
  const int64_t tiles = (R / TT) * (C / TT);
  if (tiles == 0) return y;
  SXE_CHECK(tiles < (1ll << 31), "transpose16: too many tiles");
  hipLaunchKernelGGL(transpose16_kernel, dim3((unsigned)tiles), dim3(256), 0, cur_stream(),
                     reinterpret_cast<const unsigned short*>(x.data_ptr()),
                     reinterpret_cast<unsigned short*>(y.data_ptr()), R, C);
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) { m.def("transpose16(Tensor x) -> Tensor"); }
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("transpose16", &sxe::transpose16); }

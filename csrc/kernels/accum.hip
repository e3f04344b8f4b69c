// Two-operand gradient accumulate for gfx950: dst(fp32) = [dst +] a(bf16) + b(bf16), one pass.
//
// Why: the MLP / LM-head weight gradients are bf16 TN GEMM outputs added into the ZeRO fp32
// accumulator (ops/mlp.py weight_grad_tn). With gradient accumulation every micro-step paid its
// own pass over the fp32 accumulator: a bf16 -> fp32 copy (6 B/element) on the first and a
// read-modify-write add (10 B/element) on each later one. Keeping the first micro-step's bf16
// product until the next one and folding both into the accumulator here costs 8 B/element for the
// pair (12 with `accumulate`), and the result is bit-identical: (dst + a) + b in fp32, the order
// of the per-micro-step writes.
// Geometry: grid-stride loop, 8 elements per thread per iteration (one 16-byte load of each bf16
// operand, two 16-byte fp32 stores); the tail (n % 8) is handled by scalar lanes.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {

__global__ void __launch_bounds__(256) acc2_bf16_kernel(float* __restrict__ dst, const unsigned short* __restrict__ a,
                                                        const unsigned short* __restrict__ b, int64_t n, int acc) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const u16x8 va = reinterpret_cast<const u16x8*>(a)[i];
    const u16x8 vb = reinterpret_cast<const u16x8*>(b)[i];
    f32x4 lo, hi;
    if (acc) {
      lo = reinterpret_cast<const f32x4*>(dst)[2 * i];
      hi = reinterpret_cast<const f32x4*>(dst)[2 * i + 1];
    } else {
      lo = f32x4{0.f, 0.f, 0.f, 0.f};
      hi = lo;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lo[j] = (lo[j] + bf16_to_f32(va[j])) + bf16_to_f32(vb[j]);
      hi[j] = (hi[j] + bf16_to_f32(va[4 + j])) + bf16_to_f32(vb[4 + j]);
    }
    reinterpret_cast<f32x4*>(dst)[2 * i] = lo;
    reinterpret_cast<f32x4*>(dst)[2 * i + 1] = hi;
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = ((acc ? dst[i] : 0.f) + bf16_to_f32(a[i])) + bf16_to_f32(b[i]);
}

void acc2_bf16_(at::Tensor dst, const at::Tensor& a, const at::Tensor& b, bool accumulate) {
  SXE_CHECK_CUDA(dst);
  SXE_CHECK(dst.is_contiguous() && a.is_contiguous() && b.is_contiguous(), "acc2_bf16_: contiguous operands");
  SXE_CHECK(dst.scalar_type() == at::kFloat && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
            "acc2_bf16_: fp32 dst, bf16 a / b");
  SXE_CHECK(dst.numel() == a.numel() && dst.numel() == b.numel(), "acc2_bf16_: sizes differ");
  SXE_CHECK(reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
            "acc2_bf16_: 16-byte aligned operands");
  const int64_t n = dst.numel();
  if (n == 0) return;
  c10::DeviceGuard guard(dst.device());
  const int64_t blocks = std::min<int64_t>((n / 8 + 255) / 256 + 1, 8 * kNumCUs);
  hipLaunchKernelGGL(acc2_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, cur_stream(), dst.data_ptr<float>(),
                     reinterpret_cast<const unsigned short*>(a.data_ptr()),
                     reinterpret_cast<const unsigned short*>(b.data_ptr()), n, accumulate ? 1 : 0);
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) { m.def("acc2_bf16_(Tensor(a!) dst, Tensor a, Tensor b, bool accumulate) -> ()"); }
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("acc2_bf16_", &sxe::acc2_bf16_); }

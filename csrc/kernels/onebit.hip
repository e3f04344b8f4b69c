// 1-bit compression kernels for the error-compensated compressed all-reduce (1-bit Adam / Lamb,
// 0/1 Adam).
//
// Parity: reference runtime/comm/{nccl,compressed}.py compressed_allreduce + csrc packbits
// (``packbits/unpackbits``, PackbitsBuilder). Fused here:
//   sign_pack_ef_ : x (already error-corrected) -> packed sign bits (LSB first, 8 values per byte),
//                   and the new error  e = x - scale * sign(x)  in the same pass;
//   unpack_avg    : mean over W workers of  scale_w * sign_w  (the server-side average), decoded
//                   straight from the packed bytes -- the reference unpacks to a bool tensor per
//                   worker and reduces in separate launches.
// Each thread owns 8 bytes of packed output (64 values) so the fp32 traffic is 16-byte vectors.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace onebit {

__global__ void sign_pack_ef_kernel(const float* __restrict x, float* __restrict err, const float* __restrict scale,
                                    uint8_t* __restrict packed, int64_t nbytes) {
  const float s = scale[0];
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nbytes; b += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(x + b * 8);
    const f32x4 c = *reinterpret_cast<const f32x4*>(x + b * 8 + 4);
    float v[8] = {a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]};
    uint8_t bits = 0;
    f32x4 e0, e1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool pos = v[j] >= 0.f;
      bits |= (uint8_t)pos << j;
      const float e = v[j] - (pos ? s : -s);
      if (j < 4) e0[j] = e; else e1[j - 4] = e;
    }
    *reinterpret_cast<f32x4*>(err + b * 8) = e0;
    *reinterpret_cast<f32x4*>(err + b * 8 + 4) = e1;
    packed[b] = bits;
  }
}

__global__ void unpack_avg_kernel(const uint8_t* __restrict packed, const float* __restrict scales, int W,
                                  int64_t nbytes, float* __restrict out) {
  const float invW = 1.f / (float)W;
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nbytes; b += (int64_t)gridDim.x * blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < W; ++w) {
      const uint8_t bits = packed[(int64_t)w * nbytes + b];
      const float s = scales[w];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += ((bits >> j) & 1) ? s : -s;
    }
    f32x4 o0 = {acc[0] * invW, acc[1] * invW, acc[2] * invW, acc[3] * invW};
    f32x4 o1 = {acc[4] * invW, acc[5] * invW, acc[6] * invW, acc[7] * invW};
    *reinterpret_cast<f32x4*>(out + b * 8) = o0;
    *reinterpret_cast<f32x4*>(out + b * 8 + 4) = o1;
  }
}

}  // namespace onebit

// x, err: fp32 [n] (n % 8 == 0); scale: fp32 [1]; packed: uint8 [n / 8]
void sign_pack_ef_(const at::Tensor& x, at::Tensor err, const at::Tensor& scale, at::Tensor packed) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.scalar_type() == at::kFloat && err.scalar_type() == at::kFloat && x.is_contiguous() &&
                err.is_contiguous(), "fp32 contiguous");
  SXE_CHECK(x.numel() % 8 == 0 && err.numel() == x.numel() && packed.numel() * 8 == x.numel() &&
                packed.scalar_type() == at::kByte, "sizes");
  c10::DeviceGuard g(x.device());
  const int64_t nb = packed.numel();
  if (nb == 0) return;
  hipLaunchKernelGGL(onebit::sign_pack_ef_kernel, dim3(stream_grid(nb, 256)), dim3(256), 0, cur_stream(),
                     x.data_ptr<float>(), err.data_ptr<float>(), scale.data_ptr<float>(), packed.data_ptr<uint8_t>(), nb);
  SXE_LAUNCH_CHECK();
}

// packed: uint8 [W, m / 8]; scales: fp32 [W]; out: fp32 [m]
void unpack_avg(const at::Tensor& packed, const at::Tensor& scales, at::Tensor out) {
  SXE_CHECK_CUDA(packed);
  SXE_CHECK(packed.dim() == 2 && packed.is_contiguous() && packed.scalar_type() == at::kByte, "packed [W, m/8]");
  SXE_CHECK(scales.numel() == packed.size(0) && out.numel() == packed.size(1) * 8 && out.is_contiguous(), "sizes");
  c10::DeviceGuard g(packed.device());
  const int64_t nb = packed.size(1);
  if (nb == 0) return;
  hipLaunchKernelGGL(onebit::unpack_avg_kernel, dim3(stream_grid(nb, 256)), dim3(256), 0, cur_stream(),
                     packed.data_ptr<uint8_t>(), scales.data_ptr<float>(), (int)packed.size(0), nb, out.data_ptr<float>());
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("sign_pack_ef_(Tensor x, Tensor(a!) err, Tensor scale, Tensor(b!) packed) -> ()");
  m.def("unpack_avg(Tensor packed, Tensor scales, Tensor(a!) out) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("sign_pack_ef_", &sxe::sign_pack_ef_);
  m.impl("unpack_avg", &sxe::unpack_avg);
}

// Group-wise quantization kernels (ZeRO++ quantized weights / gradients, MoQ, FP8 quantizer).
//
// Parity: reference csrc/quantization (``quantize`` / ``dequantize`` / ``swizzle_quant`` /
// ``quantized_reduction``, symmetric int8 / int4) and ops/fp_quantizer (FP8 e4m3 with per-group
// scales). MI355X design:
//  * one wave per quantization group (group sizes are multiples of 64): a lane handles
//    group/64 contiguous values, the absmax is a wave butterfly, no LDS;
//  * int4 packs two values per byte (low nibble first), int8 as-is, scales fp32 per group;
//  * FP8 e4m3 conversion uses CDNA4's hardware converters (v_cvt_pk_fp8_f32 via the
//    __builtin_amdgcn_cvt_pk_fp8_f32 builtin, OCP e4m3 on gfx950) and v_cvt_f32_fp8 back;
//  * dequant_reduce fuses the qgZ receive side: W quantized chunks -> fp32 sum in one pass.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace quant {

template <DT T, int BITS>
__global__ void quant_kernel(const typename dt_traits<T>::storage* __restrict x, int64_t n_groups, int group,
                             uint8_t* __restrict q, float* __restrict scales) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int per = group / 64;
  constexpr float qmax = BITS == 8 ? 127.f : 7.f;
  for (int64_t gi = wid; gi < n_groups; gi += nw) {
    const typename dt_traits<T>::storage* src = x + gi * group + lane * per;
    float m = 0.f;
    for (int i = 0; i < per; ++i) m = fmaxf(m, fabsf(to_f32<T>(src[i])));
    m = wave_max(m);
    const float s = m > 0.f ? m / qmax : 1.f;
    const float inv = 1.f / s;
    if (lane == 0) scales[gi] = s;
    if constexpr (BITS == 8) {
      int8_t* dst = reinterpret_cast<int8_t*>(q) + gi * group + lane * per;
      for (int i = 0; i < per; ++i) dst[i] = (int8_t)fmaxf(-qmax, fminf(qmax, rintf(to_f32<T>(src[i]) * inv)));
    } else {
      uint8_t* dst = q + (gi * group + lane * per) / 2;
      for (int i = 0; i < per; i += 2) {
        const int a = (int)fmaxf(-qmax, fminf(qmax, rintf(to_f32<T>(src[i]) * inv)));
        const int b = (int)fmaxf(-qmax, fminf(qmax, rintf(to_f32<T>(src[i + 1]) * inv)));
        dst[i / 2] = (uint8_t)((a & 0xF) | ((b & 0xF) << 4));
      }
    }
  }
}

template <DT T, int BITS>
__global__ void dequant_kernel(const uint8_t* __restrict q, const float* __restrict scales, int64_t n, int group,
                               typename dt_traits<T>::storage* __restrict out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float s = scales[i / group];
    float v;
    if constexpr (BITS == 8) {
      v = (float)reinterpret_cast<const int8_t*>(q)[i];
    } else {
      const uint8_t b = q[i >> 1];
      int nib = (i & 1) ? (b >> 4) : (b & 0xF);
      if (nib & 0x8) nib -= 16;
      v = (float)nib;
    }
    out[i] = from_f32<T>(v * s);
  }
}

// q: [W, m] quantized chunks (m values each), scales: [W, m / group]; out fp32 [m] = sum_w deq_w
template <int BITS>
__global__ void dequant_reduce_kernel(const uint8_t* __restrict q, const float* __restrict scales, int W, int64_t m,
                                      int group, float* __restrict out, float alpha, bool accumulate) {
  const int64_t bytes_per = BITS == 8 ? m : m / 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int w = 0; w < W; ++w) {
      const float s = scales[(int64_t)w * (m / group) + i / group];
      float v;
      if constexpr (BITS == 8) {
        v = (float)reinterpret_cast<const int8_t*>(q)[(int64_t)w * bytes_per + i];
      } else {
        const uint8_t b = q[(int64_t)w * bytes_per + (i >> 1)];
        int nib = (i & 1) ? (b >> 4) : (b & 0xF);
        if (nib & 0x8) nib -= 16;
        v = (float)nib;
      }
      acc += v * s;
    }
    out[i] = accumulate ? out[i] + alpha * acc : alpha * acc;
  }
}

// ---- FP8 e4m3 (OCP on gfx950) ---------------------------------------------------------------
template <DT T>
__global__ void fp8_quant_kernel(const typename dt_traits<T>::storage* __restrict x, int64_t n_groups, int group,
                                 uint8_t* __restrict q, float* __restrict scales) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int per = group / 64;
  constexpr float fmax8 = 448.f;
  for (int64_t gi = wid; gi < n_groups; gi += nw) {
    const typename dt_traits<T>::storage* src = x + gi * group + lane * per;
    float m = 0.f;
    for (int i = 0; i < per; ++i) m = fmaxf(m, fabsf(to_f32<T>(src[i])));
    m = wave_max(m);
    const float s = m > 0.f ? m / fmax8 : 1.f;
    const float inv = 1.f / s;
    if (lane == 0) scales[gi] = s;
    uint8_t* dst = q + gi * group + lane * per;
    for (int i = 0; i < per; i += 2) {
      const float a = fmaxf(-fmax8, fminf(fmax8, to_f32<T>(src[i]) * inv));
      const float b = fmaxf(-fmax8, fminf(fmax8, to_f32<T>(src[i + 1]) * inv));
      const int packed = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
      dst[i] = (uint8_t)(packed & 0xFF);
      dst[i + 1] = (uint8_t)((packed >> 8) & 0xFF);
    }
  }
}

template <DT T>
__global__ void fp8_dequant_kernel(const uint8_t* __restrict q, const float* __restrict scales, int64_t n, int group,
                                   typename dt_traits<T>::storage* __restrict out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = __builtin_amdgcn_cvt_f32_fp8((int)q[i], 0);
    out[i] = from_f32<T>(v * scales[i / group]);
  }
}

}  // namespace quant

static void check_group(const at::Tensor& x, int64_t group) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.is_contiguous(), "contiguous input");
  SXE_CHECK(group % 64 == 0 && group > 0, "group size must be a positive multiple of 64");
  SXE_CHECK(x.numel() % group == 0, "numel must be a multiple of the group size");
}

// bits in {4, 8}: returns [q (uint8/int8 storage), scales fp32 [numel / group]]
std::vector<at::Tensor> quantize_sym(const at::Tensor& x, int64_t group, int64_t bits) {
  check_group(x, group);
  SXE_CHECK(bits == 8 || bits == 4, "bits must be 4 or 8");
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel(), ng = n / group;
  auto q = at::empty({bits == 8 ? n : n / 2}, x.options().dtype(at::kByte));
  auto s = at::empty({ng}, x.options().dtype(at::kFloat));
  if (n == 0) return {q, s};
  const int blocks = stream_grid(ng * 64, 256);
  SXE_DISPATCH_DT(dtype_of(x), T, {
    using st = typename dt_traits<T>::storage;
    if (bits == 8)
      hipLaunchKernelGGL((quant::quant_kernel<T, 8>), dim3(blocks), dim3(256), 0, cur_stream(),
                         reinterpret_cast<const st*>(x.data_ptr()), ng, (int)group, q.data_ptr<uint8_t>(), s.data_ptr<float>());
    else
      hipLaunchKernelGGL((quant::quant_kernel<T, 4>), dim3(blocks), dim3(256), 0, cur_stream(),
                         reinterpret_cast<const st*>(x.data_ptr()), ng, (int)group, q.data_ptr<uint8_t>(), s.data_ptr<float>());
  });
  SXE_LAUNCH_CHECK();
  return {q, s};
}

void dequantize_sym_(const at::Tensor& q, const at::Tensor& scales, int64_t group, int64_t bits, at::Tensor out) {
  SXE_CHECK_CUDA(q);
  SXE_CHECK(out.is_contiguous() && (bits == 8 || bits == 4), "bad args");
  c10::DeviceGuard g(q.device());
  const int64_t n = out.numel();
  SXE_CHECK(scales.numel() * group == n && q.numel() == (bits == 8 ? n : n / 2), "size mismatch");
  if (n == 0) return;
  SXE_DISPATCH_DT(dtype_of(out), T, {
    using st = typename dt_traits<T>::storage;
    if (bits == 8)
      hipLaunchKernelGGL((quant::dequant_kernel<T, 8>), dim3(stream_grid(n, 256)), dim3(256), 0, cur_stream(),
                         q.data_ptr<uint8_t>(), scales.data_ptr<float>(), n, (int)group, reinterpret_cast<st*>(out.data_ptr()));
    else
      hipLaunchKernelGGL((quant::dequant_kernel<T, 4>), dim3(stream_grid(n, 256)), dim3(256), 0, cur_stream(),
                         q.data_ptr<uint8_t>(), scales.data_ptr<float>(), n, (int)group, reinterpret_cast<st*>(out.data_ptr()));
  });
  SXE_LAUNCH_CHECK();
}

// q: [W * bytes(m)] chunks of m values, scales [W * m / group]; out fp32 [m] (+)= alpha * sum_w
void dequant_reduce_(const at::Tensor& q, const at::Tensor& scales, int64_t W, int64_t group, int64_t bits,
                     at::Tensor out, double alpha, bool accumulate) {
  SXE_CHECK_CUDA(q);
  SXE_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous(), "out fp32");
  c10::DeviceGuard g(q.device());
  const int64_t m = out.numel();
  SXE_CHECK(scales.numel() == W * (m / group) && m % group == 0, "scales size");
  if (m == 0) return;
  if (bits == 8)
    hipLaunchKernelGGL(quant::dequant_reduce_kernel<8>, dim3(stream_grid(m, 256)), dim3(256), 0, cur_stream(),
                       q.data_ptr<uint8_t>(), scales.data_ptr<float>(), (int)W, m, (int)group, out.data_ptr<float>(),
                       (float)alpha, accumulate);
  else
    hipLaunchKernelGGL(quant::dequant_reduce_kernel<4>, dim3(stream_grid(m, 256)), dim3(256), 0, cur_stream(),
                       q.data_ptr<uint8_t>(), scales.data_ptr<float>(), (int)W, m, (int)group, out.data_ptr<float>(),
                       (float)alpha, accumulate);
  SXE_LAUNCH_CHECK();
}

std::vector<at::Tensor> quantize_fp8(const at::Tensor& x, int64_t group) {
  check_group(x, group);
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel(), ng = n / group;
  auto q = at::empty({n}, x.options().dtype(at::kByte));
  auto s = at::empty({ng}, x.options().dtype(at::kFloat));
  if (n == 0) return {q, s};
  SXE_DISPATCH_DT(dtype_of(x), T, {
    using st = typename dt_traits<T>::storage;
    hipLaunchKernelGGL((quant::fp8_quant_kernel<T>), dim3(stream_grid(ng * 64, 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const st*>(x.data_ptr()), ng, (int)group, q.data_ptr<uint8_t>(), s.data_ptr<float>());
  });
  SXE_LAUNCH_CHECK();
  return {q, s};
}

void dequantize_fp8_(const at::Tensor& q, const at::Tensor& scales, int64_t group, at::Tensor out) {
  SXE_CHECK_CUDA(q);
  c10::DeviceGuard g(q.device());
  const int64_t n = out.numel();
  SXE_CHECK(q.numel() == n && scales.numel() * group == n && out.is_contiguous(), "size mismatch");
  if (n == 0) return;
  SXE_DISPATCH_DT(dtype_of(out), T, {
    using st = typename dt_traits<T>::storage;
    hipLaunchKernelGGL((quant::fp8_dequant_kernel<T>), dim3(stream_grid(n, 256)), dim3(256), 0, cur_stream(),
                       q.data_ptr<uint8_t>(), scales.data_ptr<float>(), n, (int)group, reinterpret_cast<st*>(out.data_ptr()));
  });
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("quantize_sym(Tensor x, int group, int bits) -> Tensor[]");
  m.def("dequantize_sym_(Tensor q, Tensor scales, int group, int bits, Tensor(a!) out) -> ()");
  m.def("dequant_reduce_(Tensor q, Tensor scales, int W, int group, int bits, Tensor(a!) out, float alpha, "
        "bool accumulate) -> ()");
  m.def("quantize_fp8(Tensor x, int group) -> Tensor[]");
  m.def("dequantize_fp8_(Tensor q, Tensor scales, int group, Tensor(a!) out) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("quantize_sym", &sxe::quantize_sym);
  m.impl("dequantize_sym_", &sxe::dequantize_sym_);
  m.impl("dequant_reduce_", &sxe::dequant_reduce_);
  m.impl("quantize_fp8", &sxe::quantize_fp8);
  m.impl("dequantize_fp8_", &sxe::dequantize_fp8_);
}

// Activation kernels for gfx950: SwiGLU/GeGLU (gated, concatenated [gate | up] layout) and
// bias + activation (GELU-tanh / exact GELU / ReLU / SiLU / identity), forward and backward.
//
// Reference semantics: core_ops/bias_activations/bias_activation_cuda.cu:17-51 (in-place
// act(x + b)) and core_ops/gated_activations/gated_activation_kernels_cuda.cu:45 (gated act).
// Differences, MI355X-first: the training path stores the gate/up projection as ONE GEMM output
// [T, 2I] = [gate | up] (one hipBLASLt call with N = 2I instead of two), so the gated kernel
// reads two 16-byte vectors at a fixed I offset instead of the reference's interleaved pairs.
// Every lane moves 16 B per access; the grid is capped at 256 CUs x 8 blocks and grid-strides.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {

enum Act : int { ACT_IDENTITY = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_SILU = 3, ACT_GELU_ERF = 4, ACT_QUICK_GELU = 5 };

__device__ __forceinline__ float act_f(float x, int act) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_GELU: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float t = tanhf(k0 * (x + k1 * x * x * x));
      return 0.5f * x * (1.f + t);
    }
    case ACT_SILU: return x / (1.f + __expf(-x));
    case ACT_GELU_ERF: return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
    case ACT_QUICK_GELU: return x / (1.f + __expf(-1.702f * x));  // CLIP
    default: return x;
  }
}
__device__ __forceinline__ float act_df(float x, int act) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_GELU: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float u = k0 * (x + k1 * x * x * x);
      float t = tanhf(u);
      float du = k0 * (1.f + 3.f * k1 * x * x);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
    }
    case ACT_SILU: {
      float s = 1.f / (1.f + __expf(-x));
      return s * (1.f + x * (1.f - s));
    }
    case ACT_GELU_ERF: {
      const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
      return cdf + x * 0.3989422804014327f * __expf(-0.5f * x * x);
    }
    case ACT_QUICK_GELU: {
      const float sg = 1.f / (1.f + __expf(-1.702f * x));
      return sg + 1.702f * x * sg * (1.f - sg);
    }
    default: return 1.f;
  }
}

// gated: out[t, j] = act(gu[t, j]) * gu[t, I + j]
template <DT T>
__global__ void __launch_bounds__(256) gated_fwd_kernel(const typename dt_traits<T>::storage* __restrict__ gu,
                                                        typename dt_traits<T>::storage* __restrict__ out, int64_t rows,
                                                        int I, int act) {
  const int per_row = I / 8;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x)
  for (int cc = threadIdx.x; cc < per_row; cc += blockDim.x) {
    const int c = cc * 8;
    float g[8], u[8], o[8];
    load8<T>(gu + r * 2 * I + c, g);
    load8<T>(gu + r * 2 * I + I + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_f(g[j], act) * u[j];
    store8<T>(out + r * I + c, o);
  }
}

template <DT T>
__global__ void __launch_bounds__(256) gated_bwd_kernel(const typename dt_traits<T>::storage* __restrict__ dout,
                                                        const typename dt_traits<T>::storage* __restrict__ gu,
                                                        typename dt_traits<T>::storage* __restrict__ dgu, int64_t rows,
                                                        int I, int act) {
  const int per_row = I / 8;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x)
  for (int cc = threadIdx.x; cc < per_row; cc += blockDim.x) {
    const int c = cc * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    load8<T>(gu + r * 2 * I + c, g);
    load8<T>(gu + r * 2 * I + I + c, u);
    load8<T>(dout + r * I + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      du[j] = d[j] * act_f(g[j], act);
      dg[j] = d[j] * u[j] * act_df(g[j], act);
    }
    store8<T>(dgu + r * 2 * I + c, dg);
    store8<T>(dgu + r * 2 * I + I + c, du);
  }
}

at::Tensor gated_act_fwd(at::Tensor gu, int64_t act) {
  SXE_CHECK(gu.is_contiguous(), "gated_act_fwd: contiguous");
  const int64_t two_i = gu.size(-1);
  SXE_CHECK(two_i % 16 == 0, "gated_act_fwd: inner size must be a multiple of 16");
  const int I = (int)(two_i / 2);
  const int64_t rows = gu.numel() / two_i;
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  c10::DeviceGuard guard(gu.device());
  auto out = at::empty(sizes, gu.options());
  if (rows == 0) return out;
  DT d = dtype_of(gu);
  SXE_DISPATCH_DT(d, TT, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((gated_fwd_kernel<TT>), dim3((int)std::min<int64_t>(rows, 4096)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(gu.data_ptr()), reinterpret_cast<S*>(out.data_ptr()), rows, I, (int)act);
  });
  SXE_LAUNCH_CHECK();
  return out;
}

at::Tensor gated_act_bwd(at::Tensor dout, at::Tensor gu, int64_t act) {
  SXE_CHECK(gu.is_contiguous() && dout.is_contiguous(), "gated_act_bwd: contiguous");
  const int64_t two_i = gu.size(-1);
  const int I = (int)(two_i / 2);
  const int64_t rows = gu.numel() / two_i;
  SXE_CHECK(dout.numel() == rows * I, "gated_act_bwd: shape");
  c10::DeviceGuard guard(gu.device());
  auto dgu = at::empty_like(gu);
  if (rows == 0) return dgu;
  DT d = dtype_of(gu);
  SXE_DISPATCH_DT(d, TT, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((gated_bwd_kernel<TT>), dim3((int)std::min<int64_t>(rows, 4096)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(dout.data_ptr()), reinterpret_cast<const S*>(gu.data_ptr()),
                       reinterpret_cast<S*>(dgu.data_ptr()), rows, I, (int)act);
  });
  SXE_LAUNCH_CHECK();
  return dgu;
}

// y = act(x + b) ; b broadcast over rows (optional)
template <DT T>
__global__ void __launch_bounds__(256) bias_act_fwd_kernel(const typename dt_traits<T>::storage* __restrict__ x,
                                                           const typename dt_traits<T>::storage* __restrict__ b,
                                                           typename dt_traits<T>::storage* __restrict__ y, int64_t n,
                                                           int C, int act) {
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8], bv[8];
    load8<T>(x + i * 8, v);
    if (b) {
      load8<T>(b + (int)((i * 8) % C), bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bv[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_f(v[j], act);
    store8<T>(y + i * 8, v);
  }
}

template <DT T>
__global__ void __launch_bounds__(256) bias_act_bwd_kernel(const typename dt_traits<T>::storage* __restrict__ dy,
                                                           const typename dt_traits<T>::storage* __restrict__ x,
                                                           const typename dt_traits<T>::storage* __restrict__ b,
                                                           typename dt_traits<T>::storage* __restrict__ dx, int64_t n,
                                                           int C, int act) {
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8], d[8], bv[8];
    load8<T>(x + i * 8, v);
    load8<T>(dy + i * 8, d);
    if (b) {
      load8<T>(b + (int)((i * 8) % C), bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bv[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= act_df(v[j], act);
    store8<T>(dx + i * 8, d);
  }
}

at::Tensor bias_act_fwd(at::Tensor x, c10::optional<at::Tensor> bias, int64_t act) {
  SXE_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "bias_act_fwd: contiguous, numel % 8 == 0");
  const int C = (int)x.size(-1);
  SXE_CHECK(C % 8 == 0, "bias_act_fwd: channels % 8");
  const bool hb = bias.has_value() && bias->defined();
  if (hb) SXE_CHECK(bias->numel() == C && bias->scalar_type() == x.scalar_type(), "bias_act_fwd: bias");
  c10::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  const int64_t n = x.numel();
  if (n == 0) return y;
  DT d = dtype_of(x);
  SXE_DISPATCH_DT(d, TT, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((bias_act_fwd_kernel<TT>), dim3(stream_grid(n / 8, 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(x.data_ptr()), hb ? reinterpret_cast<const S*>(bias->data_ptr()) : nullptr,
                       reinterpret_cast<S*>(y.data_ptr()), n, C, (int)act);
  });
  SXE_LAUNCH_CHECK();
  return y;
}

at::Tensor bias_act_bwd(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> bias, int64_t act) {
  SXE_CHECK(x.is_contiguous() && dy.is_contiguous() && dy.sizes() == x.sizes(), "bias_act_bwd: shapes");
  const int C = (int)x.size(-1);
  const bool hb = bias.has_value() && bias->defined();
  c10::DeviceGuard guard(x.device());
  auto dx = at::empty_like(x);
  const int64_t n = x.numel();
  if (n == 0) return dx;
  DT d = dtype_of(x);
  SXE_DISPATCH_DT(d, TT, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((bias_act_bwd_kernel<TT>), dim3(stream_grid(n / 8, 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(dy.data_ptr()), reinterpret_cast<const S*>(x.data_ptr()),
                       hb ? reinterpret_cast<const S*>(bias->data_ptr()) : nullptr, reinterpret_cast<S*>(dx.data_ptr()),
                       n, C, (int)act);
  });
  SXE_LAUNCH_CHECK();
  return dx;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("gated_act_fwd(Tensor gu, int act) -> Tensor");
  m.def("gated_act_bwd(Tensor dout, Tensor gu, int act) -> Tensor");
  m.def("bias_act_fwd(Tensor x, Tensor? bias, int act) -> Tensor");
  m.def("bias_act_bwd(Tensor dy, Tensor x, Tensor? bias, int act) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("gated_act_fwd", &sxe::gated_act_fwd);
  m.impl("gated_act_bwd", &sxe::gated_act_bwd);
  m.impl("bias_act_fwd", &sxe::bias_act_fwd);
  m.impl("bias_act_bwd", &sxe::bias_act_bwd);
}

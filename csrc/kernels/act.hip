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
  // flat over (row, 8-column chunk): a single decode row spreads over I/8/256 blocks instead of
  // one block looping over the whole row
  const int per_row = I / 8;
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per_row;
    const int c = (int)(i - r * per_row) * 8;
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
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per_row;
    const int c = (int)(i - r * per_row) * 8;
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
    hipLaunchKernelGGL((gated_fwd_kernel<TT>), dim3(stream_grid(rows * (I / 8), 256)), dim3(256), 0, cur_stream(),
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
    hipLaunchKernelGGL((gated_bwd_kernel<TT>), dim3(stream_grid(rows * (I / 8), 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(dout.data_ptr()), reinterpret_cast<const S*>(gu.data_ptr()),
                       reinterpret_cast<S*>(dgu.data_ptr()), rows, I, (int)act);
  });
  SXE_LAUNCH_CHECK();
  return dgu;
}

// ---------------------------------------------------------------------------------------------
// Dual-layout gated kernels (bf16): the token-major result PLUS a token-minor (transposed) copy,
// so the MLP's weight-gradient GEMMs dW = dY^T X get both operands K-contiguous -- hipBLASLt's
// fast "TN" layout (1.34-1.48 PF vs 1.06-1.18 PF for the k-strided product at 16k tokens,
// tools/wgrad_tn16k_exp.py) -- without a separate transpose pass over HBM (the transposed tile is
// written from LDS while the token-major tile is still in registers).
//   fwd: out[t, j] = act(gu[t, j]) * gu[t, I + j]; outT[j, t] = out[t, j]
//   bwd: dgu[t, j] = d * u * act'(g), dgu[t, I + j] = d * act(g); dguT = dgu^T   (d = dout[t, j])
// Geometry (template TR tokens x TC columns per workgroup, TR*TC/16 threads): thread t loads
// row t/(TC/16), 16 columns from (t%(TC/16))*16 as two 16-byte vectors per operand (TC*2-byte row
// segments), and stores 16 tokens of one output column as two 16-byte vectors of the transposed
// row (TR*2-byte segments). LDS rows are padded by 2 elements (an odd dword stride) so the
// column-wise reads of a wave spread over the banks. The variant is
// chosen per intermediate size by ops/mlp.py (64 x 256 where it divides: 5.0-5.2 TB/s vs 4.1 for
// 64 x 64 at 16k tokens x 14336, profiles/act_layout_exp.log); the others remain for A/B.
__device__ __forceinline__ void ld16(const unsigned short* p, float (&v)[16]) {
  const u16x8 a = *reinterpret_cast<const u16x8*>(p), b = *reinterpret_cast<const u16x8*>(p + 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = bf16_to_f32(a[j]);
    v[8 + j] = bf16_to_f32(b[j]);
  }
}

// token-major store of 16 values + their copy into the LDS tile row (as 8 dword writes)
__device__ __forceinline__ void st16(unsigned short* p, unsigned short* lds_row, const float (&v)[16]) {
  u16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = f32_to_bf16(v[j]);
    b[j] = f32_to_bf16(v[8 + j]);
  }
  *reinterpret_cast<u16x8*>(p) = a;
  *reinterpret_cast<u16x8*>(p + 8) = b;
  unsigned* l = reinterpret_cast<unsigned*>(lds_row);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    l[j] = (unsigned)a[2 * j] | ((unsigned)a[2 * j + 1] << 16);
    l[4 + j] = (unsigned)b[2 * j] | ((unsigned)b[2 * j + 1] << 16);
  }
}

// transposed store of one LDS tile: output row = tile column t/(TR/16), 16 tokens from
// (t%(TR/16))*16
template <int TR, int LD>
__device__ __forceinline__ void st_t(const unsigned short* tile, unsigned short* dstT, int64_t T) {
  const int t = threadIdx.x, oc = t / (TR / 16), r0 = (t % (TR / 16)) * 16;
  u16x8 o0, o1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o0[j] = tile[(r0 + j) * LD + oc];
    o1[j] = tile[(r0 + 8 + j) * LD + oc];
  }
  unsigned short* d = dstT + (int64_t)oc * T + r0;
  *reinterpret_cast<u16x8*>(d) = o0;
  *reinterpret_cast<u16x8*>(d + 8) = o1;
}

template <bool BWD, int TR, int TC>
__global__ void __launch_bounds__(TR * TC / 16) gated_dual_kernel(const unsigned short* __restrict__ gu,
                                                                  const unsigned short* __restrict__ dout,
                                                                  unsigned short* __restrict__ out,
                                                                  unsigned short* __restrict__ outT, int64_t T,
                                                                  int I, int act) {
  constexpr int LD = TC + 2;
  __shared__ __attribute__((aligned(16))) unsigned short tile[BWD ? 2 : 1][TR * LD];
  const int tiles_c = I / TC;
  const int64_t tr = blockIdx.x / tiles_c;
  const int tc = (int)(blockIdx.x - tr * tiles_c);
  const int t = threadIdx.x, r = t / (TC / 16), c0 = (t % (TC / 16)) * 16;
  const int64_t row = tr * TR + r;
  const int col = tc * TC + c0;
  float g[16], u[16];
  ld16(gu + row * 2 * I + col, g);
  ld16(gu + row * 2 * I + I + col, u);
  if constexpr (!BWD) {
    float o[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) o[j] = act_f(g[j], act) * u[j];
    st16(out + row * I + col, &tile[0][r * LD + c0], o);
    __syncthreads();
    st_t<TR, LD>(tile[0], outT + (int64_t)(tc * TC) * T + tr * TR, T);
  } else {
    float d[16], dg[16], du[16];
    ld16(dout + row * I + col, d);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      du[j] = d[j] * act_f(g[j], act);
      dg[j] = d[j] * u[j] * act_df(g[j], act);
    }
    st16(out + row * 2 * I + col, &tile[0][r * LD + c0], dg);
    st16(out + row * 2 * I + I + col, &tile[1][r * LD + c0], du);
    __syncthreads();
    st_t<TR, LD>(tile[0], outT + (int64_t)(tc * TC) * T + tr * TR, T);
    st_t<TR, LD>(tile[1], outT + (int64_t)(I + tc * TC) * T + tr * TR, T);
  }
}

// variant -> (TR, TC): 0 = 64 x 64, 1 = 64 x 128, 2 = 128 x 64, 3 = 128 x 128, 4 = 64 x 256
static void dual_tile(int64_t variant, int& TR, int& TC) {
  SXE_CHECK(variant >= 0 && variant <= 4, "gated dual: variant must be 0..4");
  TR = (variant == 2 || variant == 3) ? 128 : 64;
  TC = variant == 4 ? 256 : (variant & 1) ? 128 : 64;
}

static void check_dual(const at::Tensor& gu, int TR, int TC, int64_t& T, int& I) {
  SXE_CHECK_CUDA(gu);
  SXE_CHECK(gu.is_contiguous() && gu.scalar_type() == at::kBFloat16, "gated dual: contiguous bf16 gate|up");
  const int64_t two_i = gu.size(-1);
  I = (int)(two_i / 2);
  T = gu.numel() / two_i;
  SXE_CHECK(T % TR == 0 && I % TC == 0, "gated dual: tokens / intermediate size must be multiples of the tile (",
            TR, " x ", TC, ")");
  SXE_CHECK((T / TR) * (I / TC) < (1ll << 31), "gated dual: too many tiles");
}

template <bool BWD>
static void launch_dual(int TR, int TC, const unsigned short* gu, const unsigned short* dout, unsigned short* out,
                        unsigned short* outT, int64_t T, int I, int act) {
  const dim3 grid((unsigned)((T / TR) * (I / TC)));
  hipStream_t s = cur_stream();
  if (TR == 64 && TC == 64)
    hipLaunchKernelGGL((gated_dual_kernel<BWD, 64, 64>), grid, dim3(256), 0, s, gu, dout, out, outT, T, I, act);
  else if (TR == 64 && TC == 256)
    hipLaunchKernelGGL((gated_dual_kernel<BWD, 64, 256>), grid, dim3(1024), 0, s, gu, dout, out, outT, T, I, act);
  else if (TR == 64)
    hipLaunchKernelGGL((gated_dual_kernel<BWD, 64, 128>), grid, dim3(512), 0, s, gu, dout, out, outT, T, I, act);
  else if (TC == 64)
    hipLaunchKernelGGL((gated_dual_kernel<BWD, 128, 64>), grid, dim3(512), 0, s, gu, dout, out, outT, T, I, act);
  else
    hipLaunchKernelGGL((gated_dual_kernel<BWD, 128, 128>), grid, dim3(1024), 0, s, gu, dout, out, outT, T, I, act);
  SXE_LAUNCH_CHECK();
}

// -> (out [..., I], outT [I, T])
std::tuple<at::Tensor, at::Tensor> gated_act_fwd_dual(at::Tensor gu, int64_t act, int64_t variant) {
  int TR, TC, I;
  int64_t T;
  dual_tile(variant, TR, TC);
  check_dual(gu, TR, TC, T, I);
  c10::DeviceGuard guard(gu.device());
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  auto out = at::empty(sizes, gu.options());
  auto outT = at::empty({I, T}, gu.options());
  if (T == 0) return {out, outT};
  launch_dual<false>(TR, TC, reinterpret_cast<const unsigned short*>(gu.data_ptr()), nullptr,
                     reinterpret_cast<unsigned short*>(out.data_ptr()), reinterpret_cast<unsigned short*>(outT.data_ptr()),
                     T, I, (int)act);
  return {out, outT};
}

// -> (dgu [..., 2I], dguT [2I, T])
std::tuple<at::Tensor, at::Tensor> gated_act_bwd_dual(at::Tensor dout, at::Tensor gu, int64_t act, int64_t variant) {
  int TR, TC, I;
  int64_t T;
  dual_tile(variant, TR, TC);
  check_dual(gu, TR, TC, T, I);
  SXE_CHECK(dout.is_contiguous() && dout.scalar_type() == at::kBFloat16 && dout.numel() == T * I,
            "gated dual bwd: dout shape");
  c10::DeviceGuard guard(gu.device());
  auto dgu = at::empty_like(gu);
  auto dguT = at::empty({2 * (int64_t)I, T}, gu.options());
  if (T == 0) return {dgu, dguT};
  launch_dual<true>(TR, TC, reinterpret_cast<const unsigned short*>(gu.data_ptr()),
                    reinterpret_cast<const unsigned short*>(dout.data_ptr()),
                    reinterpret_cast<unsigned short*>(dgu.data_ptr()), reinterpret_cast<unsigned short*>(dguT.data_ptr()),
                    T, I, (int)act);
  return {dgu, dguT};
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
  m.def("gated_act_fwd_dual(Tensor gu, int act, int variant=0) -> (Tensor, Tensor)");
  m.def("gated_act_bwd_dual(Tensor dout, Tensor gu, int act, int variant=0) -> (Tensor, Tensor)");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("gated_act_fwd_dual", &sxe::gated_act_fwd_dual);
  m.impl("gated_act_bwd_dual", &sxe::gated_act_bwd_dual);
  m.impl("gated_act_fwd", &sxe::gated_act_fwd);
  m.impl("gated_act_bwd", &sxe::gated_act_bwd);
  m.impl("bias_act_fwd", &sxe::bias_act_fwd);
  m.impl("bias_act_bwd", &sxe::bias_act_bwd);
}

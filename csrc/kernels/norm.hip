// RMSNorm / LayerNorm forward + backward for gfx950, with the residual add fused in.
//
// Semantics match the reference's inference kernels (rms_norm / pre_rms_norm in
// deepspeed/inference/v2/kernels/core_ops/cuda_rms_norm/rms_norm_cuda.cu:19,84 and fused_ln /
// fused_residual_ln in core_ops/cuda_layer_norm/layer_norm_cuda.cu:31,220) but this file is a
// training kernel set (forward saves rstd/mean, backward produces dx, dgamma, dbeta).
//
// MI355X mapping: ONE WAVE PER ROW (no __syncthreads on the row path). A lane owns NCH chunks of
// 8 contiguous elements (16-byte loads) at stride 512 elements, so a 4096-wide bf16 row is one
// 8-KiB coalesced sweep held entirely in registers (NCH = 8 -> 64 fp32 values per lane). dgamma
// and dbeta are accumulated per wave in registers across all rows the wave visits, reduced across
// the block's 4 waves in LDS and written as one fp32 partial row per block; the caller sums the
// (grid x H) partial matrix (a single small reduction instead of per-row atomics).
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {

template <DT T, bool WF32>
struct WType { using type = typename dt_traits<T>::storage; };
template <DT T>
struct WType<T, true> { using type = float; };

template <DT T, bool WF32>
__device__ __forceinline__ void load_w8(const typename WType<T, WF32>::type* w, float (&v)[8]) {
  if constexpr (WF32) load8<DT::F32>(w, v);
  else load8<T>(w, v);
}

// ---------------------------------------------------------------------------------------------
// WPR = waves per row: 1 (the default: one wave per row, no barrier) or 4 (the whole 256-thread
// block on one row, block-level reductions) for launches with few rows -- decode's single-token
// RMSNorm took 9 us as one wave sweeping 4096 elements in 8 dependent-latency chunks.
// EXACT: H == NCH * 8 * lanes per row, so no chunk needs its bounds check -- the loads of every
// chunk then issue back to back (a per-chunk `if` makes hipcc wait for each chunk's loads in turn).
template <DT T, bool WF32, bool LN, bool RES, int NCH, int WPR = 1, bool EXACT = false>
__global__ void __launch_bounds__(256) norm_fwd_kernel(const typename dt_traits<T>::storage* __restrict__ x,
                                                       const typename dt_traits<T>::storage* __restrict__ res,
                                                       const typename WType<T, WF32>::type* __restrict__ w,
                                                       const typename WType<T, WF32>::type* __restrict__ b,
                                                       typename dt_traits<T>::storage* __restrict__ y,
                                                       typename dt_traits<T>::storage* __restrict__ h_out,
                                                       float* __restrict__ rstd_out, float* __restrict__ mean_out,
                                                       int64_t rows, int H, float eps) {
  using S = typename dt_traits<T>::storage;
  constexpr int LPR = 64 * WPR;  // lanes per row
  __shared__ float red[4];
  const int lane = WPR == 1 ? (threadIdx.x & 63) : threadIdx.x;
  const int64_t wid = WPR == 1 ? ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6 : blockIdx.x;
  const int64_t nw = WPR == 1 ? ((int64_t)gridDim.x * blockDim.x) >> 6 : gridDim.x;
  auto row_sum = [&](float v) { return WPR == 1 ? wave_sum(v) : block_sum<4>(v, red); };
  for (int64_t r = wid; r < rows; r += nw) {
    const S* xr = x + r * H;
    float v[NCH][8];
    float s = 0.f;
    // every chunk's loads first, then the residual stores: a store between two chunks' loads makes
    // the next wait cover it (vmcnt counts stores too)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * LPR + lane) * 8;
      if (EXACT || col < H) load8<T>(xr + col, v[c]);
    }
    if constexpr (RES) {
      float t[NCH][8];
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (c * LPR + lane) * 8;
        if (EXACT || col < H) load8<T>(res + r * H + col, t[c]);
      }
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (c * LPR + lane) * 8;
        if (EXACT || col < H) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += t[c][j];
          // the residual stream is kept in the activation dtype (as the unfused path would)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] = to_f32<T>(from_f32<T>(v[c][j]));
          store8<T>(h_out + r * H + col, v[c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * LPR + lane) * 8;
      if (EXACT || col < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[c][j];
      }
    }
    float mean = 0.f;
    if constexpr (LN) {
      mean = row_sum(s) / (float)H;
      s = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (c * LPR + lane) * 8;
        if (EXACT || col < H) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { float d = v[c][j] - mean; s += d * d; }
        }
      }
    } else {
      s = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (c * LPR + lane) * 8;
        if (EXACT || col < H) {
#pragma unroll
          for (int j = 0; j < 8; ++j) s += v[c][j] * v[c][j];
        }
      }
    }
    const float rstd = rsqrtf(row_sum(s) / (float)H + eps);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * LPR + lane) * 8;
      if (EXACT || col < H) {
        float wv[8], o[8];
        load_w8<T, WF32>(w + col, wv);
        if constexpr (LN) {
          float bv[8];
          if (b) load_w8<T, WF32>(b + col, bv);
          else {
#pragma unroll
            for (int j = 0; j < 8; ++j) bv[j] = 0.f;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wv[j] + bv[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rstd * wv[j];
        }
        store8<T>(y + r * H + col, o);
      }
    }
    if (lane == 0) {
      rstd_out[r] = rstd;
      if constexpr (LN) mean_out[r] = mean;
    }
  }
}

// ---------------------------------------------------------------------------------------------
template <DT T, bool WF32, bool LN, bool DRES, int NCH, bool EXACT = false>
__global__ void __launch_bounds__(256) norm_bwd_kernel(const typename dt_traits<T>::storage* __restrict__ dy,
                                                       const typename dt_traits<T>::storage* __restrict__ x,
                                                       const float* __restrict__ rstd_in, const float* __restrict__ mean_in,
                                                       const typename WType<T, WF32>::type* __restrict__ w,
                                                       const typename dt_traits<T>::storage* __restrict__ dres,
                                                       typename dt_traits<T>::storage* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int64_t rows, int H) {
  using S = typename dt_traits<T>::storage;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wv_id = threadIdx.x >> 6;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float dw_acc[NCH][8], db_acc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dw_acc[c][j] = 0.f; db_acc[c][j] = 0.f; }
  for (int64_t r = wid; r < rows; r += nw) {
    const float rstd = rstd_in[r];
    const float mean = LN ? mean_in[r] : 0.f;
    float xh[NCH][8], g[NCH][8];
    float s1 = 0.f, s2 = 0.f;  // s1 = sum(g*xhat), s2 = sum(g)   with g = dy * w
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (EXACT || col < H) {
        float dyv[8], wv[8];
        load8<T>(dy + r * H + col, dyv);
        load8<T>(x + r * H + col, xh[c]);
        load_w8<T, WF32>(w + col, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xh[c][j] - mean) * rstd;
          g[c][j] = dyv[j] * wv[j];
          s1 += g[c][j] * xh[c][j];
          s2 += g[c][j];
          dw_acc[c][j] += dyv[j] * xh[c][j];
          db_acc[c][j] += dyv[j];
        }
      }
    }
    s1 = wave_sum(s1) / (float)H;
    if constexpr (LN) s2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (EXACT || col < H) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = g[c][j] - xh[c][j] * s1;
          if constexpr (LN) t -= s2;
          o[j] = t * rstd;
        }
        if constexpr (DRES) {
          float d[8];
          load8<T>(dres + r * H + col, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += d[j];
        }
        store8<T>(dx + r * H + col, o);
      }
    }
  }
  // block reduction of the per-wave dgamma/dbeta partials through LDS: [4 waves][H] floats
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (EXACT || col < H) {
#pragma unroll
      for (int j = 0; j < 8; ++j) lds[wv_id * H + col + j] = dw_acc[c][j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < H; i += blockDim.x) {
    dw_part[(int64_t)blockIdx.x * H + i] = lds[i] + lds[H + i] + lds[2 * H + i] + lds[3 * H + i];
  }
  if constexpr (LN) {
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (EXACT || col < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[wv_id * H + col + j] = db_acc[c][j];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < H; i += blockDim.x) {
      db_part[(int64_t)blockIdx.x * H + i] = lds[i] + lds[H + i] + lds[2 * H + i] + lds[3 * H + i];
    }
  }
}

// SXE_NORM_EXACT=0 keeps the bounds-checked variants (A/B of the exact-width kernels)
static bool exact_ok(int H, int nch) {
  const char* e = getenv("SXE_NORM_EXACT");
  return H == nch * 512 && !(e && e[0] == '0');
}

static int pick_nch(int H) {
  const int need = (H + 511) / 512;
  if (need <= 1) return 1;
  if (need <= 2) return 2;
  if (need <= 4) return 4;
  if (need <= 8) return 8;
  if (need <= 16) return 16;
  return 32;
}

#define SXE_DISPATCH_NCH(nch, NAME, ...)                 \
  switch (nch) {                                         \
    case 1: { constexpr int NAME = 1; __VA_ARGS__; break; }   \
    case 2: { constexpr int NAME = 2; __VA_ARGS__; break; }   \
    case 4: { constexpr int NAME = 4; __VA_ARGS__; break; }   \
    case 8: { constexpr int NAME = 8; __VA_ARGS__; break; }   \
    case 16: { constexpr int NAME = 16; __VA_ARGS__; break; } \
    default: TORCH_CHECK(false, "sxe norm: hidden size too large (max 16384)"); \
  }


// Returns (y, rstd, mean_or_empty, h_or_empty).
std::vector<at::Tensor> norm_fwd(at::Tensor x, c10::optional<at::Tensor> residual, at::Tensor weight,
                                 c10::optional<at::Tensor> bias, double eps, bool layernorm) {
  SXE_CHECK(x.is_contiguous() && weight.is_contiguous(), "norm_fwd: contiguous inputs");
  const int H = (int)x.size(-1);
  SXE_CHECK(H % 8 == 0 && H <= 16384, "norm_fwd: hidden size must be a multiple of 8 and <= 16384");
  SXE_CHECK(weight.numel() == H, "norm_fwd: weight size");
  const int64_t rows = x.numel() / H;
  c10::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  auto mean = layernorm ? at::empty({rows}, x.options().dtype(at::kFloat)) : at::empty({0}, x.options().dtype(at::kFloat));
  const bool has_res = residual.has_value() && residual->defined();
  at::Tensor h = has_res ? at::empty_like(x) : at::empty({0}, x.options());
  if (has_res) SXE_CHECK(residual->sizes() == x.sizes() && residual->is_contiguous() && residual->scalar_type() == x.scalar_type(), "norm_fwd: residual");
  const bool has_b = bias.has_value() && bias->defined();
  const bool wf32 = weight.scalar_type() == at::kFloat;
  SXE_CHECK(wf32 || weight.scalar_type() == x.scalar_type(), "norm_fwd: weight dtype must be fp32 or match x");
  if (has_b) SXE_CHECK(bias->scalar_type() == weight.scalar_type() && bias->numel() == H, "norm_fwd: bias");
  if (rows == 0) return {y, rstd, mean, h};
  // few rows (decode, small batches): a whole block per row; otherwise one wave per row
  const bool block_rows = rows <= 256 && H >= 1024;
  const int grid = block_rows ? (int)rows : (int)std::min<int64_t>((rows + 3) / 4, 2048);
  DT d = dtype_of(x);
  const int nch = block_rows ? pick_nch((H + 3) / 4) : pick_nch(H);
  SXE_DISPATCH_DT(d, TT, SXE_DISPATCH_BOOL(wf32, WF, SXE_DISPATCH_BOOL(layernorm, LNB, SXE_DISPATCH_BOOL(has_res, RB, SXE_DISPATCH_NCH(nch, NC, {
    using S = typename dt_traits<TT>::storage;
    using W = typename WType<TT, WF>::type;
    auto kern = block_rows ? norm_fwd_kernel<TT, WF, LNB, RB, NC, 4>
                : (exact_ok(H, NC) ? norm_fwd_kernel<TT, WF, LNB, RB, NC, 1, true> : norm_fwd_kernel<TT, WF, LNB, RB, NC, 1>);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(x.data_ptr()), has_res ? reinterpret_cast<const S*>(residual->data_ptr()) : nullptr,
                       reinterpret_cast<const W*>(weight.data_ptr()), has_b ? reinterpret_cast<const W*>(bias->data_ptr()) : nullptr,
                       reinterpret_cast<S*>(y.data_ptr()), has_res ? reinterpret_cast<S*>(h.data_ptr()) : nullptr,
                       rstd.data_ptr<float>(), layernorm ? mean.data_ptr<float>() : nullptr, rows, H, (float)eps);
  })))));
  SXE_LAUNCH_CHECK();
  return {y, rstd, mean, h};
}

// Returns (dx, dweight_fp32, dbias_fp32_or_empty). `dres` (optional) is added into dx.
std::vector<at::Tensor> norm_bwd(at::Tensor dy, at::Tensor x, at::Tensor rstd, c10::optional<at::Tensor> mean,
                                 at::Tensor weight, c10::optional<at::Tensor> dres, bool layernorm) {
  SXE_CHECK(dy.is_contiguous() && x.is_contiguous() && weight.is_contiguous(), "norm_bwd: contiguous");
  const int H = (int)x.size(-1);
  const int64_t rows = x.numel() / H;
  SXE_CHECK(dy.sizes() == x.sizes(), "norm_bwd: dy shape");
  c10::DeviceGuard guard(x.device());
  auto dx = at::empty_like(x);
  const bool has_dres = dres.has_value() && dres->defined();
  if (has_dres) SXE_CHECK(dres->sizes() == x.sizes() && dres->is_contiguous() && dres->scalar_type() == x.scalar_type(), "norm_bwd: dres");
  const bool wf32 = weight.scalar_type() == at::kFloat;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 512));
  auto dw_part = at::empty({grid, H}, x.options().dtype(at::kFloat));
  auto db_part = layernorm ? at::empty({grid, H}, x.options().dtype(at::kFloat)) : at::empty({0}, x.options().dtype(at::kFloat));
  if (rows == 0) {
    return {dx, at::zeros({H}, x.options().dtype(at::kFloat)), layernorm ? at::zeros({H}, x.options().dtype(at::kFloat)) : db_part};
  }
  const size_t lds = (size_t)4 * H * sizeof(float);
  SXE_CHECK(lds <= 160 * 1024, "norm_bwd: hidden too large for LDS reduction");
  DT d = dtype_of(x);
  const int nch = pick_nch(H);
  SXE_DISPATCH_DT(d, TT, SXE_DISPATCH_BOOL(wf32, WF, SXE_DISPATCH_BOOL(layernorm, LNB, SXE_DISPATCH_BOOL(has_dres, DR, SXE_DISPATCH_NCH(nch, NC, {
    using S = typename dt_traits<TT>::storage;
    using W = typename WType<TT, WF>::type;
    auto kern = exact_ok(H, NC) ? norm_bwd_kernel<TT, WF, LNB, DR, NC, true> : norm_bwd_kernel<TT, WF, LNB, DR, NC>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, cur_stream(),
                       reinterpret_cast<const S*>(dy.data_ptr()), reinterpret_cast<const S*>(x.data_ptr()),
                       rstd.data_ptr<float>(), layernorm ? mean->data_ptr<float>() : nullptr,
                       reinterpret_cast<const W*>(weight.data_ptr()),
                       has_dres ? reinterpret_cast<const S*>(dres->data_ptr()) : nullptr,
                       reinterpret_cast<S*>(dx.data_ptr()), dw_part.data_ptr<float>(),
                       layernorm ? db_part.data_ptr<float>() : nullptr, rows, H);
  })))));
  SXE_LAUNCH_CHECK();
  auto dw = dw_part.sum(0);
  auto db = layernorm ? db_part.sum(0) : db_part;
  return {dx, dw, db};
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("norm_fwd(Tensor x, Tensor? residual, Tensor weight, Tensor? bias, float eps, bool layernorm) -> Tensor[]");
  m.def("norm_bwd(Tensor dy, Tensor x, Tensor rstd, Tensor? mean, Tensor weight, Tensor? dres, bool layernorm) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("norm_fwd", &sxe::norm_fwd);
  m.impl("norm_bwd", &sxe::norm_bwd);
}

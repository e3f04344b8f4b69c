// Mixture-of-Experts routing kernels for gfx950: fused softmax + top-k gating, token -> expert-slot
// dispatch and weighted expert -> token combine, each with its backward.
//
// Reference semantics: inference/v2/kernels/ragged_ops/top_k_gating/top_k_gating_cuda.cu:15
// (softmax + top-k per token), moe_scatter/moe_scatter_cuda.cu:23 (rows into expert-ordered slots),
// moe_gather/moe_gather_cuda.cu:21 (weighted gather back to tokens); training-side the reference
// builds one-hot dispatch/combine masks and runs einsums (runtime moe/sharded_moe.py:512-540).
//
// MI355X-first layout: a routing decision is `slots[S, k]` (expert * C + position, -1 = dropped)
// plus its inverse `slot_src[E * C]` (assignment t * k + c, or -1 for an empty capacity slot).
// Every kernel is then a gather with exactly one writer per output row -- no atomics, no memset:
//   dispatch    one block per slot row:  disp[r]  = x[slot_src[r] / k]        (or 0)
//   dispatch'   one block per token:     dx[t]    = sum_c ddisp[slots[t, c]]
//   combine     one block per token:     y[t]     = sum_c w[t, c] * out[slots[t, c]]
//   combine'    one block per slot row:  dout[r]  = w[a] * dy[a / k]   (or 0), dw[a] = <out[r], dy[a / k]>
// Rows move as 16-byte vectors; sums accumulate in fp32. Gating: one wave per token, E <= 512
// experts in registers (8 per lane), k rounds of a 64-lane argmax butterfly.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace moe {

constexpr int NT = 256;

// ------------------------------------------------------------------------------------ gating
template <int EPL>  // experts per lane (E <= 64 * EPL)
__global__ void __launch_bounds__(NT) topk_softmax_kernel(const float* __restrict__ logits, float* __restrict__ probs,
                                                          float* __restrict__ topv, int64_t* __restrict__ topi,
                                                          int64_t S, int E, int k) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (t >= S) return;  // wave-uniform exit
  const float* row = logits + t * E;
  float v[EPL];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < E ? row[e] : -INFINITY;
    mx = fmaxf(mx, v[j]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < E ? __expf(v[j] - mx) : 0.f;
    sum += v[j];
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  float* prow = probs + t * E;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = j * 64 + lane;
    v[j] *= inv;
    if (e < E) prow[e] = v[j];
  }
  // k rounds: wave argmax (largest value, lowest index on ties), then knock the winner out
  for (int r = 0; r < k; ++r) {
    float bv = -1.f;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      const int e = j * 64 + lane;
      if (e < E && (v[j] > bv || (v[j] == bv && e < bi))) { bv = v[j]; bi = e; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) {
      topv[t * k + r] = bv;
      topi[t * k + r] = bi;
    }
#pragma unroll
    for (int j = 0; j < EPL; ++j)
      if (j * 64 + lane == bi) v[j] = -2.f;  // below every probability
  }
}

// --------------------------------------------------------------------------------- data path
template <DT T>
__global__ void __launch_bounds__(NT) dispatch_kernel(const typename dt_traits<T>::storage* __restrict__ x,
                                                      const int64_t* __restrict__ slot_src,
                                                      typename dt_traits<T>::storage* __restrict__ disp,
                                                      int64_t rows, int H, int k) {
  using st = typename dt_traits<T>::storage;
  const int nv = H / 8;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t a = slot_src[r];
    st* dst = disp + r * H;
    if (a < 0) {
      float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int c = threadIdx.x; c < nv; c += NT) store8<T>(dst + c * 8, z);
    } else {
      const st* src = x + (a / k) * H;
      float v[8];
      for (int c = threadIdx.x; c < nv; c += NT) {
        load8<T>(src + c * 8, v);
        store8<T>(dst + c * 8, v);
      }
    }
  }
}

// out[t] = sum_c coef[t, c] * src[slots[t, c]]  (coef == nullptr: 1). Serves dispatch' and combine.
template <DT T>
__global__ void __launch_bounds__(NT) gather_sum_kernel(const typename dt_traits<T>::storage* __restrict__ src,
                                                        const int64_t* __restrict__ slots,
                                                        const float* __restrict__ coef,
                                                        typename dt_traits<T>::storage* __restrict__ out,
                                                        int64_t S, int H, int k) {
  const int nv = H / 8;
  for (int64_t t = blockIdx.x; t < S; t += gridDim.x) {
    for (int c8 = threadIdx.x; c8 < nv; c8 += NT) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int c = 0; c < k; ++c) {
        const int64_t s = slots[t * k + c];
        if (s < 0) continue;
        const float w = coef ? coef[t * k + c] : 1.f;
        float v[8];
        load8<T>(src + s * H + c8 * 8, v);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += w * v[i];
      }
      store8<T>(out + t * H + c8 * 8, acc);
    }
  }
}

template <DT T>
__global__ void __launch_bounds__(NT) combine_bwd_kernel(const typename dt_traits<T>::storage* __restrict__ gy,
                                                         const typename dt_traits<T>::storage* __restrict__ expert_out,
                                                         const int64_t* __restrict__ slot_src,
                                                         const float* __restrict__ w,
                                                         typename dt_traits<T>::storage* __restrict__ gout,
                                                         float* __restrict__ gw, int64_t rows, int H, int k) {
  __shared__ float red[NT / 64];
  const int nv = H / 8;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t a = slot_src[r];
    typename dt_traits<T>::storage* dst = gout + r * H;
    if (a < 0) {
      float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int c = threadIdx.x; c < nv; c += NT) store8<T>(dst + c * 8, z);
      continue;  // block-uniform
    }
    const float wa = w[a];
    const auto* g = gy + (a / k) * H;
    const auto* o = expert_out + r * H;
    float dot = 0.f;
    for (int c = threadIdx.x; c < nv; c += NT) {
      float gv[8], ov[8], d[8];
      load8<T>(g + c * 8, gv);
      load8<T>(o + c * 8, ov);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        d[i] = wa * gv[i];
        dot += ov[i] * gv[i];
      }
      store8<T>(dst + c * 8, d);
    }
    dot = block_sum<NT / 64>(dot, red);
    if (threadIdx.x == 0) gw[a] = dot;
  }
}

inline int row_grid(int64_t rows) { return (int)std::max<int64_t>(1, std::min<int64_t>(rows, (int64_t)kNumCUs * 16)); }

}  // namespace moe

// probs [S, E] fp32, top values [S, k] fp32, top indices [S, k] int64
std::tuple<at::Tensor, at::Tensor, at::Tensor> moe_topk_softmax(const at::Tensor& logits, int64_t k) {
  SXE_CHECK_CUDA(logits);
  SXE_CHECK(logits.dim() == 2 && logits.scalar_type() == at::kFloat && logits.is_contiguous(),
            "moe_topk_softmax: contiguous fp32 [S, E] logits");
  const int64_t S = logits.size(0);
  const int E = logits.size(1);
  SXE_CHECK(E <= 512 && k >= 1 && k <= E, "moe_topk_softmax: E <= 512, 1 <= k <= E");
  c10::DeviceGuard g(logits.device());
  auto probs = at::empty_like(logits);
  auto topv = at::empty({S, k}, logits.options());
  auto topi = at::empty({S, k}, logits.options().dtype(at::kLong));
  if (S == 0) return {probs, topv, topi};
  const int grid = (int)((S + moe::NT / 64 - 1) / (moe::NT / 64));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(moe::NT), 0, cur_stream(), logits.data_ptr<float>(),
                       probs.data_ptr<float>(), topv.data_ptr<float>(), topi.data_ptr<int64_t>(), S, E, (int)k);
  };
  if (E <= 64) launch(moe::topk_softmax_kernel<1>);
  else if (E <= 128) launch(moe::topk_softmax_kernel<2>);
  else if (E <= 256) launch(moe::topk_softmax_kernel<4>);
  else launch(moe::topk_softmax_kernel<8>);
  SXE_LAUNCH_CHECK();
  return {probs, topv, topi};
}

static void check_rows(const at::Tensor& t, const char* name) {
  SXE_CHECK(t.is_cuda() && t.dim() == 2 && t.is_contiguous() && t.size(1) % 8 == 0, name,
            ": contiguous GPU [rows, H] with H % 8 == 0");
}

at::Tensor moe_dispatch(const at::Tensor& x, const at::Tensor& slot_src, int64_t k) {
  check_rows(x, "moe_dispatch x");
  SXE_CHECK(slot_src.scalar_type() == at::kLong && slot_src.is_contiguous() && slot_src.is_cuda(),
            "moe_dispatch: int64 slot_src");
  c10::DeviceGuard g(x.device());
  const int64_t rows = slot_src.numel();
  const int H = x.size(1);
  auto disp = at::empty({rows, H}, x.options());
  if (rows == 0) return disp;
  SXE_DISPATCH_DT(dtype_of(x), T, {
    using st = typename dt_traits<T>::storage;
    hipLaunchKernelGGL(moe::dispatch_kernel<T>, dim3(moe::row_grid(rows)), dim3(moe::NT), 0, cur_stream(),
                       reinterpret_cast<const st*>(x.data_ptr()), slot_src.data_ptr<int64_t>(),
                       reinterpret_cast<st*>(disp.data_ptr()), rows, H, (int)k);
  });
  SXE_LAUNCH_CHECK();
  return disp;
}

// out[t] = sum_c coef[t, c] * src[slots[t, c]] (coef optional): the dispatch backward (coef = None)
// and the combine forward
at::Tensor moe_gather_sum(const at::Tensor& src, const at::Tensor& slots, const c10::optional<at::Tensor>& coef) {
  check_rows(src, "moe_gather_sum src");
  SXE_CHECK(slots.scalar_type() == at::kLong && slots.dim() == 2 && slots.is_contiguous() && slots.is_cuda(),
            "moe_gather_sum: int64 [S, k] slots");
  const float* cp = nullptr;
  if (coef.has_value()) {
    SXE_CHECK(coef->scalar_type() == at::kFloat && coef->is_contiguous() && coef->numel() == slots.numel(),
              "moe_gather_sum: fp32 [S, k] coef");
    cp = coef->data_ptr<float>();
  }
  c10::DeviceGuard g(src.device());
  const int64_t S = slots.size(0);
  const int k = slots.size(1), H = src.size(1);
  auto out = at::empty({S, H}, src.options());
  if (S == 0) return out;
  SXE_DISPATCH_DT(dtype_of(src), T, {
    using st = typename dt_traits<T>::storage;
    hipLaunchKernelGGL(moe::gather_sum_kernel<T>, dim3(moe::row_grid(S)), dim3(moe::NT), 0, cur_stream(),
                       reinterpret_cast<const st*>(src.data_ptr()), slots.data_ptr<int64_t>(), cp,
                       reinterpret_cast<st*>(out.data_ptr()), S, H, k);
  });
  SXE_LAUNCH_CHECK();
  return out;
}

// combine backward: (d expert_out [rows, H], d w [S, k] fp32)
std::tuple<at::Tensor, at::Tensor> moe_combine_bwd(const at::Tensor& gy, const at::Tensor& expert_out,
                                                   const at::Tensor& slot_src, const at::Tensor& w) {
  check_rows(gy, "moe_combine_bwd gy");
  check_rows(expert_out, "moe_combine_bwd expert_out");
  SXE_CHECK(gy.scalar_type() == expert_out.scalar_type() && gy.size(1) == expert_out.size(1),
            "moe_combine_bwd: dtype / H mismatch");
  SXE_CHECK(slot_src.scalar_type() == at::kLong && slot_src.numel() == expert_out.size(0),
            "moe_combine_bwd: int64 slot_src per expert row");
  SXE_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 2 && w.size(0) == gy.size(0),
            "moe_combine_bwd: fp32 [S, k] w");
  c10::DeviceGuard g(gy.device());
  const int64_t rows = expert_out.size(0);
  const int H = gy.size(1), k = w.size(1);
  auto gout = at::empty_like(expert_out);
  auto gw = at::zeros_like(w);  // dropped assignments keep a zero weight gradient
  if (rows == 0) return {gout, gw};
  SXE_DISPATCH_DT(dtype_of(gy), T, {
    using st = typename dt_traits<T>::storage;
    hipLaunchKernelGGL(moe::combine_bwd_kernel<T>, dim3(moe::row_grid(rows)), dim3(moe::NT), 0, cur_stream(),
                       reinterpret_cast<const st*>(gy.data_ptr()), reinterpret_cast<const st*>(expert_out.data_ptr()),
                       slot_src.data_ptr<int64_t>(), w.data_ptr<float>(), reinterpret_cast<st*>(gout.data_ptr()),
                       gw.data_ptr<float>(), rows, H, k);
  });
  SXE_LAUNCH_CHECK();
  return {gout, gw};
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("moe_topk_softmax(Tensor logits, int k) -> (Tensor, Tensor, Tensor)");
  m.def("moe_dispatch(Tensor x, Tensor slot_src, int k) -> Tensor");
  m.def("moe_gather_sum(Tensor src, Tensor slots, Tensor? coef) -> Tensor");
  m.def("moe_combine_bwd(Tensor gy, Tensor expert_out, Tensor slot_src, Tensor w) -> (Tensor, Tensor)");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("moe_topk_softmax", &sxe::moe_topk_softmax);
  m.impl("moe_dispatch", &sxe::moe_dispatch);
  m.impl("moe_gather_sum", &sxe::moe_gather_sum);
  m.impl("moe_combine_bwd", &sxe::moe_combine_bwd);
}

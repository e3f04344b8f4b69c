// Softmax cross-entropy over large vocabularies for gfx950 (forward, backward, and a fused
// forward+backward that overwrites the logits with their gradient).
//
// The reference computes the LM loss with torch (and, for sequence parallelism, a vocab/sequence
// sharded variant: deepspeed/sequence/cross_entropy.py:11-60; ALST's TiledLoss,
// runtime/sequence_parallel/ulysses_sp.py:915). Here one workgroup owns one token row
// (V up to ~256K): a single 16-byte-vectorised sweep computes the running (max, sum-exp) per lane
// (online softmax), the 4 waves merge through LDS, and the backward sweep re-reads the row
// (Infinity-Cache resident at these row sizes) and writes bf16 gradients IN PLACE, so the
// [tokens, vocab] logits tensor is never duplicated (4 GiB at 16K tokens x 128K vocab).
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {

__device__ __forceinline__ void ms_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) { m = mn; s = 0.f; return; }
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <DT T, bool VEC>
__device__ __forceinline__ float row_lse(const typename dt_traits<T>::storage* __restrict__ row, int V, float* red) {
  float m = -INFINITY, s = 0.f;
  if constexpr (VEC) {
    for (int c = threadIdx.x * 8; c < V; c += blockDim.x * 8) {
      float v[8];
      load8<T>(row + c, v);
      float lm = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ls += __expf(v[j] - lm);
      ms_merge(m, s, lm, ls);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += blockDim.x) ms_merge(m, s, to_f32<T>(row[c]), 1.f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { red[2 * w] = m; red[2 * w + 1] = s; }
  __syncthreads();
  float M = red[0], Ssum = red[1];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) ms_merge(M, Ssum, red[2 * i], red[2 * i + 1]);
  __syncthreads();
  return M + __logf(Ssum);
}

// mode: 0 = forward only; 1 = forward + in-place gradient with grad = scale * (softmax - onehot)
template <DT T, bool VEC>
__global__ void __launch_bounds__(256) xent_kernel(typename dt_traits<T>::storage* __restrict__ logits, int64_t rows, int V,
                                                   const int64_t* __restrict__ target, int64_t ignore_index,
                                                   float* __restrict__ loss, float* __restrict__ lse_out, int mode,
                                                   const float* __restrict__ scale_t, float scale) {
  __shared__ float red[8];
  if (scale_t) scale *= *scale_t;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    typename dt_traits<T>::storage* row = logits + r * V;
    const int64_t tgt = target[r];
    const bool ign = (tgt == ignore_index);
    const float lse = row_lse<T, VEC>(row, V, red);
    if (threadIdx.x == 0) {
      const float xt = ign ? 0.f : to_f32<T>(row[tgt]);
      loss[r] = ign ? 0.f : (lse - xt);
      if (lse_out) lse_out[r] = lse;
    }
    __syncthreads();  // the target logit is read above before the gradient overwrites it
    if (mode == 1) {
      const float sc = ign ? 0.f : scale;
      if constexpr (VEC) {
        for (int c = threadIdx.x * 8; c < V; c += blockDim.x * 8) {
          float v[8];
          load8<T>(row + c, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = sc * (__expf(v[j] - lse) - ((c + j) == tgt ? 1.f : 0.f));
          store8<T>(row + c, v);
        }
      } else {
        for (int c = threadIdx.x; c < V; c += blockDim.x) {
          float v = to_f32<T>(row[c]);
          row[c] = from_f32<T>(sc * (__expf(v - lse) - (c == tgt ? 1.f : 0.f)));
        }
      }
    }
  }
}

// grad = dloss[r] * (softmax - onehot), written into grad_out (may alias logits).
template <DT T, bool VEC>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const typename dt_traits<T>::storage* __restrict__ logits,
                                                       typename dt_traits<T>::storage* __restrict__ grad, int64_t rows, int V,
                                                       const int64_t* __restrict__ target, int64_t ignore_index,
                                                       const float* __restrict__ lse, const float* __restrict__ dloss) {
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t tgt = target[r];
    const float sc = (tgt == ignore_index) ? 0.f : dloss[r];
    const float l = lse[r];
    const typename dt_traits<T>::storage* in = logits + r * V;
    typename dt_traits<T>::storage* out = grad + r * V;
    if constexpr (VEC) {
      for (int c = threadIdx.x * 8; c < V; c += blockDim.x * 8) {
        float v[8];
        load8<T>(in + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = sc * (__expf(v[j] - l) - ((c + j) == tgt ? 1.f : 0.f));
        store8<T>(out + c, v);
      }
    } else {
      for (int c = threadIdx.x; c < V; c += blockDim.x) {
        float v = to_f32<T>(in[c]);
        out[c] = from_f32<T>(sc * (__expf(v - l) - (c == tgt ? 1.f : 0.f)));
      }
    }
  }
}

// Dual-layout LM-head gradient (bf16): g = sc[r] * (softmax - onehot) with sc = dloss * scale_a * scale_b
// (all device scalars; 0 on ignored rows), written IN PLACE over the logits (token-major, for the
// data-gradient GEMM) AND as g^T [V, rows] (vocab-major, so the weight-gradient GEMM dW = g^T h
// reads K-contiguous operands: hipBLASLt's TN layout, 12.1 vs 14.6 ms for transposes + TN at 16k
// tokens x 128256, profiles/r06/wgrad_variants_16k.log). Running in the backward, where the
// upstream scalar is known, it also replaces the forward's in-place gradient write and the
// backward's scaling pass: 16.8 GB of HBM traffic per 16k-token micro-step instead of 25.2.
// Geometry: one 1024-thread workgroup per 64-token x 256-column tile; thread t owns row t/16 and
// 16 columns from (t%16)*16 (two 16-byte vectors), stages the bf16 result in an LDS tile with a
// 258-element row stride (odd dword stride: the column-wise reads spread over the banks), then
// stores 16 tokens of one vocab row of g^T as two 16-byte vectors.
constexpr int XG_TR = 64, XG_TC = 256, XG_LD = XG_TC + 2;

__global__ void __launch_bounds__(1024) xent_grad_dual_kernel(unsigned short* __restrict__ logits,
                                                              unsigned short* __restrict__ gT, int64_t rows, int V,
                                                              const int64_t* __restrict__ target, int64_t ignore_index,
                                                              const float* __restrict__ lse, const float* __restrict__ s_a,
                                                              const float* __restrict__ s_b) {
  __shared__ __attribute__((aligned(16))) unsigned short tile[XG_TR * XG_LD];
  const int tiles_c = V / XG_TC;
  const int64_t tr = blockIdx.x / tiles_c;
  const int tc = (int)(blockIdx.x - tr * tiles_c);
  const int t = threadIdx.x, r = t >> 4, c0 = (t & 15) * 16;
  const int64_t row = tr * XG_TR + r;
  const int col = tc * XG_TC + c0;
  const int64_t tgt = target[row];
  const float sc = (tgt == ignore_index) ? 0.f : s_a[0] * (s_b ? s_b[0] : 1.f);
  const float l = lse[row];
  unsigned short* p = logits + row * V + col;
  const u16x8 a = *reinterpret_cast<const u16x8*>(p), b = *reinterpret_cast<const u16x8*>(p + 8);
  u16x8 oa, ob;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    oa[j] = f32_to_bf16(sc * (__expf(bf16_to_f32(a[j]) - l) - ((col + j) == tgt ? 1.f : 0.f)));
    ob[j] = f32_to_bf16(sc * (__expf(bf16_to_f32(b[j]) - l) - ((col + 8 + j) == tgt ? 1.f : 0.f)));
  }
  *reinterpret_cast<u16x8*>(p) = oa;
  *reinterpret_cast<u16x8*>(p + 8) = ob;
  unsigned* ld = reinterpret_cast<unsigned*>(&tile[r * XG_LD + c0]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ld[j] = (unsigned)oa[2 * j] | ((unsigned)oa[2 * j + 1] << 16);
    ld[4 + j] = (unsigned)ob[2 * j] | ((unsigned)ob[2 * j + 1] << 16);
  }
  __syncthreads();
  // transposed store: output row = tile column t/4, 16 tokens from (t%4)*16
  const int oc = t >> 2, r0 = (t & 3) * 16;
  u16x8 o0, o1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o0[j] = tile[(r0 + j) * XG_LD + oc];
    o1[j] = tile[(r0 + 8 + j) * XG_LD + oc];
  }
  unsigned short* d = gT + (int64_t)(tc * XG_TC + oc) * rows + tr * XG_TR + r0;
  *reinterpret_cast<u16x8*>(d) = o0;
  *reinterpret_cast<u16x8*>(d + 8) = o1;
}

// -> g^T [V, rows]; the logits are overwritten with g. rows % 64 == 0, V % 256 == 0, bf16.
at::Tensor xent_grad_dual(at::Tensor logits, at::Tensor target, at::Tensor lse, int64_t ignore_index, at::Tensor scale_a,
                          c10::optional<at::Tensor> scale_b) {
  SXE_CHECK_CUDA(logits);
  SXE_CHECK(logits.dim() == 2 && logits.is_contiguous() && logits.scalar_type() == at::kBFloat16,
            "xent_grad_dual: contiguous bf16 [rows, vocab] logits");
  SXE_CHECK(target.scalar_type() == at::kLong && target.numel() == logits.size(0) && target.is_contiguous(),
            "xent_grad_dual: target must be int64 [rows]");
  const int64_t rows = logits.size(0);
  const int V = (int)logits.size(1);
  SXE_CHECK(rows % XG_TR == 0 && V % XG_TC == 0, "xent_grad_dual: rows % 64 and vocab % 256 must be 0");
  SXE_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == rows && lse.is_contiguous(), "xent_grad_dual: lse fp32 [rows]");
  SXE_CHECK(scale_a.scalar_type() == at::kFloat && scale_a.is_cuda() && scale_a.numel() == 1, "xent_grad_dual: scale_a fp32 [1]");
  const float* sb = nullptr;
  if (scale_b.has_value() && scale_b->defined()) {
    SXE_CHECK(scale_b->scalar_type() == at::kFloat && scale_b->is_cuda() && scale_b->numel() == 1,
              "xent_grad_dual: scale_b fp32 [1]");
    sb = scale_b->data_ptr<float>();
  }
  c10::DeviceGuard guard(logits.device());
  auto gT = at::empty({(int64_t)V, rows}, logits.options());
  const int64_t tiles = (rows / XG_TR) * (V / XG_TC);
  if (tiles == 0) return gT;
  SXE_CHECK(tiles < (1ll << 31), "xent_grad_dual: too many tiles");
  hipLaunchKernelGGL(xent_grad_dual_kernel, dim3((unsigned)tiles), dim3(1024), 0, cur_stream(),
                     reinterpret_cast<unsigned short*>(logits.data_ptr()), reinterpret_cast<unsigned short*>(gT.data_ptr()),
                     rows, V, target.data_ptr<int64_t>(), ignore_index, lse.data_ptr<float>(), scale_a.data_ptr<float>(), sb);
  SXE_LAUNCH_CHECK();
  return gT;
}

static void xent_checks(const at::Tensor& logits, const at::Tensor& target) {
  SXE_CHECK(logits.dim() == 2 && logits.is_contiguous(), "xent: logits must be contiguous [rows, vocab]");
  SXE_CHECK(target.scalar_type() == at::kLong && target.numel() == logits.size(0) && target.is_contiguous(),
            "xent: target must be int64 [rows]");
}

// Returns (loss [rows] fp32, lse [rows] fp32). If `inplace_grad`, logits are overwritten with
// scale * (softmax - onehot) where scale = grad_scale * (*scale_t if given).
std::tuple<at::Tensor, at::Tensor> xent_fwd(at::Tensor logits, at::Tensor target, int64_t ignore_index, bool inplace_grad,
                                 c10::optional<at::Tensor> scale_t, double grad_scale) {
  xent_checks(logits, target);
  const int64_t rows = logits.size(0);
  const int V = (int)logits.size(1);
  c10::DeviceGuard guard(logits.device());
  auto loss = at::empty({rows}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({rows}, logits.options().dtype(at::kFloat));
  if (rows == 0) return {loss, lse};
  const float* sp = nullptr;
  if (scale_t.has_value() && scale_t->defined()) {
    SXE_CHECK(scale_t->scalar_type() == at::kFloat && scale_t->is_cuda(), "xent: scale tensor fp32");
    sp = scale_t->data_ptr<float>();
  }
  const bool vec = (V % 8 == 0);
  const int grid = (int)std::min<int64_t>(rows, 8192);
  DT d = dtype_of(logits);
  SXE_DISPATCH_DT(d, TT, SXE_DISPATCH_BOOL(vec, VB, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((xent_kernel<TT, VB>), dim3(grid), dim3(256), 0, cur_stream(), reinterpret_cast<S*>(logits.data_ptr()),
                       rows, V, target.data_ptr<int64_t>(), ignore_index, loss.data_ptr<float>(), lse.data_ptr<float>(),
                       inplace_grad ? 1 : 0, sp, (float)grad_scale);
  }));
  SXE_LAUNCH_CHECK();
  return {loss, lse};
}

at::Tensor xent_bwd(at::Tensor logits, at::Tensor target, at::Tensor lse, at::Tensor dloss, int64_t ignore_index,
                    bool inplace) {
  xent_checks(logits, target);
  const int64_t rows = logits.size(0);
  const int V = (int)logits.size(1);
  SXE_CHECK(dloss.scalar_type() == at::kFloat && dloss.numel() == rows && dloss.is_contiguous(), "xent_bwd: dloss fp32 [rows]");
  c10::DeviceGuard guard(logits.device());
  at::Tensor grad = inplace ? logits : at::empty_like(logits);
  if (rows == 0) return grad;
  const bool vec = (V % 8 == 0);
  const int grid = (int)std::min<int64_t>(rows, 8192);
  DT d = dtype_of(logits);
  SXE_DISPATCH_DT(d, TT, SXE_DISPATCH_BOOL(vec, VB, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((xent_bwd_kernel<TT, VB>), dim3(grid), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const S*>(logits.data_ptr()), reinterpret_cast<S*>(grad.data_ptr()), rows, V,
                       target.data_ptr<int64_t>(), ignore_index, lse.data_ptr<float>(), dloss.data_ptr<float>());
  }));
  SXE_LAUNCH_CHECK();
  return grad;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("xent_fwd(Tensor(a!) logits, Tensor target, int ignore_index, bool inplace_grad, Tensor? scale, float grad_scale) -> (Tensor, Tensor)");
  m.def("xent_bwd(Tensor(a!) logits, Tensor target, Tensor lse, Tensor dloss, int ignore_index, bool inplace) -> Tensor");
  m.def("xent_grad_dual(Tensor(a!) logits, Tensor target, Tensor lse, int ignore_index, Tensor scale_a, Tensor? scale_b) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("xent_grad_dual", &sxe::xent_grad_dual);
  m.impl("xent_fwd", &sxe::xent_fwd);
  m.impl("xent_bwd", &sxe::xent_bwd);
}

// Fused optimizer kernels for gfx950: Adam/AdamW, Lion, Adagrad over flat fp32 master
// partitions (the ZeRO layout) and over tensor lists (multi-tensor apply).
//
// Replaces the reference's missing `multi_tensor_adam` CUDA op
// (deepspeed/ops/adam/fused_adam.py:96,175-191) and the Lion/Adagrad ops
// (deepspeed/ops/lion/fused_lion.py:42). MI355X design points:
//  * one pass over HBM: read g, p32, m, v; write p32, m, v and (optionally) the bf16/fp16
//    working copy of the parameter, so the fp32->bit16 copy of the ZeRO step
//    (reference stage_1_and_2.py:2174-2176) costs no extra pass;
//  * 16-byte accesses (float4 for fp32 state, 8-byte for bf16 grads), grid-stride over
//    256 CUs x 8 blocks;
//  * device-side `scale` (1/loss_scale * clip coefficient) and `skip` flag tensors so the
//    step never needs a host sync for clipping or overflow skipping.
#include "sxe_common.h"
#include <torch/library.h>
#include <vector>

namespace sxe {

struct AdamHP {
  float lr, beta1, beta2, eps, wd, bc1, bc2;  // bc* = 1 - beta^step (or 1 when disabled)
  int adamw;
};

template <DT G, DT L>
__device__ __forceinline__ void adam_vec4(float* __restrict__ p, const typename dt_traits<G>::storage* __restrict__ g,
                                          float* __restrict__ m, float* __restrict__ v,
                                          typename dt_traits<L>::storage* __restrict__ lp, const AdamHP& hp,
                                          float gscale) {
  f32x4 pv = *reinterpret_cast<const f32x4*>(p);
  f32x4 mv = *reinterpret_cast<const f32x4*>(m);
  f32x4 vv = *reinterpret_cast<const f32x4*>(v);
  float gv[4];
  if constexpr (G == DT::F32) {
    f32x4 t = *reinterpret_cast<const f32x4*>(g);
#pragma unroll
    for (int i = 0; i < 4; ++i) gv[i] = t[i];
  } else {
    u16x4 t = *reinterpret_cast<const u16x4*>(g);
#pragma unroll
    for (int i = 0; i < 4; ++i) gv[i] = to_f32<G>(t[i]);
  }
  const float step_size = hp.lr / hp.bc1;
  const float inv_bc2_sqrt = 1.0f / sqrtf(hp.bc2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float gi = gv[i] * gscale;
    float pi = pv[i];
    if (!hp.adamw && hp.wd != 0.f) gi += hp.wd * pi;
    float mi = hp.beta1 * mv[i] + (1.f - hp.beta1) * gi;
    float vi = hp.beta2 * vv[i] + (1.f - hp.beta2) * gi * gi;
    float denom = sqrtf(vi) * inv_bc2_sqrt + hp.eps;
    if (hp.adamw && hp.wd != 0.f) pi -= hp.lr * hp.wd * pi;
    pi -= step_size * mi / denom;
    pv[i] = pi; mv[i] = mi; vv[i] = vi;
  }
  *reinterpret_cast<f32x4*>(p) = pv;
  *reinterpret_cast<f32x4*>(m) = mv;
  *reinterpret_cast<f32x4*>(v) = vv;
  if (lp) {
    if constexpr (L == DT::F32) {
      *reinterpret_cast<f32x4*>(lp) = pv;
    } else {
      u16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = from_f32<L>(pv[i]);
      *reinterpret_cast<u16x4*>(lp) = o;
    }
  }
}

template <DT G, DT L>
__global__ void __launch_bounds__(256) adam_flat_kernel(float* __restrict__ p, const typename dt_traits<G>::storage* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        typename dt_traits<L>::storage* __restrict__ lp, int64_t n, AdamHP hp,
                                                        float gscale, const float* __restrict__ scale_t,
                                                        const float* __restrict__ skip_t) {
  if (skip_t && *skip_t != 0.f) return;
  if (scale_t) gscale *= *scale_t;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t o = i << 2;
    adam_vec4<G, L>(p + o, g + o, m + o, v + o, lp ? lp + o : nullptr, hp, gscale);
  }
  // scalar tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t o = (n4 << 2) + threadIdx.x;
    float gi = to_f32<G>(g[o]) * gscale, pi = p[o];
    if (!hp.adamw && hp.wd != 0.f) gi += hp.wd * pi;
    float mi = hp.beta1 * m[o] + (1.f - hp.beta1) * gi;
    float vi = hp.beta2 * v[o] + (1.f - hp.beta2) * gi * gi;
    float denom = sqrtf(vi) / sqrtf(hp.bc2) + hp.eps;
    if (hp.adamw && hp.wd != 0.f) pi -= hp.lr * hp.wd * pi;
    pi -= (hp.lr / hp.bc1) * mi / denom;
    p[o] = pi; m[o] = mi; v[o] = vi;
    if (lp) lp[o] = from_f32<L>(pi);
  }
}

static AdamHP make_hp(double lr, double b1, double b2, double eps, double wd, int64_t step, bool adamw, bool bias_corr) {
  AdamHP hp;
  hp.lr = (float)lr; hp.beta1 = (float)b1; hp.beta2 = (float)b2; hp.eps = (float)eps; hp.wd = (float)wd;
  hp.bc1 = bias_corr ? (float)(1.0 - std::pow(b1, (double)step)) : 1.f;
  hp.bc2 = bias_corr ? (float)(1.0 - std::pow(b2, (double)step)) : 1.f;
  hp.adamw = adamw ? 1 : 0;
  return hp;
}

static const float* opt_f32_ptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  SXE_CHECK(t->scalar_type() == at::kFloat && t->numel() >= 1 && t->is_cuda(), "scale/skip tensors must be fp32 GPU scalars");
  return t->data_ptr<float>();
}

void adam_flat_(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, c10::optional<at::Tensor> lp,
                c10::optional<at::Tensor> scale_t, c10::optional<at::Tensor> skip_t, double lr, double beta1,
                double beta2, double eps, double weight_decay, int64_t step, bool adamw, bool bias_correction,
                double grad_scale) {
  SXE_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
            "adam_flat_: master/state must be fp32");
  SXE_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adam_flat_: contiguous");
  const int64_t n = p.numel();
  SXE_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam_flat_: size mismatch");
  if (n == 0) return;
  const bool has_lp = lp.has_value() && lp->defined();
  if (has_lp) SXE_CHECK(lp->numel() == n && lp->is_contiguous(), "adam_flat_: lp size");
  // 16-byte alignment of every operand is required for the vector path.
  auto al = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
  SXE_CHECK(al(p) && al(m) && al(v), "adam_flat_: fp32 operands must be 16-byte aligned");
  SXE_CHECK((reinterpret_cast<uintptr_t>(g.data_ptr()) & 7) == 0, "adam_flat_: grad must be 8-byte aligned");
  c10::DeviceGuard guard(p.device());
  AdamHP hp = make_hp(lr, beta1, beta2, eps, weight_decay, step, adamw, bias_correction);
  const int block = 256;
  const int grid = stream_grid((n + 3) / 4, block);
  const float* sp = opt_f32_ptr(scale_t);
  const float* kp = opt_f32_ptr(skip_t);
  DT gd = dtype_of(g);
  DT ld = has_lp ? dtype_of(*lp) : DT::BF16;
  SXE_DISPATCH_DT(gd, GT, SXE_DISPATCH_DT(ld, LT, {
    using GS = typename dt_traits<GT>::storage;
    using LS = typename dt_traits<LT>::storage;
    hipLaunchKernelGGL((adam_flat_kernel<GT, LT>), dim3(grid), dim3(block), 0, cur_stream(), p.data_ptr<float>(),
                       reinterpret_cast<const GS*>(g.data_ptr()), m.data_ptr<float>(), v.data_ptr<float>(),
                       has_lp ? reinterpret_cast<LS*>(lp->data_ptr()) : nullptr, n, hp, (float)grad_scale, sp, kp);
  }));
  SXE_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Multi-tensor Adam: one launch over a list of (p, g, m, v[, lp]) tensors. The chunk table is
// built on the host into a pinned buffer and copied with the launch stream, so the call is
// graph-capture safe apart from the H2D copy node.
struct MTChunk {
  float* p; const void* g; float* m; float* v; void* lp; int64_t n;
};

template <DT G, DT L>
__global__ void __launch_bounds__(256) adam_mt_kernel(const MTChunk* __restrict__ chunks, AdamHP hp, float gscale,
                                                      const float* __restrict__ scale_t, const float* __restrict__ skip_t) {
  if (skip_t && *skip_t != 0.f) return;
  if (scale_t) gscale *= *scale_t;
  const MTChunk c = chunks[blockIdx.x];
  using GS = typename dt_traits<G>::storage;
  using LS = typename dt_traits<L>::storage;
  const GS* g = reinterpret_cast<const GS*>(c.g);
  LS* lp = reinterpret_cast<LS*>(c.lp);
  const bool vec_ok = ((reinterpret_cast<uintptr_t>(c.p) | reinterpret_cast<uintptr_t>(c.m) |
                        reinterpret_cast<uintptr_t>(c.v)) & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(c.g) & 7) == 0 && (reinterpret_cast<uintptr_t>(c.lp) & 7) == 0;
  int64_t start = 0;
  if (vec_ok) {
    const int64_t n4 = c.n >> 2;
    for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
      const int64_t o = i << 2;
      adam_vec4<G, L>(c.p + o, g + o, c.m + o, c.v + o, lp ? lp + o : nullptr, hp, gscale);
    }
    start = n4 << 2;
  }
  for (int64_t o = start + threadIdx.x; o < c.n; o += blockDim.x) {
    float gi = to_f32<G>(g[o]) * gscale, pi = c.p[o];
    if (!hp.adamw && hp.wd != 0.f) gi += hp.wd * pi;
    float mi = hp.beta1 * c.m[o] + (1.f - hp.beta1) * gi;
    float vi = hp.beta2 * c.v[o] + (1.f - hp.beta2) * gi * gi;
    float denom = sqrtf(vi) / sqrtf(hp.bc2) + hp.eps;
    if (hp.adamw && hp.wd != 0.f) pi -= hp.lr * hp.wd * pi;
    pi -= (hp.lr / hp.bc1) * mi / denom;
    c.p[o] = pi; c.m[o] = mi; c.v[o] = vi;
    if (lp) lp[o] = from_f32<L>(pi);
  }
}

void multi_tensor_adam_(at::TensorList p, at::TensorList g, at::TensorList m, at::TensorList v, at::TensorList lp,
                        c10::optional<at::Tensor> scale_t, c10::optional<at::Tensor> skip_t, double lr, double beta1,
                        double beta2, double eps, double weight_decay, int64_t step, bool adamw, bool bias_correction,
                        double grad_scale) {
  const size_t nt = p.size();
  if (nt == 0) return;
  SXE_CHECK(g.size() == nt && m.size() == nt && v.size() == nt, "multi_tensor_adam_: list sizes");
  SXE_CHECK(lp.size() == 0 || lp.size() == nt, "multi_tensor_adam_: lp list size");
  const int64_t kChunk = 65536;
  std::vector<MTChunk> host;
  DT gd = dtype_of(g[0]);
  DT ld = lp.size() ? dtype_of(lp[0]) : DT::BF16;
  for (size_t i = 0; i < nt; ++i) {
    SXE_CHECK(p[i].scalar_type() == at::kFloat && p[i].is_contiguous() && g[i].is_contiguous() &&
                  m[i].is_contiguous() && v[i].is_contiguous(), "multi_tensor_adam_: fp32 contiguous");
    SXE_CHECK(dtype_of(g[i]) == gd, "multi_tensor_adam_: mixed grad dtypes");
    const int64_t n = p[i].numel();
    for (int64_t s = 0; s < n; s += kChunk) {
      MTChunk c;
      c.p = p[i].data_ptr<float>() + s;
      c.g = static_cast<const char*>(g[i].data_ptr()) + s * g[i].element_size();
      c.m = m[i].data_ptr<float>() + s;
      c.v = v[i].data_ptr<float>() + s;
      c.lp = lp.size() ? static_cast<char*>(lp[i].data_ptr()) + s * lp[i].element_size() : nullptr;
      c.n = std::min(kChunk, n - s);
      host.push_back(c);
    }
  }
  if (host.empty()) return;
  c10::DeviceGuard guard(p[0].device());
  auto bytes = (int64_t)(host.size() * sizeof(MTChunk));
  auto h = at::empty({bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  std::memcpy(h.data_ptr(), host.data(), bytes);
  auto d = h.to(p[0].device(), /*non_blocking=*/true);
  AdamHP hp = make_hp(lr, beta1, beta2, eps, weight_decay, step, adamw, bias_correction);
  const float* sp = opt_f32_ptr(scale_t);
  const float* kp = opt_f32_ptr(skip_t);
  SXE_DISPATCH_DT(gd, GT, SXE_DISPATCH_DT(ld, LT, {
    hipLaunchKernelGGL((adam_mt_kernel<GT, LT>), dim3(host.size()), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const MTChunk*>(d.data_ptr()), hp, (float)grad_scale, sp, kp);
  }));
  SXE_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Lion (reference deepspeed/ops/lion/fused_lion.py): u = sign(b1*m + (1-b1)*g); p -= lr*(u + wd*p);
// m = b2*m + (1-b2)*g.
template <DT G, DT L>
__global__ void __launch_bounds__(256) lion_flat_kernel(float* __restrict__ p, const typename dt_traits<G>::storage* __restrict__ g,
                                                        float* __restrict__ m, typename dt_traits<L>::storage* __restrict__ lp,
                                                        int64_t n, float lr, float b1, float b2, float wd, float gscale,
                                                        const float* __restrict__ scale_t, const float* __restrict__ skip_t) {
  if (skip_t && *skip_t != 0.f) return;
  if (scale_t) gscale *= *scale_t;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gi = to_f32<G>(g[i]) * gscale, mi = m[i], pi = p[i];
    float c = b1 * mi + (1.f - b1) * gi;
    float u = (c > 0.f) ? 1.f : ((c < 0.f) ? -1.f : 0.f);
    pi -= lr * (u + wd * pi);
    m[i] = b2 * mi + (1.f - b2) * gi;
    p[i] = pi;
    if (lp) lp[i] = from_f32<L>(pi);
  }
}

void lion_flat_(at::Tensor p, at::Tensor g, at::Tensor m, c10::optional<at::Tensor> lp, c10::optional<at::Tensor> scale_t,
                c10::optional<at::Tensor> skip_t, double lr, double beta1, double beta2, double weight_decay,
                double grad_scale) {
  SXE_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat, "lion_flat_: fp32 master/state");
  const int64_t n = p.numel();
  if (n == 0) return;
  const bool has_lp = lp.has_value() && lp->defined();
  c10::DeviceGuard guard(p.device());
  DT gd = dtype_of(g);
  DT ld = has_lp ? dtype_of(*lp) : DT::BF16;
  SXE_DISPATCH_DT(gd, GT, SXE_DISPATCH_DT(ld, LT, {
    using GS = typename dt_traits<GT>::storage;
    using LS = typename dt_traits<LT>::storage;
    hipLaunchKernelGGL((lion_flat_kernel<GT, LT>), dim3(stream_grid(n, 256)), dim3(256), 0, cur_stream(),
                       p.data_ptr<float>(), reinterpret_cast<const GS*>(g.data_ptr()), m.data_ptr<float>(),
                       has_lp ? reinterpret_cast<LS*>(lp->data_ptr()) : nullptr, n, (float)lr, (float)beta1,
                       (float)beta2, (float)weight_decay, (float)grad_scale, opt_f32_ptr(scale_t), opt_f32_ptr(skip_t));
  }));
  SXE_LAUNCH_CHECK();
}

// Adagrad (reference deepspeed/ops/adagrad/cpu_adagrad.py): s += g^2; p -= lr * g / (sqrt(s) + eps).
template <DT G, DT L>
__global__ void __launch_bounds__(256) adagrad_flat_kernel(float* __restrict__ p, const typename dt_traits<G>::storage* __restrict__ g,
                                                           float* __restrict__ s, typename dt_traits<L>::storage* __restrict__ lp,
                                                           int64_t n, float lr, float eps, float wd, float gscale,
                                                           const float* __restrict__ scale_t, const float* __restrict__ skip_t) {
  if (skip_t && *skip_t != 0.f) return;
  if (scale_t) gscale *= *scale_t;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pi = p[i];
    float gi = to_f32<G>(g[i]) * gscale + wd * pi;
    float si = s[i] + gi * gi;
    pi -= lr * gi / (sqrtf(si) + eps);
    s[i] = si; p[i] = pi;
    if (lp) lp[i] = from_f32<L>(pi);
  }
}

void adagrad_flat_(at::Tensor p, at::Tensor g, at::Tensor s, c10::optional<at::Tensor> lp, c10::optional<at::Tensor> scale_t,
                   c10::optional<at::Tensor> skip_t, double lr, double eps, double weight_decay, double grad_scale) {
  const int64_t n = p.numel();
  if (n == 0) return;
  const bool has_lp = lp.has_value() && lp->defined();
  c10::DeviceGuard guard(p.device());
  DT gd = dtype_of(g);
  DT ld = has_lp ? dtype_of(*lp) : DT::BF16;
  SXE_DISPATCH_DT(gd, GT, SXE_DISPATCH_DT(ld, LT, {
    using GS = typename dt_traits<GT>::storage;
    using LS = typename dt_traits<LT>::storage;
    hipLaunchKernelGGL((adagrad_flat_kernel<GT, LT>), dim3(stream_grid(n, 256)), dim3(256), 0, cur_stream(),
                       p.data_ptr<float>(), reinterpret_cast<const GS*>(g.data_ptr()), s.data_ptr<float>(),
                       has_lp ? reinterpret_cast<LS*>(lp->data_ptr()) : nullptr, n, (float)lr, (float)eps,
                       (float)weight_decay, (float)grad_scale, opt_f32_ptr(scale_t), opt_f32_ptr(skip_t));
  }));
  SXE_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Sum of squares of a flat buffer (any float dtype) into per-block fp32 partials; inf/NaN
// propagate naturally, so the caller gets the overflow check for free from the same pass.
template <DT T>
__global__ void __launch_bounds__(256) sumsq_kernel(const typename dt_traits<T>::storage* __restrict__ x, int64_t n,
                                                    float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n8 = n >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8];
    load8<T>(x + (i << 3), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    float t = to_f32<T>(x[(n8 << 3) + threadIdx.x]);
    acc += t * t;
  }
  acc = block_sum<4>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

at::Tensor sumsq(at::Tensor x) {
  SXE_CHECK(x.is_contiguous(), "sumsq: contiguous");
  const int64_t n = x.numel();
  c10::DeviceGuard guard(x.device());
  const int grid = std::min<int64_t>(stream_grid((n + 7) / 8, 256), 1024);
  auto partial = at::empty({grid}, x.options().dtype(at::kFloat));
  SXE_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, "sumsq: 16-byte alignment");
  DT d = dtype_of(x);
  SXE_DISPATCH_DT(d, T, {
    using S = typename dt_traits<T>::storage;
    hipLaunchKernelGGL((sumsq_kernel<T>), dim3(grid), dim3(256), 0, cur_stream(), reinterpret_cast<const S*>(x.data_ptr()),
                       n, partial.data_ptr<float>());
  });
  SXE_LAUNCH_CHECK();
  return partial.sum();
}

// ---------------------------------------------------------------------------------------------
// LAMB over a flat fp32 master with PER-PARAMETER trust ratios (reference ops/lamb/fused_lamb.py:14,
// csrc/lamb/fused_lamb_cuda_kernel.cu): the flat is cut into segments (this rank's fragment of each
// original parameter); `blk` maps every block to (segment, begin, end) so a block never straddles
// two parameters. Stage 1 updates m / v and accumulates, per segment, ||p||^2 and ||u||^2 of the
// Adam direction u = m^ / (sqrt(v^) + eps) + wd p into `sums` [nseg, 2] (one atomic per block and
// segment). The caller all-reduces `sums` over the partition group when a parameter is split across
// ranks, so the ratio is the whole parameter's. Stage 2 recomputes u (p, m, v unchanged since) and
// applies p -= lr * clamp(||p|| / ||u||, min_coeff, max_coeff) * u, writing the bit16 copy too.
struct LambHP {
  float lr, b1, b2, eps, wd, bc1, bc2, min_coeff, max_coeff;
};

template <DT G>
__global__ void __launch_bounds__(256) lamb_stage1_kernel(const float* __restrict__ p,
                                                          const typename dt_traits<G>::storage* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          const int64_t* __restrict__ blk, const int64_t* __restrict__ seg_id,
                                                          float* __restrict__ sums, LambHP hp, float gscale,
                                                          const float* __restrict__ scale_t, const float* __restrict__ skip_t) {
  __shared__ float red[4];
  if (skip_t && *skip_t != 0.f) return;
  if (scale_t) gscale *= *scale_t;
  const int64_t b0 = blk[2 * blockIdx.x], b1e = blk[2 * blockIdx.x + 1];
  float pn = 0.f, un = 0.f;
  for (int64_t i = b0 + threadIdx.x; i < b1e; i += blockDim.x) {
    const float gi = to_f32<G>(g[i]) * gscale;
    const float mi = hp.b1 * m[i] + (1.f - hp.b1) * gi;
    const float vi = hp.b2 * v[i] + (1.f - hp.b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float pi = p[i];
    const float u = (mi / hp.bc1) / (sqrtf(vi / hp.bc2) + hp.eps) + hp.wd * pi;
    pn += pi * pi;
    un += u * u;
  }
  pn = block_sum<4>(pn, red);
  un = block_sum<4>(un, red);
  if (threadIdx.x == 0) {
    const int64_t sidx = seg_id[blockIdx.x];
    atomicAdd(sums + 2 * sidx, pn);
    atomicAdd(sums + 2 * sidx + 1, un);
  }
}

template <DT L>
__global__ void __launch_bounds__(256) lamb_stage2_kernel(float* __restrict__ p, const float* __restrict__ m,
                                                          const float* __restrict__ v,
                                                          typename dt_traits<L>::storage* __restrict__ lp,
                                                          const int64_t* __restrict__ blk, const int64_t* __restrict__ seg_id,
                                                          const float* __restrict__ sums, float* __restrict__ coeffs,
                                                          LambHP hp, const float* __restrict__ skip_t) {
  if (skip_t && *skip_t != 0.f) return;
  const int64_t sidx = seg_id[blockIdx.x];
  const float wn = sqrtf(sums[2 * sidx]), un = sqrtf(sums[2 * sidx + 1]);
  float coeff = (wn > 0.f && un > 0.f) ? wn / un : 1.f;
  coeff = fminf(fmaxf(coeff, hp.min_coeff), hp.max_coeff);
  if (coeffs && threadIdx.x == 0) coeffs[sidx] = coeff;
  const float step = hp.lr * coeff;
  const int64_t b0 = blk[2 * blockIdx.x], b1e = blk[2 * blockIdx.x + 1];
  for (int64_t i = b0 + threadIdx.x; i < b1e; i += blockDim.x) {
    const float pi = p[i];
    const float u = (m[i] / hp.bc1) / (sqrtf(v[i] / hp.bc2) + hp.eps) + hp.wd * pi;
    const float np = pi - step * u;
    p[i] = np;
    if (lp) lp[i] = from_f32<L>(np);
  }
}

// blk: [nblk, 2] int64 (begin, end) element ranges, seg_id: [nblk] int64, sums: [nseg, 2] fp32 (zeroed)
void lamb_stage1_(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor blk, at::Tensor seg_id,
                  at::Tensor sums, c10::optional<at::Tensor> scale_t, c10::optional<at::Tensor> skip_t, double lr,
                  double b1, double b2, double eps, double wd, double bc1, double bc2, double grad_scale) {
  SXE_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat &&
                sums.scalar_type() == at::kFloat && blk.scalar_type() == at::kLong && seg_id.scalar_type() == at::kLong,
            "lamb_stage1_: dtypes");
  const int64_t nblk = seg_id.numel();
  if (nblk == 0) return;
  c10::DeviceGuard guard(p.device());
  LambHP hp{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2, 0.f, 0.f};
  SXE_DISPATCH_DT(dtype_of(g), GT, {
    using GS = typename dt_traits<GT>::storage;
    hipLaunchKernelGGL((lamb_stage1_kernel<GT>), dim3(nblk), dim3(256), 0, cur_stream(), p.data_ptr<float>(),
                       reinterpret_cast<const GS*>(g.data_ptr()), m.data_ptr<float>(), v.data_ptr<float>(),
                       blk.data_ptr<int64_t>(), seg_id.data_ptr<int64_t>(), sums.data_ptr<float>(), hp,
                       (float)grad_scale, opt_f32_ptr(scale_t), opt_f32_ptr(skip_t));
  });
  SXE_LAUNCH_CHECK();
}

void lamb_stage2_(at::Tensor p, at::Tensor m, at::Tensor v, c10::optional<at::Tensor> lp, at::Tensor blk,
                  at::Tensor seg_id, at::Tensor sums, c10::optional<at::Tensor> coeffs, c10::optional<at::Tensor> skip_t,
                  double lr, double eps, double wd, double bc1, double bc2, double min_coeff, double max_coeff) {
  const int64_t nblk = seg_id.numel();
  if (nblk == 0) return;
  const bool has_lp = lp.has_value() && lp->defined();
  c10::DeviceGuard guard(p.device());
  LambHP hp{(float)lr, 0.f, 0.f, (float)eps, (float)wd, (float)bc1, (float)bc2, (float)min_coeff, (float)max_coeff};
  float* cp = (coeffs.has_value() && coeffs->defined()) ? coeffs->data_ptr<float>() : nullptr;
  DT ld = has_lp ? dtype_of(*lp) : DT::BF16;
  SXE_DISPATCH_DT(ld, LT, {
    using LS = typename dt_traits<LT>::storage;
    hipLaunchKernelGGL((lamb_stage2_kernel<LT>), dim3(nblk), dim3(256), 0, cur_stream(), p.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), has_lp ? reinterpret_cast<LS*>(lp->data_ptr()) : nullptr,
                       blk.data_ptr<int64_t>(), seg_id.data_ptr<int64_t>(), sums.data_ptr<float>(), cp, hp,
                       opt_f32_ptr(skip_t));
  });
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("adam_flat_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? lp, Tensor? scale, Tensor? skip, "
        "float lr, float beta1, float beta2, float eps, float weight_decay, int step, bool adamw, bool bias_correction, "
        "float grad_scale) -> ()");
  m.def("multi_tensor_adam_(Tensor(a!)[] p, Tensor[] g, Tensor(b!)[] m, Tensor(c!)[] v, Tensor(d!)[] lp, Tensor? scale, "
        "Tensor? skip, float lr, float beta1, float beta2, float eps, float weight_decay, int step, bool adamw, "
        "bool bias_correction, float grad_scale) -> ()");
  m.def("lion_flat_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(d!)? lp, Tensor? scale, Tensor? skip, float lr, "
        "float beta1, float beta2, float weight_decay, float grad_scale) -> ()");
  m.def("adagrad_flat_(Tensor(a!) p, Tensor g, Tensor(b!) s, Tensor(d!)? lp, Tensor? scale, Tensor? skip, float lr, "
        "float eps, float weight_decay, float grad_scale) -> ()");
  m.def("sumsq(Tensor x) -> Tensor");
  m.def("lamb_stage1_(Tensor p, Tensor g, Tensor(a!) m, Tensor(b!) v, Tensor blk, Tensor seg_id, Tensor(c!) sums, "
        "Tensor? scale, Tensor? skip, float lr, float beta1, float beta2, float eps, float weight_decay, float bc1, "
        "float bc2, float grad_scale) -> ()");
  m.def("lamb_stage2_(Tensor(a!) p, Tensor m, Tensor v, Tensor(b!)? lp, Tensor blk, Tensor seg_id, Tensor sums, "
        "Tensor(c!)? coeffs, Tensor? skip, float lr, float eps, float weight_decay, float bc1, float bc2, "
        "float min_coeff, float max_coeff) -> ()");
}

TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("adam_flat_", &sxe::adam_flat_);
  m.impl("multi_tensor_adam_", &sxe::multi_tensor_adam_);
  m.impl("lion_flat_", &sxe::lion_flat_);
  m.impl("adagrad_flat_", &sxe::adagrad_flat_);
  m.impl("sumsq", &sxe::sumsq);
  m.impl("lamb_stage1_", &sxe::lamb_stage1_);
  m.impl("lamb_stage2_", &sxe::lamb_stage2_);
}

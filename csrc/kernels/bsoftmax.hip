// Block-sparse row softmax for gfx950 (MI355X): the reference's ops/sparse_attention/softmax.py:37
// ``Softmax`` (Triton forward / backward kernels over the non-zero blocks of a layout [H, M, N]).
// Scores are in the reference's sparse format [B, nnz, blk, blk] (blocks in layout.nonzero() order,
// so the blocks of one block row (h, i) are contiguous: a CSR row pointer `ptr` [H M + 1] and the
// block column `col` [nnz] describe them). A softmax row is one query row r of a block row: the
// r-th rows of all its blocks, i.e. up to N blk keys.
//
//   forward   s = x * scale (+ rpe) (+|* attn_mask) (+|* key_padding_mask);  y = softmax_row(s)
//   backward  dx = y (dy - sum_row(dy y)) * ds/dx,   ds/dx = scale (* attn_mask) (* key_padding_mask)
//
// One workgroup per (block row, batch), one wave per query row (4 waves stride over the blk rows);
// each lane takes 8 consecutive keys at a time (16-byte loads of x, 32-byte loads of the fp32
// rpe / masks), three sweeps over the row (max, sum of exponentials, normalised write), the row's
// data L2-resident after the first. A fully masked row writes zeros (as the PyTorch path does).
#include "sxe_common.h"

#include <torch/library.h>

namespace sxe {
namespace bsf {

struct Args {
  const int* ptr;
  const int* col;
  int M, blk, scols;   // scols = N * blk: row length of the dense [S, S] rpe / mask images
  int64_t nnz;
  float scale;
  const float* rpe;    // [(B,) H, S, S] fp32 or null
  int64_t rpe_bs, rpe_hs;
  const float* am;     // [S, S] fp32 or null
  const float* kpm;    // [B, S] fp32 or null
  int am_mul, kpm_mul;
};

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[4 + e] = b[e];
  }
}

// the 8 scores s[c0 .. c0+7] of row r of block n (column block j) of block row (h, i), batch b
template <DT T>
__device__ __forceinline__ void scores8(const typename dt_traits<T>::storage* __restrict__ x, const Args& a, int b,
                                        int h, int i, int r, int n, int c0, float (&s)[8]) {
  load8<T>(x + (((int64_t)b * a.nnz + n) * a.blk + r) * a.blk + c0, s);
  const int j = a.col[n];
  const int64_t row = (int64_t)(i * a.blk + r) * a.scols + (int64_t)j * a.blk + c0;
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] *= a.scale;
  float t[8];
  if (a.rpe != nullptr) {
    ld8f(a.rpe + b * a.rpe_bs + h * a.rpe_hs + row, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += t[e];
  }
  if (a.am != nullptr) {
    ld8f(a.am + row, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = a.am_mul ? s[e] * t[e] : s[e] + t[e];
  }
  if (a.kpm != nullptr) {
    ld8f(a.kpm + (int64_t)b * a.scols + (int64_t)j * a.blk + c0, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = a.kpm_mul ? s[e] * t[e] : s[e] + t[e];
  }
}

template <DT T>
__global__ __launch_bounds__(256) void fwd_kernel(const typename dt_traits<T>::storage* __restrict__ x,
                                                  typename dt_traits<T>::storage* __restrict__ y, Args a) {
  const int g = blockIdx.x, b = blockIdx.y, h = g / a.M, i = g - h * a.M;
  const int p0 = a.ptr[g], cpr = a.blk / 8, total = (a.ptr[g + 1] - p0) * cpr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = wave; r < a.blk; r += 4) {
    float mx = -INFINITY;
    for (int idx = lane; idx < total; idx += 64) {
      float s[8];
      scores8<T>(x, a, b, h, i, r, p0 + idx / cpr, (idx % cpr) * 8, s);
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = fmaxf(mx, s[e]);
    }
    mx = wave_max(mx);
    const float mref = mx == -INFINITY ? 0.f : mx;
    float sum = 0.f;
    for (int idx = lane; idx < total; idx += 64) {
      float s[8];
      scores8<T>(x, a, b, h, i, r, p0 + idx / cpr, (idx % cpr) * 8, s);
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += expf(s[e] - mref);
    }
    sum = wave_sum(sum);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    for (int idx = lane; idx < total; idx += 64) {
      const int n = p0 + idx / cpr, c0 = (idx % cpr) * 8;
      float s[8];
      scores8<T>(x, a, b, h, i, r, n, c0, s);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] = expf(s[e] - mref) * inv;
      store8<T>(y + (((int64_t)b * a.nnz + n) * a.blk + r) * a.blk + c0, s);
    }
  }
}

template <DT T>
__global__ __launch_bounds__(256) void bwd_kernel(const typename dt_traits<T>::storage* __restrict__ y,
                                                  const typename dt_traits<T>::storage* __restrict__ dy,
                                                  typename dt_traits<T>::storage* __restrict__ dx, Args a) {
  const int g = blockIdx.x, b = blockIdx.y, i = g % a.M;
  const int p0 = a.ptr[g], cpr = a.blk / 8, total = (a.ptr[g + 1] - p0) * cpr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = wave; r < a.blk; r += 4) {
    float dot = 0.f;
    for (int idx = lane; idx < total; idx += 64) {
      const int64_t off = (((int64_t)b * a.nnz + p0 + idx / cpr) * a.blk + r) * a.blk + (idx % cpr) * 8;
      float yv[8], gv[8];
      load8<T>(y + off, yv);
      load8<T>(dy + off, gv);
#pragma unroll
      for (int e = 0; e < 8; ++e) dot += yv[e] * gv[e];
    }
    dot = wave_sum(dot);
    for (int idx = lane; idx < total; idx += 64) {
      const int n = p0 + idx / cpr, c0 = (idx % cpr) * 8;
      const int64_t off = (((int64_t)b * a.nnz + n) * a.blk + r) * a.blk + c0;
      float yv[8], gv[8], d[8];
      load8<T>(y + off, yv);
      load8<T>(dy + off, gv);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = yv[e] * (gv[e] - dot) * a.scale;
      const int j = a.col[n];
      float t[8];
      if (a.am != nullptr && a.am_mul) {
        ld8f(a.am + (int64_t)(i * a.blk + r) * a.scols + (int64_t)j * a.blk + c0, t);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] *= t[e];
      }
      if (a.kpm != nullptr && a.kpm_mul) {
        ld8f(a.kpm + (int64_t)b * a.scols + (int64_t)j * a.blk + c0, t);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] *= t[e];
      }
      store8<T>(dx + off, d);
    }
  }
}

static Args make_args(const at::Tensor& x, const at::Tensor& ptr, const at::Tensor& col, int64_t H, int64_t M,
                      int64_t N, double scale, const c10::optional<at::Tensor>& rpe,
                      const c10::optional<at::Tensor>& am, bool am_mul, const c10::optional<at::Tensor>& kpm,
                      bool kpm_mul) {
  SXE_CHECK(x.dim() == 4 && x.is_contiguous() && x.size(2) == x.size(3), "block-sparse softmax: x [B, nnz, blk, blk]");
  const int64_t blk = x.size(2), S = N * blk;
  SXE_CHECK(blk % 8 == 0, "block-sparse softmax: block must be a multiple of 8");
  SXE_CHECK(ptr.scalar_type() == at::kInt && ptr.is_contiguous() && ptr.numel() == H * M + 1,
            "block-sparse softmax: ptr int32 [H * M + 1]");
  SXE_CHECK(col.scalar_type() == at::kInt && col.is_contiguous() && col.numel() == x.size(1),
            "block-sparse softmax: col int32 [nnz]");
  Args a;
  a.ptr = ptr.data_ptr<int>();
  a.col = col.data_ptr<int>();
  a.M = (int)M;
  a.blk = (int)blk;
  a.scols = (int)S;
  a.nnz = x.size(1);
  a.scale = (float)scale;
  a.rpe = nullptr;
  a.rpe_bs = a.rpe_hs = 0;
  if (rpe.has_value()) {
    const at::Tensor& t = *rpe;
    SXE_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && (t.dim() == 3 || t.dim() == 4) &&
                  t.size(-1) == S && t.size(-2) == S && (t.size(-3) == 1 || t.size(-3) == H) &&
                  (t.dim() == 3 || t.size(0) == 1 || t.size(0) == x.size(0)),
              "block-sparse softmax: rpe fp32 [(B,) H or 1, S, S]");
    a.rpe = t.data_ptr<float>();
    a.rpe_hs = t.size(-3) > 1 ? S * S : 0;
    a.rpe_bs = (t.dim() == 4 && t.size(0) > 1) ? t.size(-3) * S * S : 0;
  }
  a.am = nullptr;
  if (am.has_value()) {
    SXE_CHECK(am->scalar_type() == at::kFloat && am->is_contiguous() && am->numel() == S * S,
              "block-sparse softmax: attn_mask fp32 [S, S]");
    a.am = am->data_ptr<float>();
  }
  a.kpm = nullptr;
  if (kpm.has_value()) {
    SXE_CHECK(kpm->scalar_type() == at::kFloat && kpm->is_contiguous() && kpm->numel() == x.size(0) * S,
              "block-sparse softmax: key_padding_mask fp32 [B, S]");
    a.kpm = kpm->data_ptr<float>();
  }
  a.am_mul = am_mul ? 1 : 0;
  a.kpm_mul = kpm_mul ? 1 : 0;
  return a;
}

}  // namespace bsf

at::Tensor bsparse_softmax_fwd(at::Tensor x, at::Tensor ptr, at::Tensor col, int64_t H, int64_t M, int64_t N,
                               double scale, c10::optional<at::Tensor> rpe, c10::optional<at::Tensor> am,
                               bool am_mul, c10::optional<at::Tensor> kpm, bool kpm_mul) {
  SXE_CHECK_CUDA(x);
  c10::DeviceGuard guard(x.device());
  bsf::Args a = bsf::make_args(x, ptr, col, H, M, N, scale, rpe, am, am_mul, kpm, kpm_mul);
  auto y = at::empty_like(x);
  if (x.numel() == 0 || H * M == 0) return y;
  const dim3 grid((unsigned)(H * M), (unsigned)x.size(0));
  SXE_DISPATCH_DT(dtype_of(x), T, {
    using S = typename dt_traits<T>::storage;
    hipLaunchKernelGGL(bsf::fwd_kernel<T>, grid, dim3(256), 0, cur_stream(), reinterpret_cast<const S*>(x.data_ptr()),
                       reinterpret_cast<S*>(y.data_ptr()), a);
  });
  SXE_LAUNCH_CHECK();
  return y;
}

at::Tensor bsparse_softmax_bwd(at::Tensor y, at::Tensor dy, at::Tensor ptr, at::Tensor col, int64_t H, int64_t M,
                               int64_t N, double scale, c10::optional<at::Tensor> am, bool am_mul,
                               c10::optional<at::Tensor> kpm, bool kpm_mul) {
  SXE_CHECK_CUDA(y);
  SXE_CHECK(dy.sizes() == y.sizes() && dy.scalar_type() == y.scalar_type() && dy.is_contiguous(),
            "block-sparse softmax backward: dy like y");
  c10::DeviceGuard guard(y.device());
  bsf::Args a = bsf::make_args(y, ptr, col, H, M, N, scale, c10::nullopt, am, am_mul, kpm, kpm_mul);
  auto dx = at::empty_like(y);
  if (y.numel() == 0 || H * M == 0) return dx;
  const dim3 grid((unsigned)(H * M), (unsigned)y.size(0));
  SXE_DISPATCH_DT(dtype_of(y), T, {
    using S = typename dt_traits<T>::storage;
    hipLaunchKernelGGL(bsf::bwd_kernel<T>, grid, dim3(256), 0, cur_stream(), reinterpret_cast<const S*>(y.data_ptr()),
                       reinterpret_cast<const S*>(dy.data_ptr()), reinterpret_cast<S*>(dx.data_ptr()), a);
  });
  SXE_LAUNCH_CHECK();
  return dx;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("bsparse_softmax_fwd(Tensor x, Tensor ptr, Tensor col, int H, int M, int N, float scale, Tensor? rpe, "
        "Tensor? am, bool am_mul, Tensor? kpm, bool kpm_mul) -> Tensor");
  m.def("bsparse_softmax_bwd(Tensor y, Tensor dy, Tensor ptr, Tensor col, int H, int M, int N, float scale, "
        "Tensor? am, bool am_mul, Tensor? kpm, bool kpm_mul) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("bsparse_softmax_fwd", &sxe::bsparse_softmax_fwd);
  m.impl("bsparse_softmax_bwd", &sxe::bsparse_softmax_bwd);
}

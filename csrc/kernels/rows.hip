// Row gather / scatter over 16-byte chunks: the one memory pattern behind several reference ops,
// done as one gfx950 kernel pair instead of a PyTorch index op per site.
//
//  * gather_rows(src [R, W], idx [N], offset, add) -> out [N, W]:
//      out[i] = src[idx[i] - offset] (+ add[idx[i] - offset]); an index outside [0, R) gives a zero
//      row. Users: ragged embedding lookup (reference inference/v2/kernels/ragged_ops/embed/
//      embed.cu:21; with ``offset`` = a vocab shard's first id, out-of-shard tokens read zero, as in
//      a vocab-parallel embedding), last-token logits gather (ragged_ops/logits_gather/
//      logits_gather.cu:20; ``add`` folds the fused-residual sum x + res into the gather), and the
//      random-LTD token gather (ops/random_ltd/gather_scatter.cu:22).
//  * scatter_rows_(dst [R, W], idx [N], src [N, W]): dst[idx[i]] = src[i] (indices unique):
//      the random-LTD scatter back into the full sequence (gather_scatter.cu:72) and the backward of
//      a unique-index gather.
//
// One wave per row and 16 bytes per lane per access (Guideline 13): a 4 KiB bf16 row (H = 2048)
// is 4 wave-instructions of 1 KiB, each fully coalesced. Rows are opaque bytes, so every dtype
// uses the same code; only ``add`` (an elementwise sum) needs the type.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace rows {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename I, DT T, bool ADD>
__global__ void __launch_bounds__(256) gather_kernel(const u32x4* __restrict__ src, const u32x4* __restrict__ add,
                                                     const I* __restrict__ idx, u32x4* __restrict__ out, int64_t N,
                                                     int64_t R, int64_t offset, int chunks) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < N; row += (int64_t)gridDim.x * 4) {
    const int64_t s = (int64_t)idx[row] - offset;
    const bool ok = s >= 0 && s < R;
    u32x4* o = out + row * chunks;
    const u32x4* a = src + (ok ? s : 0) * chunks;
    const u32x4* b = ADD ? add + (ok ? s : 0) * chunks : nullptr;
    for (int c = lane; c < chunks; c += 64) {
      u32x4 v = ok ? a[c] : u32x4{0u, 0u, 0u, 0u};
      if constexpr (ADD) {
        if (ok) {
          float x[8], y[8];
          using S = typename dt_traits<T>::storage;
          constexpr int E = 16 / sizeof(S);  // elements per chunk: 8 (16-bit) or 4 (f32)
          const S* pa = reinterpret_cast<const S*>(&v);
          const u32x4 w = b[c];
          const S* pb = reinterpret_cast<const S*>(&w);
          S r[E];
#pragma unroll
          for (int e = 0; e < E; ++e) {
            x[e] = to_f32<T>(pa[e]);
            y[e] = to_f32<T>(pb[e]);
            r[e] = from_f32<T>(x[e] + y[e]);
          }
          v = *reinterpret_cast<const u32x4*>(r);
        }
      }
      o[c] = v;
    }
  }
}

template <typename I>
__global__ void __launch_bounds__(256) scatter_kernel(u32x4* __restrict__ dst, const I* __restrict__ idx,
                                                      const u32x4* __restrict__ src, int64_t N, int64_t R, int chunks) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < N; row += (int64_t)gridDim.x * 4) {
    const int64_t d = (int64_t)idx[row];
    if (d < 0 || d >= R) continue;  // wave-uniform: the whole wave skips the row
    u32x4* o = dst + d * chunks;
    const u32x4* a = src + row * chunks;
    for (int c = lane; c < chunks; c += 64) o[c] = a[c];
  }
}

}  // namespace rows

static int row_chunks(const at::Tensor& t, const char* what) {
  SXE_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) == t.size(1), what, ": contiguous [rows, width]");
  const int64_t bytes = t.size(1) * t.element_size();
  SXE_CHECK(bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what,
            ": row bytes a multiple of 16 and a 16-byte aligned base");
  return (int)(bytes / 16);
}

static int rows_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, 8 * kNumCUs)); }

at::Tensor gather_rows(const at::Tensor& src, const at::Tensor& idx, int64_t offset, const c10::optional<at::Tensor>& add) {
  SXE_CHECK_CUDA(src);
  const int chunks = row_chunks(src, "gather_rows src");
  SXE_CHECK(idx.dim() == 1 && idx.is_contiguous() && (idx.scalar_type() == at::kLong || idx.scalar_type() == at::kInt),
            "gather_rows: idx int32/int64 [N]");
  const bool has_add = add.has_value() && add->defined();
  if (has_add) {
    SXE_CHECK(add->sizes() == src.sizes() && add->scalar_type() == src.scalar_type(), "gather_rows: add like src");
    row_chunks(*add, "gather_rows add");
  }
  const int64_t N = idx.numel(), R = src.size(0);
  auto out = at::empty({N, src.size(1)}, src.options());
  if (N == 0) return out;
  c10::DeviceGuard g(src.device());
  auto* s = reinterpret_cast<const rows::u32x4*>(src.data_ptr());
  auto* a = has_add ? reinterpret_cast<const rows::u32x4*>(add->data_ptr()) : nullptr;
  auto* o = reinterpret_cast<rows::u32x4*>(out.data_ptr());
  const dim3 grid(rows_grid(N)), block(256);
  auto launch = [&](auto ip) {
    using I = std::remove_const_t<std::remove_pointer_t<decltype(ip)>>;
    if (!has_add) {
      hipLaunchKernelGGL((rows::gather_kernel<I, DT::BF16, false>), grid, block, 0, cur_stream(), s, a, ip, o, N, R,
                         offset, chunks);
    } else if (src.scalar_type() == at::kFloat) {
      hipLaunchKernelGGL((rows::gather_kernel<I, DT::F32, true>), grid, block, 0, cur_stream(), s, a, ip, o, N, R,
                         offset, chunks);
    } else if (src.scalar_type() == at::kBFloat16) {
      hipLaunchKernelGGL((rows::gather_kernel<I, DT::BF16, true>), grid, block, 0, cur_stream(), s, a, ip, o, N, R,
                         offset, chunks);
    } else {
      SXE_CHECK(src.scalar_type() == at::kHalf, "gather_rows add: fp32 / bf16 / fp16");
      hipLaunchKernelGGL((rows::gather_kernel<I, DT::F16, true>), grid, block, 0, cur_stream(), s, a, ip, o, N, R,
                         offset, chunks);
    }
  };
  if (idx.scalar_type() == at::kLong) launch(idx.data_ptr<int64_t>());
  else launch(idx.data_ptr<int32_t>());
  SXE_LAUNCH_CHECK();
  return out;
}

void scatter_rows_(at::Tensor dst, const at::Tensor& idx, const at::Tensor& src) {
  SXE_CHECK_CUDA(dst);
  const int chunks = row_chunks(dst, "scatter_rows dst");
  SXE_CHECK(row_chunks(src, "scatter_rows src") == chunks && src.scalar_type() == dst.scalar_type(),
            "scatter_rows: src rows like dst rows");
  SXE_CHECK(idx.dim() == 1 && idx.is_contiguous() && idx.numel() == src.size(0) &&
                (idx.scalar_type() == at::kLong || idx.scalar_type() == at::kInt),
            "scatter_rows: idx int32/int64 [src rows]");
  const int64_t N = idx.numel();
  if (N == 0) return;
  c10::DeviceGuard g(dst.device());
  auto* d = reinterpret_cast<rows::u32x4*>(dst.data_ptr());
  auto* s = reinterpret_cast<const rows::u32x4*>(src.data_ptr());
  if (idx.scalar_type() == at::kLong)
    hipLaunchKernelGGL(rows::scatter_kernel<int64_t>, dim3(rows_grid(N)), dim3(256), 0, cur_stream(), d,
                       idx.data_ptr<int64_t>(), s, N, dst.size(0), chunks);
  else
    hipLaunchKernelGGL(rows::scatter_kernel<int32_t>, dim3(rows_grid(N)), dim3(256), 0, cur_stream(), d,
                       idx.data_ptr<int32_t>(), s, N, dst.size(0), chunks);
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("gather_rows(Tensor src, Tensor idx, int offset=0, Tensor? add=None) -> Tensor");
  m.def("scatter_rows_(Tensor(a!) dst, Tensor idx, Tensor src) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("gather_rows", &sxe::gather_rows);
  m.impl("scatter_rows_", &sxe::scatter_rows_);
}

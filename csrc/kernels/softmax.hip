// Masked attention softmax for the inference op layer (reference ops/transformer/inference/triton/
// softmax.py and csrc/transformer/inference/csrc/softmax.cu: scale, additive or boolean mask, ALiBi
// bias, causal and local-window masking, fp32 math on 16-bit scores).
//
// scores [B, H, q, k] (row-contiguous last dim); mask / alibi are broadcast views passed by their
// four element strides (0 on broadcast dims), so [B, 1, 1, k] padding masks and [1, H, 1, k] ALiBi
// slopes are read in place. One wave per score row; two passes over the row (online max + sum,
// then normalise-and-store) -- rows of up to a few thousand keys stay in L2 between the passes.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace smx {

struct View4 {
  const void* p;  // nullptr = absent
  int64_t s0, s1, s2, s3;
};

template <DT T, int MASK>  // MASK: 0 none, 1 additive f32, 2 boolean (uint8, 0 = masked out)
__global__ void __launch_bounds__(256) softmax_kernel(const typename dt_traits<T>::storage* __restrict__ x,
                                                      typename dt_traits<T>::storage* __restrict__ y, int B, int H,
                                                      int Q, int K, float scale, View4 mask, View4 alibi, int causal,
                                                      int window) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = (int64_t)B * H * Q;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += (int64_t)gridDim.x * 4) {
    const int qi = (int)(row % Q);
    const int64_t bh = row / Q;
    const int h = (int)(bh % H), b = (int)(bh / H);
    const int qpos = K - Q + qi;  // absolute position of this query among the keys
    const auto* xr = x + row * K;
    auto* yr = y + row * K;
    auto val = [&](int j) -> float {
      if (causal && j > qpos) return -INFINITY;
      if (window > 0 && j <= qpos - window) return -INFINITY;
      float v = to_f32<T>(xr[j]) * scale;
      if (alibi.p) v += reinterpret_cast<const float*>(alibi.p)[b * alibi.s0 + h * alibi.s1 + qi * alibi.s2 + j * alibi.s3];
      if constexpr (MASK == 1)
        v += reinterpret_cast<const float*>(mask.p)[b * mask.s0 + h * mask.s1 + qi * mask.s2 + j * mask.s3];
      if constexpr (MASK == 2)
        if (!reinterpret_cast<const uint8_t*>(mask.p)[b * mask.s0 + h * mask.s1 + qi * mask.s2 + j * mask.s3])
          v = -INFINITY;
      return v;
    };
    float m = -INFINITY, l = 0.f;
    for (int j = lane; j < K; j += 64) {
      const float v = val(j);
      if (v > m) {
        l = l * __expf(m - v) + 1.f;
        m = v;
      } else if (v > -INFINITY) {
        l += __expf(v - m);
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float mo = __shfl_xor(m, off, 64), lo = __shfl_xor(l, off, 64);
      const float mn = fmaxf(m, mo);
      l = (m == -INFINITY ? 0.f : l * __expf(m - mn)) + (mo == -INFINITY ? 0.f : lo * __expf(mo - mn));
      m = mn;
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;  // a fully masked row outputs zeros
    for (int j = lane; j < K; j += 64) {
      const float v = val(j);
      yr[j] = from_f32<T>(v == -INFINITY ? 0.f : __expf(v - m) * inv);
    }
  }
}

}  // namespace smx

static smx::View4 view4(const c10::optional<at::Tensor>& t, const at::Tensor& like) {
  if (!t.has_value() || !t->defined()) return smx::View4{nullptr, 0, 0, 0, 0};
  SXE_CHECK(t->dim() == 4, "masked_softmax: mask / alibi must be 4-D broadcastable to scores");
  auto e = t->expand(like.sizes());
  return smx::View4{e.data_ptr(), e.stride(0), e.stride(1), e.stride(2), e.stride(3)};
}

at::Tensor masked_softmax(const at::Tensor& scores, double scale, const c10::optional<at::Tensor>& mask,
                          const c10::optional<at::Tensor>& alibi, bool causal, int64_t window) {
  SXE_CHECK_CUDA(scores);
  SXE_CHECK(scores.dim() == 4 && scores.is_contiguous(), "masked_softmax: contiguous [B, H, q, k] scores");
  const int B = scores.size(0), H = scores.size(1), Q = scores.size(2), K = scores.size(3);
  int kind = 0;
  if (mask.has_value() && mask->defined()) {
    SXE_CHECK(mask->scalar_type() == at::kFloat || mask->scalar_type() == at::kByte || mask->scalar_type() == at::kBool,
              "masked_softmax: mask fp32 (additive) or bool/uint8 (keep = nonzero)");
    kind = mask->scalar_type() == at::kFloat ? 1 : 2;
  }
  if (alibi.has_value() && alibi->defined()) SXE_CHECK(alibi->scalar_type() == at::kFloat, "masked_softmax: fp32 alibi");
  auto y = at::empty_like(scores);
  const int64_t rows = (int64_t)B * H * Q;
  if (rows == 0 || K == 0) return y;
  c10::DeviceGuard g(scores.device());
  const smx::View4 mv = view4(mask, scores), av = view4(alibi, scores);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, 16 * kNumCUs));
#define SXE_SMX(T, M)                                                                                          \
  hipLaunchKernelGGL((smx::softmax_kernel<T, M>), dim3(grid), dim3(256), 0, cur_stream(),                      \
                     reinterpret_cast<const typename dt_traits<T>::storage*>(scores.data_ptr()),              \
                     reinterpret_cast<typename dt_traits<T>::storage*>(y.data_ptr()), B, H, Q, K, (float)scale, mv, \
                     av, causal ? 1 : 0, (int)window)
#define SXE_SMX_T(T)         \
  if (kind == 0) SXE_SMX(T, 0); \
  else if (kind == 1) SXE_SMX(T, 1); \
  else SXE_SMX(T, 2);
  if (scores.scalar_type() == at::kFloat) {
    SXE_SMX_T(DT::F32)
  } else if (scores.scalar_type() == at::kBFloat16) {
    SXE_SMX_T(DT::BF16)
  } else {
    SXE_CHECK(scores.scalar_type() == at::kHalf, "masked_softmax: fp32 / bf16 / fp16 scores");
    SXE_SMX_T(DT::F16)
  }
#undef SXE_SMX_T
#undef SXE_SMX
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("masked_softmax(Tensor scores, float scale, Tensor? mask, Tensor? alibi, bool causal, int window) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("masked_softmax", &sxe::masked_softmax); }

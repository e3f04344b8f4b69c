// Rotary position embedding (rotate-half convention, Llama/Mistral/Mixtral) for gfx950,
// applied IN PLACE on the fused QKV projection output.
//
// Reference: the inference kernel kv_rotary_pos_kernel
// (deepspeed/inference/v2/kernels/ragged_ops/linear_blocked_kv_rotary/blocked_kv_rotary_cuda.cu:26)
// rotates q/k and scatters k/v into a paged cache; training uses the same math (Megatron's
// DistributedAttention applies RoPE after the Ulysses all-to-all, sequence/layer.py:429-432).
// MI355X-first layout: the QKV GEMM writes one [tokens, (Hq + 2*Hkv) * D] row per token; q-heads and
// k-heads are adjacent, so ONE launch rotates all Hq + Hkv heads of a token without any
// transpose, and the attention kernel consumes the same buffer through strides. cos/sin come
// from an fp32 table [max_pos, D/2] computed once on the host side (Appendix B: no on-device
// trig). Backward is the same kernel with sin negated (the rotation is orthogonal).
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {

// x: base pointer of token 0, head 0; token t, head h, dim d at x[t*tok_stride + h*head_stride + d]
// (head_stride > D: partial rotary -- only the first D dims of each head rotate, Phi/GPT-NeoX style).
// Each thread rotates 8 consecutive pairs (16-byte vectors from both halves of one head).
template <DT T>
__global__ void __launch_bounds__(256) rope_kernel(typename dt_traits<T>::storage* __restrict__ x, int64_t tokens,
                                                   int64_t tok_stride, int64_t head_stride, int nheads, int D,
                                                   const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t, const int64_t* __restrict__ pos,
                                                   int64_t seq_len, int64_t pos_offset, float sign) {
  const int half = D / 2;
  const int vec_per_head = half / 8;
  const int64_t per_tok = (int64_t)nheads * vec_per_head;
  const int64_t total = tokens * per_tok;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t t = i / per_tok;
    const int rem = (int)(i - t * per_tok);
    const int h = rem / vec_per_head;
    const int c = (rem - h * vec_per_head) * 8;
    const int64_t p = pos ? pos[t] : (t % seq_len) + pos_offset;
    typename dt_traits<T>::storage* base = x + t * tok_stride + (int64_t)h * head_stride;
    float a[8], b[8], cs[8], sn[8];
    load8<T>(base + c, a);
    load8<T>(base + half + c, b);
    load8<DT::F32>(cos_t + p * half + c, cs);
    load8<DT::F32>(sin_t + p * half + c, sn);
    float oa[8], ob[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sign * sn[j];
      oa[j] = a[j] * cs[j] - b[j] * s;
      ob[j] = b[j] * cs[j] + a[j] * s;
    }
    store8<T>(base + c, oa);
    store8<T>(base + half + c, ob);
  }
}

// x: [..., tokens, heads, D] view with unit stride on D, head stride >= D (a partial-rotary view
// x[..., :rot] of the full heads is allowed) and a uniform token stride.
void rope_(at::Tensor x, at::Tensor cos_t, at::Tensor sin_t, c10::optional<at::Tensor> pos, int64_t seq_len,
           int64_t pos_offset, bool inverse) {
  SXE_CHECK(x.dim() >= 3, "rope_: x must be [..., tokens, heads, D]");
  const int D = (int)x.size(-1);
  const int nheads = (int)x.size(-2);
  SXE_CHECK(D % 16 == 0, "rope_: head dim must be a multiple of 16");
  SXE_CHECK(x.stride(-1) == 1 && x.stride(-2) >= D && x.stride(-2) % 8 == 0,
            "rope_: unit stride on D, 16-byte aligned head stride >= D");
  const int64_t head_stride = x.stride(-2);
  const int64_t tok_stride = x.stride(-3);
  const int64_t tokens = x.numel() / ((int64_t)nheads * D);
  // tokens must be uniformly strided across the leading dims ([B, S] flattened).
  if (x.dim() > 3 && x.size(-4) > 1)
    SXE_CHECK(x.stride(-4) == tok_stride * x.size(-3), "rope_: leading dims must flatten uniformly");
  SXE_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                sin_t.is_contiguous() && cos_t.size(-1) == D / 2, "rope_: cos/sin tables must be fp32 [max_pos, D/2]");
  const bool hp = pos.has_value() && pos->defined();
  if (hp) {
    SXE_CHECK(pos->scalar_type() == at::kLong && pos->numel() == tokens && pos->is_contiguous(), "rope_: pos must be int64 [tokens]");
  } else {
    SXE_CHECK(seq_len > 0 && seq_len + pos_offset <= cos_t.size(0), "rope_: table too short for seq_len");
  }
  c10::DeviceGuard guard(x.device());
  if (tokens == 0) return;
  DT d = dtype_of(x);
  const int64_t work = tokens * nheads * (D / 16);
  SXE_DISPATCH_DT(d, TT, {
    using S = typename dt_traits<TT>::storage;
    hipLaunchKernelGGL((rope_kernel<TT>), dim3(stream_grid(work, 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<S*>(x.data_ptr()), tokens, tok_stride, head_stride, nheads, D,
                       cos_t.data_ptr<float>(),
                       sin_t.data_ptr<float>(), hp ? pos->data_ptr<int64_t>() : nullptr, seq_len > 0 ? seq_len : 1,
                       pos_offset, inverse ? -1.f : 1.f);
  });
  SXE_LAUNCH_CHECK();
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, Tensor? pos, int seq_len, int pos_offset, bool inverse) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("rope_", &sxe::rope_); }

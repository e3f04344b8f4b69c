// FP6 (e3m2) / FP4 (e2m1) weights on gfx950: group-scaled quantize / dequantize for the
// FP_Quantize API, and the decode-shaped weight-only GEMMs that stream 6- or 4-bit weights.
//
// Reference: ops/fp_quantizer (FP_Quantize, fp_quantize_impl.cu) and the FP6-LLM weight GEMM of
// inference/v2/kernels/core_ops/cuda_linear (linear_kernels_cuda.cu:70, 'wf6af16': fp6 weights,
// fp16 activations, one scale per output channel).
//
// Formats (MX element encodings, no inf/nan; codes are sign | magnitude index):
//   FP4 e2m1 magnitudes {0, .5, 1, 1.5, 2, 3, 4, 6}; FP6 e3m2 magnitudes m/16 (e = 0) and
//   (1 + m/4) 2^(e-3) (e = 1..7), max 28. Rounding: nearest, ties to the smaller magnitude
//   (identical to the PyTorch value-table path of ops/fp_quantizer.py).
//
// GEMM weight layouts (built by ops/fp_quantizer.pack_*; [N, K] row-major, per-row fp32 scale):
//   FP4: [N, K/2] bytes; in every 32-bit word (8 weights w0..w7) byte b = w_b | w_{b+4} << 4.
//   FP6: plane A [N, K/2] = the 4 high code bits (sign | e) in the FP4 word layout, plane B
//        [N, K/4] = the 2 mantissa bits; in every 32-bit word of B (16 weights) byte b holds
//        m(w_b) | m(w_{b+4}) << 2 | m(w_{b+8}) << 4 | m(w_{b+12}) << 6. 0.75 bytes per weight.
// Decode to bf16 in registers is byte-parallel: v_perm_b32 table lookups (8-entry byte tables of
// the bf16 high / low bytes), byte masks and v_bfi -- ~2 VALU per weight for FP4, ~4 for FP6 --
// so the kernel stays HBM-bound while reading 1/4 (FP4) or 3/8 (FP6) of the bf16 bytes.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace mx {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

// ---------------------------------------------------------------------------- element codecs
__device__ __forceinline__ int fp4_index(float a) {  // a >= 0, already scaled into [0, 6]
  const float mid[7] = {0.25f, 0.75f, 1.25f, 1.75f, 2.5f, 3.5f, 5.f};
  int i = 0;
#pragma unroll
  for (int t = 0; t < 7; ++t) i += (a > mid[t]) ? 1 : 0;
  return i;
}
__device__ __forceinline__ float fp4_value(int i) {
  const float v[8] = {0.f, .5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
  return v[i & 7];
}
__device__ __forceinline__ float fp6_value(int i) {  // magnitude index 0..31
  const int e = i >> 2, m = i & 3;
  return e == 0 ? m * 0.0625f : (1.f + m * 0.25f) * __builtin_ldexpf(1.f, e - 3);
}
__device__ __forceinline__ int fp6_index(float a) {
  int i = 0;
#pragma unroll
  for (int t = 0; t < 31; ++t) i += (a > 0.5f * (fp6_value(t) + fp6_value(t + 1))) ? 1 : 0;
  return i;
}

// ------------------------------------------------------------ group quantize / dequantize
// One wave per group: amax -> scale = amax / fmax (1 if the group is zero), then codes. FP4 writes
// two codes per byte (element 2j in the low nibble), FP6 one code per byte (FP_Quantize layout).
template <int BITS, DT T>
__global__ void __launch_bounds__(256) quant_kernel(const typename dt_traits<T>::storage* __restrict__ x,
                                                    uint8_t* __restrict__ q, float* __restrict__ scales,
                                                    int64_t groups, int gsize) {
  const int lane = threadIdx.x & 63;
  constexpr float FMAX = BITS == 4 ? 6.f : 28.f;
  for (int64_t gi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); gi < groups; gi += (int64_t)gridDim.x * 4) {
    const auto* xg = x + gi * gsize;
    float amax = 0.f;
    for (int j = lane; j < gsize; j += 64) amax = fmaxf(amax, fabsf(to_f32<T>(xg[j])));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
    const float s = amax > 0.f ? amax / FMAX : 1.f;
    if (lane == 0) scales[gi] = s;
    if constexpr (BITS == 4) {
      uint8_t* qg = q + gi * (gsize / 2);
      for (int j = lane; j < gsize / 2; j += 64) {
        const float a = to_f32<T>(xg[2 * j]) / s, b = to_f32<T>(xg[2 * j + 1]) / s;
        const int ca = fp4_index(fabsf(a)) | (a < 0.f ? 8 : 0), cb = fp4_index(fabsf(b)) | (b < 0.f ? 8 : 0);
        qg[j] = (uint8_t)(ca | (cb << 4));
      }
    } else {
      uint8_t* qg = q + gi * gsize;
      for (int j = lane; j < gsize; j += 64) {
        const float a = to_f32<T>(xg[j]) / s;
        qg[j] = (uint8_t)(fp6_index(fabsf(a)) | (a < 0.f ? 32 : 0));
      }
    }
  }
}

template <int BITS, DT T>
__global__ void __launch_bounds__(256) dequant_kernel(const uint8_t* __restrict__ q, const float* __restrict__ scales,
                                                      typename dt_traits<T>::storage* __restrict__ y, int64_t n,
                                                      int gsize) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if constexpr (BITS == 4) {
      const int c = (q[i >> 1] >> (4 * (i & 1))) & 15;
      v = (c & 8) ? -fp4_value(c & 7) : fp4_value(c & 7);
    } else {
      const int c = q[i];
      v = (c & 32) ? -fp6_value(c & 31) : fp6_value(c & 31);
    }
    y[i] = from_f32<T>(v * scales[i / gsize]);
  }
}

// ------------------------------------------------------------------------ register decode
__device__ __forceinline__ unsigned perm(unsigned hi4, unsigned lo4, unsigned sel) {
  return __builtin_amdgcn_perm(hi4, lo4, sel);
}
// byte tables (entries 0..3 in the low word, 4..7 in the high word)
constexpr unsigned F4H_LO = 0x3F3F3F00u, F4H_HI = 0x40404040u;  // bf16 high bytes of e2m1
constexpr unsigned F4L_LO = 0xC0800000u, F4L_HI = 0xC0804000u;  // bf16 low bytes
// e3m2, indexed by e (normals; entry 0 unused) and by m (subnormals, e = 0)
constexpr unsigned F6H_LO = 0x3F3F3E00u, F6H_HI = 0x41414040u;
constexpr unsigned F6SH = 0x3E3E3D00u, F6SL = 0x40008000u;
constexpr unsigned ZMASK_LO = 0x000000FFu;                  // 0xFF where e == 0

// 4 bytes of bf16 high bytes H and low bytes L (element b in byte b) -> two dwords of bf16 pairs
__device__ __forceinline__ void interleave(unsigned H, unsigned L, unsigned& d01, unsigned& d23) {
  d01 = perm(H, L, 0x05010400u);  // [L0, H0, L1, H1]
  d23 = perm(H, L, 0x07030602u);  // [L2, H2, L3, H3]
}

// 8 FP4 codes (one word in the GEMM layout) -> 8 bf16 (magnitudes; per-row scale applied later)
__device__ __forceinline__ void fp4x8(unsigned w, unsigned (&o)[4]) {
  const unsigned lo = w & 0x07070707u, hi = (w >> 4) & 0x07070707u;
  const unsigned slo = (w & 0x08080808u) << 4, shi = w & 0x80808080u;
  interleave(perm(F4H_HI, F4H_LO, lo) | slo, perm(F4L_HI, F4L_LO, lo), o[0], o[1]);
  interleave(perm(F4H_HI, F4H_LO, hi) | shi, perm(F4L_HI, F4L_LO, hi), o[2], o[3]);
}

// 4 FP6 weights: se = (sign << 3 | e) per byte, m = mantissa bits per byte
__device__ __forceinline__ void fp6x4(unsigned se, unsigned m, unsigned& d01, unsigned& d23) {
  const unsigned e = se & 0x07070707u, s = (se & 0x08080808u) << 4;
  const unsigned z = perm(0u, ZMASK_LO, e);                            // 0xFF bytes where e == 0
  const unsigned hn = perm(F6H_HI, F6H_LO, e), ln = ((e & 0x01010101u) << 7) | (m << 5);
  const unsigned hs = perm(0u, F6SH, m), ls = perm(0u, F6SL, m);
  const unsigned H = ((z & hs) | (~z & hn)) | s, L = (z & ls) | (~z & ln);
  interleave(H, L, d01, d23);
}

__device__ __forceinline__ bf16x8 as_bf16x8(const unsigned (&o)[4]) {
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  u32x4v v = {o[0], o[1], o[2], o[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// ------------------------------------------------------------------- weight-only skinny GEMM
// y[M, N] = x[M, K] . (W[N, K] * scale[N])^T (+ bias), M <= 16. Same structure as the W8A16
// kernel of skinny_gemm.hip: one workgroup per 16 output columns, K split over NW waves; per
// step each lane reads 32 weights (16 B of FP4, 16 + 8 B of FP6) and 32 activations, i.e. 4
// v_mfma_f32_16x16x32_bf16 with lane group g = lane >> 4 on K = k0 + 128 j + 32 g + [0, 32).
template <int BITS, int NW>
__global__ void __launch_bounds__(NW * 64) skinny_fpxw_kernel(const unsigned short* __restrict__ x, int64_t ldx,
                                                              const uint8_t* __restrict__ wa, int64_t lda,
                                                              const uint8_t* __restrict__ wb, int64_t ldb,
                                                              const float* __restrict__ wscale,
                                                              const unsigned short* __restrict__ bias,
                                                              unsigned short* __restrict__ y, int64_t ldy, int M, int N,
                                                              int K, int steps_per_wave) {
  __shared__ f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * 16 + col;
  const bool wok = n < N, xok = col < M;
  const uint8_t* arow = wa + (int64_t)(wok ? n : 0) * lda;
  const uint8_t* brow = BITS == 6 ? wb + (int64_t)(wok ? n : 0) * ldb : nullptr;
  const unsigned short* xrow = x + (int64_t)(xok ? col : 0) * ldx;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < steps_per_wave; ++i) {
    const int k = (wave * steps_per_wave + i) * 128 + 32 * g;  // this lane's 32 weights
    const bool in = k < K;
    uint4 av = (wok && in) ? *reinterpret_cast<const uint4*>(arow + k / 2) : uint4{0u, 0u, 0u, 0u};
    uint2 bv = uint2{0u, 0u};
    if constexpr (BITS == 6) bv = (wok && in) ? *reinterpret_cast<const uint2*>(brow + k / 4) : uint2{0u, 0u};
    bf16x8 xs[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      xs[t] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k + 8 * t) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned aw[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      unsigned o[4];
      if constexpr (BITS == 4) {
        fp4x8(aw[t], o);
      } else {
        const unsigned bw = (t < 2) ? bv.x : bv.y;       // 16 weights per B word
        const int sh = 4 * (t & 1);                       // w0..7 of the word: bits 0/2, w8..15: 4/6
        const unsigned m_lo = (bw >> sh) & 0x03030303u, m_hi = (bw >> (sh + 2)) & 0x03030303u;
        fp6x4(aw[t] & 0x0F0F0F0Fu, m_lo, o[0], o[1]);
        fp6x4((aw[t] >> 4) & 0x0F0F0F0Fu, m_hi, o[2], o[3]);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xs[t], as_bf16x8(o), acc, 0, 0, 0);
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int v = 1; v < NW; ++v) {
      const f32x4 u = red[v][lane];
      t[0] += u[0];
      t[1] += u[1];
      t[2] += u[2];
      t[3] += u[3];
    }
    if (n < N) {
      const float sc = wscale[n];
      const float b = bias ? bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        if (m < M) y[(int64_t)m * ldy + n] = f32_to_bf16(t[r] * sc + b);
      }
    }
  }
}

// Full-weight decode (prefill-sized inputs take hipBLASLt on the bf16 weight): one thread per
// 8 weights of the GEMM layout -> bf16 [N, K] * scale[n].
template <int BITS>
__global__ void __launch_bounds__(256) unpack_kernel(const uint8_t* __restrict__ wa, const uint8_t* __restrict__ wb,
                                                     const float* __restrict__ wscale, unsigned short* __restrict__ out,
                                                     int N, int K) {
  const int64_t words = (int64_t)N * (K / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / (K / 8));
    const int k8 = (int)(i % (K / 8));
    const unsigned aw = reinterpret_cast<const unsigned*>(wa + (int64_t)n * (K / 2))[k8];
    unsigned o[4];
    if constexpr (BITS == 4) {
      fp4x8(aw, o);
    } else {
      const unsigned bw = reinterpret_cast<const unsigned*>(wb + (int64_t)n * (K / 4))[k8 >> 1];
      const int sh = 4 * (k8 & 1);
      fp6x4(aw & 0x0F0F0F0Fu, (bw >> sh) & 0x03030303u, o[0], o[1]);
      fp6x4((aw >> 4) & 0x0F0F0F0Fu, (bw >> (sh + 2)) & 0x03030303u, o[2], o[3]);
    }
    const float sc = wscale[n];
    u16x8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const unsigned short h = (unsigned short)(o[e >> 1] >> (16 * (e & 1)));
      r[e] = f32_to_bf16(bf16_to_f32(h) * sc);
    }
    *reinterpret_cast<u16x8*>(out + (int64_t)n * K + 8 * k8) = r;
  }
}

}  // namespace mx

// ------------------------------------------------------------------------------- host side
std::vector<at::Tensor> fpx_quantize(const at::Tensor& x, int64_t bits, int64_t group_size) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(bits == 4 || bits == 6, "fpx_quantize: bits 4 (e2m1) or 6 (e3m2)");
  SXE_CHECK(x.is_contiguous() && x.numel() % group_size == 0 && group_size % 2 == 0,
            "fpx_quantize: contiguous input, numel a multiple of an even group_size");
  const int64_t n = x.numel(), groups = n / group_size;
  auto q = at::empty({bits == 4 ? n / 2 : n}, x.options().dtype(at::kByte));
  auto s = at::empty({groups}, x.options().dtype(at::kFloat));
  if (n == 0) return {q, s};
  c10::DeviceGuard g(x.device());
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, 16 * kNumCUs));
#define SXE_FQ(B, T)                                                                                         \
  hipLaunchKernelGGL((mx::quant_kernel<B, T>), dim3(grid), dim3(256), 0, cur_stream(),                       \
                     reinterpret_cast<const typename dt_traits<T>::storage*>(x.data_ptr()), q.data_ptr<uint8_t>(), \
                     s.data_ptr<float>(), groups, (int)group_size)
#define SXE_FQ_B(T) \
  if (bits == 4) SXE_FQ(4, T); \
  else SXE_FQ(6, T);
  if (x.scalar_type() == at::kFloat) {
    SXE_FQ_B(DT::F32)
  } else if (x.scalar_type() == at::kBFloat16) {
    SXE_FQ_B(DT::BF16)
  } else {
    SXE_CHECK(x.scalar_type() == at::kHalf, "fpx_quantize: fp32 / bf16 / fp16 input");
    SXE_FQ_B(DT::F16)
  }
#undef SXE_FQ_B
#undef SXE_FQ
  SXE_LAUNCH_CHECK();
  return {q, s};
}

at::Tensor fpx_dequantize(const at::Tensor& q, const at::Tensor& scales, int64_t bits, int64_t group_size, int64_t n,
                          at::ScalarType dtype) {
  SXE_CHECK_CUDA(q);
  SXE_CHECK(bits == 4 || bits == 6, "fpx_dequantize: bits 4 or 6");
  SXE_CHECK(q.scalar_type() == at::kByte && q.is_contiguous() && scales.scalar_type() == at::kFloat &&
                scales.is_contiguous(), "fpx_dequantize: uint8 codes, fp32 scales");
  SXE_CHECK(q.numel() >= (bits == 4 ? n / 2 : n) && scales.numel() * group_size >= n, "fpx_dequantize: sizes");
  auto y = at::empty({n}, q.options().dtype(dtype));
  if (n == 0) return y;
  c10::DeviceGuard g(q.device());
  const int grid = stream_grid(n, 256);
#define SXE_FD(B, T)                                                                                          \
  hipLaunchKernelGGL((mx::dequant_kernel<B, T>), dim3(grid), dim3(256), 0, cur_stream(), q.data_ptr<uint8_t>(), \
                     scales.data_ptr<float>(), reinterpret_cast<typename dt_traits<T>::storage*>(y.data_ptr()), n,  \
                     (int)group_size)
#define SXE_FD_B(T) \
  if (bits == 4) SXE_FD(4, T); \
  else SXE_FD(6, T);
  if (dtype == at::kFloat) {
    SXE_FD_B(DT::F32)
  } else if (dtype == at::kBFloat16) {
    SXE_FD_B(DT::BF16)
  } else {
    SXE_CHECK(dtype == at::kHalf, "fpx_dequantize: fp32 / bf16 / fp16 output");
    SXE_FD_B(DT::F16)
  }
#undef SXE_FD_B
#undef SXE_FD
  SXE_LAUNCH_CHECK();
  return y;
}

static void check_fpxw(const at::Tensor& wa, const c10::optional<at::Tensor>& wb, const at::Tensor& wscale, int64_t bits,
                       int64_t K) {
  SXE_CHECK(bits == 4 || bits == 6, "fpx weight GEMM: bits 4 or 6");
  SXE_CHECK(K % 128 == 0, "fpx weight GEMM: K must be a multiple of 128");
  SXE_CHECK(wa.scalar_type() == at::kByte && wa.dim() == 2 && wa.is_contiguous() && wa.size(1) == K / 2,
            "fpx weight GEMM: plane A uint8 [N, K/2]");
  SXE_CHECK((reinterpret_cast<uintptr_t>(wa.data_ptr()) & 15) == 0, "fpx weight GEMM: 16-byte aligned plane A");
  if (bits == 6) {
    SXE_CHECK(wb.has_value() && wb->defined() && wb->scalar_type() == at::kByte && wb->dim() == 2 && wb->is_contiguous() &&
                  wb->size(0) == wa.size(0) && wb->size(1) == K / 4 && (reinterpret_cast<uintptr_t>(wb->data_ptr()) & 7) == 0,
              "fpx weight GEMM: FP6 plane B uint8 [N, K/4], 8-byte aligned");
  }
  SXE_CHECK(wscale.scalar_type() == at::kFloat && wscale.is_contiguous() && wscale.numel() == wa.size(0),
            "fpx weight GEMM: fp32 per-row scales [N]");
}

at::Tensor skinny_gemm_fpxw(const at::Tensor& x, const at::Tensor& wa, const c10::optional<at::Tensor>& wb,
                            const at::Tensor& wscale, const c10::optional<at::Tensor>& bias, int64_t bits) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "skinny_gemm_fpxw: bf16 x [M, K]");
  const int M = x.size(0), K = x.size(1), N = wa.size(0);
  check_fpxw(wa, wb, wscale, bits, K);
  SXE_CHECK(M >= 1 && M <= 16, "skinny_gemm_fpxw: 1 <= M <= 16");
  SXE_CHECK(x.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0,
            "skinny_gemm_fpxw: 16-byte aligned activation rows");
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return y;
  c10::DeviceGuard g(x.device());
  const int steps = K / 128, tiles = (N + 15) / 16;
  int nw = 4;
  while (nw < 8 && (int64_t)tiles * nw < 4096 && steps >= 2 * nw) nw *= 2;
  const int spw = (steps + nw - 1) / nw;
  const uint8_t* bptr = bits == 6 ? wb->data_ptr<uint8_t>() : nullptr;
  const int64_t ldb = bits == 6 ? wb->stride(0) : 0;
#define SXE_FW(B, NW)                                                                                                \
  hipLaunchKernelGGL((mx::skinny_fpxw_kernel<B, NW>), dim3(tiles), dim3(NW * 64), 0, cur_stream(),                   \
                     reinterpret_cast<const unsigned short*>(x.data_ptr()), x.stride(0), wa.data_ptr<uint8_t>(),      \
                     wa.stride(0), bptr, ldb, wscale.data_ptr<float>(), bp,                                          \
                     reinterpret_cast<unsigned short*>(y.data_ptr()), y.stride(0), M, N, K, spw)
  if (bits == 4) {
    if (nw == 4) SXE_FW(4, 4); else SXE_FW(4, 8);
  } else {
    if (nw == 4) SXE_FW(6, 4); else SXE_FW(6, 8);
  }
#undef SXE_FW
  SXE_LAUNCH_CHECK();
  return y;
}

at::Tensor fpxw_unpack(const at::Tensor& wa, const c10::optional<at::Tensor>& wb, const at::Tensor& wscale, int64_t bits) {
  SXE_CHECK_CUDA(wa);
  const int N = wa.size(0), K = wa.size(1) * 2;
  check_fpxw(wa, wb, wscale, bits, K);
  auto out = at::empty({N, K}, wa.options().dtype(at::kBFloat16));
  if (N == 0) return out;
  c10::DeviceGuard g(wa.device());
  const int grid = stream_grid((int64_t)N * (K / 8), 256);
  auto* op = reinterpret_cast<unsigned short*>(out.data_ptr());
  if (bits == 4)
    hipLaunchKernelGGL(mx::unpack_kernel<4>, dim3(grid), dim3(256), 0, cur_stream(), wa.data_ptr<uint8_t>(), nullptr,
                       wscale.data_ptr<float>(), op, N, K);
  else
    hipLaunchKernelGGL(mx::unpack_kernel<6>, dim3(grid), dim3(256), 0, cur_stream(), wa.data_ptr<uint8_t>(),
                       wb->data_ptr<uint8_t>(), wscale.data_ptr<float>(), op, N, K);
  SXE_LAUNCH_CHECK();
  return out;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("fpx_quantize(Tensor x, int bits, int group_size) -> Tensor[]");
  m.def("fpx_dequantize(Tensor q, Tensor scales, int bits, int group_size, int n, ScalarType dtype) -> Tensor");
  m.def("skinny_gemm_fpxw(Tensor x, Tensor wa, Tensor? wb, Tensor wscale, Tensor? bias, int bits) -> Tensor");
  m.def("fpxw_unpack(Tensor wa, Tensor? wb, Tensor wscale, int bits) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("fpx_quantize", &sxe::fpx_quantize);
  m.impl("fpx_dequantize", &sxe::fpx_dequantize);
  m.impl("skinny_gemm_fpxw", &sxe::skinny_gemm_fpxw);
  m.impl("fpxw_unpack", &sxe::fpxw_unpack);
}

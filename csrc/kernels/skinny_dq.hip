// Decode-sized (M <= 16) GEMMs over low-bit weights that have no skinny path elsewhere:
//   OCP-MX  -- e4m3 / e3m2 / e2m1 codes, one E8M0 exponent per 32 K (ops/mx.MXWeight), and
//   integer -- symmetric int8 / int4 codes with one fp32 scale per `group` K (ops/moe.IntWeight),
// y[M, N] = x[M, K] . dequant(W[N, K])^T (+ bias) with 16-bit activations (weight-only quantisation:
// the activations are NOT quantised on this path, unlike the block-scaled prefill GEMM).
//
// Memory-bound by construction: one workgroup per 16 output columns, K split over NW waves; per
// 128-K step every lane streams the 32 codes of one (column, K block) -- 32 / 24 / 16 bytes -- and
// decodes them in registers, bytewise-parallel: 4-bit / 6-bit codes are transcoded exactly to e4m3
// bytes (both formats embed in e4m3; byte tables through v_perm_b32) and widened by
// v_cvt_pk_f32_fp8, integers by unsigned byte conversions; the lane's block scale is applied by
// packed f32 multiplies / FMAs (v_pk_mul_f32, v_pk_fma_f32: the kernel is VALU-bound, not
// HBM-bound, at 4-6 bits per weight) and the 32 values are packed to bf16 for four
// v_mfma_f32_16x16x32_bf16 (lane group g = lane >> 4 covers K = 32 g .. 32 g + 31 of the step, so
// each lane's codes are exactly one scale block). Cross-wave partial sums are reduced in LDS.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace sdq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

enum Fmt : int { E4M3 = 0, E3M2 = 3, E2M1 = 4, I8 = 8, I4 = 9 };
__host__ __device__ constexpr int fmt_bytes32(int f) {  // bytes per 32 codes
  return (f == E4M3 || f == I8) ? 32 : (f == E3M2 ? 24 : 16);
}

typedef float f32x2v __attribute__((ext_vector_type(2)));

// 4 e2m1 codes (one per byte) -> 4 e4m3 bytes, exact: the 3-bit magnitude indexes an 8-byte table
// (v_perm_b32) of the e4m3 encodings of 0, 0.5, 1, 1.5, 2, 3, 4, 6; the sign moves from bit 3 to 7
__device__ __forceinline__ unsigned e2m1_to_e4m3(unsigned x) {
  return __builtin_amdgcn_perm(0x4C484440u, 0x3C383000u, x & 0x07070707u) | ((x & 0x08080808u) << 4);
}
// 4 e3m2 codes (one per byte) -> 4 e4m3 bytes, exact: normals (e >= 1) are ((e + 4) << 3) | (m << 1)
// with the exponent part from a table; subnormals (e == 0: m * 2^-4 = 0, 0x18, 0x20, 0x24 in e4m3)
// add a per-mantissa correction selected by the e == 0 byte mask
__device__ __forceinline__ unsigned e3m2_to_e4m3(unsigned c) {
  const unsigned e = (c >> 2) & 0x07070707u, m = c & 0x03030303u;
  const unsigned base = __builtin_amdgcn_perm(0x58504840u, 0x38302800u, e);   // (e + 4) << 3, 0 at e == 0
  const unsigned z = __builtin_amdgcn_perm(0u, 0x000000FFu, e);                // 0xFF where e == 0
  const unsigned corr = __builtin_amdgcn_perm(0u, 0x1E1C1600u, m);             // subnormal - (m << 1)
  return (base + (m << 1) + (z & corr)) | ((c & 0x20202020u) << 2);
}
// 4 e4m3 bytes -> 4 floats scaled by s (v_cvt_pk_f32_fp8, then packed f32 multiplies)
__device__ __forceinline__ void fp8x4s(unsigned b, f32x2v s2, f32x2v* o) {
  const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, false), hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, true);
  o[0] = f32x2v{lo[0], lo[1]} * s2;
  o[1] = f32x2v{hi[0], hi[1]} * s2;
}

// the 32 codes of one lane (raw words) -> 32 floats in K order, times the lane's block scale sc
// (pairs: v[j] holds elements 2 j, 2 j + 1). Integers go through unsigned byte conversions of the
// code + 2^(bits-1) and one packed FMA that removes the offset: (u - o) * sc = u * sc - o * sc.
template <int F>
__device__ __forceinline__ void decode32(const unsigned (&w)[8], float sc, f32x2v (&v)[16]) {
  const f32x2v s2 = {sc, sc};
  if constexpr (F == E4M3) {
#pragma unroll
    for (int d = 0; d < 8; ++d) fp8x4s(w[d], s2, v + 2 * d);
  } else if constexpr (F == I8) {
    const f32x2v o2 = {-128.f * sc, -128.f * sc};
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const unsigned u = w[d] ^ 0x80808080u;
      v[2 * d] = f32x2v{(float)(u & 0xffu), (float)((u >> 8) & 0xffu)} * s2 + o2;
      v[2 * d + 1] = f32x2v{(float)((u >> 16) & 0xffu), (float)(u >> 24)} * s2 + o2;
    }
  } else if constexpr (F == E2M1 || F == I4) {
    // word d holds codes 8d .. 8d+7, code 2b in the low nibble of byte b, 2b+1 in the high one
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const unsigned lo = w[d] & 0x0F0F0F0Fu, hi = (w[d] >> 4) & 0x0F0F0F0Fu;
      if constexpr (F == E2M1) {
        const unsigned el = e2m1_to_e4m3(lo), eh = e2m1_to_e4m3(hi);
        const auto l0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)el, false), l1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)el, true);
        const auto h0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)eh, false), h1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)eh, true);
        v[4 * d + 0] = f32x2v{l0[0], h0[0]} * s2;
        v[4 * d + 1] = f32x2v{l0[1], h0[1]} * s2;
        v[4 * d + 2] = f32x2v{l1[0], h1[0]} * s2;
        v[4 * d + 3] = f32x2v{l1[1], h1[1]} * s2;
      } else {
        const f32x2v o2 = {-8.f * sc, -8.f * sc};
        const unsigned lb = lo ^ 0x08080808u, hb = hi ^ 0x08080808u;  // q + 8 in 0 .. 15
#pragma unroll
        for (int b = 0; b < 4; ++b)
          v[4 * d + b] = f32x2v{(float)((lb >> (8 * b)) & 0xffu), (float)((hb >> (8 * b)) & 0xffu)} * s2 + o2;
      }
    }
  } else {  // E3M2: codes j at bits [6 j, 6 j + 6) of the 24 bytes; 4 codes per 3 bytes
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // 16 codes per 3 words
      const uint64_t lo64 = ((uint64_t)w[3 * q + 1] << 32) | w[3 * q];
      const uint64_t hi64 = ((uint64_t)w[3 * q + 2] << 32) | w[3 * q + 1];
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // group of 4 codes at bit 24 k of the 96
        const unsigned g = k < 2 ? (unsigned)(lo64 >> (24 * k)) & 0xFFFFFFu : (unsigned)(hi64 >> (24 * k - 32)) & 0xFFFFFFu;
        const unsigned c = (g & 0x3Fu) | ((g & 0xFC0u) << 2) | ((g & 0x3F000u) << 4) | ((g & 0xFC0000u) << 6);
        fp8x4s(e3m2_to_e4m3(c), s2, v + 8 * q + 2 * k);
      }
    }
  }
}

template <int F, int NW, int U>
__global__ void __launch_bounds__(NW * 64) skinny_dq_kernel(const unsigned short* __restrict__ x, int64_t ldx,
                                                            const uint8_t* __restrict__ wq, int64_t ldw,
                                                            const void* __restrict__ scales, int groups_per_row,
                                                            int group, const unsigned short* __restrict__ bias,
                                                            unsigned short* __restrict__ y, int64_t ldy, int M, int N,
                                                            int K, int steps_per_wave) {
  __shared__ f32x4v red[NW][64];
  constexpr int BY = fmt_bytes32(F);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * 16 + col;
  const bool wok = n < N, xok = col < M;
  const uint8_t* wrow = wq + (int64_t)(wok ? n : 0) * ldw;
  const unsigned short* xrow = x + (int64_t)(xok ? col : 0) * ldx;
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
  // U steps per round, all their loads issued before the first decode (U = 4 measured no faster
  // than 1 on Llama-3-8B decode and slower at batch 16: 140 vs 70 VGPRs, so the launch uses U = 1)
  for (int i0 = 0; i0 < steps_per_wave; i0 += U) {
    unsigned w[U][8];
    float sc[U];
    bf16x8 xs[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (wave * steps_per_wave + i0 + u) * 128 + 32 * g;  // this lane's 32 codes = one scale block
      const bool in = i0 + u < steps_per_wave && k < K;
#pragma unroll
      for (int d = 0; d < 8; ++d) w[u][d] = 0;
      sc[u] = 0.f;
      if (wok && in) {
        const uint8_t* p = wrow + (int64_t)k * BY / 32;
        if constexpr (BY == 32) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(p), b = *reinterpret_cast<const u32x4*>(p + 16);
          w[u][0] = a[0]; w[u][1] = a[1]; w[u][2] = a[2]; w[u][3] = a[3];
          w[u][4] = b[0]; w[u][5] = b[1]; w[u][6] = b[2]; w[u][7] = b[3];
        } else if constexpr (BY == 24) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(p);
          const u32x2 b = *reinterpret_cast<const u32x2*>(p + 16);
          w[u][0] = a[0]; w[u][1] = a[1]; w[u][2] = a[2]; w[u][3] = a[3]; w[u][4] = b[0]; w[u][5] = b[1];
        } else {
          const u32x4 a = *reinterpret_cast<const u32x4*>(p);
          w[u][0] = a[0]; w[u][1] = a[1]; w[u][2] = a[2]; w[u][3] = a[3];
        }
        if constexpr (F == I8 || F == I4) {
          sc[u] = reinterpret_cast<const float*>(scales)[(int64_t)n * groups_per_row + k / group];
        } else {
          const unsigned e = reinterpret_cast<const uint8_t*>(scales)[(int64_t)n * groups_per_row + k / 32];
          sc[u] = __uint_as_float(e << 23);  // 2^(e - 127); e = 0 flushes to 0 (an all-zero MX block)
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        xs[u][t] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k + 8 * t) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x2v v[16];
      decode32<F>(w[u], sc[u], v);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          b[2 * e] = (__bf16)v[4 * t + e][0];
          b[2 * e + 1] = (__bf16)v[4 * t + e][1];
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xs[u][t], b, acc, 0, 0, 0);
      }
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    f32x4v t = red[0][lane];
#pragma unroll
    for (int v = 1; v < NW; ++v) t += red[v][lane];
    if (n < N) {
      const float b = bias ? bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        if (m < M) y[(int64_t)m * ldy + n] = f32_to_bf16(t[r] + b);
      }
    }
  }
}

}  // namespace sdq

// y [M, N] = x [M, K] (bf16, M <= 16) . dequant(wq)^T (+ bias); fmt 0 / 3 / 4 = MX e4m3 / e3m2 / e2m1
// (scales uint8 E8M0 [N, K / 32]), 8 / 9 = int8 / int4 (scales fp32 [N, K / group], group % 32 == 0)
at::Tensor skinny_gemm_dq(at::Tensor x, at::Tensor wq, at::Tensor scales, int64_t fmt, int64_t group,
                          c10::optional<at::Tensor> bias) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(fmt == 0 || fmt == 3 || fmt == 4 || fmt == 8 || fmt == 9, "skinny_gemm_dq: fmt 0 / 3 / 4 (MX) or 8 / 9 (int)");
  SXE_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 &&
                reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
            "skinny_gemm_dq: bf16 x [M, K] with 16-byte aligned rows");
  const int64_t M = x.size(0), K = x.size(1);
  SXE_CHECK(M >= 1 && M <= 16, "skinny_gemm_dq: 1 <= M <= 16");
  SXE_CHECK(K % 128 == 0, "skinny_gemm_dq: K must be a multiple of 128");
  const bool is_int = fmt >= 8;
  if (!is_int) group = 32;
  SXE_CHECK(group >= 32 && group % 32 == 0 && K % group == 0, "skinny_gemm_dq: group a multiple of 32 dividing K");
  const int by = sdq::fmt_bytes32((int)fmt);
  SXE_CHECK(wq.is_cuda() && wq.is_contiguous() && wq.element_size() == 1 && wq.dim() >= 2 &&
                wq.numel() % (K * by / 32) == 0,
            "skinny_gemm_dq: wq codes [N, K * bits / 8]");
  const int64_t N = wq.numel() / (K * by / 32);
  SXE_CHECK(scales.is_cuda() && scales.is_contiguous() && scales.numel() == N * (K / group) &&
                (is_int ? scales.scalar_type() == at::kFloat : scales.scalar_type() == at::kByte),
            "skinny_gemm_dq: scales [N, K / group] (fp32 for int, uint8 E8M0 for MX)");
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N,
              "skinny_gemm_dq: bias bf16 [N]");
  }
  c10::DeviceGuard guard(x.device());
  auto y = at::empty({M, N}, x.options());
  constexpr int NW = 8;
  const unsigned tiles = (unsigned)((N + 15) / 16);
  const int steps = (int)((K / 128 + NW - 1) / NW);
  const unsigned short* b = (bias.has_value() && bias->defined()) ? reinterpret_cast<const unsigned short*>(bias->data_ptr())
                                                                   : nullptr;
#define SXE_SDQ(F)                                                                                                   \
  hipLaunchKernelGGL((sdq::skinny_dq_kernel<F, NW, 1>), dim3(tiles), dim3(NW * 64), 0, cur_stream(),                \
                     reinterpret_cast<const unsigned short*>(x.data_ptr()), x.stride(0), wq.data_ptr<uint8_t>(),     \
                     K * by / 32, scales.data_ptr(), (int)(K / group), (int)group, b,                               \
                     reinterpret_cast<unsigned short*>(y.data_ptr()), N, (int)M, (int)N, (int)K, steps)
  switch (fmt) {
    case 0: SXE_SDQ(sdq::E4M3); break;
    case 3: SXE_SDQ(sdq::E3M2); break;
    case 4: SXE_SDQ(sdq::E2M1); break;
    case 8: SXE_SDQ(sdq::I8); break;
    default: SXE_SDQ(sdq::I4); break;
  }
#undef SXE_SDQ
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("skinny_gemm_dq(Tensor x, Tensor wq, Tensor scales, int fmt, int group, Tensor? bias=None) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) { m.impl("skinny_gemm_dq", &sxe::skinny_gemm_dq); }

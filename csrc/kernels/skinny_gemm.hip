// Skinny GEMM for decode: y[M, N] = x[M, K] . W[N, K]^T (+ bias), M <= 16, bf16, fp32 accumulate.
//
// Decode GEMMs stream the weight once and touch almost no activation bytes, so the job is HBM
// streaming at the highest rate the chip sustains -- hipBLASLt's general kernels reach 3.5-4.7 TB/s
// on Llama-3-8B decode shapes (profiles/decode_*). MI355X-first design:
//  * MFMA does the math (v_mfma_f32_16x16x32_bf16, x padded to 16 rows): the VALU stays free and
//    the lane maps are the hardware's -- lane l holds W[n = l & 15][8 K values] as the B fragment
//    and x[m = l & 15][the same 8 K values] as the A fragment;
//  * MFMA step s of a 256-wide super-step takes K = k0 + 32 s + [0, 32): lane group g = l >> 4 reads
//    the 16 bytes at k0 + 32 s + 8 g, so each load instruction reads 64 contiguous bytes of each of
//    16 rows and two consecutive steps complete the 128-byte lines (a lane-owns-128-bytes map was
//    2x slower: 64 distinct lines per instruction);
//  * one workgroup per 16 output columns, K split over its NW = 4/8 waves (NW = 8 for narrow N,
//    so more waves per CU stream at once; 16 waves would cap VGPRs at 128 and spill), two super-steps of loads in flight per wave, partial
//    tiles summed through NW KB of LDS.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace sg {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kSS = 256;  // K per super-step per wave

struct Frag {
  bf16x8 w[8];
  bf16x8 x[8];
};

__device__ __forceinline__ void load_ss(Frag& f, const unsigned short* __restrict wrow, bool wok,
                                        const unsigned short* __restrict xrow, bool xok, int kbase, int K) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = kbase + s * 32;
    const bool in = k < K;
    f.w[s] = (wok && in) ? *reinterpret_cast<const bf16x8*>(wrow + k) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    f.x[s] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(const unsigned short* __restrict x, int64_t ldx,
                                                          const unsigned short* __restrict w, int64_t ldw,
                                                          const unsigned short* __restrict bias,
                                                          unsigned short* __restrict y, int64_t ldy, int M, int N,
                                                          int K, int ss_per_wave) {
  __shared__ f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int col = lane & 15, g = lane >> 4;
  const int n = n0 + col;
  const bool wok = n < N, xok = col < M;
  const unsigned short* wrow = w + (int64_t)(wok ? n : 0) * ldw;
  const unsigned short* xrow = x + (int64_t)(xok ? col : 0) * ldx;
  const int ss0 = wave * ss_per_wave;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  Frag cur, nxt;
  load_ss(cur, wrow, wok, xrow, xok, ss0 * kSS + g * 8, K);
  for (int i = 0; i < ss_per_wave; ++i) {
    if (i + 1 < ss_per_wave) load_ss(nxt, wrow, wok, xrow, xok, (ss0 + i + 1) * kSS + g * 8, K);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.x[s], cur.w[s], acc, 0, 0, 0);
    cur = nxt;
  }
  // acc: C[row m = 4 g + r][col n] -- sum the 4 waves' K partials
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
      const float b = bias ? bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        if (m < M) y[(int64_t)m * ldy + n] = f32_to_bf16(t[r] + b);
      }
    }
  }
}

// ---- FP8-weight variant (W8A16: e4m3 weights, per-output-row fp32 scale, bf16 activations) ----
// Same structure; each lane streams 16 bytes = 16 weights per load and converts them to bf16 in
// registers (v_cvt_f32_fp8; e4m3 values are exact in bf16), so the weight bytes -- the whole
// cost of a decode GEMM -- are halved. MFMA step (j, h) of a 512-wide super-step uses
// K = k0 + 64 j + 16 g + 8 h + [0, 8) for lane group g, for weights and activations alike.
constexpr int kSS8 = 512;

__device__ __forceinline__ bf16x8 fp8x8_to_bf16(uint2 w) {
  // byte-selected v_cvt_f32_fp8 (byte b of the word -> element b): explicit order, e4m3 is exact
  // in bf16 so the top half of the f32 bit pattern is the bf16 value
  bf16x8 r;
#define SXE_FP8_BYTE(word, b) (short)(__builtin_bit_cast(unsigned int, __builtin_amdgcn_cvt_f32_fp8((int)(word), b)) >> 16)
  r[0] = SXE_FP8_BYTE(w.x, 0);
  r[1] = SXE_FP8_BYTE(w.x, 1);
  r[2] = SXE_FP8_BYTE(w.x, 2);
  r[3] = SXE_FP8_BYTE(w.x, 3);
  r[4] = SXE_FP8_BYTE(w.y, 0);
  r[5] = SXE_FP8_BYTE(w.y, 1);
  r[6] = SXE_FP8_BYTE(w.y, 2);
  r[7] = SXE_FP8_BYTE(w.y, 3);
#undef SXE_FP8_BYTE
  return r;
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_fp8w_kernel(const unsigned short* __restrict x, int64_t ldx,
                                                                   const uint8_t* __restrict w, int64_t ldw,
                                                                   const float* __restrict wscale,
                                                                   const unsigned short* __restrict bias,
                                                                   unsigned short* __restrict y, int64_t ldy, int M,
                                                                   int N, int K, int ss_per_wave) {
  __shared__ f32x4 red[NW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int col = lane & 15, g = lane >> 4;
  const int n = n0 + col;
  const bool wok = n < N, xok = col < M;
  const uint8_t* wrow = w + (int64_t)(wok ? n : 0) * ldw;
  const unsigned short* xrow = x + (int64_t)(xok ? col : 0) * ldx;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < ss_per_wave; ++i) {
    const int k0 = (wave * ss_per_wave + i) * kSS8 + 16 * g;
    uint4 wv[8];
    bf16x8 xa[8], xb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + 64 * j;
      const bool in = k < K;
      wv[j] = (wok && in) ? *reinterpret_cast<const uint4*>(wrow + k) : uint4{0u, 0u, 0u, 0u};
      xa[j] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      xb[j] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k + 8) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[j], fp8x8_to_bf16(uint2{wv[j].x, wv[j].y}), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], fp8x8_to_bf16(uint2{wv[j].z, wv[j].w}), acc, 0, 0, 0);
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

}  // namespace sg

// x [M, K] (row stride free, unit column stride), w [N, K] contiguous rows, bias [N] or None.
at::Tensor skinny_gemm(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "skinny_gemm: bf16 only");
  SXE_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "skinny_gemm: x [M, K], w [N, K]");
  SXE_CHECK(x.stride(1) == 1 && w.stride(1) == 1, "skinny_gemm: unit stride along K");
  const int M = x.size(0), N = w.size(0), K = x.size(1);
  SXE_CHECK(M >= 1 && M <= 16, "skinny_gemm: 1 <= M <= 16");
  SXE_CHECK(K % 8 == 0 && x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0,
            "skinny_gemm: K and row strides must be multiples of 8 (16-byte loads)");
  SXE_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
            "skinny_gemm: 16-byte aligned operands");
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return y;
  c10::DeviceGuard gd(x.device());
  // K split over NW waves: enough waves in flight (~16 per CU) for narrow N, >= 2 super-steps each
  const int ss_total = (K + sg::kSS - 1) / sg::kSS;
  const int tiles = (N + 15) / 16;
  int nw = 4;
  while (nw < 8 && (int64_t)tiles * nw < 4096 && ss_total >= 4 * nw) nw *= 2;
  const int ss_per_wave = (ss_total + nw - 1) / nw;
  auto* xp = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto* wp = reinterpret_cast<const unsigned short*>(w.data_ptr());
  auto* yp = reinterpret_cast<unsigned short*>(y.data_ptr());
#define SXE_SG_LAUNCH(NW)                                                                                  \
  hipLaunchKernelGGL(sg::skinny_gemm_kernel<NW>, dim3(tiles), dim3(NW * 64), 0, cur_stream(), xp, x.stride(0), \
                     wp, w.stride(0), bp, yp, y.stride(0), M, N, K, ss_per_wave)
  if (nw == 4) SXE_SG_LAUNCH(4);
  else SXE_SG_LAUNCH(8);
#undef SXE_SG_LAUNCH
  SXE_LAUNCH_CHECK();
  return y;
}

// x [M, K] bf16, wq [N, K] e4m3 bytes (uint8 or float8_e4m3fn), wscale [N] fp32, bias [N] bf16 or None
at::Tensor skinny_gemm_fp8w(const at::Tensor& x, const at::Tensor& wq, const at::Tensor& wscale,
                            const c10::optional<at::Tensor>& bias) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.scalar_type() == at::kBFloat16, "skinny_gemm_fp8w: bf16 activations");
  SXE_CHECK(wq.element_size() == 1 && wq.dim() == 2 && wq.stride(1) == 1, "skinny_gemm_fp8w: wq [N, K] bytes");
  SXE_CHECK(wscale.scalar_type() == at::kFloat && wscale.is_contiguous() && wscale.numel() == wq.size(0),
            "skinny_gemm_fp8w: wscale fp32 [N]");
  SXE_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) == wq.size(1), "skinny_gemm_fp8w: x [M, K]");
  const int M = x.size(0), N = wq.size(0), K = x.size(1);
  SXE_CHECK(M >= 1 && M <= 16, "skinny_gemm_fp8w: 1 <= M <= 16");
  SXE_CHECK(K % 16 == 0 && wq.stride(0) % 16 == 0 && x.stride(0) % 8 == 0,
            "skinny_gemm_fp8w: K and row strides must allow 16-byte loads");
  SXE_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(wq.data_ptr()) % 16 == 0,
            "skinny_gemm_fp8w: 16-byte aligned operands");
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return y;
  c10::DeviceGuard gd(x.device());
  const int ss_total = (K + sg::kSS8 - 1) / sg::kSS8;
  const int tiles = (N + 15) / 16;
  int nw = 4;
  while (nw < 8 && (int64_t)tiles * nw < 4096 && ss_total >= 2 * nw) nw *= 2;
  const int ss_per_wave = (ss_total + nw - 1) / nw;
  auto* xp = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto* wp = reinterpret_cast<const uint8_t*>(wq.data_ptr());
  auto* yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  if (nw == 4)
    hipLaunchKernelGGL(sg::skinny_gemm_fp8w_kernel<4>, dim3(tiles), dim3(256), 0, cur_stream(), xp, x.stride(0), wp,
                       wq.stride(0), wscale.data_ptr<float>(), bp, yp, y.stride(0), M, N, K, ss_per_wave);
  else
    hipLaunchKernelGGL(sg::skinny_gemm_fp8w_kernel<8>, dim3(tiles), dim3(512), 0, cur_stream(), xp, x.stride(0), wp,
                       wq.stride(0), wscale.data_ptr<float>(), bp, yp, y.stride(0), M, N, K, ss_per_wave);
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("skinny_gemm(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("skinny_gemm_fp8w(Tensor x, Tensor wq, Tensor wscale, Tensor? bias) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("skinny_gemm", &sxe::skinny_gemm);
  m.impl("skinny_gemm_fp8w", &sxe::skinny_gemm_fp8w);
}

// OCP-MX block-scaled GEMM on gfx950's scaled matrix cores (v_mfma_scale_f32_32x32x64_f8f6f4):
//   Y[M, N] = dequant(Xq, Xs) @ dequant(Wq, Ws)^T  (+ bias[N]) (* col_scale[N])
// with X quantized per 32-element K block to MXFP8 (e4m3 + one E8M0 exponent) by mx_quant_fp8 and
// W stored as MXFP8 (e4m3), MXFP6 (e3m2 or e2m3) or MXFP4 (e2m1) codes with one E8M0 exponent per
// 32 K elements. The dequantisation is done by the MFMA itself: each lane hands the instruction its
// 32 K-contiguous codes plus the block's exponent byte, so the weight never exists in bf16 -- in HBM,
// LDS or registers (the FP6-LLM counterpart, reference inference/v2/kernels/core_ops/cuda_linear/
// linear_kernels_cuda.cu:70,216, decodes FP6 to fp16 in registers and runs fp16 tensor cores).
//
// Operand maps (measured by tools/probes/mx_mfma_layout.hip + mx_layout_check.py on MI355X,
// profiles/mx_mfma_layout.log): in a 32x32x64 MFMA lane l feeds row / column (l & 31), half
// h = l >> 5, 32 codes (element j at bits [w j, w j + w) of the 8-dword operand, w = 8 / 6 / 4):
//   * 6- and 4-bit operands: K = 32 h + j -- the lane's codes are exactly K block h;
//   * 8-bit operands: K = 16 h + j for j < 16 and K = 32 + 16 h + (j - 16) for j >= 16 -- the
//     two 16-byte halves of the operand cover the two K blocks;
//   * the lane's E8M0 byte scales K block h of its row / column, wherever those codes sit (so an
//     fp8 lane's codes use its own exponent and its partner half's).
// Both operands are K-contiguous rows -- X as [M, K], W in nn.Linear's [N, K] layout -- so the
// layouts only decide which bytes of an LDS row a lane reads; no data is ever permuted.
//
// Geometry: BM x BN output tile (256x256 / 256x128 / 128x128), 8 waves as 2 (M) x 4 (N), each wave
// (BM/2) x (BN/4) as 32x32 accumulators; K in stages of 128 (two MFMA k-steps). Operand tiles are
// staged global -> registers -> LDS with rows padded by 16 B (row strides of 144 / 112 / 80 B put
// the 16 lanes of a ds_read_b128 phase on distinct banks); the next stage's loads (tiles + the
// lanes' scale words) are in flight while the current stage's MFMAs run. Workgroups are mapped
// XCD-major: the 8 XCDs each take a contiguous range of output tiles (M fastest), so the weight
// column tiles a workgroup streams are shared through its XCD's L2.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace mx {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 128, NTHR = 512;
constexpr int SA = 128 + 16;  // padded LDS row stride of the fp8 activation tile

// MFMA format codes (cbsz / blgp): 0 e4m3, 1 e5m2, 2 e2m3, 3 e3m2, 4 e2m1
__host__ __device__ constexpr int fmt_bits(int f) { return f <= 1 ? 8 : (f <= 3 ? 6 : 4); }

template <int FB>
struct BLayout {
  static constexpr int BITS = fmt_bits(FB);
  static constexpr int RB = 16 * BITS;  // bytes per row per 128-element K stage
  static constexpr int SB = RB + 16;    // padded LDS stride
  static constexpr int CPR = RB / 16;   // 16-byte chunks per row
  static constexpr int LB = 4 * BITS;   // bytes one lane feeds per MFMA (32 elements)
};

template <int ROWS, int CPR, int STRIDE>
struct Stager {
  static constexpr int N = (ROWS * CPR + NTHR - 1) / NTHR;
  u32x4 r[N];
  __device__ __forceinline__ void load(const uint8_t* base, int64_t row_bytes, int row0, int valid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHR;
      const int row = c / CPR, ch = c % CPR;
      r[i] = (c < ROWS * CPR && row0 + row < valid)
                 ? *reinterpret_cast<const u32x4*>(base + (int64_t)(row0 + row) * row_bytes + ch * 16)
                 : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(char* lds) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHR;
      if (c < ROWS * CPR) *reinterpret_cast<u32x4*>(lds + (c / CPR) * STRIDE + (c % CPR) * 16) = r[i];
    }
  }
};

// The 32 codes a lane feeds to one 64-K MFMA step, from the step's bytes of an LDS row (`p` points
// at the step's first byte): fp8 = bytes [16 h, 16 h + 16) and [32 + 16 h, 32 + 16 h + 16); fp6 /
// fp4 = the LB contiguous bytes of block h.
template <int LB>
__device__ __forceinline__ i32x8 lds_operand(const char* p, int h) {
  i32x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (LB == 32) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(p + 16 * h), b = *reinterpret_cast<const u32x4*>(p + 32 + 16 * h);
    v = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
    return v;
  }
  p += LB * h;
  if constexpr (LB == 24) {
    const u32x2 a = *reinterpret_cast<const u32x2*>(p), b = *reinterpret_cast<const u32x2*>(p + 8),
                c = *reinterpret_cast<const u32x2*>(p + 16);
    v = i32x8{(int)a[0], (int)a[1], (int)b[0], (int)b[1], (int)c[0], (int)c[1], 0, 0};
  } else {
    const u32x4 a = *reinterpret_cast<const u32x4*>(p);
    v = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], 0, 0, 0, 0};
  }
  return v;
}

template <int BM, int BN, int FB>
__global__ void __launch_bounds__(NTHR, 1)
    mx_gemm_kernel(const uint8_t* __restrict__ Xq, const uint8_t* __restrict__ Xs, const uint8_t* __restrict__ Wq,
                   const uint8_t* __restrict__ Ws, const unsigned short* __restrict__ bias,
                   const float* __restrict__ col_scale, unsigned short* __restrict__ Y, int M, int N, int K) {
  using L = BLayout<FB>;
  constexpr int TM = BM / 2, TN = BN / 4, MI = TM / 32, NJ = TN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* lA = smem;
  char* lB = smem + BM * SA;

  // ---- XCD-major tile order: XCD x (= blockIdx % 8) owns tiles [x G/8, (x+1) G/8), M fastest -----
  const int tm = (M + BM - 1) / BM, tn = N / BN, G = tm * tn;
  int pid = blockIdx.x;
  if ((G & 7) == 0) pid = (pid & 7) * (G >> 3) + (pid >> 3);
  const int m0 = (pid % tm) * BM, n0 = (pid / tm) * BN;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3, h = lane >> 5, l32 = lane & 31;
  const int KS = K / 32;          // scale bytes per row
  const int64_t WRB = (int64_t)K * L::BITS / 8;  // weight bytes per row

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // scale words (4 E8M0 bytes = one 128-K stage) of the rows / columns this lane feeds
  unsigned sa[MI], sb[NJ];
  auto load_scales = [&](int kb) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * TM + i * 32 + l32;
      sa[i] = m < M ? *reinterpret_cast<const unsigned*>(Xs + (int64_t)m * KS + 4 * kb) : 0x7f7f7f7fu;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * TN + j * 32 + l32;
      sb[j] = *reinterpret_cast<const unsigned*>(Ws + (int64_t)n * KS + 4 * kb);
    }
  };

  Stager<BM, 8, SA> stA;
  Stager<BN, L::CPR, L::SB> stB;
  stA.load(Xq, K, m0, M);
  stB.load(Wq, WRB, n0, N);
  load_scales(0);
  const int nk = K / BK;
  for (int kb = 0; kb < nk; ++kb) {
    if (kb) __syncthreads();
    stA.store(lA);
    stB.store(lB);
    unsigned csa[MI], csb[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) csa[i] = sa[i];
#pragma unroll
    for (int j = 0; j < NJ; ++j) csb[j] = sb[j];
    __syncthreads();
    if (kb + 1 < nk) {  // the next stage's loads overlap this stage's MFMAs
      stA.load(Xq + (int64_t)(kb + 1) * BK, K, m0, M);
      stB.load(Wq + (int64_t)(kb + 1) * L::RB, WRB, n0, N);
      load_scales(kb + 1);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      i32x8 a[MI], b[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = lds_operand<32>(lA + (wm * TM + i * 32 + l32) * SA + 64 * s, h);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        b[j] = lds_operand<L::LB>(lB + (wn * TN + j * 32 + l32) * L::SB + 2 * L::LB * s, h);
      const int sh = 8 * (2 * s + h);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              a[i], b[j], acc[i][j], 0, FB, 0, (int)((csa[i] >> sh) & 0xff), 0, (int)((csb[j] >> sh) & 0xff));
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // ---- epilogue: lane holds column n of 16 rows per accumulator -------------------------------------
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn * TN + j * 32 + l32;
    const float cs = col_scale ? col_scale[n] : 1.f;
    const float bv = bias ? bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) Y[(int64_t)m * N + n] = f32_to_bf16(acc[i][j][r] * cs + bv);
      }
  }
}

// X [M, K] bf16 -> e4m3 codes [M, K] + E8M0 exponents [M, K/32]; one thread per 32-element block.
// The block exponent is ceil(log2(amax / 448)), so every scaled element is within e4m3's range and
// the hardware converter (round to nearest even) never saturates.
__global__ void mx_quant_fp8_kernel(const unsigned short* __restrict__ x, uint8_t* __restrict__ q,
                                    uint8_t* __restrict__ s, int64_t nblocks) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const u16x8* p = reinterpret_cast<const u16x8*>(x + b * 32);
  u16x8 v[4];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = p[c];
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(bf16_to_f32(v[c][e])));
  }
  int ex = -127;
  if (amax > 0.f) {
    int fe;
    const float f = frexpf(amax * (1.f / 448.f), &fe);
    ex = (f == 0.5f) ? fe - 1 : fe;
    if (ldexpf(amax, -ex) > 448.f) ++ex;
    ex = max(-127, min(127, ex));
  }
  s[b] = (uint8_t)(ex + 127);
  const float inv = ldexpf(1.f, -ex);
  unsigned out[8];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int e = 0; e < 8; e += 4) {
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[c][e]) * inv, bf16_to_f32(v[c][e + 1]) * inv, 0, false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[c][e + 2]) * inv, bf16_to_f32(v[c][e + 3]) * inv, pk, true);
      out[2 * c + e / 4] = (unsigned)pk;
    }
  u32x4* o = reinterpret_cast<u32x4*>(q + b * 32);
  o[0] = u32x4{out[0], out[1], out[2], out[3]};
  o[1] = u32x4{out[4], out[5], out[6], out[7]};
}

template <int BM, int BN, int FB>
void launch(const at::Tensor& xq, const at::Tensor& xs, const at::Tensor& wq, const at::Tensor& ws,
            const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& col_scale, at::Tensor& y, int M,
            int N, int K) {
  const size_t lds = (size_t)BM * SA + (size_t)BN * BLayout<FB>::SB;
  static bool attr = [&] {
    SXE_HIP_CHECK(hipFuncSetAttribute((const void*)mx_gemm_kernel<BM, BN, FB>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return true;
  }();
  (void)attr;
  const int G = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((mx_gemm_kernel<BM, BN, FB>), dim3(G), dim3(NTHR), lds, cur_stream(), xq.data_ptr<uint8_t>(),
                     xs.data_ptr<uint8_t>(), wq.data_ptr<uint8_t>(), ws.data_ptr<uint8_t>(),
                     bias ? reinterpret_cast<const unsigned short*>(bias->data_ptr()) : nullptr,
                     col_scale ? col_scale->data_ptr<float>() : nullptr,
                     reinterpret_cast<unsigned short*>(y.data_ptr()), M, N, K);
}

template <int FB>
void dispatch_tile(const at::Tensor& xq, const at::Tensor& xs, const at::Tensor& wq, const at::Tensor& ws,
                   const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& cs, at::Tensor& y, int M,
                   int N, int K) {
  // largest tile that still gives >= 1 workgroup per CU; 128 x 128 for small problems
  const int64_t g256 = (int64_t)((M + 255) / 256) * (N / 256), g2561 = (int64_t)((M + 255) / 256) * (N / 128);
  if (N % 256 == 0 && M > 128 && g256 >= kNumCUs)
    launch<256, 256, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K);
  else if (M > 128 && g2561 >= kNumCUs)
    launch<256, 128, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K);
  else
    launch<128, 128, FB>(xq, xs, wq, ws, bias, cs, y, M, N, K);
}

}  // namespace mx

// x [M, K] bf16 (K % 32 == 0) -> (e4m3 codes uint8 [M, K], E8M0 exponents uint8 [M, K / 32])
std::vector<at::Tensor> mx_quant_fp8(at::Tensor x) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.dim() == 2 && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "mx_quant_fp8: x [M, K] bf16");
  SXE_CHECK(x.size(1) % 32 == 0, "mx_quant_fp8: K must be a multiple of 32");
  c10::DeviceGuard guard(x.device());
  auto q = at::empty({x.size(0), x.size(1)}, x.options().dtype(at::kByte));
  auto s = at::empty({x.size(0), x.size(1) / 32}, x.options().dtype(at::kByte));
  const int64_t nb = x.numel() / 32;
  if (nb)
    hipLaunchKernelGGL(mx::mx_quant_fp8_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, cur_stream(),
                       reinterpret_cast<const unsigned short*>(x.data_ptr()), q.data_ptr<uint8_t>(),
                       s.data_ptr<uint8_t>(), nb);
  SXE_LAUNCH_CHECK();
  return {q, s};
}

// y [M, N] bf16 = MX(xq, xs) @ MX(wq, ws)^T (+ bias) (* col_scale); fmt: 0 e4m3, 2 e2m3, 3 e3m2, 4 e2m1
at::Tensor mx_gemm(at::Tensor xq, at::Tensor xs, at::Tensor wq, at::Tensor ws, int64_t fmt,
                   c10::optional<at::Tensor> bias, c10::optional<at::Tensor> col_scale) {
  SXE_CHECK_CUDA(xq);
  SXE_CHECK(fmt == 0 || fmt == 2 || fmt == 3 || fmt == 4, "mx_gemm: weight format 0 (e4m3) / 2 (e2m3) / 3 (e3m2) / 4 (e2m1)");
  SXE_CHECK(xq.dim() == 2 && xq.is_contiguous() && xq.scalar_type() == at::kByte, "mx_gemm: xq uint8 [M, K]");
  const int64_t M = xq.size(0), K = xq.size(1), N = ws.size(0);
  const int bits = mx::fmt_bits((int)fmt);
  SXE_CHECK(K % mx::BK == 0, "mx_gemm: K must be a multiple of 128");
  SXE_CHECK(N % 128 == 0, "mx_gemm: N must be a multiple of 128");
  SXE_CHECK(xs.is_contiguous() && xs.scalar_type() == at::kByte && xs.numel() == M * (K / 32), "mx_gemm: xs uint8 [M, K/32]");
  SXE_CHECK(wq.is_contiguous() && wq.scalar_type() == at::kByte && wq.numel() == N * K * bits / 8,
            "mx_gemm: wq packed codes [N, K * bits / 8]");
  SXE_CHECK(ws.dim() == 2 && ws.is_contiguous() && ws.scalar_type() == at::kByte && ws.size(1) == K / 32,
            "mx_gemm: ws uint8 [N, K/32]");
  SXE_CHECK(xs.is_cuda() && wq.is_cuda() && ws.is_cuda(), "mx_gemm: operands on the GPU");
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N,
              "mx_gemm: bias bf16 [N]");
  } else {
    bias = c10::nullopt;
  }
  if (col_scale.has_value() && col_scale->defined()) {
    SXE_CHECK(col_scale->is_cuda() && col_scale->is_contiguous() && col_scale->scalar_type() == at::kFloat &&
                  col_scale->numel() == N,
              "mx_gemm: col_scale fp32 [N]");
  } else {
    col_scale = c10::nullopt;
  }
  SXE_CHECK(M * N < (1ll << 31) && N * K < (1ll << 31), "mx_gemm: problem too large");
  c10::DeviceGuard guard(xq.device());
  auto y = at::empty({M, N}, xq.options().dtype(at::kBFloat16));
  if (M == 0) return y;
  switch (fmt) {
    case 0: mx::dispatch_tile<0>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
    case 2: mx::dispatch_tile<2>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
    case 3: mx::dispatch_tile<3>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
    default: mx::dispatch_tile<4>(xq, xs, wq, ws, bias, col_scale, y, (int)M, (int)N, (int)K); break;
  }
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("mx_quant_fp8(Tensor x) -> Tensor[]");
  m.def("mx_gemm(Tensor xq, Tensor xs, Tensor wq, Tensor ws, int fmt, Tensor? bias=None, Tensor? col_scale=None) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("mx_quant_fp8", &sxe::mx_quant_fp8);
  m.impl("mx_gemm", &sxe::mx_gemm);
}

// Block-sparse matrix multiplication for gfx950 (MI355X): the three products of the reference's
// ops/sparse_attention/matmul.py:628 ``MatMul`` (Triton SDD / DSD / DDS kernels), bf16 / fp16 in,
// fp32 accumulate, 16-bit out. Sparse operands use the reference format [B, nnz, blk, blk] (the
// non-zero blocks of a layout [H, M, N] in layout.nonzero() order).
//
//   sdd: C[b, nz] = A[b, h, i-block rows, :] . B[b, h, :, j-block cols]          (nz = (h, i, j))
//   dsd: C[b, h, r-block, :] = sum_{nz in row r} S[b, nz] . D[b, h, c(nz)-block rows, :]
//   dds: C[b, h, :, c-block] = sum_{nz in col c} D[b, h, :, r(nz)-block cols] . S[b, nz]
//
// Every operand is read in place through element strides (transposed inputs and broadcast heads
// cost nothing): no gathered copies of the dense panels, no [nnz, blk, K] intermediates and no
// index_add of partial products -- the DSD / DDS kernels walk the layout's CSR / CSC lists and sum
// a block row's (column's) products in registers. MFMA: v_mfma_f32_16x16x32_{bf16,f16}, each wave
// owning 16x16 output tiles (blk 16 .. 128 -> 1 .. 64 tiles per block); A / B fragments are 16-byte
// vector loads along the reduction dim when it is unit-stride, element gathers otherwise (the
// transposed operand of a backward product); operands stay L2-resident across the tiles of a block.
#include "sxe_common.h"

#include <torch/library.h>

namespace sxe {
namespace bsm {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <DT T>
__device__ __forceinline__ f32x4 mma(u16x8 a, u16x8 b, f32x4 c) {
  if constexpr (T == DT::BF16) {
    const bf16x8 x = __builtin_bit_cast(bf16x8, a);
    const bf16x8 y = __builtin_bit_cast(bf16x8, b);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c, 0, 0, 0);
  } else {
    const f16x8 x = __builtin_bit_cast(f16x8, a);
    const f16x8 y = __builtin_bit_cast(f16x8, b);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
  }
}

// 8 reduction-consecutive elements (k0 .. k0+7) of one operand row / column; zero past K
__device__ __forceinline__ u16x8 frag(const unsigned short* base, int64_t sk, int k0, int K) {
  if (sk == 1 && k0 + 8 <= K && (((uintptr_t)(base + k0)) & 15) == 0)
    return *reinterpret_cast<const u16x8*>(base + k0);
  u16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (k0 + j < K) ? base[(int64_t)(k0 + j) * sk] : (unsigned short)0;
  return v;
}

// acc (16x16, lane layout col = lane & 15, rows 4 (lane >> 4) + e) += A[16 rows, 0:K] . B[0:K, 16 cols]
// arow: this lane's A row at k = 0 (row r0 + (lane & 15)); bcol: this lane's B column at k = 0
template <DT T>
__device__ __forceinline__ void tile_mma(f32x4& acc, const unsigned short* arow, int64_t ask,
                                         const unsigned short* bcol, int64_t bsk, int K, int lane) {
  const int kq = 8 * (lane >> 4);
  for (int k0 = 0; k0 < K; k0 += 32) {
    const u16x8 a = frag(arow, ask, k0 + kq, K);
    const u16x8 b = frag(bcol, bsk, k0 + kq, K);
    acc = mma<T>(a, b, acc);
  }
}

struct Dense {  // logical [B, H, rows, cols] view: element (b, h, r, c) at p[b sb + h sh + r sr + c sc]
  const unsigned short* p;
  int64_t sb, sh, sr, sc;
};

// grid (nnz, B); 256 threads; the waves split the block's 16x16 tiles
template <DT T>
__global__ void __launch_bounds__(256) sdd_kernel(Dense A, Dense Bm, const int* __restrict__ hij,
                                                  unsigned short* __restrict__ C, int nnz, int blk, int K) {
  const int nz = blockIdx.x, b = blockIdx.y;
  const int h = hij[3 * nz], i = hij[3 * nz + 1], j = hij[3 * nz + 2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = blk / 16;
  const unsigned short* ab = A.p + b * A.sb + h * A.sh;
  const unsigned short* bb = Bm.p + b * Bm.sb + h * Bm.sh;
  unsigned short* cb = C + ((int64_t)b * nnz + nz) * blk * blk;
  for (int t = w; t < nt * nt; t += 4) {
    const int tr = t / nt, tc = t - tr * nt;
    const int64_t r = (int64_t)i * blk + tr * 16 + (lane & 15);
    const int64_t c = (int64_t)j * blk + tc * 16 + (lane & 15);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    tile_mma<T>(acc, ab + r * A.sr, A.sc, bb + c * Bm.sc, Bm.sr, K, lane);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      cb[(tr * 16 + 4 * (lane >> 4) + e) * blk + tc * 16 + (lane & 15)] = from_f32<T>(acc[e]);
  }
}

// grid (H * rows, ceil(Nd / 64), B); output row block g = (h, r): blk rows x 64 columns per workgroup
// S element (row, k) of block nz at S + nz blk^2 + row ssr + k ssk (trans: the block is read transposed)
template <DT T>
__global__ void __launch_bounds__(256) dsd_kernel(const unsigned short* __restrict__ S, int64_t s_sb, int ssr, int ssk,
                                                  Dense D, const int* __restrict__ ptr, const int* __restrict__ ent,
                                                  unsigned short* __restrict__ C, int rows, int blk, int Nd) {
  const int g = blockIdx.x, n0 = blockIdx.y * 64, b = blockIdx.z;
  const int h = g / rows;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = blk / 16;
  const int ncol = min(4, (Nd - n0) / 16);
  const int e0 = ptr[g], e1 = ptr[g + 1];
  const unsigned short* db = D.p + b * D.sb + h * D.sh;
  const unsigned short* sb = S + b * s_sb;
  unsigned short* cb = C + (((int64_t)b * gridDim.x + g) * blk) * Nd;
  for (int t = w; t < nt * ncol; t += 4) {
    const int tr = t / ncol, tc = t - tr * ncol;
    const int64_t col = n0 + tc * 16 + (lane & 15);
    const int row = tr * 16 + (lane & 15);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e = e0; e < e1; ++e) {
      const int nz = ent[2 * e], ci = ent[2 * e + 1];
      tile_mma<T>(acc, sb + (int64_t)nz * blk * blk + row * ssr, ssk, db + (int64_t)ci * blk * D.sr + col * D.sc, D.sr,
                  blk, lane);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) cb[(int64_t)(tr * 16 + 4 * (lane >> 4) + e) * Nd + col] = from_f32<T>(acc[e]);
  }
}

// grid (H * cols, ceil(Md / 64), B); output column block g = (h, c): 64 rows x blk columns per
// workgroup; S element (k, col) of block nz at S + nz blk^2 + k ssk + col ssc
template <DT T>
__global__ void __launch_bounds__(256) dds_kernel(Dense D, const unsigned short* __restrict__ S, int64_t s_sb, int ssk,
                                                  int ssc, const int* __restrict__ ptr, const int* __restrict__ ent,
                                                  unsigned short* __restrict__ C, int cols, int blk, int Md) {
  const int g = blockIdx.x, m0 = blockIdx.y * 64, b = blockIdx.z;
  const int h = g / cols, cj = g - h * cols;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = blk / 16;
  const int nrow = min(4, (Md - m0) / 16);
  const int e0 = ptr[g], e1 = ptr[g + 1];
  const unsigned short* db = D.p + b * D.sb + h * D.sh;
  const unsigned short* sb = S + b * s_sb;
  const int64_t ldc = (int64_t)cols * blk;
  unsigned short* cb = C + (((int64_t)b * (gridDim.x / cols) + h) * Md) * ldc + (int64_t)cj * blk;
  for (int t = w; t < nrow * nt; t += 4) {
    const int tr = t / nt, tc = t - tr * nt;
    const int64_t row = m0 + tr * 16 + (lane & 15);
    const int col = tc * 16 + (lane & 15);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e = e0; e < e1; ++e) {
      const int nz = ent[2 * e], ri = ent[2 * e + 1];
      tile_mma<T>(acc, db + row * D.sr + (int64_t)ri * blk * D.sc, D.sc, sb + (int64_t)nz * blk * blk + col * ssc, ssk,
                  blk, lane);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      cb[(int64_t)(m0 + tr * 16 + 4 * (lane >> 4) + e) * ldc + tc * 16 + (lane & 15)] = from_f32<T>(acc[e]);
  }
}

Dense dense_of(const at::Tensor& t, int64_t sb, int64_t sh, int64_t sr, int64_t sc) {
  return Dense{reinterpret_cast<const unsigned short*>(t.data_ptr()), sb, sh, sr, sc};
}

void check16(const at::Tensor& t, const char* what) {
  SXE_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  SXE_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, what, " must be bf16 or fp16");
}

}  // namespace bsm

// a / b: the logical operands (any strides) [B, Ha|1, M*blk, K] and [B, Hb|1, K, N*blk]
at::Tensor bsmm_sdd(at::Tensor a, at::Tensor b, at::Tensor hij, int64_t blk) {
  bsm::check16(a, "a");
  bsm::check16(b, "b");
  SXE_CHECK(a.scalar_type() == b.scalar_type(), "bsmm_sdd: a and b dtypes differ");
  SXE_CHECK(a.dim() == 4 && b.dim() == 4 && a.size(3) == b.size(2), "bsmm_sdd: [B, H, M, K] x [B, H, K, N]");
  SXE_CHECK(blk % 16 == 0 && blk >= 16 && blk <= 128, "bsmm_sdd: block must be 16, 32, 64 or 128");
  SXE_CHECK(hij.scalar_type() == at::kInt && hij.is_contiguous() && hij.dim() == 2 && hij.size(1) == 3,
            "bsmm_sdd: hij int32 [nnz, 3]");
  const int64_t B = std::max(a.size(0), b.size(0)), nnz = hij.size(0), K = a.size(3);
  c10::DeviceGuard guard(a.device());
  auto c = at::empty({B, nnz, blk, blk}, a.options());
  if (nnz == 0 || B == 0) return c;
  auto A = bsm::dense_of(a, a.size(0) > 1 ? a.stride(0) : 0, a.size(1) > 1 ? a.stride(1) : 0, a.stride(2), a.stride(3));
  auto Bm = bsm::dense_of(b, b.size(0) > 1 ? b.stride(0) : 0, b.size(1) > 1 ? b.stride(1) : 0, b.stride(2), b.stride(3));
  dim3 grid((unsigned)nnz, (unsigned)B);
  auto* cp = reinterpret_cast<unsigned short*>(c.data_ptr());
  if (a.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(bsm::sdd_kernel<DT::BF16>, grid, dim3(256), 0, cur_stream(), A, Bm, hij.data_ptr<int>(), cp,
                       (int)nnz, (int)blk, (int)K);
  else
    hipLaunchKernelGGL(bsm::sdd_kernel<DT::F16>, grid, dim3(256), 0, cur_stream(), A, Bm, hij.data_ptr<int>(), cp,
                       (int)nnz, (int)blk, (int)K);
  SXE_LAUNCH_CHECK();
  return c;
}

// s: [B|1, nnz, blk, blk] contiguous; trans: read each block transposed; d: logical [B, Hd|1, cols*blk, Nd];
// ptr [H*rows + 1] / ent [nnz, 2] = (nz, block column) CSR of the output block rows
at::Tensor bsmm_dsd(at::Tensor s, bool trans, at::Tensor d, at::Tensor ptr, at::Tensor ent, int64_t H, int64_t rows,
                    int64_t blk) {
  bsm::check16(s, "s");
  bsm::check16(d, "d");
  SXE_CHECK(s.scalar_type() == d.scalar_type(), "bsmm_dsd: dtypes differ");
  SXE_CHECK(s.dim() == 4 && s.is_contiguous() && s.size(2) == blk && s.size(3) == blk, "bsmm_dsd: s [B, nnz, blk, blk]");
  SXE_CHECK(d.dim() == 4, "bsmm_dsd: d [B, H, K, N]");
  SXE_CHECK(blk % 16 == 0 && blk >= 16 && blk <= 128, "bsmm_dsd: block must be 16, 32, 64 or 128");
  const int64_t Nd = d.size(3);
  SXE_CHECK(Nd % 16 == 0, "bsmm_dsd: dense columns must be a multiple of 16");
  SXE_CHECK(ptr.scalar_type() == at::kInt && ent.scalar_type() == at::kInt && ptr.numel() == H * rows + 1,
            "bsmm_dsd: CSR lists");
  const int64_t B = std::max(s.size(0), d.size(0));
  c10::DeviceGuard guard(s.device());
  auto c = at::empty({B, H, rows * blk, Nd}, s.options());
  if (B == 0 || Nd == 0) return c;
  auto D = bsm::dense_of(d, d.size(0) > 1 ? d.stride(0) : 0, d.size(1) > 1 ? d.stride(1) : 0, d.stride(2), d.stride(3));
  const int64_t s_sb = s.size(0) > 1 ? s.stride(0) : 0;
  const int ssr = trans ? 1 : (int)blk, ssk = trans ? (int)blk : 1;
  dim3 grid((unsigned)(H * rows), (unsigned)((Nd + 63) / 64), (unsigned)B);
  auto* sp = reinterpret_cast<const unsigned short*>(s.data_ptr());
  auto* cp = reinterpret_cast<unsigned short*>(c.data_ptr());
  if (s.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(bsm::dsd_kernel<DT::BF16>, grid, dim3(256), 0, cur_stream(), sp, s_sb, ssr, ssk, D,
                       ptr.data_ptr<int>(), ent.data_ptr<int>(), cp, (int)rows, (int)blk, (int)Nd);
  else
    hipLaunchKernelGGL(bsm::dsd_kernel<DT::F16>, grid, dim3(256), 0, cur_stream(), sp, s_sb, ssr, ssk, D,
                       ptr.data_ptr<int>(), ent.data_ptr<int>(), cp, (int)rows, (int)blk, (int)Nd);
  SXE_LAUNCH_CHECK();
  return c;
}

// d: logical [B, Hd|1, Md, rows*blk]; s: [B|1, nnz, blk, blk]; ptr / ent = (nz, block row) CSC lists
at::Tensor bsmm_dds(at::Tensor d, at::Tensor s, bool trans, at::Tensor ptr, at::Tensor ent, int64_t H, int64_t cols,
                    int64_t blk) {
  bsm::check16(s, "s");
  bsm::check16(d, "d");
  SXE_CHECK(s.scalar_type() == d.scalar_type(), "bsmm_dds: dtypes differ");
  SXE_CHECK(s.dim() == 4 && s.is_contiguous() && s.size(2) == blk && s.size(3) == blk, "bsmm_dds: s [B, nnz, blk, blk]");
  SXE_CHECK(d.dim() == 4, "bsmm_dds: d [B, H, M, K]");
  SXE_CHECK(blk % 16 == 0 && blk >= 16 && blk <= 128, "bsmm_dds: block must be 16, 32, 64 or 128");
  const int64_t Md = d.size(2);
  SXE_CHECK(Md % 16 == 0, "bsmm_dds: dense rows must be a multiple of 16");
  SXE_CHECK(ptr.scalar_type() == at::kInt && ent.scalar_type() == at::kInt && ptr.numel() == H * cols + 1,
            "bsmm_dds: CSC lists");
  const int64_t B = std::max(s.size(0), d.size(0));
  c10::DeviceGuard guard(s.device());
  auto c = at::empty({B, H, Md, cols * blk}, s.options());
  if (B == 0 || Md == 0) return c;
  auto D = bsm::dense_of(d, d.size(0) > 1 ? d.stride(0) : 0, d.size(1) > 1 ? d.stride(1) : 0, d.stride(2), d.stride(3));
  const int64_t s_sb = s.size(0) > 1 ? s.stride(0) : 0;
  const int ssk = trans ? 1 : (int)blk, ssc = trans ? (int)blk : 1;
  dim3 grid((unsigned)(H * cols), (unsigned)((Md + 63) / 64), (unsigned)B);
  auto* sp = reinterpret_cast<const unsigned short*>(s.data_ptr());
  auto* cp = reinterpret_cast<unsigned short*>(c.data_ptr());
  if (s.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(bsm::dds_kernel<DT::BF16>, grid, dim3(256), 0, cur_stream(), D, sp, s_sb, ssk, ssc,
                       ptr.data_ptr<int>(), ent.data_ptr<int>(), cp, (int)cols, (int)blk, (int)Md);
  else
    hipLaunchKernelGGL(bsm::dds_kernel<DT::F16>, grid, dim3(256), 0, cur_stream(), D, sp, s_sb, ssk, ssc,
                       ptr.data_ptr<int>(), ent.data_ptr<int>(), cp, (int)cols, (int)blk, (int)Md);
  SXE_LAUNCH_CHECK();
  return c;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("bsmm_sdd(Tensor a, Tensor b, Tensor hij, int blk) -> Tensor");
  m.def("bsmm_dsd(Tensor s, bool trans, Tensor d, Tensor ptr, Tensor ent, int H, int rows, int blk) -> Tensor");
  m.def("bsmm_dds(Tensor d, Tensor s, bool trans, Tensor ptr, Tensor ent, int H, int cols, int blk) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("bsmm_sdd", &sxe::bsmm_sdd);
  m.impl("bsmm_dsd", &sxe::bsmm_dsd);
  m.impl("bsmm_dds", &sxe::bsmm_dds);
}

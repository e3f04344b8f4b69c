// MFMA / LDS building blocks shared by the attention-shaped kernels (32x32x16 bf16 MFMA, 64-wide
// waves, XOR-swizzled 256-byte LDS rows readable both by rows (ds_read_b128) and transposed
// (ds_read_b64_tr_b16)). See csrc/kernels/flash_attn.hip for the derivation of every map.
#pragma once
#include <hip/hip_runtime.h>
#include "sxe_common.h"

namespace sxe {
namespace mf {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int ROWB = 256;  // bytes per LDS row (128 bf16); narrower heads use the first chunks
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// byte offset of 16-byte chunk `ch` (0..15) of row `row` in a swizzled [rows][256 B] tile
__device__ __forceinline__ int soff(int row, int ch) {
  return row * ROWB + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ bf16x8 lds_row16(const char* base, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(base + soff(row, ch));
}

__device__ __forceinline__ i16x4 lds_tr(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(const_cast<char*>(base) + byte_off));
}

// A operand of a 32x32x16 MFMA read transposed from a row-major tile: A[m = d][k = row], rows
// permuted to match an accumulator reused as the B operand (see flash_attn.hip lds_trA)
__device__ __forceinline__ bf16x8 lds_trA(const char* base, int row0, int dt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const int row = row0 + 4 * h + q;
  i16x4 lo = lds_tr(base, soff(row, ch) + 8 * (p & 1));
  i16x4 hi = lds_tr(base, soff(row + 8, ch) + 8 * (p & 1));
  const i16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

__device__ __forceinline__ bf16x8 acc_to_b(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)a[8 * s + e];
  return r;
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// accumulator register i <-> row within a 32x32 tile for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Epilogue of a TRANSPOSED accumulator (the weight was the MFMA's A operand, so the 32x32 tile is
// Y^T): lane (l32, h) owns one output row and registers 4g .. 4g+3 are its columns 8g + 4h + 0..3.
// `y` points at that row's column 4h of the tile; one 8-byte store per run, no per-element branch
// or load (a per-element `if` + scale load makes hipcc wait vmcnt(0) -- i.e. for the previous
// store -- before every element).
__device__ __forceinline__ void store_acc_t(const f32x16& c, unsigned short* y, float s) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const unsigned lo = (unsigned)f32_to_bf16(c[4 * g] * s) | ((unsigned)f32_to_bf16(c[4 * g + 1] * s) << 16);
    const unsigned hi = (unsigned)f32_to_bf16(c[4 * g + 2] * s) | ((unsigned)f32_to_bf16(c[4 * g + 3] * s) << 16);
    *reinterpret_cast<unsigned long long*>(y + 8 * g) = (unsigned long long)lo | ((unsigned long long)hi << 32);
  }
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// Stage ROWS rows x DH bf16 (DH/8 chunks per row) from global into swizzled LDS through registers
// (issue early with load(), write late with store()); rows at or beyond `valid` read as zeros.
template <int ROWS, int DH, int NTHREADS>
struct RowStager {
  static constexpr int CPR = DH / 8;  // 16-byte chunks per row
  static constexpr int N = (ROWS * CPR + NTHREADS - 1) / NTHREADS;
  u32x4 r[N];
  __device__ __forceinline__ void load(const unsigned short* base, int64_t row_stride, int row0, int valid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHREADS;
      const int row = c / CPR, ch = c % CPR;
      r[i] = (c < ROWS * CPR && row0 + row < valid)
                 ? *reinterpret_cast<const u32x4*>(base + (int64_t)(row0 + row) * row_stride + ch * 8)
                 : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(char* lds) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NTHREADS;
      if (c < ROWS * CPR) *reinterpret_cast<u32x4*>(lds + soff(c / CPR, c % CPR)) = r[i];
    }
  }
};

}  // namespace mf
}  // namespace sxe

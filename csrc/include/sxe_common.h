// Shared device helpers for the gfx950 (CDNA4) kernels of shuffle_exchange_amd.
//
// Conventions (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md):
//  * wave = 64 lanes, always; reductions use 64-wide butterflies (__shfl_xor up to 32).
//  * every memory-bound kernel moves 16 bytes per lane per access (Guideline 13): bf16 as
//    8-element vectors, fp32 as float4.
//  * bf16 <-> f32 conversion: widening is a shift; narrowing is a plain cast to __bf16, which
//    hipcc lowers to v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserving).
#pragma once
#include <hip/hip_runtime.h>
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <stdint.h>

#define SXE_CHECK(cond, ...) TORCH_CHECK(cond, "sxe: ", __VA_ARGS__)
#define SXE_CHECK_CUDA(t) SXE_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define SXE_CHECK_CONTIG(t) SXE_CHECK((t).is_contiguous(), #t " must be contiguous")
#define SXE_HIP_CHECK(expr)                                                          \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    TORCH_CHECK(_e == hipSuccess, "sxe HIP error: ", hipGetErrorString(_e), " @ ",   \
                __FILE__, ":", __LINE__);                                            \
  } while (0)
#define SXE_LAUNCH_CHECK() SXE_HIP_CHECK(hipGetLastError())

namespace sxe {

constexpr int kWave = 64;
constexpr int kNumCUs = 256;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(unsigned short u) {
  return __uint_as_float(((unsigned)u) << 16);
}
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float f16_to_f32(unsigned short u) {
  return (float)__builtin_bit_cast(_Float16, u);
}
__device__ __forceinline__ unsigned short f32_to_f16(float f) {
  return __builtin_bit_cast(unsigned short, (_Float16)f);
}

// Element-type traits for the three floating types the framework moves around.
enum class DT : int { F32 = 0, BF16 = 1, F16 = 2 };

template <DT T> struct dt_traits;
template <> struct dt_traits<DT::F32> { using storage = float; };
template <> struct dt_traits<DT::BF16> { using storage = unsigned short; };
template <> struct dt_traits<DT::F16> { using storage = unsigned short; };

template <DT T>
__device__ __forceinline__ float to_f32(typename dt_traits<T>::storage v) {
  if constexpr (T == DT::F32) return v;
  else if constexpr (T == DT::BF16) return bf16_to_f32(v);
  else return f16_to_f32(v);
}
template <DT T>
__device__ __forceinline__ typename dt_traits<T>::storage from_f32(float v) {
  if constexpr (T == DT::F32) return v;
  else if constexpr (T == DT::BF16) return f32_to_bf16(v);
  else return f32_to_f16(v);
}

// Load/store 8 consecutive elements (16 B for 16-bit types, 2 x 16 B for f32) as f32.
template <DT T>
__device__ __forceinline__ void load8(const typename dt_traits<T>::storage* p, float (&v)[8]) {
  if constexpr (T == DT::F32) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[4 + i] = b[i]; }
  } else {
    u16x8 a = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = to_f32<T>(a[i]);
  }
}
template <DT T>
__device__ __forceinline__ void store8(typename dt_traits<T>::storage* p, const float (&v)[8]) {
  if constexpr (T == DT::F32) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = v[i]; b[i] = v[4 + i]; }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  } else {
    u16x8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = from_f32<T>(v[i]);
    *reinterpret_cast<u16x8*>(p) = a;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of NW waves; `red` must hold NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  __syncthreads();
  return t;
}

inline DT dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DT::F32;
    case at::kBFloat16: return DT::BF16;
    case at::kHalf: return DT::F16;
    default: TORCH_CHECK(false, "sxe: unsupported dtype ", t.scalar_type());
  }
}

// Memory-bound grid sizing (Guideline 11): enough blocks to fill 256 CUs x 8, grid-stride rest.
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > (int64_t)kNumCUs * 8) g = (int64_t)kNumCUs * 8;
  return (int)(g < 1 ? 1 : g);
}

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

}  // namespace sxe

// Dispatch helper over {f32, bf16, f16} -> constexpr DT.
#define SXE_DISPATCH_DT(dt, NAME, ...)                               \
  switch (dt) {                                                      \
    case ::sxe::DT::F32: { constexpr ::sxe::DT NAME = ::sxe::DT::F32; __VA_ARGS__; break; }   \
    case ::sxe::DT::BF16: { constexpr ::sxe::DT NAME = ::sxe::DT::BF16; __VA_ARGS__; break; } \
    case ::sxe::DT::F16: { constexpr ::sxe::DT NAME = ::sxe::DT::F16; __VA_ARGS__; break; }   \
  }

#define SXE_DISPATCH_BOOL(cond, NAME, ...) \
  if (cond) { constexpr bool NAME = true; __VA_ARGS__; } else { constexpr bool NAME = false; __VA_ARGS__; }

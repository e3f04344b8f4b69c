// Probe: O^T (32 d x 32 n) = V^T (32 d x 32 keys) * X (32 keys x 32 n) with X held as a 32x32x16
// accumulator and V^T read from a swizzled row-major LDS tile through ds_read_b64_tr_b16.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ int soff(int row, int ch) { return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }
__device__ i16x4 lds_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(const_cast<char*>(base) + off));
}
__device__ bf16x8 lds_trA(const char* base, int row0, int dt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const int row = row0 + 4 * h + q;
  i16x4 lo = lds_tr(base, soff(row, ch) + 8 * (p & 1));
  i16x4 hi = lds_tr(base, soff(row + 8, ch) + 8 * (p & 1));
  // whole-vector bitcast: element-wise bf16 inserts from the tr-read result miscompile (hipcc 7.2)
  const i16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}
__global__ void k(const float* V /*32x128*/, const float* X /*32x32*/, float* O /*128 x 32 (d,n)*/, int dyn) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  for (int idx = lane; idx < 32 * 16; idx += 64) {
    int row = idx >> 4, ch = idx & 15;
    __bf16 tmp[8];
    for (int e = 0; e < 8; ++e) tmp[e] = (__bf16)V[row * 128 + ch * 8 + e];
    *reinterpret_cast<bf16x8*>(smem + soff(row, ch)) = *reinterpret_cast<bf16x8*>(tmp);
  }
  __syncthreads();
  f32x16 x;
  for (int i = 0; i < 16; ++i) x[i] = X[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
  for (int dt = 0; dt < 4; ++dt) {
    f32x16 o; for (int i = 0; i < 16; ++i) o[i] = 0.f;
    for (int s = 0; s < 2; ++s) {
      bf16x8 b; for (int e = 0; e < 8; ++e) b[e] = (__bf16)x[8 * s + e];
      o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_trA(smem, 16 * s, dt, lane), b, o, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) O[(32 * dt + (i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = o[i];
  }
}
int main() {
  float hV[32 * 128], hX[32 * 32], hO[128 * 32];
  srand(1);
  for (int i = 0; i < 32 * 128; ++i) hV[i] = (float)(rand() % 7 - 3);
  for (int i = 0; i < 32 * 32; ++i) hX[i] = (float)(rand() % 5 - 2);
  float *dV, *dX, *dO;
  (void)hipMalloc(&dV, sizeof(hV)); (void)hipMalloc(&dX, sizeof(hX)); (void)hipMalloc(&dO, sizeof(hO));
  (void)hipMemcpy(dV, hV, sizeof(hV), hipMemcpyHostToDevice); (void)hipMemcpy(dX, hX, sizeof(hX), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 16384, 0, dV, dX, dO, 1);
  (void)hipMemcpy(hO, dO, sizeof(hO), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int d = 0; d < 128; ++d) for (int n = 0; n < 32; ++n) {
    float ref = 0; for (int kk = 0; kk < 32; ++kk) ref += hV[kk * 128 + d] * hX[kk * 32 + n];
    if (fabsf(ref - hO[d * 32 + n]) > 1e-3) { if (bad < 10) printf("d=%d n=%d got %f ref %f\n", d, n, hO[d * 32 + n], ref); ++bad; }
  }
  printf("mismatches: %d / %d\n", bad, 128 * 32);
  return 0;
}

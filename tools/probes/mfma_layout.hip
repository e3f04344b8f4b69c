// Reveal v_mfma_f32_32x32x16_bf16 operand pairing and C/D layout empirically.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void pairing(float* out) {  // out[pos] = code of B position paired with A position pos
  const int l = threadIdx.x, h = l >> 5;
  for (int pos = 0; pos < 16; ++pos) {
    const int h0 = pos >> 3, j0 = pos & 7;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)((h == h0 && j == j0) ? 1.f : 0.f); b[j] = (__bf16)(float)(16 * h + j + 1); }
    f32x16 c; for (int i = 0; i < 16; ++i) c[i] = 0.f;
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    if (l == 0) out[pos] = c[0];
  }
}
__global__ void clayout(float* rows, float* cols) {
  const int l = threadIdx.x, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)((h == 0 && j == 0) ? (float)((l & 31) + 1) : 0.f); b[j] = (__bf16)((h == 0 && j == 0) ? 1.f : 0.f); }
  f32x16 c; for (int i = 0; i < 16; ++i) c[i] = 0.f;
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) rows[l * 16 + i] = c[i] - 1;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)((h == 0 && j == 0) ? 1.f : 0.f); b[j] = (__bf16)((h == 0 && j == 0) ? (float)((l & 31) + 1) : 0.f); }
  for (int i = 0; i < 16; ++i) c[i] = 0.f;
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) cols[l * 16 + i] = c[i] - 1;
}
int main() {
  float *d1, *d2, *d3; (void)hipMalloc(&d1, 64); (void)hipMalloc(&d2, 4096); (void)hipMalloc(&d3, 4096);
  hipLaunchKernelGGL(pairing, dim3(1), dim3(64), 0, 0, d1);
  hipLaunchKernelGGL(clayout, dim3(1), dim3(64), 0, 0, d2, d3);
  float p[16], r[1024], c[1024];
  (void)hipMemcpy(p, d1, 64, hipMemcpyDeviceToHost); (void)hipMemcpy(r, d2, 4096, hipMemcpyDeviceToHost); (void)hipMemcpy(c, d3, 4096, hipMemcpyDeviceToHost);
  printf("pairing (A pos h0,j0 -> B code 16h+j+1):\n");
  for (int pos = 0; pos < 16; ++pos) printf(" A(h%d,j%d)->B code %.0f\n", pos >> 3, pos & 7, p[pos]);
  for (int l : {0, 1, 31, 32, 33, 63}) {
    printf("lane %2d rows:", l); for (int i = 0; i < 16; ++i) printf(" %2.0f", r[l * 16 + i]);
    printf(" | cols:"); for (int i = 0; i < 16; ++i) printf(" %2.0f", c[l * 16 + i]); printf("\n");
  }
}

// Probe of ds_read_b64_tr_b16 semantics: LDS[k] = k (16-bit), lane L supplies byte address 8*L
// (elements 4L..4L+3). Prints the 4 elements each lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short i16x4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int mode) {
  __shared__ __attribute__((aligned(16))) short lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = i;
  __syncthreads();
  int L = threadIdx.x;
  int addr;
  if (mode == 0) addr = 8 * L;                       // identity
  else { int g = L >> 4, i = L & 15, q = i >> 2, p = i & 3;  // my scheme: row q (stride 64 elems), cols 4p
         addr = 2 * (g * 1024 / 4 + q * 64 + 4 * p); }
  i16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)((char*)lds + addr));
  for (int e = 0; e < 4; ++e) out[L * 4 + e] = t[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d\n", mode);
    for (int L = 0; L < 64; ++L) printf("L%02d:[%4d %4d %4d %4d]%s", L, h[4*L], h[4*L+1], h[4*L+2], h[4*L+3], (L % 4 == 3) ? "\n" : " ");
  }
  return 0;
}

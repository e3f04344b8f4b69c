#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
__device__ int soff(int row, int ch) { return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }
__device__ i16x4 lds_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(const_cast<char*>(base) + off));
}
__global__ void k(short* out, int which) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  for (int idx = lane; idx < 32 * 16; idx += 64) {
    int row = idx >> 4, ch = idx & 15;
    short tmp[8];
    for (int e = 0; e < 8; ++e) tmp[e] = which ? (short)(ch * 8 + e) : (short)row;
    *reinterpret_cast<bf16x8*>(smem + soff(row, ch)) = *reinterpret_cast<bf16x8*>(tmp);
  }
  __syncthreads();
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int dt = 0, row0 = 0;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const int row = row0 + 4 * h + q;
  i16x4 lo = lds_tr(smem, soff(row, ch) + 8 * (p & 1));
  i16x4 hi = lds_tr(smem, soff(row + 8, ch) + 8 * (p & 1));
  for (int e = 0; e < 4; ++e) { out[lane * 8 + e] = lo[e]; out[lane * 8 + 4 + e] = hi[e]; }
}
int main() {
  short* d; (void)hipMalloc(&d, 64 * 8 * 2); short rows[512], cols[512];
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 16384, 0, d, 0); (void)hipMemcpy(rows, d, 1024, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 16384, 0, d, 1); (void)hipMemcpy(cols, d, 1024, hipMemcpyDeviceToHost);
  for (int L = 0; L < 64; ++L) {
    printf("L%02d:", L);
    for (int e = 0; e < 8; ++e) printf(" (%d,%d)", rows[L * 8 + e], cols[L * 8 + e]);
    printf("\n");
  }
}

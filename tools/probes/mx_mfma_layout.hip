// Empirical operand/scale layout of gfx950's block-scaled MFMA (v_mfma_scale_f32_{32x32x64,16x16x128}_f8f6f4).
// Runs T independent experiments (one workgroup each): A/B register images (64 lanes x 8 dwords) and
// per-lane E8M0 scale words from mx_in.bin (int32 T, then a[T][64][8], b[T][64][8], sa[T][64],
// sb[T][64]); writes C of both shapes (c32[T][64][16], c16[T][64][4]) to mx_out.bin.
// tools/probes/mx_layout_check.py builds the experiments (one-hot pairing, scale ownership, random
// products) and derives / verifies the maps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int FA, int FB>
__global__ void run(const int* a, const int* b, const int* sa, const int* sb, float* c32, float* c16) {
  const int l = threadIdx.x, t = blockIdx.x;
  a += t * 512; b += t * 512; sa += t * 64; sb += t * 64; c32 += t * 1024; c16 += t * 256;
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) { av[i] = a[l * 8 + i]; bv[i] = b[l * 8 + i]; }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, FA, FB, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 16; ++i) c32[l * 16 + i] = acc[i];
  f32x4 acc4 = {};
  acc4 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc4, FA, FB, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 4; ++i) c16[l * 4 + i] = acc4[i];
}

int main(int argc, char** argv) {
  const int fa = atoi(argv[1]), fb = atoi(argv[2]);
  FILE* f = fopen("mx_in.bin", "rb");
  int T = 0;
  if (!f || fread(&T, 4, 1, f) != 1 || T <= 0 || T > 100000) { printf("bad input\n"); return 1; }
  const size_t n_in = (size_t)T * (1024 + 128);
  std::vector<int> h(n_in);
  if (fread(h.data(), 4, n_in, f) != n_in) { printf("short input\n"); return 1; }
  fclose(f);
  int *da, *db, *dsa, *dsb; float *dc, *dc4;
  (void)hipMalloc(&da, T * 2048); (void)hipMalloc(&db, T * 2048); (void)hipMalloc(&dsa, T * 256);
  (void)hipMalloc(&dsb, T * 256); (void)hipMalloc(&dc, T * 4096); (void)hipMalloc(&dc4, T * 1024);
  (void)hipMemcpy(da, h.data(), T * 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, h.data() + (size_t)T * 512, T * 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsa, h.data() + (size_t)T * 1024, T * 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsb, h.data() + (size_t)T * 1088, T * 256, hipMemcpyHostToDevice);
  bool ran = false;
#define CASE(A, B) if (fa == A && fb == B) { hipLaunchKernelGGL((run<A, B>), dim3(T), dim3(64), 0, 0, da, db, dsa, dsb, dc, dc4); ran = true; }
  CASE(0, 0) CASE(0, 2) CASE(0, 3) CASE(0, 4) CASE(2, 2) CASE(3, 3) CASE(4, 4) CASE(2, 0) CASE(3, 0) CASE(4, 0)
  if (!ran) { printf("unsupported pair\n"); return 1; }
  std::vector<float> o((size_t)T * 1280);
  (void)hipMemcpy(o.data(), dc, T * 4096, hipMemcpyDeviceToHost);
  (void)hipMemcpy(o.data() + (size_t)T * 1024, dc4, T * 1024, hipMemcpyDeviceToHost);
  f = fopen("mx_out.bin", "wb"); fwrite(o.data(), 4, o.size(), f); fclose(f);
  printf("ok %d %d T=%d\n", fa, fb, T);
  return 0;
}

// Host-side optimizers for ZeRO-Offload: Adam/AdamW, Lion, Adagrad on fp32 master partitions in
// (pinned) host memory.
//
// Replaces the reference's missing CPUAdamBuilder / CPULionBuilder / CPUAdagradBuilder ops
// (deepspeed/ops/adam/cpu_adam.py:13 create_adam/adam_update, ops/lion/cpu_lion.py:13,
// ops/adagrad/cpu_adagrad.py:11). Design:
//  * OpenMP over 16 KiB tiles (stays in L1/L2 per core), SIMD inner loops compiled for AVX-512,
//    AVX2 and baseline via GCC target_clones (the binary is built on one host and run on another);
//  * optional fused write of the updated parameter as bf16/fp16 into a pinned staging buffer, so
//    the H2D copy of the new bit16 weights can start immediately (no extra host pass);
//  * grads may arrive as fp32 or bf16 (what the GPU reduce-scatter produced).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <omp.h>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace sxe_cpu {

static inline float bf16_to_f32(uint16_t u) {
  uint32_t x = ((uint32_t)u) << 16;
  float f;
  std::memcpy(&f, &x, 4);
  return f;
}
static inline uint16_t f32_to_bf16(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  if ((x & 0x7f800000u) == 0x7f800000u && (x & 0x007fffffu)) return (uint16_t)((x >> 16) | 0x40);  // quiet NaN
  x += 0x7fffu + ((x >> 16) & 1u);
  return (uint16_t)(x >> 16);
}
static inline uint16_t f32_to_f16(float f) {
  return c10::Half(f).x;
}

enum GKind { G_F32 = 0, G_BF16 = 1 };
enum LKind { L_NONE = 0, L_BF16 = 1, L_F16 = 2 };

struct AdamArgs {
  float lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt, gscale;
  int adamw;
};

// branch-free round-to-nearest-even bf16 (quiet NaN kept): vectorises inside the update loop
static inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t r = (x + 0x7fffu + ((x >> 16) & 1u)) >> 16;
  const uint32_t q = (x >> 16) | 0x40u;
  return (uint16_t)(((x & 0x7fffffffu) > 0x7f800000u) ? q : r);
}

// The bit16 copy of the updated parameter is written in the same SIMD loop as the update (one pass
// over the tile; the separate scalar conversion loop it replaces ran once more over every element).
template <int LK>
__attribute__((target_clones("avx512f", "avx2", "default")))
static void adam_tile(float* __restrict p, const void* __restrict gv, int gk, float* __restrict m,
                      float* __restrict v, void* __restrict lpv, int64_t n, AdamArgs a) {
  float gbuf[4096];
  if (gk == G_F32) {
    const float* g = (const float*)gv;
#pragma omp simd
    for (int64_t i = 0; i < n; ++i) gbuf[i] = g[i] * a.gscale;
  } else {
    const uint16_t* g = (const uint16_t*)gv;
#pragma omp simd
    for (int64_t i = 0; i < n; ++i) gbuf[i] = bf16_to_f32(g[i]) * a.gscale;
  }
  uint16_t* lp = (uint16_t*)lpv;
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    float gi = gbuf[i];
    float pi = p[i];
    if (!a.adamw) gi += a.wd * pi;
    float mi = a.b1 * m[i] + (1.f - a.b1) * gi;
    float vi = a.b2 * v[i] + (1.f - a.b2) * gi * gi;
    float denom = std::sqrt(vi) * a.inv_bc2_sqrt + a.eps;
    if (a.adamw) pi -= a.lr * a.wd * pi;
    pi -= a.step_size * mi / denom;
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if constexpr (LK == L_BF16) lp[i] = f32_to_bf16_rne(pi);
  }
  if constexpr (LK == L_F16) {
    for (int64_t i = 0; i < n; ++i) lp[i] = f32_to_f16(p[i]);
  }
}

static int gkind(const at::Tensor& g) {
  if (g.scalar_type() == at::kFloat) return G_F32;
  TORCH_CHECK(g.scalar_type() == at::kBFloat16, "cpu_adam: grads must be fp32 or bf16");
  return G_BF16;
}
static int lkind(const c10::optional<at::Tensor>& lp) {
  if (!lp.has_value() || !lp->defined()) return L_NONE;
  if (lp->scalar_type() == at::kBFloat16) return L_BF16;
  TORCH_CHECK(lp->scalar_type() == at::kHalf, "cpu_adam: lp must be bf16 or fp16");
  return L_F16;
}

void adam_step_(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, c10::optional<at::Tensor> lp, double lr,
                double beta1, double beta2, double eps, double weight_decay, int64_t step, bool adamw,
                bool bias_correction, double grad_scale) {
  TORCH_CHECK(!p.is_cuda() && p.scalar_type() == at::kFloat && p.is_contiguous(), "cpu_adam: host fp32 contiguous");
  TORCH_CHECK(m.is_contiguous() && v.is_contiguous() && g.is_contiguous(), "cpu_adam: contiguous state");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "cpu_adam: size mismatch");
  const int gk = gkind(g), lk = lkind(lp);
  AdamArgs a;
  a.lr = (float)lr; a.b1 = (float)beta1; a.b2 = (float)beta2; a.eps = (float)eps; a.wd = (float)weight_decay;
  const double bc1 = bias_correction ? 1.0 - std::pow(beta1, (double)step) : 1.0;
  const double bc2 = bias_correction ? 1.0 - std::pow(beta2, (double)step) : 1.0;
  a.step_size = (float)(lr / bc1);
  a.inv_bc2_sqrt = (float)(1.0 / std::sqrt(bc2));
  a.gscale = (float)grad_scale;
  a.adamw = adamw ? 1 : 0;
  float* pp = p.data_ptr<float>();
  float* mp = m.data_ptr<float>();
  float* vp = v.data_ptr<float>();
  const char* gp = (const char*)g.data_ptr();
  char* lpp = lk ? (char*)lp->data_ptr() : nullptr;
  const int64_t gsz = g.element_size();
  const int64_t T = 4096;
  const int64_t tiles = (n + T - 1) / T;
  // dynamic chunks of 16 tiles (256 KB of each array): the asynchronous host tier runs this team
  // beside the training thread, and under a static split one preempted thread stalls the whole
  // update by its share
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t t = 0; t < tiles; ++t) {
    const int64_t o = t * T;
    const int64_t len = std::min(T, n - o);
    char* lo = lpp ? lpp + o * 2 : nullptr;
    if (lk == L_BF16) adam_tile<L_BF16>(pp + o, gp + o * gsz, gk, mp + o, vp + o, lo, len, a);
    else if (lk == L_F16) adam_tile<L_F16>(pp + o, gp + o * gsz, gk, mp + o, vp + o, lo, len, a);
    else adam_tile<L_NONE>(pp + o, gp + o * gsz, gk, mp + o, vp + o, nullptr, len, a);
  }
}

__attribute__((target_clones("avx512f", "avx2", "default")))
static void lion_tile(float* __restrict p, const float* __restrict g, float* __restrict m, int64_t n, float lr,
                      float b1, float b2, float wd) {
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    float c = b1 * m[i] + (1.f - b1) * g[i];
    float u = (c > 0.f) ? 1.f : ((c < 0.f) ? -1.f : 0.f);
    p[i] -= lr * (u + wd * p[i]);
    m[i] = b2 * m[i] + (1.f - b2) * g[i];
  }
}

void lion_step_(at::Tensor p, at::Tensor g, at::Tensor m, double lr, double beta1, double beta2, double wd) {
  TORCH_CHECK(g.scalar_type() == at::kFloat, "cpu_lion: fp32 grads");
  const int64_t n = p.numel(), T = 4096, tiles = (n + T - 1) / T;
  float *pp = p.data_ptr<float>(), *mp = m.data_ptr<float>();
  const float* gp = g.data_ptr<float>();
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < tiles; ++t) {
    const int64_t o = t * T;
    lion_tile(pp + o, gp + o, mp + o, std::min(T, n - o), (float)lr, (float)beta1, (float)beta2, (float)wd);
  }
}

__attribute__((target_clones("avx512f", "avx2", "default")))
static void adagrad_tile(float* __restrict p, const float* __restrict g, float* __restrict s, int64_t n, float lr,
                         float eps, float wd) {
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    float gi = g[i] + wd * p[i];
    float si = s[i] + gi * gi;
    s[i] = si;
    p[i] -= lr * gi / (std::sqrt(si) + eps);
  }
}

void adagrad_step_(at::Tensor p, at::Tensor g, at::Tensor s, double lr, double eps, double wd) {
  TORCH_CHECK(g.scalar_type() == at::kFloat, "cpu_adagrad: fp32 grads");
  const int64_t n = p.numel(), T = 4096, tiles = (n + T - 1) / T;
  float *pp = p.data_ptr<float>(), *sp = s.data_ptr<float>();
  const float* gp = g.data_ptr<float>();
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < tiles; ++t) {
    const int64_t o = t * T;
    adagrad_tile(pp + o, gp + o, sp + o, std::min(T, n - o), (float)lr, (float)eps, (float)wd);
  }
}

// sum of squares (fp32 accumulate in double per tile) for host-side grad norms
double sumsq(at::Tensor x) {
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), "cpu sumsq: fp32 contiguous");
  const float* p = x.data_ptr<float>();
  const int64_t n = x.numel();
  double acc = 0.0;
#pragma omp parallel for reduction(+ : acc) schedule(static)
  for (int64_t i = 0; i < n; ++i) acc += (double)p[i] * p[i];
  return acc;
}

int64_t num_threads() { return omp_get_max_threads(); }

// OpenMP team size of the CALLING thread's later updates (a per-thread setting): the asynchronous
// host-optimizer worker leaves one CPU to the thread that keeps launching GPU work
void set_num_threads(int64_t n) { omp_set_num_threads((int)std::max<int64_t>(1, n)); }

}  // namespace sxe_cpu

TORCH_LIBRARY(sxe_cpu, m) {
  m.def("adam_step_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? lp, float lr, float beta1, "
        "float beta2, float eps, float weight_decay, int step, bool adamw, bool bias_correction, float grad_scale) -> ()");
  m.def("lion_step_(Tensor(a!) p, Tensor g, Tensor(b!) m, float lr, float beta1, float beta2, float wd) -> ()");
  m.def("adagrad_step_(Tensor(a!) p, Tensor g, Tensor(b!) s, float lr, float eps, float wd) -> ()");
  m.def("sumsq(Tensor x) -> float");
  m.def("num_threads() -> int", &sxe_cpu::num_threads);
  m.def("set_num_threads(int n) -> ()", &sxe_cpu::set_num_threads);
}
TORCH_LIBRARY_IMPL(sxe_cpu, CPU, m) {
  m.impl("adam_step_", &sxe_cpu::adam_step_);
  m.impl("lion_step_", &sxe_cpu::lion_step_);
  m.impl("adagrad_step_", &sxe_cpu::adagrad_step_);
  m.impl("sumsq", &sxe_cpu::sumsq);
}

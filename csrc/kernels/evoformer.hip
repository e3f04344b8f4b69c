// Evoformer attention (DS4Sci_EvoformerAttention) on gfx950: O = softmax(Q K^T / sqrt(D) + bias1 +
// bias2) V over Q/K/V [B, N, L, H, D] with bias1 [B, N, 1, 1, L] (MSA row mask) and bias2
// [B, 1, H, L, L] (pair bias), head dims 32 / 64; backward with dQ, dK, dV, dbias1, dbias2.
//
// Reference: ops/deepspeed4science/evoformer_attn.py (CUTLASS kernels of csrc/deepspeed4science,
// not in the snapshot; kMax = 64 there too).
//
// The flash-attention structure of flash_attn.hip, generalised to narrow heads and additive biases:
//  * swapped products (S^T = K Q^T: one lane = one query's scores, lane-local softmax) on
//    v_mfma_f32_32x32x16_bf16, the score accumulator reused as the B operand of O^T += V^T P^T;
//  * K/V (or Q/dO) tiles staged through registers into XOR-swizzled 256-byte LDS rows (a D-wide
//    row uses its first D/8 chunks), row reads + ds_read_b64_tr_b16 transposed reads;
//  * biases are added in the log2 domain inside the online softmax, so no [L, L] matrix is ever
//    materialised; rows past L are zero-staged and masked (any L > 0);
//  * workgroups of the N MSA rows that share one (b, h, query block) are adjacent in the grid, so
//    their pair-bias tile is read from L2 once per row group rather than from HBM per row;
//  * dbias2 = sum over the N rows of dS: fp32 global atomics (vector memory) from the dK/dV
//    kernel; dbias1 = sum over heads and queries: per-lane register sums, one atomic per key.
#include "sxe_common.h"
#include "sxe_mfma.h"
#include <torch/library.h>

namespace sxe {
namespace evo {

using namespace mf;

constexpr int QW = 32, NWV = 4, QB = QW * NWV, KT = 64, QT = 32;

struct Args {
  const unsigned short *q, *k, *v, *dout, *o;
  const float *lse, *delta;   // [BN, H, Lp]
  const float *b1, *b2;       // [BN, L], [B, H, L, L] fp32 or null
  int B, N, L, H, Lp;
  float scale;
};

__device__ __forceinline__ void map_q(const Args& a, int nblk, int& b, int& n, int& h, int& blk) {
  int idx = blockIdx.x;
  n = idx % a.N;
  idx /= a.N;
  blk = idx % nblk;
  idx /= nblk;
  h = idx % a.H;
  b = idx / a.H;
}

// (bias1[key] + bias2[query][key]) * log2(e) for the lane's 16 scores of key-half j
__device__ __forceinline__ float bias_term(const Args& a, int bn, int b, int h, int q, int key) {
  key = key < a.L ? key : a.L - 1;  // callers mask keys past L; the clamp keeps every load in bounds
  q = q < a.L ? q : a.L - 1;
  float t = 0.f;
  if (a.b1) t += a.b1[(int64_t)bn * a.L + key];
  if (a.b2) t += a.b2[(((int64_t)b * a.H + h) * a.L + q) * a.L + key];
  return t * LOG2E;
}

// ------------------------------------------------------------------------------------ forward
template <int DH>
__global__ void __launch_bounds__(256, 2) fwd_kernel(Args a, unsigned short* __restrict__ out, float* __restrict__ lse) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BUF = 2 * KT * ROWB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hf = lane >> 5;
  const int nqb = (a.L + QB - 1) / QB;
  int b, n, h, qb;
  map_q(a, nqb, b, n, h, qb);
  const int bn = b * a.N + n;
  const int64_t rs = (int64_t)a.H * DH;  // row stride of [.., L, H, D]
  const int64_t base = (int64_t)bn * a.L * rs + (int64_t)h * DH;
  const int q = qb * QB + w * QW + r;
  const int qc = q < a.L ? q : a.L - 1;
  const float c = a.scale * LOG2E;

  bf16x8 qf[DH / 16];
#pragma unroll
  for (int t = 0; t < DH / 16; ++t)
    qf[t] = q < a.L ? *reinterpret_cast<const bf16x8*>(a.q + base + (int64_t)q * rs + 16 * t + 8 * hf)
                    : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  f32x16 oacc[DH / 32];
#pragma unroll
  for (int t = 0; t < DH / 32; ++t) oacc[t] = zero16();
  float m = -INFINITY, l = 0.f;

  const int ntiles = (a.L + KT - 1) / KT;
  RowStager<KT, DH, 256> sk, sv;
  sk.load(a.k + base, rs, 0, a.L);
  sv.load(a.v + base, rs, 0, a.L);
  sk.store(smem);
  sv.store(smem + KT * ROWB);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    if (more) {
      sk.load(a.k + base, rs, (t + 1) * KT, a.L);
      sv.load(a.v + base, rs, (t + 1) * KT, a.L);
    }
    const int kbase = t * KT;
    const char* kt = smem + cur * BUF;
    const char* vt = kt + KT * ROWB;
    f32x16 s[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      s[j] = zero16();
#pragma unroll
      for (int t2 = 0; t2 < DH / 16; ++t2) s[j] = mfma(lds_row16(kt, 32 * j + r, 2 * t2 + hf), qf[t2], s[j]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kbase + 32 * j + acc_row(i, hf);
        const float bt = bias_term(a, bn, b, h, qc, key);
        const float x = key < a.L ? __builtin_fmaf(s[j][i], c, bt) : -INFINITY;
        s[j][i] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, xor32(mx));
    const bool grow = mx > m + 8.f;
    const float mnew = grow ? mx : m;
    const float mref = (mnew == -INFINITY) ? 0.f : mnew;
    const float alpha = fast_exp2(m - mref);
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fast_exp2(s[j][i] - mref);
        s[j][i] = p;
        ps += p;
      }
    l = l * alpha + ps;
    m = mnew;
    if (__any(grow)) {
#pragma unroll
      for (int dt = 0; dt < DH / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pb = acc_to_b(s[j], s2);
#pragma unroll
        for (int dt = 0; dt < DH / 32; ++dt) oacc[dt] = mfma(lds_trA(vt, 32 * j + 16 * s2, dt, lane), pb, oacc[dt]);
      }
    if (more) {
      sk.store(smem + (cur ^ 1) * BUF);
      sv.store(smem + (cur ^ 1) * BUF + KT * ROWB);
    }
    __syncthreads();
    cur ^= 1;
  }
  const float lt = l + xor32(l);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (q < a.L) {
    unsigned short* op = out + base + (int64_t)q * rs;
#pragma unroll
    for (int dt = 0; dt < DH / 32; ++dt)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        u16x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = f32_to_bf16(oacc[dt][4 * rg + e] * inv);
        *reinterpret_cast<u16x4*>(op + 32 * dt + 8 * rg + 4 * hf) = pk;
      }
  }
  if (hf == 0 && q < a.Lp)
    lse[((int64_t)bn * a.H + h) * a.Lp + q] = (q < a.L && lt > 0.f) ? (m + log2f(lt)) * LN2 : INFINITY;
}

// ----------------------------------------------------------------------------------------- dQ
template <int DH>
__global__ void __launch_bounds__(256, 2) dq_kernel(Args a, unsigned short* __restrict__ dq) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BUF = 2 * KT * ROWB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hf = lane >> 5;
  const int nqb = (a.L + QB - 1) / QB;
  int b, n, h, qb;
  map_q(a, nqb, b, n, h, qb);
  const int bn = b * a.N + n;
  const int64_t rs = (int64_t)a.H * DH;
  const int64_t base = (int64_t)bn * a.L * rs + (int64_t)h * DH;
  const int q = qb * QB + w * QW + r;
  const int qc = q < a.L ? q : a.L - 1;
  const float c = a.scale * LOG2E;
  const int64_t li = ((int64_t)bn * a.H + h) * a.Lp + q;
  const float lse2 = a.lse[li] * LOG2E, dlt = a.delta[li];
  bf16x8 qf[DH / 16], df[DH / 16];
#pragma unroll
  for (int t = 0; t < DH / 16; ++t) {
    const bool ok = q < a.L;
    qf[t] = ok ? *reinterpret_cast<const bf16x8*>(a.q + base + (int64_t)q * rs + 16 * t + 8 * hf)
               : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    df[t] = ok ? *reinterpret_cast<const bf16x8*>(a.dout + base + (int64_t)q * rs + 16 * t + 8 * hf)
               : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x16 acc[DH / 32];
#pragma unroll
  for (int t = 0; t < DH / 32; ++t) acc[t] = zero16();
  const int ntiles = (a.L + KT - 1) / KT;
  RowStager<KT, DH, 256> sk, sv;
  sk.load(a.k + base, rs, 0, a.L);
  sv.load(a.v + base, rs, 0, a.L);
  sk.store(smem);
  sv.store(smem + KT * ROWB);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    if (more) {
      sk.load(a.k + base, rs, (t + 1) * KT, a.L);
      sv.load(a.v + base, rs, (t + 1) * KT, a.L);
    }
    const int kbase = t * KT;
    const char* kt = smem + cur * BUF;
    const char* vt = kt + KT * ROWB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int t2 = 0; t2 < DH / 16; ++t2) {
        s = mfma(lds_row16(kt, 32 * j + r, 2 * t2 + hf), qf[t2], s);
        dp = mfma(lds_row16(vt, 32 * j + r, 2 * t2 + hf), df[t2], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kbase + 32 * j + acc_row(i, hf);
        const float bt = bias_term(a, bn, b, h, qc, key);
        const float p = key < a.L ? fast_exp2(__builtin_fmaf(s[i], c, bt) - lse2) : 0.f;
        s[i] = p * (dp[i] - dlt);  // dS^T
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 db = acc_to_b(s, s2);
#pragma unroll
        for (int dt = 0; dt < DH / 32; ++dt) acc[dt] = mfma(lds_trA(kt, 32 * j + 16 * s2, dt, lane), db, acc[dt]);
      }
    }
    if (more) {
      sk.store(smem + (cur ^ 1) * BUF);
      sv.store(smem + (cur ^ 1) * BUF + KT * ROWB);
    }
    __syncthreads();
    cur ^= 1;
  }
  if (q < a.L) {
    unsigned short* op = dq + base + (int64_t)q * rs;
#pragma unroll
    for (int dt = 0; dt < DH / 32; ++dt)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        u16x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = f32_to_bf16(acc[dt][4 * rg + e] * a.scale);
        *reinterpret_cast<u16x4*>(op + 32 * dt + 8 * rg + 4 * hf) = pk;
      }
  }
}

// -------------------------------------------------------------------------------------- dK, dV
// Keys on the lanes (32 per wave, 128 per workgroup); sweep every 32-query tile; Q / dO tiles and
// their lse / delta staged through registers into a 2-slot LDS ring.
constexpr int SLOT = 2 * QT * ROWB + 2 * QT * 4;

template <int DH>
__global__ void __launch_bounds__(256, 2) dkdv_kernel(Args a, unsigned short* __restrict__ dk,
                                                      unsigned short* __restrict__ dv, float* __restrict__ db1,
                                                      float* __restrict__ db2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hf = lane >> 5;
  const int nkb = (a.L + QB - 1) / QB;
  int b, n, h, kb;
  map_q(a, nkb, b, n, h, kb);
  const int bn = b * a.N + n;
  const int64_t rs = (int64_t)a.H * DH;
  const int64_t base = (int64_t)bn * a.L * rs + (int64_t)h * DH;
  const int key = kb * QB + w * QW + r;
  const bool kok = key < a.L;
  const float c = a.scale * LOG2E;
  bf16x8 kf[DH / 16], vf[DH / 16];
#pragma unroll
  for (int t = 0; t < DH / 16; ++t) {
    kf[t] = kok ? *reinterpret_cast<const bf16x8*>(a.k + base + (int64_t)key * rs + 16 * t + 8 * hf)
                : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    vf[t] = kok ? *reinterpret_cast<const bf16x8*>(a.v + base + (int64_t)key * rs + 16 * t + 8 * hf)
                : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x16 dka[DH / 32], dva[DH / 32];
#pragma unroll
  for (int t = 0; t < DH / 32; ++t) {
    dka[t] = zero16();
    dva[t] = zero16();
  }
  float b1acc = 0.f;
  const int ntq = (a.L + QT - 1) / QT;
  const int64_t lrow = ((int64_t)bn * a.H + h) * a.Lp;
  RowStager<QT, DH, 256> sq, sd;
  float lreg = 0.f;
  auto load = [&](int it) {
    sq.load(a.q + base, rs, it * QT, a.L);
    sd.load(a.dout + base, rs, it * QT, a.L);
    if (threadIdx.x < 2 * QT) {
      const int qq = it * QT + (threadIdx.x & (QT - 1));
      lreg = threadIdx.x < QT ? a.lse[lrow + qq] : a.delta[lrow + qq];
    }
  };
  auto store = [&](char* slot) {
    sq.store(slot);
    sd.store(slot + QT * ROWB);
    if (threadIdx.x < 2 * QT) reinterpret_cast<float*>(slot + 2 * QT * ROWB)[threadIdx.x] = lreg;
  };
  load(0);
  store(smem);
  __syncthreads();
  int cur = 0;
  for (int it = 0; it < ntq; ++it) {
    const bool more = it + 1 < ntq;
    if (more) load(it + 1);
    const char* slot = smem + cur * SLOT;
    const char* qt = slot;
    const char* dt_ = slot + QT * ROWB;
    const float* l2 = reinterpret_cast<const float*>(slot + 2 * QT * ROWB);
    const float* dl = l2 + QT;
    const int qt0 = it * QT;
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int t2 = 0; t2 < DH / 16; ++t2) {
      s = mfma(lds_row16(qt, r, 2 * t2 + hf), kf[t2], s);    // S  [query][key]
      dp = mfma(lds_row16(dt_, r, 2 * t2 + hf), vf[t2], dp);  // dP [query][key]
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = acc_row(i, hf), qq = qt0 + qi;
      const bool ok = kok && qq < a.L;
      const float bt = bias_term(a, bn, b, h, qq, key);
      const float p = ok ? fast_exp2(__builtin_fmaf(s[i], c, bt) - l2[qi] * LOG2E) : 0.f;
      const float ds = p * (dp[i] - dl[qi]);
      if (db2 != nullptr && ok) atomicAdd(db2 + (((int64_t)b * a.H + h) * a.L + qq) * a.L + key, ds);
      b1acc += ds;
      s[i] = p;
      dp[i] = ds;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = acc_to_b(s, s2);
      const bf16x8 db = acc_to_b(dp, s2);
#pragma unroll
      for (int t = 0; t < DH / 32; ++t) {
        dva[t] = mfma(lds_trA(dt_, 16 * s2, t, lane), pb, dva[t]);  // dV^T += dO^T P
        dka[t] = mfma(lds_trA(qt, 16 * s2, t, lane), db, dka[t]);   // dK^T += Q^T dS
      }
    }
    if (more) store(smem + (cur ^ 1) * SLOT);
    __syncthreads();
    cur ^= 1;
  }
  const float b1tot = b1acc + xor32(b1acc);
  if (db1 != nullptr && kok && hf == 0) atomicAdd(db1 + (int64_t)bn * a.L + key, b1tot);
  if (kok) {
    unsigned short* kop = dk + base + (int64_t)key * rs;
    unsigned short* vop = dv + base + (int64_t)key * rs;
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        u16x4 pk, pv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pk[e] = f32_to_bf16(dka[t][4 * rg + e] * a.scale);
          pv[e] = f32_to_bf16(dva[t][4 * rg + e]);
        }
        *reinterpret_cast<u16x4*>(kop + 32 * t + 8 * rg + 4 * hf) = pk;
        *reinterpret_cast<u16x4*>(vop + 32 * t + 8 * rg + 4 * hf) = pv;
      }
  }
}

}  // namespace evo

// ------------------------------------------------------------------------------- host side
static evo::Args evo_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                          const c10::optional<at::Tensor>& b1, const c10::optional<at::Tensor>& b2) {
  SXE_CHECK(q.dim() == 5 && q.sizes() == k.sizes() && q.sizes() == v.sizes(), "evoformer: q/k/v [B, N, L, H, D]");
  for (const at::Tensor* t : {&q, &k, &v})
    SXE_CHECK(t->is_contiguous() && t->scalar_type() == at::kBFloat16, "evoformer: contiguous bf16 q/k/v");
  const int D = q.size(4);
  SXE_CHECK(D == 32 || D == 64, "evoformer: head dim 32 or 64");
  evo::Args a{};
  a.B = q.size(0);
  a.N = q.size(1);
  a.L = q.size(2);
  a.H = q.size(3);
  a.Lp = (a.L + evo::QB - 1) / evo::QB * evo::QB;
  a.scale = 1.f / std::sqrt((float)D);
  a.q = reinterpret_cast<const unsigned short*>(q.data_ptr());
  a.k = reinterpret_cast<const unsigned short*>(k.data_ptr());
  a.v = reinterpret_cast<const unsigned short*>(v.data_ptr());
  if (b1.has_value() && b1->defined()) {
    SXE_CHECK(b1->scalar_type() == at::kFloat && b1->is_contiguous() && b1->numel() == (int64_t)a.B * a.N * a.L,
              "evoformer: bias1 fp32 [B, N, 1, 1, L]");
    a.b1 = b1->data_ptr<float>();
  }
  if (b2.has_value() && b2->defined()) {
    SXE_CHECK(b2->scalar_type() == at::kFloat && b2->is_contiguous() &&
                  b2->numel() == (int64_t)a.B * a.H * a.L * a.L, "evoformer: bias2 fp32 [B, 1, H, L, L]");
    a.b2 = b2->data_ptr<float>();
  }
  return a;
}

std::vector<at::Tensor> evoformer_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                      const c10::optional<at::Tensor>& b1, const c10::optional<at::Tensor>& b2) {
  SXE_CHECK_CUDA(q);
  evo::Args a = evo_args(q, k, v, b1, b2);
  c10::DeviceGuard g(q.device());
  auto o = at::empty_like(q);
  auto lse = at::empty({(int64_t)a.B * a.N, a.H, a.Lp}, q.options().dtype(at::kFloat));
  const int grid = a.B * a.N * a.H * (a.Lp / evo::QB);
  const size_t lds = 4 * evo::KT * mf::ROWB;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {reinterpret_cast<const void*>(&evo::fwd_kernel<32>), reinterpret_cast<const void*>(&evo::fwd_kernel<64>),
                          reinterpret_cast<const void*>(&evo::dq_kernel<32>), reinterpret_cast<const void*>(&evo::dq_kernel<64>)})
      SXE_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  auto* op = reinterpret_cast<unsigned short*>(o.data_ptr());
  if (q.size(4) == 32)
    hipLaunchKernelGGL(evo::fwd_kernel<32>, dim3(grid), dim3(256), lds, cur_stream(), a, op, lse.data_ptr<float>());
  else
    hipLaunchKernelGGL(evo::fwd_kernel<64>, dim3(grid), dim3(256), lds, cur_stream(), a, op, lse.data_ptr<float>());
  SXE_LAUNCH_CHECK();
  return {o, lse};
}

// delta [BN, H, Lp] = rowsum(dO * O) (padded rows 0) is computed by the caller.
std::vector<at::Tensor> evoformer_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                                      const at::Tensor& v, const at::Tensor& lse, const at::Tensor& delta,
                                      const c10::optional<at::Tensor>& b1, const c10::optional<at::Tensor>& b2,
                                      bool need_db1, bool need_db2) {
  SXE_CHECK_CUDA(q);
  evo::Args a = evo_args(q, k, v, b1, b2);
  SXE_CHECK(dout.sizes() == q.sizes() && dout.is_contiguous() && dout.scalar_type() == at::kBFloat16,
            "evoformer_bwd: dout like q");
  SXE_CHECK(lse.numel() == (int64_t)a.B * a.N * a.H * a.Lp && delta.numel() == lse.numel() &&
                lse.scalar_type() == at::kFloat && delta.scalar_type() == at::kFloat && lse.is_contiguous() &&
                delta.is_contiguous(), "evoformer_bwd: lse / delta fp32 [B*N, H, Lp]");
  c10::DeviceGuard g(q.device());
  a.dout = reinterpret_cast<const unsigned short*>(dout.data_ptr());
  a.lse = lse.data_ptr<float>();
  a.delta = delta.data_ptr<float>();
  auto dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  at::Tensor db1, db2;
  if (need_db1) db1 = at::zeros({a.B, a.N, 1, 1, a.L}, q.options().dtype(at::kFloat));
  if (need_db2) db2 = at::zeros({a.B, 1, a.H, a.L, a.L}, q.options().dtype(at::kFloat));
  const int grid = a.B * a.N * a.H * (a.Lp / evo::QB);
  const size_t lds_q = 4 * evo::KT * mf::ROWB, lds_kv = 2 * evo::SLOT;
  auto* dqp = reinterpret_cast<unsigned short*>(dq.data_ptr());
  auto* dkp = reinterpret_cast<unsigned short*>(dk.data_ptr());
  auto* dvp = reinterpret_cast<unsigned short*>(dv.data_ptr());
  float* b1p = need_db1 ? db1.data_ptr<float>() : nullptr;
  float* b2p = need_db2 ? db2.data_ptr<float>() : nullptr;
  if (q.size(4) == 32) {
    hipLaunchKernelGGL(evo::dq_kernel<32>, dim3(grid), dim3(256), lds_q, cur_stream(), a, dqp);
    hipLaunchKernelGGL(evo::dkdv_kernel<32>, dim3(grid), dim3(256), lds_kv, cur_stream(), a, dkp, dvp, b1p, b2p);
  } else {
    hipLaunchKernelGGL(evo::dq_kernel<64>, dim3(grid), dim3(256), lds_q, cur_stream(), a, dqp);
    hipLaunchKernelGGL(evo::dkdv_kernel<64>, dim3(grid), dim3(256), lds_kv, cur_stream(), a, dkp, dvp, b1p, b2p);
  }
  SXE_LAUNCH_CHECK();
  return {dq, dk, dv, need_db1 ? db1 : at::Tensor(), need_db2 ? db2 : at::Tensor()};
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("evoformer_fwd(Tensor q, Tensor k, Tensor v, Tensor? bias1, Tensor? bias2) -> Tensor[]");
  m.def("evoformer_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor lse, Tensor delta, Tensor? bias1, "
        "Tensor? bias2, bool need_db1, bool need_db2) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("evoformer_fwd", &sxe::evoformer_fwd);
  m.impl("evoformer_bwd", &sxe::evoformer_bwd);
}

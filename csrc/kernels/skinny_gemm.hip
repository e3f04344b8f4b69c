// Skinny GEMM for decode: y[M, N] = x[M, K] . W[N, K]^T (+ bias), M <= 16, bf16, fp32 accumulate.
//
// Decode GEMMs stream the weight once and touch almost no activation bytes, so the job is HBM
// streaming at the highest rate the chip sustains -- hipBLASLt's general kernels reach 3.5-4.7 TB/s
// on Llama-3-8B decode shapes (profiles/decode_*). MI355X-first design:
//  * MFMA does the math (v_mfma_f32_16x16x32_bf16, x padded to 16 rows): the VALU stays free and
//    the lane maps are the hardware's -- lane l holds W[n = l & 15][8 K values] as the B fragment
//    and x[m = l & 15][the same 8 K values] as the A fragment;
//  * MFMA step s of a 256-wide super-step takes K = k0 + 32 s + [0, 32): lane group g = l >> 4 reads
//    the 16 bytes at k0 + 32 s + 8 g, so each load instruction reads 64 contiguous bytes of each of
//    16 rows and two consecutive steps complete the 128-byte lines (a lane-owns-128-bytes map was
//    2x slower: 64 distinct lines per instruction);
//  * one workgroup per 16 output columns, K split over its NW = 4/8 waves (NW = 8 for narrow N,
//    so more waves per CU stream at once; 16 waves would cap VGPRs at 128 and spill), two super-steps of loads in flight per wave, partial
//    tiles summed through NW KB of LDS.
//  * fused prologues (decode, M <= 4): PRO_RMS builds the GEMM input (residual add + RMSNorm) and
//    PRO_SWIGLU (silu(gate) * up) in LDS inside the GEMM launch -- every workgroup recomputes the
//    few KB of activations it needs (L2 hits) while its first weight super-step is already in
//    flight, so the norm / gated-activation launches (4-5 us each at batch 1, latency-bound) are
//    gone from the decode layer. Workgroup 0 also writes the new residual stream h = x + res.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace sg {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kSS = 256;  // K per super-step per wave

struct Frag {
  bf16x8 w[8];
  bf16x8 x[8];
};

// nt: non-temporal weight loads (`global_load ... nt`) -- a decode GEMM reads each weight byte once,
// so it need not displace the activations / KV cache from L2 and the Infinity Cache (the MI355X
// guide measures issued -> landed -18 % for a once-read cold weight stream)
// (a kernel template parameter: with a runtime flag the compiler merges the two loads of one address
// and drops the non-temporal hint)
template <bool NT = false>
__device__ __forceinline__ void load_w(Frag& f, const unsigned short* __restrict wrow, bool wok, int kbase, int K) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = kbase + s * 32;
    const bf16x8* p = reinterpret_cast<const bf16x8*>(wrow + k);
    if (wok && k < K) f.w[s] = NT ? __builtin_nontemporal_load(p) : *p;
    else f.w[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}
__device__ __forceinline__ void load_x(Frag& f, const unsigned short* __restrict xrow, bool xok, int kbase, int K) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = kbase + s * 32;
    f.x[s] = (xok && k < K) ? *reinterpret_cast<const bf16x8*>(xrow + k) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

enum : int { PRO_NONE = 0, PRO_RMS = 1, PRO_SWIGLU = 2, PRO_MERGE = 3 };
constexpr int kProMaxM = 4;

struct ProArgs {
  const unsigned short* res;  // RMS: residual added to x (nullptr: none), same row stride as x
  const unsigned short* gw;   // RMS: norm weight [K]
  unsigned short* hout;       // RMS: h = x + res [M, K] (written by workgroup 0; nullptr: not wanted)
  float eps;
  const float* po;            // MERGE: split-KV attention partials [splits, M, nq, D] (unnormalised)
  const float* pml;           // MERGE: their (max, sum) [splits, M, nq, 2], log2 domain
  int splits, nq;
  // RMS + RoPE epilogue (rcos != nullptr; the decode QKV projection, head dim 128): the output's q
  // and k heads are rotated (rotate-half, fp32 cos/sin [max_pos, 64] at rpos[m]) and the rotated k
  // plus v rows are written to the paged cache [blocks, 2, nkv, bs, 128] at rslots[m] -- the
  // RoPE + KV-append launch is gone from the decode layer. Each 16-column tile of a q / k head
  // holds 8 rotation pairs (columns 8 j + c and 64 + 8 j + c), partners 8 lanes apart.
  const float* rcos;
  const float* rsin;
  const int64_t* rpos;
  const int64_t* rslots;
  unsigned short* rcache;
  int rnq, rnkv, rbs;
  int nt;  // non-temporal weight loads (SXE_SKINNY_NT)
};

// output column of lane `col` in tile `tile` (identity unless the RoPE epilogue pairs columns)
__device__ __forceinline__ int out_col(const ProArgs& p, int tile, int col) {
  const int h = tile >> 3, j = tile & 7;
  if (p.rcos == nullptr || h >= p.rnq + p.rnkv) return tile * 16 + col;
  return h * 128 + (col < 8 ? 8 * j + col : 56 + 8 * j + col);
}

// Wave-0 epilogue store of output (m, n) = v under the RoPE epilogue; every lane calls it (the pair
// exchange is a whole-wave shuffle).
__device__ __forceinline__ void rope_store(const ProArgs& p, float v, int m, int M, int n, int tile, int col,
                                           unsigned short* __restrict y, int64_t ldy) {
  const int h = tile >> 3;
  const float pv = __shfl_xor(v, 8, 64);
  if (m >= M) return;
  const int d = n - h * 128;
  float out = v;
  if (h < p.rnq + p.rnkv) {
    const int64_t ps = p.rpos[m];
    const float c = p.rcos[ps * 64 + (d & 63)], sn = p.rsin[ps * 64 + (d & 63)];
    out = col < 8 ? v * c - pv * sn : v * c + pv * sn;
  }
  const unsigned short ob = f32_to_bf16(out);
  y[(int64_t)m * ldy + n] = ob;
  if (h >= p.rnq) {
    const int64_t slot = p.rslots[m];
    if (slot >= 0) {
      const int kv = h >= p.rnq + p.rnkv ? 1 : 0, hh = h - p.rnq - kv * p.rnkv;
      const int64_t blk = slot / p.rbs, off = slot - blk * p.rbs;
      p.rcache[(((blk * 2 + kv) * p.rnkv + hh) * p.rbs + off) * 128 + d] = ob;
    }
  }
}

// The M x K GEMM input, built in LDS (bf16, row stride K) by the whole workgroup in ONE pass:
//   PRO_RMS    act = bf16(h * g), h = bf16(x + res) (the unfused norm's rounding); the row's
//              rsqrt(mean(h^2) + eps) goes to rinv[] and scales the GEMM output in the epilogue
//   PRO_SWIGLU act = bf16(silu(x[:, :K]) * x[:, K:])
// PRO_MERGE: act[m][h D + d] = the flash-decoding merge of the KV splits' partials (paged_attn.hip
// merge_kernel's math): sum_s 2^(M_s - M) o_s / sum_s 2^(M_s - M) L_s. One thread per 8 d of one
// (row, head); every load of a group of 8 splits is issued before the first use.
template <int NT>
__device__ __forceinline__ void build_merge(int M, int K, int klo, int khi, const ProArgs& p, unsigned short* act) {
  constexpr int U = 8;
  const int D = K / p.nq, per = (khi - klo) / 8, n = M * per;
  for (int idx = threadIdx.x; idx < n; idx += NT) {
    const int m = idx / per, c = klo + (idx - m * per) * 8, h = c / D, d = c - h * D;
    const int64_t th = (int64_t)m * p.nq + h, sstride = (int64_t)M * p.nq;
    float Mx = -INFINITY, L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < p.splits; s0 += U) {
      float ms[U], ls[U];
      f32x4 o0[U], o1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i2 = (int64_t)min(s0 + u, p.splits - 1) * sstride + th;
        ms[u] = p.pml[i2 * 2];
        ls[u] = p.pml[i2 * 2 + 1];
        o0[u] = *reinterpret_cast<const f32x4*>(p.po + i2 * D + d);
        o1[u] = *reinterpret_cast<const f32x4*>(p.po + i2 * D + d + 4);
      }
      float Mc = Mx;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (s0 + u < p.splits) Mc = fmaxf(Mc, ms[u]);
      const float r = Mx == -INFINITY ? 0.f : exp2f(Mx - Mc);
      L *= r;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= r;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (s0 + u < p.splits && ms[u] != -INFINITY) {
          const float f = exp2f(ms[u] - Mc);
          L += f * ls[u];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] += f * o0[u][j];
            acc[4 + j] += f * o1[u][j];
          }
        }
      }
      Mx = Mc;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = L > 0.f ? acc[j] / L : 0.f;
    store8<DT::BF16>(act + (int64_t)m * K + c, acc);
  }
  __syncthreads();
}

// Only columns [klo, khi) of the input are built (a split-K part needs no more), except under
// PRO_RMS, whose row norm needs the whole row.
template <int MODE, int NT>
__device__ __forceinline__ void build_act(const unsigned short* __restrict x, int64_t ldx, int M, int K, int klo,
                                          int khi, const ProArgs& p, unsigned short* act, float* rinv) {
  if constexpr (MODE == PRO_MERGE) {
    build_merge<NT>(M, K, klo, khi, p, act);
    return;
  }
  if constexpr (MODE == PRO_RMS) {
    klo = 0;
    khi = K;
  }
  // U chunks of 8 per thread per round, every load of a round issued before the first use: a loop
  // that consumes each chunk before loading the next is a chain of dependent L2 round trips (it made
  // the fused down projection 9 us slower than the separate SwiGLU launch)
  constexpr int U = 4;
  __shared__ float red[NT / 64][kProMaxM];
  const int per = (khi - klo) / 8, n = M * per;
  float ss[kProMaxM] = {0.f, 0.f, 0.f, 0.f};
  for (int base = 0; base < n; base += U * NT) {
    u16x8 a[U], b[U], gw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * NT + threadIdx.x;
      const int m = idx / per, c = klo + (idx - m * per) * 8;
      const bool ok = idx < n;
      const unsigned short* xr = x + (int64_t)(ok ? m : 0) * ldx + (ok ? c : 0);
      a[u] = *reinterpret_cast<const u16x8*>(xr);
      if constexpr (MODE == PRO_SWIGLU) {
        b[u] = *reinterpret_cast<const u16x8*>(xr + K);
      } else {
        gw[u] = *reinterpret_cast<const u16x8*>(p.gw + (ok ? c : 0));
        if (p.res != nullptr) b[u] = *reinterpret_cast<const u16x8*>(p.res + (int64_t)(ok ? m : 0) * ldx + (ok ? c : 0));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * NT + threadIdx.x;
      if (idx >= n) continue;
      const int m = idx / per, c = klo + (idx - m * per) * 8;
      float o[8];
      if constexpr (MODE == PRO_SWIGLU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gv = bf16_to_f32(a[u][j]);
          o[j] = gv / (1.f + __expf(-gv)) * bf16_to_f32(b[u][j]);
        }
      } else {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(a[u][j]);
        if (p.res != nullptr) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(f32_to_bf16(v[j] + bf16_to_f32(b[u][j])));
          if (p.hout != nullptr && blockIdx.x == 0) store8<DT::BF16>(p.hout + (int64_t)m * K + c, v);
        }
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          q += v[j] * v[j];
          o[j] = v[j] * bf16_to_f32(gw[u][j]);
        }
#pragma unroll
        for (int mm = 0; mm < kProMaxM; ++mm)
          if (mm == m) ss[mm] += q;
      }
      store8<DT::BF16>(act + (int64_t)m * K + c, o);
    }
  }
  if constexpr (MODE == PRO_RMS) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int mm = 0; mm < kProMaxM; ++mm) {
      const float t = wave_sum(ss[mm]);
      if (lane == 0) red[wave][mm] = t;
    }
    __syncthreads();
    if (threadIdx.x < kProMaxM) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) t += red[w][threadIdx.x];
      rinv[threadIdx.x] = rsqrtf(t / (float)K + p.eps);
    }
  }
  __syncthreads();
}

template <int NW, int MODE = PRO_NONE, bool NT = false>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(const unsigned short* __restrict x, int64_t ldx,
                                                          const unsigned short* __restrict w, int64_t ldw,
                                                          const unsigned short* __restrict bias,
                                                          unsigned short* __restrict y, int64_t ldy, int M, int N,
                                                          int K, int ss_per_wave, ProArgs pro) {
  __shared__ f32x4 red[NW][64];
  extern __shared__ __attribute__((aligned(16))) unsigned short act_lds[];  // PRO_*: the M x K input
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x;
  const int n = MODE == PRO_RMS ? out_col(pro, tile, col) : tile * 16 + col;
  const bool wok = n < N, xok = col < M;
  const unsigned short* wrow = w + (int64_t)(wok ? n : 0) * ldw;
  const unsigned short* xrow = MODE == PRO_NONE ? x + (int64_t)(xok ? col : 0) * ldx
                                                : act_lds + (int64_t)(xok ? col : 0) * K;
  const int ss0 = wave * ss_per_wave;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  __shared__ float rinv[kProMaxM];
  Frag cur, nxt;
  if constexpr (MODE == PRO_NONE) {
    load_w<NT>(cur, wrow, wok, ss0 * kSS + g * 8, K);
    load_x(cur, xrow, xok, ss0 * kSS + g * 8, K);
    for (int i = 0; i < ss_per_wave; ++i) {
      if (i + 1 < ss_per_wave) {
        load_w<NT>(nxt, wrow, wok, (ss0 + i + 1) * kSS + g * 8, K);
        load_x(nxt, xrow, xok, (ss0 + i + 1) * kSS + g * 8, K);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.x[s], cur.w[s], acc, 0, 0, 0);
      cur = nxt;
    }
  } else {
    // the weight stream runs two super-steps ahead of the prologue, which builds the input in LDS
    Frag nx2;
    load_w<NT>(cur, wrow, wok, ss0 * kSS + g * 8, K);
    if (ss_per_wave > 1) load_w<NT>(nxt, wrow, wok, (ss0 + 1) * kSS + g * 8, K);
    build_act<MODE, NW * 64>(x, ldx, M, K, 0, K, pro, act_lds, rinv);
    for (int i = 0; i < ss_per_wave; ++i) {
      if (i + 2 < ss_per_wave) load_w<NT>(nx2, wrow, wok, (ss0 + i + 2) * kSS + g * 8, K);
      load_x(cur, xrow, xok, (ss0 + i) * kSS + g * 8, K);
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.x[s], cur.w[s], acc, 0, 0, 0);
      cur = nxt;
      nxt = nx2;
    }
  }
  // acc: C[row m = 4 g + r][col n] -- sum the 4 waves' K partials
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int v = 1; v < NW; ++v) {
      const f32x4 u = red[v][lane];
      t[0] += u[0];
      t[1] += u[1];
      t[2] += u[2];
      t[3] += u[3];
    }
    if (MODE == PRO_RMS && pro.rcos != nullptr) {  // RoPE epilogue (no bias: checked on the host)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        rope_store(pro, t[r] * rinv[m < kProMaxM ? m : 0], m, M, n, tile, col, y, ldy);
      }
    } else if (n < N) {
      const float b = bias ? bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        const float sc = MODE == PRO_RMS ? rinv[m < kProMaxM ? m : 0] : 1.f;
        if (m < M) y[(int64_t)m * ldy + n] = f32_to_bf16(t[r] * sc + b);
      }
    }
  }
}

// Waves per workgroup: NW = 8 (more waves streaming per CU) while the tiles still fit on the chip
// in ONE round -- at ~150 VGPRs (bf16) one 8-wave workgroup fits per CU, at ~115 (fp8) two -- and
// every wave keeps >= `min_ss` super-steps; otherwise NW = 4 (three / four workgroups per CU), so
// e.g. the 384-tile QKV projection does not run a second, half-empty round of 8-wave workgroups.
// SXE_SKINNY_NT (read per call; a captured decode graph keeps the value of its capture)
inline int nt_loads() {
  const char* e = std::getenv("SXE_SKINNY_NT");
  return (e != nullptr && *e != 0 && *e != '0') ? 1 : 0;
}

inline int pick_nw(int tiles, int ss_total, int min_ss, int wg8_per_cu) {
  int nw = 4;
  while (nw < 8 && (int64_t)tiles * nw < 4096 && ss_total >= min_ss * nw) nw *= 2;
  if (nw == 8 && tiles > kNumCUs * wg8_per_cu) nw = 4;
  return nw;
}

// ---- FP8-weight variant (W8A16: e4m3 weights, per-output-row fp32 scale, bf16 activations) ----
// Same structure; each lane streams 16 bytes = 16 weights per load and converts them to bf16 in
// registers (v_cvt_f32_fp8; e4m3 values are exact in bf16), so the weight bytes -- the whole
// cost of a decode GEMM -- are halved. MFMA step (j, h) of a 512-wide super-step uses
// K = k0 + 64 j + 16 g + 8 h + [0, 8) for lane group g, for weights and activations alike.
constexpr int kSS8 = 512;

__device__ __forceinline__ bf16x8 fp8x8_to_bf16(uint2 w) {
  // byte-selected v_cvt_f32_fp8 (byte b of the word -> element b): explicit order, e4m3 is exact
  // in bf16 so the top half of the f32 bit pattern is the bf16 value
  bf16x8 r;
#define SXE_FP8_BYTE(word, b) (short)(__builtin_bit_cast(unsigned int, __builtin_amdgcn_cvt_f32_fp8((int)(word), b)) >> 16)
  r[0] = SXE_FP8_BYTE(w.x, 0);
  r[1] = SXE_FP8_BYTE(w.x, 1);
  r[2] = SXE_FP8_BYTE(w.x, 2);
  r[3] = SXE_FP8_BYTE(w.x, 3);
  r[4] = SXE_FP8_BYTE(w.y, 0);
  r[5] = SXE_FP8_BYTE(w.y, 1);
  r[6] = SXE_FP8_BYTE(w.y, 2);
  r[7] = SXE_FP8_BYTE(w.y, 3);
#undef SXE_FP8_BYTE
  return r;
}

template <int NW, int MODE = PRO_NONE>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_fp8w_kernel(const unsigned short* __restrict x, int64_t ldx,
                                                                   const uint8_t* __restrict w, int64_t ldw,
                                                                   const float* __restrict wscale,
                                                                   const unsigned short* __restrict bias,
                                                                   unsigned short* __restrict y, int64_t ldy, int M,
                                                                   int N, int K, int ss_per_wave, ProArgs pro) {
  __shared__ f32x4 red[NW][64];
  extern __shared__ __attribute__((aligned(16))) unsigned short act_lds[];  // PRO_*: the M x K input
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int n = MODE == PRO_RMS ? out_col(pro, blockIdx.x, col) : blockIdx.x * 16 + col;
  const bool wok = n < N, xok = col < M;
  const uint8_t* wrow = w + (int64_t)(wok ? n : 0) * ldw;
  const unsigned short* xrow = MODE == PRO_NONE ? x + (int64_t)(xok ? col : 0) * ldx
                                                : act_lds + (int64_t)(xok ? col : 0) * K;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  __shared__ float rinv[kProMaxM];
  uint4 wv0[8];  // first super-step's weights: in flight while the prologue builds the input
  if constexpr (MODE != PRO_NONE) {
    const int k0 = (wave * ss_per_wave) * kSS8 + 16 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + 64 * j;
      wv0[j] = (wok && k < K && ss_per_wave > 0) ? *reinterpret_cast<const uint4*>(wrow + k) : uint4{0u, 0u, 0u, 0u};
    }
    build_act<MODE, NW * 64>(x, ldx, M, K, 0, K, pro, act_lds, rinv);
  }
  for (int i = 0; i < ss_per_wave; ++i) {
    const int k0 = (wave * ss_per_wave + i) * kSS8 + 16 * g;
    uint4 wv[8];
    bf16x8 xa[8], xb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + 64 * j;
      const bool in = k < K;
      if (MODE != PRO_NONE && i == 0) wv[j] = wv0[j];
      else wv[j] = (wok && in) ? *reinterpret_cast<const uint4*>(wrow + k) : uint4{0u, 0u, 0u, 0u};
      xa[j] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      xb[j] = (xok && in) ? *reinterpret_cast<const bf16x8*>(xrow + k + 8) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[j], fp8x8_to_bf16(uint2{wv[j].x, wv[j].y}), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb[j], fp8x8_to_bf16(uint2{wv[j].z, wv[j].w}), acc, 0, 0, 0);
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int v = 1; v < NW; ++v) {
      const f32x4 u = red[v][lane];
      t[0] += u[0];
      t[1] += u[1];
      t[2] += u[2];
      t[3] += u[3];
    }
    if (MODE == PRO_RMS && pro.rcos != nullptr) {  // RoPE epilogue (no bias: checked on the host)
      const float sc = wscale[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        rope_store(pro, t[r] * sc * rinv[m < kProMaxM ? m : 0], m, M, n, blockIdx.x, col, y, ldy);
      }
    } else if (n < N) {
      const float sc = wscale[n];
      const float b = bias ? bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 4 * g + r;
        const float rs = MODE == PRO_RMS ? rinv[m < kProMaxM ? m : 0] : 1.f;
        if (m < M) y[(int64_t)m * ldy + n] = f32_to_bf16(t[r] * sc * rs + b);
      }
    }
  }
}

// Waves per workgroup and super-steps per wave of the bf16 kernel. (A split-K variant -- K split
// over 2-4 workgroups with a last-arrival reduction -- was measured and removed: 5.9 vs 3.7 ms per
// batch-1 decode step, profiles/r05/decode_splitk_ab.log.)
inline void plan(int tiles, int ss_total, int& nw, int& spw) {
  nw = pick_nw(tiles, ss_total, 4, 1);
  spw = (ss_total + nw - 1) / nw;
}

}  // namespace sg

// x [M, K] (row stride free, unit column stride), w [N, K] contiguous rows, bias [N] or None.
at::Tensor skinny_gemm(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "skinny_gemm: bf16 only");
  SXE_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "skinny_gemm: x [M, K], w [N, K]");
  SXE_CHECK(x.stride(1) == 1 && w.stride(1) == 1, "skinny_gemm: unit stride along K");
  const int M = x.size(0), N = w.size(0), K = x.size(1);
  SXE_CHECK(M >= 1 && M <= 16, "skinny_gemm: 1 <= M <= 16");
  SXE_CHECK(K % 8 == 0 && x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0,
            "skinny_gemm: K and row strides must be multiples of 8 (16-byte loads)");
  SXE_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
            "skinny_gemm: 16-byte aligned operands");
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return y;
  c10::DeviceGuard gd(x.device());
  const int ss_total = (K + sg::kSS - 1) / sg::kSS;
  const int tiles = (N + 15) / 16;
  int nw = 4, ss_per_wave = 1;
  sg::ProArgs pro{};
  pro.nt = sg::nt_loads();
  sg::plan(tiles, ss_total, nw, ss_per_wave);
  auto* xp = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto* wp = reinterpret_cast<const unsigned short*>(w.data_ptr());
  auto* yp = reinterpret_cast<unsigned short*>(y.data_ptr());
#define SXE_SG_LAUNCH(NW, NT)                                                                              \
  hipLaunchKernelGGL((sg::skinny_gemm_kernel<NW, sg::PRO_NONE, NT>), dim3(tiles), dim3(NW * 64), 0, cur_stream(), \
                     xp, x.stride(0), wp, w.stride(0), bp, yp, y.stride(0), M, N, K, ss_per_wave, pro)
  if (pro.nt) { if (nw == 4) SXE_SG_LAUNCH(4, true); else SXE_SG_LAUNCH(8, true); }
  else { if (nw == 4) SXE_SG_LAUNCH(4, false); else SXE_SG_LAUNCH(8, false); }
#undef SXE_SG_LAUNCH
  SXE_LAUNCH_CHECK();
  return y;
}

// x [M, K] bf16, wq [N, K] e4m3 bytes (uint8 or float8_e4m3fn), wscale [N] fp32, bias [N] bf16 or None
at::Tensor skinny_gemm_fp8w(const at::Tensor& x, const at::Tensor& wq, const at::Tensor& wscale,
                            const c10::optional<at::Tensor>& bias) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(x.scalar_type() == at::kBFloat16, "skinny_gemm_fp8w: bf16 activations");
  SXE_CHECK(wq.element_size() == 1 && wq.dim() == 2 && wq.stride(1) == 1, "skinny_gemm_fp8w: wq [N, K] bytes");
  SXE_CHECK(wscale.scalar_type() == at::kFloat && wscale.is_contiguous() && wscale.numel() == wq.size(0),
            "skinny_gemm_fp8w: wscale fp32 [N]");
  SXE_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) == wq.size(1), "skinny_gemm_fp8w: x [M, K]");
  const int M = x.size(0), N = wq.size(0), K = x.size(1);
  SXE_CHECK(M >= 1 && M <= 16, "skinny_gemm_fp8w: 1 <= M <= 16");
  SXE_CHECK(K % 16 == 0 && wq.stride(0) % 16 == 0 && x.stride(0) % 8 == 0,
            "skinny_gemm_fp8w: K and row strides must allow 16-byte loads");
  SXE_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(wq.data_ptr()) % 16 == 0,
            "skinny_gemm_fp8w: 16-byte aligned operands");
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return y;
  c10::DeviceGuard gd(x.device());
  const int ss_total = (K + sg::kSS8 - 1) / sg::kSS8;
  const int tiles = (N + 15) / 16;
  const int nw = sg::pick_nw(tiles, ss_total, 2, 2);
  const int ss_per_wave = (ss_total + nw - 1) / nw;
  auto* xp = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto* wp = reinterpret_cast<const uint8_t*>(wq.data_ptr());
  auto* yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  if (nw == 4)
    hipLaunchKernelGGL(sg::skinny_gemm_fp8w_kernel<4>, dim3(tiles), dim3(256), 0, cur_stream(), xp, x.stride(0), wp,
                       wq.stride(0), wscale.data_ptr<float>(), bp, yp, y.stride(0), M, N, K, ss_per_wave,
                       sg::ProArgs{});
  else
    hipLaunchKernelGGL(sg::skinny_gemm_fp8w_kernel<8>, dim3(tiles), dim3(512), 0, cur_stream(), xp, x.stride(0), wp,
                       wq.stride(0), wscale.data_ptr<float>(), bp, yp, y.stride(0), M, N, K, ss_per_wave,
                       sg::ProArgs{});
  SXE_LAUNCH_CHECK();
  return y;
}

// ---- fused-prologue entry points (decode, M <= 4) ----------------------------------------------
// mode 1 (rms): x [M, K], res [M, K] or None (same row stride), gw [K], eps -> (y [M, N], h [M, K] = x + res)
// mode 2 (swiglu): x = gu [M, 2K] (gate | up halves) -> y [M, N]
// wq: bf16 [N, K] (wscale None) or e4m3 bytes [N, K] with wscale fp32 [N]
struct RopeTensors {
  const at::Tensor *cos, *sin, *pos, *slots, *cache;
  int64_t nq, nkv;
};

static std::vector<at::Tensor> skinny_gemm_pro_impl(const at::Tensor& x, const c10::optional<at::Tensor>& res,
                                                    const c10::optional<at::Tensor>& gw, double eps,
                                                    const at::Tensor& w, const c10::optional<at::Tensor>& wscale,
                                                    const c10::optional<at::Tensor>& bias, int64_t mode,
                                                    const RopeTensors* rope) {
  SXE_CHECK_CUDA(x);
  SXE_CHECK(mode == sg::PRO_RMS || mode == sg::PRO_SWIGLU, "skinny_gemm_pro: mode 1 (rms) or 2 (swiglu)");
  SXE_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 &&
                reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "skinny_gemm_pro: x bf16 [M, *], 16-B rows");
  const bool fp8 = wscale.has_value() && wscale->defined();
  SXE_CHECK(w.dim() == 2 && w.stride(1) == 1 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
            "skinny_gemm_pro: w [N, K] row-major, 16-B aligned");
  SXE_CHECK(fp8 ? w.element_size() == 1 : w.scalar_type() == at::kBFloat16, "skinny_gemm_pro: w bf16 or fp8 bytes");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  SXE_CHECK(M >= 1 && M <= sg::kProMaxM, "skinny_gemm_pro: 1 <= M <= 4");
  SXE_CHECK(x.size(1) == (mode == sg::PRO_SWIGLU ? 2 * K : K), "skinny_gemm_pro: x width");
  SXE_CHECK(K % (fp8 ? 16 : 8) == 0 && w.stride(0) % (fp8 ? 16 : 8) == 0, "skinny_gemm_pro: K alignment");
  sg::ProArgs pro{nullptr, nullptr, nullptr, (float)eps};
  pro.nt = sg::nt_loads();
  if (rope != nullptr) {
    SXE_CHECK(mode == sg::PRO_RMS && !(bias.has_value() && bias->defined()), "skinny_gemm_pro_rope: RMS mode, no bias");
    const int64_t nq = rope->nq, nkv = rope->nkv;
    SXE_CHECK(nq > 0 && nkv > 0 && w.size(0) == (nq + 2 * nkv) * 128, "skinny_gemm_pro_rope: w rows = (nq + 2 nkv) * 128");
    const at::Tensor &c = *rope->cos, &sn = *rope->sin, &ps = *rope->pos, &sl = *rope->slots, &kc = *rope->cache;
    SXE_CHECK(c.scalar_type() == at::kFloat && sn.scalar_type() == at::kFloat && c.is_contiguous() && sn.is_contiguous() &&
                  c.dim() == 2 && c.size(1) == 64 && sn.sizes() == c.sizes(),
              "skinny_gemm_pro_rope: cos/sin fp32 [max_pos, 64]");
    SXE_CHECK(ps.scalar_type() == at::kLong && ps.is_contiguous() && ps.numel() == x.size(0) &&
                  sl.scalar_type() == at::kLong && sl.is_contiguous() && sl.numel() == x.size(0),
              "skinny_gemm_pro_rope: pos / slots int64 [M]");
    SXE_CHECK(kc.scalar_type() == at::kBFloat16 && kc.is_contiguous() && kc.dim() == 5 && kc.size(1) == 2 &&
                  kc.size(2) == nkv && kc.size(4) == 128,
              "skinny_gemm_pro_rope: cache bf16 [blocks, 2, nkv, bs, 128]");
    pro.rcos = c.data_ptr<float>();
    pro.rsin = sn.data_ptr<float>();
    pro.rpos = ps.data_ptr<int64_t>();
    pro.rslots = sl.data_ptr<int64_t>();
    pro.rcache = reinterpret_cast<unsigned short*>(kc.data_ptr());
    pro.rnq = (int)nq;
    pro.rnkv = (int)nkv;
    pro.rbs = (int)kc.size(3);
  }
  at::Tensor h;
  if (mode == sg::PRO_RMS) {
    SXE_CHECK(gw.has_value() && gw->scalar_type() == at::kBFloat16 && gw->is_contiguous() && gw->numel() == K,
              "skinny_gemm_pro: norm weight bf16 [K]");
    pro.gw = reinterpret_cast<const unsigned short*>(gw->data_ptr());
    if (res.has_value() && res->defined()) {
      SXE_CHECK(res->scalar_type() == at::kBFloat16 && res->sizes() == x.sizes() && res->strides() == x.strides(),
                "skinny_gemm_pro: residual like x");
      pro.res = reinterpret_cast<const unsigned short*>(res->data_ptr());
      h = at::empty({M, K}, x.options());
      pro.hout = reinterpret_cast<unsigned short*>(h.data_ptr());
    }
  }
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return {y, h.defined() ? h : x};
  c10::DeviceGuard gd(x.device());
  const size_t lds = (size_t)M * K * 2;
  SXE_CHECK(lds <= 144 * 1024, "skinny_gemm_pro: M x K input exceeds the LDS budget");
  const int tiles = (N + 15) / 16;
  auto* xp = reinterpret_cast<const unsigned short*>(x.data_ptr());
  auto* yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  static bool attr[3][2][2] = {};  // [bf16 / fp8 / bf16 nt][NW == 8][mode]
  auto set = [&](const void* f, int a, int b, int c) {
    if (!attr[a][b][c]) {
      SXE_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024));
      attr[a][b][c] = true;
    }
  };
  const int mi = mode == sg::PRO_RMS ? 0 : 1;
  if (!fp8) {
    const int ss_total = (K + sg::kSS - 1) / sg::kSS;
    int nw = 4, spw = 1;
    sg::plan(tiles, ss_total, nw, spw);
    auto* wp = reinterpret_cast<const unsigned short*>(w.data_ptr());
#define SXE_SGP1(NW, MODE, NT)                                                                                       \
  do {                                                                                                               \
    set(reinterpret_cast<const void*>(&sg::skinny_gemm_kernel<NW, MODE, NT>), NT ? 2 : 0, NW == 8, mi);              \
    hipLaunchKernelGGL((sg::skinny_gemm_kernel<NW, MODE, NT>), dim3(tiles), dim3(NW * 64), lds, cur_stream(), xp,     \
                       x.stride(0), wp, w.stride(0), bp, yp, y.stride(0), M, N, K, spw, pro);                         \
  } while (0)
#define SXE_SGP(NW, MODE)                                                                                            \
  do {                                                                                                               \
    if (pro.nt) SXE_SGP1(NW, MODE, true);                                                                            \
    else SXE_SGP1(NW, MODE, false);                                                                                  \
  } while (0)
    if (mode == sg::PRO_RMS) { if (nw == 4) SXE_SGP(4, sg::PRO_RMS); else SXE_SGP(8, sg::PRO_RMS); }
    else { if (nw == 4) SXE_SGP(4, sg::PRO_SWIGLU); else SXE_SGP(8, sg::PRO_SWIGLU); }
#undef SXE_SGP
#undef SXE_SGP1
  } else {
    SXE_CHECK(wscale->scalar_type() == at::kFloat && wscale->is_contiguous() && wscale->numel() == N,
              "skinny_gemm_pro: wscale fp32 [N]");
    const int ss_total = (K + sg::kSS8 - 1) / sg::kSS8;
    const int nw = sg::pick_nw(tiles, ss_total, 2, 2);
    const int spw = (ss_total + nw - 1) / nw;
    auto* wp = reinterpret_cast<const uint8_t*>(w.data_ptr());
    const float* sp = wscale->data_ptr<float>();
#define SXE_SGP8(NW, MODE)                                                                                           \
  do {                                                                                                               \
    set(reinterpret_cast<const void*>(&sg::skinny_gemm_fp8w_kernel<NW, MODE>), 1, NW == 8, mi);                      \
    hipLaunchKernelGGL((sg::skinny_gemm_fp8w_kernel<NW, MODE>), dim3(tiles), dim3(NW * 64), lds, cur_stream(), xp,    \
                       x.stride(0), wp, w.stride(0), sp, bp, yp, y.stride(0), M, N, K, spw, pro);                     \
  } while (0)
    if (mode == sg::PRO_RMS) { if (nw == 4) SXE_SGP8(4, sg::PRO_RMS); else SXE_SGP8(8, sg::PRO_RMS); }
    else { if (nw == 4) SXE_SGP8(4, sg::PRO_SWIGLU); else SXE_SGP8(8, sg::PRO_SWIGLU); }
#undef SXE_SGP8
  }
  SXE_LAUNCH_CHECK();
  return {y, h.defined() ? h : x};
}

std::vector<at::Tensor> skinny_gemm_pro(const at::Tensor& x, const c10::optional<at::Tensor>& res,
                                        const c10::optional<at::Tensor>& gw, double eps, const at::Tensor& w,
                                        const c10::optional<at::Tensor>& wscale, const c10::optional<at::Tensor>& bias,
                                        int64_t mode) {
  return skinny_gemm_pro_impl(x, res, gw, eps, w, wscale, bias, mode, nullptr);
}

// The decode QKV projection with residual + RMSNorm prologue AND the RoPE + paged-KV-append
// epilogue: returns [qkv (q / k rotated), h]; the rotated k and v rows land in `cache`.
std::vector<at::Tensor> skinny_gemm_pro_rope(const at::Tensor& x, const c10::optional<at::Tensor>& res,
                                             const at::Tensor& gw, double eps, const at::Tensor& w,
                                             const c10::optional<at::Tensor>& wscale, const at::Tensor& cos_t,
                                             const at::Tensor& sin_t, const at::Tensor& pos, const at::Tensor& slots,
                                             at::Tensor cache, int64_t nq, int64_t nkv) {
  RopeTensors r{&cos_t, &sin_t, &pos, &slots, &cache, nq, nkv};
  return skinny_gemm_pro_impl(x, res, gw, eps, w, wscale, c10::nullopt, sg::PRO_RMS, &r);
}

// Decode o_proj with the flash-decoding merge as its prologue (PRO_MERGE): part_o fp32
// [splits, M, nq, D] and part_ml fp32 [splits, M, nq, 2] from paged_attention_parts; w bf16 [N, K]
// (wscale None) or e4m3 bytes with wscale fp32 [N]; K = nq * D. One launch instead of merge + GEMM.
at::Tensor skinny_gemm_merge(const at::Tensor& part_o, const at::Tensor& part_ml, const at::Tensor& w,
                             const c10::optional<at::Tensor>& wscale, const c10::optional<at::Tensor>& bias) {
  SXE_CHECK_CUDA(part_o);
  SXE_CHECK(part_o.scalar_type() == at::kFloat && part_o.dim() == 4 && part_o.is_contiguous() &&
                part_ml.scalar_type() == at::kFloat && part_ml.is_contiguous() && part_ml.dim() == 4 &&
                part_ml.size(0) == part_o.size(0) && part_ml.size(1) == part_o.size(1) &&
                part_ml.size(2) == part_o.size(2) && part_ml.size(3) == 2,
            "skinny_gemm_merge: part_o fp32 [S, M, nq, D], part_ml fp32 [S, M, nq, 2]");
  const int S = part_o.size(0), M = part_o.size(1), nq = part_o.size(2), D = part_o.size(3);
  const bool fp8 = wscale.has_value() && wscale->defined();
  SXE_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.is_contiguous() && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
            "skinny_gemm_merge: w [N, K] row-major, 16-B aligned");
  SXE_CHECK(fp8 ? w.element_size() == 1 : w.scalar_type() == at::kBFloat16, "skinny_gemm_merge: w bf16 or fp8 bytes");
  const int N = w.size(0), K = w.size(1);
  SXE_CHECK(K == nq * D && D % 8 == 0 && M >= 1 && M <= sg::kProMaxM && S >= 1, "skinny_gemm_merge: K = nq * D, M <= 4");
  SXE_CHECK(K % (fp8 ? 16 : 8) == 0, "skinny_gemm_merge: K alignment");
  sg::ProArgs pro{nullptr, nullptr, nullptr, 0.f, part_o.data_ptr<float>(), part_ml.data_ptr<float>(), S, nq};
  pro.nt = sg::nt_loads();
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    SXE_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias: bf16 [N]");
    bp = reinterpret_cast<const unsigned short*>(bias->data_ptr());
  }
  auto y = at::empty({M, N}, part_o.options().dtype(at::kBFloat16));
  if (N == 0) return y;
  c10::DeviceGuard gd(part_o.device());
  const size_t lds = (size_t)M * K * 2;
  SXE_CHECK(lds <= 144 * 1024, "skinny_gemm_merge: M x K input exceeds the LDS budget");
  const int tiles = (N + 15) / 16;
  auto* yp = reinterpret_cast<unsigned short*>(y.data_ptr());
  static bool attr[3][2] = {};  // [bf16 / fp8 / bf16 nt][NW == 8]
  auto set = [&](const void* f, int a, int b) {
    if (!attr[a][b]) {
      SXE_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024));
      attr[a][b] = true;
    }
  };
  if (!fp8) {
    const int ss_total = (K + sg::kSS - 1) / sg::kSS;
    int nw = 4, spw = 1;
    sg::plan(tiles, ss_total, nw, spw);
    auto* wp = reinterpret_cast<const unsigned short*>(w.data_ptr());
#define SXE_SGM1(NW, NT)                                                                                             \
  do {                                                                                                               \
    set(reinterpret_cast<const void*>(&sg::skinny_gemm_kernel<NW, sg::PRO_MERGE, NT>), NT ? 2 : 0, NW == 8);         \
    hipLaunchKernelGGL((sg::skinny_gemm_kernel<NW, sg::PRO_MERGE, NT>), dim3(tiles), dim3(NW * 64), lds,              \
                       cur_stream(),                                                                                 \
                       nullptr, K, wp, w.stride(0), bp, yp, y.stride(0), M, N, K, spw, pro);                          \
  } while (0)
#define SXE_SGM(NW)                                                                                                  \
  do {                                                                                                               \
    if (pro.nt) SXE_SGM1(NW, true);                                                                                  \
    else SXE_SGM1(NW, false);                                                                                        \
  } while (0)
    if (nw == 4) SXE_SGM(4); else SXE_SGM(8);
#undef SXE_SGM
#undef SXE_SGM1
  } else {
    SXE_CHECK(wscale->scalar_type() == at::kFloat && wscale->is_contiguous() && wscale->numel() == N,
              "skinny_gemm_merge: wscale fp32 [N]");
    const int ss_total = (K + sg::kSS8 - 1) / sg::kSS8;
    const int nw = sg::pick_nw(tiles, ss_total, 2, 2);
    const int spw = (ss_total + nw - 1) / nw;
    auto* wp = reinterpret_cast<const uint8_t*>(w.data_ptr());
    const float* sp = wscale->data_ptr<float>();
#define SXE_SGM8(NW)                                                                                                 \
  do {                                                                                                               \
    set(reinterpret_cast<const void*>(&sg::skinny_gemm_fp8w_kernel<NW, sg::PRO_MERGE>), 1, NW == 8);                 \
    hipLaunchKernelGGL((sg::skinny_gemm_fp8w_kernel<NW, sg::PRO_MERGE>), dim3(tiles), dim3(NW * 64), lds,            \
                       cur_stream(), nullptr, K, wp, w.stride(0), sp, bp, yp, y.stride(0), M, N, K, spw, pro);        \
  } while (0)
    if (nw == 4) SXE_SGM8(4); else SXE_SGM8(8);
#undef SXE_SGM8
  }
  SXE_LAUNCH_CHECK();
  return y;
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("skinny_gemm(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("skinny_gemm_fp8w(Tensor x, Tensor wq, Tensor wscale, Tensor? bias) -> Tensor");
  m.def("skinny_gemm_pro(Tensor x, Tensor? res, Tensor? gw, float eps, Tensor w, Tensor? wscale, Tensor? bias, "
        "int mode) -> Tensor[]");
  m.def("skinny_gemm_merge(Tensor part_o, Tensor part_ml, Tensor w, Tensor? wscale, Tensor? bias) -> Tensor");
  m.def("skinny_gemm_pro_rope(Tensor x, Tensor? res, Tensor gw, float eps, Tensor w, Tensor? wscale, Tensor cos, "
        "Tensor sin, Tensor pos, Tensor slots, Tensor(a!) cache, int nq, int nkv) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("skinny_gemm", &sxe::skinny_gemm);
  m.impl("skinny_gemm_fp8w", &sxe::skinny_gemm_fp8w);
  m.impl("skinny_gemm_pro", &sxe::skinny_gemm_pro);
  m.impl("skinny_gemm_merge", &sxe::skinny_gemm_merge);
  m.impl("skinny_gemm_pro_rope", &sxe::skinny_gemm_pro_rope);
}

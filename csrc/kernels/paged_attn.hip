// Ragged / paged-KV attention for the FastGen-style inference engine (gfx950).
//
// Parity: reference inference/v2/kernels/ragged_ops/linear_blocked_kv_rotary (KV append into the
// blocked cache) and ragged_ops/blocked_flash (attention over blocked KV; the reference links an
// external flash-attn build for sm80+). Designed for MI355X instead:
//
//  * cache layout per layer: [num_blocks, 2 (k|v), n_kv_heads, block_size, D] bf16 -- the keys of
//    one (block, head) are one contiguous run, so a wave reading 64 consecutive keys streams
//    64 x 256 B = 16 KB with no stride;
//  * one workgroup (4 waves, 256 threads) per (sequence, kv head, KV split): all G = nq/nkv query
//    heads of the GQA group (x the sequence's new tokens) share every K/V byte loaded, so decode is
//    pure HBM streaming at the GQA-reduced byte count;
//  * both products on the matrix cores (v_mfma_f32_16x16x32_bf16), 16 query rows (token x head of
//    the group) per pass: S^T = K Q^T with K fragments loaded straight from the cache into the A
//    operand (lane = key row of a 16-key tile) and Q^T in the B operand, so each lane holds one
//    query row's scores (online softmax per lane, max/sum folded over the 4 lane groups with two
//    shuffles); O^T += V^T P^T takes P^T directly from the score accumulators (the
//    accumulator-as-operand identity: the 16x16 C layout's k order is matched by the order the V
//    rows are read) and V^T through ds_read_b64_tr_b16 from a per-wave V image in LDS, loaded by
//    global_load_lds (no staging registers) with the XOR-swizzled 2D-byte rows; the key rows of a
//    tile are permuted (0, 8, 4, 12 + e) so each 32-lane half's transposed read is conflict-free;
//  * decode (4 rows of 16 used for Llama-3's G = 4) wastes MFMA lanes, not bandwidth: the previous
//    VALU kernel spent 512 FMA instructions per wave per 64 keys on Q K^T alone;
//  * flash-decoding split over the KV length when (sequences x kv heads) is too small to fill the
//    256 CUs, merged by a second kernel (fp32 partials);
//  * causal masking by absolute position (chunked prefill / speculative tokens just work), sliding
//    windows skip the key chunks they mask entirely.
#include "sxe_common.h"
#include <torch/library.h>

namespace sxe {
namespace pa {

constexpr int kWaves = 4;
constexpr float kLog2e = 1.4426950408889634f;

template <int D>
__global__ __launch_bounds__(256) void kv_append_kernel(const unsigned short* __restrict qkv, int64_t tok_stride,
                                                        int nq, int nkv, const int64_t* __restrict slots,
                                                        unsigned short* __restrict cache, int bs) {
  const int t = blockIdx.x;
  const int64_t slot = slots[t];
  if (slot < 0) return;
  const int64_t blk = slot / bs, off = slot % bs;
  constexpr int V = D / 8;
  const int total = 2 * nkv * V;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int kv = i / (nkv * V);
    const int rem = i - kv * nkv * V;
    const int h = rem / V, v = rem - h * V;
    const unsigned short* src = qkv + (int64_t)t * tok_stride + (int64_t)(nq + kv * nkv + h) * D + v * 8;
    unsigned short* dst = cache + (((blk * 2 + kv) * nkv + h) * bs + off) * D + v * 8;
    *reinterpret_cast<u16x8*>(dst) = *reinterpret_cast<const u16x8*>(src);
  }
}

// Decode/prefill prologue in ONE launch: rotate the q and k heads of each token in place
// (rotate-half RoPE, fp32 cos/sin table [max_pos, D/2] at the token's absolute position) and write
// the rotated k plus v into the paged cache -- the separate rope_ + kv_append launches were ~7 us
// of latency per layer at batch 1. One workgroup per token; a thread handles 8 rotation pairs.
template <int D>
__global__ __launch_bounds__(256) void rope_kv_append_kernel(unsigned short* __restrict qkv, int64_t tok_stride,
                                                             int nq, int nkv, const int64_t* __restrict pos,
                                                             const float* __restrict cos_t,
                                                             const float* __restrict sin_t,
                                                             const int64_t* __restrict slots,
                                                             unsigned short* __restrict cache, int bs) {
  constexpr int HALF = D / 2, VR = HALF / 8, VV = D / 8;
  const int t = blockIdx.x;
  const int64_t slot = slots[t];
  const int64_t blk = slot / bs, off = slot % bs;
  const int64_t p = pos[t];
  unsigned short* row = qkv + (int64_t)t * tok_stride;
  const int nrot = (nq + nkv) * VR;
  for (int i = threadIdx.x; i < nrot + nkv * VV; i += blockDim.x) {
    if (i < nrot) {
      const int h = i / VR, c = (i - h * VR) * 8;
      unsigned short* base = row + (int64_t)h * D;
      float a[8], b[8], cs[8], sn[8], oa[8], ob[8];
      load8<DT::BF16>(base + c, a);
      load8<DT::BF16>(base + HALF + c, b);
      load8<DT::F32>(cos_t + p * HALF + c, cs);
      load8<DT::F32>(sin_t + p * HALF + c, sn);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        oa[j] = a[j] * cs[j] - b[j] * sn[j];
        ob[j] = b[j] * cs[j] + a[j] * sn[j];
      }
      store8<DT::BF16>(base + c, oa);
      store8<DT::BF16>(base + HALF + c, ob);
      if (h >= nq && slot >= 0) {  // rotated k -> cache
        unsigned short* dst = cache + (((blk * 2 + 0) * nkv + (h - nq)) * bs + off) * D;
        store8<DT::BF16>(dst + c, oa);
        store8<DT::BF16>(dst + HALF + c, ob);
      }
    } else if (slot >= 0) {  // v -> cache
      const int j = i - nrot, h = j / VV, v = j - h * VV;
      const unsigned short* src = row + (int64_t)(nq + nkv + h) * D + v * 8;
      unsigned short* dst = cache + (((blk * 2 + 1) * nkv + h) * bs + off) * D + v * 8;
      *reinterpret_cast<u16x8*>(dst) = *reinterpret_cast<const u16x8*>(src);
    }
  }
}

struct Args {
  const unsigned short* q;
  int64_t q_tok_stride;  // elements between consecutive tokens (heads are D apart)
  const unsigned short* cache;
  const int* block_table;
  int max_blocks;
  const int* q_start;
  const int* q_len;
  const int* kv_len;
  int nq, nkv, bs;
  float scale_log2;
  int splits, keys_per_split;
  unsigned short* out;
  int64_t out_tok_stride;
  float* part_o;   // [splits, T, nq, D]
  float* part_ml;  // [splits, T, nq, 2]
  int T;
  int window;      // sliding window (Mistral / Qwen2): keys older than `window` positions are masked; 0 = off
  int* counters;   // [S * nkv] zeroed split-arrival counters: the last split of a (seq, kv head) merges; or null
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-byte chunk `ch` of row `row` in a swizzled [rows][D bf16] image (see flash_attn.hip)
template <int D>
__device__ __forceinline__ int soff(int row, int ch) {
  constexpr int CH = D / 8;
  const int f = (((row & 3) << 2) | ((row >> 2) & 3)) & (CH >= 16 ? 15 : CH - 1);
  return row * (2 * D) + 16 * (ch ^ f);
}

// first key row of lane group g's 4-row block in a 16-key tile (C rows 4g..4g+3 <-> keys kperm(g)+e):
// the two groups of a 32-lane half read blocks 8 rows apart -> conflict-free transposed reads
__device__ __forceinline__ int kperm(int g) { return ((g & 1) << 3) | ((g & 2) << 1); }

constexpr int PR = 16;  // query rows per pass

template <int D>
struct PaGeo {
  static constexpr int NT = D >= 256 ? 2 : 4;  // 16-key tiles per wave chunk (register budget at D = 256)
  static constexpr int KC = 16 * NT;           // keys per wave chunk
  static constexpr int KS = D / 32;            // k-steps of the Q K^T product
  static constexpr int DT = D / 16;            // 16-wide d tiles of O^T
  static constexpr int VIMG = KC * 2 * D;      // bytes of one wave's V image
  static constexpr int MERGE = kWaves * PR * D * 4;
  static constexpr int LDS = (kWaves * VIMG > MERGE ? kWaves * VIMG : MERGE);
};

template <int D>
__global__ __launch_bounds__(256) void paged_attn_kernel(Args a) {
  using P = PaGeo<D>;
  constexpr int NT = P::NT, KC = P::KC, KS = P::KS, DT = P::DT;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // V images, then the wave-merge buffer
  __shared__ int64_t koff_lds[kWaves][KC];
  __shared__ float mrg_ml[kWaves][PR][2];

  const int seq = blockIdx.x / a.nkv, kvh = blockIdx.x - (blockIdx.x / a.nkv) * a.nkv;
  const int split = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int G = a.nq / a.nkv;
  const int qs = a.q_start[seq], ql = a.q_len[seq], kl = a.kv_len[seq];
  const int k_begin = split * a.keys_per_split;
  const int k_end = min(kl, k_begin + a.keys_per_split);
  const int nrows_total = ql * G;
  const int* bt = a.block_table + (int64_t)seq * a.max_blocks;
  const int64_t head_stride = (int64_t)a.bs * D;             // between kv heads inside a block half
  const int64_t half_stride = (int64_t)a.nkv * head_stride;  // k half -> v half
  const int64_t block_stride = 2 * half_stride;
  char* vimg = smem + wave * P::VIMG;
  float* mrg_o = reinterpret_cast<float*>(smem);  // [kWaves][PR][D] after the key loop
  const int krow = kperm(i >> 2) + (i & 3);        // this lane's key row in a tile (A operand of Q K^T)

  for (int row0 = 0; row0 < nrows_total; row0 += PR) {
    const int nrows = min(PR, nrows_total - row0);
    // ---- Q^T B operand: lane holds row i's d = 32 ks + 8 g .. +7 ---------------------------------
    bf16x8 qb[KS];
    const bool row_ok = i < nrows;
    int pos = -1;  // absolute position of this lane's query row (causal horizon)
    {
      const int row = row0 + (row_ok ? i : 0), tok = row / G, gh = row - tok * G;
      const unsigned short* qp = a.q + (int64_t)(qs + tok) * a.q_tok_stride + (int64_t)(kvh * G + gh) * D + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        u32x4 v = *reinterpret_cast<const u32x4*>(qp + 32 * ks);
        if (!row_ok) v = u32x4{0u, 0u, 0u, 0u};
        qb[ks] = __builtin_bit_cast(bf16x8, v);
      }
      if (row_ok) pos = kl - ql + tok;
    }
    const int max_pos = kl - ql + (row0 + nrows - 1) / G;  // causal horizon of the pass
    const int k_hi = min(k_end, max_pos + 1);
    int k_start = k_begin;
    if (a.window > 0) {  // first chunk holding a key visible to the pass's oldest row
      const int k_lo = kl - ql + row0 / G - a.window + 1;
      if (k_lo > k_begin) k_start = k_begin + ((k_lo - k_begin) / KC) * KC;
    }
    float m = -INFINITY, lsum = 0.f;
    f32x4 o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kb = k_start + wave * KC; kb < k_hi; kb += kWaves * KC) {
      // ---- cache offsets of the chunk's keys (lane = key; keys past k_hi re-read key kb) ----------
      if (lane < KC) {
        const int key = kb + lane;
        const int kc = key < k_hi ? key : kb;
        const int blk = bt[kc / a.bs], off = kc - (kc / a.bs) * a.bs;
        koff_lds[wave][lane] = (int64_t)blk * block_stride + kvh * head_stride + (int64_t)off * D;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      // ---- K fragments straight into the A operand: tile t, key row krow, d = 32 ks + 8 g ---------
      bf16x8 kr[NT][KS];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const unsigned short* kp = a.cache + koff_lds[wave][16 * t + krow] + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kr[t][ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(kp + 32 * ks));
      }
      // ---- V rows -> this wave's LDS image (global_load_lds, swizzled source chunk) -------------
      {
        constexpr int CH = D / 8, RPK = 64 / CH;  // rows per 1 KiB wave-instruction
#pragma unroll
        for (int n = 0; n < KC / RPK; ++n) {
          const int row = RPK * n + lane / CH;
          const int cpos = lane % CH;
          const int ch = cpos ^ ((((row & 3) << 2) | ((row >> 2) & 3)) & (CH >= 16 ? 15 : CH - 1));
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(a.cache + koff_lds[wave][row] + half_stride + ch * 8),
              (__attribute__((address_space(3))) void*)(vimg + n * 1024), 16, 0, 0);
        }
      }
      // ---- S^T = K Q^T: lane holds keys 16t + kperm(g) + e of row i ------------------------------
      f32x4 sc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) sc[t] = mfma16(kr[t][ks], qb[ks], sc[t]);
      }
      // ---- online softmax of row i over the chunk -------------------------------------------------
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int key = kb + 16 * t + kperm(g) + e;
          const bool vis = key < k_hi && key <= pos && (a.window <= 0 || key > pos - a.window);
          const float x = vis ? sc[t][e] * a.scale_log2 : -INFINITY;
          sc[t][e] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float mref = mn == -INFINITY ? 0.f : mn;
      const float alpha = m == -INFINITY ? 0.f : exp2f(m - mref);
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = exp2f(sc[t][e] - mref);  // exp2(-inf) = 0 for masked keys
          sc[t][e] = p;
          ps += p;
        }
      lsum = lsum * alpha + ps;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's V image has landed
      __builtin_amdgcn_wave_barrier();
      // ---- O^T += V^T P^T over key-tile pairs: P^T straight from the score registers -------------
#pragma unroll
      for (int pp = 0; pp < NT / 2; ++pp) {
        bf16x8 pb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pb[e] = (__bf16)sc[2 * pp][e];
          pb[4 + e] = (__bf16)sc[2 * pp + 1][e];
        }
        const int q4 = i >> 2, p4 = i & 3;
        const int r0 = 32 * pp + kperm(g) + q4;  // row of this lane's address in the first tile
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int ch = 2 * dt + (p4 >> 1);
          const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) i16x4*)(vimg + soff<D>(r0, ch) + 8 * (p4 & 1)));
          const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) i16x4*)(vimg + soff<D>(r0 + 16, ch) + 8 * (p4 & 1)));
          const i16x8 va = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          o[dt] = mfma16(__builtin_bit_cast(bf16x8, va), pb, o[dt]);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // the V image is read before the next chunk overwrites it
      __builtin_amdgcn_wave_barrier();
    }
    // ---- fold the row sum over the 4 lane groups; merge the 4 waves through LDS --------------------
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    __syncthreads();  // every wave is done with its V image (the merge buffer aliases it)
    if (row_ok) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int e = 0; e < 4; ++e) mrg_o[(wave * PR + i) * D + 16 * dt + 4 * g + e] = o[dt][e];
      if (g == 0) {
        mrg_ml[wave][i][0] = m;
        mrg_ml[wave][i][1] = lsum;
      }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nrows * D; idx += 256) {
      const int r = idx / D, d = idx - r * D;
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) M = fmaxf(M, mrg_ml[w][r][0]);
      float sum = 0.f, L = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const float mw = mrg_ml[w][r][0];
        const float f = (mw == -INFINITY) ? 0.f : exp2f(mw - M);
        sum += f * mrg_o[(w * PR + r) * D + d];
        L += f * mrg_ml[w][r][1];
      }
      const int row = row0 + r, tok = row / G, gh = row - tok * G;
      const int t = qs + tok, h = kvh * G + gh;
      if (a.splits == 1) {
        a.out[(int64_t)t * a.out_tok_stride + (int64_t)h * D + d] = f32_to_bf16(L > 0.f ? sum / L : 0.f);
      } else {
        const int64_t pidx = ((int64_t)split * a.T + t) * a.nq + h;
        a.part_o[pidx * D + d] = sum;
        if (d == 0) {
          a.part_ml[pidx * 2 + 0] = M;
          a.part_ml[pidx * 2 + 1] = L;
        }
      }
    }
    __syncthreads();
  }
  if (a.counters != nullptr) {
    // In-kernel split merge: the last of the `splits` workgroups of this (sequence, kv head) to
    // finish combines every split's partials (merge_kernel's math) and writes the bf16 output --
    // no second launch. Release: each split's partials are made visible device-wide (across the
    // XCDs' L2s) before its arrival is counted; acquire: the last one fences again before reading.
    __shared__ int is_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = atomicAdd(a.counters + blockIdx.x, 1);
      is_last = prev == a.splits - 1;
      if (is_last) atomicExch(a.counters + blockIdx.x, 0);  // self-resetting: ready for the next launch / replay
    }
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    constexpr int U = 8;
    const int64_t sstride = (int64_t)a.T * a.nq;
    for (int idx = threadIdx.x; idx < nrows_total * D; idx += 256) {
      const int r = idx / D, d = idx - r * D, tok = r / G, gh = r - tok * G;
      const int t = qs + tok, h = kvh * G + gh;
      const int64_t th = (int64_t)t * a.nq + h;
      float M = -INFINITY, acc = 0.f, L = 0.f;
      for (int s0 = 0; s0 < a.splits; s0 += U) {
        float ms[U], ls[U], os[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i2 = (int64_t)min(s0 + u, a.splits - 1) * sstride + th;
          ms[u] = a.part_ml[i2 * 2];
          ls[u] = a.part_ml[i2 * 2 + 1];
          os[u] = a.part_o[i2 * D + d];
        }
        float Mc = M;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (s0 + u < a.splits) Mc = fmaxf(Mc, ms[u]);
        const float rs = (M == -INFINITY) ? 0.f : exp2f(M - Mc);
        acc *= rs;
        L *= rs;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (s0 + u < a.splits && ms[u] != -INFINITY) {
            const float f = exp2f(ms[u] - Mc);
            acc += f * os[u];
            L += f * ls[u];
          }
        }
        M = Mc;
      }
      a.out[(int64_t)t * a.out_tok_stride + (int64_t)h * D + d] = f32_to_bf16(L > 0.f ? acc / L : 0.f);
    }
  }
}

// Combine the splits' fp32 partials of one (token, head): every load of a group of up to 16 splits is
// issued before the first use (a loop that consumes each partial before loading the next makes a
// chain of dependent ~1 us memory round trips: 10 us at 16 splits).
template <int D>
__global__ __launch_bounds__(D) void merge_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                                                  int splits, int T, int nq, unsigned short* __restrict__ out,
                                                  int64_t out_tok_stride) {
  constexpr int U = 16;
  const int th = blockIdx.x;  // t * nq + h
  const int t = th / nq, h = th - t * nq;
  const int d = threadIdx.x;
  const int64_t sstride = (int64_t)T * nq;
  float M = -INFINITY, acc = 0.f, L = 0.f;
  for (int s0 = 0; s0 < splits; s0 += U) {
    float ms[U], ls[U], os[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = min(s0 + u, splits - 1);
      const int64_t idx = s * sstride + th;
      ms[u] = part_ml[idx * 2];
      ls[u] = part_ml[idx * 2 + 1];
      os[u] = part_o[idx * D + d];
    }
    float Mc = M;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s0 + u < splits) Mc = fmaxf(Mc, ms[u]);
    const float r = (M == -INFINITY) ? 0.f : exp2f(M - Mc);
    acc *= r;
    L *= r;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s0 + u < splits && ms[u] != -INFINITY) {
        const float f = exp2f(ms[u] - Mc);
        acc += f * os[u];
        L += f * ls[u];
      }
    }
    M = Mc;
  }
  out[(int64_t)t * out_tok_stride + (int64_t)h * D + d] = f32_to_bf16(L > 0.f ? acc / L : 0.f);
}

}  // namespace pa

// qkv: [T, nq + 2 nkv, D] bf16 (token stride may exceed the row); slots: [T] int64 (-1 = skip)
void rope_kv_cache_append(at::Tensor qkv, const at::Tensor& cos_t, const at::Tensor& sin_t, const at::Tensor& pos,
                          at::Tensor cache, const at::Tensor& slots, int64_t nq, int64_t nkv) {
  SXE_CHECK_CUDA(qkv);
  SXE_CHECK(qkv.scalar_type() == at::kBFloat16 && cache.scalar_type() == at::kBFloat16, "bf16 only");
  SXE_CHECK(qkv.dim() == 3 && qkv.stride(2) == 1 && qkv.stride(1) == qkv.size(2), "qkv must be [T, H, D] row-major");
  SXE_CHECK(qkv.size(1) == nq + 2 * nkv, "qkv heads != nq + 2 nkv");
  SXE_CHECK(cache.dim() == 5 && cache.is_contiguous() && cache.size(2) == nkv && cache.size(4) == qkv.size(2),
            "cache must be [blocks, 2, nkv, bs, D]");
  SXE_CHECK(slots.scalar_type() == at::kLong && slots.numel() == qkv.size(0), "slots: int64 [T]");
  SXE_CHECK(pos.scalar_type() == at::kLong && pos.numel() == qkv.size(0) && pos.is_contiguous(), "pos: int64 [T]");
  const int D = qkv.size(2);
  SXE_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                sin_t.is_contiguous() && cos_t.dim() == 2 && cos_t.size(1) == D / 2 && sin_t.sizes() == cos_t.sizes(),
            "cos/sin: fp32 [max_pos, D/2]");
  const int T = qkv.size(0);
  if (T == 0) return;
  c10::DeviceGuard g(qkv.device());
  auto* q = reinterpret_cast<unsigned short*>(qkv.data_ptr());
  auto* c = reinterpret_cast<unsigned short*>(cache.data_ptr());
  const int bs = cache.size(3);
#define SXE_RKA(DD)                                                                                              \
  hipLaunchKernelGGL(pa::rope_kv_append_kernel<DD>, dim3(T), dim3(256), 0, cur_stream(), q, qkv.stride(0), (int)nq, \
                     (int)nkv, pos.data_ptr<int64_t>(), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(),       \
                     slots.data_ptr<int64_t>(), c, bs)
  if (D == 128) SXE_RKA(128);
  else if (D == 64) SXE_RKA(64);
  else if (D == 256) SXE_RKA(256);
  else SXE_CHECK(false, "rope_kv_cache_append: head_dim must be 64, 128 or 256");
#undef SXE_RKA
  SXE_LAUNCH_CHECK();
}

void kv_cache_append(const at::Tensor& qkv, at::Tensor cache, const at::Tensor& slots, int64_t nq, int64_t nkv) {
  SXE_CHECK_CUDA(qkv);
  SXE_CHECK(qkv.scalar_type() == at::kBFloat16 && cache.scalar_type() == at::kBFloat16, "bf16 only");
  SXE_CHECK(qkv.dim() == 3 && qkv.stride(2) == 1 && qkv.stride(1) == qkv.size(2), "qkv must be [T, H, D] row-major");
  SXE_CHECK(cache.dim() == 5 && cache.is_contiguous(), "cache must be [blocks, 2, nkv, bs, D]");
  SXE_CHECK(slots.scalar_type() == at::kLong && slots.numel() == qkv.size(0), "slots: int64 [T]");
  const int D = qkv.size(2);
  const int T = qkv.size(0);
  if (T == 0) return;
  c10::DeviceGuard g(qkv.device());
  auto* q = reinterpret_cast<const unsigned short*>(qkv.data_ptr());
  auto* c = reinterpret_cast<unsigned short*>(cache.data_ptr());
  const int bs = cache.size(3);
  if (D == 128)
    hipLaunchKernelGGL(pa::kv_append_kernel<128>, dim3(T), dim3(256), 0, cur_stream(), q, qkv.stride(0), (int)nq,
                       (int)nkv, slots.data_ptr<int64_t>(), c, bs);
  else if (D == 64)
    hipLaunchKernelGGL(pa::kv_append_kernel<64>, dim3(T), dim3(256), 0, cur_stream(), q, qkv.stride(0), (int)nq,
                       (int)nkv, slots.data_ptr<int64_t>(), c, bs);
  else if (D == 256)
    hipLaunchKernelGGL(pa::kv_append_kernel<256>, dim3(T), dim3(256), 0, cur_stream(), q, qkv.stride(0), (int)nq,
                       (int)nkv, slots.data_ptr<int64_t>(), c, bs);
  else
    SXE_CHECK(false, "kv_cache_append: head_dim must be 64, 128 or 256");
  SXE_LAUNCH_CHECK();
}

// q: [T, nq, D] (token stride free); returns out [T, nq, D] bf16. parts != nullptr (and splits > 1):
// no merge launch -- the fp32 partials go to (*parts)[0] = part_o [splits, T, nq, D] and
// (*parts)[1] = part_ml [splits, T, nq, 2] for a consumer that merges them itself (skinny_gemm_merge)
static at::Tensor paged_attention_impl(const at::Tensor& q, const at::Tensor& cache, const at::Tensor& block_table,
                                       const at::Tensor& q_start, const at::Tensor& q_len, const at::Tensor& kv_len,
                                       double scale, int64_t max_kv_len, int64_t splits, int64_t window,
                                       std::vector<at::Tensor>* parts, const c10::optional<at::Tensor>& counters = {}) {
  SXE_CHECK_CUDA(q);
  SXE_CHECK(q.scalar_type() == at::kBFloat16 && cache.scalar_type() == at::kBFloat16, "bf16 only");
  SXE_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == q.size(2), "q must be [T, nq, D] with head stride D");
  SXE_CHECK(cache.dim() == 5 && cache.is_contiguous(), "cache must be [blocks, 2, nkv, bs, D]");
  SXE_CHECK(block_table.scalar_type() == at::kInt && block_table.is_contiguous() && block_table.dim() == 2,
            "block_table int32 [S, max_blocks]");
  for (auto* t : {&q_start, &q_len, &kv_len})
    SXE_CHECK(t->scalar_type() == at::kInt && t->is_contiguous() && t->numel() == block_table.size(0),
              "q_start/q_len/kv_len: int32 [S]");
  const int T = q.size(0), nq = q.size(1), D = q.size(2);
  const int nkv = cache.size(2), bs = cache.size(3);
  SXE_CHECK(cache.size(4) == D && nq % nkv == 0, "head layout mismatch");
  const int S = block_table.size(0);
  auto out = at::empty({T, nq, D}, q.options());
  if (T == 0 || S == 0) return out;
  c10::DeviceGuard g(q.device());
  splits = std::max<int64_t>(1, splits);
  int64_t kps = (std::max<int64_t>(max_kv_len, 1) + splits - 1) / splits;
  kps = (kps + 63) / 64 * 64;  // whole wave chunks (64 keys; 32 at head dim 256)
  splits = (std::max<int64_t>(max_kv_len, 1) + kps - 1) / kps;
  at::Tensor part_o, part_ml;
  pa::Args a;
  a.q = reinterpret_cast<const unsigned short*>(q.data_ptr());
  a.q_tok_stride = q.stride(0);
  a.cache = reinterpret_cast<const unsigned short*>(cache.data_ptr());
  a.block_table = block_table.data_ptr<int>();
  a.max_blocks = block_table.size(1);
  a.q_start = q_start.data_ptr<int>();
  a.q_len = q_len.data_ptr<int>();
  a.kv_len = kv_len.data_ptr<int>();
  a.nq = nq;
  a.nkv = nkv;
  a.bs = bs;
  a.scale_log2 = (float)scale * pa::kLog2e;
  a.splits = (int)splits;
  a.keys_per_split = (int)kps;
  a.out = reinterpret_cast<unsigned short*>(out.data_ptr());
  a.out_tok_stride = out.stride(0);
  a.T = T;
  a.part_o = nullptr;
  a.part_ml = nullptr;
  a.window = (int)std::max<int64_t>(0, window);
  a.counters = nullptr;
  if (splits > 1 && parts == nullptr && counters.has_value()) {
    SXE_CHECK(counters->is_cuda() && counters->scalar_type() == at::kInt && counters->is_contiguous() &&
                  counters->numel() >= (int64_t)S * nkv,
              "paged_attention: counters int32 [>= S * nkv] on the device, zeroed");
    a.counters = counters->data_ptr<int>();
  }
  if (splits > 1) {
    part_o = at::empty({splits, T, nq, D}, q.options().dtype(at::kFloat));
    part_ml = at::empty({splits, T, nq, 2}, q.options().dtype(at::kFloat));
    a.part_o = part_o.data_ptr<float>();
    a.part_ml = part_ml.data_ptr<float>();
  }
  dim3 grid(S * nkv, splits);
  SXE_CHECK(D == 128 || D == 64 || D == 256, "paged_attention: head_dim must be 64, 128 or 256");
  static bool attr_set[3] = {false, false, false};
  auto launch = [&](void (*kern)(pa::Args), size_t lds, int slot) {
    if (!attr_set[slot]) {  // > 64 KiB of dynamic LDS must be opted into (gfx950: 160 KiB per CU)
      SXE_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr_set[slot] = true;
    }
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, cur_stream(), a);
  };
  if (D == 128) launch(pa::paged_attn_kernel<128>, pa::PaGeo<128>::LDS, 0);
  else if (D == 256) launch(pa::paged_attn_kernel<256>, pa::PaGeo<256>::LDS, 1);
  else launch(pa::paged_attn_kernel<64>, pa::PaGeo<64>::LDS, 2);
  SXE_LAUNCH_CHECK();
  if (splits > 1 && parts != nullptr) {
    *parts = {part_o, part_ml};
    return out;
  }
  if (splits > 1 && a.counters == nullptr) {
    if (D == 128)
      hipLaunchKernelGGL(pa::merge_kernel<128>, dim3(T * nq), dim3(128), 0, cur_stream(), a.part_o, a.part_ml,
                         (int)splits, T, nq, a.out, a.out_tok_stride);
    else if (D == 256)
      hipLaunchKernelGGL(pa::merge_kernel<256>, dim3(T * nq), dim3(256), 0, cur_stream(), a.part_o, a.part_ml,
                         (int)splits, T, nq, a.out, a.out_tok_stride);
    else
      hipLaunchKernelGGL(pa::merge_kernel<64>, dim3(T * nq), dim3(64), 0, cur_stream(), a.part_o, a.part_ml,
                         (int)splits, T, nq, a.out, a.out_tok_stride);
    SXE_LAUNCH_CHECK();
  }
  return out;
}

at::Tensor paged_attention(const at::Tensor& q, const at::Tensor& cache, const at::Tensor& block_table,
                           const at::Tensor& q_start, const at::Tensor& q_len, const at::Tensor& kv_len, double scale,
                           int64_t max_kv_len, int64_t splits, int64_t window, const c10::optional<at::Tensor>& counters) {
  return paged_attention_impl(q, cache, block_table, q_start, q_len, kv_len, scale, max_kv_len, splits, window, nullptr,
                              counters);
}

// [out, part_o, part_ml]: with one split `out` is the attention output and the partials are empty;
// with several, `out` is unwritten and the partials are returned unmerged
std::vector<at::Tensor> paged_attention_parts(const at::Tensor& q, const at::Tensor& cache,
                                              const at::Tensor& block_table, const at::Tensor& q_start,
                                              const at::Tensor& q_len, const at::Tensor& kv_len, double scale,
                                              int64_t max_kv_len, int64_t splits, int64_t window) {
  std::vector<at::Tensor> parts;
  auto out = paged_attention_impl(q, cache, block_table, q_start, q_len, kv_len, scale, max_kv_len, splits, window,
                                  &parts);
  if (parts.empty()) {
    auto e = at::empty({0}, q.options().dtype(at::kFloat));
    return {out, e, e};
  }
  return {out, parts[0], parts[1]};
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("kv_cache_append(Tensor qkv, Tensor(a!) cache, Tensor slots, int nq, int nkv) -> ()");
  m.def("rope_kv_cache_append(Tensor(a!) qkv, Tensor cos, Tensor sin, Tensor pos, Tensor(b!) cache, Tensor slots, "
        "int nq, int nkv) -> ()");
  m.def("paged_attention(Tensor q, Tensor cache, Tensor block_table, Tensor q_start, Tensor q_len, Tensor kv_len, "
        "float scale, int max_kv_len, int splits, int window=0, Tensor(a!)? counters=None) -> Tensor");
  m.def("paged_attention_parts(Tensor q, Tensor cache, Tensor block_table, Tensor q_start, Tensor q_len, "
        "Tensor kv_len, float scale, int max_kv_len, int splits, int window=0) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("kv_cache_append", &sxe::kv_cache_append);
  m.impl("rope_kv_cache_append", &sxe::rope_kv_cache_append);
  m.impl("paged_attention", &sxe::paged_attention);
  m.impl("paged_attention_parts", &sxe::paged_attention_parts);
}

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
//  * key phase: lane = key (K row in 16 B vector registers, q rows broadcast from LDS); value phase:
//    lane = 4 output dims of one of KG V rows per load instruction, the 64 rows' cache offsets
//    precomputed in the key phase so all V loads of a chunk are in flight together (a per-key
//    block-table lookup -> load chain made the value phase latency-bound); probabilities hop
//    through LDS; key-group partial sums fold once per pass with lane shuffles;
//  * flash-decoding split over the KV length when (sequences x kv heads) is too small to fill the
//    256 CUs, merged by a second kernel (fp32 partials);
//  * causal masking by absolute position (chunked prefill / speculative tokens just work).
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
  int* counters;   // [S * nkv] self-resetting split counters (nullptr: separate merge kernel)
  int T;
  int window;      // sliding window (Mistral / Qwen2): keys older than `window` positions are masked; 0 = off
};

// R = query rows (token x head-in-group) per pass: 4 / 8 / 16 picked on the host from the GQA group
// size so decode rows (q_len = 1) fill one pass without idle row slots.
template <int D, int R>
__global__ __launch_bounds__(256) void paged_attn_kernel(Args a) {
  constexpr int KV16 = D / 8;   // 16-byte vectors per K row
  constexpr int LPR = D / 4;    // value phase: lanes per V row (4 dims = 8 bytes each)
  constexpr int KG = 64 / LPR;  // V rows per wave load instruction
  __shared__ float q_lds[R][D];
  __shared__ float p_lds[kWaves][R][64];
  __shared__ int64_t voff_lds[kWaves][64];
  __shared__ float mrg_o[kWaves][R][D];
  __shared__ float mrg_ml[kWaves][R][2];

  const int seq = blockIdx.x / a.nkv, kvh = blockIdx.x - (blockIdx.x / a.nkv) * a.nkv;
  const int split = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kg = lane / LPR, dl = lane - (lane / LPR) * LPR;
  const int G = a.nq / a.nkv;
  const int qs = a.q_start[seq], ql = a.q_len[seq], kl = a.kv_len[seq];
  const int k_begin = split * a.keys_per_split;
  const int k_end = min(kl, k_begin + a.keys_per_split);
  const int nrows_total = ql * G;
  const int* bt = a.block_table + (int64_t)seq * a.max_blocks;
  const int64_t head_stride = (int64_t)a.bs * D;          // between kv heads inside a block half
  const int64_t half_stride = (int64_t)a.nkv * head_stride;  // k half -> v half
  const int64_t block_stride = 2 * half_stride;

  for (int row0 = 0; row0 < nrows_total; row0 += R) {
    const int nrows = min(R, nrows_total - row0);
    // ---- q rows -> LDS (fp32, pre-scaled by softmax scale * log2 e) -------------------------
    for (int i = threadIdx.x; i < R * D; i += 256) {
      const int r = i / D, d = i - r * D;
      float v = 0.f;
      if (r < nrows) {
        const int row = row0 + r, tok = row / G, g = row - tok * G;
        v = bf16_to_f32(a.q[(int64_t)(qs + tok) * a.q_tok_stride + (int64_t)(kvh * G + g) * D + d]) * a.scale_log2;
      }
      q_lds[r][d] = v;
    }
    __syncthreads();
    const int max_pos = kl - ql + (row0 + nrows - 1) / G;  // causal horizon of this tile
    const int k_hi = min(k_end, max_pos + 1);
    // sliding window: keys below the oldest row's window are masked for every row of the pass --
    // start at the 64-key chunk holding the first visible key (the waves keep their interleave)
    int k_start = k_begin;
    if (a.window > 0) {
      const int k_lo = kl - ql + row0 / G - a.window + 1;
      if (k_lo > k_begin) k_start = k_begin + ((k_lo - k_begin) / 64) * 64;
    }
    float m[R], l[R], acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      m[r] = -INFINITY;
      l[r] = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[r][e] = 0.f;
    }
    for (int kb = k_start + wave * 64; kb < k_hi; kb += kWaves * 64) {
      // q rows are re-read from LDS every chunk: without this fence LICM hoists all R x D of them
      // into registers (R = 4 alone would need 512 VGPRs and spill to scratch)
      asm volatile("" ::: "memory");
      // ---- key phase: lane = key; invalid lanes re-read key kb (in range) and get p = 0 ------
      const int key = kb + lane;
      const bool valid = key < k_hi;
      const int kc = valid ? key : kb;
      const int blk = bt[kc / a.bs], off = kc - (kc / a.bs) * a.bs;
      const int64_t koff = (int64_t)blk * block_stride + kvh * head_stride + (int64_t)off * D;
      voff_lds[wave][lane] = koff + half_stride;
      u16x8 kr[KV16];
#pragma unroll
      for (int v = 0; v < KV16; ++v) kr[v] = *reinterpret_cast<const u16x8*>(a.cache + koff + v * 8);
      float s[R];
#pragma unroll
      for (int r = 0; r < R; ++r) s[r] = 0.f;
#pragma unroll
      for (int v = 0; v < KV16; ++v) {
        float kf[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) kf[e] = bf16_to_f32(kr[v][e]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (r < nrows) {  // (uniform) guard also keeps the scheduler from hoisting all R x D q reads
            const f32x4 q0 = *reinterpret_cast<const f32x4*>(&q_lds[r][v * 8]);
            const f32x4 q1 = *reinterpret_cast<const f32x4*>(&q_lds[r][v * 8 + 4]);
            s[r] += q0[0] * kf[0] + q0[1] * kf[1] + q0[2] * kf[2] + q0[3] * kf[3] + q1[0] * kf[4] + q1[1] * kf[5] +
                    q1[2] * kf[6] + q1[3] * kf[7];
          }
        }
      }
      // ---- online softmax per row -----------------------------------------------------------
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < nrows) {
          const int pos = kl - ql + (row0 + r) / G;
          const bool vis = valid && key <= pos && (a.window <= 0 || key > pos - a.window);
          const float sv = vis ? s[r] : -INFINITY;
          const float mx = wave_max(sv);
          const float mn = fmaxf(m[r], mx);
          float p = 0.f, alpha = 1.f;
          if (mn != -INFINITY) {
            p = (sv == -INFINITY) ? 0.f : exp2f(sv - mn);
            alpha = (m[r] == -INFINITY) ? 0.f : exp2f(m[r] - mn);
          }
          l[r] = l[r] * alpha + wave_sum(p);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[r][e] *= alpha;
          m[r] = mn;
          p_lds[wave][r][lane] = p;
        } else {
          p_lds[wave][r][lane] = 0.f;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): p_lds / voff_lds visible within the wave
      __builtin_amdgcn_wave_barrier();
      // ---- value phase: KG V rows per load, lane = 4 dims of one row; all 64 rows issued
      //      back to back (offsets precomputed in the key phase, so no dependent block lookups) --
#pragma unroll 16
      for (int j0 = 0; j0 < 64; j0 += KG) {
        const int j = j0 + kg;
        const uint2 w = *reinterpret_cast<const uint2*>(a.cache + voff_lds[wave][j] + dl * 4);
        const float v0 = bf16_to_f32(w.x & 0xffff), v1 = bf16_to_f32(w.x >> 16);
        const float v2 = bf16_to_f32(w.y & 0xffff), v3 = bf16_to_f32(w.y >> 16);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float p = p_lds[wave][r][j];
          acc[r][0] += p * v0;
          acc[r][1] += p * v1;
          acc[r][2] += p * v2;
          acc[r][3] += p * v3;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    // ---- fold the KG key groups of each wave, then merge the 4 waves ---------------------------
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) acc[r][e] += __shfl_xor(acc[r][e], o, 64);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < nrows) {
        if (kg == 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) mrg_o[wave][r][dl * 4 + e] = acc[r][e];
        }
        if (lane == 0) {
          mrg_ml[wave][r][0] = m[r];
          mrg_ml[wave][r][1] = l[r];
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nrows * D; i += 256) {
      const int r = i / D, d = i - r * D;
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) M = fmaxf(M, mrg_ml[w][r][0]);
      float sum = 0.f, L = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const float mw = mrg_ml[w][r][0];
        const float f = (mw == -INFINITY) ? 0.f : exp2f(mw - M);
        sum += f * mrg_o[w][r][d];
        L += f * mrg_ml[w][r][1];
      }
      const int row = row0 + r, tok = row / G, g = row - tok * G;
      const int t = qs + tok, h = kvh * G + g;
      if (a.splits == 1) {
        a.out[(int64_t)t * a.out_tok_stride + (int64_t)h * D + d] = f32_to_bf16(L > 0.f ? sum / L : 0.f);
      } else {
        const int64_t idx = ((int64_t)split * a.T + t) * a.nq + h;
        a.part_o[idx * D + d] = sum;
        if (d == 0) {
          a.part_ml[idx * 2 + 0] = M;
          a.part_ml[idx * 2 + 1] = L;
        }
      }
    }
    __syncthreads();
  }
  // split-KV merge fused in: the LAST workgroup of (seq, kv head) to finish (device-scope counter,
  // release fence before / acquire fence after the vector atomic) combines every split's partial
  // o / (max, sum) for this sequence's rows and resets the counter for the next launch. No
  // workgroup waits on another, so there is nothing to deadlock on.
  if (a.splits > 1 && a.counters != nullptr) {
    __shared__ int is_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) is_last = atomicAdd(&a.counters[blockIdx.x], 1) == a.splits - 1;
    __syncthreads();
    if (is_last) {
      __threadfence();
      for (int i = threadIdx.x; i < nrows_total * D; i += 256) {
        const int row = i / D, d = i - row * D, tok = row / G, g = row - tok * G;
        const int64_t th = (int64_t)(qs + tok) * a.nq + kvh * G + g;
        float M = -INFINITY;
        for (int s = 0; s < a.splits; ++s) M = fmaxf(M, __builtin_nontemporal_load(&a.part_ml[((int64_t)s * a.T * a.nq + th) * 2]));
        float acc = 0.f, L = 0.f;
        for (int s = 0; s < a.splits; ++s) {
          const int64_t idx = (int64_t)s * a.T * a.nq + th;
          const float ms = __builtin_nontemporal_load(&a.part_ml[idx * 2]);
          if (ms == -INFINITY) continue;
          const float f = exp2f(ms - M);
          acc += f * __builtin_nontemporal_load(&a.part_o[idx * D + d]);
          L += f * __builtin_nontemporal_load(&a.part_ml[idx * 2 + 1]);
        }
        a.out[(int64_t)(qs + tok) * a.out_tok_stride + (int64_t)(kvh * G + g) * D + d] =
            f32_to_bf16(L > 0.f ? acc / L : 0.f);
      }
      if (threadIdx.x == 0) atomicExch(&a.counters[blockIdx.x], 0);
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void merge_kernel(const float* __restrict part_o, const float* __restrict part_ml,
                                                  int splits, int T, int nq, unsigned short* __restrict out,
                                                  int64_t out_tok_stride) {
  const int th = blockIdx.x;  // t * nq + h
  const int t = th / nq, h = th - t * nq;
  const int d = threadIdx.x;
  float M = -INFINITY;
  for (int s = 0; s < splits; ++s) M = fmaxf(M, part_ml[((int64_t)s * T * nq + th) * 2]);
  float acc = 0.f, L = 0.f;
  for (int s = 0; s < splits; ++s) {
    const int64_t idx = (int64_t)s * T * nq + th;
    const float ms = part_ml[idx * 2];
    if (ms == -INFINITY) continue;
    const float f = exp2f(ms - M);
    acc += f * part_o[idx * D + d];
    L += f * part_ml[idx * 2 + 1];
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

// q: [T, nq, D] (token stride free); returns out [T, nq, D] bf16
// Persistent, self-resetting per-(seq, kv head) split counters for the fused merge: allocated zeroed
// once per device OUTSIDE any stream capture (a buffer first allocated inside a HIP-graph capture
// would belong to the graph's pool); while capturing with too small a buffer, or without
// SXE_PA_FUSED_MERGE=1, the separate merge kernel runs instead.
static int* split_counters(const c10::Device& dev, int64_t need) {
  static at::Tensor buf[64];
  // opt-in: measured SLOWER than the separate merge kernel on Llama-3-8B decode (batch 1: 4.56 vs
  // 4.31 ms/token; batch 16: 7.90 vs 5.97 ms -- the device-scope release/acquire fences write back
  // and invalidate L2 per workgroup, and the merge serialises into one workgroup per head group)
  static const bool enabled = [] {
    const char* e = std::getenv("SXE_PA_FUSED_MERGE");
    return e && e[0] == '1';
  }();
  if (!enabled || dev.index() < 0 || dev.index() >= 64) return nullptr;
  at::Tensor& b = buf[dev.index()];
  if (b.defined() && b.numel() >= need) return b.data_ptr<int>();
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(cur_stream(), &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  b = at::zeros({std::max<int64_t>(need, 1 << 16)}, at::TensorOptions().device(dev).dtype(at::kInt));
  return b.data_ptr<int>();
}

at::Tensor paged_attention(const at::Tensor& q, const at::Tensor& cache, const at::Tensor& block_table,
                           const at::Tensor& q_start, const at::Tensor& q_len, const at::Tensor& kv_len, double scale,
                           int64_t max_kv_len, int64_t splits, int64_t window) {
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
  kps = (kps + 63) / 64 * 64;
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
  a.counters = nullptr;
  a.window = (int)std::max<int64_t>(0, window);
  if (splits > 1) {
    part_o = at::empty({splits, T, nq, D}, q.options().dtype(at::kFloat));
    part_ml = at::empty({splits, T, nq, 2}, q.options().dtype(at::kFloat));
    a.part_o = part_o.data_ptr<float>();
    a.part_ml = part_ml.data_ptr<float>();
    a.counters = split_counters(q.device(), S * nkv);
  }
  dim3 grid(S * nkv, splits);
  const int G = nq / nkv;
  SXE_CHECK(D == 128 || D == 64 || D == 256, "paged_attention: head_dim must be 64, 128 or 256");
#define SXE_PA_LAUNCH(DD, RR) hipLaunchKernelGGL((pa::paged_attn_kernel<DD, RR>), grid, dim3(256), 0, cur_stream(), a)
  if (D == 128) {
    if (G <= 4) SXE_PA_LAUNCH(128, 4);
    else if (G <= 8) SXE_PA_LAUNCH(128, 8);
    else SXE_PA_LAUNCH(128, 16);
  } else if (D == 256) {  // 64 lanes per V row: one row per load; R <= 8 keeps LDS + VGPRs in budget
    if (G <= 4) SXE_PA_LAUNCH(256, 4);
    else SXE_PA_LAUNCH(256, 8);
  } else {
    if (G <= 4) SXE_PA_LAUNCH(64, 4);
    else if (G <= 8) SXE_PA_LAUNCH(64, 8);
    else SXE_PA_LAUNCH(64, 16);
  }
#undef SXE_PA_LAUNCH
  SXE_LAUNCH_CHECK();
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

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  m.def("kv_cache_append(Tensor qkv, Tensor(a!) cache, Tensor slots, int nq, int nkv) -> ()");
  m.def("rope_kv_cache_append(Tensor(a!) qkv, Tensor cos, Tensor sin, Tensor pos, Tensor(b!) cache, Tensor slots, "
        "int nq, int nkv) -> ()");
  m.def("paged_attention(Tensor q, Tensor cache, Tensor block_table, Tensor q_start, Tensor q_len, Tensor kv_len, "
        "float scale, int max_kv_len, int splits, int window=0) -> Tensor");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("kv_cache_append", &sxe::kv_cache_append);
  m.impl("rope_kv_cache_append", &sxe::rope_kv_cache_append);
  m.impl("paged_attention", &sxe::paged_attention);
}

// Flash attention forward + backward for gfx950 (MI355X), bf16 in / fp32 accumulate, head dims 64,
// 128 and 256 (templated: no zero-padding of the head dim), causal or full, GQA, query length !=
// key length (cross / prefix / chunked-prefill attention: the causal mask is bottom-right aligned by
// `qoff`, query i sees keys <= i + qoff), arbitrary [B, S, H, D] strides (so the fused QKV projection
// output is read in place and dq/dk/dv are written straight into one dqkv buffer).
//
// Reference users: FPDT's chunked attention with LSE merging (deepspeed/sequence/fpdt_layer.py:134-460),
// Ulysses local attention (sequence/layer.py:434), the Triton flash kernels of the inference path
// (ops/transformer/inference/triton/attention.py:263, triton_ops.py:16) and the external
// flash-attn the FastGen blocked_flash op calls (inference/v2/kernels/ragged_ops/blocked_flash/).
//
// CDNA4 design (see /opt/skills/guides/cdna_hip_programming.md §3, §5.5 T2/T10/T12-T14, App. B):
//  * v_mfma_f32_32x32x16_bf16 everywhere; 64-wide waves; one wave owns 32 query rows (fwd, dQ)
//    or 32 key rows (dK/dV);
//  * "swapped" products: the forward computes S^T = K Q^T so one lane holds one query's scores
//    (softmax max/sum are lane-local + one lane^32 exchange, the rescale is a per-lane scalar),
//    and S^T is consumed directly as the B operand of O^T += V^T P^T (the accumulator-as-operand
//    identity of guide §3, with its permuted k order), so P never touches LDS;
//  * V^T / K^T / Q^T / dO^T operands come from row-major LDS tiles through ds_read_b64_tr_b16
//    (hardware transpose), with the XOR-swizzled 256-byte-row image that is conflict-free for
//    both the row reads (ds_read_b128) and the transposed reads (guide T10, image (b));
//  * K/V (or Q/dO) tiles are register-staged one tile ahead (T14 issue-early/write-late) into a
//    double-buffered LDS ring: one barrier per tile;
//  * backward = pre-pass (-delta = -rowsum(dO * O), lse * log2(e)) + dQ kernel (forward-shaped) +
//    dK/dV kernel (keys on lanes, dK^T/dV^T accumulated in registers across the GQA query heads): no
//    atomics, deterministic.
//  * heavy-first block order for the causal triangle.
#include "sxe_common.h"
#include <torch/library.h>
#include <type_traits>

namespace sxe {
namespace fa {

constexpr int NW = 4;           // waves per workgroup
constexpr int QW = 32;          // rows per wave
constexpr int QB = NW * QW;     // 128 rows per workgroup
constexpr int KT = 64;          // keys per K/V tile (forward / dQ)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Byte offset of 16-byte chunk `ch` (0..D/8-1) of row `row` in a swizzled [rows][D bf16] tile: the
// chunk index is XORed with a 4-bit function of the row (3 bits when a row has only 8 chunks) so
// both the row reads (ds_read_b128) and the transposed 4-row reads (ds_read_b64_tr_b16) spread over
// the banks (guide T10, image (b)); the XOR is an involution, which the direct-to-LDS loader uses.
template <int D>
__device__ __forceinline__ int soff(int row, int ch) {
  constexpr int CH = D / 8;
  const int f = (((row & 3) << 2) | ((row >> 2) & 3)) & (CH >= 16 ? 15 : CH - 1);
  return row * (2 * D) + 16 * (ch ^ f);
}

template <int D>
__device__ __forceinline__ bf16x8 lds_row16(const char* base, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(base + soff<D>(row, ch));
}

// Transposed read: 4 consecutive rows x one column per lane (ds_read_b64_tr_b16).
__device__ __forceinline__ i16x4 lds_tr(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(const_cast<char*>(base) + byte_off));
}

// A operand of a 32x32x16 MFMA taken from a row-major [rows][d] LDS tile, transposed:
// A[m = d][k] with d = 32*dt + (lane&31), k permuted to match an accumulator used as B operand:
// element j of lane half h <- tile row (row0 + 8*(j>>2) + 4h + (j&3)), column d.
template <int D>
__device__ __forceinline__ bf16x8 lds_trA(const char* base, int row0, int dt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const int row = row0 + 4 * h + q;
  i16x4 lo = lds_tr(base, soff<D>(row, ch) + 8 * (p & 1));
  i16x4 hi = lds_tr(base, soff<D>(row + 8, ch) + 8 * (p & 1));
  // whole-vector bitcast: element-wise bf16 inserts from the tr-read result miscompile (hipcc 7.2)
  const i16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

// Per-lane byte offsets of the two LDS read forms above, computed once per kernel: the swizzle only
// looks at the low 4 row bits, so for a tile row base row0 that is a multiple of 16
//   lds_row16(base, row0 + r, 2 t2 + h)  = base + 2D row0 + row[t2]
//   lds_trA(base, row0, dt, lane)        = tr_read(base + 2D row0, tr[dt][0], tr[dt][1])
// and every read in a tile loop is a hoisted VGPR plus an instruction immediate (recomputed per read,
// the XOR'd offsets cost ~40 VALU adds per forward tile).
template <int D>
struct LaneOffs {
  int row[D / 16];
  int tr[D / 32][2];
  __device__ __forceinline__ void init(int lane) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t2 = 0; t2 < D / 16; ++t2) row[t2] = soff<D>(r, 2 * t2 + h);
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, hh = g >> 1;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
      tr[dt][0] = soff<D>(4 * hh + q, ch) + 8 * (p & 1);
      tr[dt][1] = soff<D>(4 * hh + q + 8, ch) + 8 * (p & 1);
    }
  }
};
__device__ __forceinline__ bf16x8 lds_row_at(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}
__device__ __forceinline__ bf16x8 lds_tr_at(const char* base, const int (&o)[2]) {
  i16x4 lo = lds_tr(base, o[0]);
  i16x4 hi = lds_tr(base, o[1]);
  const i16x8 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

// Accumulator registers 8s..8s+7 -> bf16 B operand (k-step s of the accumulator-as-operand trick).
__device__ __forceinline__ bf16x8 acc_to_b(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)a[8 * s + e];
  return r;
}

// value of the lane 32 apart (lane ^ 32) via v_permlane32_swap: a VALU op instead of a
// ds_bpermute round trip through the LDS
__device__ __forceinline__ float xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// raw v_exp_f32: exp2f() wraps it in denormal range reduction, pure VALU overhead for softmax
// probabilities (a denormal p is 0 for every purpose here)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// accumulator register i <-> row offset within a 32x32 tile for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

struct Strides {
  int64_t b, s, h;  // element strides; d is unit stride
};

// Stage a [rows=ROWS][D] tile of 16-byte chunks from global into registers (each thread owns
// ROWS*(D/8)/threads chunks), then into swizzled LDS. Rows at or beyond `nrows_valid` read as zeros.
template <int ROWS, int NWAVES, int D>
struct Stager {
  static constexpr int CH = D / 8;
  static constexpr int N = ROWS * CH / (NWAVES * 64);
  u32x4 r[N];
  __device__ __forceinline__ void load(const unsigned short* base, int64_t row_stride, int row0, int nrows_valid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NWAVES * 64;
      const int row = c / CH, ch = c % CH;
      if (row0 + row < nrows_valid)
        r[i] = *reinterpret_cast<const u32x4*>(base + (int64_t)(row0 + row) * row_stride + ch * 8);
      else
        r[i] = u32x4{0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(char* lds) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = threadIdx.x + i * NWAVES * 64;
      *reinterpret_cast<u32x4*>(lds + soff<D>(c / CH, c % CH)) = r[i];
    }
  }
};


// Block-sparse attention (reference ops/sparse_attention: Triton SDD/DSD matmuls + block softmax):
// a uint8 layout [H, nb, nb] over blk x blk blocks (blk in {16, 32, 64, 128, ...}, a multiple of 16)
// says which (query block, key block) pairs exist. The kernels below walk only the K (or Q) tiles
// that intersect a non-zero block -- a compacted tile list built in LDS at kernel start -- and mask
// scores element-wise inside them, so compute and HBM traffic scale with the layout's density.
struct Sparse {
  const uint8_t* layout;  // nullptr = dense
  int blk, nb;
};

// Build the list of tiles [t_lo, t_hi) of `tile` rows along one axis whose block range intersects
// a non-zero block of rows [r_lo, r_hi) along the other axis; `q_axis_rows` says whether the fixed
// range is the query axis. Returns the count (also in list[-1]); all threads participate.
__device__ __forceinline__ int build_tile_list(const Sparse sp, int head, int t_lo, int t_hi, int tile, int r_lo,
                                               int r_hi, bool fixed_is_query, int* list) {
  int* flags = list + 1024;  // scratch after the list (t_hi - t_lo <= 1024)
  for (int t = t_lo + (int)threadIdx.x; t < t_hi; t += blockDim.x) {
    const int a0 = r_lo / sp.blk, a1 = (r_hi - 1) / sp.blk;
    const int b0 = (t * tile) / sp.blk, b1 = (t * tile + tile - 1) / sp.blk;
    int act = 0;
    for (int a = a0; a <= a1 && !act; ++a)
      for (int bb = b0; bb <= b1; ++bb) {
        const int qb_ = fixed_is_query ? a : bb, kb_ = fixed_is_query ? bb : a;
        if (sp.layout[((int64_t)head * sp.nb + qb_) * sp.nb + kb_]) { act = 1; break; }
      }
    flags[t - t_lo] = act;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int n = 0;
    for (int t = t_lo; t < t_hi; ++t)
      if (flags[t - t_lo]) list[n++] = t;
    list[-1] = n;
  }
  __syncthreads();
  return list[-1];
}

// Heavy-first mapping of the flat block index onto (b, head, row-block) for the causal triangle.
__device__ __forceinline__ void map_block(int nblk, int BH, bool heavy_last_index, int& bh, int& blk) {
  const int idx = blockIdx.x;
  const int rank = idx / BH;
  bh = idx - rank * BH;
  blk = heavy_last_index ? (nblk - 1 - rank) : rank;
}

// =============================================================================================
// Direct-to-LDS tile loads (global_load_lds_dwordx4): no staging registers. A wave-instruction
// writes 1 KiB = 1024 / (2 D) rows linearly, so the XOR swizzle goes on the per-lane SOURCE chunk
// (the swizzle is an involution: position c' of row `row` holds logical chunk c' ^ f(row)).
// =============================================================================================
//
// Issued from inline asm, not __builtin_amdgcn_global_load_lds: the compiler's wait-count pass
// cannot tell a builtin DMA's LDS writes from the ring's LDS reads, so it put an `s_waitcnt
// vmcnt(0)` before the first ds_read after every issue -- each dK/dV tile waited for the NEXT
// tile's load before its first MFMA (no prefetch at all), and dQ before its dQ MFMAs. Completion is
// tracked by hand instead: every consumer runs vm_wait_all() + a barrier before it reads a slot.
extern __shared__ __attribute__((aligned(16))) char smem[];  // every kernel's dynamic LDS
// M0 value of a wave-uniform pointer into smem: the symbol's LDS address plus the byte offset (a
// generic-to-LDS cast of the pointer itself costs a 64-bit null check per DMA instruction)
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem +
                                        (unsigned)(p - smem));
}
__device__ __forceinline__ void glds16(const void* gsrc, char* lds_wave_base) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds_addr(lds_wave_base)), "v"(gsrc)
               : "memory", "m0");
}
__device__ __forceinline__ void glds4(const void* gsrc, char* lds_wave_base) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(lds_addr(lds_wave_base)), "v"(gsrc)
               : "memory", "m0");
}
template <int ROWS, int D, int NWV = NW>
__device__ __forceinline__ void tile_glds(const unsigned short* base, int64_t row_stride, int row0, char* lds) {
  constexpr int CH = D / 8, RPK = 64 / CH;  // rows per 1 KiB wave-instruction
  static_assert(ROWS % (RPK * NWV) == 0, "tile rows must split evenly over the waves");
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < ROWS / RPK / NWV; ++i) {
    const int n = i * NWV + w;
    const int row = RPK * n + lane / CH;
    const int cpos = lane % CH;
    const int ch = cpos ^ ((((row & 3) << 2) | ((row >> 2) & 3)) & (CH >= 16 ? 15 : CH - 1));
    glds16(base + (int64_t)(row0 + row) * row_stride + ch * 8, lds + n * 1024);
  }
}
// s_waitcnt vmcnt(0) through the builtin (expcnt / lgkmcnt fields left at their maxima), not inline
// asm: the compiler's wait-count pass then knows every load it tracks has landed, so it does not
// keep counting the operand loads issued before a tile loop as pending inside the loop (where its
// counted waits would also wait for the hand-tracked LDS-DMA below)
__device__ __forceinline__ void vm_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }


// =============================================================================================
// Forward. Grid: (Sq / rows per workgroup) * B * H blocks. q: [B, Sq, *, D], k/v/o: [B, Sk, *, D]
// strided; lse [B, H, Sq]. Causal: query i sees keys <= i + qoff (qoff = Sk - Sq unless padded).
// =============================================================================================
// One K/V tile of a wave's online softmax. MASK = false is the interior-tile body (no causal
// diagonal, no padded tail, dense): none of the per-score compares / selects are emitted -- on
// the Llama-3 shape ~90 % of the tiles take it; the masked body handles the diagonal, the kv_len
// tail and block-sparse layouts.
template <bool MASK, int D>
__device__ __forceinline__ void fwd_tile(const LaneOffs<D>& lo, const char* kt, const char* vt, const bf16x8 (&qf)[D / 16],
                                         f32x16 (&oacc)[D / 32], float& m, float& l, float c, int kbase, int qpos,
                                         int r, int h, int lane, bool diag, bool tail, int kvlen, const uint8_t* lrow,
                                         int blk) {
  // causal diagonal tile whose second 32-key half lies entirely above this wave's last query
  // (the wave's queries start at the tile's first key): that half's QK^T and PV MFMAs are skipped
  const bool skip1 = MASK && diag && !tail && lrow == nullptr && kbase + 32 > qpos + QW - 1;
  f32x16 s[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    s[j] = zero16();
    if (j == 1 && skip1) break;
#pragma unroll
    for (int t2 = 0; t2 < D / 16; ++t2) s[j] = mfma(lds_row_at(kt + 32 * j * 2 * D, lo.row[t2]), qf[t2], s[j]);
  }
  // raw scores: the max is taken before scaling (c > 0) and the scale folds into the exp's FMA
  float mx = -INFINITY;
  // key - query offsets of this lane's first score row; opaque, so the compares below keep
  // compile-time row constants instead of 32 hoisted per-row thresholds per mask (VGPRs)
  int dd = kbase + 4 * h - qpos - r, dl = kbase + 4 * h - kvlen;
  if (MASK) asm volatile("" : "+v"(dd), "+v"(dl));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    bool b0 = true, b1 = true;  // layout bits of keys kbase+32j+[0,16) and +[16,32)
    if (MASK && lrow) {
      b0 = lrow[(kbase + 32 * j) / blk] != 0;
      b1 = lrow[(kbase + 32 * j + 16) / blk] != 0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float x = s[j][i];
      if (MASK) {
        if (diag && dd + 32 * j + acc_row(i, 0) > 0) x = -INFINITY;
        if (tail && dl + 32 * j + acc_row(i, 0) >= 0) x = -INFINITY;
        if (!(i < 8 ? b0 : b1)) x = -INFINITY;
        s[j][i] = x;
      }
      mx = fmaxf(mx, x);
    }
  }
  mx = fmaxf(mx, xor32(mx)) * c;
  // lazy rescale: the reference max only moves when the tile max exceeds it by > 2^8, so
  // p <= 256 (harmless in fp32 / bf16) and the O rescale is skipped whenever no lane of the wave
  // moved (most tiles after the first few)
  const bool grow = mx > m + 8.f;
  const float mnew = grow ? mx : m;
  const float mref = (mnew == -INFINITY) ? 0.f : mnew;
  const float alpha = fast_exp2(m - mref);
  float ps = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = fast_exp2(__builtin_fmaf(s[j][i], c, -mref));
      s[j][i] = p;
      ps += p;
    }
  l = l * alpha + ps;
  m = mnew;
  if (__any(grow)) {
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j == 1 && skip1) break;  // its p are all exp2(-inf) = 0
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = acc_to_b(s[j], s2);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
        oacc[dt] = mfma(lds_tr_at(vt + (32 * j + 16 * s2) * 2 * D, lo.tr[dt]), pb, oacc[dt]);
    }
  }
}

// Waves per workgroup (each 32 queries): NWF = 8 (256 queries; one workgroup of 2 waves per SIMD
// per CU) shares every staged K/V tile among twice the queries of NWF = 4, which serves sequences
// that are not a multiple of 256 and head dim 256 (whose accumulators need a whole SIMD's
// register file: 1 wave per SIMD).
template <int D, int NWF>
constexpr int fwd_min_waves() { return D >= 256 ? 1 : 8 / NWF; }

// DMA: K/V tiles go straight to LDS (global_load_lds from inline asm, see glds16) instead of through
// the register Stager; head dim 256 always (staging registers would not fit next to its 128
// accumulator + 64 Q-fragment registers), smaller head dims by default (SXE_FA_FWD_DMA=0 selects the
// register Stager: 4-7 % slower at D 128, B4 S2048 to B1 S32k, equal at D 64 --
// profiles/r05/attn_fwd_dma_ab.log)
template <bool SPARSE, int NWF, int D, bool DMA = (D >= 256)>
__global__ void __launch_bounds__(NWF * 64, (fwd_min_waves<D, NWF>())) fwd_kernel(
    const unsigned short* __restrict__ q, Strides qs, const unsigned short* __restrict__ k, Strides ks,
    const unsigned short* __restrict__ v, Strides vs, unsigned short* __restrict__ o, Strides os,
    float* __restrict__ lse, int B, int H, int Hk, int Sq, int Sk, float scale, int causal, Sparse sp, int kvlen,
    int qoff) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ROWB = 2 * D;
  constexpr int BUF = 2 * KT * ROWB;  // one ring slot = K tile + V tile
  int* tlist = reinterpret_cast<int*>(smem + 4 * KT * ROWB) + 1;
  constexpr int QBF = NWF * QW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int nqb = Sq / QBF;
  int bh, qb;
  map_block(nqb, B * H, causal != 0, bh, qb);
  const int b = bh / H, head = bh - b * H;
  const int kh = head / (H / Hk);
  const int q0 = qb * QBF + w * QW;  // this wave's first query
  const int qpos = q0 + qoff;        // its position on the key axis (causal diagonal)
  const unsigned short* qp = q + b * qs.b + head * qs.h;
  const unsigned short* kp = k + b * ks.b + kh * ks.h;
  const unsigned short* vp = v + b * vs.b + kh * vs.h;
  const float c = scale * LOG2E;

  bf16x8 qf[D / 16];
#pragma unroll
  for (int t = 0; t < D / 16; ++t)
    qf[t] = *reinterpret_cast<const bf16x8*>(qp + (int64_t)(q0 + r) * qs.s + 16 * t + 8 * h);

  f32x16 oacc[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) oacc[t] = zero16();
  float m = -INFINITY, l = 0.f;

  // keys needed by the workgroup (causal: up to its last query's diagonal)
  const int kend = causal ? min(Sk, (qb + 1) * QBF + qoff) : Sk;
  const int nkt = (max(kend, 0) + KT - 1) / KT;
  const int ntiles = SPARSE ? build_tile_list(sp, head, 0, nkt, KT, qb * QBF, qb * QBF + QBF, true, tlist) : nkt;
  auto tile_at = [&](int i) { return SPARSE ? tlist[i] : i; };
  const uint8_t* lrow = SPARSE ? sp.layout + ((int64_t)head * sp.nb + (q0 + r) / sp.blk) * sp.nb : nullptr;
  Stager<KT, NWF, D> sk, sv;
  const int t0 = ntiles > 0 ? tile_at(0) : 0;
  if constexpr (DMA) {
    if (ntiles > 0) {
      tile_glds<KT, D, NWF>(kp, ks.s, t0 * KT, smem);
      tile_glds<KT, D, NWF>(vp, vs.s, t0 * KT, smem + KT * ROWB);
    }
    vm_wait_all();
  } else {
    sk.load(kp, ks.s, t0 * KT, Sk);
    sv.load(vp, vs.s, t0 * KT, Sk);
    sk.store(smem);
    sv.store(smem + KT * ROWB);
  }
  __syncthreads();
  LaneOffs<D> lo;
  lo.init(lane);
  // the tile loop runs unrolled by two so the ring slot is a compile-time constant in each copy: every
  // LDS address is then a hoisted per-lane offset plus an instruction immediate (with a runtime slot
  // each K / V read paid a VALU add per tile -- ~50 of the interior tile's ~200 VALU instructions)
  auto step = [&](const int t, auto slot) {
    constexpr int CUR = decltype(slot)::value;
    const bool more = (t + 1) < ntiles;
    if (more) {
      if constexpr (DMA) {
        tile_glds<KT, D, NWF>(kp, ks.s, tile_at(t + 1) * KT, smem + (CUR ^ 1) * BUF);
        tile_glds<KT, D, NWF>(vp, vs.s, tile_at(t + 1) * KT, smem + (CUR ^ 1) * BUF + KT * ROWB);
      } else {
        sk.load(kp, ks.s, tile_at(t + 1) * KT, Sk);
        sv.load(vp, vs.s, tile_at(t + 1) * KT, Sk);
      }
    }
    const int kbase = tile_at(t) * KT;
    // a wave whose queries all precede this tile has nothing to add (causal)
    const bool active = !causal || kbase <= qpos + QW - 1;
    if (active) {
      const char* kt = smem + CUR * BUF;
      const char* vt = kt + KT * ROWB;
      const bool diag = causal && (kbase + KT - 1 > qpos);
      const bool tail = kbase + KT > kvlen;  // keys past the valid length (padded key axis)
      if (SPARSE || diag || tail)
        fwd_tile<true, D>(lo, kt, vt, qf, oacc, m, l, c, kbase, qpos, r, h, lane, diag, tail, kvlen, lrow,
                          SPARSE ? sp.blk : 1);
      else
        fwd_tile<false, D>(lo, kt, vt, qf, oacc, m, l, c, kbase, qpos, r, h, lane, false, false, kvlen, nullptr, 1);
    }
    if constexpr (DMA) {
      vm_wait_all();
    } else if (more) {
      sk.store(smem + (CUR ^ 1) * BUF);
      sv.store(smem + (CUR ^ 1) * BUF + KT * ROWB);
    }
    __syncthreads();
  };
  for (int t = 0; t < ntiles; t += 2) {
    step(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) step(t + 1, std::integral_constant<int, 1>{});
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;  // a fully masked row outputs zeros
  unsigned short* op = o + b * os.b + head * os.h + (int64_t)(q0 + r) * os.s;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      u16x4 pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) pk[e] = f32_to_bf16(oacc[dt][4 * rg + e] * inv);
      *reinterpret_cast<u16x4*>(op + 32 * dt + 8 * rg + 4 * h) = pk;
    }
  if (h == 0) lse[((int64_t)b * H + head) * Sq + q0 + r] = lt > 0.f ? (m + log2f(lt)) * LN2 : INFINITY;
}

// =============================================================================================
// Backward pre-pass, per (batch, head, query) row: -delta = -sum_d dO * O and lse * log2(e) (fp32),
// D/8 threads per row. (Computing delta inside the dQ kernel instead -- it holds the dO rows --
// measured neutral: the dQ prologue's extra O load cost what the launch saved.)
// =============================================================================================
template <int D>
__global__ void __launch_bounds__(256) delta_kernel(const unsigned short* __restrict__ dout, Strides ds,
                                                    const unsigned short* __restrict__ o, Strides os,
                                                    const float* __restrict__ lse, float* __restrict__ ndelta,
                                                    float* __restrict__ lse2, int B, int H, int S) {
  constexpr int TPR = D / 8, RPB = 256 / TPR;
  const int64_t row = (int64_t)blockIdx.x * RPB + (threadIdx.x / TPR);
  const int part = threadIdx.x % TPR;
  if (row >= (int64_t)B * H * S) return;
  const int s = (int)(row % S);
  const int64_t bh = row / S;
  const int hh = (int)(bh % H), b = (int)(bh / H);
  float x[8], y[8];
  load8<DT::BF16>(dout + b * ds.b + hh * ds.h + (int64_t)s * ds.s + part * 8, x);
  load8<DT::BF16>(o + b * os.b + hh * os.h + (int64_t)s * os.s + part * 8, y);
  float acc = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc += x[e] * y[e];
#pragma unroll
  for (int off = TPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, TPR);
  if (part == 0) {
    ndelta[row] = -acc;
    lse2[row] = lse[row] * LOG2E;
  }
}

template <int D>
constexpr int bwd_min_waves() { return D >= 256 ? 1 : 2; }

// =============================================================================================
// dQ: forward-shaped. Per wave 32 queries; per K/V tile recompute S^T, P^T, dP^T = V dO^T,
// dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T.
// =============================================================================================
template <bool MASK, int D>
__device__ __forceinline__ void dq_tile(const LaneOffs<D>& lo, const char* kt, const char* vt, const bf16x8 (&qf)[D / 16],
                                        const bf16x8 (&df)[D / 16], f32x16 (&dqacc)[D / 32], float c, float lse2,
                                        float ndlt, int kbase, int qpos, int r, int h, int lane, bool diag, bool tail,
                                        int kvlen, const uint8_t* lay_row, int blk) {
  int dd = kbase + 4 * h - qpos - r, dl = kbase + 4 * h - kvlen;  // see fwd_tile
  if (MASK) asm volatile("" : "+v"(dd), "+v"(dl));
  const bool skip1 = MASK && diag && !tail && lay_row == nullptr && kbase + 32 > qpos + QW - 1;  // see fwd_tile
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j == 1 && skip1) break;
    f32x16 s = zero16(), dp = zero16();
#pragma unroll
    for (int t2 = 0; t2 < D / 16; ++t2) {
      s = mfma(lds_row_at(kt + 32 * j * 2 * D, lo.row[t2]), qf[t2], s);
      dp = mfma(lds_row_at(vt + 32 * j * 2 * D, lo.row[t2]), df[t2], dp);
    }
    bool b0 = true, b1 = true;
    if (MASK && lay_row) {
      b0 = lay_row[(kbase + 32 * j) / blk] != 0;
      b1 = lay_row[(kbase + 32 * j + 16) / blk] != 0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = fast_exp2(__builtin_fmaf(s[i], c, -lse2));
      if (MASK) {
        if (diag && dd + 32 * j + acc_row(i, 0) > 0) p = 0.f;
        if (tail && dl + 32 * j + acc_row(i, 0) >= 0) p = 0.f;
        if (!(i < 8 ? b0 : b1)) p = 0.f;
      }
      s[i] = p * (dp[i] + ndlt);  // dS^T (ndlt = -delta)
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 db = acc_to_b(s, s2);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
        dqacc[dt] = mfma(lds_tr_at(kt + (32 * j + 16 * s2) * 2 * D, lo.tr[dt]), db, dqacc[dt]);
    }
  }
}

// NWF waves per workgroup, 32 queries each: 8 (256 queries) shares every staged K/V tile among twice
// the queries of 4 -- half the L2-to-LDS tile traffic per query, at one workgroup per CU
// (SXE_FA_DQ_WAVES, read per call; Sq a multiple of 256, head dims 64 / 128)
template <bool SPARSE, int D, int NWF = 4>
__global__ void __launch_bounds__(NWF * 64, (NWF == 8 ? 1 : bwd_min_waves<D>())) dq_kernel(
    const unsigned short* __restrict__ q, Strides qs, const unsigned short* __restrict__ k, Strides ks,
    const unsigned short* __restrict__ v, Strides vs, const unsigned short* __restrict__ dout, Strides dos,
    const float* __restrict__ lse, const float* __restrict__ ndelta, unsigned short* __restrict__ dq, Strides dqs,
    int B, int H, int Hk, int Sq, int Sk, float scale, int causal, Sparse sp, int kvlen, int qoff) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ROWB = 2 * D;
  constexpr int BUF = 2 * KT * ROWB;
  int* tlist = reinterpret_cast<int*>(smem + 4 * KT * ROWB) + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  constexpr int QBF = NWF * QW;
  const int nqb = Sq / QBF;
  int bh, qb;
  map_block(nqb, B * H, causal != 0, bh, qb);
  const int b = bh / H, head = bh - b * H;
  const int kh = head / (H / Hk);
  const int q0 = qb * QBF + w * QW;
  const int qpos = q0 + qoff;
  const unsigned short* qp = q + b * qs.b + head * qs.h;
  const unsigned short* dop = dout + b * dos.b + head * dos.h;
  const unsigned short* kp = k + b * ks.b + kh * ks.h;
  const unsigned short* vp = v + b * vs.b + kh * vs.h;
  const float c = scale * LOG2E;
  const int64_t lrow = ((int64_t)b * H + head) * Sq + q0 + r;
  const int kend = causal ? min(Sk, (qb + 1) * QBF + qoff) : Sk;
  const int nkt = (max(kend, 0) + KT - 1) / KT;
  const int ntiles = SPARSE ? build_tile_list(sp, head, 0, nkt, KT, qb * QBF, qb * QBF + QBF, true, tlist) : nkt;
  auto tile_at = [&](int i) { return SPARSE ? tlist[i] : i; };
  const uint8_t* lay_row = SPARSE ? sp.layout + ((int64_t)head * sp.nb + (q0 + r) / sp.blk) * sp.nb : nullptr;
  if (ntiles > 0) {
    tile_glds<KT, D, NWF>(kp, ks.s, tile_at(0) * KT, smem);
    tile_glds<KT, D, NWF>(vp, vs.s, tile_at(0) * KT, smem + KT * ROWB);
  }

  const float lse2 = lse[lrow] * LOG2E;
  bf16x8 qf[D / 16], df[D / 16];
#pragma unroll
  for (int t = 0; t < D / 16; ++t) {
    qf[t] = *reinterpret_cast<const bf16x8*>(qp + (int64_t)(q0 + r) * qs.s + 16 * t + 8 * h);
    df[t] = *reinterpret_cast<const bf16x8*>(dop + (int64_t)(q0 + r) * dos.s + 16 * t + 8 * h);
  }
  const float ndlt = ndelta[lrow];
  f32x16 dqacc[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) dqacc[t] = zero16();
  vm_wait_all();
  // pin the Q / dO fragments and row constants as loaded before the loop (see dkdv_kernel)
#pragma unroll
  for (int t = 0; t < D / 16; ++t) asm volatile("" ::"v"(qf[t]), "v"(df[t]));
  asm volatile("" ::"v"(lse2), "v"(ndlt));
  __syncthreads();
  LaneOffs<D> lo;
  lo.init(lane);
  // unrolled by two: compile-time ring slot, hoisted LDS offsets (see fwd_kernel)
  auto step = [&](const int t, auto slot) {
    constexpr int CUR = decltype(slot)::value;
    if (t + 1 < ntiles) {
      tile_glds<KT, D, NWF>(kp, ks.s, tile_at(t + 1) * KT, smem + (CUR ^ 1) * BUF);
      tile_glds<KT, D, NWF>(vp, vs.s, tile_at(t + 1) * KT, smem + (CUR ^ 1) * BUF + KT * ROWB);
    }
    const int kbase = tile_at(t) * KT;
    const bool active = !causal || kbase <= qpos + QW - 1;
    if (active) {
      const char* kt = smem + CUR * BUF;
      const char* vt = smem + CUR * BUF + KT * ROWB;
      const bool diag = causal && (kbase + KT - 1 > qpos);
      const bool tail = kbase + KT > kvlen;
      if (SPARSE || diag || tail)
        dq_tile<true, D>(lo, kt, vt, qf, df, dqacc, c, lse2, ndlt, kbase, qpos, r, h, lane, diag, tail, kvlen,
                         lay_row, SPARSE ? sp.blk : 1);
      else
        dq_tile<false, D>(lo, kt, vt, qf, df, dqacc, c, lse2, ndlt, kbase, qpos, r, h, lane, false, false, kvlen,
                          nullptr, 1);
    }
    vm_wait_all();
    __syncthreads();
  };
  for (int t = 0; t < ntiles; t += 2) {
    step(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) step(t + 1, std::integral_constant<int, 1>{});
  }
  unsigned short* op = dq + b * dqs.b + head * dqs.h + (int64_t)(q0 + r) * dqs.s;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      u16x4 pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) pk[e] = f32_to_bf16(dqacc[dt][4 * rg + e] * scale);
      *reinterpret_cast<u16x4*>(op + 32 * dt + 8 * rg + 4 * h) = pk;
    }
}

// =============================================================================================
// dK, dV: per wave 32 keys held on the lanes; sweep every query head of the GQA group and every
// 32-query tile at or after the keys (causal). Q/dO tiles + LSE/delta arrive by LDS-DMA into a
// 2-slot ring; the workgroup's V block (128 keys) sits in LDS for the whole kernel (V fragments in
// registers too would exceed the VGPR budget and spill); K fragments, dK^T and dV^T live in
// registers.
// =============================================================================================
constexpr int QT = 32;  // queries per tile in the dK/dV sweep
template <int D, int KB = QB> struct KVL {
  static constexpr int TILE = QT * 2 * D;              // one Q (or dO) tile
  static constexpr int SLOT = 2 * TILE + 2 * QT * 4;   // Q, dO, lse[32], delta[32]
  static constexpr int VBLK = KB * 2 * D;              // the V block of KB keys
};

// PART: 3 = dK and dV in one sweep; 1 = dV only; 2 = dK only (head dim 256: the two 128-register
// accumulators of one sweep would spill, so two sweeps each recompute S = Q K^T)
template <bool MASK, int D, int PART>
__device__ __forceinline__ void dkdv_tile(const LaneOffs<D>& lo, const char* slot, const char* vblk,
                                          const bf16x8 (&kf)[D / 16],
                                          f32x16 (&dka)[D / 32], f32x16 (&dva)[D / 32], float c, int qt0, int k0,
                                          int w, int r, int h, int lane, bool diag, const Sparse& sp, int hq0,
                                          int kbl, int qoff) {
  const char* qt = slot;
  const char* dt_ = slot + KVL<D>::TILE;
  const float* l2 = reinterpret_cast<const float*>(slot + 2 * KVL<D>::TILE);
  const float* dl = l2 + QT;
  f32x16 s = zero16(), dp = zero16();
#pragma unroll
  for (int t2 = 0; t2 < D / 16; ++t2) {
    s = mfma(lds_row_at(qt, lo.row[t2]), kf[t2], s);  // S  [query][key]
    if constexpr ((PART & 2) != 0)
      dp = mfma(lds_row_at(dt_, lo.row[t2]), lds_row_at(vblk + w * QW * 2 * D, lo.row[t2]), dp);  // dP
  }
  bool b0 = true, b1 = true;  // layout bits of query rows qt0+[0,16) and qt0+[16,32) vs this key
  if (MASK && sp.layout) {
    b0 = sp.layout[((int64_t)hq0 * sp.nb + qt0 / sp.blk) * sp.nb + kbl] != 0;
    b1 = sp.layout[((int64_t)hq0 * sp.nb + (qt0 + 16) / sp.blk) * sp.nb + kbl] != 0;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = fast_exp2(__builtin_fmaf(s[i], c, -l2[acc_row(i, h)]));  // P; l2 = lse log2(e)
  // masks under wave-uniform (scalar) branches: interior tiles -- most of them -- run no per-score
  // compares / selects (`diag` and the layout pointer are SGPR values; see the readfirstlane of w)
  if (MASK && diag) {
    int dd = k0 + r - 4 * h - qt0 - qoff;  // masked iff key > query + qoff, i.e. dd > row(i, 0)
    asm volatile("" : "+v"(dd));            // keep the per-row compares against constants (see fwd_tile)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (dd > acc_row(i, 0)) s[i] = 0.f;
  }
  if (MASK && sp.layout) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!(acc_row(i, h) < 16 ? b0 : b1)) s[i] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) dp[i] = s[i] * (dp[i] + dl[acc_row(i, h)]);  // dS = P (dP - delta); dl = -delta
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const bf16x8 pb = acc_to_b(s, s2);
    const bf16x8 db = acc_to_b(dp, s2);
#pragma unroll
    for (int t = 0; t < D / 32; ++t) {
      if constexpr ((PART & 1) != 0) dva[t] = mfma(lds_tr_at(dt_ + 16 * s2 * 2 * D, lo.tr[t]), pb, dva[t]);  // dV^T
      if constexpr ((PART & 2) != 0) dka[t] = mfma(lds_tr_at(qt + 16 * s2 * 2 * D, lo.tr[t]), db, dka[t]);   // dK^T
    }
  }
}

// SPLIT (GQA): one workgroup per (batch, group of `hpw` QUERY heads, key block) instead of per KV
// head: under a causal mask the KV-head form gives key block 0 G x (Sq/128) query tiles while the
// mean block has half of that, and with B*Hk*Sk/128 ~ 2 workgroups per CU the whole launch waits for
// block 0 (measured 650 us at B4 S2048 H32/8). Splitting the G query heads into G/hpw groups cuts the
// longest job by G/hpw; the per-group fp32 dK/dV partials [B, Sk, H/hpw, D] are summed by
// dkdv_reduce_kernel (hpw = 2 halves that partial traffic against hpw = 1).
// NWK waves per workgroup, 32 keys each: 8 (256 keys, head dim 128; SXE_FA_DKDV_WAVES, read per
// call) shares every staged Q / dO tile among twice the keys of 4 -- half the L2-to-LDS traffic per
// key, at one workgroup per CU
template <bool SPLIT, int D, int PART = 3, int NWK = 4>
__global__ void __launch_bounds__(NWK * 64, (NWK == 8 ? 1 : bwd_min_waves<D>())) dkdv_kernel(
    const unsigned short* __restrict__ q, Strides qs, const unsigned short* __restrict__ k, Strides ks,
    const unsigned short* __restrict__ v, Strides vs, const unsigned short* __restrict__ dout, Strides dos,
    const float* __restrict__ lse, const float* __restrict__ delta, unsigned short* __restrict__ dk, Strides dks,
    unsigned short* __restrict__ dv, Strides dvs, float* __restrict__ pk, float* __restrict__ pv, int B, int H,
    int Hk, int Sq, int Sk, float scale, int causal, Sparse sp, int qoff, int hpw) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KB = NWK * QW;  // keys per workgroup
  using G_ = KVL<D, KB>;
  char* vblk = smem;
  char* ring = smem + G_::VBLK;
  int* tlist = reinterpret_cast<int*>(ring + 2 * G_::SLOT) + 1;
  // w via readfirstlane: the compiler then knows it (and k0, the causal `diag` test) is wave-uniform,
  // so the diagonal mask is a scalar branch rather than per-lane selects on every tile
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), r = lane & 31,
            h = lane >> 5;
  const int nkb = Sk / KB;
  int bh, kb;
  const int G = SPLIT ? hpw : H / Hk;  // query heads swept by this workgroup (sparse: 1)
  const int HB = H / G;                 // workgroups along the head axis
  map_block(nkb, B * HB, false, bh, kb);  // key block 0 is the heaviest under causality
  const int b = bh / HB, hsel = bh - b * HB;
  const int hq0 = hsel * G;             // first query head swept by this workgroup
  const int kh = hq0 / (H / Hk);
  const int k0 = kb * KB + w * QW;  // this wave's first key
  const unsigned short* kp = k + b * ks.b + kh * ks.h;
  const unsigned short* vp = v + b * vs.b + kh * vs.h;
  const float c = scale * LOG2E;
  // causal: the first query that sees key block kb (query i sees keys <= i + qoff)
  const int qstart = causal ? min(Sq, max(0, kb * KB - qoff) / QT * QT) : 0;
  const int ntq = (Sq - qstart) / QT;
  // sparse: SPLIT mode (G == 1), list of the active 32-query tiles of this key block
  const int total = sp.layout ? build_tile_list(sp, hq0, qstart / QT, Sq / QT, QT, kb * KB, kb * KB + KB, false, tlist)
                              : ntq * G;
  const int kbl = sp.layout ? (k0 + r) / sp.blk : 0;
  // dense tile order: the query tiles qstart .. Sq of head hq0, then of hq0 + 1, ... -- walked by
  // incremented iterators (a runtime `it % ntq` / `it / ntq` per tile was a scalar division
  // sequence, a third of the kernel's instructions as SALU)
  int is_h = hq0, is_q = qstart;  // next tile to issue
  int c_q = qstart;               // tile being computed
  auto issue = [&](int it, char* slot) {
    const int hq = sp.layout ? hq0 : is_h;
    const int qt0 = sp.layout ? tlist[it] * QT : is_q;
    if (!sp.layout) {
      is_q += QT;
      if (is_q >= Sq) {
        is_q = qstart;
        ++is_h;
      }
    }
    tile_glds<QT, D, NWK>(q + b * qs.b + hq * qs.h, qs.s, qt0, slot);
    tile_glds<QT, D, NWK>(dout + b * dos.b + hq * dos.h, dos.s, qt0, slot + G_::TILE);
    if (w == 0) {  // 64 lanes x 4 B: lse[32] then delta[32]
      const int64_t lr = ((int64_t)b * H + hq) * Sq + qt0 + (lane & 31);
      glds4(lane < 32 ? (const void*)(lse + lr) : (const void*)(delta + lr), slot + 2 * G_::TILE);
    }
  };
  if constexpr ((PART & 2) != 0) tile_glds<KB, D, NWK>(vp, vs.s, kb * KB, vblk);
  if (total > 0) issue(0, ring);
  bf16x8 kf[D / 16];
#pragma unroll
  for (int t = 0; t < D / 16; ++t)
    kf[t] = *reinterpret_cast<const bf16x8*>(kp + (int64_t)(k0 + r) * ks.s + 16 * t + 8 * h);
  f32x16 dka[D / 32], dva[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t) {
    dka[t] = zero16();
    dva[t] = zero16();
  }
  vm_wait_all();
  // pin the K fragments as loaded before the loop: left to itself the compiler sinks their loads
  // below the barrier, and its counted waits for them inside the loop then also wait on the
  // hand-tracked LDS-DMA of the next tile
#pragma unroll
  for (int t = 0; t < D / 16; ++t) asm volatile("" ::"v"(kf[t]));
  __syncthreads();
  LaneOffs<D> lo;
  lo.init(lane);
  // unrolled by two: compile-time ring slot, hoisted LDS offsets (see fwd_kernel)
  auto step = [&](const int it, auto slotc) {
    constexpr int CUR = decltype(slotc)::value;
    const int qt0 = sp.layout ? tlist[it] * QT : c_q;
    c_q = c_q + QT >= Sq ? qstart : c_q + QT;
    const bool active = !causal || (qt0 + QT - 1 + qoff >= k0);
    const bool diag = causal && (qt0 + qoff < k0 + QW);
    if (it + 1 < total) issue(it + 1, ring + (CUR ^ 1) * G_::SLOT);
    if (active)
      dkdv_tile<true, D, PART>(lo, ring + CUR * G_::SLOT, vblk, kf, dka, dva, c, qt0, k0, w, r, h, lane, diag, sp,
                               hq0, kbl, qoff);
    vm_wait_all();
    __syncthreads();
  };
  for (int it = 0; it < total; it += 2) {
    step(it, std::integral_constant<int, 0>{});
    if (it + 1 < total) step(it + 1, std::integral_constant<int, 1>{});
  }
  if (SPLIT && pk != nullptr) {  // fp32 partials, layout [B, Sk, H / hpw, D] contiguous
    float* kp32 = pk + (((int64_t)b * Sk + k0 + r) * HB + hsel) * D;
    float* vp32 = pv + (((int64_t)b * Sk + k0 + r) * HB + hsel) * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        f32x4 a, cc;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dka[t][4 * rg + e] * scale;
          cc[e] = dva[t][4 * rg + e];
        }
        if constexpr ((PART & 2) != 0) *reinterpret_cast<f32x4*>(kp32 + 32 * t + 8 * rg + 4 * h) = a;
        if constexpr ((PART & 1) != 0) *reinterpret_cast<f32x4*>(vp32 + 32 * t + 8 * rg + 4 * h) = cc;
      }
    return;
  }
  unsigned short* kop = dk + b * dks.b + kh * dks.h + (int64_t)(k0 + r) * dks.s;
  unsigned short* vop = dv + b * dvs.b + kh * dvs.h + (int64_t)(k0 + r) * dvs.s;
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      u16x4 pk4, pv4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pk4[e] = f32_to_bf16(dka[t][4 * rg + e] * scale);
        pv4[e] = f32_to_bf16(dva[t][4 * rg + e]);
      }
      if constexpr ((PART & 2) != 0) *reinterpret_cast<u16x4*>(kop + 32 * t + 8 * rg + 4 * h) = pk4;
      if constexpr ((PART & 1) != 0) *reinterpret_cast<u16x4*>(vop + 32 * t + 8 * rg + 4 * h) = pv4;
    }
}


// dk[b, s, kh, :] = sum_g pk[b, s, kh*G + g, :] (dv likewise) over the G = H / Hk partial groups of
// each KV head (H here = the partial count, query heads / hpw); one thread per 8 output elements.
template <int D>
__global__ void __launch_bounds__(256) dkdv_reduce_kernel(const float* __restrict__ pk, const float* __restrict__ pv,
                                                          unsigned short* __restrict__ dk, Strides dks,
                                                          unsigned short* __restrict__ dv, Strides dvs, int B, int S,
                                                          int H, int Hk) {
  const int G = H / Hk;
  const int64_t n8 = (int64_t)B * S * Hk * (D / 8);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % (D / 8)) * 8;
    const int64_t rest = i / (D / 8);
    const int kh = (int)(rest % Hk);
    const int64_t bs = rest / Hk;  // b * S + s
    const int b = (int)(bs / S), s_ = (int)(bs - (int64_t)b * S);
    float ak[8] = {0, 0, 0, 0, 0, 0, 0, 0}, av[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = 0; g < G; ++g) {
      const int64_t off = (bs * H + kh * G + g) * D + c;
      float x[8], y[8];
      load8<DT::F32>(pk + off, x);
      load8<DT::F32>(pv + off, y);
#pragma unroll
      for (int e = 0; e < 8; ++e) { ak[e] += x[e]; av[e] += y[e]; }
    }
    store8<DT::BF16>(dk + b * dks.b + (int64_t)s_ * dks.s + kh * dks.h + c, ak);
    store8<DT::BF16>(dv + b * dvs.b + (int64_t)s_ * dvs.s + kh * dvs.h + c, av);
  }
}

}  // namespace fa

// ---------------------------------------------------------------------------------------------
static fa::Strides strides_of(const at::Tensor& t) {
  return fa::Strides{t.stride(0), t.stride(1), t.stride(2)};
}

// q: [B, Sq, Hq, D]; k, v: [B, Sk, Hk, D]; D in {64, 128, 256}; Sq, Sk multiples of 128
static void check_qkv(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  SXE_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "flash_attn: tensors must be [B, S, H, D]");
  SXE_CHECK(q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 && v.scalar_type() == at::kBFloat16,
            "flash_attn: bf16 only");
  const int64_t D = q.size(3);
  SXE_CHECK(D == 64 || D == 128 || D == 256, "flash_attn: head dim must be 64, 128 or 256");
  SXE_CHECK(k.size(3) == D && v.size(3) == D, "flash_attn: q/k/v head dims differ");
  SXE_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1, "flash_attn: unit stride on D");
  SXE_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0), "flash_attn: q/k/v shapes");
  SXE_CHECK(q.size(2) % k.size(2) == 0, "flash_attn: Hq must be a multiple of Hkv");
  SXE_CHECK(q.size(1) % fa::QB == 0 && k.size(1) % fa::QB == 0, "flash_attn: seq lengths must be multiples of 128");
  for (const at::Tensor* t : {&q, &k, &v})
    SXE_CHECK((t->stride(1) % 8) == 0 && (t->stride(2) % 8) == 0 && (t->stride(0) % 8) == 0 &&
                  (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "flash_attn: 16-byte aligned rows required");
}

static fa::Sparse sparse_of(const c10::optional<at::Tensor>& layout, int64_t block, const at::Tensor& q) {
  if (!layout.has_value() || !layout->defined()) return fa::Sparse{nullptr, 0, 0};
  const at::Tensor& L = *layout;
  const int S = q.size(1), H = q.size(2);
  SXE_CHECK(L.is_cuda() && L.scalar_type() == at::kByte && L.is_contiguous() && L.dim() == 3, "layout: uint8 [H, nb, nb]");
  SXE_CHECK(block >= 16 && block % 16 == 0 && S % block == 0, "layout block must be a multiple of 16 dividing seq_len");
  SXE_CHECK(L.size(0) == H && L.size(1) == S / block && L.size(2) == S / block, "layout shape must be [H, S/block, S/block]");
  SXE_CHECK(S / fa::KT <= 1024, "sparse attention: seq_len <= 65536");
  return fa::Sparse{L.data_ptr<uint8_t>(), (int)block, (int)(S / block)};
}

constexpr size_t kListBytes = (1 + 2048) * sizeof(int) + 16;  // tile list + scratch flags (sparse mode)

// Kernel-variant knob, read on every call (not cached at static init) so a test or an A/B run can
// switch variants inside one process: SXE_FA_FWD_WAVES=4 forces the 4-wave forward.
static int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e != nullptr && *e != 0) ? std::atoi(e) : dflt;
}
// 4-wave forward workgroups only when forced (SXE_FA_FWD_WAVES=4): 8 waves are equal or faster on
// every measured shape -- causal equal at head dims 64 / 128, non-causal 3-7 % faster
// (profiles/r05/attn_fwd_waves_ab.log, attn_fwd_waves_d64_ab.log; one earlier box showed 4 waves
// 6 % ahead at D64 causal, which a second box did not reproduce)
static bool fwd_narrow(int D) {
  (void)D;
  return env_int("SXE_FA_FWD_WAVES", 8) == 4;
}
static bool fwd_dma() { return env_int("SXE_FA_FWD_DMA", 1) != 0; }

template <typename F>
static void set_lds_limit(F* f, size_t bytes) {
  SXE_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)bytes));
}

// kv_len: valid keys (the rest of the padded key axis is masked); qoff: causal offset (query i sees
// keys <= i + qoff), default Sk - Sq (bottom-right aligned)
template <int D>
static std::vector<at::Tensor> fwd_impl_d(at::Tensor q, at::Tensor k, at::Tensor v, bool causal, double scale,
                                          fa::Sparse sp, int kvlen, int qoff) {
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1), Hk = k.size(2);
  auto o = at::empty({B, Sq, H, D}, q.options());
  auto lse = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  constexpr int ROWB = 2 * D;
  const size_t lds = 4 * fa::KT * ROWB + (sp.layout ? kListBytes : 0);
  static bool attr = false;
  if (!attr) {
    const size_t mx = 4 * fa::KT * ROWB + kListBytes;
    set_lds_limit(&fa::fwd_kernel<false, 4, D>, mx);
    set_lds_limit(&fa::fwd_kernel<true, 4, D>, mx);
    if constexpr (D < 256) {
      set_lds_limit(&fa::fwd_kernel<false, 8, D>, mx);
      set_lds_limit(&fa::fwd_kernel<true, 8, D>, mx);
      set_lds_limit(&fa::fwd_kernel<false, 4, D, true>, mx);
      set_lds_limit(&fa::fwd_kernel<true, 4, D, true>, mx);
      set_lds_limit(&fa::fwd_kernel<false, 8, D, true>, mx);
      set_lds_limit(&fa::fwd_kernel<true, 8, D, true>, mx);
    }
    attr = true;
  }
  // 8 waves share each staged K/V tile when the query axis allows; head dim 256 runs 4 (register budget)
  const bool wide = D < 256 && Sq % 256 == 0 && !fwd_narrow(D);
  const int grid = (Sq / fa::QB) * B * H;
  auto launch = [&](auto kern, int nwf) {
    hipLaunchKernelGGL(kern, dim3(nwf == 8 ? grid / 2 : grid), dim3(nwf * 64), lds, cur_stream(),
                       reinterpret_cast<const unsigned short*>(q.data_ptr()), strides_of(q),
                       reinterpret_cast<const unsigned short*>(k.data_ptr()), strides_of(k),
                       reinterpret_cast<const unsigned short*>(v.data_ptr()), strides_of(v),
                       reinterpret_cast<unsigned short*>(o.data_ptr()), strides_of(o), lse.data_ptr<float>(), B, H, Hk,
                       Sq, Sk, (float)scale, causal ? 1 : 0, sp, kvlen, qoff);
  };
  if constexpr (D < 256) {
    if (fwd_dma()) {
      if (wide)
        sp.layout ? launch(fa::fwd_kernel<true, 8, D, true>, 8) : launch(fa::fwd_kernel<false, 8, D, true>, 8);
      else
        sp.layout ? launch(fa::fwd_kernel<true, 4, D, true>, 4) : launch(fa::fwd_kernel<false, 4, D, true>, 4);
      SXE_LAUNCH_CHECK();
      return {o, lse};
    }
    if (wide) {
      sp.layout ? launch(fa::fwd_kernel<true, 8, D>, 8) : launch(fa::fwd_kernel<false, 8, D>, 8);
      SXE_LAUNCH_CHECK();
      return {o, lse};
    }
  }
  sp.layout ? launch(fa::fwd_kernel<true, 4, D>, 4) : launch(fa::fwd_kernel<false, 4, D>, 4);
  SXE_LAUNCH_CHECK();
  return {o, lse};
}

static std::vector<at::Tensor> fwd_impl(at::Tensor q, at::Tensor k, at::Tensor v, bool causal, double scale,
                                        fa::Sparse sp, int64_t kv_len = -1, int64_t causal_offset = INT64_MIN) {
  check_qkv(q, k, v);
  const int Sq = q.size(1), Sk = k.size(1);
  const int kvlen = kv_len < 0 ? Sk : (int)kv_len;
  SXE_CHECK(kvlen >= 1 && kvlen <= Sk, "flash_attn: kv_len must be in [1, Sk]");
  const int qoff = causal_offset == INT64_MIN ? Sk - Sq : (int)causal_offset;
  SXE_CHECK(!sp.layout || (Sq == Sk && qoff == 0), "block-sparse attention needs Sq == Sk");
  c10::DeviceGuard guard(q.device());
  switch (q.size(3)) {
    case 64: return fwd_impl_d<64>(q, k, v, causal, scale, sp, kvlen, qoff);
    case 256: return fwd_impl_d<256>(q, k, v, causal, scale, sp, kvlen, qoff);
    default: return fwd_impl_d<128>(q, k, v, causal, scale, sp, kvlen, qoff);
  }
}

template <int D>
static void bwd_impl_d(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse,
                       at::Tensor dq, at::Tensor dk, at::Tensor dv, bool causal, double scale, fa::Sparse sp,
                       int kvlen, int qoff) {
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1), Hk = k.size(2);
  constexpr int ROWB = 2 * D;
  using G_ = fa::KVL<D>;
  auto ndelta = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  auto lse2 = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  const int64_t rows = (int64_t)B * H * Sq;
  constexpr int RPB = 256 / (D / 8);
  hipLaunchKernelGGL(fa::delta_kernel<D>, dim3((rows + RPB - 1) / RPB), dim3(256), 0, cur_stream(),
                     reinterpret_cast<const unsigned short*>(dout.data_ptr()), strides_of(dout),
                     reinterpret_cast<const unsigned short*>(o.data_ptr()), strides_of(o), lse.data_ptr<float>(),
                     ndelta.data_ptr<float>(), lse2.data_ptr<float>(), B, H, Sq);
  SXE_LAUNCH_CHECK();
  const size_t lds_dq = 4 * fa::KT * ROWB + (sp.layout ? kListBytes : 0);
  const size_t lds_kv_max = G_::VBLK + 2 * G_::SLOT + kListBytes;
  static bool attr_set = false;
  if (!attr_set) {  // > 64 KiB of dynamic LDS must be opted into (gfx950 has 160 KiB per CU)
    set_lds_limit(&fa::dq_kernel<false, D>, 4 * fa::KT * ROWB + kListBytes);
    set_lds_limit(&fa::dq_kernel<true, D>, 4 * fa::KT * ROWB + kListBytes);
    if constexpr (D < 256) {
      set_lds_limit(&fa::dq_kernel<false, D, 8>, 4 * fa::KT * ROWB + kListBytes);
      set_lds_limit(&fa::dq_kernel<true, D, 8>, 4 * fa::KT * ROWB + kListBytes);
    }
    set_lds_limit(&fa::dkdv_kernel<false, D>, lds_kv_max);
    set_lds_limit(&fa::dkdv_kernel<true, D>, lds_kv_max);
    if constexpr (D == 128) {
      const size_t mx8 = fa::KVL<D, 256>::VBLK + 2 * G_::SLOT + kListBytes;
      set_lds_limit(&fa::dkdv_kernel<false, D, 3, 8>, mx8);
      set_lds_limit(&fa::dkdv_kernel<true, D, 3, 8>, mx8);
    }
    if constexpr (D >= 256) {
      set_lds_limit(&fa::dkdv_kernel<false, D, 1>, lds_kv_max);
      set_lds_limit(&fa::dkdv_kernel<true, D, 1>, lds_kv_max);
      set_lds_limit(&fa::dkdv_kernel<false, D, 2>, lds_kv_max);
      set_lds_limit(&fa::dkdv_kernel<true, D, 2>, lds_kv_max);
    }
    attr_set = true;
  }
  // 8-wave dQ workgroups from 8k queries on (auto; SXE_FA_DQ_WAVES=4 / 8 forces): 1.5-2 % faster
  // fwd+bwd at S8k / S32k, neutral at 2k (profiles/r05/attn_bwd_waves_ab.log)
  const int dqw = env_int("SXE_FA_DQ_WAVES", 0);
  const bool dq8 = D < 256 && Sq % 256 == 0 && (dqw == 8 || (dqw == 0 && Sq >= 8192));
  auto* dqk = sp.layout ? fa::dq_kernel<true, D> : fa::dq_kernel<false, D>;
  if constexpr (D < 256) {
    if (dq8) dqk = sp.layout ? fa::dq_kernel<true, D, 8> : fa::dq_kernel<false, D, 8>;
  }
  hipLaunchKernelGGL(dqk, dim3((Sq / (dq8 ? 2 * fa::QB : fa::QB)) * B * H),
                     dim3(dq8 ? 512 : 256), lds_dq, cur_stream(),
                     reinterpret_cast<const unsigned short*>(q.data_ptr()), strides_of(q),
                     reinterpret_cast<const unsigned short*>(k.data_ptr()), strides_of(k),
                     reinterpret_cast<const unsigned short*>(v.data_ptr()), strides_of(v),
                     reinterpret_cast<const unsigned short*>(dout.data_ptr()), strides_of(dout),
                     lse.data_ptr<float>(), ndelta.data_ptr<float>(),
                     reinterpret_cast<unsigned short*>(dq.data_ptr()), strides_of(dq), B, H, Hk, Sq, Sk, (float)scale,
                     causal ? 1 : 0, sp, kvlen, qoff);
  SXE_LAUNCH_CHECK();
  // sparse: always one workgroup per query head (per-head tile lists); with GQA the per-head fp32
  // partials are reduced; causal GQA: split to remove the key-block-0 tail (see dkdv_kernel)
  // query heads per dK/dV workgroup in the split form (a divisor of the GQA group; sparse: 1). Auto
  // (SXE_FA_DKDV_HPW unset / 0): the largest divisor whose heaviest workgroup -- key block 0 sweeps
  // hpw x Sq/32 query tiles under the causal mask -- still fits the mean load of the 2 x CUs
  // workgroup slots (hpw <= B H nkb / (4 CUs)), and at most 2 from 8k keys on, where the partials'
  // traffic no longer matters and the balance does. Measured fwd+bwd (H32/8 D128 causal; 1 / 2 / 4
  // heads per workgroup): B8 S2048 1.88 / 1.76 / 1.69 ms, B4 S2048 0.84 / 0.76 / 0.88, B1 S32k
  // 36.4 / 36.2 / 37.3; B1 S32k H4/1 4.75 / 6.14 / 9.15 (profiles/r05/attn_dkdv_hpw_sweep.log)
  int hpw = sp.layout != nullptr ? 1 : env_int("SXE_FA_DKDV_HPW", 0);
  if (hpw == 0) {
    int64_t cap = (int64_t)B * H * (Sk / fa::QB) / (4 * kNumCUs);
    if (Sk >= 8192 && cap > 2) cap = 2;
    for (int d = H / Hk; d >= 1; --d)
      if ((H / Hk) % d == 0 && d <= cap) {
        hpw = d;
        break;
      }
  }
  if (hpw < 1 || (H / Hk) % hpw != 0) hpw = 1;
  const bool split = sp.layout != nullptr || (causal && H / Hk > hpw);
  const bool partials = split && H / hpw > Hk;
  const int np = H / hpw;  // partial head groups
  // head dim 256: dV and dK in one sweep (S once, 256 accumulators, a few spilled registers; default)
  // or two (SXE_FA_DKDV_ONE_SWEEP=0: PART 1 / 2, each recomputes S): one sweep is 1-9 % faster
  // fwd+bwd (profiles/r05/attn_d256_one_sweep_ab.log)
  const bool one_sweep = D >= 256 && env_int("SXE_FA_DKDV_ONE_SWEEP", 1) != 0;
  // head dim 128: 8-wave dK/dV workgroups of 256 keys (SXE_FA_DKDV_WAVES=8, read per call)
  // (auto from 8k keys on, as the dQ kernel; SXE_FA_DKDV_WAVES=4 / 8 forces)
  const int kvw = env_int("SXE_FA_DKDV_WAVES", 0);
  const bool kv8 = D == 128 && Sk % 256 == 0 && (kvw == 8 || (kvw == 0 && Sk >= 8192));
  const size_t lds_kv = (kv8 ? fa::KVL<D, 256>::VBLK : G_::VBLK) + 2 * G_::SLOT + (sp.layout ? kListBytes : 0);
  at::Tensor pk, pv;
  if (partials) {
    pk = at::empty({B, Sk, np, D}, q.options().dtype(at::kFloat));
    pv = at::empty({B, Sk, np, D}, q.options().dtype(at::kFloat));
  }
  auto launch = [&](auto kern, int heads, int nwk = 4) {
    hipLaunchKernelGGL(kern, dim3((Sk / (nwk * fa::QW)) * B * heads), dim3(nwk * 64), lds_kv, cur_stream(),
                       reinterpret_cast<const unsigned short*>(q.data_ptr()), strides_of(q),
                       reinterpret_cast<const unsigned short*>(k.data_ptr()), strides_of(k),
                       reinterpret_cast<const unsigned short*>(v.data_ptr()), strides_of(v),
                       reinterpret_cast<const unsigned short*>(dout.data_ptr()), strides_of(dout),
                       lse2.data_ptr<float>(), ndelta.data_ptr<float>(),
                       reinterpret_cast<unsigned short*>(dk.data_ptr()), strides_of(dk),
                       reinterpret_cast<unsigned short*>(dv.data_ptr()), strides_of(dv),
                       partials ? pk.data_ptr<float>() : nullptr, partials ? pv.data_ptr<float>() : nullptr, B, H, Hk,
                       Sq, Sk, (float)scale, causal ? 1 : 0, sp, qoff, hpw);
  };
  // the dK/dV launch(es) of one form: SPLIT = one workgroup per query-head group (partials / direct)
  auto run_dkdv = [&](auto splitc, int heads) {
    constexpr bool SP = decltype(splitc)::value;
    if constexpr (D >= 256) {
      if (!one_sweep) {
        launch(fa::dkdv_kernel<SP, D, 1>, heads);
        SXE_LAUNCH_CHECK();
        launch(fa::dkdv_kernel<SP, D, 2>, heads);
        return;
      }
    }
    if constexpr (D == 128) {
      if (kv8) {
        launch(fa::dkdv_kernel<SP, D, 3, 8>, heads, 8);
        return;
      }
    }
    launch(fa::dkdv_kernel<SP, D>, heads);
  };
  if (split) {
    run_dkdv(std::true_type{}, np);
    SXE_LAUNCH_CHECK();
    if (partials) {
      const int64_t n8 = (int64_t)B * Sk * Hk * (D / 8);
      hipLaunchKernelGGL(fa::dkdv_reduce_kernel<D>, dim3(stream_grid(n8, 256)), dim3(256), 0, cur_stream(),
                         pk.data_ptr<float>(), pv.data_ptr<float>(), reinterpret_cast<unsigned short*>(dk.data_ptr()),
                         strides_of(dk), reinterpret_cast<unsigned short*>(dv.data_ptr()), strides_of(dv), B, Sk, np,
                         Hk);
    }
  } else {
    run_dkdv(std::false_type{}, Hk);
  }
  SXE_LAUNCH_CHECK();
}

// dq/dk/dv are caller-provided (possibly strided views of one dqkv buffer).
static void bwd_impl(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse,
                     at::Tensor dq, at::Tensor dk, at::Tensor dv, bool causal, double scale, fa::Sparse sp,
                     int64_t kv_len = -1, int64_t causal_offset = INT64_MIN) {
  check_qkv(q, k, v);
  check_qkv(dq, dk, dv);
  const int Sq = q.size(1), Sk = k.size(1);
  const int kvlen = kv_len < 0 ? Sk : (int)kv_len;
  SXE_CHECK(kvlen >= 1 && kvlen <= Sk, "flash_attn_bwd: kv_len must be in [1, Sk]");
  const int qoff = causal_offset == INT64_MIN ? Sk - Sq : (int)causal_offset;
  SXE_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && dout.stride(3) == 1 && o.stride(3) == 1,
            "flash_attn_bwd: dout/o shapes");
  SXE_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "flash_attn_bwd: grad shapes");
  SXE_CHECK(lse.is_contiguous() && lse.size(2) == Sq, "flash_attn_bwd: lse [B, H, Sq]");
  c10::DeviceGuard guard(q.device());
  switch (q.size(3)) {
    case 64: return bwd_impl_d<64>(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, sp, kvlen, qoff);
    case 256: return bwd_impl_d<256>(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, sp, kvlen, qoff);
    default: return bwd_impl_d<128>(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, sp, kvlen, qoff);
  }
}

static int64_t offset_arg(int64_t causal_offset) { return causal_offset == -(int64_t(1) << 40) ? INT64_MIN : causal_offset; }

std::vector<at::Tensor> flash_attn_fwd(at::Tensor q, at::Tensor k, at::Tensor v, bool causal, double scale,
                                       int64_t kv_len, int64_t causal_offset) {
  return fwd_impl(q, k, v, causal, scale, fa::Sparse{nullptr, 0, 0}, kv_len, offset_arg(causal_offset));
}

void flash_attn_bwd(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse,
                    at::Tensor dq, at::Tensor dk, at::Tensor dv, bool causal, double scale, int64_t kv_len,
                    int64_t causal_offset) {
  bwd_impl(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, fa::Sparse{nullptr, 0, 0}, kv_len,
           offset_arg(causal_offset));
}

std::vector<at::Tensor> flash_attn_fwd_sparse(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor layout,
                                              int64_t block, bool causal, double scale) {
  return fwd_impl(q, k, v, causal, scale, sparse_of(layout, block, q));
}

void flash_attn_bwd_sparse(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse,
                           at::Tensor dq, at::Tensor dk, at::Tensor dv, at::Tensor layout, int64_t block, bool causal,
                           double scale) {
  bwd_impl(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, sparse_of(layout, block, q));
}

}  // namespace sxe

TORCH_LIBRARY_FRAGMENT(sxe, m) {
  // causal_offset: query i sees keys <= i + causal_offset; the default sentinel means Sk - Sq
  m.def("flash_attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale, int kv_len=-1, "
        "int causal_offset=-1099511627776) -> Tensor[]");
  m.def("flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, "
        "Tensor(c!) dv, bool causal, float scale, int kv_len=-1, int causal_offset=-1099511627776) -> ()");
  m.def("flash_attn_fwd_sparse(Tensor q, Tensor k, Tensor v, Tensor layout, int block, bool causal, float scale) -> Tensor[]");
  m.def("flash_attn_bwd_sparse(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor(a!) dq, "
        "Tensor(b!) dk, Tensor(c!) dv, Tensor layout, int block, bool causal, float scale) -> ()");
}
TORCH_LIBRARY_IMPL(sxe, CUDA, m) {
  m.impl("flash_attn_fwd", &sxe::flash_attn_fwd);
  m.impl("flash_attn_bwd", &sxe::flash_attn_bwd);
  m.impl("flash_attn_fwd_sparse", &sxe::flash_attn_fwd_sparse);
  m.impl("flash_attn_bwd_sparse", &sxe::flash_attn_bwd_sparse);
}

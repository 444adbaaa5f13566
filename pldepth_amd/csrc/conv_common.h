// Shared pieces of the implicit-GEMM convolution kernels (conv_igemm.hip: exact fp32 MFMA;
// conv_x3.hip: fp32 through three bf16 MFMA products): the GEMM view of one NHWC convolution,
// buffer-descriptor operand fetch, the fused input prologue and the accumulator epilogue.
#pragma once
#include "common.h"

namespace pld {

enum ConvMode { MODE_FWD = 0, MODE_WGRAD = 1 };

// One NHWC convolution seen as C[M][N] = A[M][K] . B[K][N]:
//   FWD   : m = (img,oy,ox), n = co, k = (ty,tx,ci); A = im2col(x1 ++ x2), B = Wn^T ([N][K])
//   DGRAD : FWD on (dY, flipped filter), output columns routed to dx1 / dx2 at `split`
//   WGRAD : m = (ty,tx,ci), n = co, k = (img,oy,ox) pixels; A = im2col^T, B = dY ([K][N])
struct GemmConvParams {
  const float* x1;
  const float* x2;
  int c1, c2, C;
  int n, h, w, kh, kw, sh, sw, pt, pl, oh, ow;
  const float* in_scale;
  const float* in_shift;
  int in_act;
  const float* bmat;    // FWD: Wn [N][K]; WGRAD: dY [K][N]
  const float* bsplit;  // FWD, bf16x3 kernel only: Wn pre-split (pld_filter_split) or NULL
  int M, N, K;
  const float* bias;
  float* out1;
  int ld1, acc1;
  float* out2;
  int ld2, acc2, split;
  long zstride;
  int ktiles_per_split;
  FastDiv dC, dKW, dOW, dOH;
  // bf16x3 FWD/DGRAD K-step order: 0 = linear in k = (tap, ci); > 0 = tap-inner, K-step
  // (chunk, tap) covers 32 channels of ONE source at one tap: kc1 = ceil(c1/32) chunks of x1,
  // then ceil(c2/32) of x2 (kc_tap in all) — one load per element instead of one per source,
  // and consecutive steps re-read the same channels at shifted taps (L2 hits)
  int kc_tap, kc1;
  FastDiv dTaps;
  // BatchNorm batch statistics of the stored output (FWD, unsplit, overwrite, no routing):
  // fp64 (sum, sum of squares) per output channel and per wave row tile, channel-major
  // [N][stats_parts][2], stats_parts = M tiles x (BM / wave rows); NULL = off
  double* stats;
  int stats_parts;
  // bf16x3 tile-stream schedule (conv_x3_kernel, sk_nk > 0): a 1-D grid of G workgroups walks
  // the (tile, K-step) space tile-major, tile t = (mb = t / sk_nnb, nb = t % sk_nnb), sk_nk
  // K-steps per tile. sk_align = 1: workgroup w owns whole tiles [w T/G, (w+1) T/G) (T =
  // sk_tiles); 0: steps [w S/G, (w+1) S/G) (S = T sk_nk), a tile cut between workgroups leaves
  // raw fp32 partial sums in sk_slab ([G][2][BM][BN]: a workgroup's first, then last tile) that
  // pld's stream fixup kernel sums in K order and stores through the epilogue.
  int sk_nk, sk_tiles, sk_nnb, sk_align;
  float* sk_slab;
  int sk_q;  // steps per cut unit of a non-aligned range (0 / 1: any step)
  // halo kernel grid order: 0 = N tiles fastest (the M tile's band shared in L2), 1 = M tiles
  // fastest (the N panel of the filter shared in L2: filters larger than an XCD's L2)
  int raster;
  // tile-stream tile order (halo kernel): sk_perm = P > 1 maps stream tile t to tile
  // (t % P) Q + t / P over the first P Q tiles (Q = sk_tiles / P); 0 / 1: identity (sk_tile)
  int sk_perm;
};

// the tile at stream position t. With workgroup ranges about P tiles long, P-way interleaving
// puts consecutive workgroups — one XCD's, which run together — on neighbouring tiles (whose
// input bands overlap in that XCD's L2) instead of P tiles apart
__host__ __device__ inline int sk_tile(const GemmConvParams& p, int t) {
  if (p.sk_perm <= 1) return t;
  const int q = p.sk_tiles / p.sk_perm;
  return t < q * p.sk_perm ? (t % p.sk_perm) * q + t / p.sk_perm : t;
}

// first global step of workgroup w of G in the tile-stream schedule (GemmConvParams sk_*)
// XCD-aware workgroup order: workgroups are dealt round-robin to the 8 XCDs (flat ids b, b + 8,
// ... share one), so virtual id = the flat id's slot in a contiguous run per XCD. Bijective on
// [0, nwg); neighbouring virtual ids (which share operands) meet in one XCD's L2.
__device__ __forceinline__ int xcd_order(int flat, int nwg) {
  const int xcd = flat & 7, slot = flat >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
}

// (sk_q > 1: non-aligned ranges cut on multiples of sk_q steps — the halo kernel's chunks)
__host__ __device__ inline long sk_begin(const GemmConvParams& p, long w, long G) {
  if (p.sk_align) return (w * p.sk_tiles / G) * p.sk_nk;
  const long q = p.sk_q > 1 ? p.sk_q : 1;
  return (w * ((long)p.sk_tiles * p.sk_nk / q) / G) * q;
}
// the workgroup whose range holds global step s (non-aligned schedule)
__host__ __device__ inline long sk_owner(const GemmConvParams& p, long s, long G) {
  const long q = p.sk_q > 1 ? p.sk_q : 1;
  return ((s / q + 1) * G - 1) / ((long)p.sk_tiles * p.sk_nk / q);
}

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---- operand fetch: raw buffer loads through wave-uniform descriptors. An out-of-range offset
// (OOB) returns zeros, so padding taps, ragged tiles and the idle source of a concat need no
// branch around the load.
constexpr unsigned OOB = 0x80000000u;
constexpr long MAX_RECORDS = 0x7FFFFFF0L;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, long bytes) {
  const int n = (int)(bytes < MAX_RECORDS ? (bytes > 0 ? bytes : 0) : MAX_RECORDS);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, n, 0x00020000);
}

__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 prologue4(int act, float4 v, float4 s, float4 t) {
  return make_float4(act_fwd(act, v.x * s.x + t.x), act_fwd(act, v.y * s.y + t.y),
                     act_fwd(act, v.z * s.z + t.z), act_fwd(act, v.w * s.w + t.w));
}

// the BN statistics partial of a wave's accumulators (store_acc's layout; p.stats set)
template <int TM, int TN>
__device__ __forceinline__ void acc_stats(const GemmConvParams& p, const floatx16 (&acc)[TM][TN],
                                          int m_w, int n_w, int lane) {
  const int h = lane >> 5, l32 = lane & 31;
  // per column: this wave's rows summed in fp64 (the lane's 16 x TM rows, then the other half
  // wave's through a cross-half swap); lanes 0-31 own one column each. Written for every wave
  // row tile (zeros past M), so the finalize reads stats_parts whole slots per channel.
  const int part = m_w / (TM * 32);
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = n_w + b * 32 + l32;
    const float bias = (p.bias && col < p.N) ? p.bias[col] : 0.f;
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m_w + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const double v = row < p.M ? (double)(acc[a][b][r] + bias) : 0.0;
        s += v;
        q += v * v;
      }
    s += __shfl_xor(s, 32);
    q += __shfl_xor(q, 32);
    if (h == 0 && col < p.N)
      *reinterpret_cast<double2*>(p.stats + ((long)col * p.stats_parts + part) * 2) =
          make_double2(s, q);
  }
}

// ---- staged epilogue (round 4): whole float4 column quads only (N, split, leading dims in 4s,
// 16-byte bases), no split-K slab
__device__ __forceinline__ bool staged_ok(const GemmConvParams& p) {
  return p.zstride == 0 && (p.N & 3) == 0 && (p.split >= p.N || (p.split & 3) == 0) &&
         (p.ld1 & 3) == 0 && (reinterpret_cast<uintptr_t>(p.out1) & 15) == 0 &&
         (p.split >= p.N ||
          ((p.ld2 & 3) == 0 && (reinterpret_cast<uintptr_t>(p.out2) & 15) == 0));
}

// A wave's TM x TN accumulators (+ bias, routing, accumulate) through its private LDS region
// `buf` of 32 x (32 TN + 8) floats, one 32-row sub-tile at a time: written in the MFMA C layout,
// read back as row-contiguous float4, stored as 16-byte streaming (nt) stores. The caller
// guarantees that no other wave touches `buf` any more (after the K loop's last barrier).
template <int TM, int TN>
__device__ __forceinline__ void store_acc_staged(const GemmConvParams& p,
                                                 const floatx16 (&acc)[TM][TN], int m_w, int n_w,
                                                 int lane, float* buf) {
  constexpr int WTN = TN * 32, LD = WTN + 8, Q = WTN / 4, IT = 32 * Q / 64;
  static_assert(IT >= 1 && (32 * Q) % 64 == 0, "whole float4 passes");
  const int h = lane >> 5, l32 = lane & 31;
  float bias[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = n_w + b * 32 + l32;
    bias[b] = (p.bias && col < p.N) ? p.bias[col] : 0.f;
  }
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[a][b][r];  // (through a scalar: see store_partial)
        buf[((r & 3) + 8 * (r >> 2) + 4 * h) * LD + b * 32 + l32] = v + bias[b];
      }
    // (one wave's LDS accesses complete in order: its reads see its writes, and the next
    // sub-tile's writes follow these reads)
    // in chunks of up to 4 quads per lane (registers: the wide tiles hold 128 accumulators)
    constexpr int CH = IT < 4 ? IT : 4;
    static_assert(IT % CH == 0, "whole chunks");
#pragma unroll
    for (int c = 0; c < IT; c += CH) {
      float4 v[CH], prev[CH];
      float* dst[CH];
      bool ok[CH], accum[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) {  // the chunk's destinations read before its stores
        const int e = lane + 64 * (c + i), row = e / Q, q = e - row * Q;
        const int grow = m_w + a * 32 + row, gcol = n_w + 4 * q;
        v[i] = *reinterpret_cast<const float4*>(buf + row * LD + 4 * q);
        ok[i] = grow < p.M && gcol < p.N;
        const bool first = gcol < p.split;
        dst[i] = first ? p.out1 + (long)grow * p.ld1 + gcol
                       : p.out2 + (long)grow * p.ld2 + (gcol - p.split);
        accum[i] = ok[i] && (first ? p.acc1 : p.acc2);
        prev[i] = accum[i] ? *reinterpret_cast<const float4*>(dst[i]) : make_float4(0, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < CH; ++i)
        if (ok[i]) st_nt4(dst[i], accum[i] ? add4(prev[i], v[i]) : v[i]);
    }
  }
}

// ---- epilogue of a wave's TM x TN grid of 32x32 accumulators (C/D map of the 32x32 MFMA
// forms: column = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)). m_w/n_w: the wave's first
// output row/column. Split-K slabs (zstride > 0) get the raw sums; otherwise bias, two-way
// column routing (dgrad of a concat) and accumulate-or-overwrite are applied.
template <int TM, int TN>
__device__ __forceinline__ void store_acc(const GemmConvParams& p, const floatx16 (&acc)[TM][TN],
                                          int m_w, int n_w, int lane, int zb = -1) {
  const int h = lane >> 5, l32 = lane & 31;
  if (p.zstride > 0) {
    float* out1 = p.out1 + (long)(zb >= 0 ? zb : (int)blockIdx.z) * p.zstride;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n_w + b * 32 + l32;
        if (col >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m_w + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row < p.M) out1[(long)row * p.N + col] = acc[a][b][r];
        }
      }
    return;
  }
  if (p.stats) acc_stats<TM, TN>(p, acc, m_w, n_w, lane);
  if (!p.acc1 && !p.acc2) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n_w + b * 32 + l32;
        if (col >= p.N) continue;
        const float bias = p.bias ? p.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m_w + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row >= p.M) continue;
          const float v = acc[a][b][r] + bias;
          if (col < p.split) p.out1[(long)row * p.ld1 + col] = v;
          else p.out2[(long)row * p.ld2 + (col - p.split)] = v;
        }
      }
    return;
  }
  // accumulate: the tile's 16 destination values are fetched together before any store (one
  // HBM latency per tile instead of one per element: the compiler cannot prove the
  // read-modify-writes independent, so it would not batch them itself; 0.80 -> 0.55 ms on a
  // 401408 x 512 -> 256 dgrad)
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n_w + b * 32 + l32;
      if (col >= p.N) continue;
      const float bias = p.bias ? p.bias[col] : 0.f;
      const bool first = col < p.split;  // two-way column routing (dgrad of a concat)
      float* base = first ? p.out1 + col : p.out2 + (col - p.split);
      const long ld = first ? p.ld1 : p.ld2;
      const int accum = first ? p.acc1 : p.acc2;
      float prev[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m_w + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        prev[r] = (accum && row < p.M) ? base[(long)row * ld] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m_w + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        const float v = acc[a][b][r] + bias;
        base[(long)row * ld] = accum ? prev[r] + v : v;
      }
    }
}

}  // namespace pld

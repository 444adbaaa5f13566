// Implicit-GEMM convolution in fp32 through three bf16 MFMA products ("bf16x3").
//
// Every fp32 operand value v is split once, when its tile is staged into LDS, into
//   hi = bf16_rne(v),  lo = bf16_rne(v - hi)            (|v - hi - lo| <= 2^-17 |v|)
// and each product is formed as  a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi  on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation. The dropped a_lo.b_lo term and the split
// residuals bound the error of one product by ~2^-16 relative (~1.5e-5), two orders of magnitude
// inside BASELINE.json's 1e-3 fp32 parity bar (and ~30x tighter than the TF32 that the
// reference's TF2 applies to convolutions on tensor-core GPUs). Throughput: three
// 32x32x16 MFMAs (96 cycles) do the work of eight 32x32x2 fp32 MFMAs (512 cycles).
//
// Same three GEMM views, same C-ABI entry points and epilogue as conv_igemm.hip (which keeps the
// exact-fp32 path and the scalar shapes this kernel does not take):
//   FWD/DGRAD: C[m=(img,oy,ox)][n] = sum_k im2col(x)[m][k=(ty,tx,ci)] * Wn[n][k]
//   WGRAD    : C[i=(ty,tx,ci)][co] = sum_{p=(img,oy,ox)} im2col(x)[p][i] * dY[p][co]
//
// Tiling: 512 threads = 8 waves, warp-specialised. Waves 0-3 (consumers) own (BM/WM) x (BN/WN)
// of the BM x BN block tile as 32x32 MFMA tiles; waves 4-7 (producers) stage the next 32-deep
// K-step (global loads two steps ahead, hi/lo split, LDS stores), so the VALU split work of one
// wave overlaps the matrix work of its SIMD partner. LDS holds, per operand and buffer, a hi
// plane and a lo plane of [rows][4 x 16-byte k-chunks], XOR-swizzled (chunk_off) so that the
// ds_read_b128 fragment reads (lane = row, 16 B = 8 k) and the producers' stores are
// conflict-free. Double-buffered, one barrier per K-step. Workgroups are mapped to tiles
// XCD-aware (neighbouring tiles share an XCD's L2).
//   FWD/DGRAD staging: full 128-byte lines — 8 lanes per row, 4 consecutive k (channels of one
//     tap and one source, since C % 8 == 0) per lane; the filter operand is pre-split
//     (pld_filter_split; the host splits into the workspace when the caller has no copy) and
//     staged as-is. A one-source FWD conv may carry the fused input prologue act(x*s[c] + t[c])
//     (the BatchNorm apply + activation of the layer that produced x, never materialised): the
//     producers apply it to in-image elements between the global load and the split (PRO).
//   WGRAD staging: lanes over 4-channel quads of one pixel (coalesced), stored row-contiguous
//     into a [k = pixel][channel] image that the consumers read with ds_read_b64_tr_b16
//     (hardware transpose) into the k-contiguous MFMA fragments.
#include <algorithm>
#include <cstdlib>

#include "conv_x3_core.h"

namespace pld {
namespace x3 {

// --------------------------------------------------------------------- patch mode
// 3x3 stride-1 FWD/DGRAD convs whose input has exactly 32 channels (one source): the whole K =
// 9 taps x 32 channels is ONE input patch. A workgroup stages the 10 x 34-pixel halo patch of an
// 8 x 32-pixel output tile once (hi/lo planes, [pixel][32 k] rows, chunk_off-swizzled) plus the
// pre-split filter of its BN output channels for all 9 taps, then each of its 8 waves computes
// one 32-pixel output row: per tap the A fragments are the patch rows shifted by (ty, tx) —
// every input value is fetched once per tile instead of once per tap (the im2col GEMM re-reads
// each input 9 times, which bounds the N <= 96 decoder convs by operand fetch, not MFMA).
constexpr int PT_H = 8, PT_W = 32, P_H = PT_H + 2, P_W = PT_W + 2, P_PIX = P_H * P_W;

template <int BN>
struct PatchSmem {
  static constexpr int A_PLANE = P_PIX * 64;   // [patch pixel][32 k] bf16
  static constexpr int B_TAP = BN * 64;        // [n][32 k] bf16, one tap
  static constexpr int B_PLANE = 9 * B_TAP;
  static constexpr int BYTES = 2 * A_PLANE + 2 * B_PLANE;
};

template <int BN>
__global__ __launch_bounds__(512) void conv_x3_patch_kernel(GemmConvParams p) {
  using S = PatchSmem<BN>;
  constexpr int TN = BN / 32;
  __shared__ __attribute__((aligned(16))) unsigned char smem[S::BYTES];
  unsigned char* Ah = smem;
  unsigned char* Al = smem + S::A_PLANE;
  unsigned char* Bh = smem + 2 * S::A_PLANE;
  unsigned char* Bl = Bh + S::B_PLANE;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int tiles_x = (p.ow + PT_W - 1) / PT_W, tiles_y = (p.oh + PT_H - 1) / PT_H;
  // XCD-aware order (as conv_x3_kernel): neighbouring tiles, which share halo rows, on one XCD
  const int nwg = gridDim.x * gridDim.y;
  const int flat = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = flat & 7, slot = flat >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int nb = wid % gridDim.y;
  int t = wid / gridDim.y;
  const int tx0 = t % tiles_x;
  t /= tiles_x;
  const int ty0 = t % tiles_y;
  const int img = t / tiles_y;
  const int oy0 = ty0 * PT_H, ox0 = tx0 * PT_W, n0 = nb * BN;

  // ---- stage: patch (all 512 threads; loads first, then split + stores) ----
  {
    const long img_elems = (long)p.h * p.w * 32;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.x1 + img * img_elems, img_elems * 4);
    constexpr int EA = P_PIX * 8, IA = (EA + 511) / 512;  // 4-channel quads of the patch
    float4 va[IA];
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int e = threadIdx.x + 512 * i;
      const int px = e >> 3, q = e & 7;
      const int py = px / P_W, pxx = px - py * P_W;
      const int iy = oy0 - p.pt + py, ix = ox0 - p.pl + pxx;
      const bool ok = e < EA && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
      va[i] = bload4(rs, ok ? (unsigned)(((iy * p.w + ix) * 32 + 4 * q) * 4) : OOB);
    }
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.bsplit, (long)p.N * p.K * 4);
    constexpr int EB = 9 * BN * 8, IB = (EB + 511) / 512;  // 16-byte halves of 8-k chunks
    float4 vb[IB];
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int e = threadIdx.x + 512 * i;
      const int half = e & 1, c = (e >> 1) & 3, nt = e >> 3;
      const int tap = nt / BN, n = nt - tap * BN;
      const bool ok = e < EB && n0 + n < p.N;
      vb[i] = bload4(rb, ok ? (unsigned)(((n0 + n) * p.K + tap * 32 + 8 * c) * 4 + 16 * half)
                            : OOB);
    }
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int e = threadIdx.x + 512 * i;
      if (e < EA) {
        const int px = e >> 3, q = e & 7;
        unsigned h0, l0, h1, l1;
        split2(va[i].x, va[i].y, h0, l0);
        split2(va[i].z, va[i].w, h1, l1);
        const int o = chunk_off(px, q >> 1) + 8 * (q & 1);
        *reinterpret_cast<u32x2*>(Ah + o) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(Al + o) = u32x2{l0, l1};
      }
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int e = threadIdx.x + 512 * i;
      if (e < EB) {
        const int half = e & 1, c = (e >> 1) & 3, nt = e >> 3;
        const int tap = nt / BN, n = nt - tap * BN;
        *reinterpret_cast<float4*>((half ? Bl : Bh) + tap * S::B_TAP + chunk_off(n, c)) = vb[i];
      }
    }
  }
  __syncthreads();

  // ---- compute: wave w = output row oy0 + w, 32 pixels x BN channels ----
  const int h = lane >> 5, l32 = lane & 31;
  floatx16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int r = (wave + tap / 3) * P_W + l32 + tap % 3;  // this lane's patch pixel
    const unsigned char* bh_t = Bh + tap * S::B_TAP;
    const unsigned char* bl_t = Bl + tap * S::B_TAP;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 ah = lds_frag(Ah, r, 2 * s + h), al = lds_frag(Al, r, 2 * s + h);
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const bf16x8 bh = lds_frag(bh_t, b * 32 + l32, 2 * s + h);
        const bf16x8 bl = lds_frag(bl_t, b * 32 + l32, 2 * s + h);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[b], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: tile row i = output pixel ox0 + i of row oy0 + wave (bias, routing, acc) ----
  const int oy = oy0 + wave;
  // whole float4 column quads (N, split, leading dims in 4s, 16-byte bases): the wave's
  // [32 px][BN] block through LDS (after every wave's last fragment read), out as 16-byte
  // streaming stores of contiguous pixel runs — the conv_x3_kernel grid epilogue's form
  const bool quads = (p.N & 3) == 0 && (p.split >= p.N || (p.split & 3) == 0) &&
                     (p.ld1 & 3) == 0 && (reinterpret_cast<uintptr_t>(p.out1) & 15) == 0 &&
                     (p.split >= p.N ||
                      ((p.ld2 & 3) == 0 && (reinterpret_cast<uintptr_t>(p.out2) & 15) == 0));
  if (quads) {
    constexpr int LD = BN + 8;  // the two half-waves' rows (4 apart) 32 banks apart
    static_assert(8 * 32 * LD * 4 <= S::BYTES, "epilogue staging fits the LDS");
    __syncthreads();
    float* buf = reinterpret_cast<float*>(smem) + wave * 32 * LD;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + b * 32 + l32;
      const float bias = (p.bias && col < p.N) ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[b][r];
        buf[((r & 3) + 8 * (r >> 2) + 4 * h) * LD + b * 32 + l32] = v + bias;
      }
    }
    if (oy >= p.oh) return;
    constexpr int Q = BN / 4, IT = 32 * Q / 64;
    float4 v[IT], prev[IT];
    float* dst[IT];
    bool ok[IT], accum[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {  // every destination read before any store (accumulate)
      const int e = lane + 64 * i, px = e / Q, q = e - px * Q;
      const int ox = ox0 + px, col = n0 + 4 * q;
      v[i] = *reinterpret_cast<const float4*>(buf + px * LD + 4 * q);
      ok[i] = ox < p.ow && col < p.N;
      const long row = ((long)img * p.oh + oy) * p.ow + ox;
      const bool first = col < p.split;
      dst[i] = first ? p.out1 + row * p.ld1 + col : p.out2 + row * p.ld2 + (col - p.split);
      accum[i] = ok[i] && (first ? p.acc1 : p.acc2);
      prev[i] = accum[i] ? *reinterpret_cast<const float4*>(dst[i]) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i)
      if (ok[i]) st_nt4(dst[i], accum[i] ? add4(prev[i], v[i]) : v[i]);
    return;
  }
  if (oy >= p.oh) return;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = n0 + b * 32 + l32;
    if (col >= p.N) continue;
    const float bias = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ox = ox0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (ox >= p.ow) continue;
      const long row = ((long)img * p.oh + oy) * p.ow + ox;
      const float v = acc[b][r] + bias;
      if (col < p.split) {
        float* dst = p.out1 + row * p.ld1 + col;
        *dst = p.acc1 ? *dst + v : v;
      } else {
        float* dst = p.out2 + row * p.ld2 + (col - p.split);
        *dst = p.acc2 ? *dst + v : v;
      }
    }
  }
}

// Inputs of several 32-channel chunks (C % 16 == 0 per source; a concat's sources chunked
// separately, a ragged 16-channel chunk masked): 32 output channels per workgroup, one (patch,
// filter) stage per chunk, double buffered in LDS (2 x 80 KB).
constexpr int MC_STAGE = 2 * PatchSmem<32>::A_PLANE + 2 * PatchSmem<32>::B_PLANE;

// The multi-chunk patch conv, warp-specialised (the pattern of conv_x3_patch_wgrad_pc_kernel):
// waves 0-3 compute two output rows each (2 accumulators, the
// filter fragments of a (tap, k-half) shared by both rows, the next fragments read while the
// current ones multiply), waves 4-7 stage the next chunk (global loads one chunk ahead in
// registers, patch hi/lo split, pre-split filter copied) into the other LDS buffer. One barrier
// per chunk.
template <bool CAT>
__global__ __launch_bounds__(512) void conv_x3_patch_mc_pc_kernel(GemmConvParams p) {
  using S = PatchSmem<32>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * MC_STAGE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int tiles_x = (p.ow + PT_W - 1) / PT_W, tiles_y = (p.oh + PT_H - 1) / PT_H;
  const int nwg = gridDim.x * gridDim.y;
  const int flat = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = flat & 7, slot = flat >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int nb = wid % gridDim.y;
  int t = wid / gridDim.y;
  const int tx0 = t % tiles_x;
  t /= tiles_x;
  const int ty0 = t % tiles_y;
  const int img = t / tiles_y;
  const int oy0 = ty0 * PT_H, ox0 = tx0 * PT_W, n0 = nb * 32;
  const int nch = p.kc_tap;  // chunks: kc1 of x1, then those of x2

  floatx16 acc[2];  // compute waves only
  if (wave >= 4) {  // ------------------------------------------------------------ staging
    const int ptid = threadIdx.x - 256;
    const long img1 = (long)p.h * p.w * p.c1, img2 = (long)p.h * p.w * p.c2;
    const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.x1 + img * img1, img1 * 4);
    const __amdgpu_buffer_rsrc_t rs2 = CAT ? make_rsrc(p.x2 + img * img2, img2 * 4) : rs1;
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.bsplit, (long)p.N * p.K * 4);
    constexpr int EA = P_PIX * 8, IA = (EA + 255) / 256;
    constexpr int EB = 9 * 32 * 8, IB = (EB + 255) / 256;
    float4 va[IA], vb[IB];
    auto load = [&](int ch) {
      ch = min(ch, nch - 1);  // past the end: a harmless re-load of the last chunk
      const bool s2 = CAT && ch >= p.kc1;
      const int cb = (s2 ? ch - p.kc1 : ch) * 32, cs = s2 ? p.c2 : p.c1;
      const __amdgpu_buffer_rsrc_t rs = s2 ? rs2 : rs1;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int e = ptid + 256 * i;
        const int px = e >> 3, c4 = (e & 7) * 4;
        const int py = px / P_W, pxx = px - py * P_W;
        const int iy = oy0 - p.pt + py, ix = ox0 - p.pl + pxx;
        const bool ok = e < EA && cb + c4 < cs && (unsigned)iy < (unsigned)p.h &&
                        (unsigned)ix < (unsigned)p.w;
        va[i] = bload4(rs, ok ? (unsigned)(((iy * p.w + ix) * cs + cb + c4) * 4) : OOB);
      }
      const int kb = (s2 ? p.c1 : 0) + cb;
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int e = ptid + 256 * i;
        const int half = e & 1, c = (e >> 1) & 3, nt = e >> 3;
        const int tap = nt >> 5, n = nt & 31;
        const bool ok = e < EB && n0 + n < p.N && cb + 8 * c < cs;
        vb[i] = bload4(rb, ok ? (unsigned)(((n0 + n) * p.K + tap * p.C + kb + 8 * c) * 4 +
                                           16 * half)
                              : OOB);
      }
    };
    auto store = [&](int buf) {
      unsigned char* Ah = smem + buf * MC_STAGE;
      unsigned char* Al = Ah + S::A_PLANE;
      unsigned char* Bh = Ah + 2 * S::A_PLANE;
      unsigned char* Bl = Bh + S::B_PLANE;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int e = ptid + 256 * i;
        if (e < EA) {
          const int px = e >> 3, q = e & 7;
          unsigned h0, l0, h1, l1;
          split2(va[i].x, va[i].y, h0, l0);
          split2(va[i].z, va[i].w, h1, l1);
          const int o = chunk_off(px, q >> 1) + 8 * (q & 1);
          *reinterpret_cast<u32x2*>(Ah + o) = u32x2{h0, h1};
          *reinterpret_cast<u32x2*>(Al + o) = u32x2{l0, l1};
        }
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int e = ptid + 256 * i;
        if (e < EB) {
          const int half = e & 1, c = (e >> 1) & 3, nt = e >> 3;
          const int tap = nt >> 5, n = nt & 31;
          *reinterpret_cast<float4*>((half ? Bl : Bh) + tap * S::B_TAP + chunk_off(n, c)) =
              vb[i];
        }
      }
    };
    // barriers: 1 + nch, matching the compute waves
    load(0);
    store(0);
    load(1);
    lds_barrier();
    for (int i = 0;; ++i) {
      store((i + 1) & 1);  // chunk i+1 while the compute waves multiply chunk i
      load(i + 2);
      lds_barrier();
      if (i + 1 >= nch) break;
    }
    return;
  }
  // ------------------------------------------------------------------------ compute
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  lds_barrier();
  for (int ch = 0; ch < nch; ++ch) {
    const unsigned char* Ah = smem + (ch & 1) * MC_STAGE;
    const unsigned char* Al = Ah + S::A_PLANE;
    const unsigned char* Bh = Ah + 2 * S::A_PLANE;
    const unsigned char* Bl = Bh + S::B_PLANE;
    // step j = 2 tap + s: the A rows of output rows 2 wave, 2 wave + 1 shifted by the tap,
    // k-chunk 2 s + h; the filter of the tap
    auto frags = [&](int j, bf16x8 (&a)[4], bf16x8 (&b)[2]) {
      const int tap = j >> 1, s = j & 1;
      const int r0 = (2 * wave + tap / 3) * P_W + l32 + tap % 3;
      a[0] = lds_frag(Ah, r0, 2 * s + h);
      a[1] = lds_frag(Al, r0, 2 * s + h);
      a[2] = lds_frag(Ah, r0 + P_W, 2 * s + h);
      a[3] = lds_frag(Al, r0 + P_W, 2 * s + h);
      b[0] = lds_frag(Bh + tap * S::B_TAP, l32, 2 * s + h);
      b[1] = lds_frag(Bl + tap * S::B_TAP, l32, 2 * s + h);
    };
    bf16x8 a[4], b[2], na[4], nb2[2];
    frags(0, a, b);
#pragma unroll
    for (int j = 0; j < 18; ++j) {
      if (j < 17) frags(j + 1, na, nb2);
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);  // the next step's reads first
      __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);  // then this step's products
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2 * r + 1], b[0], acc[r], 0, 0, 0);
        acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2 * r], b[1], acc[r], 0, 0, 0);
        acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2 * r], b[0], acc[r], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = na[u];
      b[0] = nb2[0];
      b[1] = nb2[1];
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
  }
  const int col = n0 + l32;
  if (col >= p.N) return;
  const float bias = p.bias ? p.bias[col] : 0.f;
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int oy = oy0 + 2 * wave + rr;
    if (oy >= p.oh) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ox = ox0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (ox >= p.ow) continue;
      const long row = ((long)img * p.oh + oy) * p.ow + ox;
      const float v = acc[rr][r] + bias;
      if (col < p.split) {
        float* dst = p.out1 + row * p.ld1 + col;
        *dst = p.acc1 ? *dst + v : v;
      } else {
        float* dst = p.out2 + row * p.ld2 + (col - p.split);
        *dst = p.acc2 ? *dst + v : v;
      }
    }
  }
}

constexpr int kPatchBN[] = {32, 64, 96};
constexpr int kNumPatch = 3;

// WGRAD in patch form, 3x3 stride 1: dW[tap][ci][co] = sum_p X[p + tap][ci] dY[p][co]. A
// workgroup owns one 32-channel chunk of ONE source (all 9 taps: 9 MFMA row tiles) x 32 output
// channels, and loops over a range of 8 x 32-pixel output tiles (its split-K share). Per tile it
// stages the 10 x 34 input patch of the chunk and the 256 x 32 dY tile as [pixel][channel] hi/lo
// images, double-buffered; the A fragment of tap (ty, tx) is the patch image read transposed
// (ds_read_b64_tr_b16) from row (row + ty) * 34 + tx on, the dY fragment is shared by the 9
// taps. Every input value is staged once per tile, not once per tap.
constexpr int PW_A = P_PIX * 64;       // patch image plane: [340 pixels][32 ch] bf16
constexpr int PW_B = PT_H * PT_W * 64; // dY image plane: [256 pixels][32 co] bf16
constexpr int PW_STAGE = 2 * PW_A + 2 * PW_B;

__device__ __forceinline__ bf16x8 tr_frag_rows(const unsigned char* plane, int row0, int lane) {
  // 32x32x16 operand from a [row][32 col] bf16 image (64-byte rows, no swizzle: 4 consecutive
  // rows land 16 banks apart): lane l needs column l & 31 and rows row0 + 8 (l >> 5) .. +7
  const int i16 = lane & 15, grp = (lane >> 4) & 1, h = lane >> 5;
  const int r = row0 + 8 * h + (i16 >> 2);
  const int col = 16 * grp + 4 * (i16 & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plane + r * 64 + col * 2));
  const v4s hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plane + (r + 4) * 64 + col * 2));
  const v4s v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v);
}

// Warp-specialised (round 3; a uniform-role form, where every wave holds 9 accumulator tiles +
// the next tile's loads, left the matrix pipes idle while all waves split and stored: MFMA 31 %
// busy). Waves 0-3 only compute — wave c owns output rows 2c, 2c+1 of the 8 x 32 tile (four
// 16-pixel k-steps, all 9 taps), with the next tap's A fragments and the next k-step's dY
// fragments read while the current ones multiply — and waves 4-7 only stage: global loads two
// tiles ahead in registers, bf16 hi/lo split, LDS stores into the other buffer. One barrier per
// tile; the 4 consumers' partial sums meet in LDS in a fixed order (deterministic).
__device__ __forceinline__ void pw_frag_pair(const unsigned char* plane, int plane_bytes, int row0,
                                             int lane, bf16x8& hi, bf16x8& lo) {
  hi = tr_frag_rows(plane, row0, lane);
  lo = tr_frag_rows(plane + plane_bytes, row0, lane);
}

__global__ __launch_bounds__(512) void conv_x3_patch_wgrad_pc_kernel(GemmConvParams p, int tiles,
                                                                     int tiles_per_split) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * PW_STAGE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // several cout tiles (N > 32): XCD-aware order, cout tile fastest, then chunk, then split —
  // the workgroups an XCD runs at once share one tile range, so a chunk's patch is fetched once
  // for its cout tiles and a dY tile once for the concurrent chunks (dec2 dW, N = 144: 873 ->
  // 501 MB fetched per launch, time unchanged); one cout tile: launch order (dec3 dW measured 6 %
  // slower with the XCD order, nothing to share across cout tiles)
  const int flat = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int wid = gridDim.y > 1 ? xcd_order(flat, gridDim.x * gridDim.y * gridDim.z) : flat;
  const int nb = wid % gridDim.y, q = (wid / gridDim.y) % gridDim.x,
            zb = wid / (gridDim.x * gridDim.y);
  const bool s2 = q >= p.kc1;
  const int cb = (s2 ? q - p.kc1 : q) * 32;
  const int cs = s2 ? p.c2 : p.c1;
  const int nv = min(32, cs - cb);
  const int n0 = nb * 32;
  const int t_begin = zb * tiles_per_split, t_end = min(tiles, t_begin + tiles_per_split);
  const int n = t_end - t_begin;

  floatx16 acc[9];  // consumers only (the producers' path never defines it: no registers)
  if (wave >= 4) {  // ------------------------------------------------------------ producer
    const int ptid = threadIdx.x - 256;
    const int tiles_x = (p.ow + PT_W - 1) / PT_W, tiles_y = (p.oh + PT_H - 1) / PT_H;
    const long img_in = (long)p.h * p.w * cs;
    const long img_out = (long)p.oh * p.ow;
    const float* xsrc = s2 ? p.x2 : p.x1;
    constexpr int EA = P_PIX * 8, IA = (EA + 255) / 256;  // patch: 4-channel quads
    constexpr int EB = PT_H * PT_W * 8, IB = EB / 256;    // dY: 4-channel quads
    struct Stage {
      float4 a[IA], b[IB];
    };
    auto load = [&](int t, Stage& st) {
      t = min(t, t_end - 1);  // past the end: a harmless re-load of the last tile
      const int tx0 = t % tiles_x, r1 = t / tiles_x, ty0 = r1 % tiles_y, img = r1 / tiles_y;
      const int oy0 = ty0 * PT_H, ox0 = tx0 * PT_W;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(xsrc + img * img_in, img_in * 4);
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int e = ptid + 256 * i;
        const int px = e >> 3, c4 = (e & 7) * 4;
        const int py = px / P_W, pxx = px - py * P_W;
        const int iy = oy0 - p.pt + py, ix = ox0 - p.pl + pxx;
        const bool ok = e < EA && c4 < nv && (unsigned)iy < (unsigned)p.h &&
                        (unsigned)ix < (unsigned)p.w;
        st.a[i] = bload4(rs, ok ? (unsigned)(((iy * p.w + ix) * cs + cb + c4) * 4) : OOB);
      }
      const __amdgpu_buffer_rsrc_t rd =
          make_rsrc(p.bmat + img * img_out * p.N, img_out * p.N * 4);
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int e = ptid + 256 * i;
        const int k = e >> 3, c4 = (e & 7) * 4;
        const int oy = oy0 + (k >> 5), ox = ox0 + (k & 31);
        const bool ok = oy < p.oh && ox < p.ow && n0 + c4 < p.N;
        st.b[i] = bload4(rd, ok ? (unsigned)(((oy * p.ow + ox) * p.N + n0 + c4) * 4) : OOB);
      }
    };
    auto store = [&](int buf, const Stage& st) {
      unsigned char* A = smem + buf * PW_STAGE;
      unsigned char* B = A + 2 * PW_A;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int e = ptid + 256 * i;
        if (e < EA) {
          unsigned h0, l0, h1, l1;
          split2(st.a[i].x, st.a[i].y, h0, l0);
          split2(st.a[i].z, st.a[i].w, h1, l1);
          const int o = (e >> 3) * 64 + (e & 7) * 8;
          *reinterpret_cast<u32x2*>(A + o) = u32x2{h0, h1};
          *reinterpret_cast<u32x2*>(A + PW_A + o) = u32x2{l0, l1};
        }
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int e = ptid + 256 * i;
        unsigned h0, l0, h1, l1;
        split2(st.b[i].x, st.b[i].y, h0, l0);
        split2(st.b[i].z, st.b[i].w, h1, l1);
        const int o = (e >> 3) * 64 + (e & 7) * 8;
        *reinterpret_cast<u32x2*>(B + o) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(B + PW_B + o) = u32x2{l0, l1};
      }
    };
    if (n > 0) {
      // one register stage (a tile's loads land during the previous tile's ~3.5k MFMA
      // cycles); barriers 1 + n, matching the consumers
      Stage st;
      load(t_begin, st);
      store(0, st);
      load(t_begin + 1, st);
      lds_barrier();
      for (int i = 0;; ++i) {
        store((i + 1) & 1, st);  // tile i+1 while the consumers multiply tile i
        load(t_begin + i + 2, st);
        lds_barrier();
        if (i + 1 >= n) break;
      }
    }
  } else {  // ----------------------------------------------------------------- consumer
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    if (n > 0) {
      lds_barrier();
      for (int t = 0; t < n; ++t) {
        const unsigned char* A = smem + (t & 1) * PW_STAGE;
        const unsigned char* B = A + 2 * PW_A;
        // k-step s: output row 2 wave + (s >> 1), pixels 16 (s & 1) .. +15
        bf16x8 bh, bl, ah, al, nh, nl;
        pw_frag_pair(B, PW_B, 32 * (2 * wave), lane, bh, bl);
        pw_frag_pair(A, PW_A, (2 * wave) * P_W, lane, ah, al);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = 2 * wave + (s >> 1), px0 = 16 * (s & 1);
          bf16x8 bh2 = bh, bl2 = bl;
          if (s < 3) {
            const int s1 = s + 1;
            pw_frag_pair(B, PW_B, 32 * (2 * wave + (s1 >> 1)) + 16 * (s1 & 1), lane, bh2, bl2);
          }
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            // the next A fragments (next tap, or tap 0 of the next k-step) in flight during
            // this tap's three products
            if (tap < 8) {
              const int t1 = tap + 1;
              pw_frag_pair(A, PW_A, (row + t1 / 3) * P_W + px0 + t1 % 3, lane, nh, nl);
            } else if (s < 3) {
              const int s1 = s + 1;
              pw_frag_pair(A, PW_A, (2 * wave + (s1 >> 1)) * P_W + 16 * (s1 & 1), lane, nh, nl);
            }
            // the reads above issue before this tap's products (then the 3 MFMAs); one
            // fragment set ahead and no more: the scheduler otherwise hoists every read of the
            // tile (register blow-up, spills)
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // MFMA
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[tap], 0, 0, 0);
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[tap], 0, 0, 0);
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[tap], 0, 0, 0);
            ah = nh;
            al = nl;
            __builtin_amdgcn_sched_barrier(0);
          }
          bh = bh2;
          bl = bl2;
        }
        lds_barrier();
      }
    }
  }
  // the 4 consumers' partial sums through LDS: each writes its 9 tiles to its own slot, then
  // all 512 threads add the 4 slots per element in a fixed order ((0 + 1) + (2 + 3)) and store
  // (deterministic; no wave holds two sets of accumulators)
  constexpr int SLOT = 9 * 16 * 64;  // floats: tile t, register r, lane
  static_assert(4 * SLOT * 4 <= 2 * PW_STAGE, "reduction slots fit the staging LDS");
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();  // the last tile's LDS reads are done
  if (wave < 4) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[wave * SLOT + (t * 16 + r) * 64 + lane] = acc[t][r];
  }
  __syncthreads();
  float* out = p.out1 + (p.zstride > 0 ? (long)zb * p.zstride : 0);
  for (int e = threadIdx.x; e < SLOT; e += 512) {
    const int ln = e & 63, r = (e >> 6) & 15, t = e >> 10;
    const int h = ln >> 5, col = n0 + (ln & 31);
    const int ci = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (col >= p.N || ci >= nv) continue;
    const float v = (red[e] + red[SLOT + e]) + (red[2 * SLOT + e] + red[3 * SLOT + e]);
    const long m = (long)t * p.C + (s2 ? p.c1 : 0) + cb + ci;
    float* dst = out + m * p.N + col;
    *dst = (p.zstride == 0 && p.acc1) ? *dst + v : v;
  }
}

// 64 output channels per workgroup (N > 32): the input patch of a tile is staged ONCE for both
// 32-wide cout tiles (the 32-wide kernel re-stages it per cout tile: fetch-bound, PMC 2.9x the
// algorithmic bytes for N = 240). dY rows are 128 B: the 32-byte column blocks are XOR-swizzled
// by 2 ((row >> 1) & 1) so the transposed reads of 4 consecutive rows hit 4 distinct bank ranges.
__device__ __forceinline__ int dy64_off(int k, int col) {  // byte offset of (row k, cout col)
  return k * 128 + (((col >> 4) ^ (((k >> 1) & 1) << 1)) << 5) + (col & 15) * 2;
}

__device__ __forceinline__ bf16x8 tr_frag_dy64(const unsigned char* plane, int row0, int c0,
                                               int lane) {
  const int i16 = lane & 15, grp = (lane >> 4) & 1, h = lane >> 5;
  const int r = row0 + 8 * h + (i16 >> 2);
  const int col = c0 + 16 * grp + 4 * (i16 & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plane + dy64_off(r, col)));
  const v4s hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plane + dy64_off(r + 4, col)));
  const v4s v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v);
}

// The 64-cout weight gradient in the producer/consumer form of conv_x3_patch_wgrad_pc_kernel.
// Double-buffering needs a smaller tile than the 8 x 32 one above (two 107 KB stages do not fit):
// 4 x 32 output pixels, a 6 x 34 input patch (26 KB) + the [128 px][64 co] dY image (32 KB) per
// stage. Waves 0-3 compute: wave c = (cout tile c & 1, output rows 2 (c >> 1), +1), all 9 taps
// (9 accumulators, the next fragments read under the current products); waves 4-7 stage the next
// tile. The two row pairs of a cout tile meet in LDS in a fixed order (deterministic). The
// 4-row tile also fits the 28-row decoder maps exactly (8 rows: 4 tiles, 12.5 % padding).
constexpr int Q_H = 4, Q_PH = Q_H + 2, Q_PIX = Q_PH * P_W;
constexpr int Q_A = Q_PIX * 64;        // patch plane: [204 px][32 ch] bf16
constexpr int Q_B = Q_H * PT_W * 128;  // dY plane: [128 px][64 co] bf16
constexpr int Q_STAGE = 2 * Q_A + 2 * Q_B;

__global__ __launch_bounds__(512) void conv_x3_patch_wgrad64_pc_kernel(GemmConvParams p,
                                                                       int tiles,
                                                                       int tiles_per_split) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * Q_STAGE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int flat = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int wid = gridDim.y > 1 ? xcd_order(flat, gridDim.x * gridDim.y * gridDim.z)
                                : flat;  // as the 32-wide kernel
  const int nb = wid % gridDim.y, q = (wid / gridDim.y) % gridDim.x,
            zb = wid / (gridDim.x * gridDim.y);
  const bool s2 = q >= p.kc1;
  const int cb = (s2 ? q - p.kc1 : q) * 32;
  const int cs = s2 ? p.c2 : p.c1;
  const int nv = min(32, cs - cb);
  const int n0 = nb * 64;
  const int t_begin = zb * tiles_per_split, t_end = min(tiles, t_begin + tiles_per_split);
  const int n = t_end - t_begin;
  const int ct = wave & 1, rp = (wave >> 1) & 1;

  floatx16 acc[9];
  if (wave >= 4) {  // ------------------------------------------------------------ producer
    const int ptid = threadIdx.x - 256;
    const int tiles_x = (p.ow + PT_W - 1) / PT_W, tiles_y = (p.oh + Q_H - 1) / Q_H;
    const long img_in = (long)p.h * p.w * cs;
    const long img_out = (long)p.oh * p.ow;
    const float* xsrc = s2 ? p.x2 : p.x1;
    constexpr int EA = Q_PIX * 8, IA = (EA + 255) / 256;  // patch: 4-channel quads
    constexpr int EB = Q_H * PT_W * 16, IB = EB / 256;    // dY: 4-cout quads
    struct Stage {
      float4 a[IA], b[IB];
    };
    auto load = [&](int t, Stage& st) {
      t = min(t, t_end - 1);  // past the end: a harmless re-load of the last tile
      const int tx0 = t % tiles_x, r1 = t / tiles_x, ty0 = r1 % tiles_y, img = r1 / tiles_y;
      const int oy0 = ty0 * Q_H, ox0 = tx0 * PT_W;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(xsrc + img * img_in, img_in * 4);
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int e = ptid + 256 * i;
        const int px = e >> 3, c4 = (e & 7) * 4;
        const int py = px / P_W, pxx = px - py * P_W;
        const int iy = oy0 - p.pt + py, ix = ox0 - p.pl + pxx;
        const bool ok = e < EA && c4 < nv && (unsigned)iy < (unsigned)p.h &&
                        (unsigned)ix < (unsigned)p.w;
        st.a[i] = bload4(rs, ok ? (unsigned)(((iy * p.w + ix) * cs + cb + c4) * 4) : OOB);
      }
      const __amdgpu_buffer_rsrc_t rd =
          make_rsrc(p.bmat + img * img_out * p.N, img_out * p.N * 4);
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int e = ptid + 256 * i;
        const int k = e >> 4, c4 = (e & 15) * 4;
        const int oy = oy0 + (k >> 5), ox = ox0 + (k & 31);
        const bool ok = oy < p.oh && ox < p.ow && n0 + c4 < p.N;
        st.b[i] = bload4(rd, ok ? (unsigned)(((oy * p.ow + ox) * p.N + n0 + c4) * 4) : OOB);
      }
    };
    auto store = [&](int buf, const Stage& st) {
      unsigned char* A = smem + buf * Q_STAGE;
      unsigned char* B = A + 2 * Q_A;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const int e = ptid + 256 * i;
        if (e < EA) {
          unsigned h0, l0, h1, l1;
          split2(st.a[i].x, st.a[i].y, h0, l0);
          split2(st.a[i].z, st.a[i].w, h1, l1);
          const int o = (e >> 3) * 64 + (e & 7) * 8;
          *reinterpret_cast<u32x2*>(A + o) = u32x2{h0, h1};
          *reinterpret_cast<u32x2*>(A + Q_A + o) = u32x2{l0, l1};
        }
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int e = ptid + 256 * i;
        unsigned h0, l0, h1, l1;
        split2(st.b[i].x, st.b[i].y, h0, l0);
        split2(st.b[i].z, st.b[i].w, h1, l1);
        const int o = dy64_off(e >> 4, (e & 15) * 4);
        *reinterpret_cast<u32x2*>(B + o) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(B + Q_B + o) = u32x2{l0, l1};
      }
    };
    if (n > 0) {  // barriers 1 + n, matching the consumers
      Stage st;
      load(t_begin, st);
      store(0, st);
      load(t_begin + 1, st);
      lds_barrier();
      for (int i = 0;; ++i) {
        store((i + 1) & 1, st);  // tile i+1 while the consumers multiply tile i
        load(t_begin + i + 2, st);
        lds_barrier();
        if (i + 1 >= n) break;
      }
    }
  } else {  // ----------------------------------------------------------------- consumer
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    if (n > 0) {
      lds_barrier();
      for (int t = 0; t < n; ++t) {
        const unsigned char* A = smem + (t & 1) * Q_STAGE;
        const unsigned char* B = A + 2 * Q_A;
        // k-step s: output row 2 rp + (s >> 1), pixels 16 (s & 1) .. +15
        bf16x8 bh, bl, ah, al, nh, nl;
        bh = tr_frag_dy64(B, 32 * (2 * rp), 32 * ct, lane);
        bl = tr_frag_dy64(B + Q_B, 32 * (2 * rp), 32 * ct, lane);
        pw_frag_pair(A, Q_A, (2 * rp) * P_W, lane, ah, al);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = 2 * rp + (s >> 1), px0 = 16 * (s & 1);
          bf16x8 bh2 = bh, bl2 = bl;
          if (s < 3) {
            const int s1 = s + 1, k1 = 32 * (2 * rp + (s1 >> 1)) + 16 * (s1 & 1);
            bh2 = tr_frag_dy64(B, k1, 32 * ct, lane);
            bl2 = tr_frag_dy64(B + Q_B, k1, 32 * ct, lane);
          }
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            if (tap < 8) {
              const int t1 = tap + 1;
              pw_frag_pair(A, Q_A, (row + t1 / 3) * P_W + px0 + t1 % 3, lane, nh, nl);
            } else if (s < 3) {
              const int s1 = s + 1;
              pw_frag_pair(A, Q_A, (2 * rp + (s1 >> 1)) * P_W + 16 * (s1 & 1), lane, nh, nl);
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // MFMA
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[tap], 0, 0, 0);
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[tap], 0, 0, 0);
            acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[tap], 0, 0, 0);
            ah = nh;
            al = nl;
            __builtin_amdgcn_sched_barrier(0);
          }
          bh = bh2;
          bl = bl2;
        }
        lds_barrier();
      }
    }
  }
  // row pair 1 -> LDS slot of its cout tile; row pair 0 adds it in place ((rp 0) + (rp 1)); then
  // all 512 threads store both cout tiles (deterministic)
  constexpr int SLOT = 9 * 16 * 64;  // floats: tile t, register r, lane
  static_assert(2 * SLOT * 4 <= 2 * Q_STAGE, "reduction slots fit the staging LDS");
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();  // the last tile's LDS reads are done
  if (wave < 4 && rp == 1) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[ct * SLOT + (t * 16 + r) * 64 + lane] = acc[t][r];
  }
  __syncthreads();
  if (wave < 4 && rp == 0) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* e = red + ct * SLOT + (t * 16 + r) * 64 + lane;
        *e = acc[t][r] + *e;
      }
  }
  __syncthreads();
  float* out = p.out1 + (p.zstride > 0 ? (long)zb * p.zstride : 0);
  for (int e = threadIdx.x; e < 2 * SLOT; e += 512) {
    const int c2t = e / SLOT, f = e - c2t * SLOT;
    const int ln = f & 63, r = (f >> 6) & 15, t = f >> 10;
    const int h = ln >> 5, col = n0 + 32 * c2t + (ln & 31);
    const int ci = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (col >= p.N || ci >= nv) continue;
    const long m = (long)t * p.C + (s2 ? p.c1 : 0) + cb + ci;
    float* dst = out + m * p.N + col;
    *dst = (p.zstride == 0 && p.acc1) ? *dst + red[e] : red[e];
  }
}

}  // namespace x3
}  // namespace pld

using namespace pld;

// ---- internal entry points used by conv_igemm.hip's C-ABI dispatch ----
__global__ void filter_split_kernel(const float* __restrict__ w, long chunks,
                                    x3::u32x4* __restrict__ out) {
  for (long c = (long)blockIdx.x * blockDim.x + threadIdx.x; c < chunks;
       c += (long)gridDim.x * blockDim.x) {
    const float4 a = reinterpret_cast<const float4*>(w)[2 * c];
    const float4 b = reinterpret_cast<const float4*>(w)[2 * c + 1];
    unsigned hs[4], ls[4];
    x3::split2(a.x, a.y, hs[0], ls[0]);
    x3::split2(a.z, a.w, hs[1], ls[1]);
    x3::split2(b.x, b.y, hs[2], ls[2]);
    x3::split2(b.z, b.w, hs[3], ls[3]);
    out[2 * c] = x3::u32x4{hs[0], hs[1], hs[2], hs[3]};
    out[2 * c + 1] = x3::u32x4{ls[0], ls[1], ls[2], ls[3]};
  }
}

extern "C" int pld_filter_split(const float* w, int64_t rows, int K, void* out, void* stream) {
  PLD_CHECK_ARG(w && out && rows > 0 && K > 0 && K % 8 == 0 && aligned16(w) && aligned16(out),
                "pld_filter_split: bad args (K %% 8 == 0, 16-byte aligned buffers)");
  const long chunks = (long)rows * K / 8;
  filter_split_kernel<<<std::min<unsigned>(cdiv(chunks, 256), 4096), 256, 0, as_stream(stream)>>>(
      w, chunks, reinterpret_cast<x3::u32x4*>(out));
  return check_launch("filter_split_kernel");
}

extern "C" int pld__x3_num_cfg(void) { return x3::kNumCfg; }
extern "C" int pld__x3_cfg_dims(int cfg, int* bm, int* bn, int* tm, int* tn, int* occ) {
  if (cfg < 0 || cfg >= x3::kNumCfg) return PLD_ERR_ARG;
  const x3::Cfg& c = x3::kCfg[cfg];
  *bm = c.bm; *bn = c.bn; *tm = c.tm; *tn = c.tn; *occ = c.occ;
  return PLD_OK;
}
extern "C" int pld__x3_wgrad_cfg_ok(int cfg) {  // every tile (widths 32..256, % 32)
  return cfg >= 0 && cfg < x3::kNumCfg;
}
extern "C" int pld__x3_num_patch(void) { return x3::kNumPatch; }
extern "C" int pld__x3_patch_bn(int cfg) {
  return cfg >= 0 && cfg < x3::kNumPatch ? x3::kPatchBN[cfg] : 0;
}
// eligibility of the patch kernels (FWD view): 3x3 stride 1, no prologue; one 32-channel source
// for every schedule, or channels in 16s per source for the multi-chunk (32-column) schedule 0
extern "C" int pld__x3_patch_ok(const GemmConvParams* p, int cfg) {
  const bool geo = p->kh == 3 && p->kw == 3 && p->sh == 1 && p->sw == 1 &&
                   p->in_scale == nullptr && p->K == 9 * p->C && p->pt >= 0 && p->pt <= 2 &&
                   p->pl >= 0 && p->pl <= 2;
  if (!geo) return 0;
  if (p->C == 32 && p->c2 == 0) return 1;
  return cfg == 0 && p->c1 % 16 == 0 && p->c2 % 16 == 0;
}
extern "C" int pld__x3_patch_launch(GemmConvParams* p, int cfg, void* stream) {
  if (!pld__x3_patch_ok(p, cfg) || cfg < 0 || cfg >= x3::kNumPatch || !p->bsplit) {
    set_error("conv_x3_patch: ineligible geometry or schedule %d", cfg);
    return PLD_ERR_ARG;
  }
  const int tiles = (int)(cdiv(p->ow, x3::PT_W) * cdiv(p->oh, x3::PT_H) * p->n);
  if (!(p->C == 32 && p->c2 == 0)) {  // multi-chunk
    p->kc1 = (int)cdiv(p->c1, 32);
    p->kc_tap = p->kc1 + (int)cdiv(p->c2, 32);
    dim3 grid(tiles, cdiv(p->N, 32));
    if (p->c2) x3::conv_x3_patch_mc_pc_kernel<true><<<grid, 512, 0, as_stream(stream)>>>(*p);
    else x3::conv_x3_patch_mc_pc_kernel<false><<<grid, 512, 0, as_stream(stream)>>>(*p);
    return check_launch("conv_x3_patch_mc_pc_kernel");
  }
  const int bn = x3::kPatchBN[cfg];
  dim3 grid(tiles, cdiv(p->N, bn));
  hipStream_t st = as_stream(stream);
  switch (cfg) {
    case 0: x3::conv_x3_patch_kernel<32><<<grid, 512, 0, st>>>(*p); break;
    case 1: x3::conv_x3_patch_kernel<64><<<grid, 512, 0, st>>>(*p); break;
    default: x3::conv_x3_patch_kernel<96><<<grid, 512, 0, st>>>(*p); break;
  }
  return check_launch("conv_x3_patch_kernel");
}
// WGRAD patch kernel: 3x3 stride 1, channel counts that split into 32-channel chunks of one
// source (c1, c2 % 16 == 0), no prologue; `splits` workgroups per (chunk, 32 cout) share the tiles
extern "C" int pld__x3_patch_wgrad_ok(const GemmConvParams* p) {
  return p->kh == 3 && p->kw == 3 && p->sh == 1 && p->sw == 1 && p->in_scale == nullptr &&
         p->c1 % 16 == 0 && p->c2 % 16 == 0 && p->N % 4 == 0 && p->pt >= 0 && p->pt <= 2 &&
         p->pl >= 0 && p->pl <= 2;
}
// output channels per workgroup of the patch WGRAD kernel: 64 (one staged patch feeds two
// 32-wide cout tiles) where that pads no more MFMA columns than 32-wide tiles do (N = 240: 256
// either way, dec1 wgrad 0.66 -> 0.56 ms); N = 144 keeps 32 (192 vs 160 padded: no gain)
extern "C" int pld__x3_patch_wgrad_cw(int N) {
  return (N > 32 && 2 * cdiv(N, 64) == cdiv(N, 32)) ? 64 : 32;
}
// output rows per tile: 8, or 4 for the double-buffered 64-cout kernel
extern "C" int pld__x3_patch_wgrad_th(int N) {
  return pld__x3_patch_wgrad_cw(N) == 64 ? x3::Q_H : x3::PT_H;
}
extern "C" int pld__x3_patch_wgrad_tiles(const GemmConvParams* p) {
  return (int)(cdiv(p->ow, x3::PT_W) * cdiv(p->oh, pld__x3_patch_wgrad_th(p->N)) * p->n);
}

extern "C" int pld__x3_patch_wgrad_launch(GemmConvParams* p, int splits, void* stream) {
  if (!pld__x3_patch_wgrad_ok(p) || splits < 1) {
    set_error("conv_x3_patch_wgrad: ineligible geometry");
    return PLD_ERR_ARG;
  }
  const int tiles = pld__x3_patch_wgrad_tiles(p);
  const int tps = (int)cdiv(tiles, splits);
  p->kc1 = (int)cdiv(p->c1, 32);
  const int chunks = p->kc1 + (int)cdiv(p->c2, 32);
  if (pld__x3_patch_wgrad_cw(p->N) == 64) {
    dim3 grid(chunks, cdiv(p->N, 64), cdiv(tiles, tps));
    x3::conv_x3_patch_wgrad64_pc_kernel<<<grid, 512, 0, as_stream(stream)>>>(*p, tiles, tps);
    return check_launch("conv_x3_patch_wgrad64_pc_kernel");
  }
  dim3 grid(chunks, cdiv(p->N, 32), cdiv(tiles, tps));
  x3::conv_x3_patch_wgrad_pc_kernel<<<grid, 512, 0, as_stream(stream)>>>(*p, tiles, tps);
  return check_launch("conv_x3_patch_wgrad_pc_kernel");
}
// sk_grid > 0: the tile-stream schedule with that many workgroups (p->sk_* filled by the host;
// non-aligned: p->sk_slab holds 2 sk_grid BM BN floats and the fixup kernel follows)
extern "C" int pld__x3_launch(GemmConvParams* p, int mode, int splits, int cfg, int sk_grid,
                              void* stream) {
  if (mode == MODE_WGRAD && !pld__x3_wgrad_cfg_ok(cfg)) {
    set_error("conv_x3: schedule %d is not a WGRAD tile", cfg);
    return PLD_ERR_ARG;
  }
  if (sk_grid > 0 && (p->in_scale || p->sk_nk <= 0 || p->sk_tiles <= 0 ||
                      (!p->sk_align && !p->sk_slab))) {
    set_error("conv_x3: bad tile-stream parameters");
    return PLD_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  if (mode == MODE_FWD) {
    if (sk_grid > 0) x3::launch_fwd_stream(*p, cfg, sk_grid, st);
    else x3::launch_fwd_grid(*p, splits, cfg, st);
  } else {
    if (sk_grid > 0) x3::launch_wgrad_stream(*p, cfg, sk_grid, st);
    else x3::launch_wgrad_grid(*p, splits, cfg, st);
  }
  return check_launch("conv_x3_kernel");
}

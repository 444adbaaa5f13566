// Row-band halo conv: the bf16x3 implicit GEMM of a 3x3 stride-1 'same' convolution (forward
// view: forward and dgrad) whose input is staged ONCE per 32-channel chunk instead of once per
// tap (round 6).
//
// A workgroup owns BM consecutive output pixels m0 .. m0 + BM - 1 of the flattened NHWC output
// (the im2col GEMM's M tile, so the epilogue, BN statistics, split-K slabs and concat routing are
// conv_x3_kernel's) and BN output channels. For input width w, every tap of those pixels reads
// inside the contiguous input pixel range [m0 - pt w - pl, m0 + BM + 2 w + 2 - pt w - pl): the
// "patch", BM + 2w + 2 rows of one chunk's 32 channels (128 contiguous bytes per pixel). The
// producer waves stage it split into bf16 hi/lo planes once per chunk; the consumer waves walk
// the chunk's 9 taps by addressing the patch rows shifted by ty w + tx, and a lane whose tap
// falls outside its image (padding, or the neighbouring image in the band) reads a zero row.
// Per 32-deep K-step (one (chunk, tap)) the producers stage only the pre-split filter slab (BN x
// 32) and 1/9 of the next chunk's patch; the im2col kernel stages BM x 32 input values per
// K-step, re-reading and re-splitting every input element 9 times. Round-5 ablations put 70 % of
// conv_x3_kernel's time in that producer path (profiles/r05_x3_ablation.txt).
//
// Structure as conv_x3_kernel (conv_x3_core.h): 512 threads, waves 0-3 consume (LDS -> MFMA,
// WM x WN grid of wave tiles), waves 4-7 produce; K-step order (chunk, tap) with the chunks of
// x1 then x2 (concat) and a ragged last chunk masked; one barrier per K-step. LDS: the patch
// double-buffered per chunk (chunk c + 1's patch is written in 8 parts during chunk c's first
// 8 K-steps, its loads issued one chunk ahead: the band comes from HBM), the filter slab
// triple-buffered (the producers run two K-steps ahead, so the consumers read the next step's
// first fragments under the current step's MFMAs). Input widths up to HALO_WMAX (the decoder
// maps of 14, 28 and 56 pixels); wider maps take the 2-D patch kernels (conv_x3.hip).
#include "conv_x3_core.h"

namespace pld {
namespace x3 {

constexpr int HALO_WMAX = 56;
constexpr int HALO_TAPS = 9;
constexpr int HALO_PARTS = 8;  // a chunk's patch is staged in the first 8 of its 9 K-steps

// WMAX: widest map an instantiation takes; NB: filter slab buffers (3: the consumers read the
// next step's first fragments under the current step's MFMAs; 2: one step at a time, the LDS
// of two resident workgroups per CU, so that one's prologue / epilogue hides under the other's
// MFMAs — the short-K dgrads)
template <int BM, int BN, int WMAX = HALO_WMAX, int NB = 3>
struct HaloSmem {
  static constexpr int NPMAX = BM + 2 * WMAX + 2;  // patch rows of the widest map
  static constexpr int ZR = NPMAX;                       // the zero row (after the patch rows)
  static constexpr int A_PLANE = (NPMAX + 1) * 64;       // [row][32 k] bf16, chunk_off layout
  static constexpr int A_BYTES = 2 * A_PLANE;            // hi + lo
  static constexpr int B_PLANE = BN * 64;
  static constexpr int B_BYTES = 2 * B_PLANE;
  static constexpr int BYTES = 2 * A_BYTES + NB * B_BYTES;
  __device__ static unsigned char* a(unsigned char* s, int buf) { return s + buf * A_BYTES; }
  __device__ static unsigned char* b(unsigned char* s, int buf) {
    return s + 2 * A_BYTES + buf * B_BYTES;
  }
};

// ---------------------------------------------------------------------------- producer
// A "unit" is one 32-channel chunk of one output tile (9 K-steps). Grid: the workgroup's tile
// (mb, nb), units = its chunks [g_begin / 9, g_end / 9). STREAM: global units u = tile x kc_tap
// + chunk over the tile-major stream, the workgroup's range cut on unit boundaries (sk_begin,
// sk_q = 9); a range may end and start mid-tile.
template <int BM, int BN, bool CAT, bool STREAM, int WMAX, int NB>
__device__ __forceinline__ void halo_producer(const GemmConvParams& p, unsigned char* smem,
                                              int g_begin, int g_end, int pw, int lane, int mb0,
                                              int nb0) {
  using S = HaloSmem<BM, BN, WMAX, NB>;
  constexpr int LEAD = NB - 1;  // K-steps the stored filter slab runs ahead of the consumers
  const int ptid = pw * 64 + lane;
  const int n = g_end - g_begin;
  if (n <= 0) {  // barriers: 1 + n, matching the consumers
    lds_barrier();
    return;
  }
  constexpr int FB = BN / 32;
  const int br = lane & 31, half = lane >> 5;
  const int np = BM + 2 * p.w + 2;  // patch rows of this map (<= NPMAX)
  const int npix = p.n * p.h * p.w;
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.x1, (long)npix * p.c1 * 4);
  const __amdgpu_buffer_rsrc_t rs2 = CAT ? make_rsrc(p.x2, (long)npix * p.c2 * 4) : rs1;
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.bsplit, (long)p.N * p.K * 4);
  const int u0 = g_begin / HALO_TAPS, nunits = n / HALO_TAPS;
  // per unit: its chunk, the input pixel of patch row 0 and the first filter row of its tile
  struct CI {
    int kq, P0, n0;
  };
  auto info = [&](int gc) {
    gc = min(gc, nunits - 1);  // past the end: a harmless re-fetch of the last unit
    CI c;
    int mb = mb0, nb = nb0;
    if constexpr (STREAM) {
      const int u = u0 + gc, t = u / p.kc_tap;
      c.kq = u - t * p.kc_tap;
      const int ta = sk_tile(p, t);
      mb = ta / p.sk_nnb;
      nb = ta - mb * p.sk_nnb;
    } else {
      c.kq = u0 + gc;
    }
    c.P0 = mb * BM - p.pt * p.w - p.pl;
    c.n0 = nb * BN;
    return c;
  };
  // patch: NPMAX rows x 8 float4 quads, in 8 parts of PART items (IAP per thread)
  constexpr int NQ = S::NPMAX * 8;
  constexpr int IAP = (NQ + HALO_PARTS * 256 - 1) / (HALO_PARTS * 256);
  constexpr int PART = IAP * 256;
  auto chunk_src = [&](int kq, int& chb, int& cs, __amdgpu_buffer_rsrc_t& rs, int& koff) {
    const bool s2 = CAT && kq >= p.kc1;
    chb = (s2 ? kq - p.kc1 : kq) * BK;
    cs = s2 ? p.c2 : p.c1;
    rs = s2 ? rs2 : rs1;
    koff = s2 ? p.c1 : 0;
  };
  auto load_part = [&](const CI& ci, int t, float4(&ra)[IAP]) {
    int chb, cs, koff;
    __amdgpu_buffer_rsrc_t rs;
    chunk_src(ci.kq, chb, cs, rs, koff);
#pragma unroll
    for (int i = 0; i < IAP; ++i) {
      const int e = t * PART + i * 256 + ptid;
      const int row = e >> 3, c = chb + 4 * (e & 7);
      const int pix = ci.P0 + row;
      const bool ok = row < np && (unsigned)pix < (unsigned)npix && c < cs;
      ra[i] = bload4(rs, ok ? (unsigned)((pix * cs + c) * 4) : OOB);
    }
  };
  auto store_part = [&](int buf, int t, const float4(&ra)[IAP]) {
    unsigned char* A = S::a(smem, buf);
#pragma unroll
    for (int i = 0; i < IAP; ++i) {
      const int e = t * PART + i * 256 + ptid;
      const int row = e >> 3, q = e & 7;
      if (row < np) {
        unsigned h0, l0, h1, l1;
        split2(ra[i].x, ra[i].y, h0, l0);
        split2(ra[i].z, ra[i].w, h1, l1);
        const int o = chunk_off(row, q >> 1) + 8 * (q & 1);
        *reinterpret_cast<u32x2*>(A + o) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(A + S::A_PLANE + o) = u32x2{l0, l1};
      }
    }
  };
  // filter slab of (unit, tap): lanes 0-31 stage the hi halves, 32-63 the lo halves of 8 rows
  // x 4 chunks per instruction
  auto load_b = [&](const CI& ci, int tap, float4(&rb)[FB]) {
    int chb, cs, koff;
    __amdgpu_buffer_rsrc_t rs;
    chunk_src(ci.kq, chb, cs, rs, koff);
    const int cb8 = chb + 8 * (br & 3);  // this lane's 8-k chunk of the filter row
    const int kc = tap * p.C + koff + cb8;
    const bool kcin = cb8 < cs;
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int nn = ci.n0 + pw * (BN / 4) + 8 * j + (br >> 2);
      const bool ok = kcin && nn < p.N;
      rb[j] = bload4(rsb, ok ? ((unsigned)(nn * p.K + kc)) * 4u + 16u * half : OOB);
    }
  };
  auto store_b = [&](int buf, const float4(&rb)[FB]) {
    unsigned char* B = S::b(smem, buf);
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int r = pw * (BN / 4) + 8 * j + (br >> 2);
      *reinterpret_cast<float4*>(B + half * S::B_PLANE + chunk_off(r, br & 3)) = rb[j];
    }
  };
  // Iteration i = 9 c + t (the consumers on relative step i, reading filter buffer i % 3 and,
  // ahead, (i + 1) % 3) stores the filter slab of step i + 2 into buffer (i + 2) % 3 (loaded two
  // iterations earlier) and, at t < 8, part t of the patch of relative unit c + 1 (loaded at the
  // same tap one unit earlier: nine K-steps for the HBM latency of the input band). Unit c + 1's
  // patch is complete one iteration before that unit starts (the pipelined consumers read its
  // first fragments one step ahead). Loop unrolled over two units: every register stage is
  // addressed at compile time. Re-fetches past the end are clamped; their stores land in
  // buffers no one reads any more.

  // the zero row of both patch buffers (hi and lo planes), never written again
  if (ptid < 16) {
    unsigned char* A = S::a(smem, ptid >> 3) + ((ptid >> 2) & 1) * S::A_PLANE;
    *reinterpret_cast<u32x4*>(A + S::ZR * 64 + 16 * (ptid & 3)) = u32x4{0u, 0u, 0u, 0u};
  }
  float4 pa[HALO_PARTS][IAP];  // the next unit's patch, in flight
  // filter slabs in flight in registers (a divisor of 18, so that the stage is addressed at
  // compile time; 3 and 6 measured no faster: the slabs are L2 hits)
  constexpr int BD = 2;
  float4 rb[BD][FB];
  // prologue: unit 0's patch and its first two filter slabs stored; unit 1's patch and slabs
  // 2, 3 in flight
  CI c0 = info(0), c1 = info(1), c2;
#pragma unroll
  for (int t = 0; t < HALO_PARTS; ++t) load_part(c0, t, pa[t]);
#pragma unroll
  for (int j = 0; j < LEAD; ++j) load_b(c0, j, rb[j]);
#pragma unroll
  for (int t = 0; t < HALO_PARTS; ++t) store_part(0, t, pa[t]);
#pragma unroll
  for (int j = 0; j < LEAD; ++j) store_b(j, rb[j]);
#pragma unroll
  for (int t = 0; t < HALO_PARTS; ++t) load_part(c1, t, pa[t]);
#pragma unroll
  for (int j = 0; j < BD; ++j) load_b(c0, LEAD + j, rb[j]);
  lds_barrier();
  for (int c = 0; c < nunits; c += 2) {
#pragma unroll
    for (int u = 0; u < 2 * HALO_TAPS; ++u) {
      const int t = u % HALO_TAPS, cc = c + u / HALO_TAPS;
      if (u == HALO_TAPS && cc >= nunits) break;
      if (t == 0) {  // units cc (c0), cc + 1 (c1), cc + 2 (c2)
        if (u != 0 || c != 0) c0 = c1, c1 = info(cc + 1);
        c2 = info(cc + 2);
      }
      const int i = HALO_TAPS * cc + t;
      store_b((i + LEAD) % NB, rb[u % BD]);
      if (t + LEAD + BD < HALO_TAPS) load_b(c0, t + LEAD + BD, rb[u % BD]);  // step i+LEAD+BD
      else load_b(c1, t + LEAD + BD - HALO_TAPS, rb[u % BD]);
      if (t < HALO_PARTS) {
        store_part((cc + 1) & 1, t, pa[t]);
        load_part(c2, t, pa[t]);
      }
      lds_barrier();
    }
  }
}

// ---------------------------------------------------------------------------- consumer
template <int BM, int BN, int WM, int WN, bool STREAM, int WMAX, int NB>
__device__ __forceinline__ void halo_consumer(const GemmConvParams& p, unsigned char* smem,
                                              int g_begin, int g_end, int wave, int lane, int mb,
                                              int nb, int zb, int wid) {
  using S = HaloSmem<BM, BN, WMAX, NB>;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, l32 = lane & 31;
  floatx16 acc[TM][TN];
  auto zero = [&]() {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  };
  zero();
  // per A fragment: this lane's patch row at tap (0, 0) (its row in the tile) and the taps of
  // its output pixel that stay inside its image (per tile)
  int pr[TM];
  unsigned vm[TM];
  auto setup = [&](int mbt) {
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int rr = wm * WTM + a * 32 + l32;
      const int m = mbt * BM + rr;
      const bool valid = m < p.M;
      const int mm = valid ? m : 0;
      const uint32_t q = p.dOW.div((uint32_t)mm);
      const int ox = mm - (int)q * p.ow;
      const uint32_t img = p.dOH.div(q);
      const int oy = (int)q - (int)img * p.oh;
      const int iy0 = oy - p.pt, ix0 = ox - p.pl;
      unsigned t = 0;
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx)
          t |= (unsigned)(valid && (unsigned)(iy0 + ty) < (unsigned)p.h &&
                          (unsigned)(ix0 + tx) < (unsigned)p.w)
               << (ty * 3 + tx);
      vm[a] = t;
      pr[a] = rr;
    }
  };
  struct Frags {
    bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
  };
  // fragments of relative step i, k-half s: the patch of its unit shifted by its tap (a lane
  // whose tap leaves its image reads the zero row), its filter slab
  auto read = [&](int i, int s, Frags& f) {
    const int ci = i / HALO_TAPS, tap = i - ci * HALO_TAPS;
    const int ty = tap / 3;
    const int toff = ty * p.w + (tap - 3 * ty);
    const unsigned char* A = S::a(smem, ci & 1);
    const unsigned char* B = S::b(smem, i % NB);
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int r = ((vm[a] >> tap) & 1u) ? pr[a] + toff : S::ZR;
      f.ah[a] = lds_frag(A, r, 2 * s + h);
      f.al[a] = lds_frag(A + S::A_PLANE, r, 2 * s + h);
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int r = wn * WTN + b * 32 + l32;
      f.bh[b] = lds_frag(B, r, 2 * s + h);
      f.bl[b] = lds_frag(B + S::B_PLANE, r, 2 * s + h);
    }
  };
  auto mma = [&](const Frags& f) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.al[a], f.bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[a], f.bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[a], f.bh[b], acc[a][b], 0, 0, 0);
      }
  };
  // the next half-step's fragment reads spread between this half-step's MFMAs (the LDS
  // array takes up to two ds_read_b128 per MFMA gap for free)
  constexpr int NR = 2 * (TM + TN), NM = 3 * TM * TN;
  constexpr int PER = NM / NR > 0 ? NM / NR : 1;
  auto interleave = [&]() {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // MFMA
    }
    if constexpr (NM > NR * PER) __builtin_amdgcn_sched_group_barrier(0x008, NM - NR * PER, 0);
  };
  Frags f0, f1;
  const int n = g_end - g_begin;
  // STREAM: the tile of the current unit, its first unit, the chunk within it
  const int u0 = g_begin / HALO_TAPS, u_end = g_end / HALO_TAPS;
  int tile = 0, kq = 0;
  if constexpr (STREAM) {
    tile = u0 / p.kc_tap;
    kq = u0 - tile * p.kc_tap;
    mb = sk_tile(p, tile) / p.sk_nnb;
    nb = sk_tile(p, tile) - mb * p.sk_nnb;
  }
  setup(mb);
  lds_barrier();
  // a tile's last step (or the range's): its sums out — whole tiles through the epilogue, a tile
  // cut between workgroups as raw partials for the fixup kernel (STREAM)
  auto tile_out = [&](int mbo, int nbo) {
    const int first = tile * p.kc_tap;
    if (first >= u0 && first + p.kc_tap <= u_end)
      store_acc<TM, TN>(p, acc, mbo * BM + wm * WTM, nbo * BN + wn * WTN, lane);
    else
      store_partial<TM, TN, BM, BN>(p, acc, wm * WTM, wn * WTN, lane, wid,
                                    tile == u0 / p.kc_tap ? 0 : 1);
    zero();
  };
  if constexpr (NB == 3) {
    if (n > 0) read(0, 0, f0);
    for (int i = 0; i < n; ++i) {
      read(i, 1, f1);  // the second half of this step while the first multiplies
      mma(f0);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      // STREAM: the last step of a tile; the next step (read below) is the next tile's first,
      // so its rows and tap masks are set up now (this step's reads are all issued)
      const bool tend = STREAM && i % HALO_TAPS == HALO_TAPS - 1 &&
                        (kq == p.kc_tap - 1 || i == n - 1);
      const int mbo = mb, nbo = nb;
      if (STREAM && tend && i + 1 < n) {
        const int ta = sk_tile(p, tile + 1);
        mb = ta / p.sk_nnb;
        nb = ta - mb * p.sk_nnb;
        setup(mb);
      }
      // the next step's first half (ready since the last barrier: the producers run two steps
      // ahead); unconditional (the last step re-reads itself) so that the LDS wait counts stay
      // exact and this half's MFMAs do not wait for these reads
      read(min(i + 1, n - 1), 0, f0);
      mma(f1);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (STREAM) {
        if (i % HALO_TAPS == HALO_TAPS - 1) {
          if (tend) {
            tile_out(mbo, nbo);
            ++tile;
            kq = 0;
          } else {
            ++kq;
          }
        }
      }
      // no LDS drain before this barrier: the reads still in flight are the next step's, from
      // buffers the producers do not write in the coming iteration (filter buffer (i + 1) % 3,
      // the current or next unit's patch); this step's reads completed under its MFMAs
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  } else {
    // NB == 2: one step at a time (the next step's filter slab is not there yet)
    for (int i = 0; i < n; ++i) {
      read(i, 0, f0);
      __builtin_amdgcn_sched_barrier(0);
      mma(f0);
      read(i, 1, f0);
      __builtin_amdgcn_sched_barrier(0);
      mma(f0);
      if (STREAM && i % HALO_TAPS == HALO_TAPS - 1) {
        if (kq == p.kc_tap - 1 || i == n - 1) {
          tile_out(mb, nb);
          ++tile;
          kq = 0;
          mb = sk_tile(p, tile) / p.sk_nnb;
          nb = sk_tile(p, tile) - mb * p.sk_nnb;
          setup(mb);
        } else {
          ++kq;
        }
      }
      lds_barrier();
    }
  }
  if constexpr (STREAM) return;
  // epilogue (conv_x3_kernel's grid form): the staging buffers are free after the last barrier
  if constexpr (4 * 32 * (WTN + 8) * 4 <= S::BYTES) {
    if (staged_ok(p)) {
      const int m_w = mb * BM + wm * WTM, n_w = nb * BN + wn * WTN;
      if (p.stats) acc_stats<TM, TN>(p, acc, m_w, n_w, lane);
      store_acc_staged<TM, TN>(p, acc, m_w, n_w, lane,
                               reinterpret_cast<float*>(smem) + wave * 32 * (WTN + 8));
      return;
    }
  }
  store_acc<TM, TN>(p, acc, mb * BM + wm * WTM, nb * BN + wn * WTN, lane, zb);
}

template <int BM, int BN, int WM, int WN, bool CAT, bool STREAM, int WMAX, int NB>
__global__ __launch_bounds__(512, NB == 2 ? 2 : 1) void conv_x3_halo_kernel(GemmConvParams p) {
  using S = HaloSmem<BM, BN, WMAX, NB>;
  static_assert(WM * WN == 4, "4 consumer waves");
  static_assert((BM / WM) % 32 == 0 && (BN / WN) % 32 == 0 && BN % 32 == 0, "wave tile");
  static_assert(S::BYTES <= (NB == 2 ? 80 : 160) * 1024, "LDS (NB == 2: two workgroups per CU)");
  __shared__ __attribute__((aligned(16))) unsigned char smem[S::BYTES];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nmb = gridDim.x, nnb = gridDim.y;
  const int nwg = nmb * nnb * gridDim.z;
  // XCD-aware order (conv_x3_kernel's): one contiguous run of virtual ids per XCD — grid: N
  // tiles of one M tile, then neighbouring M tiles (whose patches overlap), then the K split;
  // stream: neighbouring ranges
  const int wid = xcd_order(blockIdx.x + nmb * (blockIdx.y + nnb * blockIdx.z), nwg);
  int kt_begin, kt_end, mb = 0, nb = 0, zb = 0;
  if constexpr (STREAM) {
    kt_begin = (int)sk_begin(p, wid, nwg);
    kt_end = (int)sk_begin(p, wid + 1, nwg);
  } else {
    nb = p.raster ? (wid / nmb) % nnb : wid % nnb;
    mb = p.raster ? wid % nmb : (wid / nnb) % nmb;
    zb = wid / (nnb * nmb);
    kt_begin = 0;
    kt_end = p.kc_tap * HALO_TAPS;
    if (p.ktiles_per_split > 0) {  // whole chunks per split (multiple of 9 K-steps)
      kt_begin = zb * p.ktiles_per_split;
      kt_end = min(kt_end, kt_begin + p.ktiles_per_split);
    }
  }
  if (wave >= 4)
    halo_producer<BM, BN, CAT, STREAM, WMAX, NB>(p, smem, kt_begin, kt_end, wave - 4, lane, mb,
                                                 nb);
  else
    halo_consumer<BM, BN, WM, WN, STREAM, WMAX, NB>(p, smem, kt_begin, kt_end, wave, lane, mb,
                                                    nb, zb, wid);
}

// schedules: tile, consumer-wave grid, widest map, filter slab buffers
struct HaloCfg { int bm, bn, wm, wn, wmax, nb; };
inline constexpr HaloCfg kHalo[] = {
    {256, 128, 2, 2, HALO_WMAX, 3}, {128, 256, 2, 2, HALO_WMAX, 3}, {128, 128, 2, 2, HALO_WMAX, 3},
    {256, 64, 4, 1, HALO_WMAX, 3},  {128, 160, 4, 1, HALO_WMAX, 3},
    // two workgroups per CU on maps up to 28 wide (the 28^2 / 14^2 decoder and ResNet convs)
    {128, 128, 2, 2, 28, 2},        {128, 64, 2, 2, 28, 2},
    // ... and up to 56 wide (smaller tiles: the 56^2 band is BM + 114 rows)
    {128, 64, 2, 2, HALO_WMAX, 2},  {64, 128, 2, 2, HALO_WMAX, 2},
};
constexpr int kNumHalo = (int)(sizeof(kHalo) / sizeof(kHalo[0]));

template <int BM, int BN, int WM, int WN, int WMAX, int NB>
static void halo_launch(GemmConvParams& p, int splits, int sk_grid, hipStream_t st) {
  if (sk_grid > 0) {  // tile stream (+ the fixup of the tiles cut between workgroups)
    const dim3 grid(sk_grid);
    if (p.c2) conv_x3_halo_kernel<BM, BN, WM, WN, true, true, WMAX, NB><<<grid, 512, 0, st>>>(p);
    else conv_x3_halo_kernel<BM, BN, WM, WN, false, true, WMAX, NB><<<grid, 512, 0, st>>>(p);
    if (!p.sk_align)
      x3_stream_fixup_kernel<BM, BN, WM><<<dim3(sk_grid, WM), 256, 0, st>>>(p, sk_grid);
    return;
  }
  const dim3 grid(cdiv(p.M, BM), cdiv(p.N, BN), splits);
  if (p.c2) conv_x3_halo_kernel<BM, BN, WM, WN, true, false, WMAX, NB><<<grid, 512, 0, st>>>(p);
  else conv_x3_halo_kernel<BM, BN, WM, WN, false, false, WMAX, NB><<<grid, 512, 0, st>>>(p);
}

}  // namespace x3
}  // namespace pld

using namespace pld;

extern "C" int pld__x3_num_halo(void) { return x3::kNumHalo; }
// the widest input map schedule cfg takes (0: no such schedule)
extern "C" int pld__x3_halo_wmax(int cfg) {
  return cfg >= 0 && cfg < x3::kNumHalo ? x3::kHalo[cfg].wmax : 0;
}
// 1: two workgroups per CU (double-buffered filter slab)
extern "C" int pld__x3_halo_occ2(int cfg) {
  return cfg >= 0 && cfg < x3::kNumHalo && x3::kHalo[cfg].nb == 2;
}
extern "C" int pld__x3_halo_dims(int cfg, int* bm, int* bn, int* tm, int* tn) {
  if (cfg < 0 || cfg >= x3::kNumHalo) return PLD_ERR_ARG;
  const x3::HaloCfg& c = x3::kHalo[cfg];
  *bm = c.bm;
  *bn = c.bn;
  *tm = c.bm / c.wm / 32;
  *tn = c.bn / c.wn / 32;
  return PLD_OK;
}
// eligibility (FWD view): 3x3 stride 1 'same' geometry, no input prologue, maps up to
// HALO_WMAX wide, channel counts in 8s, 32-bit buffer offsets
extern "C" int pld__x3_halo_ok(const GemmConvParams* p) {
  return p->kh == 3 && p->kw == 3 && p->sh == 1 && p->sw == 1 && p->oh == p->h &&
         p->ow == p->w && p->in_scale == nullptr && p->pt >= 0 && p->pt <= 2 && p->pl >= 0 &&
         p->pl <= 2 && p->w <= x3::HALO_WMAX && p->c1 % 8 == 0 && p->c2 % 8 == 0 &&
         p->K == 9 * p->C && (long)p->n * p->h * p->w * std::max(p->c1, p->c2) * 4 < MAX_RECORDS &&
         (long)p->N * p->K * 4 < MAX_RECORDS;
}
// kc_tap / kc1 / ktiles_per_split / zstride / out1 (grid) or sk_* (sk_grid > 0: the tile
// stream, planned by pld__x3_halo_stream_plan) are the caller's (pld's run_fwd_gemm)
extern "C" int pld__x3_halo_launch(GemmConvParams* p, int cfg, int splits, int sk_grid,
                                   void* stream) {
  if (!pld__x3_halo_ok(p) || cfg < 0 || cfg >= x3::kNumHalo || p->w > x3::kHalo[cfg].wmax ||
      !p->bsplit || splits < 1 ||
      p->kc_tap <= 0 || (p->ktiles_per_split % x3::HALO_TAPS) != 0 ||
      (sk_grid > 0 && (p->sk_nk != p->kc_tap * x3::HALO_TAPS || p->sk_q != x3::HALO_TAPS ||
                       p->sk_tiles <= 0 || (!p->sk_align && !p->sk_slab)))) {
    set_error("conv_x3_halo: ineligible geometry or schedule %d", cfg);
    return PLD_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  // grid order: M tiles fastest where the filter outgrows an XCD's 4 MB L2 (every N panel
  // re-read per M tile otherwise); PLD_HALO_RASTER=0/1 forces one (A/B)
  static const int raster_env = [] {
    const char* e = std::getenv("PLD_HALO_RASTER");
    return e ? std::atoi(e) : -1;
  }();
  p->raster = raster_env >= 0 ? raster_env : ((long)p->N * p->K * 4 > (4L << 20) ? 1 : 0);
  switch (cfg) {
    case 0: x3::halo_launch<256, 128, 2, 2, x3::HALO_WMAX, 3>(*p, splits, sk_grid, st); break;
    case 1: x3::halo_launch<128, 256, 2, 2, x3::HALO_WMAX, 3>(*p, splits, sk_grid, st); break;
    case 2: x3::halo_launch<128, 128, 2, 2, x3::HALO_WMAX, 3>(*p, splits, sk_grid, st); break;
    case 3: x3::halo_launch<256, 64, 4, 1, x3::HALO_WMAX, 3>(*p, splits, sk_grid, st); break;
    case 4: x3::halo_launch<128, 160, 4, 1, x3::HALO_WMAX, 3>(*p, splits, sk_grid, st); break;
    case 5: x3::halo_launch<128, 128, 2, 2, 28, 2>(*p, splits, sk_grid, st); break;
    case 6: x3::halo_launch<128, 64, 2, 2, 28, 2>(*p, splits, sk_grid, st); break;
    case 7: x3::halo_launch<128, 64, 2, 2, x3::HALO_WMAX, 2>(*p, splits, sk_grid, st); break;
    default: x3::halo_launch<64, 128, 2, 2, x3::HALO_WMAX, 2>(*p, splits, sk_grid, st); break;
  }
  return check_launch("conv_x3_halo_kernel");
}
// the tile-stream plan (fills p->sk_*; returns the grid): T tiles of kc_tap units (chunks of 9
// K-steps) cut evenly over one resident workgroup per CU, at least 4 units each; whole tiles
// per workgroup only where that divides evenly (then no fixup)
extern "C" int pld__x3_halo_stream_plan(GemmConvParams* p, int cfg) {
  int bm, bn, tm, tn;
  if (pld__x3_halo_dims(cfg, &bm, &bn, &tm, &tn)) return 0;
  const long tiles = (long)cdiv(p->M, bm) * cdiv(p->N, bn);
  const long units = tiles * p->kc_tap;
  p->sk_nk = p->kc_tap * x3::HALO_TAPS;
  p->sk_tiles = (int)tiles;
  p->sk_nnb = (int)cdiv(p->N, bn);
  p->sk_q = x3::HALO_TAPS;
  const long G = std::max<long>(1, std::min<long>(256L * (x3::kHalo[cfg].nb == 2 ? 2 : 1),
                                                  units / 4));
  p->sk_align = (tiles % G == 0) ? 1 : 0;
  // P-way interleaved tile order where each workgroup walks P >= 2 tiles (sk_tile);
  // PLD_HALO_PERM=0 keeps the plain order (A/B)
  static const int perm_env = [] {
    const char* e = std::getenv("PLD_HALO_PERM");
    return e ? std::atoi(e) : 1;
  }();
  p->sk_perm = perm_env && tiles >= 2 * G ? (int)((tiles + G / 2) / G) : 0;
  return (int)G;
}
extern "C" size_t pld__x3_halo_stream_slab_bytes(int cfg, int G, int aligned) {
  int bm, bn, tm, tn;
  if (aligned || pld__x3_halo_dims(cfg, &bm, &bn, &tm, &tn)) return 0;
  return sizeof(float) * 2 * (size_t)G * bm * bn;
}

// The bf16x3 implicit-GEMM tile kernel (conv_x3_kernel) and its launch templates, shared by
// the translation units that instantiate it (conv_x3_grid.hip: tile grids; conv_x3_stream.hip:
// tile streams) and by conv_x3.hip (patch kernels, C-ABI entry points). See conv_x3.hip for the
// arithmetic and the structure.
#pragma once
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "conv_common.h"


namespace pld {
namespace x3 {

constexpr int BK = 32;

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// two floats -> packed bf16 (hi pair, lo pair)
__device__ __forceinline__ void split2(float x, float y, unsigned& hi, unsigned& lo) {
  const bf16x2 h = {(__bf16)x, (__bf16)y};
  hi = __builtin_bit_cast(unsigned, h);
  const float xr = x - __uint_as_float(hi << 16);
  const float yr = y - __uint_as_float(hi & 0xffff0000u);
  const bf16x2 l = {(__bf16)xr, (__bf16)yr};
  lo = __builtin_bit_cast(unsigned, l);
}

// byte offset of 16-byte k-chunk `c` of row `r` inside one plane. The chunk is stored in slot
// c ^ g(r), g(r) = (r1 ^ r3) | r2 << 1 (r_i = bit i of r): conflict-free for the ds_read_b128
// fragment reads (16-lane groups of rows, one chunk) and for the producers' ds_write_b128 of 8
// consecutive rows (searched exhaustively over linear GF(2) swizzles of the row bits).
__device__ __forceinline__ int chunk_off(int r, int c) {
  const int g = (((r >> 1) ^ (r >> 3)) & 1) | ((r >> 1) & 2);
  return r * 64 + 16 * (c ^ g);
}

__device__ __forceinline__ bf16x8 lds_frag(const unsigned char* plane, int r, int c) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(plane + chunk_off(r, c)));
}

// WGRAD image: [32 k rows][R columns] bf16 per plane. A transposed read (4 consecutive k rows x
// 32 bytes per 16-lane group, the second group 32 bytes further) must touch distinct banks:
// with a row pitch that is a multiple of 256 B (R = 32, 64, 128, 256) the 32-byte column blocks
// are XOR-swizzled by 2(k & 3); a pitch of 320, 192 or 448 B (R = 160, 96, 224) already puts the
// four rows 16 banks apart; R = 192 (384 B: rows alternate between two bank offsets) swaps block
// pairs on k & 2.
template <int R>
__device__ __forceinline__ int tr_off(int k, int col) {
  constexpr int NB = R / 16;  // 32-byte blocks per row
  static_assert(R % 32 == 0 && R >= 32 && R <= 256, "WGRAD image width");
  int sw = 0;
  if constexpr ((NB & (NB - 1)) == 0) sw = ((k & 3) << 1) & (NB - 1);
  else if constexpr (NB == 12) sw = k & 2;
  const int b = (col >> 4) ^ sw;
  return k * (2 * R) + b * 32 + (col & 15) * 2;
}

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

// 32x32x16 operand fragment from a [k][col] image with ds_read_b64_tr_b16: lane l needs
// column c0 + (l & 31), k = 16 s + 8 (l >> 5) .. +7; each 16-lane group reads 4 k-rows x 16
// columns per instruction (lane 4q+p supplies row q, columns 4p..4p+3) and receives its column
template <int R>
__device__ __forceinline__ bf16x8 lds_frag_tr(const unsigned char* plane, int c0, int s,
                                              int lane) {
  const int i16 = lane & 15, grp = (lane >> 4) & 1, h = lane >> 5;
  const int k = 16 * s + 8 * h + (i16 >> 2);
  const int col = c0 + 16 * grp + 4 * (i16 & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4s*)(plane + tr_off<R>(k, col)));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4s*)(plane + tr_off<R>(k + 4, col)));
  const v4s v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v);
}

// LDS hand-off between the producer and consumer waves: the writer's ds_writes are complete
// (lgkmcnt) before the barrier; no vmcnt wait, so the producers' next global loads stay in
// flight across it. The empty asm statements keep the compiler from moving LDS accesses across.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM, int BN>
struct X3Smem {
  static constexpr int A_PLANE = BM * 64, B_PLANE = BN * 64;  // bytes of one bf16 plane
  static constexpr int A_BYTES = 2 * A_PLANE, B_BYTES = 2 * B_PLANE;
  static constexpr int BYTES = 2 * (A_BYTES + B_BYTES);         // double-buffered
  __device__ static unsigned char* a(unsigned char* s, int buf) { return s + buf * A_BYTES; }
  __device__ static unsigned char* b(unsigned char* s, int buf) {
    return s + 2 * A_BYTES + buf * B_BYTES;
  }
};

// ---------------------------------------------------------------------------- producer
// Four waves (pw = 0..3) stage K-steps: global fp32 -> bf16 hi/lo -> LDS. Every K-step issues
// the same, unconditional set of loads (the concat's second source is a template parameter, the
// last steps re-fetch the final tile), so the compiler can count the loads in flight and wait
// for exactly one stage (vmcnt(N)), never draining the prefetch (vmcnt(0)).
template <int BM, int BN, int MODE, bool CAT, bool TI, bool PRO, bool STREAM>
__device__ __forceinline__ void x3_producer(const GemmConvParams& p, unsigned char* smem,
                                            int g_begin, int g_end, int nk, int pw, int lane,
                                            int mb0, int nb0) {
  using S = X3Smem<BM, BN>;
  const int ptid = pw * 64 + lane;

  // x1/x2 addressed relative to the first image this workgroup touches (32-bit offsets); a
  // tile-stream workgroup walks many tiles, its descriptors span the whole tensors (the host
  // keeps them under 2 GiB)
  int img_base = 0, pix_base = 0;
  if (!STREAM) {
    if (MODE == MODE_FWD) {
      img_base = (int)p.dOH.div(p.dOW.div((uint32_t)(mb0 * BM)));
    } else {
      pix_base = g_begin * BK;
      img_base = (int)p.dOH.div(p.dOW.div((uint32_t)min(pix_base, p.K - 1)));
    }
  }
  const long img_elems = (long)p.h * p.w;
  const __amdgpu_buffer_rsrc_t rs1 =
      make_rsrc(p.x1 + img_base * img_elems * p.c1, (p.n - img_base) * img_elems * p.c1 * 4);
  const __amdgpu_buffer_rsrc_t rs2 =
      CAT ? make_rsrc(p.x2 + img_base * img_elems * p.c2, (p.n - img_base) * img_elems * p.c2 * 4)
          : rs1;
  // FWD: B is the pre-split filter (pld_filter_split layout); WGRAD: B = dY fp32
  const __amdgpu_buffer_rsrc_t rsb =
      (MODE == MODE_FWD)
          ? make_rsrc(p.bsplit, (long)p.N * p.K * 4)
          : make_rsrc(p.bmat + (long)pix_base * p.N, (long)(p.K - pix_base) * p.N * 4);

  // FWD: full-line staging. A wave-instruction covers 8 rows x 128 B: lane = (row lr = lane/8,
  // 4-k group ks = lane%8); producer wave pw owns rows [pw BM/4, (pw+1) BM/4) of A and
  // [pw BN/4, ...) of B, in groups of 8. B lanes 0-31 stage the hi halves, 32-63 the lo halves
  // of 8 rows x 4 chunks (chunk = 32 B: [8 hi][8 lo] bf16).
  static_assert(MODE != MODE_FWD || (BM % 32 == 0 && BN % 32 == 0), "FWD tiles: rows % 32");
  constexpr int FA = BM / 32, FB = BN / 32;
  const int lr = lane >> 3, ks = lane & 7;
  const int br = lane & 31, half = lane >> 5;
  // per A row: pixel index of tap (0,0) relative to the descriptor base, and the taps that land
  // inside the image (bit t, taps <= 32); per B row: byte offset and validity
  int a_base[FA];
  unsigned a_taps[FA];
  unsigned b_off[FB];
  bool b_ok[FB];
  // WGRAD: a thread owns 16 consecutive columns (fixed channels: one tap, one source, since
  // C, c1 % 16 == 0) of P pixel slots g, g + G, ... of each K-step (NQ = R/16 threads per pixel
  // row, G = floor(256/NQ) rows per pass, P = ceil(32/G); threads past row 31, and the
  // 256 mod NQ threads past the last full pass, idle). One pixel decomposition serves 16
  // channels; lanes run along a pixel row: 64-byte coalesced loads, and each thread fills one
  // whole 32-byte block of the [k][col] image read back transposed.
  constexpr int NQA = BM / 16, NQB = BN / 16;
  constexpr int GA = 256 / NQA, GB = 256 / NQB;
  constexpr int PA = (BK + GA - 1) / GA, PB = (BK + GB - 1) / GB;
  static_assert(MODE == MODE_FWD || (BM >= 32 && BN >= 32 && BM <= 256 && BN <= 256),
                "WGRAD tile columns must be 32..256");
  int w_ty = 0, w_tx = 0, w_ci = 0;
  bool w_ok = false, w_in1 = true;
  int w_cs = 0;                // WGRAD concat: this thread's source channel count and
  const float* w_src = p.x1;   // its first channel's address in the workgroup's first image
  int w_n = 0;                 // WGRAD: this thread's first dY column

  // per-thread row / column state of tile (mb, nb)
  auto setup = [&](int mb, int nb) {
  const int m0 = mb * BM;
  const int n0 = nb * BN;
  if (MODE == MODE_FWD) {
#pragma unroll
    for (int j = 0; j < FA; ++j) {
      const int r = pw * (BM / 4) + 8 * j + lr;
      const int m = m0 + r;
      const bool mok = m < p.M;
      const int mm = mok ? m : m0;
      const uint32_t q = p.dOW.div((uint32_t)mm);
      const int ox = mm - (int)q * p.ow;
      const uint32_t img = p.dOH.div(q);
      const int oy = (int)q - (int)img * p.oh;
      const int iy0 = oy * p.sh - p.pt, ix0 = ox * p.sw - p.pl;
      a_base[j] = (((int)img - img_base) * p.h + iy0) * p.w + ix0;
      unsigned t = 0;
      for (int ty = 0; ty < p.kh; ++ty)
        for (int tx = 0; tx < p.kw; ++tx)
          t |= (unsigned)(mok && (unsigned)(iy0 + ty) < (unsigned)p.h &&
                          (unsigned)(ix0 + tx) < (unsigned)p.w) << (ty * p.kw + tx);
      a_taps[j] = t;
    }
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int nn = n0 + pw * (BN / 4) + 8 * j + (br >> 2);
      b_ok[j] = nn < p.N;
      b_off[j] = (unsigned)(b_ok[j] ? nn : 0) * (unsigned)p.K * 4u + 16u * half;
    }
  } else {
    const int i = m0 + 16 * (ptid % NQA);
    w_ok = i < p.M;
    const int ii = w_ok ? i : 0;
    const uint32_t tap = p.dC.div((uint32_t)ii);
    w_ci = ii - (int)tap * p.C;
    const uint32_t ty = p.dKW.div(tap);
    w_ty = (int)ty;
    w_tx = (int)tap - (int)ty * p.kw;
    w_in1 = w_ci < p.c1;
    w_cs = w_in1 ? p.c1 : p.c2;
    w_src = w_in1 ? p.x1 + img_base * img_elems * p.c1 + w_ci
                  : p.x2 + img_base * img_elems * p.c2 + (w_ci - p.c1);
    w_n = n0 + 16 * (ptid % NQB);
  }
  };
  // tile-stream: the tile of the next load and its first global step
  int tile_g0 = 0, next_switch = STREAM ? g_begin : 0x7fffffff;
  if (!STREAM) setup(mb0, nb0);

  constexpr int RA = (MODE == MODE_FWD) ? FA : 4 * PA;  // float4 staging registers, A
  constexpr int RB = (MODE == MODE_FWD) ? FB : 4 * PB;  // and B
  struct Stage {  // one K-step in flight
    float4 ra[RA], rb[RB];
    float4 ps, pt;  // PRO: this lane's 4 channels' prologue scale / shift
    unsigned okm;   // PRO: bit j = A row j's element lies inside the image (else it stays 0)
  };
  static_assert(!PRO || (MODE == MODE_FWD && !CAT), "prologue: one-source FWD view only");

  auto load_tile = [&](int g, Stage& st) {
    if (STREAM && g >= next_switch) {  // wave-uniform: a new tile's row / column state
      const int t = g / nk;
      setup(t / p.sk_nnb, t % p.sk_nnb);
      tile_g0 = t * nk;
      next_switch = tile_g0 + nk;
    }
    const int kt = g - tile_g0;
    const int k0 = kt * BK;
    if (MODE == MODE_FWD && TI) {
      // tap-inner order: K-step kt = (chunk kq, tap) with the chunks of x1 first, then x2, each
      // 32 channels of ONE source (ragged last chunk masked): one load per element and the
      // source's descriptor picked per step (wave-uniform), where the linear order needs both
      const int kq = (int)p.dTaps.div((uint32_t)kt);
      const int tap = kt - kq * p.kh * p.kw;
      const bool s2 = CAT && kq >= p.kc1;
      const int chb = (s2 ? kq - p.kc1 : kq) * BK;  // first channel of the chunk in its source
      const int cs = s2 ? p.c2 : p.c1;
      const __amdgpu_buffer_rsrc_t rs = s2 ? rs2 : rs1;
      const int c = chb + 4 * ks;
      const bool kin = c < cs;
      const int ty = (int)p.dKW.div((uint32_t)tap);
      const int toff = ty * p.w + (tap - ty * p.kw);  // pixel offset of the tap
      unsigned okm = 0;
#pragma unroll
      for (int j = 0; j < FA; ++j) {
        const bool ok = kin && ((a_taps[j] >> tap) & 1u);
        okm |= (unsigned)ok << j;
        st.ra[j] = bload4(rs, ok ? (unsigned)(((a_base[j] + toff) * cs + c) * 4) : OOB);
      }
      if constexpr (PRO) {  // unconditional loads (clamped channel): no branch around them
        const int cc = kin ? c : 0;
        st.ps = *reinterpret_cast<const float4*>(p.in_scale + cc);
        st.pt = *reinterpret_cast<const float4*>(p.in_shift + cc);
        st.okm = okm;
      }
      const int cb8 = chb + 8 * (br & 3);  // this lane's 8-k chunk of the filter
      const int kc = tap * p.C + (s2 ? p.c1 : 0) + cb8;
      const bool kcin = cb8 < cs;
#pragma unroll
      for (int j = 0; j < FB; ++j)
        st.rb[j] = bload4(rsb, (b_ok[j] && kcin) ? b_off[j] + 4u * (unsigned)kc : OOB);
    } else if (MODE == MODE_FWD) {
      const int k = k0 + 4 * ks;  // this lane's 4 consecutive k (C % 8 == 0: one tap, one source)
      const bool kin = k < p.K;
      const int kk = kin ? k : 0;
      const int tap = (int)p.dC.div((uint32_t)kk);
      const int ci = kk - tap * p.C;
      const int ty = (int)p.dKW.div((uint32_t)tap);
      const int toff = ty * p.w + (tap - ty * p.kw);  // pixel offset of the tap
      const bool src2 = CAT && ci >= p.c1;
      const int cs = src2 ? p.c2 : p.c1;
      const int cb = src2 ? ci - p.c1 : ci;
      unsigned okm = 0;
#pragma unroll
      for (int j = 0; j < FA; ++j) {
        const bool ok = kin && ((a_taps[j] >> tap) & 1u);
        okm |= (unsigned)ok << j;
        const unsigned off = (unsigned)(((a_base[j] + toff) * cs + cb) * 4);
        if (CAT)  // both sources, the other one out of range (reads as 0)
          st.ra[j] = add4(bload4(rs1, (ok && !src2) ? off : OOB), bload4(rs2, (ok && src2) ? off : OOB));
        else
          st.ra[j] = bload4(rs1, ok ? off : OOB);
      }
      if constexpr (PRO) {
        const int cc = kin ? cb : 0;
        st.ps = *reinterpret_cast<const float4*>(p.in_scale + cc);
        st.pt = *reinterpret_cast<const float4*>(p.in_shift + cc);
        st.okm = okm;
      }
      const int kc = k0 + 8 * (br & 3);
      const bool kcin = kc < p.K;
#pragma unroll
      for (int j = 0; j < FB; ++j)
        st.rb[j] = bload4(rsb, (b_ok[j] && kcin) ? b_off[j] + 4u * (unsigned)kc : OOB);
    } else {
      const int ga = ptid / NQA;
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int slot = ga + GA * j;
        const int pix = k0 + slot;
        const bool rok = ga < GA && slot < BK && pix < p.K;
        const int pp = rok ? pix : pix_base;
        const uint32_t q = p.dOW.div((uint32_t)pp);
        const int ox = pp - (int)q * p.ow;
        const uint32_t img = p.dOH.div(q);
        const int oy = (int)q - (int)img * p.oh;
        const int ir = ((int)img - img_base) * p.h;
        const int iy = oy * p.sh - p.pt + w_ty, ix = ox * p.sw - p.pl + w_tx;
        const bool ok = rok && w_ok && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
        const int px = (ir + iy) * p.w + ix;
        if (CAT) {  // this thread's source is fixed: one (per-lane address) load per element;
                    // masked lanes re-read their first 16 channels and zero the data
          const float4* a = reinterpret_cast<const float4*>(w_src + (ok ? px * w_cs : 0));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float4 v = a[u];
            st.ra[4 * j + u] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        } else {
          const unsigned o1 = ok ? (unsigned)((px * p.c1 + w_ci) * 4) : OOB;
#pragma unroll
          for (int u = 0; u < 4; ++u) st.ra[4 * j + u] = bload4(rs1, o1 == OOB ? OOB : o1 + 16 * u);
        }
      }
      const int gb = ptid / NQB;
      const int n = w_n;
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int slot = gb + GB * j;
        const int pix = k0 + slot;
        const bool ok = gb < GB && slot < BK && pix < p.K && n < p.N;
        const unsigned o = ok ? (unsigned)(((pix - pix_base) * p.N + n) * 4) : OOB;
#pragma unroll
        for (int u = 0; u < 4; ++u) st.rb[4 * j + u] = bload4(rsb, o == OOB ? OOB : o + 16 * u);
      }
    }
  };

  // 16 columns of one k row -> one 32-byte block in each plane of the [k][col] image
  auto store_row16 = [&](unsigned char* plane, int plane_bytes, auto rcols, int k, int col,
                         const float4* v) {
    unsigned h[8], l[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      split2(v[u].x, v[u].y, h[2 * u], l[2 * u]);
      split2(v[u].z, v[u].w, h[2 * u + 1], l[2 * u + 1]);
    }
    const int o = tr_off<decltype(rcols)::value>(k, col);
    *reinterpret_cast<u32x4*>(plane + o) = u32x4{h[0], h[1], h[2], h[3]};
    *reinterpret_cast<u32x4*>(plane + o + 16) = u32x4{h[4], h[5], h[6], h[7]};
    *reinterpret_cast<u32x4*>(plane + plane_bytes + o) = u32x4{l[0], l[1], l[2], l[3]};
    *reinterpret_cast<u32x4*>(plane + plane_bytes + o + 16) = u32x4{l[4], l[5], l[6], l[7]};
  };

  auto store_tile = [&](int buf, const Stage& st) {
    unsigned char* A = S::a(smem, buf);
    unsigned char* B = S::b(smem, buf);
    if (MODE == MODE_FWD) {
      const int ob = 8 * (ks & 1);  // byte offset of this lane's 4 k inside its 16-byte chunk
#pragma unroll
      for (int j = 0; j < FA; ++j) {
        const int r = pw * (BM / 4) + 8 * j + lr;
        float4 v = st.ra[j];
        if constexpr (PRO)
          v = ((st.okm >> j) & 1u) ? prologue4(p.in_act, v, st.ps, st.pt)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        unsigned h0, l0, h1, l1;
        split2(v.x, v.y, h0, l0);
        split2(v.z, v.w, h1, l1);
        const int o = chunk_off(r, ks >> 1) + ob;
        *reinterpret_cast<u32x2*>(A + o) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(A + S::A_PLANE + o) = u32x2{l0, l1};
      }
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int r = pw * (BN / 4) + 8 * j + (br >> 2);
        *reinterpret_cast<float4*>(B + half * S::B_PLANE + chunk_off(r, br & 3)) = st.rb[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int slot = ptid / NQA + GA * j;
        if (ptid / NQA < GA && slot < BK)
          store_row16(A, S::A_PLANE, std::integral_constant<int, BM>{}, slot,
                      16 * (ptid % NQA), &st.ra[4 * j]);
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int slot = ptid / NQB + GB * j;
        if (ptid / NQB < GB && slot < BK)
          store_row16(B, S::B_PLANE, std::integral_constant<int, BN>{}, slot,
                      16 * (ptid % NQB), &st.rb[4 * j]);
      }
    }
  };

  // Two register stages: K-step i+1 is stored while i runs on the MFMAs and its registers are
  // refilled with step i+3 (clamped to the last step: a harmless re-fetch) — every global load
  // has two K-steps of MFMA work to land. Barriers (match the consumer): 1 + n.
  const int n = g_end - g_begin;
  if (n <= 0) {
    lds_barrier();
    return;
  }
  const int last = g_end - 1;
  Stage s0, s1;
  load_tile(g_begin, s0);
  store_tile(0, s0);
  load_tile(min(g_begin + 1, last), s0);
  load_tile(min(g_begin + 2, last), s1);
  lds_barrier();
  for (int i = 0;; i += 2) {
    store_tile(1, s0);  // step i+1 (odd) -> buffer 1 (unused past the end)
    load_tile(min(g_begin + i + 3, last), s0);
    lds_barrier();
    if (i + 1 >= n) break;
    store_tile(0, s1);  // step i+2 (even) -> buffer 0
    load_tile(min(g_begin + i + 4, last), s1);
    lds_barrier();
    if (i + 2 >= n) break;
  }
}

// ---------------------------------------------------------------------------- consumer
// a tile-stream workgroup's raw partial sums of a tile cut between workgroups: slab
// [wid][slot][BM][BN] (slot 0 = the workgroup's first tile, 1 = its last), row-major
template <int TM, int TN, int BM, int BN>
__device__ __forceinline__ void store_partial(const GemmConvParams& p,
                                              const floatx16 (&acc)[TM][TN], int r_w, int c_w,
                                              int lane, long wid, int slot) {
  // one per-lane byte offset; each element's constant offset rides in the SGPR operand (plain
  // per-element addresses cost ~100 VGPRs across the tile stream's K loop)
  const __amdgpu_buffer_rsrc_t rs =
      make_rsrc(p.sk_slab + (wid * 2 + slot) * (long)(BM * BN), (long)BM * BN * 4);
  const int h = lane >> 5, l32 = lane & 31;
  const unsigned voff = (unsigned)(((r_w + 4 * h) * BN + c_w + l32) * 4);
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // (through a scalar: hipcc/ROCm 7.2 reads element 0 for __builtin_bit_cast of a
        // vector-element lvalue)
        const float v = acc[a][b][r];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff,
                                              ((a * 32 + (r & 3) + 8 * (r >> 2)) * BN + b * 32) * 4,
                                              0);
      }
}

// Grid-schedule epilogue: after the last K-step barrier the staging buffers are free and each
// consumer wave owns a private region, so its sums go out through store_acc_staged (LDS, 16-byte
// streaming row stores) where the output takes whole float4 quads. The short-K 1x1 convs are
// epilogue-heavy: 192 -> 1152 at 14^2 x 32: 22.9 -> 18.3 us, the other 1x1 shapes -6 to -12 %,
// 3x3 decoder convs unchanged (profiles/r04_epilogue_store_ab.txt: plain 16-B stores 20.0,
// write-through 19.1).
template <int BM, int BN, int WM, int WN, int MODE, bool STREAM>
__device__ __forceinline__ void x3_consumer(const GemmConvParams& p, unsigned char* smem,
                                            int g_begin, int g_end, int nk, int wave, int lane,
                                            int mb0, int nb0, int zb, int wid) {
  using S = X3Smem<BM, BN>;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, l32 = lane & 31;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  struct Frags {
    bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
  };
  auto read_frags = [&](const unsigned char* A, const unsigned char* B, int s, Frags& f) {
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      if constexpr (MODE == MODE_WGRAD) {
        f.ah[a] = lds_frag_tr<BM>(A, wm * WTM + a * 32, s, lane);
        f.al[a] = lds_frag_tr<BM>(A + S::A_PLANE, wm * WTM + a * 32, s, lane);
      } else {
        const int r = wm * WTM + a * 32 + l32;
        f.ah[a] = lds_frag(A, r, 2 * s + h);
        f.al[a] = lds_frag(A + S::A_PLANE, r, 2 * s + h);
      }
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      if constexpr (MODE == MODE_WGRAD) {
        f.bh[b] = lds_frag_tr<BN>(B, wn * WTN + b * 32, s, lane);
        f.bl[b] = lds_frag_tr<BN>(B + S::B_PLANE, wn * WTN + b * 32, s, lane);
      } else {
        const int r = wn * WTN + b * 32 + l32;
        f.bh[b] = lds_frag(B, r, 2 * s + h);
        f.bl[b] = lds_frag(B + S::B_PLANE, r, 2 * s + h);
      }
    }
  };
  auto mfmas = [&](const Frags& f) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.al[a], f.bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[a], f.bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[a], f.bh[b], acc[a][b], 0, 0, 0);
      }
  };
  Frags f0;

  lds_barrier();
  // one segment per tile the range touches (the whole range when !STREAM); the epilogue sits
  // between segments, outside the K loop (fragment registers dead there)
  int g = g_begin;
  while (g < g_end) {
    const int t = STREAM ? g / nk : 0;
    const int seg_end = STREAM ? min(g_end, (t + 1) * nk) : g_end;
    if (g != g_begin) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    }
    for (; g < seg_end; ++g) {
      const int buf = (g - g_begin) & 1;
      const unsigned char* A = S::a(smem, buf);
      const unsigned char* B = S::b(smem, buf);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        read_frags(A, B, s, f0);
        // keep the substep's fragment reads together ahead of its MFMAs (one LDS wait per
        // substep instead of the scheduler's register-saving read-wait-MFMA interleave)
        __builtin_amdgcn_sched_barrier(0);
        mfmas(f0);
      }
      lds_barrier();
    }
    if constexpr (STREAM) {
      const int mb = t / p.sk_nnb, nb = t - mb * p.sk_nnb;
      if (t * nk >= g_begin && (t + 1) * nk <= g_end)
        store_acc<TM, TN>(p, acc, mb * BM + wm * WTM, nb * BN + wn * WTN, lane);
      else
        store_partial<TM, TN, BM, BN>(p, acc, wm * WTM, wn * WTN, lane, wid,
                                      t == g_begin / nk ? 0 : 1);
    }
  }
  if constexpr (!STREAM) {
    if constexpr (4 * 32 * (WTN + 8) * 4 <= S::BYTES) {
      if (staged_ok(p)) {
        const int m_w = mb0 * BM + wm * WTM, n_w = nb0 * BN + wn * WTN;
        if (p.stats) acc_stats<TM, TN>(p, acc, m_w, n_w, lane);
        store_acc_staged<TM, TN>(p, acc, m_w, n_w, lane,
                                 reinterpret_cast<float*>(smem) + wave * 32 * (WTN + 8));
        return;
      }
    }
    store_acc<TM, TN>(p, acc, mb0 * BM + wm * WTM, nb0 * BN + wn * WTN, lane, zb);
  }
}

// 512 threads: waves 0-3 consume (LDS fragments -> MFMA), waves 4-7 produce the next K-step
// (global loads, prologue, hi/lo split, LDS stores) — a VALU-heavy wave and an MFMA-heavy
// wave share each SIMD, so the split overlaps the matrix work.
//   STREAM = false: grid (M tiles, N tiles, K splits), one tile (or K slice) per workgroup.
//   STREAM = true : 1-D grid of G workgroups, each walking a contiguous range of the
//     (tile, K-step) space (GemmConvParams sk_*): the pipeline runs on across tile boundaries
//     (no per-tile prologue / drain: the short-K 1x1 convs), and a non-aligned range balances
//     long-K convs whose tile count does not fill the 256 CUs (stream-K).
template <int BM, int BN, int WM, int WN, int MODE, bool CAT, bool TI, bool PRO = false,
          bool STREAM = false>
__global__ __launch_bounds__((WM * WN + 4) * 64) void conv_x3_kernel(GemmConvParams p) {
  static_assert(WM * WN == 4, "4 consumer waves");
  static_assert((BM / WM) % 32 == 0 && (BN / WN) % 32 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) unsigned char smem[X3Smem<BM, BN>::BYTES];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs (b, b+8, ... share one),
  // so each XCD gets a contiguous run of virtual ids: for the tile grid N fastest, then M, then
  // the K split — the N tiles of one M tile (same A rows) and neighbouring M tiles (overlapping
  // im2col halos) share that XCD's L2; for the tile stream, neighbouring ranges. Bijective for
  // any grid size (speed only, never correctness).
  const int nmb = gridDim.x, nnb = gridDim.y;
  const int nwg = nmb * nnb * gridDim.z;
  const int flat = blockIdx.x + nmb * (blockIdx.y + nnb * blockIdx.z);
  const int xcd = flat & 7, slot = flat >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  if constexpr (STREAM) {
    const int g_begin = (int)sk_begin(p, wid, nwg), g_end = (int)sk_begin(p, wid + 1, nwg);
    if (wave >= WM * WN)
      x3_producer<BM, BN, MODE, CAT, TI, PRO, true>(p, smem, g_begin, g_end, p.sk_nk,
                                                    wave - WM * WN, lane, 0, 0);
    else
      x3_consumer<BM, BN, WM, WN, MODE, true>(p, smem, g_begin, g_end, p.sk_nk, wave, lane, 0,
                                              0, 0, wid);
    return;
  }
  const int nb = wid % nnb;
  const int mb = (wid / nnb) % nmb;
  const int zb = wid / (nnb * nmb);
  int kt_begin = 0, kt_end = p.kc_tap ? p.kc_tap * p.kh * p.kw : (p.K + BK - 1) / BK;
  if (p.ktiles_per_split > 0) {
    kt_begin = zb * p.ktiles_per_split;
    kt_end = min(kt_end, kt_begin + p.ktiles_per_split);
  }
  if (wave >= WM * WN)
    x3_producer<BM, BN, MODE, CAT, TI, PRO, false>(p, smem, kt_begin, kt_end, 0x7fffffff,
                                                   wave - WM * WN, lane, mb, nb);
  else
    x3_consumer<BM, BN, WM, WN, MODE, false>(p, smem, kt_begin, kt_end, 0x7fffffff, wave, lane,
                                             mb, nb, zb, wid);
}

// The tile-stream schedule's fixup (non-aligned ranges): per tile cut between workgroups and
// per wave row tile of it (blockIdx.y: BM / WM rows), one workgroup sums the cut pieces' raw
// partials in K order (fixed: deterministic), then applies conv_x3_kernel's epilogue — bias,
// concat routing, accumulate, the BN statistics partial of that wave row tile (store_acc's
// layout); thread = column, 4 rows in flight. Launched on the same stream right after the main
// kernel (its slabs are complete).
template <int BM, int BN, int WM>
__global__ __launch_bounds__(256) void x3_stream_fixup_kernel(GemmConvParams p, int G) {
  static_assert(BN <= 256, "one column per thread");
  constexpr int WTM = BM / WM;
  const int j = blockIdx.x, wm = blockIdx.y;  // the cut at the start of workgroup j's range
  const long nk = p.sk_nk, S = (long)p.sk_tiles * nk;
  const long s = sk_begin(p, j, G);
  if (j == 0 || s >= S || s % nk == 0) return;
  const long t = s / nk, ts = t * nk;
  if (sk_begin(p, j - 1, G) > ts) return;  // an earlier cut of the same tile handles it
  const long c0 = sk_owner(p, ts, G), c1 = sk_owner(p, ts + nk - 1, G);
  const int col = threadIdx.x;
  const int ta = sk_tile(p, (int)t);
  const int mb = ta / p.sk_nnb, nb = ta - mb * p.sk_nnb;
  const int gc = nb * BN + col;
  if (col >= BN || gc >= p.N) return;
  const float bias = p.bias ? p.bias[gc] : 0.f;
  const bool first = gc < p.split;  // two-way column routing (dgrad of a concat)
  float* base = first ? p.out1 + gc : p.out2 + (gc - p.split);
  const long ld = first ? p.ld1 : p.ld2;
  const int accum = first ? p.acc1 : p.acc2;
  const int r0 = wm * WTM, rows = min(WTM, p.M - mb * BM - r0);
  double s1 = 0.0, s2 = 0.0;
  for (int r = 0; r < rows; r += 4) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (long c = c0; c <= c1; ++c) {
      const int slot = (t == sk_begin(p, c, G) / nk) ? 0 : 1;
      const float* sl = p.sk_slab + (c * 2 + slot) * (long)(BM * BN) + (r0 + r) * BN + col;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += (r + u < rows) ? sl[u * BN] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (r + u >= rows) break;
      const float y = v[u] + bias;
      float* d = base + (long)(mb * BM + r0 + r + u) * ld;
      *d = accum ? *d + y : y;
      s1 += (double)y;
      s2 += (double)y * (double)y;
    }
  }
  if (p.stats)
    *reinterpret_cast<double2*>(p.stats + ((long)gc * p.stats_parts + mb * WM + wm) * 2) =
        make_double2(s1, s2);
}

// ------------------------------------------------------------------------ schedules
struct Cfg { int bm, bn, tm, tn, occ; };
// occ: resident blocks per CU (LDS 2 (BM+BN) 128 B of 160 KiB; registers). tm x tn: 32x32 MFMA
// tiles per consumer wave.
inline constexpr Cfg kCfg[] = {
    {256, 32, 2, 1, 2},  {128, 64, 2, 1, 3},  {128, 96, 1, 3, 2},  {128, 128, 2, 2, 2},
    {128, 160, 1, 5, 2}, {128, 192, 1, 6, 1}, {128, 224, 1, 7, 1}, {256, 64, 2, 2, 1},
    {256, 128, 4, 2, 1}, {128, 256, 2, 4, 1},
    // short-M / long-K launches (the encoder's 14x14 and 28x28 1x1 convs at batch 32: 147-294
    // tiles of 128 x 64 leave most of the 256 CUs idle): 4x the workgroups, 4 resident per CU
    {64, 64, 1, 1, 4},
    // short-M launches with narrow-but-not-tiny N (N = 112..320 at M = 6272 / 25088): one
    // workgroup covers 2-3x the columns of a 64 x 64 tile, so the A strip is staged once per
    // 128 / 192 columns instead of once per 64
    {64, 128, 1, 2, 3},  {64, 192, 1, 3, 2},
};
constexpr int kNumCfg = (int)(sizeof(kCfg) / sizeof(kCfg[0]));

template <int MODE, int BM, int BN, int WM, int WN>
inline void launch_cfg_grid(GemmConvParams& p, int splits, hipStream_t st) {
  constexpr int T = (WM * WN + 4) * 64;
  dim3 grid(cdiv(p.M, BM), cdiv(p.N, BN), splits);
  if constexpr (MODE == MODE_FWD) {
    if (p.in_scale) {  // one source (x3_fwd_geom)
      if (p.kc_tap) conv_x3_kernel<BM, BN, WM, WN, MODE, false, true, true><<<grid, T, 0, st>>>(p);
      else conv_x3_kernel<BM, BN, WM, WN, MODE, false, false, true><<<grid, T, 0, st>>>(p);
      return;
    }
  }
  if (MODE == MODE_FWD && p.kc_tap) {
    if (p.c2) conv_x3_kernel<BM, BN, WM, WN, MODE, true, true><<<grid, T, 0, st>>>(p);
    else conv_x3_kernel<BM, BN, WM, WN, MODE, false, true><<<grid, T, 0, st>>>(p);
  } else {
    if (p.c2) conv_x3_kernel<BM, BN, WM, WN, MODE, true, false><<<grid, T, 0, st>>>(p);
    else conv_x3_kernel<BM, BN, WM, WN, MODE, false, false><<<grid, T, 0, st>>>(p);
  }
}

// tile stream (no input prologue: the host keeps those on the grid)
template <int MODE, int BM, int BN, int WM, int WN>
inline void launch_cfg_stream(GemmConvParams& p, int sk_grid, hipStream_t st) {
  constexpr int T = (WM * WN + 4) * 64;
  const dim3 grid(sk_grid);
  if (MODE == MODE_FWD && p.kc_tap) {
    if (p.c2) conv_x3_kernel<BM, BN, WM, WN, MODE, true, true, false, true><<<grid, T, 0, st>>>(p);
    else conv_x3_kernel<BM, BN, WM, WN, MODE, false, true, false, true><<<grid, T, 0, st>>>(p);
  } else {
    if (p.c2) conv_x3_kernel<BM, BN, WM, WN, MODE, true, false, false, true><<<grid, T, 0, st>>>(p);
    else conv_x3_kernel<BM, BN, WM, WN, MODE, false, false, false, true><<<grid, T, 0, st>>>(p);
  }
  if (!p.sk_align)
    x3_stream_fixup_kernel<BM, BN, WM><<<dim3(sk_grid, WM), 256, 0, st>>>(p, sk_grid);
}

// schedule cfg -> (BM, BN, WM, WN): kCfg's tiles with their consumer-wave grids
#define PLD_X3_DISPATCH(cfg, CALL)  \
  switch (cfg) {                    \
    case 0: CALL(256, 32, 4, 1); break;  \
    case 1: CALL(128, 64, 2, 2); break;  \
    case 2: CALL(128, 96, 4, 1); break;  \
    case 3: CALL(128, 128, 2, 2); break; \
    case 4: CALL(128, 160, 4, 1); break; \
    case 5: CALL(128, 192, 4, 1); break; \
    case 6: CALL(128, 224, 4, 1); break; \
    case 7: CALL(256, 64, 4, 1); break;  \
    case 8: CALL(256, 128, 2, 2); break; \
    case 9: CALL(128, 256, 2, 2); break; \
    case 10: CALL(64, 64, 2, 2); break;  \
    case 11: CALL(64, 128, 2, 2); break; \
    default: CALL(64, 192, 2, 2); break; \
  }

}  // namespace x3
}  // namespace pld

// entry points of the instantiating translation units (one per launch family, so the template
// instantiations compile in parallel)
namespace pld {
namespace x3 {
void launch_fwd_grid(GemmConvParams& p, int splits, int cfg, hipStream_t st);
void launch_fwd_stream(GemmConvParams& p, int cfg, int sk_grid, hipStream_t st);
void launch_wgrad_grid(GemmConvParams& p, int splits, int cfg, hipStream_t st);
void launch_wgrad_stream(GemmConvParams& p, int cfg, int sk_grid, hipStream_t st);
}  // namespace x3
}  // namespace pld

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
// K-step (global loads two steps ahead, fused prologue, hi/lo split, LDS stores), so the VALU
// split work of one wave overlaps the matrix work of its SIMD partner. LDS holds, per operand
// and buffer, a hi plane and a lo plane of [rows][4 x 16-byte k-chunks], XOR-swizzled (chunk_off) so that
// the ds_read_b128 fragment reads (lane = row, 16 B = 8 k) and the row-per-lane stores are
// conflict-free. Double-buffered, one barrier per K-step.
//   FWD staging: wave w owns k-chunk w (8 consecutive k = 8 channels of one tap and one source,
//     since C % 8 == 0), lane = row: the tap decomposition, the concat source and the fused
//     input prologue's scale/shift are wave-uniform (scalar registers, one descriptor). A filter
//     pre-split by pld_filter_split is staged as-is (no conversion).
//   WGRAD staging: a thread owns 4 consecutive rows (channels) x P consecutive pixels and
//     transposes them in registers into P-wide k runs of the 4 rows.
#include <algorithm>
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

// act(x*s+t) on N values, the activation switch hoisted out of the element loop
template <int N>
__device__ __forceinline__ void prologue_n(int act, float (&e)[N], const float* s, const float* t) {
  switch (act) {
    case ACT_RELU:
#pragma unroll
      for (int u = 0; u < N; ++u) e[u] = fmaxf(e[u] * s[u] + t[u], 0.f);
      break;
    case ACT_SWISH:
#pragma unroll
      for (int u = 0; u < N; ++u) {
        const float z = e[u] * s[u] + t[u];
        e[u] = z * sigmoidf_(z);
      }
      break;
    case ACT_SIGMOID:
#pragma unroll
      for (int u = 0; u < N; ++u) e[u] = sigmoidf_(e[u] * s[u] + t[u]);
      break;
    default:
#pragma unroll
      for (int u = 0; u < N; ++u) e[u] = e[u] * s[u] + t[u];
  }
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
// Four waves (pw = 0..3) stage K-steps: global fp32 -> (prologue) -> bf16 hi/lo -> LDS.
template <int BM, int BN, int MODE>
__device__ __forceinline__ void x3_producer(const GemmConvParams& p, unsigned char* smem,
                                            int kt_begin, int kt_end, int pw, int lane) {
  using S = X3Smem<BM, BN>;
  const int ptid = pw * 64 + lane;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;

  // x1/x2 addressed relative to the first image this workgroup touches (32-bit offsets)
  int img_base, pix_base = 0;
  if (MODE == MODE_FWD) {
    img_base = (int)p.dOH.div(p.dOW.div((uint32_t)m0));
  } else {
    pix_base = kt_begin * BK;
    img_base = (int)p.dOH.div(p.dOW.div((uint32_t)min(pix_base, p.K - 1)));
  }
  const long img_elems = (long)p.h * p.w;
  const __amdgpu_buffer_rsrc_t rs1 =
      make_rsrc(p.x1 + img_base * img_elems * p.c1, (p.n - img_base) * img_elems * p.c1 * 4);
  const __amdgpu_buffer_rsrc_t rs2 =
      p.c2 ? make_rsrc(p.x2 + img_base * img_elems * p.c2, (p.n - img_base) * img_elems * p.c2 * 4)
           : make_rsrc(p.x1, 0);
  const bool bsplit = MODE == MODE_FWD && p.bsplit != nullptr;  // B already hi/lo split
  const __amdgpu_buffer_rsrc_t rsb =
      (MODE == MODE_FWD)
          ? make_rsrc(bsplit ? p.bsplit : p.bmat, (long)p.N * p.K * 4)
          : make_rsrc(p.bmat + (long)pix_base * p.N, (long)(p.K - pix_base) * p.N * 4);

  // FWD: lane = row (rows lane + 64 j), wave pw = k-chunk pw of the K-step
  constexpr int FA = (BM + 63) / 64, FB = (BN + 63) / 64;
  int a_ir[FA], a_iy0[FA], a_ix0[FA];
  bool a_ok[FA];
  // WGRAD: thread = 4 rows (quad) x P consecutive pixels
  constexpr int QA = BM / 4, QB = BN / 4;
  constexpr int GA = 256 / QA, GB = 256 / QB;
  constexpr int PA = BK / GA, PB = BK / GB;
  static_assert(MODE == MODE_FWD || (GA * PA == BK && GB * PB == BK && PA >= 1 && PB >= 1),
                "WGRAD tile rows must be 32..256");
  int w_ty = 0, w_tx = 0, w_ci = 0;
  bool w_ok = false, w_in1 = true, wpro = false;
  float wsc[4] = {0.f, 0.f, 0.f, 0.f}, wsh[4] = {0.f, 0.f, 0.f, 0.f};

  if (MODE == MODE_FWD) {
#pragma unroll
    for (int j = 0; j < FA; ++j) {
      const int r = lane + 64 * j;
      const int m = m0 + r;
      a_ok[j] = (r < BM) && (m < p.M);
      const int mm = a_ok[j] ? m : m0;
      const uint32_t q = p.dOW.div((uint32_t)mm);
      const int ox = mm - (int)q * p.ow;
      const uint32_t img = p.dOH.div(q);
      const int oy = (int)q - (int)img * p.oh;
      a_ir[j] = ((int)img - img_base) * p.h;
      a_iy0[j] = oy * p.sh - p.pt;
      a_ix0[j] = ox * p.sw - p.pl;
    }
  } else {
    const int i = m0 + 4 * (ptid % QA);
    w_ok = i < p.M;
    const int ii = w_ok ? i : 0;
    const uint32_t tap = p.dC.div((uint32_t)ii);
    w_ci = ii - (int)tap * p.C;
    const uint32_t ty = p.dKW.div(tap);
    w_ty = (int)ty;
    w_tx = (int)tap - (int)ty * p.kw;
    w_in1 = w_ci < p.c1;
    wpro = p.in_scale && w_ok && w_in1;
    if (wpro) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        wsc[u] = p.in_scale[w_ci + u];
        wsh[u] = p.in_shift[w_ci + u];
      }
    }
  }

  constexpr int RA = (MODE == MODE_FWD) ? 2 * FA : PA;  // float4 staging registers, A
  constexpr int RB = (MODE == MODE_FWD) ? 2 * FB : PB;  // and B
  // one K-step in flight: its staging registers and per-step flags
  struct Stage {
    float4 ra[RA], rb[RB];
    unsigned vmask;
    bool fpro;  // FWD: the prologue applies to this K-step's chunk (wave-uniform)
    int fci;    // FWD: first channel of the chunk (prologue coefficients)
  };

  auto load_tile = [&](int kt, Stage& st) {
    float4* ra = st.ra;
    float4* rb = st.rb;
    unsigned& vmask = st.vmask;
    const int k0 = kt * BK;
    vmask = 0;
    if (MODE == MODE_FWD) {
      const int k = k0 + 8 * pw;  // wave-uniform
      const bool kin = k < p.K;
      const int kk = kin ? k : 0;
      const int tap = (int)p.dC.div((uint32_t)kk);
      const int ci = kk - tap * p.C;
      const int ty = (int)p.dKW.div((uint32_t)tap);
      const int tx = tap - ty * p.kw;
      const bool src2 = ci >= p.c1;
      const int cs = src2 ? p.c2 : p.c1;
      const int cb = src2 ? ci - p.c1 : ci;
      const __amdgpu_buffer_rsrc_t rs = src2 ? rs2 : rs1;
#pragma unroll
      for (int j = 0; j < FA; ++j) {
        const int iy = a_iy0[j] + ty, ix = a_ix0[j] + tx;
        const bool ok = kin && a_ok[j] && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
        const unsigned off = ok ? (unsigned)((((a_ir[j] + iy) * p.w + ix) * cs + cb) * 4) : OOB;
        ra[2 * j] = bload4(rs, off);
        ra[2 * j + 1] = bload4(rs, ok ? off + 16 : OOB);
        vmask |= (unsigned)ok << j;
      }
      st.fpro = p.in_scale && kin && !src2;
      st.fci = ci;
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int r = lane + 64 * j;
        const int n = n0 + r;
        const bool ok = kin && r < BN && n < p.N;
        const unsigned off = ok ? (unsigned)((n * p.K + k) * 4) : OOB;
        rb[2 * j] = bload4(rsb, off);
        rb[2 * j + 1] = bload4(rsb, ok ? off + 16 : OOB);
      }
    } else {
      const int ga = ptid / QA;
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int pix = k0 + PA * ga + j;
        const bool rok = pix < p.K;
        const int pp = rok ? pix : pix_base;
        const uint32_t q = p.dOW.div((uint32_t)pp);
        const int ox = pp - (int)q * p.ow;
        const uint32_t img = p.dOH.div(q);
        const int oy = (int)q - (int)img * p.oh;
        const int ir = ((int)img - img_base) * p.h;
        const int iy = oy * p.sh - p.pt + w_ty, ix = ox * p.sw - p.pl + w_tx;
        const bool ok = rok && w_ok && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
        const int px = (ir + iy) * p.w + ix;
        float4 v = bload4(rs1, (ok && w_in1) ? (unsigned)((px * p.c1 + w_ci) * 4) : OOB);
        if (p.c2)
          v = add4(v, bload4(rs2, (ok && !w_in1) ? (unsigned)((px * p.c2 + w_ci - p.c1) * 4) : OOB));
        ra[j] = v;
        vmask |= (unsigned)ok << j;
      }
      const int gb = ptid / QB;
      const int n = n0 + 4 * (ptid % QB);
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int pix = k0 + PB * gb + j;
        const bool ok = pix < p.K && n < p.N;
        rb[j] = bload4(rsb, ok ? (unsigned)(((pix - pix_base) * p.N + n) * 4) : OOB);
      }
    }
  };

  // rows of 4-row quads x P k values -> P-wide runs in the hi and lo planes
  auto store_quad = [&](unsigned char* plane, int plane_bytes, int q, int g, auto& e) {
    constexpr int P = sizeof(e[0]) / sizeof(float);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = 4 * q + u;
      const int slot = P * g;
      const int o = chunk_off(r, slot >> 3) + 2 * (slot & 7);
      if constexpr (P == 1) {
        const __bf16 hv = (__bf16)e[u][0];
        const __bf16 lv = (__bf16)(e[u][0] - (float)hv);
        *reinterpret_cast<__bf16*>(plane + o) = hv;
        *reinterpret_cast<__bf16*>(plane + plane_bytes + o) = lv;
      } else {
        unsigned hi[P / 2], lo[P / 2];
#pragma unroll
        for (int t = 0; t < P / 2; ++t) split2(e[u][2 * t], e[u][2 * t + 1], hi[t], lo[t]);
        if constexpr (P == 2) {
          *reinterpret_cast<unsigned*>(plane + o) = hi[0];
          *reinterpret_cast<unsigned*>(plane + plane_bytes + o) = lo[0];
        } else if constexpr (P == 4) {
          *reinterpret_cast<u32x2*>(plane + o) = u32x2{hi[0], hi[1]};
          *reinterpret_cast<u32x2*>(plane + plane_bytes + o) = u32x2{lo[0], lo[1]};
        } else {
          *reinterpret_cast<u32x4*>(plane + o) = u32x4{hi[0], hi[1], hi[2], hi[3]};
          *reinterpret_cast<u32x4*>(plane + plane_bytes + o) = u32x4{lo[0], lo[1], lo[2], lo[3]};
        }
      }
    }
  };

  auto store_tile = [&](int buf, const Stage& st) {
    const float4* ra = st.ra;
    const float4* rb = st.rb;
    const unsigned vmask = st.vmask;
    const bool fpro = st.fpro;
    const int fci = st.fci;
    unsigned char* A = S::a(smem, buf);
    unsigned char* B = S::b(smem, buf);
    if (MODE == MODE_FWD) {
      float sc[8], sh[8];
      if (fpro) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          sc[u] = p.in_scale[fci + u];
          sh[u] = p.in_shift[fci + u];
        }
      }
#pragma unroll
      for (int j = 0; j < FA; ++j) {
        const int r = lane + 64 * j;
        if (r >= BM) continue;
        float e[8] = {ra[2 * j].x, ra[2 * j].y, ra[2 * j].z, ra[2 * j].w,
                      ra[2 * j + 1].x, ra[2 * j + 1].y, ra[2 * j + 1].z, ra[2 * j + 1].w};
        if (fpro && ((vmask >> j) & 1u)) prologue_n<8>(p.in_act, e, sc, sh);
        unsigned hs[4], ls[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) split2(e[2 * u], e[2 * u + 1], hs[u], ls[u]);
        const int o = chunk_off(r, pw);
        *reinterpret_cast<u32x4*>(A + o) = u32x4{hs[0], hs[1], hs[2], hs[3]};
        *reinterpret_cast<u32x4*>(A + S::A_PLANE + o) = u32x4{ls[0], ls[1], ls[2], ls[3]};
      }
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int r = lane + 64 * j;
        if (r >= BN) continue;
        const int o = chunk_off(r, pw);
        if (bsplit) {  // chunk = [8 hi][8 lo] bf16, as written by pld_filter_split
          *reinterpret_cast<float4*>(B + o) = rb[2 * j];
          *reinterpret_cast<float4*>(B + S::B_PLANE + o) = rb[2 * j + 1];
        } else {
          const float e[8] = {rb[2 * j].x, rb[2 * j].y, rb[2 * j].z, rb[2 * j].w,
                              rb[2 * j + 1].x, rb[2 * j + 1].y, rb[2 * j + 1].z, rb[2 * j + 1].w};
          unsigned hs[4], ls[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) split2(e[2 * u], e[2 * u + 1], hs[u], ls[u]);
          *reinterpret_cast<u32x4*>(B + o) = u32x4{hs[0], hs[1], hs[2], hs[3]};
          *reinterpret_cast<u32x4*>(B + S::B_PLANE + o) = u32x4{ls[0], ls[1], ls[2], ls[3]};
        }
      }
    } else {
      {
        float e[4][PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) {
          float v[4] = {ra[j].x, ra[j].y, ra[j].z, ra[j].w};
          if (wpro && ((vmask >> j) & 1u)) prologue_n<4>(p.in_act, v, wsc, wsh);
#pragma unroll
          for (int u = 0; u < 4; ++u) e[u][j] = v[u];
        }
        store_quad(A, S::A_PLANE, ptid % QA, ptid / QA, e);
      }
      {
        float e[4][PB];
#pragma unroll
        for (int j = 0; j < PB; ++j) {
          e[0][j] = rb[j].x; e[1][j] = rb[j].y; e[2][j] = rb[j].z; e[3][j] = rb[j].w;
        }
        store_quad(B, S::B_PLANE, ptid % QB, ptid / QB, e);
      }
    }
  };

  // Two register stages: K-step i+1 is stored while i runs on the MFMAs, and its registers
  // are refilled with step i+3 — every global load has two K-steps of MFMA work to land.
  // Barrier schedule (matches the consumer): 1 + n barriers.
  const int n = kt_end - kt_begin;
  Stage s0, s1;
  if (n > 0) {
    load_tile(kt_begin, s0);
    store_tile(0, s0);
  }
  if (n > 1) load_tile(kt_begin + 1, s0);
  if (n > 2) load_tile(kt_begin + 2, s1);
  lds_barrier();
  for (int i = 0; i < n; i += 2) {
    if (i + 1 < n) {
      store_tile(1, s0);  // step i+1 (odd) -> buffer 1
      if (i + 3 < n) load_tile(kt_begin + i + 3, s0);
    }
    lds_barrier();
    if (i + 1 < n) {
      if (i + 2 < n) {
        store_tile(0, s1);  // step i+2 (even) -> buffer 0
        if (i + 4 < n) load_tile(kt_begin + i + 4, s1);
      }
      lds_barrier();
    }
  }
}

// ---------------------------------------------------------------------------- consumer
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void x3_consumer(const GemmConvParams& p, unsigned char* smem,
                                            int kt_begin, int kt_end, int wave, int lane) {
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

  lds_barrier();
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    const unsigned char* A = S::a(smem, buf);
    const unsigned char* B = S::b(smem, buf);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int r = wm * WTM + a * 32 + l32;
        ah[a] = lds_frag(A, r, 2 * s + h);
        al[a] = lds_frag(A + S::A_PLANE, r, 2 * s + h);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int r = wn * WTN + b * 32 + l32;
        bh[b] = lds_frag(B, r, 2 * s + h);
        bl[b] = lds_frag(B + S::B_PLANE, r, 2 * s + h);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    }
    lds_barrier();
  }
  store_acc<TM, TN>(p, acc, blockIdx.x * BM + wm * WTM, blockIdx.y * BN + wn * WTN, lane);
}

// 512 threads: waves 0-3 consume (LDS fragments -> MFMA), waves 4-7 produce the next K-step
// (global loads, prologue, hi/lo split, LDS stores) — a VALU-heavy wave and an MFMA-heavy
// wave share each SIMD, so the split overlaps the matrix work.
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(512) void conv_x3_kernel(GemmConvParams p) {
  static_assert(WM * WN == 4, "4 consumer waves");
  static_assert((BM / WM) % 32 == 0 && (BN / WN) % 32 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) unsigned char smem[X3Smem<BM, BN>::BYTES];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int kt_begin = 0, kt_end = (p.K + BK - 1) / BK;
  if (p.ktiles_per_split > 0) {
    kt_begin = blockIdx.z * p.ktiles_per_split;
    kt_end = min(kt_end, kt_begin + p.ktiles_per_split);
  }
  if (wave >= 4) x3_producer<BM, BN, MODE>(p, smem, kt_begin, kt_end, wave - 4, lane);
  else x3_consumer<BM, BN, WM, WN>(p, smem, kt_begin, kt_end, wave, lane);
}

// ------------------------------------------------------------------------ schedules
struct Cfg { int bm, bn, tm, tn, occ; };
// occ: resident 512-thread blocks per CU (LDS 2 (BM+BN) 128 B of 160 KiB; registers)
static const Cfg kCfg[] = {
    {256, 32, 2, 1, 2},  {128, 64, 2, 1, 3},  {128, 96, 1, 3, 2},  {128, 128, 2, 2, 2},
    {128, 160, 1, 5, 2}, {128, 192, 1, 6, 1}, {128, 224, 1, 7, 1}, {256, 64, 2, 2, 1},
    {256, 128, 4, 2, 1}, {128, 256, 2, 4, 1},
};
constexpr int kNumCfg = (int)(sizeof(kCfg) / sizeof(kCfg[0]));

// WGRAD stages rows as 4-row quads x P pixels: BM and BN must be powers of two in [32, 256]
constexpr bool pow2_rows(int r) { return r == 32 || r == 64 || r == 128 || r == 256; }

template <int MODE, int BM, int BN, int WM, int WN>
static void launch_cfg(GemmConvParams& p, int splits, hipStream_t st) {
  if constexpr (MODE == MODE_FWD || (pow2_rows(BM) && pow2_rows(BN))) {
    dim3 grid(cdiv(p.M, BM), cdiv(p.N, BN), splits);
    conv_x3_kernel<BM, BN, WM, WN, MODE><<<grid, 512, 0, st>>>(p);
  }
}

template <int MODE>
static void launch(GemmConvParams& p, int splits, int cfg, hipStream_t st) {
  switch (cfg) {
    case 0: launch_cfg<MODE, 256, 32, 4, 1>(p, splits, st); break;
    case 1: launch_cfg<MODE, 128, 64, 2, 2>(p, splits, st); break;
    case 2: launch_cfg<MODE, 128, 96, 4, 1>(p, splits, st); break;
    case 3: launch_cfg<MODE, 128, 128, 2, 2>(p, splits, st); break;
    case 4: launch_cfg<MODE, 128, 160, 4, 1>(p, splits, st); break;
    case 5: launch_cfg<MODE, 128, 192, 4, 1>(p, splits, st); break;
    case 6: launch_cfg<MODE, 128, 224, 4, 1>(p, splits, st); break;
    case 7: launch_cfg<MODE, 256, 64, 4, 1>(p, splits, st); break;
    case 8: launch_cfg<MODE, 256, 128, 2, 2>(p, splits, st); break;
    default: launch_cfg<MODE, 128, 256, 2, 2>(p, splits, st); break;
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
extern "C" int pld__x3_wgrad_cfg_ok(int cfg) {
  return cfg >= 0 && cfg < x3::kNumCfg && x3::pow2_rows(x3::kCfg[cfg].bm) &&
         x3::pow2_rows(x3::kCfg[cfg].bn);
}
extern "C" int pld__x3_launch(GemmConvParams* p, int mode, int splits, int cfg, void* stream) {
  if (mode == MODE_WGRAD && !pld__x3_wgrad_cfg_ok(cfg)) {
    set_error("conv_x3: schedule %d is not a WGRAD tile", cfg);
    return PLD_ERR_ARG;
  }
  if (mode == MODE_FWD) x3::launch<MODE_FWD>(*p, splits, cfg, as_stream(stream));
  else x3::launch<MODE_WGRAD>(*p, splits, cfg, as_stream(stream));
  return check_launch("conv_x3_kernel");
}

// Wide 1x1 convolutions on bf16x3 MFMA: out[m][n] = sum_k a[m][k] * w[n][k] for the 1x1,
// stride-1 convs whose reduction is short (K <= 128) and whose output is wide — the
// EfficientNetB0 expand convs of stages 3-6 (40->240, 80->480, 112->672; pl_hourglass.py:52-57
// via Keras EfficientNetB0) and the data-gradients of the project convs (240->40 backward is
// 40->240 ...). Their cost is the output write (6-12 floats written per float read), and
// the im2col tile kernel (conv_x3.hip) reaches only ~2 TB/s on them: 1-4 K-steps per tile leave
// its producer/consumer pipeline all prologue and epilogue.
//
// Here a workgroup streams 32-row strips of `a` (each one contiguous 32*K-float block) through
// LDS for a fixed group of output columns, warp-specialised like conv_x3.hip: 2 loader waves
// fetch strip j+2 with fully coalesced 16-byte loads, split strip j+1 into bf16 hi/lo and store
// it as an LDS image, while 4 compute waves — each holding the filter fragments of its NT
// 32-column tiles in VGPRs for the whole launch — read strip j's A fragments and run 3 MFMAs per
// 16-k substep (same bf16x3 arithmetic as conv_x3.hip), then store their tiles straight from
// the accumulators. One barrier per strip. Loads and stores live in different waves, so neither
// waits on the other's vmcnt. Workgroups of one strip set are dealt to one XCD (the column
// groups' re-reads of a strip hit that XCD's L2).
// Optional epilogue: the BatchNormalization batch statistics of the output (sum, sum of squares
// per column: fp32 over a lane's 16 rows of a strip, fp64 across strips), written as fp64
// partials [N][strip groups][2] in bn.hip's finalize layout — the output is never read back.
// Algorithmic bytes: M*K*4 read + M*N*4 written (+ read when accumulating).
#include <cstdlib>

#include "conv_common.h"

namespace pld {
namespace w1 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 8 floats -> bf16 hi = rne(v), lo = rne(v - hi)
__device__ __forceinline__ void split8(float4 a, float4 b, bf16x8& hi, bf16x8& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const __bf16 h = (__bf16)v[i];
    hi[i] = h;
    lo[i] = (__bf16)(v[i] - (float)h);
  }
}

// 4 floats -> packed bf16 hi / lo quads (8 bytes each)
__device__ __forceinline__ void split4(float4 v, u32x2& hi, u32x2& lo) {
  const float f[4] = {v.x, v.y, v.z, v.w};
  unsigned short hs[4], ls[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const __bf16 h = (__bf16)f[i];
    hs[i] = __builtin_bit_cast(unsigned short, h);
    ls[i] = __builtin_bit_cast(unsigned short, (__bf16)(f[i] - (float)h));
  }
  hi = u32x2{hs[0] | (unsigned)hs[1] << 16, hs[2] | (unsigned)hs[3] << 16};
  lo = u32x2{ls[0] | (unsigned)ls[1] << 16, ls[2] | (unsigned)ls[3] << 16};
}

// LDS hand-off (as conv_x3.hip): the writers' ds_writes complete, no vmcnt wait — the loader
// waves' prefetches stay in flight across the barrier
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int NC = 4;  // compute waves per workgroup
constexpr int NL = 2;  // loader waves per workgroup
constexpr int OLS = 40;  // row pitch (floats) of a compute wave's output staging tile

// LDS strip image: [32 rows][16 KS k] bf16 per plane (hi, lo), row pitch 32 KS + 16 bytes (an
// odd multiple of 16: the 16-lane groups of a fragment read hit 16 distinct 16-byte slots)
template <int KS>
struct Strip {
  static constexpr int RS = 32 * KS + 16, PLANE = 32 * RS, BYTES = 2 * PLANE;
};

template <int KS, int NT, bool ACC>
__global__ __launch_bounds__((NC + NL) * 64) void wide1x1_kernel(
    const float* __restrict__ a, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ out, int M, int K, int N, double* __restrict__ stats, int nsx, int ncy) {
  using S = Strip<KS>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * S::BYTES];
  __shared__ __attribute__((aligned(16))) float obuf[NC][32 * OLS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware order (workgroups are dealt round-robin to the 8 XCDs): each XCD gets a contiguous
  // run of (strip group, column group) ids, column group fastest
  const int nwg = gridDim.x, flat = blockIdx.x;
  const int xcd = flat & 7, slot = flat >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int cy = wid % ncy, sx = wid / ncy;
  const int nstrips = (M + 31) / 32;
  const int n = (nstrips - sx + nsx - 1) / nsx;  // strips sx, sx + nsx, ... of this workgroup
  // (grid = nsx x ncy exactly, sx < nsx <= nstrips: n >= 1 for every workgroup)

  if (wave >= NC) {
    // ---- loader waves: strip j (rows 32 (sx + j nsx) ..) -> hi/lo bf16 LDS image. Thread
    // float4 e = lt + 64 NL i covers row e / (4 KS), k 4 (e % (4 KS)) of the K-padded image
    // (NQ = KS per thread exactly): every load and LDS store is unconditional — pad columns and
    // rows past M load zeros through the descriptor — so hipcc counts vmcnt precisely
    const int lt = threadIdx.x - NC * 64;
    static_assert(64 * NL == 128, "two loader waves");
    constexpr int NQ = KS;
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(a, (long)M * K * 4);
    const int k4 = K / 4;
    auto load = [&](int j, float4 (&v)[NQ]) {
      const int row0 = 32 * (sx + min(j, n - 1) * nsx);
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int e = lt + 128 * i;
        const int r = e / (4 * KS), c = e % (4 * KS);
        const bool ok = c < k4 && row0 + r < M;
        // volatile (aux bit 31): the load stays where it is issued — a load sunk into the next
        // stage's code puts the two paths into the loop header out of order, and hipcc then
        // falls back to near-vmcnt(0) waits
        v[i] = __builtin_bit_cast(
            float4, __builtin_amdgcn_raw_buffer_load_b128(
                        ra, ok ? (unsigned)(((row0 + r) * K + 4 * c) * 4) : OOB, 0,
                        (int)0x80000000u));
      }
    };
    auto store = [&](int buf, const float4 (&v)[NQ]) {
      unsigned char* hi = smem + buf * S::BYTES;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int e = lt + 128 * i;
        const int r = e / (4 * KS), c = e % (4 * KS);
        u32x2 h, l;
        split4(v[i], h, l);
        *reinterpret_cast<u32x2*>(hi + r * S::RS + 8 * c) = h;
        *reinterpret_cast<u32x2*>(hi + S::PLANE + r * S::RS + 8 * c) = l;
      }
    };
    // two register stages (as conv_x3.hip's producer): strip i+1 stored while i is on the
    // MFMAs and its registers refilled with i+3 (clamped past the end);
    // strip j goes to LDS image j & 1; barriers 1 + n (the compute waves' count)
    float4 s0[NQ], s1[NQ];
    load(0, s0);
    store(0, s0);
    load(1, s0);
    load(2, s1);
    lds_barrier();
    for (int i = 0;; i += 2) {
      store(1, s0);
      if (i + 1 >= n) {
        lds_barrier();
        break;
      }
      load(i + 3, s0);
      lds_barrier();
      store(0, s1);
      if (i + 2 >= n) {
        lds_barrier();
        break;
      }
      load(i + 4, s1);
      lds_barrier();
    }
    return;
  }

  // ---- compute waves: NT 32-column tiles each, filter fragments in VGPRs for the launch
  const int h = lane >> 5, l32 = lane & 31;
  const int col0 = (cy * NC + wave) * NT * 32;
  const bool active = col0 < N;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(w, (long)N * K * 4);
  bf16x8 bh[NT][KS], bl[NT][KS];
  float bs[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nn = col0 + 32 * t + l32;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 16 * s + 8 * h;
      const bool ok = nn < N && k < K;
      const unsigned off = (unsigned)(nn * K + k) * 4u;
      split8(bload4(rw, ok ? off : OOB), bload4(rw, ok ? off + 16u : OOB), bh[t][s], bl[t][s]);
    }
    bs[t] = (bias && nn < N) ? bias[nn] : 0.f;
  }
  double s1[NT], s2[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) s1[t] = s2[t] = 0.0;

  // accumulate: the destination rows of strip j are fetched before its MFMAs, so their HBM
  // latency hides under the matrix work instead of stalling every row-segment store
  lds_barrier();
  for (int j = 0; j < n; ++j) {
    if (active) {
      const unsigned char* img = smem + (j & 1) * S::BYTES;
      const int rs = 32 * (sx + j * nsx);
      float4 old[NT][4];
      if constexpr (ACC) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int cq = col0 + 32 * t + 4 * (lane & 7);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rr = (lane >> 3) + 8 * i;
            old[t][i] = (rs + rr < M && cq < N)
                            ? *reinterpret_cast<const float4*>(out + (long)(rs + rr) * N + cq)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
      }
      floatx16 c[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) c[t][r] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int o = l32 * S::RS + 32 * s + 16 * h;
        const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + o));
        const bf16x8 al =
            __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + S::PLANE + o));
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[t][s], c[t], 0, 0, 0);
          c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[t][s], c[t], 0, 0, 0);
          c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[t][s], c[t], 0, 0, 0);
        }
      }
      // lane holds column col0 + 32 t + l32, rows (r & 3) + 8 (r >> 2) + 4 h of the strip; the
      // tile goes out through the wave's LDS buffer (row pitch OLS: the two row groups of a
      // write land 32 banks apart) as float4 rows — each store instruction writes 8 full
      // 128-byte row segments
      float* ob = obuf[wave];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float f1 = 0.f, f2 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
          const float v = c[t][r] + bs[t];
          ob[rr * OLS + l32] = v;
          if (rs + rr < M) {
            f1 += v;
            f2 = fmaf(v, v, f2);
          }
        }
        s1[t] += (double)f1;
        s2[t] += (double)f2;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const int cq = col0 + 32 * t + 4 * (lane & 7);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = (lane >> 3) + 8 * i;
          if (rs + rr < M && cq < N) {
            float4 v = *reinterpret_cast<const float4*>(ob + rr * OLS + 4 * (lane & 7));
            float4* d = reinterpret_cast<float4*>(out + (long)(rs + rr) * N + cq);
            if constexpr (ACC) v = add4(v, old[t][i]);
            *d = v;
          }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
    }
    lds_barrier();
  }
  if (stats && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const double a1 = s1[t] + __shfl_xor(s1[t], 32);
      const double a2 = s2[t] + __shfl_xor(s2[t], 32);
      const int nn = col0 + 32 * t + l32;
      if (h == 0 && nn < N)
        *reinterpret_cast<double2*>(stats + ((long)nn * nsx + sx) * 2) = make_double2(a1, a2);
    }
  }
}

constexpr int MAX_K = 128;

// NT = 32-column tiles per wave: ~64 VGPRs of filter fragments whatever K
constexpr int nt_for(int ks) { return ks <= 4 ? 2 : 1; }

// launch geometry: column groups of 4 waves x NT tiles; strip groups so that ~PER_CU
// workgroups land on each of the 256 CUs (the loop covers the rest)
static void geometry(long M, int K, int N, int& nsx, int& ncy) {
  static const int per_cu = [] {
    const char* e = std::getenv("PLD_WIDE_PER_CU");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 2;
  }();
  const int ks = (K + 15) / 16;
  ncy = (int)cdiv(N, NC * 32 * nt_for(ks));
  const long nstrips = cdiv(M, 32);
  nsx = (int)std::max<long>(1, std::min<long>(nstrips, cdiv(256L * per_cu, ncy)));
}

template <int KS>
static void launch(const float* a, const float* w, const float* bias, float* out, int M, int K,
                   int N, int acc, double* stats, hipStream_t st) {
  int nsx, ncy;
  geometry(M, K, N, nsx, ncy);
  // the accumulating form is its own instantiation: its prefetch registers would otherwise
  // cost the overwrite form occupancy (measured 0.028 -> 0.037 ms on 40 -> 240)
  if (acc)
    wide1x1_kernel<KS, nt_for(KS), true><<<nsx * ncy, (NC + NL) * 64, 0, st>>>(
        a, w, bias, out, M, K, N, stats, nsx, ncy);
  else
    wide1x1_kernel<KS, nt_for(KS), false><<<nsx * ncy, (NC + NL) * 64, 0, st>>>(
        a, w, bias, out, M, K, N, stats, nsx, ncy);
}

}  // namespace w1
}  // namespace pld

using namespace pld;

// (K, N) of the GEMM a wide 1x1 conv runs: fwd K = cin, N = cout; dgrad K = cout, N = cin.
// Taken where the exact-fp32 thin kernel does not apply (pld__thin_ok) and the output is wide.
extern "C" int pld__wide_ok(int K, int N) {
  static const int off = [] {
    const char* e = getenv("PLD_NO_WIDE");  // debug knob: route these to the im2col tiles
    return e && e[0] == '1';
  }();
  return !off && K % 8 == 0 && K >= 8 && K <= w1::MAX_K && N % 4 == 0 && N >= 64 && N >= 2 * K;
}

// stats partials per column of a wide 1x1 GEMM (the strip groups)
extern "C" int pld__wide_stats_parts(long M, int K, int N) {
  int nsx, ncy;
  w1::geometry(M, K, N, nsx, ncy);
  return nsx;
}

// stats: NULL, or [N][pld__wide_stats_parts][2] fp64 BN partials of the output (acc must be 0)
extern "C" int pld__wide_gemm(const float* a, const float* w, const float* bias, float* out,
                              long M, int K, int N, int acc, void* stream, double* stats) {
  PLD_CHECK_ARG(a && w && out && M > 0 && aligned16(a) && aligned16(w) && aligned16(out) &&
                    N % 4 == 0,
                "wide1x1: bad args");
  PLD_CHECK_ARG(M * (long)K < (1L << 29) && M * (long)N < (1L << 31) && (long)N * K < (1L << 29),
                "wide1x1: tensor too large");
  PLD_CHECK_ARG(K % 8 == 0 && K >= 8 && K <= w1::MAX_K, "wide1x1: unsupported K=%d", K);
  PLD_CHECK_ARG(!(stats && acc), "wide1x1: statistics of an accumulated output");
  hipStream_t st = as_stream(stream);
  const int m = (int)M;
  switch ((K + 15) / 16) {
    case 1: w1::launch<1>(a, w, bias, out, m, K, N, acc, stats, st); break;
    case 2: w1::launch<2>(a, w, bias, out, m, K, N, acc, stats, st); break;
    case 3: w1::launch<3>(a, w, bias, out, m, K, N, acc, stats, st); break;
    case 4: w1::launch<4>(a, w, bias, out, m, K, N, acc, stats, st); break;
    case 5: w1::launch<5>(a, w, bias, out, m, K, N, acc, stats, st); break;
    case 6: w1::launch<6>(a, w, bias, out, m, K, N, acc, stats, st); break;
    case 7: w1::launch<7>(a, w, bias, out, m, K, N, acc, stats, st); break;
    default: w1::launch<8>(a, w, bias, out, m, K, N, acc, stats, st); break;
  }
  return check_launch("wide1x1_kernel");
}

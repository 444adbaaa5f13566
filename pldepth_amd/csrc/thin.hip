// Thin 1x1 convolutions: out[m][n] = sum_k a[m][k] * b[n][k] with a small reduction (K <= 48, K % 8
// == 0, N <= 256) — the EfficientNet expand / project convs of the early stages
// (pl_hourglass.py:52-57 via Keras EfficientNetB0: 16->96, 24->144, 40->240 expand; 96->24,
// 144->24, 240->40 project) and their data-gradients. These are HBM-bound (2-9 FMAs per byte),
// so an MFMA tile buys nothing: the 64x32 / 256x32 MFMA tiles re-read `a` once per N tile and
// reach ~3.5 TB/s on them. Here a 256-thread workgroup owns 64 consecutive rows (one contiguous
// 64*K-float block of `a`, read fully coalesced and transposed through LDS so each lane holds
// its row in VGPRs); its 4 waves split the output columns, the filter row of each column is
// wave-uniform (scalar loads: the FMAs take it as an SGPR operand), and the workgroup's whole
// [64][N] output tile goes back through LDS, to be stored as the one contiguous run of `out` it
// is (round 3: the per-wave column chunks wrote 32-64-byte pieces of 64 rows per instruction,
// 3.1-3.6 TB/s on the 16->96 and 24->144 expand convs). Exact fp32 fmaf chains in k order.
#include <algorithm>

#include "common.h"
#include "conv_common.h"

namespace pld {

constexpr int THIN_PAD = 4;  // LDS row padding (floats): spreads the lane-per-row reads over banks

template <int KR, int CH>
__global__ __launch_bounds__(256) void thin1x1_kernel(const float* __restrict__ a,
                                                      const float* __restrict__ b,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ out, int M, int N,
                                                      int acc, double* __restrict__ stats) {
  constexpr int LA = KR + THIN_PAD;  // LDS row stride of the staged a tile
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sa = smem;                  // [64][LA]
  float* so = smem;                  // [64][N + THIN_PAD]: the whole output tile (over sa, once
                                     // every wave holds its row in registers)
  const int LO = N + THIN_PAD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar filter loads
  const long m0 = (long)blockIdx.x * 64;
  const int rows = (int)min(64L, (long)M - m0);
  // stage the contiguous [rows][KR] block of a: float4 index e = tid + 256 j
  constexpr int NV = 64 * KR / 4;
  const float4* src = reinterpret_cast<const float4*>(a + m0 * KR);
  const int nv = rows * KR / 4;
#pragma unroll
  for (int j = 0; j < (NV + 255) / 256; ++j) {
    const int e = tid + 256 * j;
    if (e < NV) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < nv) v = src[e];
      const int r = (4 * e) / KR, c = (4 * e) % KR;
      *reinterpret_cast<float4*>(sa + r * LA + c) = v;
    }
  }
  __syncthreads();
  float x[KR];
#pragma unroll
  for (int k = 0; k < KR; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(sa + lane * LA + k);
    x[k] = v.x; x[k + 1] = v.y; x[k + 2] = v.z; x[k + 3] = v.w;
  }
  __syncthreads();  // sa is dead: the output tile reuses its space (one more block per CU)
  // the 4 waves share the 64 rows and take CH-column chunks round-robin into the LDS tile
  for (int n0 = wave * CH; n0 < N; n0 += 4 * CH) {
    float o[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const float* br = b + (long)(n0 + j) * KR;  // wave-uniform row: scalar loads
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < KR; ++k) s = fmaf(x[k], br[k], s);
      o[j] = bias ? s + bias[n0 + j] : s;
    }
#pragma unroll
    for (int j = 0; j < CH; j += 4)
      *reinterpret_cast<float4*>(so + lane * LO + n0 + j) =
          make_float4(o[j], o[j + 1], o[j + 2], o[j + 3]);
  }
  __syncthreads();
  if (stats) {
    // BN batch statistics of the output (the BatchNormalization that follows the conv): per
    // column, sum and sum of squares over this workgroup's rows in fp64 (thread = column; rows
    // in order). Partials [N][gridDim.x][2] (bn.hip's finalize layout).
    for (int j = tid; j < N; j += 256) {
      double s1 = 0.0, s2 = 0.0;
      for (int r = 0; r < rows; ++r) {
        const double v = (double)so[r * LO + j];
        s1 += v;
        s2 += v * v;
      }
      *reinterpret_cast<double2*>(stats + ((long)j * gridDim.x + blockIdx.x) * 2) =
          make_double2(s1, s2);
    }
  }
  // the tile's rows are one contiguous [rows][N] run of out: fully coalesced float4 stores
  // (chunked per wave, each instruction wrote 32-64-byte pieces of 64 different rows)
  const int nq = N / 4, tq = rows * nq;
  constexpr int U = 4;  // accumulate: U destination quads fetched before their stores
  float4* dst = reinterpret_cast<float4*>(out + m0 * N);
  for (int e0 = tid; e0 < tq; e0 += 256 * U) {
    float4 old[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 256 * u;
      old[u] = (acc && e < tq) ? dst[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 256 * u;
      if (e < tq) {
        const int r = e / nq, q = e - r * nq;
        float4 v = *reinterpret_cast<const float4*>(so + r * LO + 4 * q);
        if (acc) v = add4(v, old[u]);
        dst[e] = v;
      }
    }
  }
}

template <int KR>
static void thin_launch(const float* a, const float* b, const float* bias, float* out, int M,
                        int N, int acc, double* stats, hipStream_t st) {
  const unsigned grid = (unsigned)cdiv(M, 64);
  const size_t lds = sizeof(float) * 64 * (std::max(KR, N) + THIN_PAD);
  // CH = 16 only when the chunks split evenly over the 4 waves (N = 144: 18 chunks of 8 balance
  // 5/5/4/4, 9 chunks of 16 would leave three waves idle a third of the time)
  if (N % 64 == 0 && N >= 128)
    thin1x1_kernel<KR, 16><<<grid, 256, lds, st>>>(a, b, bias, out, M, N, acc, stats);
  else thin1x1_kernel<KR, 8><<<grid, 256, lds, st>>>(a, b, bias, out, M, N, acc, stats);
}

static bool thin_kr_ok(int kr) { return kr % 8 == 0 && kr >= 8 && kr <= 48; }

}  // namespace pld

using namespace pld;

// (K, N) of the GEMM a thin 1x1 conv runs: fwd K = cin, N = cout; dgrad K = cout, N = cin
extern "C" int pld__thin_ok(int K, int N) {
  static const int off = [] {
    const char* e = getenv("PLD_NO_THIN");  // debug knob: route everything to the MFMA tiles
    return e && e[0] == '1';
  }();
  if (off || N % 8 != 0 || !thin_kr_ok(K)) return 0;
  // K x N <= 4096: above it (40 -> 240, 40 -> 144) the per-lane FMA chains outlast the HBM time
  // and the MFMA tiles are as fast or faster (measured, profiles/r01_conv_table.txt)
  return N <= 256 && K * N <= 4096;
}

// 1x1, stride 1, unpadded, single source, no prologue
extern "C" int pld__thin_geom(const pld_conv_args* a) {
  return a && a->kh == 1 && a->kw == 1 && a->sh == 1 && a->sw == 1 && a->pad_t == 0 &&
         a->pad_l == 0 && a->c2 == 0 && a->x2 == nullptr && a->in_scale == nullptr &&
         a->oh == a->h && a->ow == a->w;
}

// stats: NULL, or [N][cdiv(M, 64)][2] fp64 BN partials of the output (pld__thin_stats_parts)
extern "C" int pld__thin_stats_parts(long M) { return (int)cdiv(M, 64); }

extern "C" int pld__thin_gemm(const float* a, const float* b, const float* bias, float* out,
                              long M, int K, int N, int acc, void* stream, double* stats) {
  PLD_CHECK_ARG(a && b && out && M > 0 && aligned16(a) && aligned16(out) && aligned16(b),
                "thin1x1: bad args");
  PLD_CHECK_ARG(M * (long)(K > N ? K : N) < (1L << 31), "thin1x1: tensor too large");
  PLD_CHECK_ARG(pld__thin_ok(K, N), "thin1x1: unsupported K=%d N=%d", K, N);
  hipStream_t st = as_stream(stream);
  const int m = (int)M;
  switch (K) {
    case 8: thin_launch<8>(a, b, bias, out, m, N, acc, stats, st); break;
    case 16: thin_launch<16>(a, b, bias, out, m, N, acc, stats, st); break;
    case 24: thin_launch<24>(a, b, bias, out, m, N, acc, stats, st); break;
    case 32: thin_launch<32>(a, b, bias, out, m, N, acc, stats, st); break;
    case 40: thin_launch<40>(a, b, bias, out, m, N, acc, stats, st); break;
    default: thin_launch<48>(a, b, bias, out, m, N, acc, stats, st); break;
  }
  return check_launch("thin1x1_kernel");
}

// Thin-N 1x1 convolutions whose input operand is produced on the fly by the elementwise op that
// precedes them, so that operand is never written to HBM and read back:
//   PRO_BNACT : y[m][n] = sum_k (act(bn(x[m][k])) * gate[img(m)][k]) * w[n][k]
//               — an EfficientNet block's project conv reading the pre-BN depthwise output
//                 through the block's BN + swish + SE gate (keras efficientnet block(): bn ->
//                 activation -> se multiply -> project_conv; pl_hourglass.py:52-57); replaces
//                 pld_bn_apply(gate) + pld_conv2d_fwd;
//   PRO_BNBWD : y[m][n] = sum_k bnbwd(x, dy)[m][k] * w[n][k],
//               bnbwd = (invstd gamma) (dy act'(z) - k1 - xhat k2)  (bn_bwd_apply's arithmetic)
//               — the expand conv's input gradient reading (expand_pre, d expand_activation)
//                 through the expand BN's backward; replaces the apply pass of pld_bn_bwd +
//                 pld_conv2d_dgrad (the reduction + finalize still run first: k1, k2).
// Shapes: the early MBConv blocks (K = 32..240 expanded channels, N = 16..40 block channels,
// M = n h w up to 1.6 M rows at 448^2, batch 32): HBM-bound, so plain fp32 FMA chains (exact
// fp32, more accurate than the bf16x3 tiles they replace). A 256-thread workgroup owns 64
// consecutive rows: the contiguous [64][K] block (one or two sources) is read with coalesced
// float4 loads, the prologue applied once per element, and stored in LDS (row stride K + 4:
// conflict-free ds_read_b128 of a row per lane); each lane then owns a row, the 4 waves split the
// N columns (filter rows wave-uniform: scalar loads), and the outputs go back through LDS for
// whole-row-segment stores (thin.hip's layout).
#include <algorithm>

#include "common.h"
#include "conv_common.h"

namespace pld {

enum PgPro { PRO_BNACT = 0, PRO_BNBWD = 1 };

struct PgParams {
  const float* x;       // [M][K]
  const float* dy;      // [M][K] (PRO_BNBWD)
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  const float* gate;    // [n_img][K] or NULL (PRO_BNACT)
  const float* k12;     // [2][K] (PRO_BNBWD)
  const float* w;       // [N][K]
  float* y;             // [M][N]
  int M, K, N, act, acc;
  FastDiv dHW;          // rows per image (gate)
};

constexpr int PG_KMAX = 240;  // [64][K + 4] floats of LDS stay within 64 KiB

// NW: output columns per wave (N <= 4 NW); MQ: float4 loads per thread per source (>= K / 16)
template <int PRO, int NW, int MQ>
__global__ __launch_bounds__(256) void pgemm_kernel(PgParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = p.K, LA = K + 4;
  float* sa = smem;                       // [64][LA]; after the MACs: [4][64][NW + 4] outputs
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long m0 = (long)blockIdx.x * 64;
  const int rows = (int)min(64L, (long)p.M - m0);
  // a thread owns ONE channel quad q of rows r0, r0 + rpp, ... (rpp = 256 / (K/4) rows per pass,
  // each pass a contiguous run of rpp rows): the BN coefficients of its quad are loaded once,
  // not once per element (bn_apply_kernel's scheme); every load is in flight before any is used
  const int kq = K / 4, rpp = 256 / kq;
  const int q = tid % kq, r0 = tid / kq, c = 4 * q;
  const bool act_t = r0 < rpp;
  const float4* s1 = reinterpret_cast<const float4*>(p.x + m0 * K);
  const float4* s2 = reinterpret_cast<const float4*>((PRO == PRO_BNBWD ? p.dy : p.x) + m0 * K);
  float4 va[MQ], vb[MQ];
#pragma unroll
  for (int j = 0; j < MQ; ++j) {  // clamped, unconditional loads (rows past the tile: zeroed)
    const int r = min(r0 + j * rpp, rows - 1);
    va[j] = s1[r * kq + q];
    if (PRO == PRO_BNBWD) vb[j] = s2[r * kq + q];
  }
  const float4 mu4 = *reinterpret_cast<const float4*>(p.mean + c);
  const float4 is4 = *reinterpret_cast<const float4*>(p.invstd + c);
  const float4 ga4 = *reinterpret_cast<const float4*>(p.gamma + c);
  const float4 be4 = *reinterpret_cast<const float4*>(p.beta + c);
  const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, is[4] = {is4.x, is4.y, is4.z, is4.w};
  const float ga[4] = {ga4.x, ga4.y, ga4.z, ga4.w}, be[4] = {be4.x, be4.y, be4.z, be4.w};
  float k1[4] = {0.f, 0.f, 0.f, 0.f}, k2[4] = {0.f, 0.f, 0.f, 0.f};
  if (PRO == PRO_BNBWD) {
    const float4 k14 = *reinterpret_cast<const float4*>(p.k12 + c);
    const float4 k24 = *reinterpret_cast<const float4*>(p.k12 + K + c);
    k1[0] = k14.x; k1[1] = k14.y; k1[2] = k14.z; k1[3] = k14.w;
    k2[0] = k24.x; k2[1] = k24.y; k2[2] = k24.z; k2[3] = k24.w;
  }
#pragma unroll
  for (int j = 0; j < MQ; ++j) {
    const int r = r0 + j * rpp;
    if (!act_t || r >= 64) break;
    const float xs[4] = {va[j].x, va[j].y, va[j].z, va[j].w};
    const float ds[4] = {vb[j].x, vb[j].y, vb[j].z, vb[j].w};
    float o[4];
    if (PRO == PRO_BNACT) {
      float g[4] = {1.f, 1.f, 1.f, 1.f};
      if (p.gate && r < rows) {
        const long img = (long)p.dHW.div((uint32_t)(m0 + r));
        const float4 g4 = *reinterpret_cast<const float4*>(p.gate + img * K + c);
        g[0] = g4.x; g[1] = g4.y; g[2] = g4.z; g[3] = g4.w;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)  // bn_apply_kernel's arithmetic (then act, then the gate)
        o[u] = act_fwd(p.act, ((xs[u] - mu[u]) * is[u]) * ga[u] + be[u]) * g[u];
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // bn_bwd_apply_kernel's arithmetic
        const float xh = (xs[u] - mu[u]) * is[u];
        const float z = xh * ga[u] + be[u];
        const float dz = ds[u] * act_grad(p.act, z);
        o[u] = (is[u] * ga[u]) * (dz - k1[u] - xh * k2[u]);
      }
    }
    if (r >= rows) o[0] = o[1] = o[2] = o[3] = 0.f;
    *reinterpret_cast<float4*>(sa + r * LA + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
  __syncthreads();
  // lane = row; wave w owns columns n = w NW .. w NW + NW - 1 (zero-padded past N)
  float acc[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) acc[j] = 0.f;
  const int nb = wave * NW;
  // K in chunks of 16 held in VGPRs (4 ds_read_b128 of the lane's row); per column the 16 filter
  // values are wave-uniform: one scalar s_load_dwordx16 feeds 16 FMAs (thin.hip's scheme; one
  // load per 4 FMAs left the loop bound by load issue and lgkmcnt waits)
  constexpr int KC = 16;
  for (int kc = 0; kc < K; kc += KC) {
    float xr[KC];
#pragma unroll
    for (int q = 0; q < KC / 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(sa + lane * LA + kc + 4 * q);
      xr[4 * q] = v.x; xr[4 * q + 1] = v.y; xr[4 * q + 2] = v.z; xr[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      if (nb + j < p.N) {  // wave-uniform
        const float* br = p.w + (long)(nb + j) * K + kc;
        float t = acc[j];
#pragma unroll
        for (int k = 0; k < KC; ++k) t = fmaf(xr[k], br[k], t);
        acc[j] = t;
      }
    }
  }
  // the workgroup's [64 rows][N] output tile through LDS (the input tile's space, once every
  // wave is done reading it), then stored as the one contiguous run of y it is: float4 stores
  // when N % 4 == 0 (the per-wave column chunks wrote 16-40-byte pieces of 64 rows)
  __syncthreads();
  const int LO = p.N + 4;
#pragma unroll
  for (int j = 0; j < NW; ++j)
    if (nb + j < p.N) sa[lane * LO + nb + j] = acc[j];
  __syncthreads();
  const int N = p.N;
  if (N % 4 == 0 && (reinterpret_cast<uintptr_t>(p.y) & 15) == 0) {
    const int nq = N / 4, tq = rows * nq;
    float4* dst = reinterpret_cast<float4*>(p.y + m0 * N);
    constexpr int U = 4;  // accumulate: U destination quads fetched before their stores
    for (int e0 = tid; e0 < tq; e0 += 256 * U) {
      float4 old[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + 256 * u;
        old[u] = (p.acc && e < tq) ? dst[e] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + 256 * u;
        if (e < tq) {
          const int r = e / nq, q = e - r * nq;
          float4 v = *reinterpret_cast<const float4*>(sa + r * LO + 4 * q);
          if (p.acc) v = add4(v, old[u]);
          dst[e] = v;
        }
      }
    }
    return;
  }
  for (int e = tid; e < rows * N; e += 256) {
    const int r = e / N, j = e - r * N;
    const float v = sa[r * LO + j];
    float* d = p.y + (m0 + r) * N + j;
    *d = p.acc ? *d + v : v;
  }
}

static int pg_launch(PgParams& p, int pro, hipStream_t st) {
  const int nw = (p.N + 3) / 4;
  const size_t lds = sizeof(float) * 64 * (std::max(p.K, p.N) + 4);
  const unsigned grid = cdiv(p.M, 64);
  const int mq = (int)cdiv(64, 256 / (p.K / 4));  // passes of rpp rows per thread
#define PG3(NWV, MQV)                                                                      \
  if (pro == PRO_BNACT) pgemm_kernel<PRO_BNACT, NWV, MQV><<<grid, 256, lds, st>>>(p);      \
  else pgemm_kernel<PRO_BNBWD, NWV, MQV><<<grid, 256, lds, st>>>(p);
#define PG(NWV)                                    \
  if (mq <= 4) { PG3(NWV, 4) }                     \
  else if (mq <= 8) { PG3(NWV, 8) }                \
  else if (mq <= 12) { PG3(NWV, 12) }              \
  else { PG3(NWV, 16) }
  if (nw <= 4) { PG(4) }
  else if (nw <= 6) { PG(6) }
  else if (nw <= 10) { PG(10) }
  else { PG(12) }
#undef PG
#undef PG3
  return check_launch("pgemm_kernel");
}

}  // namespace pld

using namespace pld;

extern "C" int pld_pgemm_ok(int k, int n) {
  return k > 0 && k % 16 == 0 && k <= PG_KMAX && n > 0 && n <= 48;
}

static int pg_check(const float* x, int64_t rows, int k, const float* mean, const float* invstd,
                    const float* gamma, const float* beta, const float* w, int n, float* y) {
  PLD_CHECK_ARG(x && mean && invstd && gamma && beta && w && y && rows > 0,
                "pld_pgemm: bad args");
  PLD_CHECK_ARG(pld_pgemm_ok(k, n), "pld_pgemm: K=%d N=%d unsupported (K %% 16 == 0, K <= %d, "
                "N <= 48)", k, n, PG_KMAX);
  PLD_CHECK_ARG(aligned16(x) && aligned16(mean) && aligned16(invstd) && aligned16(gamma) &&
                    aligned16(beta) && aligned16(w),
                "pld_pgemm: operands must be 16-byte aligned");
  PLD_CHECK_ARG(rows * (int64_t)k < (1L << 31), "pld_pgemm: tensor too large");
  return PLD_OK;
}

extern "C" int pld_pgemm_bn_act(const float* x, int64_t rows, int k, const float* mean,
                                const float* invstd, const float* gamma, const float* beta,
                                int act, const float* gate, int hw, const float* w, int n,
                                float* y, int accumulate, void* stream) {
  int rc = pg_check(x, rows, k, mean, invstd, gamma, beta, w, n, y);
  if (rc) return rc;
  PLD_CHECK_ARG(!gate || (hw > 0 && aligned16(gate)), "pld_pgemm_bn_act: gate needs hw > 0");
  PgParams p{};
  p.x = x; p.mean = mean; p.invstd = invstd; p.gamma = gamma; p.beta = beta;
  p.gate = gate; p.w = w; p.y = y;
  p.M = (int)rows; p.K = k; p.N = n; p.act = act; p.acc = accumulate;
  p.dHW = FastDiv((uint32_t)(hw > 0 ? hw : 1));
  return pg_launch(p, PRO_BNACT, as_stream(stream));
}

extern "C" int pld_pgemm_bn_bwd(const float* x, const float* dy, int64_t rows, int k,
                                const float* mean, const float* invstd, const float* gamma,
                                const float* beta, int act, const float* k12, const float* w,
                                int n, float* y, int accumulate, void* stream) {
  int rc = pg_check(x, rows, k, mean, invstd, gamma, beta, w, n, y);
  if (rc) return rc;
  PLD_CHECK_ARG(dy && k12 && aligned16(dy) && aligned16(k12), "pld_pgemm_bn_bwd: bad dy / k12");
  PgParams p{};
  p.x = x; p.dy = dy; p.mean = mean; p.invstd = invstd; p.gamma = gamma; p.beta = beta;
  p.k12 = k12; p.w = w; p.y = y;
  p.M = (int)rows; p.K = k; p.N = n; p.act = act; p.acc = accumulate;
  return pg_launch(p, PRO_BNBWD, as_stream(stream));
}

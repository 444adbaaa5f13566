// EfficientNetB0 MBConv pieces that are not GEMMs: depthwise conv (fwd + input gradient; the
// filters are frozen, pldepth/models/pl_hourglass.py:52-57) and squeeze-and-excitation.
//
// DepthwiseConv2D (keras efficientnet.py block(): k3/k5, stride 1 'same' or stride 2 after
// ZeroPadding2D(correct_pad) = asymmetric (k//2 - 1, k//2) padding on even inputs):
//   y[i][oy][ox][c] = sum_{ty,tx} x[i][oy*s+ty-pt][ox*s+tx-pl][c] * w[ty][tx][c]
//   dx[i][iy][ix][c] = sum_{ty,tx : (iy+pt-ty) % s == 0} dy[i][(iy+pt-ty)/s][(ix+pl-tx)/s][c] * w
// One thread per (pixel, 4 channels); HBM/L2-bound, no MFMA (no reduction over channels).
//
// Squeeze-and-excitation (GlobalAveragePooling2D -> Conv2D 1x1 swish -> Conv2D 1x1 sigmoid ->
// multiply): pooling and its adjoint reductions are per-image channel reductions (fp64 partials,
// fixed-order finalize); the two tiny FCs run one workgroup per image.
#include <algorithm>

#include "conv_common.h"

namespace pld {

// Index decomposition of a flat (img, row, column-tile, channel-quad) id with 32-bit magic
// divisions (64-bit integer division is emulated and was the cost of the first version).
struct DwGeom {
  int n, h, w, c, oh, ow, s, pt, pl;
  FastDiv dCV, dTiles, dRows;
  const float* mean;  // optional input prologue: act(((x - mean) * invstd) * gamma + beta)
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
};

__device__ __forceinline__ float4 fma4(float4 acc, float4 v, float4 f) {
  // explicit fused multiply-adds: every tap rounds once whatever the compiler makes of the
  // conditional rows around it (the tiled and register-window dgrads agree bit for bit)
  acc.x = fmaf(v.x, f.x, acc.x);
  acc.y = fmaf(v.y, f.y, acc.y);
  acc.z = fmaf(v.z, f.z, acc.z);
  acc.w = fmaf(v.w, f.w, acc.w);
  return acc;
}

// forward: a thread owns an R x T block of output pixels (R rows, T consecutive columns) and 4
// channels; each of the (R-1)S+K input rows of its (T-1)S+K-column window is loaded — and, with
// the BN+activation prologue, activated — once, then feeds every output row it reaches (the
// prologue's exp/rcp were the cost of a one-row window). Per output the taps are summed in the
// same (ty, tx) order as a direct loop. The prologue activation ACT is a template parameter
// (PRO_NONE: no prologue). The loads stay behind per-row/column bounds branches on purpose:
// branch-free (buffer-descriptor) loads let hipcc hoist every row's loads ahead of the FMAs
// (> 256 VGPRs, spills for K = 5).
constexpr int PRO_NONE = -1;

template <int K, int S, int T, int R, int ACT>
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ wt, DwGeom g,
                                                         float* __restrict__ y) {
  constexpr bool PRO = ACT != PRO_NONE;
  constexpr int NC = (T - 1) * S + K;
  constexpr int NR = (R - 1) * S + K;
  const int cv = g.c / 4;
  const int tiles = (g.ow + T - 1) / T;
  const int rgroups = (g.oh + R - 1) / R;
  const int total = g.n * rgroups * tiles * cv;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int t0 = (int)g.dCV.div((uint32_t)e);
    const int q = e - t0 * cv;
    const int t1 = (int)g.dTiles.div((uint32_t)t0);
    const int ox0 = (t0 - t1 * tiles) * T;
    const int img = (int)g.dRows.div((uint32_t)t1);
    const int oy0 = (t1 - img * rgroups) * R;
    float4 mu, is, ga, be;
    if (PRO) {
      mu = *reinterpret_cast<const float4*>(g.mean + 4 * q);
      is = *reinterpret_cast<const float4*>(g.invstd + 4 * q);
      ga = *reinterpret_cast<const float4*>(g.gamma + 4 * q);
      be = *reinterpret_cast<const float4*>(g.beta + 4 * q);
    }
    float4 acc[R][T];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int o = 0; o < T; ++o) acc[r][o] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* xb = x + (long)img * g.h * g.w * g.c + 4 * q;
    const int ix0 = ox0 * S - g.pl;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int iy = oy0 * S + j - g.pt;
      if (iy < 0 || iy >= g.h) continue;
      float4 row[NC];
#pragma unroll
      for (int jc = 0; jc < NC; ++jc) {
        const int ix = ix0 + jc;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ix >= 0 && ix < g.w) {
          v = *reinterpret_cast<const float4*>(xb + ((long)iy * g.w + ix) * g.c);
          if (PRO)  // the bn_apply arithmetic, then the activation (TF pads the activated map)
            v = make_float4(act_fwd(ACT, ((v.x - mu.x) * is.x) * ga.x + be.x),
                            act_fwd(ACT, ((v.y - mu.y) * is.y) * ga.y + be.y),
                            act_fwd(ACT, ((v.z - mu.z) * is.z) * ga.z + be.z),
                            act_fwd(ACT, ((v.w - mu.w) * is.w) * ga.w + be.w));
        }
        row[jc] = v;
      }
      const float* wq = wt + 4 * q;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ty = j - r * S;  // compile-time after unrolling
        if (ty < 0 || ty >= K) continue;
#pragma unroll
        for (int tx = 0; tx < K; ++tx) {
          const float4 f = *reinterpret_cast<const float4*>(wq + (ty * K + tx) * g.c);
#pragma unroll
          for (int o = 0; o < T; ++o) acc[r][o] = fma4(acc[r][o], row[o * S + tx], f);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (oy0 + r >= g.oh) break;
      float* yb = y + (((long)img * g.oh + oy0 + r) * g.ow) * g.c + 4 * q;
#pragma unroll
      for (int o = 0; o < T; ++o)
        if (ox0 + o < g.ow) *reinterpret_cast<float4*>(yb + (long)(ox0 + o) * g.c) = acc[r][o];
    }
  }
}

// Optional epilogue of the depthwise dgrads: the backward reductions of the BN + activation
// that PRODUCED the depthwise input (an MBConv expand BN: x = its pre-BN input), gathered as the
// gradient d(act) is stored — dz = d(act) act'(bn(x)), per channel (sum dz, sum dz xhat) in fp64.
// The host sizes the grid to a multiple of the channel-quad count, so each thread's quad is fixed
// for all its trips; a block combines its threads per quad in a fixed order and writes one
// partial per channel: [C][gridDim.x][2], bn.hip's finalize layout (no separate pass over
// (x, d(act)) for the reductions).
struct DwBnb {
  const float* x;
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
  double* part;
};

// the BN parameters of this thread's (fixed) channel quad, loaded once per launch
struct BnbQuad {
  float m[4], iv[4], gv[4], bv[4];
};

__device__ __forceinline__ BnbQuad bnb_quad(const DwBnb& b, int cv) {
  const int c0 = 4 * (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) % cv);
  const float4 mu = *reinterpret_cast<const float4*>(b.mean + c0);
  const float4 is = *reinterpret_cast<const float4*>(b.invstd + c0);
  const float4 ga = *reinterpret_cast<const float4*>(b.gamma + c0);
  const float4 be = *reinterpret_cast<const float4*>(b.beta + c0);
  return BnbQuad{{mu.x, mu.y, mu.z, mu.w}, {is.x, is.y, is.z, is.w},
                 {ga.x, ga.y, ga.z, ga.w}, {be.x, be.y, be.z, be.w}};
}

// one stored quad: fp32 running sums of the trip (a trip's few outputs), folded into the
// thread's fp64 totals once per trip by bnb_fold
__device__ __forceinline__ void bnb_acc(const DwBnb& b, const BnbQuad& pq, long idx, float4 v,
                                        float (&f0)[4], float (&f1)[4]) {
  const float4 x = *reinterpret_cast<const float4*>(b.x + idx);
  const float xv[4] = {x.x, x.y, x.z, x.w}, dv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float xh = (xv[u] - pq.m[u]) * pq.iv[u];
    const float dz = dv[u] * act_grad(b.act, xh * pq.gv[u] + pq.bv[u]);
    f0[u] += dz;
    f1[u] = fmaf(dz, xh, f1[u]);
  }
}

__device__ __forceinline__ void bnb_fold(float (&f0)[4], float (&f1)[4], double (&s0)[4],
                                         double (&s1)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    s0[u] += (double)f0[u];
    s1[u] += (double)f1[u];
    f0[u] = f1[u] = 0.f;
  }
}

// block combine (all 256 threads reach it): thread j's quad is (blockIdx.x 256 + j) mod cv
__device__ __forceinline__ void bnb_flush(const DwBnb& b, int cv, const double (&s0)[4],
                                          const double (&s1)[4]) {
  __shared__ double red[256][8];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    red[threadIdx.x][u] = s0[u];
    red[threadIdx.x][4 + u] = s1[u];
  }
  __syncthreads();
  const int base = (int)(((long)blockIdx.x * 256) % cv);
  for (int qq = threadIdx.x; qq < cv; qq += 256) {
    double a[4] = {0.0, 0.0, 0.0, 0.0}, c[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = (qq - base + cv) % cv; j < 256; j += cv)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] += red[j][u];
        c[u] += red[j][4 + u];
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<double2*>(b.part + ((long)(4 * qq + u) * gridDim.x + blockIdx.x) * 2) =
          make_double2(a[u], c[u]);
  }
}

// input gradient, stride 1: dx[iy][ix] = sum dy[iy+pt-ty][ix+pl-tx] w[ty][tx]; a thread owns
// R rows x T columns of dx from an (R+K-1) x (T+K-1) window of dy, each dy row loaded once. dy
// rows are visited bottom-up so every output still sums its taps in ascending (ty, tx) order.
template <int K, int T, int R, bool BNB = false>
__global__ __launch_bounds__(256) void dwconv_dgrad_s1_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ wt,
                                                              DwGeom g, float* __restrict__ dx,
                                                              int accum, DwBnb bnb = DwBnb{}) {
  constexpr int NC = T + K - 1;
  constexpr int NR = R + K - 1;
  const int cv = g.c / 4;
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};
  float f0[4] = {0.f, 0.f, 0.f, 0.f}, f1[4] = {0.f, 0.f, 0.f, 0.f};
  BnbQuad pq{};
  if constexpr (BNB) pq = bnb_quad(bnb, cv);
  const int tiles = (g.w + T - 1) / T;
  const int rgroups = (g.h + R - 1) / R;
  const int total = g.n * rgroups * tiles * cv;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int t0 = (int)g.dCV.div((uint32_t)e);
    const int q = e - t0 * cv;
    const int t1 = (int)g.dTiles.div((uint32_t)t0);
    const int ix0 = (t0 - t1 * tiles) * T;
    const int img = (int)g.dRows.div((uint32_t)t1);
    const int iy0 = (t1 - img * rgroups) * R;
    float4 acc[R][T];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int o = 0; o < T; ++o) acc[r][o] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* db = dy + (long)img * g.oh * g.ow * g.c + 4 * q;
    const int ox_lo = ix0 + g.pl - (K - 1);
    const int oy_lo = iy0 + g.pt - (K - 1);
#pragma unroll
    for (int jr = NR - 1; jr >= 0; --jr) {
      const int oy = oy_lo + jr;
      if (oy < 0 || oy >= g.oh) continue;
      float4 row[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int ox = ox_lo + j;
        row[j] = (ox >= 0 && ox < g.ow)
                     ? *reinterpret_cast<const float4*>(db + ((long)oy * g.ow + ox) * g.c)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const float* wq = wt + 4 * q;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ty = r + K - 1 - jr;  // dx row iy0 + r reads dy row iy0 + r + pt - ty
        if (ty < 0 || ty >= K) continue;
#pragma unroll
        for (int tx = 0; tx < K; ++tx) {
          const float4 f = *reinterpret_cast<const float4*>(wq + (ty * K + tx) * g.c);
          // output o uses dy column ix0 + o + pl - tx = ox_lo + (o + K - 1 - tx)
#pragma unroll
          for (int o = 0; o < T; ++o) acc[r][o] = fma4(acc[r][o], row[o + K - 1 - tx], f);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (iy0 + r >= g.h) break;
      float* xb = dx + (((long)img * g.h + iy0 + r) * g.w) * g.c + 4 * q;
#pragma unroll
      for (int o = 0; o < T; ++o) {
        if (ix0 + o >= g.w) continue;
        float4* d = reinterpret_cast<float4*>(xb + (long)(ix0 + o) * g.c);
        float4 v = acc[r][o];
        if (accum) {
          const float4 old = *d;
          v.x += old.x; v.y += old.y; v.z += old.z; v.w += old.w;
        }
        *d = v;
        if constexpr (BNB)
          bnb_acc(bnb, pq, (((long)img * g.h + iy0 + r) * g.w + ix0 + o) * g.c + 4 * q, v, f0,
                  f1);
      }
    }
    if constexpr (BNB) bnb_fold(f0, f1, s0, s1);
  }
  if constexpr (BNB) bnb_flush(bnb, cv, s0, s1);
}

// input gradient, stride 2, one thread per 2x2 block of dx pixels (2a + u, 2b + v). With the pad
// parities PTP = pt & 1, PLP = pl & 1 fixed at compile time, the taps of output (u, v) are the
// (ty, tx) with ty = u + PTP and tx = v + PLP (mod 2) — every tap serves exactly one of the four
// outputs — and dy row (2a + u + pt - ty) / 2 = a + pt / 2 + (u + PTP - ty) / 2: a window of
// (K + 3) / 2 dy rows x columns at compile-time offsets, each loaded once (the per-pixel kernel
// re-read it for every output). Each output sums its taps in ascending (ty, tx) order.
template <int K, int PTP, int PLP, bool BNB = false>
__global__ __launch_bounds__(256) void dwconv_dgrad_s2_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ wt,
                                                              DwGeom g, float* __restrict__ dx,
                                                              int accum, DwBnb bnb = DwBnb{}) {
  constexpr int DMIN = -(K - 1) / 2;  // (u + PTP - ty) / 2 ranges over [DMIN, 1]
  constexpr int NW = 2 - DMIN;
  const int cv = g.c / 4;
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0};
  float f0[4] = {0.f, 0.f, 0.f, 0.f}, f1[4] = {0.f, 0.f, 0.f, 0.f};
  BnbQuad pq{};
  if constexpr (BNB) pq = bnb_quad(bnb, cv);
  const int bw = (g.w + 1) / 2, bh = (g.h + 1) / 2;
  const int total = g.n * bh * bw * cv;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int t0 = (int)g.dCV.div((uint32_t)e);
    const int q = e - t0 * cv;
    const int t1 = (int)g.dTiles.div((uint32_t)t0);  // tiles == bw
    const int b = t0 - t1 * bw;
    const int img = (int)g.dRows.div((uint32_t)t1);  // rows == bh
    const int a = t1 - img * bh;
    const float* db = dy + (long)img * g.oh * g.ow * g.c + 4 * q;
    const int oy0 = a + (g.pt >> 1) + DMIN, ox0 = b + (g.pl >> 1) + DMIN;
    float4 win[NW][NW];
#pragma unroll
    for (int r = 0; r < NW; ++r)
#pragma unroll
      for (int s2 = 0; s2 < NW; ++s2) {
        const int oy = oy0 + r, ox = ox0 + s2;
        win[r][s2] = ((unsigned)oy < (unsigned)g.oh && (unsigned)ox < (unsigned)g.ow)
                         ? *reinterpret_cast<const float4*>(db + ((long)oy * g.ow + ox) * g.c)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    float4 acc[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) acc[u][v] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* wq = wt + 4 * q;
#pragma unroll
    for (int ty = 0; ty < K; ++ty) {
      const int u = (ty + PTP) & 1;  // ty = u + PTP (mod 2)
      const int r = (u + PTP - ty) / 2 - DMIN;
#pragma unroll
      for (int tx = 0; tx < K; ++tx) {
        const int v = (tx + PLP) & 1;
        const int s2 = (v + PLP - tx) / 2 - DMIN;
        const float4 f = *reinterpret_cast<const float4*>(wq + (ty * K + tx) * g.c);
        acc[u][v] = fma4(acc[u][v], win[r][s2], f);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int iy = 2 * a + u;
      if (iy >= g.h) break;
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int ix = 2 * b + v;
        if (ix >= g.w) continue;
        const long idx = (((long)img * g.h + iy) * g.w + ix) * g.c + 4 * q;
        float4* d = reinterpret_cast<float4*>(dx + idx);
        float4 o = acc[u][v];
        if (accum) {
          const float4 old = *d;
          o.x += old.x; o.y += old.y; o.z += old.z; o.w += old.w;
        }
        *d = o;
        if constexpr (BNB) bnb_acc(bnb, pq, idx, o, f0, f1);
      }
    }
    if constexpr (BNB) bnb_fold(f0, f1, s0, s1);
  }
  if constexpr (BNB) bnb_flush(bnb, cv, s0, s1);
}

// ---- SE ----
// optional input prologue of the SE reductions: the squeeze reads the pre-BN depthwise output
// and applies the block's BN + activation on the fly, so the activation is never materialised
struct SePro {
  const float* mean;  // NULL: the input is already the activation
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
};

__device__ __forceinline__ float4 se_pro(const SePro& pr, float4 v, float4 mu, float4 is,
                                         float4 ga, float4 be) {
  return make_float4(act_fwd(pr.act, ((v.x - mu.x) * is.x) * ga.x + be.x),
                     act_fwd(pr.act, ((v.y - mu.y) * is.y) * ga.y + be.y),
                     act_fwd(pr.act, ((v.z - mu.z) * is.z) * ga.z + be.z),
                     act_fwd(pr.act, ((v.w - mu.w) * is.w) * ga.w + be.w));
}

// per-image channel sums of a (or of a*dy): partial[img][split][c] (fp64); 4 rows of loads in
// flight per thread (the same summation order as one row at a time).
// BNB (backward, with the BN + activation prologue): also the four per-(image, channel) sums
// from which the block BN's backward reductions follow once the SE has produced addn:
//   A1 = sum dy act'(z), A2 = sum act'(z), B1 = sum dy act'(z) xhat, B2 = sum act'(z) xhat,
// so that sum dz = gate A1 + addn A2 and sum dz xhat = gate B1 + addn B2 for
// dz = (dy gate + addn) act'(z) (chan_reduce's RED_BNBWD with gate / addn): part4[k][img][split][c].
template <bool PRO, bool BNB = false>
__global__ __launch_bounds__(256) void img_chan_sum_kernel(const float* __restrict__ a,
                                                           const float* __restrict__ b, int hw,
                                                           int c, int rsplit, SePro pr,
                                                           double* __restrict__ part,
                                                           double* __restrict__ part4 = nullptr) {
  static_assert(!BNB || PRO, "the BN-backward sums need the BN prologue");
  const int img = blockIdx.x / rsplit;
  const int sp = blockIdx.x % rsplit;
  const int cv = c / 4;
  const int cbase = blockIdx.y * 256;
  const int ncv = min(256, cv - cbase);
  const int tid = threadIdx.x;
  const int rpi = 256 / ncv;
  const int r0 = tid / ncv;
  const int q = cbase + tid % ncv;
  const int rows_per = (hw + rsplit - 1) / rsplit;
  const int rb = sp * rows_per, re = min(hw, rb + rows_per);
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  double bs[4][4];  // [A1, A2, B1, B2][channel]
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int u = 0; u < 4; ++u) bs[k][u] = 0.0;
  if (r0 < rpi) {
    const long base = (long)img * hw * c + 4 * q;
    float4 mu, is, ga, be;
    if (PRO) {
      mu = *reinterpret_cast<const float4*>(pr.mean + 4 * q);
      is = *reinterpret_cast<const float4*>(pr.invstd + 4 * q);
      ga = *reinterpret_cast<const float4*>(pr.gamma + 4 * q);
      be = *reinterpret_cast<const float4*>(pr.beta + 4 * q);
    }
    // BNB: act and act' from ONE sigmoid for swish (act_fwd and act_grad each evaluated it: two
    // exp + two rcp per element, which the compiler did not merge across the runtime switch)
    auto act2 = [&](float z, float& av, float& ag) {
      if (pr.act == ACT_SWISH) {
        const float sg = sigmoidf_(z);
        av = z * sg;
        ag = sg * (1.f + z * (1.f - sg));
      } else {
        av = act_fwd(pr.act, z);
        ag = act_grad(pr.act, z);
      }
    };
    auto acc1 = [&](float4 v, float4 u) {
      if constexpr (BNB) {
        const float xs[4] = {v.x, v.y, v.z, v.w}, us[4] = {u.x, u.y, u.z, u.w};
        const float mus[4] = {mu.x, mu.y, mu.z, mu.w}, iss[4] = {is.x, is.y, is.z, is.w};
        const float gas[4] = {ga.x, ga.y, ga.z, ga.w}, bes[4] = {be.x, be.y, be.z, be.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xs[e] - mus[e]) * iss[e];
          const float z = xh * gas[e] + bes[e];
          float av, ag;
          act2(z, av, ag);
          const float dg = us[e] * ag;
          s[e] += (double)(av * us[e]);
          bs[0][e] += (double)dg;
          bs[1][e] += (double)ag;
          bs[2][e] += (double)dg * (double)xh;
          bs[3][e] += (double)ag * (double)xh;
        }
        return;
      }
      if (PRO) v = se_pro(pr, v, mu, is, ga, be);
      if (b) {
        s[0] += (double)(v.x * u.x); s[1] += (double)(v.y * u.y);
        s[2] += (double)(v.z * u.z); s[3] += (double)(v.w * u.w);
      } else {
        s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
      }
    };
    int r = rb + r0;
    constexpr int RU = 4;
    if (b) {
      for (; r + (RU - 1) * rpi < re; r += RU * rpi) {
        float4 v[RU], u[RU];
#pragma unroll
        for (int j = 0; j < RU; ++j) {
          v[j] = *reinterpret_cast<const float4*>(a + base + (long)(r + j * rpi) * c);
          u[j] = *reinterpret_cast<const float4*>(b + base + (long)(r + j * rpi) * c);
        }
#pragma unroll
        for (int j = 0; j < RU; ++j) acc1(v[j], u[j]);
      }
    } else {
      for (; r + (RU - 1) * rpi < re; r += RU * rpi) {
        float4 v[RU];
#pragma unroll
        for (int j = 0; j < RU; ++j)
          v[j] = *reinterpret_cast<const float4*>(a + base + (long)(r + j * rpi) * c);
#pragma unroll
        for (int j = 0; j < RU; ++j) acc1(v[j], v[j]);
      }
    }
    for (; r < re; r += rpi) {
      const float4 v = *reinterpret_cast<const float4*>(a + base + (long)r * c);
      const float4 u = b ? *reinterpret_cast<const float4*>(b + base + (long)r * c) : v;
      acc1(v, u);
    }
  }
  __shared__ double red[256][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) red[tid][u] = s[u];
  __syncthreads();
  if (r0 == 0 && r0 < rpi) {
    for (int j = 1; j < rpi; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += red[tid + j * ncv][u];
    double* o = part + ((long)img * rsplit + sp) * c + 4 * q;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = s[u];
  }
  if constexpr (BNB) {
    const long plane = (long)gridDim.x * c;  // one [img][split][c] plane per sum
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 4; ++u) red[tid][u] = bs[k][u];
      __syncthreads();
      if (r0 == 0 && r0 < rpi) {
        double t[4] = {bs[k][0], bs[k][1], bs[k][2], bs[k][3]};
        for (int j = 1; j < rpi; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) t[u] += red[tid + j * ncv][u];
        double* o = part4 + k * plane + ((long)img * rsplit + sp) * c + 4 * q;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = t[u];
      }
    }
  }
}

// sum_k part[(img * rsplit + k) * c + ch] in k order, with up to 8 loads in flight (rsplit is
// up to 32: one dependent load per k would leave the workgroup latency-bound)
__device__ __forceinline__ double se_part_sum(const double* __restrict__ part, int img, int rsplit,
                                              int c, int ch) {
  const double* p = part + (long)img * rsplit * c + ch;
  double s = 0.0;
  int k = 0;
  for (; k + 8 <= rsplit; k += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(long)(k + u) * c];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < rsplit; ++k) s += p[(long)k * c];
  return s;
}

// forward excitation, one workgroup per image
// SE excitation FCs (tiny: c <= 1152, cse <= 48 per image). Grid (image, SE_SLICES) of
// 1024-thread workgroups: every workgroup rebuilds the image's full hidden vector (z1 fwd /
// dz1 bwd) with short dependency chains (16 channel slices x 64 hidden lanes, then a fixed-order
// LDS combine) and writes its own slice of the c outputs. Workgroup 0 of an image also stores
// pooled and z1 (the backward needs z1).
constexpr int SE_SLICES = 8;
constexpr int SE_THREADS = 1024;
constexpr int SE_CS = SE_THREADS / 64;  // channel slices

// out[j] = sum_ch v[ch] * w[ch * cse + j] (w row-major [c][cse]; lanes over j: coalesced)
__device__ __forceinline__ void se_vecmat_cj(const float* v, const float* __restrict__ w, int c,
                                             int cse, float* red /* [SE_THREADS] */,
                                             float* out) {
  const int jl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  for (int j0 = 0; j0 < cse; j0 += 64) {
    const int j = j0 + jl;
    float a0 = 0.f, a1 = 0.f;
    if (j < cse) {
      int ch = sl;
#pragma unroll 4
      for (; ch + SE_CS < c; ch += 2 * SE_CS) {
        a0 += v[ch] * w[(long)ch * cse + j];
        a1 += v[ch + SE_CS] * w[(long)(ch + SE_CS) * cse + j];
      }
      if (ch < c) a0 += v[ch] * w[(long)ch * cse + j];
    }
    red[threadIdx.x] = a0 + a1;
    __syncthreads();
    if (sl == 0 && j < cse) {
      float t = red[jl];
      for (int k = 1; k < SE_CS; ++k) t += red[k * 64 + jl];
      out[j] = t;
    }
    __syncthreads();
  }
}

// out[j] = sum_ch v[ch] * w[j * c + ch] (w row-major [cse][c]): one wave per j, lanes over ch
__device__ __forceinline__ void se_vecmat_jc(const float* v, const float* __restrict__ w, int c,
                                             int cse, float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int j = wave; j < cse; j += SE_THREADS / 64) {
    float acc = 0.f;
#pragma unroll 4
    for (int ch = lane; ch < c; ch += 64) acc += v[ch] * w[(long)j * c + ch];
    acc = wave_sum(acc);
    if (lane == 0) out[j] = acc;
  }
}

__global__ __launch_bounds__(SE_THREADS) void se_fc_fwd_kernel(const double* __restrict__ part,
                                                               int rsplit, int hw, int c, int cse,
                                                               const float* __restrict__ w1,
                                                               const float* __restrict__ b1,
                                                               const float* __restrict__ w2,
                                                               const float* __restrict__ b2,
                                                               float* __restrict__ pooled,
                                                               float* __restrict__ z1,
                                                               float* __restrict__ gate) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* sp = sm;             // [c] pooled
  float* sh = sm + c;         // [cse] z1 - b1, then swish(z1)
  float* red = sh + cse;      // [SE_THREADS]
  const int img = blockIdx.x, slice = blockIdx.y;
  for (int ch = threadIdx.x; ch < c; ch += SE_THREADS) {
    const double s = se_part_sum(part, img, rsplit, c, ch);
    sp[ch] = (float)(s / (double)hw);
  }
  __syncthreads();
  se_vecmat_cj(sp, w1, c, cse, red, sh);
  if ((int)threadIdx.x < cse) {
    const int j = threadIdx.x;
    const float z = sh[j] + b1[j];
    if (slice == 0) z1[(long)img * cse + j] = z;
    sh[j] = z * sigmoidf_(z);
  }
  if (slice == 0)
    for (int ch = threadIdx.x; ch < c; ch += SE_THREADS) pooled[(long)img * c + ch] = sp[ch];
  __syncthreads();
  const int per = (c + SE_SLICES - 1) / SE_SLICES;
  const int cb = slice * per, ce = min(c, cb + per);
  for (int ch = cb + threadIdx.x; ch < ce; ch += SE_THREADS) {
    float acc = b2[ch];
#pragma unroll 8
    for (int j = 0; j < cse; ++j) acc += sh[j] * w2[(long)j * c + ch];
    gate[(long)img * c + ch] = sigmoidf_(acc);
  }
}

// SE backward: given S[c] = sum_hw dy*a (squeeze partials of the product), dz2 = S g (1-g),
// dz1 = (w2 . dz2) swish'(z1), addn[c] = (w1 . dz1)[c] / hw.
__global__ __launch_bounds__(SE_THREADS) void se_fc_bwd_kernel(const double* __restrict__ part,
                                                               int rsplit, int hw, int c, int cse,
                                                               const float* __restrict__ w1,
                                                               const float* __restrict__ w2,
                                                               const float* __restrict__ z1,
                                                               const float* __restrict__ gate,
                                                               float* __restrict__ addn,
                                                               const double* __restrict__ part4,
                                                               double* __restrict__ bnpart) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dz2 = sm;       // [c]
  float* dz1 = sm + c;   // [cse]
  const int img = blockIdx.x, slice = blockIdx.y;
  for (int ch = threadIdx.x; ch < c; ch += SE_THREADS) {
    const double s = se_part_sum(part, img, rsplit, c, ch);
    const float g = gate[(long)img * c + ch];
    dz2[ch] = (float)s * g * (1.f - g);
  }
  __syncthreads();
  se_vecmat_jc(dz2, w2, c, cse, dz1);
  __syncthreads();
  if ((int)threadIdx.x < cse) {
    const int j = threadIdx.x;
    const float z = z1[(long)img * cse + j];
    const float sg = sigmoidf_(z);
    dz1[j] *= sg * (1.f + z * (1.f - sg));
  }
  __syncthreads();
  const int per = (c + SE_SLICES - 1) / SE_SLICES;
  const int cb = slice * per, ce = min(c, cb + per);
  for (int ch = cb + threadIdx.x; ch < ce; ch += SE_THREADS) {
    float acc = 0.f;
#pragma unroll 8
    for (int j = 0; j < cse; ++j) acc += dz1[j] * w1[(long)ch * cse + j];
    const float ad = acc / (float)hw;
    addn[(long)img * c + ch] = ad;
    if (bnpart) dz2[ch] = ad;  // dz2 is no longer read: the slice's addn for the BN partials
  }
  if (bnpart) {
    // the block BN's backward partials of this image: sum dz = g A1 + addn A2, sum dz xhat =
    // g B1 + addn B2 per squeeze split -> [ch][img * rsplit + k][2] (bnbwd_finalize's layout);
    // every (channel, split) pair of the slice on its own thread
    __syncthreads();
    const long plane = (long)gridDim.x * rsplit * c, nparts = (long)gridDim.x * rsplit;
    for (int e = threadIdx.x; e < (ce - cb) * rsplit; e += SE_THREADS) {
      const int ch = cb + e / rsplit, k = e % rsplit;
      const double g = gate[(long)img * c + ch], ad = dz2[ch];
      const long o = ((long)img * rsplit + k) * c + ch;
      const double d0 = g * part4[o] + ad * part4[plane + o];
      const double d1 = g * part4[2 * plane + o] + ad * part4[3 * plane + o];
      *reinterpret_cast<double2*>(bnpart + ((long)ch * nparts + (long)img * rsplit + k) * 2) =
          make_double2(d0, d1);
    }
  }
}

static unsigned grid_for(long n) { return std::min<unsigned>(std::max(cdiv(n, 256), 1u), 8192); }

static int se_rsplit(int n, int hw, int c) {
  const int cy = std::max(1, (int)cdiv(c / 4, 256));  // c < 4: one group (found by tools/asan)
  int rs = (int)std::max(1L, 1024L / ((long)std::max(n, 1) * cy));
  rs = std::min(rs, std::max(1, hw / 32));
  return rs;
}

}  // namespace pld

using namespace pld;

static DwGeom dw_geom(int n, int h, int w, int c, int s, int pt, int pl, int oh, int ow) {
  DwGeom g{};
  g.n = n; g.h = h; g.w = w; g.c = c; g.s = s; g.pt = pt; g.pl = pl; g.oh = oh; g.ow = ow;
  g.dCV = FastDiv((uint32_t)(c / 4));
  return g;
}

// dwtile.hip: the LDS-tiled forward (C % 16 == 0), optionally gathering the output's BN partials
extern "C" int pld__dw_tiled_ok(int k, int s, int c);
extern "C" int pld__dw_tiled_parts(int n, int oh, int ow, int s, int c);
extern "C" int pld__dw_dgrad_tiled(const float* dy, int n, int h, int w, int c, const float* wdw,
                                   int k, int pad_t, int pad_l, int oh, int ow, float* dx,
                                   int accumulate, hipStream_t st);
extern "C" int pld__dw_fwd_tiled(const float* x, int n, int h, int w, int c, const float* wdw,
                                 int k, int s, int pad_t, int pad_l, int oh, int ow,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, int act, float* y, double* stats,
                                 hipStream_t st);
// bn.hip
extern "C" int pld__bn_stats_finish(const double* part, int nparts, int64_t rows, int c,
                                    float eps, float momentum, float* mean, float* invstd,
                                    float* moving_mean, float* moving_var, hipStream_t st);

template <int K, int S, int T, int R>
static void dw_fwd_launch(const float* x, const float* wdw, DwGeom& g, float* y, hipStream_t st) {
  const int rgroups = (g.oh + R - 1) / R;
  g.dTiles = FastDiv((uint32_t)((g.ow + T - 1) / T));
  g.dRows = FastDiv((uint32_t)rgroups);
  const long total = (long)g.n * rgroups * ((g.ow + T - 1) / T) * (g.c / 4);
  const unsigned grid = grid_for(total);
  if (!g.mean) dwconv_fwd_kernel<K, S, T, R, PRO_NONE><<<grid, 256, 0, st>>>(x, wdw, g, y);
  else if (g.act == ACT_SWISH) dwconv_fwd_kernel<K, S, T, R, ACT_SWISH><<<grid, 256, 0, st>>>(x, wdw, g, y);
  else if (g.act == ACT_RELU) dwconv_fwd_kernel<K, S, T, R, ACT_RELU><<<grid, 256, 0, st>>>(x, wdw, g, y);
  else if (g.act == ACT_SIGMOID) dwconv_fwd_kernel<K, S, T, R, ACT_SIGMOID><<<grid, 256, 0, st>>>(x, wdw, g, y);
  else dwconv_fwd_kernel<K, S, T, R, ACT_NONE><<<grid, 256, 0, st>>>(x, wdw, g, y);
}

extern "C" int pld_dwconv_fwd_bn(const float* x, int n, int h, int w, int c, const float* wdw,
                                 int k, int s, int pad_t, int pad_l, int oh, int ow,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, int act, float* y, void* stream) {
  PLD_CHECK_ARG(x && wdw && y && n > 0 && h > 0 && w > 0 && c > 0 && s > 0 && oh > 0 && ow > 0,
                "pld_dwconv_fwd: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_dwconv_fwd: channels must be a multiple of 4");
  PLD_CHECK_ARG(!mean || (invstd && gamma && beta), "pld_dwconv_fwd_bn: incomplete BN prologue");
  PLD_CHECK_ARG((long)n * h * w * c < (1L << 31) && (long)n * oh * ow * c < (1L << 31),
                "pld_dwconv_fwd: tensor too large for 32-bit indexing");
  PLD_CHECK_ARG(s == 1 || s == 2, "pld_dwconv_fwd: stride %d unsupported (1, 2)", s);
  hipStream_t st = as_stream(stream);
  if (pld__dw_tiled_ok(k, s, c) && aligned16(x) && aligned16(y) && aligned16(wdw))
    return pld__dw_fwd_tiled(x, n, h, w, c, wdw, k, s, pad_t, pad_l, oh, ow, mean, invstd, gamma,
                             beta, act, y, nullptr, st);
  DwGeom g = dw_geom(n, h, w, c, s, pad_t, pad_l, oh, ow);
  g.mean = mean; g.invstd = invstd; g.gamma = gamma; g.beta = beta; g.act = act;
  if (k == 3 && s == 1) dw_fwd_launch<3, 1, 4, 4>(x, wdw, g, y, st);
  else if (k == 3) dw_fwd_launch<3, 2, 2, 4>(x, wdw, g, y, st);
  else if (k == 5 && s == 1) dw_fwd_launch<5, 1, 4, 4>(x, wdw, g, y, st);
  else if (k == 5) dw_fwd_launch<5, 2, 2, 4>(x, wdw, g, y, st);
  else {
    set_error("pld_dwconv_fwd: kernel size %d unsupported (3, 5)", k);
    return PLD_ERR_UNSUPPORTED;
  }
  return check_launch("dwconv_fwd_kernel");
}

extern "C" size_t pld_dwconv_fwd_bn_stats_workspace_size(int n, int oh, int ow, int c, int s) {
  if (n <= 0 || oh <= 0 || ow <= 0 || c <= 0) return 0;
  const size_t fused = sizeof(double) * 2 * (size_t)c * pld__dw_tiled_parts(n, oh, ow, s, c);
  return std::max(fused, pld_channel_reduce_workspace_size((int64_t)n * oh * ow, c));
}

extern "C" int pld_dwconv_fwd_bn_stats(const float* x, int n, int h, int w, int c,
                                       const float* wdw, int k, int s, int pad_t, int pad_l,
                                       int oh, int ow, const float* mean, const float* invstd,
                                       const float* gamma, const float* beta, int act, float* y,
                                       float eps, float momentum, float* y_mean, float* y_invstd,
                                       float* y_moving_mean, float* y_moving_var, void* ws,
                                       size_t ws_bytes, void* stream) {
  PLD_CHECK_ARG(y_mean && y_invstd && ws &&
                    ws_bytes >= pld_dwconv_fwd_bn_stats_workspace_size(n, oh, ow, c, s),
                "pld_dwconv_fwd_bn_stats: bad statistics arguments / workspace too small");
  PLD_CHECK_ARG((y_moving_mean == nullptr) == (y_moving_var == nullptr),
                "pld_dwconv_fwd_bn_stats: moving statistics must both be given or both NULL");
  PLD_CHECK_ARG(x && wdw && y && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0,
                "pld_dwconv_fwd_bn_stats: bad args");
  PLD_CHECK_ARG((long)n * h * w * c < (1L << 31) && (long)n * oh * ow * c < (1L << 31),
                "pld_dwconv_fwd_bn_stats: tensor too large for 32-bit indexing");
  PLD_CHECK_ARG(!mean || (invstd && gamma && beta), "pld_dwconv_fwd_bn_stats: incomplete BN");
  hipStream_t st = as_stream(stream);
  const int64_t rows = (int64_t)n * oh * ow;
  if (pld__dw_tiled_ok(k, s, c) && aligned16(x) && aligned16(y) && aligned16(wdw)) {
    int rc = pld__dw_fwd_tiled(x, n, h, w, c, wdw, k, s, pad_t, pad_l, oh, ow, mean, invstd,
                               gamma, beta, act, y, (double*)ws, st);
    if (rc) return rc;
    return pld__bn_stats_finish((const double*)ws, pld__dw_tiled_parts(n, oh, ow, s, c), rows, c,
                                eps, momentum, y_mean, y_invstd, y_moving_mean, y_moving_var, st);
  }
  int rc = pld_dwconv_fwd_bn(x, n, h, w, c, wdw, k, s, pad_t, pad_l, oh, ow, mean, invstd, gamma,
                             beta, act, y, stream);
  if (rc) return rc;
  return pld_bn_stats(y, rows, c, eps, momentum, y_mean, y_invstd, y_moving_mean, y_moving_var,
                      ws, stream);
}

extern "C" int pld_dwconv_fwd(const float* x, int n, int h, int w, int c, const float* wdw, int k,
                              int s, int pad_t, int pad_l, int oh, int ow, float* y,
                              void* stream) {
  return pld_dwconv_fwd_bn(x, n, h, w, c, wdw, k, s, pad_t, pad_l, oh, ow, nullptr, nullptr,
                           nullptr, nullptr, 0, y, stream);
}

// grid of a dgrad launch: with the BN epilogue a multiple of the channel-quad count's share of
// 256 (m = cv / gcd(256, cv)), so that every thread keeps one channel quad for all its trips
static unsigned dgrad_grid(long total, int cv, bool bnb) {
  const unsigned g = grid_for(total);
  if (!bnb) return g;
  int a = 256, b = cv;
  while (b) { const int t = a % b; a = b; b = t; }
  const unsigned m = (unsigned)(cv / a);
  return std::max(m, g / m * m);
}

static int dw_dgrad_impl(const float* dy, int n, int h, int w, int c, const float* wdw, int k,
                         int s, int pad_t, int pad_l, int oh, int ow, float* dx, int accumulate,
                         const DwBnb* bnb, unsigned* grid_out, void* stream) {
  PLD_CHECK_ARG(dy && wdw && dx && n > 0 && h > 0 && w > 0 && c > 0 && s > 0 && oh > 0 && ow > 0,
                "pld_dwconv_dgrad: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_dwconv_dgrad: channels must be a multiple of 4");
  PLD_CHECK_ARG((long)n * h * w * c < (1L << 31) && (long)n * oh * ow * c < (1L << 31),
                "pld_dwconv_dgrad: tensor too large for 32-bit indexing");
  PLD_CHECK_ARG(k == 3 || k == 5, "pld_dwconv_dgrad: kernel size %d unsupported (3, 5)", k);
  PLD_CHECK_ARG(s == 1 || s == 2, "pld_dwconv_dgrad: stride %d unsupported (1, 2)", s);
  DwGeom g = dw_geom(n, h, w, c, s, pad_t, pad_l, oh, ow);
  g.dRows = FastDiv((uint32_t)h);
  hipStream_t st = as_stream(stream);
  const DwBnb bb = bnb ? *bnb : DwBnb{};
  const bool B = bnb != nullptr;
  if (s == 1 && !bnb && pld__dw_tiled_ok(k, 1, c) && pad_t < k && pad_l < k && aligned16(dy) &&
      aligned16(dx) && aligned16(wdw)) {
    // LDS-tiled (each dy element read once per workgroup instead of once per overlapping
    // register window: 2-3.5x the dy bytes from HBM at 14^2-28^2); same sums bit for bit
    if (grid_out) *grid_out = 0;
    return pld__dw_dgrad_tiled(dy, n, h, w, c, wdw, k, pad_t, pad_l, oh, ow, dx, accumulate, st);
  }
  if (s == 1) {
    constexpr int T = 4, R = 4;
    const int rgroups = (h + R - 1) / R;
    g.dRows = FastDiv((uint32_t)rgroups);
    g.dTiles = FastDiv((uint32_t)((w + T - 1) / T));
    const long total = (long)n * rgroups * ((w + T - 1) / T) * (c / 4);
    const unsigned grid = dgrad_grid(total, c / 4, B);
    if (grid_out) *grid_out = grid;
#define PLD_DWS1(KK)                                                                          \
  if (B) dwconv_dgrad_s1_kernel<KK, T, R, true><<<grid, 256, 0, st>>>(dy, wdw, g, dx, accumulate, bb); \
  else dwconv_dgrad_s1_kernel<KK, T, R><<<grid, 256, 0, st>>>(dy, wdw, g, dx, accumulate);
    if (k == 3) { PLD_DWS1(3) } else { PLD_DWS1(5) }
#undef PLD_DWS1
  } else {
    const int bw = (w + 1) / 2, bh = (h + 1) / 2;
    g.dTiles = FastDiv((uint32_t)bw);
    g.dRows = FastDiv((uint32_t)bh);
    const unsigned grid = dgrad_grid((long)n * bh * bw * (c / 4), c / 4, B);
    if (grid_out) *grid_out = grid;
    const int par = (pad_t & 1) * 2 + (pad_l & 1);
#define PLD_DWS2B(KK, PY, PX)                                                                   \
  if (B) dwconv_dgrad_s2_kernel<KK, PY, PX, true><<<grid, 256, 0, st>>>(dy, wdw, g, dx, accumulate, bb); \
  else dwconv_dgrad_s2_kernel<KK, PY, PX><<<grid, 256, 0, st>>>(dy, wdw, g, dx, accumulate);
#define PLD_DWS2(KK)                                                                            \
  if (par == 0) { PLD_DWS2B(KK, 0, 0) }                                                         \
  else if (par == 1) { PLD_DWS2B(KK, 0, 1) }                                                    \
  else if (par == 2) { PLD_DWS2B(KK, 1, 0) }                                                    \
  else { PLD_DWS2B(KK, 1, 1) }
    if (k == 3) { PLD_DWS2(3) } else { PLD_DWS2(5) }
#undef PLD_DWS2
#undef PLD_DWS2B
  }
  return check_launch("dwconv_dgrad_kernel");
}

extern "C" int pld_dwconv_dgrad(const float* dy, int n, int h, int w, int c, const float* wdw,
                                int k, int s, int pad_t, int pad_l, int oh, int ow, float* dx,
                                int accumulate, void* stream) {
  return dw_dgrad_impl(dy, n, h, w, c, wdw, k, s, pad_t, pad_l, oh, ow, dx, accumulate, nullptr,
                       nullptr, stream);
}

extern "C" size_t pld_dwconv_dgrad_bn_bwd_workspace_size(int n, int h, int w, int c, int s) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || c % 4 || (s != 1 && s != 2)) return 0;
  const long total = s == 1 ? (long)n * ((h + 3) / 4) * ((w + 3) / 4) * (c / 4)
                            : (long)n * ((h + 1) / 2) * ((w + 1) / 2) * (c / 4);
  return sizeof(double) * 2 * (size_t)c * dgrad_grid(total, c / 4, true);
}

extern "C" int pld__bn_bwd_finish(const double* part, int nparts, const float* x, const float* dy,
                                  int64_t rows, int c, const float* mean, const float* invstd,
                                  const float* gamma, const float* beta, int act,
                                  const float* gate, const float* addn, int hw, float* dx,
                                  int dx_accumulate, float* dgamma, float* dbeta,
                                  int param_accumulate, float* k12, hipStream_t st);

extern "C" int pld_dwconv_dgrad_bn_bwd(const float* dy, int n, int h, int w, int c,
                                       const float* wdw, int k, int s, int pad_t, int pad_l,
                                       int oh, int ow, float* dact, int accumulate,
                                       const float* x, const float* mean, const float* invstd,
                                       const float* gamma, const float* beta, int act, float* dx,
                                       int dx_accumulate, float* dgamma, float* dbeta,
                                       int param_accumulate, float* k12, void* ws,
                                       size_t ws_bytes, void* stream) {
  PLD_CHECK_ARG(x && mean && invstd && gamma && beta && k12 && ws && aligned16(x) &&
                    aligned16(mean) && aligned16(invstd) && aligned16(gamma) && aligned16(beta),
                "pld_dwconv_dgrad_bn_bwd: bad BN args (16-byte aligned)");
  const size_t need = pld_dwconv_dgrad_bn_bwd_workspace_size(n, h, w, c, s);
  PLD_CHECK_ARG(need > 0 && ws_bytes >= need, "pld_dwconv_dgrad_bn_bwd: workspace %zu < %zu",
                ws_bytes, need);
  const DwBnb b{x, mean, invstd, gamma, beta, act, (double*)ws};
  unsigned grid = 0;
  int rc = dw_dgrad_impl(dy, n, h, w, c, wdw, k, s, pad_t, pad_l, oh, ow, dact, accumulate, &b,
                         &grid, stream);
  if (rc) return rc;
  return pld__bn_bwd_finish((const double*)ws, (int)grid, x, dact, (int64_t)n * h * w, c, mean,
                            invstd, gamma, beta, act, nullptr, nullptr, 0, dx, dx_accumulate,
                            dgamma, dbeta, param_accumulate, k12, as_stream(stream));
}

extern "C" size_t pld_se_workspace_size(int n, int hw, int c, int cse) {
  if (n <= 0 || hw <= 0 || c <= 0) return 0;
  return sizeof(double) * (size_t)n * se_rsplit(n, hw, c) * c;
}

static int se_fwd_impl(const float* a, const SePro& pr, int n, int hw, int c, int cse,
                       const float* w1, const float* b1, const float* w2, const float* b2,
                       float* pooled, float* z1, float* gate, void* ws, void* stream) {
  PLD_CHECK_ARG(a && w1 && b1 && w2 && b2 && pooled && z1 && gate && ws && n > 0 && hw > 0 &&
                    c > 0 && cse > 0,
                "pld_se_fwd: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_se_fwd: channels must be a multiple of 4");
  hipStream_t st = as_stream(stream);
  const int rs = se_rsplit(n, hw, c);
  dim3 g1(n * rs, cdiv(c / 4, 256));
  if (pr.mean) img_chan_sum_kernel<true><<<g1, 256, 0, st>>>(a, nullptr, hw, c, rs, pr, (double*)ws);
  else img_chan_sum_kernel<false><<<g1, 256, 0, st>>>(a, nullptr, hw, c, rs, pr, (double*)ws);
  int rc = check_launch("img_chan_sum_kernel");
  if (rc) return rc;
  se_fc_fwd_kernel<<<dim3(n, SE_SLICES), SE_THREADS, sizeof(float) * (c + cse + SE_THREADS), st>>>(
      (const double*)ws, rs, hw, c, cse, w1, b1, w2, b2, pooled, z1, gate);
  return check_launch("se_fc_fwd_kernel");
}

extern "C" int pld_se_fwd(const float* a, int n, int hw, int c, int cse, const float* w1,
                          const float* b1, const float* w2, const float* b2, float* pooled,
                          float* z1, float* gate, void* ws, void* stream) {
  return se_fwd_impl(a, SePro{}, n, hw, c, cse, w1, b1, w2, b2, pooled, z1, gate, ws, stream);
}

extern "C" int pld_se_fwd_bn(const float* x, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int act, int n, int hw, int c,
                             int cse, const float* w1, const float* b1, const float* w2,
                             const float* b2, float* pooled, float* z1, float* gate, void* ws,
                             void* stream) {
  PLD_CHECK_ARG(mean && invstd && gamma && beta, "pld_se_fwd_bn: incomplete BN prologue");
  return se_fwd_impl(x, SePro{mean, invstd, gamma, beta, act}, n, hw, c, cse, w1, b1, w2, b2,
                     pooled, z1, gate, ws, stream);
}

static int se_bwd_impl(const float* dy, const float* a, const SePro& pr, int n, int hw, int c,
                       int cse, const float* w1, const float* w2, const float* z1,
                       const float* gate, float* addn, void* ws, void* stream) {
  PLD_CHECK_ARG(dy && a && w1 && w2 && z1 && gate && addn && ws && n > 0 && hw > 0 && c > 0 &&
                    cse > 0,
                "pld_se_bwd: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_se_bwd: channels must be a multiple of 4");
  hipStream_t st = as_stream(stream);
  const int rs = se_rsplit(n, hw, c);
  dim3 g1(n * rs, cdiv(c / 4, 256));
  if (pr.mean) img_chan_sum_kernel<true><<<g1, 256, 0, st>>>(a, dy, hw, c, rs, pr, (double*)ws);
  else img_chan_sum_kernel<false><<<g1, 256, 0, st>>>(a, dy, hw, c, rs, pr, (double*)ws);
  int rc = check_launch("img_chan_sum_kernel(bwd)");
  if (rc) return rc;
  se_fc_bwd_kernel<<<dim3(n, SE_SLICES), SE_THREADS, sizeof(float) * (c + cse), st>>>(
      (const double*)ws, rs, hw, c, cse, w1, w2, z1, gate, addn, nullptr, nullptr);
  return check_launch("se_fc_bwd_kernel");
}

extern "C" int pld_se_bwd(const float* dy, const float* a, int n, int hw, int c, int cse,
                          const float* w1, const float* w2, const float* z1, const float* gate,
                          float* addn, void* ws, void* stream) {
  return se_bwd_impl(dy, a, SePro{}, n, hw, c, cse, w1, w2, z1, gate, addn, ws, stream);
}

extern "C" int pld_se_bwd_bn(const float* dy, const float* x, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, int act,
                             int n, int hw, int c, int cse, const float* w1, const float* w2,
                             const float* z1, const float* gate, float* addn, void* ws,
                             void* stream) {
  PLD_CHECK_ARG(mean && invstd && gamma && beta, "pld_se_bwd_bn: incomplete BN prologue");
  return se_bwd_impl(dy, x, SePro{mean, invstd, gamma, beta, act}, n, hw, c, cse, w1, w2, z1,
                     gate, addn, ws, stream);
}

// bn.hip: finalize (dgamma, dbeta, k1, k2 from channel-major partials) + apply
extern "C" int pld__bn_bwd_finish(const double* part, int nparts, const float* x, const float* dy,
                                  int64_t rows, int c, const float* mean, const float* invstd,
                                  const float* gamma, const float* beta, int act,
                                  const float* gate, const float* addn, int hw, float* dx,
                                  int dx_accumulate, float* dgamma, float* dbeta,
                                  int param_accumulate, float* k12, hipStream_t st);

// The BN-backward squeeze (img_chan_sum_kernel<true, true>) holds 136 VGPRs, i.e. 3 workgroups
// per CU: se_rsplit's 1024-workgroup grid ran as 1.33 rounds of the 768 the chip holds at once.
// One round of 768: 47.2 -> 44.1 us per launch, step +0.3 % in 4 of 4 alternating pairs; 1536
// (two rounds) 47.8 us (profiles/r04_se_squeeze_grid_ab.txt)
static int se_rsplit_bn(int n, int hw, int c) {
  const int cy = std::max(1, (int)cdiv(c / 4, 256));
  int rs = (int)std::max(1L, 768L / ((long)std::max(n, 1) * cy));
  rs = std::min(rs, std::max(1, hw / 32));
  return rs;
}

static size_t se_bn_ws_parts(int n, int hw, int c) {
  return (size_t)n * se_rsplit_bn(n, hw, c) * c;  // doubles per [img][split][c] plane
}

extern "C" size_t pld_se_bwd_bn_full_workspace_size(int n, int hw, int c, int cse) {
  if (n <= 0 || hw <= 0 || c <= 0) return 0;
  // S plane, the 4 BN-sum planes, the [c][parts][2] BN partials, k1 / k2
  return sizeof(double) * se_bn_ws_parts(n, hw, c) * 7 + 2 * sizeof(float) * (size_t)c + 64;
}

extern "C" int pld_se_bwd_bn_full(const float* dy, const float* x, const float* mean,
                                  const float* invstd, const float* gamma, const float* beta,
                                  int act, int n, int hw, int c, int cse, const float* w1,
                                  const float* w2, const float* z1, const float* gate,
                                  float* addn, float* dx, int dx_accumulate, float* dgamma,
                                  float* dbeta, int param_accumulate, void* ws, size_t ws_bytes,
                                  void* stream) {
  PLD_CHECK_ARG(dy && x && mean && invstd && gamma && beta && w1 && w2 && z1 && gate && addn &&
                    dx && dgamma && dbeta && ws && n > 0 && hw > 0 && c > 0 && cse > 0,
                "pld_se_bwd_bn_full: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_se_bwd_bn_full: channels must be a multiple of 4");
  PLD_CHECK_ARG((long)n * hw * c < (1L << 31), "pld_se_bwd_bn_full: tensor too large");
  PLD_CHECK_ARG(ws_bytes >= pld_se_bwd_bn_full_workspace_size(n, hw, c, cse),
                "pld_se_bwd_bn_full: workspace too small");
  hipStream_t st = as_stream(stream);
  const int rs = se_rsplit_bn(n, hw, c);
  const size_t np = se_bn_ws_parts(n, hw, c);
  double* part = (double*)ws;
  double* part4 = part + np;
  double* bnpart = part4 + 4 * np;
  float* k12 = (float*)(bnpart + 2 * np);
  const SePro pr{mean, invstd, gamma, beta, act};
  dim3 g1(n * rs, cdiv(c / 4, 256));
  img_chan_sum_kernel<true, true><<<g1, 256, 0, st>>>(x, dy, hw, c, rs, pr, part, part4);
  int rc = check_launch("img_chan_sum_kernel(bwd, bn)");
  if (rc) return rc;
  se_fc_bwd_kernel<<<dim3(n, SE_SLICES), SE_THREADS, sizeof(float) * (c + cse), st>>>(
      part, rs, hw, c, cse, w1, w2, z1, gate, addn, part4, bnpart);
  rc = check_launch("se_fc_bwd_kernel");
  if (rc) return rc;
  return pld__bn_bwd_finish(bnpart, n * rs, x, dy, (int64_t)n * hw, c, mean, invstd, gamma, beta,
                            act, gate, addn, hw, dx, dx_accumulate, dgamma, dbeta,
                            param_accumulate, k12, st);
}

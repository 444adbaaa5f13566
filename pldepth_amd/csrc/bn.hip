// Training-mode BatchNormalization (+ fused activation / SE gate) and per-channel reductions.
//
// Replaces Keras BatchNormalization in training mode (TF FusedBatchNormV3 / FusedBatchNormGradV3)
// for every BN on the hot path: the decoder BNs (pldepth/models/pl_hourglass.py:60,69,78,87,92),
// the 49 trainable EfficientNetB0 BNs (frozen encoder, BN trainable: pl_hourglass.py:52-57) and
// the ReDWeb/ResNet BNs (redweb.py). Keras defaults: epsilon 1e-3, momentum 0.99; the moving
// variance is updated with the unbiased (n/(n-1)) batch variance, the output uses the biased one.
//
// Channel reductions run over an NHWC tensor viewed as [rows][C]: a block owns a row range and up
// to 256 float4 channel groups; each thread accumulates in fp64 (the statistics of 6.4M-row
// tensors stay exact to ~1e-16), block partials land in a caller workspace and a finalize kernel
// sums them in a fixed order (deterministic, no atomics). HBM-bound: one read of x (stats) and
// one read of (x, dy) (backward) per element.
#include <algorithm>

#include "common.h"

namespace pld {

enum RedOp { RED_STATS = 0, RED_SUM = 1, RED_BNBWD = 2 };

struct RedParams {
  const float* x;
  const float* dy;
  long rows;
  int C;
  int rows_per_block;
  // BNBWD
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
  const float* gate;
  const float* addn;
  const float* res;  // residual added before the activation (ResNet / ReDWeb blocks), or NULL
  FastDiv dHW;
  double* partial;  // [C][gridDim.x][2]
  float* dz_out;    // BNBWD without gate/addn: also store dz = d(act input) (or NULL)
  const float* sscale;  // BNBWD: dy scaled per image (drop-connect), [rows / hw], or NULL
};

template <int VW>
__device__ __forceinline__ void ld(const float* p, float (&v)[VW]) {
  if constexpr (VW == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = *p;
  }
}

template <int VW>
__device__ __forceinline__ void st(float* p, const float (&v)[VW]) {
  if constexpr (VW == 4)
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else
    *p = v[0];
}

// ACT >= 0: the BN backward's activation as a compile-time constant (no per-element switch on
// p.act in the loop); -1: read p.act (the statistics / sum reductions do not use it)
template <int OP, int VW, int ACT = -1>
__global__ __launch_bounds__(256) void chan_reduce_kernel(RedParams p) {
  const int act_id = ACT >= 0 ? ACT : p.act;
  __shared__ double red[256][2 * VW];
  const int CV = p.C / VW;
  const int cbase = blockIdx.y * 256;
  const int ncv = min(256, CV - cbase);
  const int tid = threadIdx.x;
  const int rpi = 256 / ncv;
  const int r0 = tid / ncv;
  const int cv = cbase + tid % ncv;
  const bool act = r0 < rpi;
  const long rbeg = (long)blockIdx.x * p.rows_per_block;
  const long rend = min(p.rows, rbeg + p.rows_per_block);
  double s0[VW], s1[VW];
#pragma unroll
  for (int u = 0; u < VW; ++u) s0[u] = s1[u] = 0.0;
  if (act) {
    const int c0 = cv * VW;
    float mean[VW], inv[VW], gam[VW], bet[VW];
    if (OP == RED_BNBWD) {
      ld<VW>(p.mean + c0, mean);
      ld<VW>(p.invstd + c0, inv);
      ld<VW>(p.gamma + c0, gam);
      ld<VW>(p.beta + c0, bet);
    }
    long r = rbeg + r0;
    if (OP != RED_BNBWD) {
      // RU independent row loads in flight per thread before any is consumed (one load per
      // thread per trip leaves too few bytes in flight to cover HBM latency). Same summation
      // order as the plain loop.
      constexpr int RU = 4;
      for (; r + (RU - 1) * rpi < rend; r += RU * rpi) {
        float xv[RU][VW];
#pragma unroll
        for (int j = 0; j < RU; ++j) ld<VW>(p.x + (r + j * rpi) * p.C + c0, xv[j]);
#pragma unroll
        for (int j = 0; j < RU; ++j)
#pragma unroll
          for (int u = 0; u < VW; ++u) {
            const double d = xv[j][u];
            s0[u] += d;
            if (OP == RED_STATS) s1[u] += d * d;
          }
      }
    } else if (!p.gate && !p.addn) {  // BN(+residual)(+act) backward: same, for (x, dy[, res])
      constexpr int RU = 4;
      for (; r + (RU - 1) * rpi < rend; r += RU * rpi) {
        float xv[RU][VW], dv[RU][VW], rv[RU][VW];
#pragma unroll
        for (int j = 0; j < RU; ++j) {
          ld<VW>(p.x + (r + j * rpi) * p.C + c0, xv[j]);
          ld<VW>(p.dy + (r + j * rpi) * p.C + c0, dv[j]);
          if (p.sscale) {  // drop-connect: d(bn out) = dy * scale[img], rounded as its own product
            const float sc = p.sscale[p.dHW.div((uint32_t)(r + j * rpi))];
#pragma unroll
            for (int u = 0; u < VW; ++u) dv[j][u] = mul_rn(dv[j][u], sc);
          }
          if (p.res) {
            ld<VW>(p.res + (r + j * rpi) * p.C + c0, rv[j]);
          } else {
#pragma unroll
            for (int u = 0; u < VW; ++u) rv[j][u] = 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < RU; ++j) {
          float dzv[VW];
#pragma unroll
          for (int u = 0; u < VW; ++u) {
            const float xh = (xv[j][u] - mean[u]) * inv[u];
            const float z = (xh * gam[u] + bet[u]) + rv[j][u];
            const float dz = dv[j][u] * act_grad(act_id, z);
            dzv[u] = dz;
            s0[u] += (double)dz;
            s1[u] += (double)dz * (double)xh;
          }
          if (p.dz_out) st<VW>(p.dz_out + (r + j * rpi) * p.C + c0, dzv);
        }
      }
    }
    for (; r < rend; r += rpi) {
      float xv[VW];
      ld<VW>(p.x + r * p.C + c0, xv);
      if (OP == RED_STATS) {
#pragma unroll
        for (int u = 0; u < VW; ++u) {
          const double d = xv[u];
          s0[u] += d;
          s1[u] += d * d;
        }
      } else if (OP == RED_SUM) {
#pragma unroll
        for (int u = 0; u < VW; ++u) s0[u] += (double)xv[u];
      } else {
        float dv[VW];
        ld<VW>(p.dy + r * p.C + c0, dv);
        float g[VW], a[VW];
        const long img = (p.gate || p.addn || p.sscale) ? (long)p.dHW.div((uint32_t)r) : 0;
        if (p.sscale) {
          const float sc = p.sscale[img];
#pragma unroll
          for (int u = 0; u < VW; ++u) dv[u] = mul_rn(dv[u], sc);
        }
#pragma unroll
        for (int u = 0; u < VW; ++u) { g[u] = 1.f; a[u] = 0.f; }
        if (p.gate) ld<VW>(p.gate + img * p.C + c0, g);
        if (p.addn) ld<VW>(p.addn + img * p.C + c0, a);
        float rv[VW];
#pragma unroll
        for (int u = 0; u < VW; ++u) rv[u] = 0.f;
        if (p.res) ld<VW>(p.res + r * p.C + c0, rv);
        float dzv[VW];
#pragma unroll
        for (int u = 0; u < VW; ++u) {
          const float xh = (xv[u] - mean[u]) * inv[u];
          const float z = (xh * gam[u] + bet[u]) + rv[u];
          const float dz = (dv[u] * g[u] + a[u]) * act_grad(act_id, z);
          dzv[u] = dz;
          s0[u] += (double)dz;
          s1[u] += (double)dz * (double)xh;
        }
        if (p.dz_out) st<VW>(p.dz_out + r * p.C + c0, dzv);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < VW; ++u) {
    red[tid][u] = s0[u];
    red[tid][VW + u] = s1[u];
  }
  __syncthreads();
  if (act && r0 == 0) {
    for (int j = 1; j < rpi; ++j) {
#pragma unroll
      for (int u = 0; u < VW; ++u) {
        s0[u] += red[tid + j * ncv][u];
        s1[u] += red[tid + j * ncv][VW + u];
      }
    }
    // channel-major partials: the finalize kernel's per-channel read is one contiguous run
#pragma unroll
    for (int u = 0; u < VW; ++u)
      *reinterpret_cast<double2*>(p.partial + (((long)(cv * VW + u)) * gridDim.x + blockIdx.x) * 2) =
          make_double2(s0[u], s1[u]);
  }
}

static void red_plan(long rows, int C, int& nbx, int& rpb) {
  // ~ 2048 blocks total, >= 32 rows per block
  const int cy = (int)cdiv(C / ((C % 4 == 0) ? 4 : 1), 256);
  long want = std::max<long>(1, 2048 / cy);
  rpb = (int)std::max<long>(32, (rows + want - 1) / want);
  nbx = (int)((rows + rpb - 1) / rpb);
}

static int launch_reduce(int op, RedParams& p, hipStream_t st) {
  int nbx, rpb;
  red_plan(p.rows, p.C, nbx, rpb);
  p.rows_per_block = rpb;
  const bool v4 = (p.C % 4 == 0);
  const int CV = p.C / (v4 ? 4 : 1);
  dim3 grid(nbx, cdiv(CV, 256));
#define PLD_RED(OPV)                                                                         \
  if (v4) chan_reduce_kernel<OPV, 4><<<grid, 256, 0, st>>>(p);                               \
  else chan_reduce_kernel<OPV, 1><<<grid, 256, 0, st>>>(p);
#define PLD_RED_ACT(A)                                                                       \
  if (v4) chan_reduce_kernel<RED_BNBWD, 4, A><<<grid, 256, 0, st>>>(p);                      \
  else chan_reduce_kernel<RED_BNBWD, 1, A><<<grid, 256, 0, st>>>(p);
  if (op == RED_STATS) { PLD_RED(RED_STATS) }
  else if (op == RED_SUM) { PLD_RED(RED_SUM) }
  else if (p.act == ACT_NONE) { PLD_RED_ACT(ACT_NONE) }
  else if (p.act == ACT_RELU) { PLD_RED_ACT(ACT_RELU) }
  else if (p.act == ACT_SWISH) { PLD_RED_ACT(ACT_SWISH) }
  else { PLD_RED(RED_BNBWD) }
#undef PLD_RED_ACT
#undef PLD_RED
  return check_launch("chan_reduce_kernel");
}

// ---- finalize kernels: one workgroup per channel sums that channel's nbx partials (one
// contiguous [nbx][2] run, coalesced 16-byte loads strided over the 256 threads, then a
// fixed-shape wavefront butterfly and a 4-way LDS sum: deterministic, latency-parallel) ----
__device__ __forceinline__ void reduce_partials(const double* __restrict__ part, int nbx, int C,
                                                int c, double& s, double& q) {
  __shared__ double rs[4], rq[4];
  const double2* run = reinterpret_cast<const double2*>(part) + (long)c * nbx;
  double a = 0.0, b = 0.0;
  // U partials in flight per thread per trip (a GEMM epilogue leaves up to M/32 partials per
  // channel: 12544 at 112^2 x 32, i.e. 49 dependent round trips per thread one at a time)
  constexpr int U = 8;
  int i = threadIdx.x;
  for (; i + (U - 1) * 256 < nbx; i += U * 256) {
    double2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = run[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a += v[u].x;
      b += v[u].y;
    }
  }
  for (; i < nbx; i += 256) {
    const double2 v = run[i];
    a += v.x;
    b += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    rs[w] = a;
    rq[w] = b;
  }
  __syncthreads();
  s = (rs[0] + rs[1]) + (rs[2] + rs[3]);
  q = (rq[0] + rq[1]) + (rq[2] + rq[3]);
}

__global__ __launch_bounds__(256) void stats_finalize_kernel(
    const double* __restrict__ part, int nbx, int C, long rows, float eps, float momentum,
    float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ mmean,
    float* __restrict__ mvar) {
  const int c = blockIdx.x;
  double s, q;
  reduce_partials(part, nbx, C, c, s, q);
  if (threadIdx.x != 0) return;
  const double n = (double)rows;
  const double mu = s / n;
  double var = q / n - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (mmean) {
    const double uvar = rows > 1 ? var * n / (n - 1.0) : var;
    // Keras assign_moving_average: v -= (v - value) * (1 - momentum)
    mmean[c] = mmean[c] - (mmean[c] - (float)mu) * (1.0f - momentum);
    mvar[c] = mvar[c] - (mvar[c] - (float)uvar) * (1.0f - momentum);
  }
}

__global__ __launch_bounds__(256) void sum_finalize_kernel(const double* __restrict__ part,
                                                           int nbx, int C,
                                                           float* __restrict__ out, int acc) {
  const int c = blockIdx.x;
  double s, q;
  reduce_partials(part, nbx, C, c, s, q);
  if (threadIdx.x == 0) out[c] = acc ? out[c] + (float)s : (float)s;
}

// writes dgamma/dbeta and the per-channel coefficients k1 = mean(dz), k2 = mean(dz*xhat)
__global__ __launch_bounds__(256) void bnbwd_finalize_kernel(
    const double* __restrict__ part, int nbx, int C, long rows, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int pacc, float* __restrict__ k12) {
  const int c = blockIdx.x;
  double s, q;
  reduce_partials(part, nbx, C, c, s, q);
  if (threadIdx.x != 0) return;
  if (dbeta) dbeta[c] = pacc ? dbeta[c] + (float)s : (float)s;
  if (dgamma) dgamma[c] = pacc ? dgamma[c] + (float)q : (float)q;
  k12[c] = (float)(s / (double)rows);
  k12[C + c] = (float)(q / (double)rows);
}

// ---- elementwise ----
struct ApplyParams {
  const float* x;
  long rows;
  int C;
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  const float* scale;  // affine form (mean == NULL): y = act(x*scale + shift)
  const float* shift;
  int act;
  const float* gate;
  const float* res;
  FastDiv dHW;
  FastDiv dCV;
  float* y;
  const float* sscale;  // per image (drop-connect): y = act(bn(x) * sscale[img] + res), or NULL
};

// The host sizes the grid so that its thread count is a multiple of C / VW: every thread's
// elements then share one channel group, and the per-channel parameters are loaded once per
// thread instead of once per element (ew_grid_c).
template <int VW>
__global__ __launch_bounds__(256) void bn_apply_kernel(ApplyParams p) {
  const long nv = p.rows * p.C / VW;
  const int CV = p.C / VW;
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nv) return;
  const int c0 = (int)(e - (long)p.dCV.div((uint32_t)e) * CV) * VW;
  float mu[VW], is[VW], ga[VW], be[VW];
  if (p.mean) {
    ld<VW>(p.mean + c0, mu);
    ld<VW>(p.invstd + c0, is);
    ld<VW>(p.gamma + c0, ga);
    ld<VW>(p.beta + c0, be);
  } else {
    ld<VW>(p.scale + c0, mu);
    ld<VW>(p.shift + c0, is);
  }
  for (; e < nv; e += (long)gridDim.x * blockDim.x) {
    float xv[VW], g[VW];
    ld<VW>(p.x + e * VW, xv);
    if (p.mean) {
#pragma unroll
      for (int u = 0; u < VW; ++u) xv[u] = ((xv[u] - mu[u]) * is[u]) * ga[u] + be[u];
    } else {
#pragma unroll
      for (int u = 0; u < VW; ++u) xv[u] = xv[u] * mu[u] + is[u];
    }
    if (p.sscale) {  // drop-connect scale of the BN output, then + the residual: two roundings, as
                     // Keras' Dropout product and Add (and residual_add)
      const float sc = p.sscale[p.dHW.div((uint32_t)p.dCV.div((uint32_t)e))];
      if (p.res) {
        float rv[VW];
        ld<VW>(p.res + e * VW, rv);
#pragma unroll
        for (int u = 0; u < VW; ++u) xv[u] = add_rn(mul_rn(xv[u], sc), rv[u]);
      } else {
#pragma unroll
        for (int u = 0; u < VW; ++u) xv[u] = mul_rn(xv[u], sc);
      }
    } else if (p.res) {
      float rv[VW];
      ld<VW>(p.res + e * VW, rv);
#pragma unroll
      for (int u = 0; u < VW; ++u) xv[u] = add_rn(xv[u], rv[u]);
    }
#pragma unroll
    for (int u = 0; u < VW; ++u) g[u] = 1.f;
    if (p.gate) {
      const long r = (long)p.dCV.div((uint32_t)e);
      ld<VW>(p.gate + (long)p.dHW.div((uint32_t)r) * p.C + c0, g);
    }
#pragma unroll
    for (int u = 0; u < VW; ++u) xv[u] = act_fwd(p.act, xv[u]) * g[u];
    if constexpr (VW == 4)
      st_nt4(p.y + e * 4, make_float4(xv[0], xv[1], xv[2], xv[3]));
    else
      p.y[e] = xv[0];
  }
}

struct BwdApplyParams {
  const float* x;
  const float* dy;
  long rows;
  int C;
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
  const float* gate;
  const float* addn;
  FastDiv dHW;
  const float* k12;
  float* dx;
  int acc;
  FastDiv dCV;
  const float* res;
  float* dres;  // receives dz = d(act input), the residual branch's gradient (or NULL)
  int dres_acc;
  const float* sscale;  // dy scaled per image (drop-connect), or NULL
};

template <int VW, int ACT = -1>  // ACT >= 0: compile-time activation (as chan_reduce_kernel)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BwdApplyParams p) {
  const int act_id = ACT >= 0 ? ACT : p.act;
  const long nv = p.rows * p.C / VW;
  const int CV = p.C / VW;
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nv) return;
  // one channel group per thread (grid from ew_grid_c): parameters loaded once
  const int c0 = (int)(e - (long)p.dCV.div((uint32_t)e) * CV) * VW;
  float mu[VW], is[VW], ga[VW], be[VW], k1[VW], k2[VW];
  ld<VW>(p.mean + c0, mu);
  ld<VW>(p.invstd + c0, is);
  ld<VW>(p.gamma + c0, ga);
  ld<VW>(p.beta + c0, be);
  ld<VW>(p.k12 + c0, k1);
  ld<VW>(p.k12 + p.C + c0, k2);
  for (; e < nv; e += (long)gridDim.x * blockDim.x) {
    float xv[VW], dv[VW], g[VW], a[VW];
    ld<VW>(p.x + e * VW, xv);
    ld<VW>(p.dy + e * VW, dv);
#pragma unroll
    for (int u = 0; u < VW; ++u) { g[u] = 1.f; a[u] = 0.f; }
    if (p.gate || p.addn || p.sscale) {
      const long r = (long)p.dCV.div((uint32_t)e);
      const long img = (long)p.dHW.div((uint32_t)r);
      if (p.gate) ld<VW>(p.gate + img * p.C + c0, g);
      if (p.addn) ld<VW>(p.addn + img * p.C + c0, a);
      if (p.sscale) {
        const float sc = p.sscale[img];
#pragma unroll
        for (int u = 0; u < VW; ++u) dv[u] = mul_rn(dv[u], sc);
      }
    }
    float rv[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) rv[u] = 0.f;
    if (p.res) ld<VW>(p.res + e * VW, rv);
    float o[VW], dzs[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) {
      const float xh = (xv[u] - mu[u]) * is[u];
      const float z = (xh * ga[u] + be[u]) + rv[u];
      const float dz = (dv[u] * g[u] + a[u]) * act_grad(act_id, z);
      dzs[u] = dz;
      o[u] = (is[u] * ga[u]) * (dz - k1[u] - xh * k2[u]);
    }
    if (p.dres) {
#pragma unroll
      for (int u = 0; u < VW; ++u) {
        float* d = p.dres + e * VW + u;
        *d = p.dres_acc ? *d + dzs[u] : dzs[u];
      }
    }
    if (!p.dx) continue;
    if constexpr (VW == 4) {
      float4* d = reinterpret_cast<float4*>(p.dx + e * 4);
      float4 v = make_float4(o[0], o[1], o[2], o[3]);
      if (p.acc) {
        const float4 old = *d;
        v.x += old.x; v.y += old.y; v.z += old.z; v.w += old.w;
      }
      st_nt4(reinterpret_cast<float*>(d), v);
    } else {
      p.dx[e] = p.acc ? p.dx[e] + o[0] : o[0];
    }
  }
}

static unsigned ew_grid(long nv) { return std::min<unsigned>(std::max(cdiv(nv, 256), 1u), 8192); }

// ew_grid with 256 * grid a multiple of cv when the grid-stride loop iterates (see bn_apply_kernel)
static unsigned ew_grid_c(long nv, int cv) {
  unsigned g = ew_grid(nv);
  if ((long)g * 256 >= nv) return g;  // one element per thread
  int a = 256, b = cv;
  while (b) { const int t = a % b; a = b; b = t; }
  const unsigned m = (unsigned)(cv / a);  // 256 * g % cv == 0  <=>  g % m == 0
  return std::max(m, g / m * m);
}

static size_t red_ws_doubles(long rows, int C) {
  int nbx, rpb;
  red_plan(rows, C, nbx, rpb);
  return (size_t)nbx * C * 2;
}

__global__ void bn_infer_kernel(const float* __restrict__ g, const float* __restrict__ b,
                                const float* __restrict__ mm, const float* __restrict__ mv, int c,
                                float eps, float* __restrict__ sc, float* __restrict__ sh) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  const float s = g[i] / sqrtf(mv[i] + eps);
  sc[i] = s;
  sh[i] = b[i] - mm[i] * s;
}

__global__ void bn_train_coeffs_kernel(const float* __restrict__ mean,
                                       const float* __restrict__ invstd,
                                       const float* __restrict__ g, const float* __restrict__ b,
                                       int c, float* __restrict__ sc, float* __restrict__ sh) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  const float s = g[i] * invstd[i];
  sc[i] = s;
  sh[i] = b[i] - mean[i] * s;
}

// one output row (cout = 4 or 8 floats: 1 or 2 float4) per thread
template <int CO>
__global__ __launch_bounds__(256) void channel_pad_affine_kernel(
    const float* __restrict__ x, long rows, int cin, const float* __restrict__ sc,
    const float* __restrict__ sh, float* __restrict__ y) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float o[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    float v = 0.f;
    if (c < cin) {
      v = x[r * cin + c];
      if (sc) v = v * sc[c] + sh[c];
    }
    o[c] = v;
  }
  float4* d = reinterpret_cast<float4*>(y + r * CO);
#pragma unroll
  for (int q = 0; q < CO / 4; ++q) d[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
}

}  // namespace pld

using namespace pld;

extern "C" int pld_channel_pad_affine(const float* x, int64_t rows, int cin, int cout,
                                      const float* scale, const float* shift, float* y,
                                      void* stream) {
  PLD_CHECK_ARG(x && y && rows > 0 && cin > 0 && cin <= cout && (cout == 4 || cout == 8) &&
                    aligned16(y) && (scale == nullptr) == (shift == nullptr),
                "pld_channel_pad_affine: bad args");
  const unsigned g = (unsigned)cdiv(rows, 256);
  if (cout == 4)
    channel_pad_affine_kernel<4><<<g, 256, 0, as_stream(stream)>>>(x, rows, cin, scale, shift, y);
  else
    channel_pad_affine_kernel<8><<<g, 256, 0, as_stream(stream)>>>(x, rows, cin, scale, shift, y);
  return check_launch("channel_pad_affine_kernel");
}

extern "C" int pld_bn_train_coeffs(const float* mean, const float* invstd, const float* gamma,
                                   const float* beta, int c, float* scale, float* shift,
                                   void* stream) {
  PLD_CHECK_ARG(mean && invstd && gamma && beta && scale && shift && c > 0,
                "pld_bn_train_coeffs: bad args");
  bn_train_coeffs_kernel<<<cdiv(c, 256), 256, 0, as_stream(stream)>>>(mean, invstd, gamma, beta,
                                                                      c, scale, shift);
  return check_launch("bn_train_coeffs_kernel");
}

extern "C" int pld_bn_inference_coeffs(const float* gamma, const float* beta,
                                       const float* moving_mean, const float* moving_var, int c,
                                       float eps, float* scale, float* shift, void* stream) {
  PLD_CHECK_ARG(gamma && beta && moving_mean && moving_var && scale && shift && c > 0,
                "pld_bn_inference_coeffs: bad args");
  bn_infer_kernel<<<cdiv(c, 256), 256, 0, as_stream(stream)>>>(gamma, beta, moving_mean,
                                                                moving_var, c, eps, scale, shift);
  return check_launch("bn_infer_kernel");
}

extern "C" size_t pld_channel_reduce_workspace_size(int64_t rows, int c) {
  if (rows <= 0 || c <= 0) return 0;
  // fp64 partials + 2*C floats of BN-backward coefficients
  return red_ws_doubles(rows, c) * sizeof(double) + 2 * sizeof(float) * (size_t)c + 64;
}

extern "C" int pld_channel_sum(const float* x, int64_t rows, int c, float* out, int accumulate,
                               void* ws, void* stream) {
  PLD_CHECK_ARG(x && out && ws && rows > 0 && c > 0, "pld_channel_sum: bad args");
  PLD_CHECK_ARG(rows < (1L << 31), "pld_channel_sum: too many rows");
  RedParams p{};
  p.x = x;
  p.rows = rows;
  p.C = c;
  p.partial = (double*)ws;
  hipStream_t st = as_stream(stream);
  int rc = launch_reduce(RED_SUM, p, st);
  if (rc) return rc;
  int nbx, rpb;
  red_plan(rows, c, nbx, rpb);
  sum_finalize_kernel<<<c, 256, 0, st>>>(p.partial, nbx, c, out, accumulate);
  return check_launch("sum_finalize_kernel");
}

extern "C" int pld_bn_stats(const float* x, int64_t rows, int c, float eps, float momentum,
                            float* mean, float* invstd, float* moving_mean, float* moving_var,
                            void* ws, void* stream) {
  PLD_CHECK_ARG(x && mean && invstd && ws && rows > 0 && c > 0, "pld_bn_stats: bad args");
  PLD_CHECK_ARG(rows < (1L << 31), "pld_bn_stats: too many rows");
  PLD_CHECK_ARG((moving_mean == nullptr) == (moving_var == nullptr),
                "pld_bn_stats: moving_mean/moving_var must both be given or both NULL");
  RedParams p{};
  p.x = x;
  p.rows = rows;
  p.C = c;
  p.partial = (double*)ws;
  hipStream_t st = as_stream(stream);
  int rc = launch_reduce(RED_STATS, p, st);
  if (rc) return rc;
  int nbx, rpb;
  red_plan(rows, c, nbx, rpb);
  stats_finalize_kernel<<<c, 256, 0, st>>>(p.partial, nbx, c, rows, eps, momentum,
                                                       mean, invstd, moving_mean, moving_var);
  return check_launch("stats_finalize_kernel");
}

// internal (conv producers that gather the statistics of their output): finalize only
extern "C" int pld__bn_stats_finish(const double* part, int nparts, int64_t rows, int c,
                                    float eps, float momentum, float* mean, float* invstd,
                                    float* moving_mean, float* moving_var, hipStream_t st) {
  PLD_CHECK_ARG(part && mean && invstd && rows > 0 && c > 0 && nparts > 0,
                "pld__bn_stats_finish: bad args");
  stats_finalize_kernel<<<c, 256, 0, st>>>(part, nparts, c, rows, eps, momentum, mean, invstd,
                                           moving_mean, moving_var);
  return check_launch("stats_finalize_kernel");
}

static int bn_apply_impl(const float* x, int64_t rows, int c, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, int act,
                         const float* gate, int hw, const float* res, float* y, void* stream,
                         const float* sscale = nullptr) {
  PLD_CHECK_ARG(x && y && mean && invstd && gamma && beta && rows > 0 && c > 0,
                "pld_bn_apply: bad args");
  PLD_CHECK_ARG(!res || c % 4 != 0 || aligned16(res), "pld_bn_add_apply: res misaligned");
  PLD_CHECK_ARG(!(gate || sscale) || hw > 0, "pld_bn_apply: gate / sample scale need hw > 0");
  ApplyParams p{};
  p.x = x;
  p.rows = rows;
  p.C = c;
  p.mean = mean;
  p.invstd = invstd;
  p.gamma = gamma;
  p.beta = beta;
  p.act = act;
  p.gate = gate;
  p.res = res;
  p.sscale = sscale;
  p.dHW = FastDiv((uint32_t)std::max(hw, 1));
  p.y = y;
  p.dCV = FastDiv((uint32_t)(c % 4 == 0 ? c / 4 : c));
  PLD_CHECK_ARG(rows * c < (1L << 31), "elementwise: tensor too large");
  hipStream_t st = as_stream(stream);
  if (c % 4 == 0) {
    bn_apply_kernel<4><<<ew_grid_c(rows * c / 4, c / 4), 256, 0, st>>>(p);
  } else {
    bn_apply_kernel<1><<<ew_grid_c(rows * c, c), 256, 0, st>>>(p);
  }
  return check_launch("bn_apply_kernel");
}

extern "C" int pld_bn_apply(const float* x, int64_t rows, int c, const float* mean,
                            const float* invstd, const float* gamma, const float* beta, int act,
                            const float* gate, int hw, float* y, void* stream) {
  return bn_apply_impl(x, rows, c, mean, invstd, gamma, beta, act, gate, hw, nullptr, y, stream);
}

extern "C" int pld_bn_add_apply(const float* x, int64_t rows, int c, const float* mean,
                                const float* invstd, const float* gamma, const float* beta,
                                const float* res, int act, float* y, void* stream) {
  PLD_CHECK_ARG(res, "pld_bn_add_apply: res is NULL");
  return bn_apply_impl(x, rows, c, mean, invstd, gamma, beta, act, nullptr, 0, res, y, stream);
}

// EfficientNet's residual MBConv output (Keras EfficientNetB0 block: Dropout(noise_shape =
// (None, 1, 1, 1)) then add, applied to the project BN's output): y = act(bn(x) * sscale[img] +
// res) in one pass, with the same roundings as bn_apply followed by residual_add (scale and
// residual in one fma). sscale NULL = bn_add_apply.
extern "C" int pld_bn_scale_add_apply(const float* x, int64_t rows, int c, const float* mean,
                                      const float* invstd, const float* gamma, const float* beta,
                                      const float* sample_scale, int hw, const float* res, int act,
                                      float* y, void* stream) {
  PLD_CHECK_ARG(res, "pld_bn_scale_add_apply: res is NULL");
  return bn_apply_impl(x, rows, c, mean, invstd, gamma, beta, act, nullptr, hw, res, y, stream,
                       sample_scale);
}

extern "C" int pld_channel_affine_act(const float* x, int64_t rows, int c, const float* scale,
                                      const float* shift, int act, float* y, void* stream) {
  PLD_CHECK_ARG(x && y && scale && shift && rows > 0 && c > 0, "pld_channel_affine_act: bad args");
  ApplyParams p{};
  p.x = x;
  p.rows = rows;
  p.C = c;
  p.scale = scale;
  p.shift = shift;
  p.act = act;
  p.dHW = FastDiv(1);
  p.y = y;
  p.dCV = FastDiv((uint32_t)(c % 4 == 0 ? c / 4 : c));
  PLD_CHECK_ARG(rows * c < (1L << 31), "elementwise: tensor too large");
  hipStream_t st = as_stream(stream);
  if (c % 4 == 0) {
    bn_apply_kernel<4><<<ew_grid_c(rows * c / 4, c / 4), 256, 0, st>>>(p);
  } else {
    bn_apply_kernel<1><<<ew_grid_c(rows * c, c), 256, 0, st>>>(p);
  }
  return check_launch("bn_apply_kernel(affine)");
}

static int bn_bwd_finish(const double* part, int nbx, const float* x, const float* dy,
                         int64_t rows, int c, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int act, const float* gate,
                         const float* addn, FastDiv dHW, const float* res, float* dx,
                         int dx_accumulate, float* dres, int dres_accumulate, float* dgamma,
                         float* dbeta, int param_accumulate, float* k12, hipStream_t st,
                         const float* sscale = nullptr);

static int bn_bwd_impl(const float* x, const float* dy, int64_t rows, int c, const float* mean,
                       const float* invstd, const float* gamma, const float* beta, int act,
                       const float* gate, const float* addn, int hw, const float* res,
                       float* dx, int dx_accumulate, float* dres, int dres_accumulate,
                       float* dgamma, float* dbeta, int param_accumulate, void* ws,
                       void* stream, const float* sscale = nullptr) {
  PLD_CHECK_ARG(x && dy && mean && invstd && gamma && beta && ws && rows > 0 && c > 0,
                "pld_bn_bwd: bad args");
  PLD_CHECK_ARG(rows < (1L << 31), "pld_bn_bwd: too many rows");
  PLD_CHECK_ARG(!(gate || addn || sscale) || hw > 0, "pld_bn_bwd: gate/addn/scale need hw > 0");
  hipStream_t st = as_stream(stream);
  RedParams p{};
  p.x = x;
  p.dy = dy;
  p.rows = rows;
  p.C = c;
  p.mean = mean;
  p.invstd = invstd;
  p.gamma = gamma;
  p.beta = beta;
  p.act = act;
  p.gate = gate;
  p.addn = addn;
  p.res = res;
  p.sscale = sscale;
  p.dHW = FastDiv((uint32_t)std::max(hw, 1));
  p.partial = (double*)ws;
  // Residual form with an activation and a fresh dres: the reduction pass stores dz (= dres, the
  // residual branch's gradient) as it goes, and the elementwise pass then reads (x, dz) instead
  // of (x, dy, res): 28 instead of 32 bytes per element. Without an activation dz = dy and the
  // mask needs no residual.
  const bool dz_pass = res && act != ACT_NONE && dres && !dres_accumulate && !gate && !addn &&
                       !sscale && dres != dy && dres != x && dres != res;
  if (res && act == ACT_NONE) p.res = nullptr;
  if (dz_pass) p.dz_out = dres;
  int rc = launch_reduce(RED_BNBWD, p, st);
  if (rc) return rc;
  int nbx, rpb;
  red_plan(rows, c, nbx, rpb);
  float* k12 = reinterpret_cast<float*>((char*)ws + red_ws_doubles(rows, c) * sizeof(double));
  if (dz_pass)
    return bn_bwd_finish(p.partial, nbx, x, dres, rows, c, mean, invstd, gamma, beta, ACT_NONE,
                         nullptr, nullptr, p.dHW, nullptr, dx, dx_accumulate, nullptr, 0, dgamma,
                         dbeta, param_accumulate, k12, st);
  return bn_bwd_finish(p.partial, nbx, x, dy, rows, c, mean, invstd, gamma, beta, act, gate, addn,
                       p.dHW, p.res, dx, dx_accumulate, dres, dres_accumulate, dgamma, dbeta,
                       param_accumulate, k12, st, sscale);
}

// finalize (dgamma, dbeta, k1 = mean dz, k2 = mean dz xhat from nbx channel-major partials) +
// the elementwise dx / dres pass
static int bn_bwd_finish(const double* part, int nbx, const float* x, const float* dy,
                         int64_t rows, int c, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int act, const float* gate,
                         const float* addn, FastDiv dHW, const float* res, float* dx,
                         int dx_accumulate, float* dres, int dres_accumulate, float* dgamma,
                         float* dbeta, int param_accumulate, float* k12, hipStream_t st,
                         const float* sscale) {
  bnbwd_finalize_kernel<<<c, 256, 0, st>>>(part, nbx, c, rows, dgamma, dbeta,
                                                       param_accumulate, k12);
  int rc = check_launch("bnbwd_finalize_kernel");
  if (rc || !(dx || dres)) return rc;
  BwdApplyParams q{};
  q.x = x;
  q.dy = dy;
  q.rows = rows;
  q.C = c;
  q.mean = mean;
  q.invstd = invstd;
  q.gamma = gamma;
  q.beta = beta;
  q.act = act;
  q.gate = gate;
  q.addn = addn;
  q.dHW = dHW;
  q.k12 = k12;
  q.dx = dx;
  q.acc = dx_accumulate;
  q.dCV = FastDiv((uint32_t)(c % 4 == 0 ? c / 4 : c));
  q.res = res;
  q.dres = dres;
  q.dres_acc = dres_accumulate;
  q.sscale = sscale;
  if (c % 4 == 0) {
    const unsigned g = ew_grid_c(rows * c / 4, c / 4);
    if (act == ACT_NONE) bn_bwd_apply_kernel<4, ACT_NONE><<<g, 256, 0, st>>>(q);
    else if (act == ACT_RELU) bn_bwd_apply_kernel<4, ACT_RELU><<<g, 256, 0, st>>>(q);
    else if (act == ACT_SWISH) bn_bwd_apply_kernel<4, ACT_SWISH><<<g, 256, 0, st>>>(q);
    else bn_bwd_apply_kernel<4><<<g, 256, 0, st>>>(q);
  } else {
    bn_bwd_apply_kernel<1><<<ew_grid_c(rows * c, c), 256, 0, st>>>(q);
  }
  return check_launch("bn_bwd_apply_kernel");
}

// internal (upconv.hip): the BN backward from partials a producer kernel accumulated
extern "C" int pld__bn_bwd_finish(const double* part, int nparts, const float* x, const float* dy,
                                  int64_t rows, int c, const float* mean, const float* invstd,
                                  const float* gamma, const float* beta, int act,
                                  const float* gate, const float* addn, int hw, float* dx,
                                  int dx_accumulate, float* dgamma, float* dbeta,
                                  int param_accumulate, float* k12, hipStream_t st) {
  PLD_CHECK_ARG(part && x && dy && mean && invstd && gamma && beta && k12 && rows > 0 && c > 0,
                "pld__bn_bwd_finish: bad args");
  PLD_CHECK_ARG(rows * c < (1L << 31), "pld__bn_bwd_finish: tensor too large");
  PLD_CHECK_ARG(!(gate || addn) || hw > 0, "pld__bn_bwd_finish: gate/addn need hw > 0");
  return bn_bwd_finish(part, nparts, x, dy, rows, c, mean, invstd, gamma, beta, act, gate, addn,
                       FastDiv((uint32_t)std::max(hw, 1)), nullptr, dx, dx_accumulate, nullptr, 0,
                       dgamma, dbeta, param_accumulate, k12, st);
}

// the reductions + finalize of pld_bn_bwd without its elementwise pass: dgamma/dbeta and the
// per-channel coefficients k12 = [mean dz | mean dz xhat] for a consumer that applies the
// backward on the fly (pgemm.hip's PRO_BNBWD)
extern "C" int pld_bn_bwd_coeffs(const float* x, const float* dy, int64_t rows, int c,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, int act, float* dgamma, float* dbeta,
                                 int param_accumulate, float* k12, void* ws, void* stream) {
  PLD_CHECK_ARG(x && dy && mean && invstd && gamma && beta && k12 && ws && rows > 0 && c > 0,
                "pld_bn_bwd_coeffs: bad args");
  PLD_CHECK_ARG(rows < (1L << 31), "pld_bn_bwd_coeffs: too many rows");
  hipStream_t st = as_stream(stream);
  RedParams p{};
  p.x = x;
  p.dy = dy;
  p.rows = rows;
  p.C = c;
  p.mean = mean;
  p.invstd = invstd;
  p.gamma = gamma;
  p.beta = beta;
  p.act = act;
  p.dHW = FastDiv(1);
  p.partial = (double*)ws;
  int rc = launch_reduce(RED_BNBWD, p, st);
  if (rc) return rc;
  int nbx, rpb;
  red_plan(rows, c, nbx, rpb);
  bnbwd_finalize_kernel<<<c, 256, 0, st>>>(p.partial, nbx, c, rows, dgamma, dbeta,
                                                       param_accumulate, k12);
  return check_launch("bnbwd_finalize_kernel");
}

extern "C" int pld_bn_bwd(const float* x, const float* dy, int64_t rows, int c, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, int act,
                          const float* gate, const float* addn, int hw, float* dx,
                          int dx_accumulate, float* dgamma, float* dbeta, int param_accumulate,
                          void* ws, void* stream) {
  return bn_bwd_impl(x, dy, rows, c, mean, invstd, gamma, beta, act, gate, addn, hw, nullptr,
                     dx, dx_accumulate, nullptr, 0, dgamma, dbeta, param_accumulate, ws, stream);
}

// the backward of pld_bn_scale_add_apply's BN branch: BN(+act) backward of dy * sscale[img]
// (the drop-connect scale folded into both passes instead of a scaled copy of dy)
extern "C" int pld_bn_bwd_scaled(const float* x, const float* dy, int64_t rows, int c,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, int act, const float* sample_scale, int hw,
                                 float* dx, int dx_accumulate, float* dgamma, float* dbeta,
                                 int param_accumulate, void* ws, void* stream) {
  PLD_CHECK_ARG(sample_scale, "pld_bn_bwd_scaled: sample_scale is NULL");
  return bn_bwd_impl(x, dy, rows, c, mean, invstd, gamma, beta, act, nullptr, nullptr, hw,
                     nullptr, dx, dx_accumulate, nullptr, 0, dgamma, dbeta, param_accumulate, ws,
                     stream, sample_scale);
}

extern "C" int pld_bn_add_bwd(const float* x, const float* dy, int64_t rows, int c,
                              const float* mean, const float* invstd, const float* gamma,
                              const float* beta, const float* res, int act, float* dx,
                              int dx_accumulate, float* dres, int dres_accumulate, float* dgamma,
                              float* dbeta, int param_accumulate, void* ws, void* stream) {
  PLD_CHECK_ARG(res, "pld_bn_add_bwd: res is NULL");
  PLD_CHECK_ARG(c % 4 != 0 || ((aligned16(res)) && (!dres || aligned16(dres))),
                "pld_bn_add_bwd: res/dres misaligned");
  return bn_bwd_impl(x, dy, rows, c, mean, invstd, gamma, beta, act, nullptr, nullptr, 0, res,
                     dx, dx_accumulate, dres, dres_accumulate, dgamma, dbeta, param_accumulate,
                     ws, stream);
}

// Bilinear x2 upsampling (fwd + adjoint) and the per-sample residual combine.
//
// UpSampling2D(interpolation='bilinear') (pldepth/models/pl_hourglass.py:62,71,80,89,94) resolves
// to tf.image.resize(bilinear, half_pixel_centers=True): out row o samples in = (o+0.5)/2-0.5,
// lower = max(floor(in),0), upper = min(ceil(in), h-1), lerp = in-floor(in); computed here in the
// same lerp form (top + (bottom-top)*ylerp). The gradient (ResizeBilinearGrad) is the adjoint,
// written as a gather: input row k receives output rows 2k-1 (w .25), 2k (w .75, or 1 at k=0),
// 2k+1 (w .75, or 1 at k=h-1), 2k+2 (w .25); the 2-D weight is the product of the 1-D weights.
// Both are HBM-bound, float4 over channels.
//
// pld_residual_add: EfficientNet block output = Dropout(noise_shape=(N,1,1,1))(x) + inputs
// (keras efficientnet.py block(), drop-connect rate 0.2*b/16): a per-sample keep/(1-rate) scale.
#include <algorithm>

#include "common.h"

namespace pld {

template <int VW>
__device__ __forceinline__ void ld4(const float* p, float (&v)[VW]) {
  if constexpr (VW == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = *p;
  }
}

template <int VW>
__device__ __forceinline__ void st4(float* p, const float (&v)[VW]) {
  if constexpr (VW == 4)
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else
    *p = v[0];
}

__device__ __forceinline__ void lerp_coords(int o, int in_size, int& lo, int& hi, float& l) {
  const float in = ((float)o + 0.5f) * 0.5f - 0.5f;
  const float f = floorf(in);
  lo = max((int)f, 0);
  hi = min((int)ceilf(in), in_size - 1);
  l = in - f;
}

// optional input prologue: the decoder's BN + ReLU applied to each tap on the fly (the
// activation before the upsampling is never materialised in training)
struct UpPro {
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
};

// 2x bilinear upsample, one thread per INPUT cell (i, j) and channel quad: the four outputs
// (2i + a, 2j + b) read only rows i-1..i+1 / columns j-1..j+1 (clamped), so the 3x3 cells are
// loaded (and BN-prologued) once for four outputs instead of 4 taps per output; every output is
// still formed by lerp_coords' taps and the same top/bottom arithmetic (bit-identical).
template <bool PRO>
__global__ __launch_bounds__(256) void upsample2x_fwd_cell_kernel(
    const float* __restrict__ x, int n, int h, int w, int c, UpPro pr, float* __restrict__ y,
    FastDiv dCV, FastDiv dW, FastDiv dH) {
  const uint32_t total = (uint32_t)n * dH.d * dW.d * dCV.d;
  const int W2 = 2 * w;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    const uint32_t t = dCV.div(e);
    const int q = (int)(e - t * dCV.d);
    const uint32_t t2 = dW.div(t);
    const int j = (int)(t - t2 * dW.d);
    const uint32_t img_u = dH.div(t2);
    const int i = (int)(t2 - img_u * dH.d);
    const float* base = x + (long)img_u * h * w * c + q * 4;
    float4 mu, is, ga, be;
    if (PRO) {
      mu = *reinterpret_cast<const float4*>(pr.mean + q * 4);
      is = *reinterpret_cast<const float4*>(pr.invstd + q * 4);
      ga = *reinterpret_cast<const float4*>(pr.gamma + q * 4);
      be = *reinterpret_cast<const float4*>(pr.beta + q * 4);
    }
    // cells[r][s] = input (rr[r], cc[s]) with rr = {i-1, i, i+1} clamped (same for columns)
    const int rr[3] = {max(i - 1, 0), i, min(i + 1, h - 1)};
    const int cc[3] = {max(j - 1, 0), j, min(j + 1, w - 1)};
    float4 cell[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        float4 v = *reinterpret_cast<const float4*>(base + ((long)rr[r] * w + cc[s2]) * c);
        if (PRO) {
          v.x = act_fwd(pr.act, ((v.x - mu.x) * is.x) * ga.x + be.x);
          v.y = act_fwd(pr.act, ((v.y - mu.y) * is.y) * ga.y + be.y);
          v.z = act_fwd(pr.act, ((v.z - mu.z) * is.z) * ga.z + be.z);
          v.w = act_fwd(pr.act, ((v.w - mu.w) * is.w) * ga.w + be.w);
        }
        cell[r][s2] = v;
      }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      int y0, y1;
      float yl;
      lerp_coords(2 * i + a, h, y0, y1, yl);
      // y0 / y1 as an index into rr: y0 is i-1 (clamped) or i, y1 is i or i+1 (clamped)
      const int r0 = a == 0 ? 0 : 1, r1 = a == 0 ? 1 : 2;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        int x0, x1;
        float xl;
        lerp_coords(2 * j + b, w, x0, x1, xl);
        const int s0 = b == 0 ? 0 : 1, s1 = b == 0 ? 1 : 2;
        const float4 tl = cell[r0][s0], tr = cell[r0][s1], bl = cell[r1][s0], br = cell[r1][s1];
        float4 o;
        {
          const float top = tl.x + (tr.x - tl.x) * xl, bot = bl.x + (br.x - bl.x) * xl;
          o.x = top + (bot - top) * yl;
        }
        {
          const float top = tl.y + (tr.y - tl.y) * xl, bot = bl.y + (br.y - bl.y) * xl;
          o.y = top + (bot - top) * yl;
        }
        {
          const float top = tl.z + (tr.z - tl.z) * xl, bot = bl.z + (br.z - bl.z) * xl;
          o.z = top + (bot - top) * yl;
        }
        {
          const float top = tl.w + (tr.w - tl.w) * xl, bot = bl.w + (br.w - bl.w) * xl;
          o.w = top + (bot - top) * yl;
        }
        *reinterpret_cast<float4*>(y + (((long)img_u * 2 * h + 2 * i + a) * W2 + 2 * j + b) * c +
                                   q * 4) = o;
      }
    }
  }
}

template <int VW, bool PRO>
__global__ __launch_bounds__(256) void upsample2x_fwd_kernel(const float* __restrict__ x, int n,
                                                             int h, int w, int c, UpPro pr,
                                                             float* __restrict__ y, FastDiv dCV,
                                                             FastDiv dW2, FastDiv dH2) {
  // 32-bit index math through multiply-high dividers (the host checks total < 2^31): 64-bit
  // div/mod is a long instruction sequence per element
  const uint32_t total = (uint32_t)n * dH2.d * dW2.d * dCV.d;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    const uint32_t t = dCV.div(e);
    const int q = (int)(e - t * dCV.d);
    const uint32_t t2 = dW2.div(t);
    const int ox = (int)(t - t2 * dW2.d);
    const uint32_t img_u = dH2.div(t2);
    const int oy = (int)(t2 - img_u * dH2.d);
    const int img = (int)img_u;
    int y0, y1, x0, x1;
    float yl, xl;
    lerp_coords(oy, h, y0, y1, yl);
    lerp_coords(ox, w, x0, x1, xl);
    const float* base = x + (long)img * h * w * c + q * VW;
    float tl[VW], tr[VW], bl[VW], br[VW], o[VW];
    ld4<VW>(base + ((long)y0 * w + x0) * c, tl);
    ld4<VW>(base + ((long)y0 * w + x1) * c, tr);
    ld4<VW>(base + ((long)y1 * w + x0) * c, bl);
    ld4<VW>(base + ((long)y1 * w + x1) * c, br);
    if (PRO) {
      float mu[VW], is[VW], ga[VW], be[VW];
      ld4<VW>(pr.mean + q * VW, mu);
      ld4<VW>(pr.invstd + q * VW, is);
      ld4<VW>(pr.gamma + q * VW, ga);
      ld4<VW>(pr.beta + q * VW, be);
#pragma unroll
      for (int u = 0; u < VW; ++u) {  // the bn_apply arithmetic, then the activation
        tl[u] = act_fwd(pr.act, ((tl[u] - mu[u]) * is[u]) * ga[u] + be[u]);
        tr[u] = act_fwd(pr.act, ((tr[u] - mu[u]) * is[u]) * ga[u] + be[u]);
        bl[u] = act_fwd(pr.act, ((bl[u] - mu[u]) * is[u]) * ga[u] + be[u]);
        br[u] = act_fwd(pr.act, ((br[u] - mu[u]) * is[u]) * ga[u] + be[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < VW; ++u) {
      const float top = tl[u] + (tr[u] - tl[u]) * xl;
      const float bot = bl[u] + (br[u] - bl[u]) * xl;
      o[u] = top + (bot - top) * yl;
    }
    st4<VW>(y + (long)e * VW, o);
  }
}

// 1-D adjoint taps of input index k (size s): output indices and weights
__device__ __forceinline__ int adj_taps(int k, int s, int (&o)[4], float (&wt)[4]) {
  int cnt = 0;
  if (k >= 1) { o[cnt] = 2 * k - 1; wt[cnt++] = 0.25f; }
  o[cnt] = 2 * k; wt[cnt++] = (k == 0) ? 1.0f : 0.75f;
  o[cnt] = 2 * k + 1; wt[cnt++] = (k == s - 1) ? 1.0f : 0.75f;
  if (k <= s - 2) { o[cnt] = 2 * k + 2; wt[cnt++] = 0.25f; }
  return cnt;
}

template <int VW>
__global__ __launch_bounds__(256) void upsample2x_bwd_kernel(const float* __restrict__ dy, int n,
                                                             int h, int w, int c,
                                                             float* __restrict__ dx, int acc,
                                                             FastDiv dCV, FastDiv dW, FastDiv dH) {
  const int W2 = 2 * w;
  const uint32_t total = (uint32_t)n * dH.d * dW.d * dCV.d;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    const uint32_t t = dCV.div(e);
    const int q = (int)(e - t * dCV.d);
    const uint32_t t2 = dW.div(t);
    const int kx = (int)(t - t2 * dW.d);
    const uint32_t img_u = dH.div(t2);
    const int ky = (int)(t2 - img_u * dH.d);
    const int img = (int)img_u;
    // the 4 x 4 adjoint window at fixed positions (rows 2k-1 .. 2k+2): an absent edge tap gets
    // weight 0 and a clamped (valid) address, so all 16 loads are unconditional and in flight
    // together; fma(0, v, r) = r keeps every sum equal to adj_taps' present-taps-only order
    const int H2 = 2 * h;
    int oy[4], ox[4];
    float wy[4], wx[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      oy[a] = min(max(2 * ky - 1 + a, 0), H2 - 1);
      ox[a] = min(max(2 * kx - 1 + a, 0), W2 - 1);
    }
    wy[0] = ky >= 1 ? 0.25f : 0.f;
    wy[1] = ky == 0 ? 1.0f : 0.75f;
    wy[2] = ky == h - 1 ? 1.0f : 0.75f;
    wy[3] = ky <= h - 2 ? 0.25f : 0.f;
    wx[0] = kx >= 1 ? 0.25f : 0.f;
    wx[1] = kx == 0 ? 1.0f : 0.75f;
    wx[2] = kx == w - 1 ? 1.0f : 0.75f;
    wx[3] = kx <= w - 2 ? 0.25f : 0.f;
    const float* base = dy + (long)img * 2 * h * W2 * c + q * VW;
    float v[4][4][VW];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) ld4<VW>(base + ((long)oy[a] * W2 + ox[b]) * c, v[a][b]);
    float s[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) s[u] = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float rs[VW];
#pragma unroll
      for (int u = 0; u < VW; ++u) rs[u] = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < VW; ++u) rs[u] += wx[b] * v[a][b][u];
#pragma unroll
      for (int u = 0; u < VW; ++u) s[u] += wy[a] * rs[u];
    }
    if (acc) {
      float old[VW];
      ld4<VW>(dx + (long)e * VW, old);
#pragma unroll
      for (int u = 0; u < VW; ++u) s[u] += old[u];
    }
    st4<VW>(dx + (long)e * VW, s);
  }
}

__global__ __launch_bounds__(256) void residual_kernel(const float* __restrict__ a,
                                                       const float* __restrict__ sc,
                                                       const float* __restrict__ b, long per,
                                                       long total, float* __restrict__ y,
                                                       int acc) {
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const float s = sc ? sc[e / per] : 1.f;
    // the product and the sum rounded separately (Keras Dropout, then Add)
    float v = b ? add_rn(mul_rn(a[e], s), b[e]) : mul_rn(a[e], s);
    if (acc) v = add_rn(v, y[e]);
    y[e] = v;
  }
}

// float4 form (per % 4 == 0, 16-byte aligned, total < 2^33): 32-bit index math, the per-sample
// scale's image index through a multiply-high divider
__global__ __launch_bounds__(256) void residual4_kernel(const float4* __restrict__ a,
                                                        const float* __restrict__ sc,
                                                        const float4* __restrict__ b,
                                                        FastDiv dPer4, uint32_t total4,
                                                        float4* __restrict__ y) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total4;
       e += gridDim.x * blockDim.x) {
    const float s = sc ? sc[dPer4.div(e)] : 1.f;
    const float4 u = a[e];
    float4 v;
    if (b) {  // product and sum rounded separately, as residual_kernel
      const float4 w = b[e];
      v = make_float4(add_rn(mul_rn(u.x, s), w.x), add_rn(mul_rn(u.y, s), w.y),
                      add_rn(mul_rn(u.z, s), w.z), add_rn(mul_rn(u.w, s), w.w));
    } else {
      v = make_float4(mul_rn(u.x, s), mul_rn(u.y, s), mul_rn(u.z, s), mul_rn(u.w, s));
    }
    y[e] = v;
  }
}

__device__ __forceinline__ float dropconnect_scale(float rate, uint64_t seed, uint64_t step,
                                                   int layer, int img) {
  uint4 c = make_uint4((uint32_t)layer, (uint32_t)img, (uint32_t)step,
                       (uint32_t)(step >> 32) ^ 0x5D0Cu);
  uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int r = 0; r < 10; ++r) {  // Philox4x32-10
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  const float u = (float)(c.x >> 8) * (1.0f / 16777216.0f);  // [0, 1)
  return (u >= rate) ? 1.0f / (1.0f - rate) : 0.0f;
}

__global__ void dropconnect_kernel(float* __restrict__ sc, int n, float rate, uint64_t seed,
                                   uint64_t step_arg, const int64_t* __restrict__ step_dev,
                                   int layer, int off) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t step = step_dev ? (uint64_t)step_dev[0] : step_arg;
  sc[i] = dropconnect_scale(rate, seed, step, layer, off + i);
}

// every drop-connect layer of one step in one launch: blockIdx.y = layer slot
constexpr int DC_MAX_LAYERS = 32;
struct DcLayers {
  float rate[DC_MAX_LAYERS];
  int layer[DC_MAX_LAYERS];
};
__global__ void dropconnect_multi_kernel(float* __restrict__ sc, int n, DcLayers L, uint64_t seed,
                                         uint64_t step_arg, const int64_t* __restrict__ step_dev,
                                         int off) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t step = step_dev ? (uint64_t)step_dev[0] : step_arg;
  const int s = blockIdx.y;
  sc[(long)s * n + i] = dropconnect_scale(L.rate[s], seed, step, L.layer[s], off + i);
}

static unsigned grid_for(long n) { return std::min<unsigned>(std::max(cdiv(n, 256), 1u), 8192); }

}  // namespace pld

using namespace pld;

extern "C" int pld_upsample2x_fwd(const float* x, int n, int h, int w, int c, float* y,
                                  void* stream) {
  PLD_CHECK_ARG(x && y && n > 0 && h > 0 && w > 0 && c > 0, "pld_upsample2x_fwd: bad args");
  return pld_upsample2x_fwd_bn(x, n, h, w, c, nullptr, nullptr, nullptr, nullptr, 0, y, stream);
}

extern "C" int pld_upsample2x_fwd_bn(const float* x, int n, int h, int w, int c,
                                     const float* mean, const float* invstd, const float* gamma,
                                     const float* beta, int act, float* y, void* stream) {
  PLD_CHECK_ARG(x && y && n > 0 && h > 0 && w > 0 && c > 0, "pld_upsample2x_fwd: bad args");
  PLD_CHECK_ARG(!mean || (invstd && gamma && beta), "pld_upsample2x_fwd_bn: incomplete BN");
  hipStream_t st = as_stream(stream);
  const long total = (long)n * 4 * h * w * c;
  PLD_CHECK_ARG(total < (1L << 31), "pld_upsample2x_fwd: tensor too large for 32-bit indexing");
  const UpPro pr{mean, invstd, gamma, beta, act};
  const FastDiv dW2((uint32_t)(2 * w)), dH2((uint32_t)(2 * h));
  if (c % 4 == 0) {
    const FastDiv dCV((uint32_t)(c / 4));
    const FastDiv dW((uint32_t)w), dH((uint32_t)h);
    if (mean) upsample2x_fwd_cell_kernel<true><<<grid_for(total / 16), 256, 0, st>>>(x, n, h, w, c, pr, y, dCV, dW, dH);
    else upsample2x_fwd_cell_kernel<false><<<grid_for(total / 16), 256, 0, st>>>(x, n, h, w, c, pr, y, dCV, dW, dH);
  } else {
    const FastDiv dCV((uint32_t)c);
    if (mean) upsample2x_fwd_kernel<1, true><<<grid_for(total), 256, 0, st>>>(x, n, h, w, c, pr, y, dCV, dW2, dH2);
    else upsample2x_fwd_kernel<1, false><<<grid_for(total), 256, 0, st>>>(x, n, h, w, c, pr, y, dCV, dW2, dH2);
  }
  return check_launch("upsample2x_fwd_kernel");
}

extern "C" int pld_upsample2x_bwd(const float* dy, int n, int h, int w, int c, float* dx,
                                  int accumulate, void* stream) {
  PLD_CHECK_ARG(dy && dx && n > 0 && h > 0 && w > 0 && c > 0, "pld_upsample2x_bwd: bad args");
  hipStream_t st = as_stream(stream);
  const long total = (long)n * h * w * c;
  PLD_CHECK_ARG(4 * total < (1L << 31), "pld_upsample2x_bwd: tensor too large for 32-bit indexing");
  const FastDiv dW((uint32_t)w), dH((uint32_t)h);
  if (c % 4 == 0)
    upsample2x_bwd_kernel<4><<<grid_for(total / 4), 256, 0, st>>>(dy, n, h, w, c, dx, accumulate,
                                                                  FastDiv((uint32_t)(c / 4)), dW, dH);
  else
    upsample2x_bwd_kernel<1><<<grid_for(total), 256, 0, st>>>(dy, n, h, w, c, dx, accumulate,
                                                              FastDiv((uint32_t)c), dW, dH);
  return check_launch("upsample2x_bwd_kernel");
}

extern "C" int pld_residual_add(const float* a, const float* sample_scale, const float* b, int n,
                                int64_t elems_per_img, float* y, void* stream) {
  PLD_CHECK_ARG(a && y && n > 0 && elems_per_img > 0, "pld_residual_add: bad args");
  const long total = (long)n * elems_per_img;
  if (elems_per_img % 4 == 0 && total / 4 < (1L << 31) && aligned16(a) && aligned16(y) &&
      (!b || aligned16(b))) {
    residual4_kernel<<<grid_for(total / 4), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(a), sample_scale, reinterpret_cast<const float4*>(b),
        FastDiv((uint32_t)(elems_per_img / 4)), (uint32_t)(total / 4),
        reinterpret_cast<float4*>(y));
    return check_launch("residual4_kernel");
  }
  residual_kernel<<<grid_for(total), 256, 0, as_stream(stream)>>>(a, sample_scale, b,
                                                                  elems_per_img, total, y, 0);
  return check_launch("residual_kernel");
}

extern "C" int pld_dropconnect_scales(float* scales, int n, float rate, uint64_t seed,
                                      uint64_t step, int layer, int image_offset, void* stream) {
  PLD_CHECK_ARG(scales && n > 0 && rate >= 0.f && rate < 1.f, "pld_dropconnect_scales: bad args");
  dropconnect_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(scales, n, rate, seed, step,
                                                                  nullptr, layer, image_offset);
  return check_launch("dropconnect_kernel");
}

extern "C" int pld_dropconnect_scales_dev(float* scales, int n, float rate, uint64_t seed,
                                          const int64_t* step_dev, int layer, int image_offset,
                                          void* stream) {
  PLD_CHECK_ARG(scales && step_dev && n > 0 && rate >= 0.f && rate < 1.f,
                "pld_dropconnect_scales_dev: bad args");
  dropconnect_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(scales, n, rate, seed, 0,
                                                                  step_dev, layer, image_offset);
  return check_launch("dropconnect_kernel");
}

extern "C" int pld_dropconnect_scales_multi(float* scales, int n, int nl, const float* rates,
                                            const int* layers, uint64_t seed, uint64_t step,
                                            const int64_t* step_dev, int image_offset,
                                            void* stream) {
  PLD_CHECK_ARG(scales && rates && layers && n > 0 && nl > 0 && nl <= DC_MAX_LAYERS,
                "pld_dropconnect_scales_multi: bad args");
  DcLayers L{};
  for (int s = 0; s < nl; ++s) {
    PLD_CHECK_ARG(rates[s] >= 0.f && rates[s] < 1.f, "pld_dropconnect_scales_multi: bad rate");
    L.rate[s] = rates[s];
    L.layer[s] = layers[s];
  }
  dropconnect_multi_kernel<<<dim3(cdiv(n, 256), nl), 256, 0, as_stream(stream)>>>(
      scales, n, L, seed, step, step_dev, image_offset);
  return check_launch("dropconnect_multi_kernel");
}

extern "C" int pld_scale_per_sample(const float* x, const float* sample_scale, int n,
                                    int64_t elems_per_img, float* y, int accumulate,
                                    void* stream) {
  PLD_CHECK_ARG(x && y && n > 0 && elems_per_img > 0, "pld_scale_per_sample: bad args");
  const long total = (long)n * elems_per_img;
  residual_kernel<<<grid_for(total), 256, 0, as_stream(stream)>>>(x, sample_scale, nullptr,
                                                                  elems_per_img, total, y,
                                                                  accumulate);
  return check_launch("residual_kernel(scale)");
}

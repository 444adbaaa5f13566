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

#include "common.h"

namespace pld {

template <int K>
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ x, int n,
                                                         int h, int w, int c,
                                                         const float* __restrict__ wt, int s,
                                                         int pt, int pl, int oh, int ow,
                                                         float* __restrict__ y) {
  const int cv = c / 4;
  const long total = (long)n * oh * ow * cv;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int q = (int)(e % cv);
    long t = e / cv;
    const int ox = (int)(t % ow);
    t /= ow;
    const int oy = (int)(t % oh);
    const int img = (int)(t / oh);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* xb = x + (long)img * h * w * c + 4 * q;
#pragma unroll
    for (int ty = 0; ty < K; ++ty) {
      const int iy = oy * s + ty - pt;
      if (iy < 0 || iy >= h) continue;
#pragma unroll
      for (int tx = 0; tx < K; ++tx) {
        const int ix = ox * s + tx - pl;
        if (ix < 0 || ix >= w) continue;
        const float4 v = *reinterpret_cast<const float4*>(xb + ((long)iy * w + ix) * c);
        const float4 f = *reinterpret_cast<const float4*>(wt + (ty * K + tx) * c + 4 * q);
        acc.x += v.x * f.x;
        acc.y += v.y * f.y;
        acc.z += v.z * f.z;
        acc.w += v.w * f.w;
      }
    }
    *reinterpret_cast<float4*>(y + e * 4) = acc;
  }
}

template <int K>
__global__ __launch_bounds__(256) void dwconv_dgrad_kernel(const float* __restrict__ dy, int n,
                                                           int h, int w, int c,
                                                           const float* __restrict__ wt, int s,
                                                           int pt, int pl, int oh, int ow,
                                                           float* __restrict__ dx, int accum) {
  const int cv = c / 4;
  const long total = (long)n * h * w * cv;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int q = (int)(e % cv);
    long t = e / cv;
    const int ix = (int)(t % w);
    t /= w;
    const int iy = (int)(t % h);
    const int img = (int)(t / h);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* db = dy + (long)img * oh * ow * c + 4 * q;
#pragma unroll
    for (int ty = 0; ty < K; ++ty) {
      const int ny = iy + pt - ty;
      if (ny < 0 || ny % s) continue;
      const int oy = ny / s;
      if (oy >= oh) continue;
#pragma unroll
      for (int tx = 0; tx < K; ++tx) {
        const int nx = ix + pl - tx;
        if (nx < 0 || nx % s) continue;
        const int ox = nx / s;
        if (ox >= ow) continue;
        const float4 v = *reinterpret_cast<const float4*>(db + ((long)oy * ow + ox) * c);
        const float4 f = *reinterpret_cast<const float4*>(wt + (ty * K + tx) * c + 4 * q);
        acc.x += v.x * f.x;
        acc.y += v.y * f.y;
        acc.z += v.z * f.z;
        acc.w += v.w * f.w;
      }
    }
    float4* d = reinterpret_cast<float4*>(dx + e * 4);
    if (accum) {
      const float4 o = *d;
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
    }
    *d = acc;
  }
}

// ---- SE ----
// per-image channel sums of a (or of a*dy): partial[img][split][c] (fp64)
__global__ __launch_bounds__(256) void img_chan_sum_kernel(const float* __restrict__ a,
                                                           const float* __restrict__ b, int hw,
                                                           int c, int rsplit,
                                                           double* __restrict__ part) {
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
  if (r0 < rpi) {
    const long base = (long)img * hw * c + 4 * q;
    for (int r = rb + r0; r < re; r += rpi) {
      const float4 v = *reinterpret_cast<const float4*>(a + base + (long)r * c);
      if (b) {
        const float4 u = *reinterpret_cast<const float4*>(b + base + (long)r * c);
        s[0] += (double)(v.x * u.x); s[1] += (double)(v.y * u.y);
        s[2] += (double)(v.z * u.z); s[3] += (double)(v.w * u.w);
      } else {
        s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
      }
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
}

// forward excitation, one workgroup per image
__global__ __launch_bounds__(256) void se_fc_fwd_kernel(const double* __restrict__ part,
                                                        int rsplit, int hw, int c, int cse,
                                                        const float* __restrict__ w1,
                                                        const float* __restrict__ b1,
                                                        const float* __restrict__ w2,
                                                        const float* __restrict__ b2,
                                                        float* __restrict__ pooled,
                                                        float* __restrict__ z1,
                                                        float* __restrict__ gate) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* sp = sm;          // [c] pooled
  float* sh = sm + c;      // [cse] swish(z1)
  const int img = blockIdx.x;
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    double s = 0.0;
    for (int k = 0; k < rsplit; ++k) s += part[((long)img * rsplit + k) * c + ch];
    const float m = (float)(s / (double)hw);
    sp[ch] = m;
    pooled[(long)img * c + ch] = m;
  }
  __syncthreads();
  // z1[j] = sum_c pooled[c] w1[c][j] + b1[j]: one wave per j (round robin)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int j = wave; j < cse; j += 4) {
    float acc = 0.f;
    for (int ch = lane; ch < c; ch += 64) acc += sp[ch] * w1[(long)ch * cse + j];
    acc = wave_sum(acc);
    if (lane == 0) {
      const float z = acc + b1[j];
      z1[(long)img * cse + j] = z;
      sh[j] = z * sigmoidf_(z);
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    float acc = b2[ch];
    for (int j = 0; j < cse; ++j) acc += sh[j] * w2[(long)j * c + ch];
    gate[(long)img * c + ch] = sigmoidf_(acc);
  }
}

// backward through the excitation: addn = (d pooled) / hw
__global__ __launch_bounds__(256) void se_fc_bwd_kernel(const double* __restrict__ part,
                                                        int rsplit, int hw, int c, int cse,
                                                        const float* __restrict__ w1,
                                                        const float* __restrict__ w2,
                                                        const float* __restrict__ z1,
                                                        const float* __restrict__ gate,
                                                        float* __restrict__ addn) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dz2 = sm;       // [c]
  float* dz1 = sm + c;   // [cse]
  const int img = blockIdx.x;
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    double s = 0.0;
    for (int k = 0; k < rsplit; ++k) s += part[((long)img * rsplit + k) * c + ch];
    const float g = gate[(long)img * c + ch];
    dz2[ch] = (float)s * g * (1.f - g);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int j = wave; j < cse; j += 4) {
    float acc = 0.f;
    for (int ch = lane; ch < c; ch += 64) acc += dz2[ch] * w2[(long)j * c + ch];
    acc = wave_sum(acc);
    if (lane == 0) {
      const float z = z1[(long)img * cse + j];
      const float sg = sigmoidf_(z);
      dz1[j] = acc * (sg * (1.f + z * (1.f - sg)));
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    float acc = 0.f;
    for (int j = 0; j < cse; ++j) acc += dz1[j] * w1[(long)ch * cse + j];
    addn[(long)img * c + ch] = acc / (float)hw;
  }
}

static unsigned grid_for(long n) { return std::min<unsigned>(std::max(cdiv(n, 256), 1u), 8192); }

static int se_rsplit(int n, int hw, int c) {
  const int cy = (int)cdiv(c / 4, 256);
  int rs = (int)std::max(1L, 1024L / ((long)n * cy));
  rs = std::min(rs, std::max(1, hw / 32));
  return rs;
}

}  // namespace pld

using namespace pld;

extern "C" int pld_dwconv_fwd(const float* x, int n, int h, int w, int c, const float* wdw, int k,
                              int s, int pad_t, int pad_l, int oh, int ow, float* y,
                              void* stream) {
  PLD_CHECK_ARG(x && wdw && y && n > 0 && h > 0 && w > 0 && c > 0 && s > 0 && oh > 0 && ow > 0,
                "pld_dwconv_fwd: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_dwconv_fwd: channels must be a multiple of 4");
  const long total = (long)n * oh * ow * (c / 4);
  hipStream_t st = as_stream(stream);
  switch (k) {
    case 3: dwconv_fwd_kernel<3><<<grid_for(total), 256, 0, st>>>(x, n, h, w, c, wdw, s, pad_t, pad_l, oh, ow, y); break;
    case 5: dwconv_fwd_kernel<5><<<grid_for(total), 256, 0, st>>>(x, n, h, w, c, wdw, s, pad_t, pad_l, oh, ow, y); break;
    default: set_error("pld_dwconv_fwd: kernel size %d unsupported (3, 5)", k); return PLD_ERR_UNSUPPORTED;
  }
  return check_launch("dwconv_fwd_kernel");
}

extern "C" int pld_dwconv_dgrad(const float* dy, int n, int h, int w, int c, const float* wdw,
                                int k, int s, int pad_t, int pad_l, int oh, int ow, float* dx,
                                int accumulate, void* stream) {
  PLD_CHECK_ARG(dy && wdw && dx && n > 0 && h > 0 && w > 0 && c > 0 && s > 0 && oh > 0 && ow > 0,
                "pld_dwconv_dgrad: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_dwconv_dgrad: channels must be a multiple of 4");
  const long total = (long)n * h * w * (c / 4);
  hipStream_t st = as_stream(stream);
  switch (k) {
    case 3: dwconv_dgrad_kernel<3><<<grid_for(total), 256, 0, st>>>(dy, n, h, w, c, wdw, s, pad_t, pad_l, oh, ow, dx, accumulate); break;
    case 5: dwconv_dgrad_kernel<5><<<grid_for(total), 256, 0, st>>>(dy, n, h, w, c, wdw, s, pad_t, pad_l, oh, ow, dx, accumulate); break;
    default: set_error("pld_dwconv_dgrad: kernel size %d unsupported (3, 5)", k); return PLD_ERR_UNSUPPORTED;
  }
  return check_launch("dwconv_dgrad_kernel");
}

extern "C" size_t pld_se_workspace_size(int n, int hw, int c, int cse) {
  if (n <= 0 || hw <= 0 || c <= 0) return 0;
  return sizeof(double) * (size_t)n * se_rsplit(n, hw, c) * c;
}

extern "C" int pld_se_fwd(const float* a, int n, int hw, int c, int cse, const float* w1,
                          const float* b1, const float* w2, const float* b2, float* pooled,
                          float* z1, float* gate, void* ws, void* stream) {
  PLD_CHECK_ARG(a && w1 && b1 && w2 && b2 && pooled && z1 && gate && ws && n > 0 && hw > 0 &&
                    c > 0 && cse > 0,
                "pld_se_fwd: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_se_fwd: channels must be a multiple of 4");
  hipStream_t st = as_stream(stream);
  const int rs = se_rsplit(n, hw, c);
  dim3 g1(n * rs, cdiv(c / 4, 256));
  img_chan_sum_kernel<<<g1, 256, 0, st>>>(a, nullptr, hw, c, rs, (double*)ws);
  int rc = check_launch("img_chan_sum_kernel");
  if (rc) return rc;
  se_fc_fwd_kernel<<<n, 256, sizeof(float) * (c + cse), st>>>(
      (const double*)ws, rs, hw, c, cse, w1, b1, w2, b2, pooled, z1, gate);
  return check_launch("se_fc_fwd_kernel");
}

extern "C" int pld_se_bwd(const float* dy, const float* a, int n, int hw, int c, int cse,
                          const float* w1, const float* w2, const float* z1, const float* gate,
                          float* addn, void* ws, void* stream) {
  PLD_CHECK_ARG(dy && a && w1 && w2 && z1 && gate && addn && ws && n > 0 && hw > 0 && c > 0 &&
                    cse > 0,
                "pld_se_bwd: bad args");
  PLD_CHECK_ARG(c % 4 == 0, "pld_se_bwd: channels must be a multiple of 4");
  hipStream_t st = as_stream(stream);
  const int rs = se_rsplit(n, hw, c);
  dim3 g1(n * rs, cdiv(c / 4, 256));
  img_chan_sum_kernel<<<g1, 256, 0, st>>>(a, dy, hw, c, rs, (double*)ws);
  int rc = check_launch("img_chan_sum_kernel(bwd)");
  if (rc) return rc;
  se_fc_bwd_kernel<<<n, 256, sizeof(float) * (c + cse), st>>>((const double*)ws, rs, hw, c, cse,
                                                               w1, w2, z1, gate, addn);
  return check_launch("se_fc_bwd_kernel");
}

// Max pooling over a zero-padded input (ResNet-50 stem: ZeroPadding2D(1) -> MaxPooling2D(3, 2),
// keras.applications.resnet "pool1_pad"/"pool1_pool", reached by ReDWebNetTFVersion through
// ResNet50(include_top=False) at pldepth/models/redweb.py:410).
//
// Window positions outside the input are zeros of the padding layer and compete in the max like
// any input (value 0). Ties resolve to the first maximum in row-major window order (TF's CPU
// MaxPool/MaxPoolGrad with strict '<' updates); the forward stores that tap index (u8) so the
// backward is a deterministic gather: each input pixel sums dy over the <= ceil(k/s)^2 windows
// whose argmax tap is that pixel (a gradient routed to a padding tap is dropped, as the
// ZeroPadding2D gradient slices it away). HBM-bound; float4 over channels when C % 4 == 0.
#include <algorithm>

#include "common.h"

namespace pld {

struct PoolParams {
  int n, h, w, c, k, s, pt, pl, oh, ow;
};

template <int VW>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const float* __restrict__ x,
                                                          PoolParams p, float* __restrict__ y,
                                                          uint8_t* __restrict__ am) {
  const int CV = p.c / VW;
  const long total = (long)p.n * p.oh * p.ow * CV;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    long pix = i / CV;
    const int ox = (int)(pix % p.ow);
    pix /= p.ow;
    const int oy = (int)(pix % p.oh);
    const long img = pix / p.oh;
    float best[VW];
    int arg[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) { best[u] = 0.f; arg[u] = -1; }
    for (int ky = 0; ky < p.k; ++ky) {
      const int iy = oy * p.s - p.pt + ky;
      for (int kx = 0; kx < p.k; ++kx) {
        const int ix = ox * p.s - p.pl + kx;
        const int tap = ky * p.k + kx;
        float v[VW];
        if (iy >= 0 && iy < p.h && ix >= 0 && ix < p.w) {
          const float* src = x + ((img * p.h + iy) * p.w + ix) * p.c + cv * VW;
          if constexpr (VW == 4) {
            const float4 t = *reinterpret_cast<const float4*>(src);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
          } else {
            v[0] = *src;
          }
        } else {
#pragma unroll
          for (int u = 0; u < VW; ++u) v[u] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < VW; ++u)
          if (arg[u] < 0 || best[u] < v[u]) { best[u] = v[u]; arg[u] = tap; }
      }
    }
    const long o = ((img * p.oh + oy) * p.ow + ox) * p.c + cv * VW;
#pragma unroll
    for (int u = 0; u < VW; ++u) {
      y[o + u] = best[u];
      if (am) am[o + u] = (uint8_t)arg[u];
    }
  }
}

template <int VW>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ dy,
                                                          const uint8_t* __restrict__ am,
                                                          PoolParams p, float* __restrict__ dx,
                                                          int acc) {
  const int CV = p.c / VW;
  const long total = (long)p.n * p.h * p.w * CV;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    long pix = i / CV;
    const int ix = (int)(pix % p.w);
    pix /= p.w;
    const int iy = (int)(pix % p.h);
    const long img = pix / p.h;
    float g[VW];
#pragma unroll
    for (int u = 0; u < VW; ++u) g[u] = 0.f;
    const int ry = iy + p.pt, rx = ix + p.pl;  // position in the padded frame
    const int oy0 = max(0, (ry - p.k + p.s) / p.s), oy1 = min(p.oh - 1, ry / p.s);
    const int ox0 = max(0, (rx - p.k + p.s) / p.s), ox1 = min(p.ow - 1, rx / p.s);
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ky = ry - oy * p.s;
      if (ky < 0 || ky >= p.k) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kx = rx - ox * p.s;
        if (kx < 0 || kx >= p.k) continue;
        const int tap = ky * p.k + kx;
        const long o = ((img * p.oh + oy) * p.ow + ox) * p.c + cv * VW;
#pragma unroll
        for (int u = 0; u < VW; ++u)
          if (am[o + u] == tap) g[u] += dy[o + u];
      }
    }
    const long d = ((img * p.h + iy) * p.w + ix) * p.c + cv * VW;
#pragma unroll
    for (int u = 0; u < VW; ++u) dx[d + u] = acc ? dx[d + u] + g[u] : g[u];
  }
}

// The same for 4 channels per thread with vector loads (float4 dy, 4 argmax bytes at once)
// and 32-bit magic-number index math (< 2^31 quads): the generic form's 64-bit div/mod and
// byte-wise loads held the ResNet stem's pool backward (224^2 x 64, batch 32) at ~1 TB/s
__global__ __launch_bounds__(256) void maxpool_bwd4_kernel(const float* __restrict__ dy,
                                                           const uint8_t* __restrict__ am,
                                                           PoolParams p, FastDiv dCV,
                                                           FastDiv dW, FastDiv dH, int total,
                                                           float* __restrict__ dx, int acc) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = dCV.div((uint32_t)i);
    const int c0 = 4 * (i - (int)(pix * dCV.d));
    const uint32_t r = dW.div(pix);
    const int ix = (int)(pix - r * dW.d);
    const uint32_t img = dH.div(r);
    const int iy = (int)(r - img * dH.d);
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    const int ry = iy + p.pt, rx = ix + p.pl;
    const int oy0 = max(0, (ry - p.k + p.s) / p.s), oy1 = min(p.oh - 1, ry / p.s);
    const int ox0 = max(0, (rx - p.k + p.s) / p.s), ox1 = min(p.ow - 1, rx / p.s);
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ky = ry - oy * p.s;
      if (ky < 0 || ky >= p.k) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kx = rx - ox * p.s;
        if (kx < 0 || kx >= p.k) continue;
        const unsigned tap = (unsigned)(ky * p.k + kx);
        const long o = (((long)img * p.oh + oy) * p.ow + ox) * p.c + c0;
        const unsigned a4 = *reinterpret_cast<const unsigned*>(am + o);
        const float4 d = *reinterpret_cast<const float4*>(dy + o);
        if ((a4 & 0xffu) == tap) g.x += d.x;
        if (((a4 >> 8) & 0xffu) == tap) g.y += d.y;
        if (((a4 >> 16) & 0xffu) == tap) g.z += d.z;
        if ((a4 >> 24) == tap) g.w += d.w;
      }
    }
    float4* dst = reinterpret_cast<float4*>(dx + (long)pix * p.c + c0);
    if (acc) {
      const float4 o = *dst;
      g = make_float4(o.x + g.x, o.y + g.y, o.z + g.z, o.w + g.w);
    }
    *dst = g;
  }
}

static bool pool_ok(const PoolParams& p) {
  return p.n > 0 && p.h > 0 && p.w > 0 && p.c > 0 && p.k > 0 && p.k <= 15 && p.s > 0 &&
         p.pt >= 0 && p.pl >= 0 && p.oh > 0 && p.ow > 0 &&
         (long)(p.oh - 1) * p.s - p.pt + p.k - 1 >= 0 && (p.oh - 1) * p.s - p.pt < p.h + p.k &&
         (p.ow - 1) * p.s - p.pl < p.w + p.k;
}

}  // namespace pld

using namespace pld;

extern "C" int pld_maxpool2d_fwd(const float* x, int n, int h, int w, int c, int k, int s,
                                 int pad_t, int pad_l, int oh, int ow, float* y,
                                 uint8_t* argmax, void* stream) {
  PoolParams p{n, h, w, c, k, s, pad_t, pad_l, oh, ow};
  PLD_CHECK_ARG(x && y && pool_ok(p), "pld_maxpool2d_fwd: bad args");
  const bool v4 = c % 4 == 0 && aligned16(x) && aligned16(y) && (!argmax || aligned16(argmax));
  const long total = (long)n * oh * ow * (v4 ? c / 4 : c);
  const unsigned g = std::min<unsigned>(std::max(cdiv(total, 256), 1u), 16384);
  if (v4) maxpool_fwd_kernel<4><<<g, 256, 0, as_stream(stream)>>>(x, p, y, argmax);
  else maxpool_fwd_kernel<1><<<g, 256, 0, as_stream(stream)>>>(x, p, y, argmax);
  return check_launch("maxpool_fwd_kernel");
}

extern "C" int pld_maxpool2d_bwd(const float* dy, const uint8_t* argmax, int n, int h, int w,
                                 int c, int k, int s, int pad_t, int pad_l, int oh, int ow,
                                 float* dx, int accumulate, void* stream) {
  PoolParams p{n, h, w, c, k, s, pad_t, pad_l, oh, ow};
  PLD_CHECK_ARG(dy && argmax && dx && pool_ok(p), "pld_maxpool2d_bwd: bad args");
  const bool v4 = c % 4 == 0 && aligned16(dy) && aligned16(dx);
  const long quads = (long)n * h * w * (c / 4);
  if (v4 && ((uintptr_t)argmax & 3) == 0 && quads < (1L << 31) - (1L << 24)) {
    const unsigned g = std::min<unsigned>(std::max(cdiv(quads, 256), 1u), 16384);
    maxpool_bwd4_kernel<<<g, 256, 0, as_stream(stream)>>>(
        dy, argmax, p, FastDiv((uint32_t)(c / 4)), FastDiv((uint32_t)w), FastDiv((uint32_t)h),
        (int)quads, dx, accumulate);
    return check_launch("maxpool_bwd4_kernel");
  }
  const long total = (long)n * h * w * (v4 ? c / 4 : c);
  const unsigned g = std::min<unsigned>(std::max(cdiv(total, 256), 1u), 16384);
  if (v4) maxpool_bwd_kernel<4><<<g, 256, 0, as_stream(stream)>>>(dy, argmax, p, dx, accumulate);
  else maxpool_bwd_kernel<1><<<g, 256, 0, as_stream(stream)>>>(dy, argmax, p, dx, accumulate);
  return check_launch("maxpool_bwd_kernel");
}

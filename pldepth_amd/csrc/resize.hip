// Image resizing of the HR-WSI data-access path:
// pldepth/data/dao/hr_wsi.py:65-74 resizes decoded images and depth maps with
// tf.image.resize(..., BILINEAR) and validity masks with NEAREST_NEIGHBOR. TF2 semantics
// (antialias off, half-pixel centres):
//   bilinear: src = (dst + 0.5) * in/out - 0.5; y0 = max(floor(src), 0), y1 = min(ceil(src),
//             in - 1), weight = src - floor(src); rows then columns, fp32
//   nearest : src = min(floor((dst + 0.5) * in/out), in - 1)
// NHWC float32, one thread per output element (channel fastest): HBM-bound gathers.
#include <algorithm>

#include "common.h"

// the interpolation must round after every operation like TF's CPU kernel: no FMA contraction
// (HIP compiles with -ffp-contract=fast by default)
#pragma clang fp contract(off)

namespace pld {

struct ResizeGeom {
  int n, h, w, c, oh, ow;
  float sy, sx;  // in / out
};

__global__ __launch_bounds__(256) void resize_bilinear_kernel(const float* __restrict__ x,
                                                              ResizeGeom g,
                                                              float* __restrict__ y) {
  const long total = (long)g.n * g.oh * g.ow * g.c;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % g.c);
    long t = e / g.c;
    const int ox = (int)(t % g.ow);
    t /= g.ow;
    const int oy = (int)(t % g.oh);
    const int img = (int)(t / g.oh);
    // un-fused fp32 multiply then add/subtract, as TF's CPU kernel computes
    const float fy = ((float)oy + 0.5f) * g.sy - 0.5f;
    const float fx = ((float)ox + 0.5f) * g.sx - 0.5f;
    const float fly = floorf(fy), flx = floorf(fx);
    const int y0 = max((int)fly, 0), y1 = min((int)ceilf(fy), g.h - 1);
    const int x0 = max((int)flx, 0), x1 = min((int)ceilf(fx), g.w - 1);
    const float ly = fy - fly, lx = fx - flx;
    const float* b = x + (long)img * g.h * g.w * g.c + ch;
    const float tl = b[((long)y0 * g.w + x0) * g.c], tr = b[((long)y0 * g.w + x1) * g.c];
    const float bl = b[((long)y1 * g.w + x0) * g.c], br = b[((long)y1 * g.w + x1) * g.c];
    const float top = tl + (tr - tl) * lx;
    const float bot = bl + (br - bl) * lx;
    y[e] = top + (bot - top) * ly;
  }
}

__global__ __launch_bounds__(256) void resize_nearest_kernel(const float* __restrict__ x,
                                                             ResizeGeom g,
                                                             float* __restrict__ y) {
  const long total = (long)g.n * g.oh * g.ow * g.c;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % g.c);
    long t = e / g.c;
    const int ox = (int)(t % g.ow);
    t /= g.ow;
    const int oy = (int)(t % g.oh);
    const int img = (int)(t / g.oh);
    const int iy = min((int)floorf(((float)oy + 0.5f) * g.sy), g.h - 1);
    const int ix = min((int)floorf(((float)ox + 0.5f) * g.sx), g.w - 1);
    y[e] = x[(((long)img * g.h + iy) * g.w + ix) * g.c + ch];
  }
}

}  // namespace pld

using namespace pld;

static int resize_impl(const float* x, int n, int h, int w, int c, int oh, int ow, float* y,
                       bool bilinear, void* stream) {
  PLD_CHECK_ARG(x && y && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0,
                "pld_resize: bad args");
  ResizeGeom g{n, h, w, c, oh, ow, (float)h / (float)oh, (float)w / (float)ow};
  const long total = (long)n * oh * ow * c;
  const unsigned grid = std::min<unsigned>(cdiv(total, 256), 16384);
  if (bilinear) resize_bilinear_kernel<<<grid, 256, 0, as_stream(stream)>>>(x, g, y);
  else resize_nearest_kernel<<<grid, 256, 0, as_stream(stream)>>>(x, g, y);
  return check_launch(bilinear ? "resize_bilinear_kernel" : "resize_nearest_kernel");
}

extern "C" int pld_resize_bilinear(const float* x, int n, int h, int w, int c, int oh, int ow,
                                   float* y, void* stream) {
  return resize_impl(x, n, h, w, c, oh, ow, y, true, stream);
}

extern "C" int pld_resize_nearest(const float* x, int n, int h, int w, int c, int oh, int ow,
                                  float* y, void* stream) {
  return resize_impl(x, n, h, w, c, oh, ow, y, false, stream);
}

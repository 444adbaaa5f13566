// The EfficientNetB0 stem convolution as a direct kernel: Rescaling + Normalization (the input
// prologue x*scale + shift, in-image taps only) -> ZeroPadding2D(correct_pad) -> Conv2D(32, 3x3,
// stride 2, valid, no bias) of the [0, 1] RGB input (Keras EfficientNetB0 stem, reached through
// pl_hourglass.py:48), with the batch statistics of its output for the stem BatchNormalization in
// the epilogue.
//
// 3 input channels make the im2col GEMM K = 27: an MFMA tile pads it to 32 and re-reads the map
// per tap (conv_igemm_kernel: 0.22 ms at 448^2 x 32, 1.3 TB/s). Here a 256-thread workgroup owns
// an 8 x 32 output tile: it stages the 17 x 65 x 3 input window once (coalesced rows, prologue
// applied, padding zeros; all loads of a thread in flight together: a rolled loop waiting out
// each load's latency ran 164 us), each thread holds one output pixel's 27 taps in registers and
// forms its 32 channels with the filter as scalar (SGPR) operands, one channel's 27 contiguous
// weights at a time, accumulating in fp64 with one rounding per output, and the [256][32] tile
// leaves through LDS as contiguous 4 KB row runs.
// Algorithmic bytes: the input once + the output once (77 + 205 MB at 448^2 x 32).
#include <algorithm>

#include "common.h"
#include "conv_common.h"

namespace pld {
namespace stem {

constexpr int TH = 8, TW = 32, CO = 32, KS = 3, CI = 3, S = 2;
constexpr int IH = (TH - 1) * S + KS, IW = (TW - 1) * S + KS;  // 17 x 65 input window
constexpr int OL = CO + 4;                                       // output tile row pitch

struct Params {
  const float* x;
  const float* w;  // native [CO][KS][KS][CI]
  const float* bias;
  const float* scale;  // prologue (NULL = identity)
  const float* shift;
  int act;
  float* y;
  int n, ih, iw, oh, ow, pt, pl, acc;
  int tiles_x, tiles_y;
  double* stats;  // [CO][gridDim.x][2] or NULL
};

__global__ __launch_bounds__(256) void stem3x3_kernel(Params p) {
  // the input window, then (once every thread holds its taps' products) the output tile
  __shared__ __attribute__((aligned(16))) float lds[TH * TW * OL];
  static_assert(IH * IW * CI <= TH * TW * OL, "window fits the tile buffer");
  __shared__ double red[8][CO][2];
  float* xin = lds;
  float* so = lds;
  const int tid = threadIdx.x;
  const int tx0 = (int)(blockIdx.x % p.tiles_x) * TW;
  const int rest = (int)(blockIdx.x / p.tiles_x);
  const int ty0 = (rest % p.tiles_y) * TH;
  const int img = rest / p.tiles_y;
  const int iy0 = ty0 * S - p.pt, ix0 = tx0 * S - p.pl;
  const float* xb = p.x + (long)img * p.ih * p.iw * CI;
  float sc[CI], sh[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) {
    sc[c] = p.scale ? p.scale[c] : 1.f;
    sh[c] = p.scale ? p.shift[c] : 0.f;
  }
  // stage the input window: row r holds IW pixels x 3 channels = 195 contiguous floats of x. All
  // 13 loads of a thread are issued before the first LDS write (a rolled loop waits out each
  // load's latency in turn)
  constexpr int NE = IH * IW * CI, IT = (NE + 255) / 256;
  float v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = tid + 256 * i;
    const int r = e / (IW * CI), q = e - r * (IW * CI);
    const int iy = iy0 + r, ix = ix0 + q / CI;
    v[i] = (e < NE && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw)
               ? xb[((long)iy * p.iw + ix) * CI + (q - (q / CI) * CI)]
               : 0.f;
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = tid + 256 * i;
    if (e >= NE) continue;
    const int r = e / (IW * CI), q = e - r * (IW * CI);
    const int iy = iy0 + r, ix = ix0 + q / CI, c = q - (q / CI) * CI;
    float u = v[i];
    if (p.scale && (unsigned)iy < (unsigned)p.ih && (unsigned)ix < (unsigned)p.iw)
      // in-image taps only: padding stays zero (selects, not a dynamic index: no scratch array)
      u = act_fwd(p.act, u * (c == 0 ? sc[0] : c == 1 ? sc[1] : sc[2]) +
                             (c == 0 ? sh[0] : c == 1 ? sh[1] : sh[2]));
    xin[e] = u;
  }
  __syncthreads();
  const int ly = tid / TW, lx = tid - ly * TW;
  // the pixel's 27 taps in registers, then one output channel at a time: channel co's 27
  // weights are contiguous in the native filter, so they arrive as wide scalar loads
  float xv[KS * KS * CI];
#pragma unroll
  for (int ty = 0; ty < KS; ++ty)
#pragma unroll
    for (int tx = 0; tx < KS; ++tx)
#pragma unroll
      for (int ci = 0; ci < CI; ++ci)
        xv[(ty * KS + tx) * CI + ci] = xin[((ly * S + ty) * IW + lx * S + tx) * CI + ci];
  // fp64 accumulation, one rounding to fp32 per output: the stem's output is then within half
  // an ulp of the exact sum, whatever order an fp32 chain would take (the 64^2 batch-2 parity
  // test amplifies the stem's rounding through a training-mode BN over 8 values per channel at
  // top_activation). The 864 fp64 FMAs per pixel stay hidden under the kernel's HBM time.
  float acc[CO];
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    double a = 0.0;
#pragma unroll
    for (int t = 0; t < KS * KS * CI; ++t)
      a = fma((double)xv[t], (double)p.w[co * KS * KS * CI + t], a);
    acc[co] = (float)a;
  }
  __syncthreads();  // the window is dead: the output tile takes its space
#pragma unroll
  for (int co = 0; co < CO; co += 4) {
    float4 v = make_float4(acc[co], acc[co + 1], acc[co + 2], acc[co + 3]);
    if (p.bias) {
      v.x += p.bias[co];
      v.y += p.bias[co + 1];
      v.z += p.bias[co + 2];
      v.w += p.bias[co + 3];
    }
    *reinterpret_cast<float4*>(so + tid * OL + co) = v;
  }
  __syncthreads();
  const int rows_ok = min(TH, p.oh - ty0), cols_ok = min(TW, p.ow - tx0);
  if (p.stats) {
    // thread (g, c): channel c over the 32 pixels of tile row g, fp64, pixels in order; then the
    // 8 row sums in order (deterministic)
    const int c = tid & (CO - 1), g = tid >> 5;
    double s1 = 0.0, s2 = 0.0;
    if (g < rows_ok)
      for (int j = 0; j < cols_ok; ++j) {
        const double v = (double)so[(g * TW + j) * OL + c];
        s1 += v;
        s2 += v * v;
      }
    red[g][c][0] = s1;
    red[g][c][1] = s2;
    __syncthreads();
    if (tid < CO) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        a += red[r][tid][0];
        b += red[r][tid][1];
      }
      *reinterpret_cast<double2*>(p.stats + ((long)tid * gridDim.x + blockIdx.x) * 2) =
          make_double2(a, b);
    }
  }
  // each tile row is one contiguous run of cols_ok x 32 floats of y: float4 stores
  float* yb = p.y + (((long)img * p.oh + ty0) * p.ow + tx0) * CO;
  for (int e = tid; e < TH * TW * CO / 4; e += 256) {
    const int r = e / (TW * CO / 4), q = e - r * (TW * CO / 4);
    const int px = q / (CO / 4), c4 = q - px * (CO / 4);
    if (r >= rows_ok || px >= cols_ok) continue;
    float4 v = *reinterpret_cast<const float4*>(so + (r * TW + px) * OL + 4 * c4);
    float4* d = reinterpret_cast<float4*>(yb + ((long)r * p.ow + px) * CO + 4 * c4);
    if (p.acc) v = add4(v, *d);
    *d = v;
  }
}

}  // namespace stem
}  // namespace pld

using namespace pld;

// the geometry the direct stem kernel takes: 3x3 stride 2, 3 -> 32 channels, one source
extern "C" int pld__stem3x3_eligible(const pld_conv_args* a) {
  return a && a->kh == 3 && a->kw == 3 && a->sh == 2 && a->sw == 2 && a->c1 == 3 && a->c2 == 0 &&
         a->cout == 32 && a->pad_t >= 0 && a->pad_t <= 2 && a->pad_l >= 0 && a->pad_l <= 2 &&
         a->oh > 0 && a->ow > 0 && a->n > 0 && a->h > 0 && a->w > 0;
}

extern "C" int pld__stem3x3_parts(const pld_conv_args* a) {
  return (int)(cdiv(a->ow, stem::TW) * cdiv(a->oh, stem::TH) * a->n);
}

extern "C" int pld__stem3x3_fwd(const pld_conv_args* a, const float* w_nat, const float* bias,
                                float* y, int accumulate, double* stats, void* stream) {
  PLD_CHECK_ARG(pld__stem3x3_eligible(a) && w_nat && y && aligned16(y),
                "stem3x3: bad args (3x3 stride 2, 3 -> 32 channels, 16-byte aligned output)");
  PLD_CHECK_ARG(!(stats && accumulate), "stem3x3: statistics of an accumulated output");
  stem::Params p;
  p.x = a->x1;
  p.w = w_nat;
  p.bias = bias;
  p.scale = a->in_scale;
  p.shift = a->in_shift;
  p.act = a->in_act;
  p.y = y;
  p.n = a->n;
  p.ih = a->h;
  p.iw = a->w;
  p.oh = a->oh;
  p.ow = a->ow;
  p.pt = a->pad_t;
  p.pl = a->pad_l;
  p.acc = accumulate;
  p.tiles_x = (int)cdiv(a->ow, stem::TW);
  p.tiles_y = (int)cdiv(a->oh, stem::TH);
  p.stats = stats;
  stem::stem3x3_kernel<<<pld__stem3x3_parts(a), 256, 0, as_stream(stream)>>>(p);
  return check_launch("stem3x3_kernel");
}

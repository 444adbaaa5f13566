// 3x3 'same' convolutions with ONE output channel (the ff_effnet decoder's final Conv2D(1, 3x3),
// pldepth/models/pl_hourglass.py:96; ReDWeb's AdaptiveOutputLayer conv1, redweb.py:322) as
// direct, LDS-tiled, HBM-bound kernels.
//
// An implicit GEMM with N = 1 wastes 31/32 of every 32x32 MFMA tile; the layer's arithmetic
// (288 MACs per output pixel) is far below the HBM roofline, so each kernel instead streams its
// big operand once: a 16x16 output tile stages its 18x18 input halo (all channels, chunked by 32)
// in LDS, padded to a 36-float channel stride so 16 consecutive pixels' float4 reads hit 16
// distinct LDS slots.
//   fwd   : y[n][oy][ox] = b + sum_{ty,tx,c} x[n][oy+ty-pt][ox+tx-pl][c] * w[ty][tx][c]
//   dgrad : dx[n][iy][ix][c] = sum_{ty,tx} dy[n][iy-ty+pt][ix-tx+pl] * w[ty][tx][c]
//   wgrad : dw[ty][tx][c] = sum_{n,oy,ox} x[n][oy+ty-pt][ox+tx-pl][c] * dy[n][oy][ox]
//           (per-workgroup partials over a strided set of tiles, ordered reduction)
// Algorithmic bytes: fwd/wgrad read x once (+ dy), dgrad writes dx once.
#include <algorithm>

#include "conv_common.h"

namespace pld {

constexpr int ST = 16;        // output tile edge
constexpr int HT = ST + 2;    // halo edge (3x3)
constexpr int CH = 32;        // channels per LDS chunk
constexpr int CS = CH + 4;    // padded channel stride

struct SkinnyParams {
  const float* x;   // [n][h][w][c]
  const float* dy;  // [n][h][w]
  const float* wt;  // fwd: [3][3][c] (tap-major, = HWIO with cout 1); dgrad: [c][3][3] flipped
  const float* bias;
  float* y;         // fwd: [n][h][w]; dgrad: [n][h][w][c]
  float* part;      // wgrad partials [gridDim.x][9*c]
  int n, h, w, c, pt, pl, acc;
  int tiles_x, tiles_y;
};

constexpr int MAX_C = 2 * CH;  // eligibility bound (ReDWeb's aol/conv1 has 64 input channels)
constexpr int NT = 256;        // workgroup size of the halo kernels

// One 32-channel chunk of a tile's 18x18 input halo in flight in registers: every load issued
// at once through a buffer descriptor (zeros outside the image and past the last channel) — no
// branch around a load — so the next tile's halo streams in while the current one is computed.
// halo[(hy*HT + hx)*CS + cc] = x[img][y0+hy-pt][x0+hx-pl][c0+cc]
struct HaloRegs {
  static constexpr int NQ = CH / 4, TOTAL = HT * HT * NQ, IT = (TOTAL + NT - 1) / NT;
  float4 v[IT];
  float dy;  // wgrad: this thread's dy pixel of the tile
};

__device__ __forceinline__ void tile_origin(const SkinnyParams& p, int tile, int& img, int& y0,
                                            int& x0) {
  img = tile / (p.tiles_x * p.tiles_y);
  const int r = tile - img * p.tiles_x * p.tiles_y;
  y0 = (r / p.tiles_x) * ST;
  x0 = (r % p.tiles_x) * ST;
}

__device__ __forceinline__ void halo_load(const SkinnyParams& p, HaloRegs& h, int tile, int c0,
                                          bool with_dy) {
  int img, y0, x0;
  tile_origin(p, tile, img, y0, x0);
  const int nc = min(CH, p.c - c0);
  const int img_elems = p.h * p.w * p.c;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.x + (long)img * img_elems, (long)img_elems * 4);
#pragma unroll
  for (int i = 0; i < HaloRegs::IT; ++i) {
    const int e = threadIdx.x + NT * i;
    const int q = e % HaloRegs::NQ, pix = e / HaloRegs::NQ;
    const int hy = pix / HT, hx = pix % HT;
    const int iy = y0 + hy - p.pt, ix = x0 + hx - p.pl;
    const bool ok = e < HaloRegs::TOTAL && 4 * q < nc && (unsigned)iy < (unsigned)p.h &&
                    (unsigned)ix < (unsigned)p.w;
    h.v[i] = bload4(rs, ok ? (unsigned)(((iy * p.w + ix) * p.c + c0 + 4 * q) * 4) : OOB);
  }
  if (with_dy) {
    const int hw = p.h * p.w;
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(p.dy + (long)img * hw, (long)hw * 4);
    const int oy = y0 + threadIdx.x / ST, ox = x0 + threadIdx.x % ST;
    h.dy = bload1(rd, (oy < p.h && ox < p.w) ? (unsigned)((oy * p.w + ox) * 4) : OOB);
  }
}

__device__ __forceinline__ void halo_store(const HaloRegs& h, float* halo) {
#pragma unroll
  for (int i = 0; i < HaloRegs::IT; ++i) {
    const int e = threadIdx.x + NT * i;
    if (e < HaloRegs::TOTAL)
      *reinterpret_cast<float4*>(halo + (e / HaloRegs::NQ) * CS + 4 * (e % HaloRegs::NQ)) = h.v[i];
  }
}

// persistent workgroups over the tiles; the halo chunk of the next (tile, chunk) stage is loaded
// before the current one is computed (the index is clamped at the end: a harmless re-load)
template <int NCH>
__global__ __launch_bounds__(NT) void skinny_fwd_kernel(SkinnyParams p) {
  __shared__ __attribute__((aligned(16))) float halo[HT * HT * CS];
  __shared__ __attribute__((aligned(16))) float wl[9 * MAX_C];
  const int tx = threadIdx.x % ST, ty = threadIdx.x / ST;
  const int ntiles = p.tiles_x * p.tiles_y * p.n;
  for (int e = threadIdx.x; e < 9 * p.c; e += NT) wl[(e / p.c) * MAX_C + e % p.c] = p.wt[e];
  HaloRegs hr;
  halo_load(p, hr, min((int)blockIdx.x, ntiles - 1), 0, false);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      __syncthreads();
      halo_store(hr, halo);
      __syncthreads();
      if (k + 1 < NCH) halo_load(p, hr, tile, (k + 1) * CH, false);
      else halo_load(p, hr, min(tile + (int)gridDim.x, ntiles - 1), 0, false);
      const int nc = min(CH, p.c - k * CH);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float* hp = halo + ((ty + t / 3) * HT + tx + t % 3) * CS;
        const float* wp = wl + t * MAX_C + k * CH;
        for (int q = 0; q < nc; q += 4) {
          const float4 v = *reinterpret_cast<const float4*>(hp + q);
          const float4 f = *reinterpret_cast<const float4*>(wp + q);
          acc += v.x * f.x + v.y * f.y + v.z * f.z + v.w * f.w;
        }
      }
    }
    int img, y0, x0;
    tile_origin(p, tile, img, y0, x0);
    const int oy = y0 + ty, ox = x0 + tx;
    if (oy < p.h && ox < p.w) {
      float* d = p.y + ((long)img * p.h + oy) * p.w + ox;
      const float v = acc + (p.bias ? p.bias[0] : 0.f);
      *d = p.acc ? *d + v : v;
    }
  }
}

__global__ __launch_bounds__(256) void skinny_dgrad_kernel(SkinnyParams p) {
  __shared__ float dyl[HT * HT];
  __shared__ __attribute__((aligned(16))) float wl[9 * 64];
  const int tx = threadIdx.x % ST, ty = threadIdx.x / ST;
  const int x0 = blockIdx.x * ST, y0 = blockIdx.y * ST, img = blockIdx.z;
  // dy halo: dyl[hy][hx] = dy[img][y0+hy-(2-pt)][x0+hx-(2-pl)]
  const int qt = 2 - p.pt, ql = 2 - p.pl;
  for (int e = threadIdx.x; e < HT * HT; e += blockDim.x) {
    const int iy = y0 + e / HT - qt, ix = x0 + e % HT - ql;
    dyl[e] = (iy >= 0 && iy < p.h && ix >= 0 && ix < p.w)
                 ? p.dy[((long)img * p.h + iy) * p.w + ix] : 0.f;
  }
  (void)tx;
  (void)ty;
  for (int c0 = 0; c0 < p.c; c0 += 64) {
    const int nc = min(64, p.c - c0);
    const int nq = nc / 4;
    __syncthreads();
    // p.w is the dgrad-native filter [c][3][3] with flipped taps: W[t][c] = Wd[c][8 - t]
    for (int e = threadIdx.x; e < 9 * nc; e += blockDim.x)
      wl[(e / nc) * 64 + e % nc] = p.wt[(long)(c0 + e % nc) * 9 + (8 - e / nc)];
    __syncthreads();
    // one (pixel, 4-channel quad) per thread and pass: neighbouring lanes write neighbouring
    // 16-byte quads of one pixel, then of the next pixel (full-line stores of the dx rows)
    for (int e = threadIdx.x; e < ST * ST * nq; e += blockDim.x) {
      const int q = e % nq, pix = e / nq;
      const int py = pix / ST, px = pix % ST;
      const int iy = y0 + py, ix = x0 + px;
      if (iy >= p.h || ix >= p.w) continue;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        // output (iy - ty + pt) contributes through tap ty: halo row iy-ty+pt-(y0-qt)
        const float g = dyl[(py + 2 - t / 3) * HT + px + 2 - t % 3];
        const float4 f = *reinterpret_cast<const float4*>(wl + t * 64 + 4 * q);
        a.x += g * f.x; a.y += g * f.y; a.z += g * f.z; a.w += g * f.w;
      }
      float4* dp = reinterpret_cast<float4*>(p.y + (((long)img * p.h + iy) * p.w + ix) * p.c +
                                             c0 + 4 * q);
      if (p.acc) {
        const float4 o = *dp;
        a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
      }
      *dp = a;
    }
  }
}

// 256 threads = 8 channel quads x 32 pixel groups of 8 pixels: per pixel a thread reads dy once
// and the 9 tap quads of its halo column, 4 FMAs per 16-byte LDS read; persistent workgroups
// over a strided set of tiles with the next halo chunk in flight during the current one's
// compute. Groups are combined by a fixed shuffle tree inside each wave, then across the 4 waves
// in LDS (deterministic).
template <int NCH>
__global__ __launch_bounds__(NT) void skinny_wgrad_kernel(SkinnyParams p) {
  __shared__ __attribute__((aligned(16))) float halo[HT * HT * CS];
  __shared__ float dyl[ST * ST];
  __shared__ __attribute__((aligned(16))) float comb[4][9 * MAX_C];
  const int ntiles = p.tiles_x * p.tiles_y * p.n;
  const int q = threadIdx.x & 7, pg = threadIdx.x >> 3;
  float4 acc[NCH][9];
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[k][t] = make_float4(0.f, 0.f, 0.f, 0.f);
  HaloRegs hr;
  halo_load(p, hr, min((int)blockIdx.x, ntiles - 1), 0, true);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      __syncthreads();
      halo_store(hr, halo);
      if (k == 0) dyl[threadIdx.x] = hr.dy;
      __syncthreads();
      if (k + 1 < NCH) halo_load(p, hr, tile, (k + 1) * CH, false);
      else halo_load(p, hr, min(tile + (int)gridDim.x, ntiles - 1), 0, true);
      if (4 * q < min(CH, p.c - k * CH)) {
#pragma unroll 2
        for (int i = 0; i < 8; ++i) {
          const int pix = pg * 8 + i, py = pix / ST, px = pix % ST;
          const float g = dyl[pix];
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const float4 v = *reinterpret_cast<const float4*>(
                halo + ((py + t / 3) * HT + px + t % 3) * CS + 4 * q);
            acc[k][t].x += v.x * g;
            acc[k][t].y += v.y * g;
            acc[k][t].z += v.z * g;
            acc[k][t].w += v.w * g;
          }
        }
      }
    }
  }
  // reduce the 8 pixel groups of each wave (lane bits 3..5), then the 4 waves
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        acc[k][t].x += __shfl_xor(acc[k][t].x, o);
        acc[k][t].y += __shfl_xor(acc[k][t].y, o);
        acc[k][t].z += __shfl_xor(acc[k][t].z, o);
        acc[k][t].w += __shfl_xor(acc[k][t].w, o);
      }
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    if (lane < 8 && 4 * lane < min(CH, p.c - k * CH)) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
        *reinterpret_cast<float4*>(&comb[wave][t * MAX_C + k * CH + 4 * lane]) = acc[k][t];
    }
  }
  __syncthreads();
  // partial index = tap * c + channel (HWIO with cout 1)
  for (int e = threadIdx.x; e < 9 * p.c; e += NT) {
    const int t = e / p.c, c = e - t * p.c;
    const int o = t * MAX_C + c;
    p.part[(long)blockIdx.x * 9 * p.c + e] = ((comb[0][o] + comb[1][o]) + comb[2][o]) + comb[3][o];
  }
}

// one workgroup per output: strided partial sums then a fixed-shape tree (deterministic)
__global__ __launch_bounds__(256) void skinny_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                  int nb, int per,
                                                                  float* __restrict__ dw,
                                                                  int acc) {
  __shared__ double red[256];
  const int e = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[(long)b * per + e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dw[e] = acc ? dw[e] + (float)red[0] : (float)red[0];
}

constexpr int SKINNY_WG_BLOCKS = 2048;
constexpr int SKINNY_FWD_BLOCKS = 2048;  // persistent: ~3 per CU, each over a strided tile set

// ---- 1x1 conv with one input and one output channel (ReDWeb's final aol/conv2, redweb.py: a
// scalar affine map of the 448^2 prediction): y = w x + b, dx = w dy, dw = sum x dy. Pure HBM
// streams — as an implicit GEMM with K = N = 1 it ran at 0.4 ms fwd / dgrad and 1.3 ms wgrad.
constexpr int SCALAR_BLOCKS = 1024;

__global__ __launch_bounds__(256) void scalar1x1_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ y, long n, int acc) {
  const float wv = w[0], bv = bias ? bias[0] : 0.f;
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    float4 o = make_float4(wv * v.x + bv, wv * v.y + bv, wv * v.z + bv, wv * v.w + bv);
    if (acc) {
      const float4 d = reinterpret_cast<const float4*>(y)[i];
      o = make_float4(d.x + o.x, d.y + o.y, d.z + o.z, d.w + o.w);
    }
    reinterpret_cast<float4*>(y)[i] = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long i = 4 * n4 + threadIdx.x;
    const float o = wv * x[i] + bv;
    y[i] = acc ? y[i] + o : o;
  }
}

// fp64 partial dot products, one per block (fixed grid-stride order), then one ordered sum
__global__ __launch_bounds__(256) void scalar1x1_wgrad_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ dy,
                                                              long n, double* __restrict__ part) {
  __shared__ double red[4];
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  double s = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(x)[i];
    const float4 b = reinterpret_cast<const float4*>(dy)[i];
    s += (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z + (double)a.w * b.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long i = 4 * n4 + threadIdx.x;
    s += (double)x[i] * dy[i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void scalar1x1_wgrad_sum_kernel(const double* __restrict__ part,
                                                                  int nb, float* __restrict__ dw,
                                                                  int acc) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)((red[0] + red[1]) + (red[2] + red[3]));
    dw[0] = acc ? dw[0] + v : v;
  }
}

}  // namespace pld

using namespace pld;

extern "C" int pld__scalar1x1_eligible(const pld_conv_args* a) {
  return a && a->kh == 1 && a->kw == 1 && a->sh == 1 && a->sw == 1 && a->pad_t == 0 &&
         a->pad_l == 0 && a->c1 == 1 && a->c2 == 0 && a->cout == 1 && a->in_scale == nullptr &&
         a->oh == a->h && a->ow == a->w;
}

static unsigned scalar_grid(long n) {
  return (unsigned)std::max<long>(1, std::min<long>(SCALAR_BLOCKS, ((n >> 2) + 255) / 256));
}

// fwd: (x, w, b) -> y; dgrad: (dy, w, NULL) -> dx (the 1x1 1->1 filter is its own transpose)
extern "C" int pld__scalar1x1_apply(const float* x, const float* w, const float* bias, float* y,
                                    long n, int accumulate, void* stream) {
  PLD_CHECK_ARG(x && w && y && aligned16(x) && aligned16(y), "scalar 1x1 conv: bad args");
  scalar1x1_kernel<<<scalar_grid(n), 256, 0, as_stream(stream)>>>(x, w, bias, y, n, accumulate);
  return check_launch("scalar1x1_kernel");
}

extern "C" size_t pld__scalar1x1_wgrad_ws(void) { return sizeof(double) * SCALAR_BLOCKS; }

extern "C" int pld__scalar1x1_wgrad(const float* x, const float* dy, float* dw, long n,
                                    int accumulate, void* ws, void* stream) {
  PLD_CHECK_ARG(x && dy && dw && ws && aligned16(x) && aligned16(dy),
                "scalar 1x1 wgrad: bad args");
  const unsigned nb = scalar_grid(n);
  hipStream_t st = as_stream(stream);
  scalar1x1_wgrad_kernel<<<nb, 256, 0, st>>>(x, dy, n, (double*)ws);
  int rc = check_launch("scalar1x1_wgrad_kernel");
  if (rc) return rc;
  scalar1x1_wgrad_sum_kernel<<<1, 256, 0, st>>>((const double*)ws, (int)nb, dw, accumulate);
  return check_launch("scalar1x1_wgrad_sum_kernel");
}

// eligibility: 3x3 stride-1 'same', single source, no prologue, cout 1, c % 4 == 0, c <= 64
extern "C" int pld__skinny_eligible(const pld_conv_args* a) {
  return a && a->cout == 1 && a->kh == 3 && a->kw == 3 && a->sh == 1 && a->sw == 1 &&
         a->c2 == 0 && a->in_scale == nullptr && a->c1 % 4 == 0 && a->c1 <= MAX_C &&
         a->oh == a->h && a->ow == a->w && a->pad_t >= 0 && a->pad_t <= 2 && a->pad_l >= 0 &&
         a->pad_l <= 2;
}

static SkinnyParams mk(const pld_conv_args* a) {
  SkinnyParams p{};
  p.x = a->x1;
  p.n = a->n; p.h = a->h; p.w = a->w; p.c = a->c1;
  p.pt = a->pad_t; p.pl = a->pad_l;
  p.tiles_x = (int)cdiv(a->w, ST);
  p.tiles_y = (int)cdiv(a->h, ST);
  return p;
}

extern "C" int pld__skinny_fwd(const pld_conv_args* a, const float* w_ohwi, const float* bias,
                               float* y, int accumulate, void* stream) {
  SkinnyParams p = mk(a);
  p.wt = w_ohwi;  // [1][3][3][c] == [tap][c]
  p.bias = bias;
  p.y = y;
  p.acc = accumulate;
  const int ntiles = p.tiles_x * p.tiles_y * p.n;
  const int nb = std::min(SKINNY_FWD_BLOCKS, ntiles);
  if (p.c > CH) skinny_fwd_kernel<2><<<nb, NT, 0, as_stream(stream)>>>(p);
  else skinny_fwd_kernel<1><<<nb, NT, 0, as_stream(stream)>>>(p);
  return check_launch("skinny_fwd_kernel");
}

extern "C" int pld__skinny_dgrad(const pld_conv_args* a, const float* dy, const float* w_dgrad,
                                 float* dx, int accumulate, void* stream) {
  SkinnyParams p = mk(a);
  p.dy = dy;
  p.wt = w_dgrad;
  p.y = dx;
  p.acc = accumulate;
  dim3 grid(p.tiles_x, p.tiles_y, p.n);
  skinny_dgrad_kernel<<<grid, 256, 0, as_stream(stream)>>>(p);
  return check_launch("skinny_dgrad_kernel");
}

extern "C" size_t pld__skinny_wgrad_ws(const pld_conv_args* a) {
  return sizeof(float) * (size_t)SKINNY_WG_BLOCKS * 9 * a->c1;
}

extern "C" int pld__skinny_wgrad(const pld_conv_args* a, const float* dy, float* dw,
                                 int accumulate, void* ws, void* stream) {
  SkinnyParams p = mk(a);
  p.dy = dy;
  p.part = (float*)ws;
  const int ntiles = p.tiles_x * p.tiles_y * p.n;
  const int nb = std::min(SKINNY_WG_BLOCKS, ntiles);
  hipStream_t st = as_stream(stream);
  if (p.c > CH) skinny_wgrad_kernel<2><<<nb, NT, 0, st>>>(p);
  else skinny_wgrad_kernel<1><<<nb, NT, 0, st>>>(p);
  int rc = check_launch("skinny_wgrad_kernel");
  if (rc) return rc;
  const int per = 9 * p.c;
  skinny_wgrad_reduce_kernel<<<per, 256, 0, st>>>(p.part, nb, per, dw, accumulate);
  return check_launch("skinny_wgrad_reduce_kernel");
}

// The ff_effnet decoder's last stage fused: BN + ReLU -> UpSampling2D(bilinear) x2 ->
// Conv2D(1, 3x3, 'same') + bias (pldepth/models/pl_hourglass.py:92-96), forward, filter gradient
// and the input gradient taken back through the upsampling, without materialising the 2x map.
//
// Unfused, the 448x448x32 upsampled map is written by the upsample (822 MB at batch 32), read by
// the conv forward and by its filter gradient, and its gradient is written by the conv dgrad and
// read back by the upsample's adjoint: ~4 passes over 822 MB. Here every kernel reads the
// 224x224 pre-BN map (or the 1-channel dpred) and builds the part of the 2x map it needs in LDS:
//   fwd   : y[p] = b + sum_{t,c} w[t][c] * up[p + t - 1][c],  up = bilinear2x(relu(bn(x)))
//   wgrad : dw[t][c] = sum_p up[p + t - 1][c] * dy[p]  (persistent partials + ordered reduce)
//   dgrad : dact = bilinear2x^T(dup),  dup[q][c] = sum_t w[t][c] * dy[q - t + 1]
// The 2x map is formed with the same taps and lerp arithmetic as upsample2x_fwd_cell_kernel
// (resample.hip), the BN prologue as its UpPro, so `up` is bit-identical to the unfused path's.
// Algorithmic bytes: fwd/wgrad read x (224^2 x c) once (+ dy), dgrad reads dy and writes dact.
#include <algorithm>

#include "common.h"

namespace pld {
namespace upc {

constexpr int NT = 256;
constexpr int ST = 16;           // 2x-map output tile edge (fwd / wgrad)
constexpr int UT = ST + 2;       // 2x-map halo edge (3x3)
constexpr int SR = ST / 2 + 2;   // source rows / cols feeding a UT x UT 2x-map window
constexpr int CMAX = 32;         // channels (the decoder's dec_conv4 output)
constexpr int CS = CMAX + 4;     // padded LDS channel stride
constexpr int DT = 8;            // dgrad: source (1x map) tile edge
constexpr int DU = 2 * DT + 2;   // its 2x-map window edge
constexpr int DY = DU + 2;       // the dy window edge feeding that

struct Params {
  const float* x;       // [n][h][w][c] pre-BN (dec4_pre)
  const float* mean;    // BN (training statistics) + ReLU prologue
  const float* invstd;
  const float* gamma;
  const float* beta;
  const float* wt;      // [3][3][c] (HWIO, cout 1)
  const float* bias;    // [1] or NULL
  const float* dy;      // [n][2h][2w]
  float* y;             // fwd: [n][2h][2w]; dgrad: dact [n][h][w][c]
  float* part;          // wgrad partials [gridDim.x][9 c]
  int n, h, w, c;
  int tiles_x, tiles_y;  // fwd / wgrad tiles of the 2x map
};

__device__ __forceinline__ void lerp_coords(int o, int in_size, int& lo, int& hi, float& l) {
  const float in = ((float)o + 0.5f) * 0.5f - 0.5f;
  const float f = floorf(in);
  lo = max((int)f, 0);
  hi = min((int)ceilf(in), in_size - 1);
  l = in - f;
}

// source window of a fwd / wgrad tile: rows sy0 .. sy0 + SR - 1 (clamped into the image: the
// clamped duplicates are what the bilinear taps clamp to), prologued, in registers then LDS
struct SrcRegs {
  static constexpr int NQ = CMAX / 4, TOTAL = SR * SR * NQ, IT = (TOTAL + NT - 1) / NT;
  float4 v[IT];
  float dy;
};

__device__ __forceinline__ void tile_origin(const Params& p, int tile, int& img, int& Y0,
                                            int& X0) {
  img = tile / (p.tiles_x * p.tiles_y);
  const int r = tile - img * p.tiles_x * p.tiles_y;
  Y0 = (r / p.tiles_x) * ST;
  X0 = (r % p.tiles_x) * ST;
}

__device__ __forceinline__ void src_load(const Params& p, SrcRegs& s, int tile, bool with_dy) {
  int img, Y0, X0;
  tile_origin(p, tile, img, Y0, X0);
  const int sy0 = Y0 / 2 - 1, sx0 = X0 / 2 - 1;
  const long img_elems = (long)p.h * p.w * p.c;
  const float* base = p.x + img * img_elems;
#pragma unroll
  for (int i = 0; i < SrcRegs::IT; ++i) {
    const int e = threadIdx.x + NT * i;
    const int q = e % SrcRegs::NQ, pix = e / SrcRegs::NQ;
    const int ry = min(max(sy0 + pix / SR, 0), p.h - 1);
    const int rx = min(max(sx0 + pix % SR, 0), p.w - 1);
    const bool ok = e < SrcRegs::TOTAL && 4 * q < p.c;
    s.v[i] = ok ? *reinterpret_cast<const float4*>(base + ((long)ry * p.w + rx) * p.c + 4 * q)
                : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (with_dy) {
    const int H2 = 2 * p.h, W2 = 2 * p.w;
    const int oy = Y0 + threadIdx.x / ST, ox = X0 + threadIdx.x % ST;
    s.dy = (oy < H2 && ox < W2) ? p.dy[((long)img * H2 + oy) * W2 + ox] : 0.f;
  }
}

// prologue (BN with batch statistics, then ReLU: UpPro act 1) and the LDS store of the window
__device__ __forceinline__ void src_store(const Params& p, const SrcRegs& s, float* src) {
#pragma unroll
  for (int i = 0; i < SrcRegs::IT; ++i) {
    const int e = threadIdx.x + NT * i;
    if (e >= SrcRegs::TOTAL) continue;
    const int q = e % SrcRegs::NQ, pix = e / SrcRegs::NQ;
    if (4 * q >= p.c) continue;
    const float4 mu = *reinterpret_cast<const float4*>(p.mean + 4 * q);
    const float4 is = *reinterpret_cast<const float4*>(p.invstd + 4 * q);
    const float4 ga = *reinterpret_cast<const float4*>(p.gamma + 4 * q);
    const float4 be = *reinterpret_cast<const float4*>(p.beta + 4 * q);
    float4 v = s.v[i];
    v.x = act_fwd(1, ((v.x - mu.x) * is.x) * ga.x + be.x);
    v.y = act_fwd(1, ((v.y - mu.y) * is.y) * ga.y + be.y);
    v.z = act_fwd(1, ((v.z - mu.z) * is.z) * ga.z + be.z);
    v.w = act_fwd(1, ((v.w - mu.w) * is.w) * ga.w + be.w);
    *reinterpret_cast<float4*>(src + pix * CS + 4 * q) = v;
  }
}

// the UT x UT window of the 2x map at (Y0 - 1, X0 - 1) from the source window in LDS: zeros
// outside the 2x map (the conv's 'same' padding), else upsample2x_fwd_cell_kernel's taps and
// top / bottom lerp arithmetic
__device__ __forceinline__ void build_up(const Params& p, int Y0, int X0, const float* src,
                                         float* up) {
  const int H2 = 2 * p.h, W2 = 2 * p.w, nq = p.c / 4;
  const int sy0 = Y0 / 2 - 1, sx0 = X0 / 2 - 1;
  for (int e = threadIdx.x; e < UT * UT * nq; e += NT) {
    const int q = e % nq, pix = e / nq;
    const int uy = Y0 - 1 + pix / UT, ux = X0 - 1 + pix % UT;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (uy >= 0 && uy < H2 && ux >= 0 && ux < W2) {
      int y0, y1, x0, x1;
      float yl, xl;
      lerp_coords(uy, p.h, y0, y1, yl);
      lerp_coords(ux, p.w, x0, x1, xl);
      const float* r0 = src + (y0 - sy0) * SR * CS + 4 * q;
      const float* r1 = src + (y1 - sy0) * SR * CS + 4 * q;
      const float4 tl = *reinterpret_cast<const float4*>(r0 + (x0 - sx0) * CS);
      const float4 tr = *reinterpret_cast<const float4*>(r0 + (x1 - sx0) * CS);
      const float4 bl = *reinterpret_cast<const float4*>(r1 + (x0 - sx0) * CS);
      const float4 br = *reinterpret_cast<const float4*>(r1 + (x1 - sx0) * CS);
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
    }
    *reinterpret_cast<float4*>(up + pix * CS + 4 * q) = o;
  }
}

// persistent workgroups over the 2x-map tiles; the next tile's source window is in flight while
// the current one is computed
__global__ __launch_bounds__(NT) void upconv_fwd_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) float src[SR * SR * CS];
  __shared__ __attribute__((aligned(16))) float up[UT * UT * CS];
  __shared__ __attribute__((aligned(16))) float wl[9 * CMAX];
  const int tx = threadIdx.x % ST, ty = threadIdx.x / ST;
  const int ntiles = p.tiles_x * p.tiles_y * p.n;
  for (int e = threadIdx.x; e < 9 * p.c; e += NT) wl[(e / p.c) * CMAX + e % p.c] = p.wt[e];
  SrcRegs sr;
  src_load(p, sr, min((int)blockIdx.x, ntiles - 1), false);
  const float b = p.bias ? p.bias[0] : 0.f;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int img, Y0, X0;
    tile_origin(p, tile, img, Y0, X0);
    __syncthreads();
    src_store(p, sr, src);
    __syncthreads();
    src_load(p, sr, min(tile + (int)gridDim.x, ntiles - 1), false);
    build_up(p, Y0, X0, src, up);
    __syncthreads();
    // skinny_fwd_kernel's accumulation: taps, then channel quads
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float* hp = up + ((ty + t / 3) * UT + tx + t % 3) * CS;
      const float* wp = wl + t * CMAX;
      for (int q = 0; q < p.c; q += 4) {
        const float4 v = *reinterpret_cast<const float4*>(hp + q);
        const float4 f = *reinterpret_cast<const float4*>(wp + q);
        acc += v.x * f.x + v.y * f.y + v.z * f.z + v.w * f.w;
      }
    }
    const int oy = Y0 + ty, ox = X0 + tx;
    if (oy < 2 * p.h && ox < 2 * p.w) p.y[((long)img * 2 * p.h + oy) * 2 * p.w + ox] = acc + b;
  }
}

// 256 threads = 8 channel quads x 32 pixel groups of 8 pixels (skinny_wgrad_kernel's layout)
__global__ __launch_bounds__(NT) void upconv_wgrad_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) float src[SR * SR * CS];
  __shared__ __attribute__((aligned(16))) float up[UT * UT * CS];
  __shared__ float dyl[ST * ST];
  __shared__ __attribute__((aligned(16))) float comb[4][9 * CMAX];
  const int ntiles = p.tiles_x * p.tiles_y * p.n;
  const int q = threadIdx.x & 7, pg = threadIdx.x >> 3;
  float4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  SrcRegs sr;
  src_load(p, sr, min((int)blockIdx.x, ntiles - 1), true);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int img, Y0, X0;
    tile_origin(p, tile, img, Y0, X0);
    __syncthreads();
    src_store(p, sr, src);
    dyl[threadIdx.x] = sr.dy;
    __syncthreads();
    src_load(p, sr, min(tile + (int)gridDim.x, ntiles - 1), true);
    build_up(p, Y0, X0, src, up);
    __syncthreads();
    if (4 * q < p.c) {
#pragma unroll 2
      for (int i = 0; i < 8; ++i) {
        const int pix = pg * 8 + i, py = pix / ST, px = pix % ST;
        const float g = dyl[pix];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const float4 v = *reinterpret_cast<const float4*>(
              up + ((py + t / 3) * UT + px + t % 3) * CS + 4 * q);
          acc[t].x += v.x * g;
          acc[t].y += v.y * g;
          acc[t].z += v.z * g;
          acc[t].w += v.w * g;
        }
      }
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      acc[t].x += __shfl_xor(acc[t].x, o);
      acc[t].y += __shfl_xor(acc[t].y, o);
      acc[t].z += __shfl_xor(acc[t].z, o);
      acc[t].w += __shfl_xor(acc[t].w, o);
    }
  if (lane < 8 && 4 * lane < p.c) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *reinterpret_cast<float4*>(&comb[wave][t * CMAX + 4 * lane]) = acc[t];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 9 * p.c; e += NT) {
    const int t = e / p.c, c = e - t * p.c;
    const int o = t * CMAX + c;
    p.part[(long)blockIdx.x * 9 * p.c + e] = ((comb[0][o] + comb[1][o]) + comb[2][o]) + comb[3][o];
  }
}

__global__ __launch_bounds__(256) void upconv_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                  int nb, int per,
                                                                  float* __restrict__ dw) {
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
  if (threadIdx.x == 0) dw[e] = (float)red[0];
}

// one workgroup per DT x DT source tile: the DU x DU window of the 2x-map gradient
// dup[q][c] = sum_t w[t][c] dy[q - t + 1] (zero outside the 2x map) in LDS, then each source
// pixel gathers its bilinear adjoint: the 2x rows u in 2i-1 .. 2i+2 whose lerp taps land on i,
// weight (1 - l) for the lower tap and l for the upper (both, at a clamped border).
__global__ __launch_bounds__(NT) void upconv_dgrad_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) float dup[DU * DU * CS];
  __shared__ float dyl[DY * DY];
  __shared__ __attribute__((aligned(16))) float wl[9 * CMAX];
  const int H2 = 2 * p.h, W2 = 2 * p.w, nq = p.c / 4;
  const int j0 = blockIdx.x * DT, i0 = blockIdx.y * DT, img = blockIdx.z;
  const int u0 = 2 * i0 - 1, v0 = 2 * j0 - 1;  // dup window origin
  for (int e = threadIdx.x; e < 9 * p.c; e += NT) wl[(e / p.c) * CMAX + e % p.c] = p.wt[e];
  // dy window: dyl[a][b] = dy[u0 - 1 + a][v0 - 1 + b]
  for (int e = threadIdx.x; e < DY * DY; e += NT) {
    const int yy = u0 - 1 + e / DY, xx = v0 - 1 + e % DY;
    dyl[e] = (yy >= 0 && yy < H2 && xx >= 0 && xx < W2) ? p.dy[((long)img * H2 + yy) * W2 + xx]
                                                         : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < DU * DU * nq; e += NT) {
    const int q = e % nq, pix = e / nq;
    const int a = pix / DU, b = pix % DU;
    const int uy = u0 + a, ux = v0 + b;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (uy >= 0 && uy < H2 && ux >= 0 && ux < W2) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        // y[p] = sum_t w[t] up[p + t - 1]  =>  dup[q] = sum_t w[t] dy[q - t + 1]
        const float g = dyl[(a + 2 - t / 3) * DY + b + 2 - t % 3];
        const float4 f = *reinterpret_cast<const float4*>(wl + t * CMAX + 4 * q);
        o.x += g * f.x; o.y += g * f.y; o.z += g * f.z; o.w += g * f.w;
      }
    }
    *reinterpret_cast<float4*>(dup + pix * CS + 4 * q) = o;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < DT * DT * nq; e += NT) {
    const int q = e % nq, pix = e / nq;
    const int i = i0 + pix / DT, j = j0 + pix % DT;
    if (i >= p.h || j >= p.w) continue;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int du = -1; du <= 2; ++du) {
      const int uy = 2 * i + du;
      if (uy < 0 || uy >= H2) continue;
      int y0, y1;
      float yl;
      lerp_coords(uy, p.h, y0, y1, yl);
      const float wy = (y0 == i ? 1.f - yl : 0.f) + (y1 == i ? yl : 0.f);
      if (wy == 0.f) continue;
#pragma unroll
      for (int dv = -1; dv <= 2; ++dv) {
        const int ux = 2 * j + dv;
        if (ux < 0 || ux >= W2) continue;
        int x0, x1;
        float xl;
        lerp_coords(ux, p.w, x0, x1, xl);
        const float wx = (x0 == j ? 1.f - xl : 0.f) + (x1 == j ? xl : 0.f);
        if (wx == 0.f) continue;
        const float ww = wy * wx;
        const float4 g = *reinterpret_cast<const float4*>(
            dup + ((uy - u0) * DU + (ux - v0)) * CS + 4 * q);
        a.x += ww * g.x; a.y += ww * g.y; a.z += ww * g.z; a.w += ww * g.w;
      }
    }
    *reinterpret_cast<float4*>(p.y + (((long)img * p.h + i) * p.w + j) * p.c + 4 * q) = a;
  }
}

constexpr int FWD_BLOCKS = 2048;
constexpr int WG_BLOCKS = 2048;

static bool args_ok(const float* x, int n, int h, int w, int c) {
  return x && n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && c <= CMAX && aligned16(x);
}

static Params mk(const float* x, int n, int h, int w, int c, const float* mean,
                 const float* invstd, const float* gamma, const float* beta) {
  Params p{};
  p.x = x;
  p.n = n; p.h = h; p.w = w; p.c = c;
  p.mean = mean; p.invstd = invstd; p.gamma = gamma; p.beta = beta;
  p.tiles_x = (int)cdiv(2 * w, ST);
  p.tiles_y = (int)cdiv(2 * h, ST);
  return p;
}

}  // namespace upc
}  // namespace pld

using namespace pld;

extern "C" size_t pld_upconv_wgrad_workspace_size(int c) {
  return c > 0 ? sizeof(float) * (size_t)upc::WG_BLOCKS * 9 * c : 0;
}

extern "C" int pld_upconv_fwd(const float* x, int n, int h, int w, int c, const float* mean,
                              const float* invstd, const float* gamma, const float* beta,
                              const float* wt, const float* bias, float* y, void* stream) {
  PLD_CHECK_ARG(upc::args_ok(x, n, h, w, c) && mean && invstd && gamma && beta && wt && y,
                "pld_upconv_fwd: bad args (c %% 4 == 0, c <= 32, 16-byte aligned x)");
  upc::Params p = upc::mk(x, n, h, w, c, mean, invstd, gamma, beta);
  p.wt = wt;
  p.bias = bias;
  p.y = y;
  const int ntiles = p.tiles_x * p.tiles_y * n;
  upc::upconv_fwd_kernel<<<std::min(upc::FWD_BLOCKS, ntiles), upc::NT, 0, as_stream(stream)>>>(p);
  return check_launch("upconv_fwd_kernel");
}

extern "C" int pld_upconv_wgrad(const float* x, int n, int h, int w, int c, const float* mean,
                                const float* invstd, const float* gamma, const float* beta,
                                const float* dy, float* dw, void* ws, size_t ws_bytes,
                                void* stream) {
  PLD_CHECK_ARG(upc::args_ok(x, n, h, w, c) && mean && invstd && gamma && beta && dy && dw,
                "pld_upconv_wgrad: bad args");
  PLD_CHECK_ARG(ws && ws_bytes >= pld_upconv_wgrad_workspace_size(c),
                "pld_upconv_wgrad: workspace too small");
  upc::Params p = upc::mk(x, n, h, w, c, mean, invstd, gamma, beta);
  p.dy = dy;
  p.part = (float*)ws;
  const int ntiles = p.tiles_x * p.tiles_y * n;
  const int nb = std::min(upc::WG_BLOCKS, ntiles);
  hipStream_t st = as_stream(stream);
  upc::upconv_wgrad_kernel<<<nb, upc::NT, 0, st>>>(p);
  int rc = check_launch("upconv_wgrad_kernel");
  if (rc) return rc;
  upc::upconv_wgrad_reduce_kernel<<<9 * c, 256, 0, st>>>(p.part, nb, 9 * c, dw);
  return check_launch("upconv_wgrad_reduce_kernel");
}

extern "C" int pld_upconv_dgrad(const float* dy, int n, int h, int w, int c, const float* wt,
                                float* dact, void* stream) {
  PLD_CHECK_ARG(dy && wt && dact && n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 &&
                    c <= upc::CMAX && aligned16(dact),
                "pld_upconv_dgrad: bad args");
  upc::Params p{};
  p.dy = dy;
  p.wt = wt;
  p.y = dact;
  p.n = n; p.h = h; p.w = w; p.c = c;
  dim3 grid(cdiv(w, upc::DT), cdiv(h, upc::DT), n);
  upc::upconv_dgrad_kernel<<<grid, upc::NT, 0, as_stream(stream)>>>(p);
  return check_launch("upconv_dgrad_kernel");
}

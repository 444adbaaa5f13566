// DepthwiseConv2D forward, LDS-tiled (keras efficientnet block(): DepthwiseConv2D k3/k5,
// stride 1 'same' or stride 2 after ZeroPadding2D; frozen filters, pl_hourglass.py:52-57), with
// the block's expand BN + swish applied to the input as it is staged and, optionally, the batch
// statistics of the output (the BN that follows) gathered in the epilogue.
//
// A workgroup walks a contiguous run of TO-wide output tiles of one group of 4 CQ = 32 channels
// (the last group masked when C % 32 == 16), the next tile's window loads issued before the
// current tile's FMAs so that they overlap (tile_plan sizes the grid to one resident round). The
// ((TO - 1) S + K)^2 input window of those channels is read once (coalesced: CQ * 16 contiguous
// bytes per pixel), activated once per element (the register-window kernel in dwse.hip
// re-activated every overlapping window load: ~4x the exp / rcp work at k5) and stored in LDS,
// for stride 2 with even and odd columns in separate planes so that neighbouring output columns
// read neighbouring LDS addresses. Each thread then owns one channel quad, one output column
// and R rows: it walks the (R - 1) S + K input rows of its column window once, feeding every tap
// of every output row it reaches from registers (filter taps preloaded), in the same (ty, tx)
// summation order as the direct loop. Statistics: per-thread fp64 sums of its outputs, combined
// over the workgroup in a fixed order into [C][workgroups][2] partials (bn.hip's finalize layout).
#include <algorithm>

#include "common.h"

namespace pld {
namespace dwt {

struct Geo {
  const float* x;
  const float* w;       // [K][K][C]
  float* y;
  const float* mean;    // input prologue act(bn(x)) or NULL
  const float* invstd;
  const float* gamma;
  const float* beta;
  double* stats;        // [C][gridDim.x][2] or NULL
  int n, h, wd, c, oh, ow, pt, pl;
  int tiles_x, tiles_y;
  int per;              // tiles per workgroup (a contiguous run of its channel group's tiles)
  int accum;            // DG: y += result
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

// output rows per tile: 4 per thread (k5 stride 1) / 2 (stride 2)
__host__ __device__ constexpr int tile_rows(int s, int cq) { return (256 / (cq * (s == 1 ? 16 : 8))) * (s == 1 ? 4 : 2); }

// Workgroups per launch: every workgroup of the grid resident at once (DW_MINB per CU: the
// launch bound holds every instantiation's VGPRs to that, the windows fit the LDS), each walking a contiguous run of
// tiles of its channel group with the next tile's window loads in flight while the current one
// is computed (one tile per workgroup left the load, the prologue and the FMA/LDS phases
// serialised: 2-3.9 TB/s at 14^2-56^2).
#ifndef PLD_DW_MINB
#define PLD_DW_MINB 2
#endif
constexpr int RESIDENT = PLD_DW_MINB * 256;

__host__ __device__ constexpr int tile_cols(int s) { return s == 1 ? 16 : 8; }

// tiles per workgroup and workgroups per channel group (grid.x = the statistics' part count)
static void tile_plan(int n, int oh, int ow, int s, int c, int& per, int& nbx) {
  const long nsp = (long)n * cdiv(oh, tile_rows(s, 8)) * cdiv(ow, tile_cols(s));
  const long ncg = cdiv(c, 32);
  const long slots = std::max<long>(1, RESIDENT / ncg);
  per = (int)cdiv(nsp, slots);
  nbx = (int)cdiv(nsp, per);
}

// DG (stride 1): the input gradient of a stride-1 depthwise conv as this correlation of dy with
// the flipped filter, window pads K - 1 - pad; the taps of every output summed in ascending
// (ty, tx) order of the unflipped filter, as dwconv_dgrad_s1_kernel (dwse.hip) sums them, so the
// two paths agree bit for bit (the BN-fused dgrad epilogue stays on that kernel).
template <int K, int S, int CQ, int ACT, bool DG = false>  // ACT < 0: no prologue
__global__ __launch_bounds__(256, PLD_DW_MINB) void dw_fwd_tile_kernel(Geo g) {
  constexpr int TO = tile_cols(S);                // output tile width
  constexpr int TOH = tile_rows(S, CQ);           // output tile height
  constexpr int TI = (TO - 1) * S + K;            // input window width
  constexpr int TIR = (TOH - 1) * S + K;          // input window height
  constexpr int TIH = (TI + 1) / 2;               // stride 2: columns per parity plane
  constexpr int COLS = S == 1 ? TI : 2 * TIH;     // LDS columns (parity planes side by side)
  constexpr int RGN = 256 / (CQ * TO);            // row groups
  constexpr int R = TOH / RGN;                    // output rows per thread
  constexpr int NR = (R - 1) * S + K;             // input rows a thread walks
  constexpr int NE = TIR * TI * CQ;               // window float4s
  constexpr int NL = (NE + 255) / 256;
  static_assert(256 % CQ == 0, "a thread's staged channel quad is tid % CQ on every load");
  static_assert(!DG || (S == 1 && ACT < 0), "the dgrad form is stride 1 without a prologue");
  extern __shared__ __attribute__((aligned(16))) float4 tile[];  // [TIR][COLS][CQ], [K K][CQ]
  float4* ftile = tile + TIR * COLS * CQ;
  const int tid = threadIdx.x;
  const int cb = blockIdx.y * CQ * 4;             // first channel of the group
  const int ntx = g.tiles_x, nt = g.tiles_x * g.tiles_y;
  const int nsp = g.n * nt;
  const int sp0 = blockIdx.x * g.per, sp1 = min(nsp, sp0 + g.per);
  const int q = tid % CQ;                         // staged quad (all loads) = computed quad
  const bool qok = cb + 4 * q < g.c;  // the last group of a C % 32 == 16 layer is half full
  const float* fq = g.w + (qok ? cb + 4 * q : 0);  // this thread's filter quad: tap t at fq + t C
  float4 mu, is, ga, be;
  if (ACT >= 0 && qok) {
    mu = *reinterpret_cast<const float4*>(g.mean + cb + 4 * q);
    is = *reinterpret_cast<const float4*>(g.invstd + cb + 4 * q);
    ga = *reinterpret_cast<const float4*>(g.gamma + cb + 4 * q);
    be = *reinterpret_cast<const float4*>(g.beta + cb + 4 * q);
  }
  // k3: the 9 taps in registers; k5: the 25 taps staged once in LDS (filter loads inside the
  // tile loop would queue behind the prefetched window and wait for it)
  float4 f3[K == 3 ? 3 : 1][K == 3 ? 3 : 1];
  if constexpr (K == 3) {
#pragma unroll
    for (int ty = 0; ty < K; ++ty)
#pragma unroll
      for (int tx = 0; tx < K; ++tx) f3[ty][tx] = *reinterpret_cast<const float4*>(fq + (ty * K + tx) * g.c);
  } else {
    for (int e = tid; e < K * K * CQ; e += 256) {
      const int t = e / CQ, qq = e % CQ;
      ftile[e] = cb + 4 * qq < g.c ? *reinterpret_cast<const float4*>(g.w + t * g.c + cb + 4 * qq)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  auto origin = [&](int sp, int& img, int& oy0, int& ox0) {
    img = sp / nt;
    const int rr = sp - img * nt;
    oy0 = (rr / ntx) * TOH;
    ox0 = (rr % ntx) * TO;
  };
  float4 v[NL];
  auto load_window = [&](int sp) {
    int img, oy0, ox0;
    origin(sp, img, oy0, ox0);
    const int iy0 = oy0 * S - g.pt, ix0 = ox0 * S - g.pl;
    const float* xb = g.x + (long)img * g.h * g.wd * g.c + cb;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 256 * i;
      const int px = e / CQ;
      const int wy = px / TI, wx = px - wy * TI;
      const int iy = iy0 + wy, ix = ix0 + wx;
      const bool ok = e < NE && (unsigned)iy < (unsigned)g.h && (unsigned)ix < (unsigned)g.wd && qok;
      v[i] = ok ? *reinterpret_cast<const float4*>(xb + ((long)iy * g.wd + ix) * g.c + 4 * q)
                : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const int oc = (tid / CQ) % TO, rg = tid / (CQ * TO);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (sp0 < sp1) load_window(sp0);
  for (int sp = sp0; sp < sp1; ++sp) {
    int img, oy0, ox0;
    origin(sp, img, oy0, ox0);
    const int iy0 = oy0 * S - g.pt, ix0 = ox0 * S - g.pl;
    __syncthreads();  // the previous tile's window is no longer read
    // ---- the prologue and the LDS stores of this tile's window ----
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 256 * i;
      if (e >= NE) break;
      const int px = e / CQ;
      const int wy = px / TI, wx = px - wy * TI;
      const int iy = iy0 + wy, ix = ix0 + wx;
      float4 a = v[i];
      if (ACT >= 0 && (unsigned)iy < (unsigned)g.h && (unsigned)ix < (unsigned)g.wd && qok) {
        // bn_apply's arithmetic, then the activation (TF pads the activated map with zeros)
        a = make_float4(act_fwd(ACT, ((a.x - mu.x) * is.x) * ga.x + be.x),
                        act_fwd(ACT, ((a.y - mu.y) * is.y) * ga.y + be.y),
                        act_fwd(ACT, ((a.z - mu.z) * is.z) * ga.z + be.z),
                        act_fwd(ACT, ((a.w - mu.w) * is.w) * ga.w + be.w));
      }
      const int col = S == 1 ? wx : (wx & 1) * TIH + (wx >> 1);
      tile[(wy * COLS + col) * CQ + q] = a;
    }
    __syncthreads();
    if (sp + 1 < sp1) load_window(sp + 1);  // in flight under this tile's FMAs
    float4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    auto lds_row = [&](int wy, float4 (&row)[K]) {
#pragma unroll
      for (int tx = 0; tx < K; ++tx) {
        const int wx = oc * S + tx;
        const int col = S == 1 ? wx : (wx & 1) * TIH + (wx >> 1);
        row[tx] = tile[(wy * COLS + col) * CQ + q];
      }
    };
    if constexpr (K == 3) {
      // each of the (R - 1) S + K input rows of the column window read once and fed to every
      // output row it reaches (DG: rows bottom-up, window offsets K - 1 - tap)
#pragma unroll
      for (int jj = 0; jj < NR; ++jj) {
        const int j = DG ? NR - 1 - jj : jj;
        float4 row[K];
        lds_row(rg * R * S + j, row);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int ty = j - r * S;  // compile-time after unrolling
          if (ty < 0 || ty >= K) continue;
#pragma unroll
          for (int tx = 0; tx < K; ++tx) {
            if constexpr (DG) acc[r] = fma4(acc[r], row[K - 1 - tx], f3[K - 1 - ty][tx]);
            else acc[r] = fma4(acc[r], row[tx], f3[ty][tx]);
          }
        }
      }
    } else {
      // k5: one filter row (5 taps) at a time, ty outer; each output row re-reads its input row
      // per ty (25 taps in registers plus the unrolled window do not fit)
#pragma unroll 1
      for (int ty = 0; ty < K; ++ty) {
        float4 f[K];
#pragma unroll
        for (int tx = 0; tx < K; ++tx) f[tx] = ftile[(ty * K + tx) * CQ + q];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float4 row[K];
          lds_row(rg * R * S + r * S + (DG ? K - 1 - ty : ty), row);
#pragma unroll
          for (int tx = 0; tx < K; ++tx) acc[r] = fma4(acc[r], row[DG ? K - 1 - tx : tx], f[tx]);
        }
      }
    }
    // ---- store (+ statistics) ----
    const int ox = ox0 + oc;
    if (ox < g.ow && qok) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int oy = oy0 + rg * R + r;
        if (oy >= g.oh) break;
        float4* yp = reinterpret_cast<float4*>(g.y + (((long)img * g.oh + oy) * g.ow + ox) * g.c + cb + 4 * q);
        if (DG && g.accum) {
          const float4 old = *yp;
          acc[r].x += old.x; acc[r].y += old.y; acc[r].z += old.z; acc[r].w += old.w;
        }
        *yp = acc[r];
        if (g.stats) {
          const float a4[4] = {acc[r].x, acc[r].y, acc[r].z, acc[r].w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const double d = a4[u];
            s1[u] += d;
            s2[u] += d * d;
          }
        }
      }
    }
  }
  if (!g.stats) return;
  __syncthreads();  // the window is no longer read: reuse it for the fixed-order combine
  double* red = reinterpret_cast<double*>(tile);  // [256][8]
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    red[tid * 8 + u] = s1[u];
    red[tid * 8 + 4 + u] = s2[u];
  }
  __syncthreads();
  if (tid < CQ && qok) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = red[tid * 8 + u];
    for (int j = 1; j < 256 / CQ; ++j)
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] += red[(tid + CQ * j) * 8 + u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<double2*>(g.stats + ((long)(cb + 4 * tid + u) * gridDim.x + blockIdx.x) * 2) =
          make_double2(t[u], t[4 + u]);
  }
}

template <int K, int S, int CQ>
static size_t lds_bytes() {
  constexpr int TO = tile_cols(S);
  constexpr int TI = (TO - 1) * S + K;
  constexpr int TIR = (tile_rows(S, CQ) - 1) * S + K;
  constexpr int COLS = S == 1 ? TI : 2 * ((TI + 1) / 2);
  const size_t win = sizeof(float4) * (TIR * COLS * CQ + (K == 5 ? K * K * CQ : 0));
  return std::max(win, sizeof(double) * 256 * 8);
}

template <int K, int S, int CQ>
static void launch(Geo& g, int act, hipStream_t st) {
  g.tiles_x = (int)cdiv(g.ow, tile_cols(S));
  g.tiles_y = (int)cdiv(g.oh, tile_rows(S, CQ));
  int nbx;
  tile_plan(g.n, g.oh, g.ow, S, g.c, g.per, nbx);
  dim3 grid(nbx, (int)cdiv(g.c, 4 * CQ));
  const size_t lds = lds_bytes<K, S, CQ>();
  if (!g.mean) dw_fwd_tile_kernel<K, S, CQ, -1><<<grid, 256, lds, st>>>(g);
  else if (act == ACT_SWISH) dw_fwd_tile_kernel<K, S, CQ, ACT_SWISH><<<grid, 256, lds, st>>>(g);
  else if (act == ACT_RELU) dw_fwd_tile_kernel<K, S, CQ, ACT_RELU><<<grid, 256, lds, st>>>(g);
  else if (act == ACT_SIGMOID) dw_fwd_tile_kernel<K, S, CQ, ACT_SIGMOID><<<grid, 256, lds, st>>>(g);
  else dw_fwd_tile_kernel<K, S, CQ, ACT_NONE><<<grid, 256, lds, st>>>(g);
}

}  // namespace dwt
}  // namespace pld

using namespace pld;

// eligible: k 3 / 5, stride 1 / 2, C % 16 == 0, 16-byte aligned tensors
extern "C" int pld__dw_tiled_ok(int k, int s, int c) {
  return (k == 3 || k == 5) && (s == 1 || s == 2) && c % 16 == 0;
}

extern "C" int pld__dw_tiled_parts(int n, int oh, int ow, int s, int c) {
  int per, nbx;
  dwt::tile_plan(n, oh, ow, s, c, per, nbx);
  return nbx;
}

extern "C" int pld__dw_fwd_tiled(const float* x, int n, int h, int w, int c, const float* wdw,
                                 int k, int s, int pad_t, int pad_l, int oh, int ow,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, int act, float* y, double* stats,
                                 hipStream_t st) {
  dwt::Geo g{};
  g.x = x; g.w = wdw; g.y = y;
  g.mean = mean; g.invstd = invstd; g.gamma = gamma; g.beta = beta;
  g.stats = stats;
  g.n = n; g.h = h; g.wd = w; g.c = c; g.oh = oh; g.ow = ow; g.pt = pad_t; g.pl = pad_l;
  // 32-channel groups (one 128-byte line per pixel), the last one masked when C % 32 == 16:
  // 16-channel groups would split every line between two workgroups that run far apart
#define DWT(KK, SS) dwt::launch<KK, SS, 8>(g, act, st);
  if (k == 3 && s == 1) { DWT(3, 1) }
  else if (k == 3) { DWT(3, 2) }
  else if (k == 5 && s == 1) { DWT(5, 1) }
  else { DWT(5, 2) }
#undef DWT
  return check_launch("dw_fwd_tile_kernel");
}

// stride-1 input gradient through the tiled kernel (DG): dx [n][h][w][c] from dy [n][oh][ow][c]
extern "C" int pld__dw_dgrad_tiled(const float* dy, int n, int h, int w, int c, const float* wdw,
                                   int k, int pad_t, int pad_l, int oh, int ow, float* dx,
                                   int accumulate, hipStream_t st) {
  dwt::Geo g{};
  g.x = dy; g.w = wdw; g.y = dx;
  g.n = n; g.h = oh; g.wd = ow; g.c = c; g.oh = h; g.ow = w;
  g.pt = k - 1 - pad_t; g.pl = k - 1 - pad_l;
  g.accum = accumulate;
  g.tiles_x = (int)cdiv(w, dwt::tile_cols(1));
  g.tiles_y = (int)cdiv(h, dwt::tile_rows(1, 8));
  int nbx;
  dwt::tile_plan(n, h, w, 1, c, g.per, nbx);
  dim3 grid(nbx, (int)cdiv(c, 32));
  if (k == 3)
    dwt::dw_fwd_tile_kernel<3, 1, 8, -1, true><<<grid, 256, dwt::lds_bytes<3, 1, 8>(), st>>>(g);
  else
    dwt::dw_fwd_tile_kernel<5, 1, 8, -1, true><<<grid, 256, dwt::lds_bytes<5, 1, 8>(), st>>>(g);
  return check_launch("dw_fwd_tile_kernel(dgrad)");
}

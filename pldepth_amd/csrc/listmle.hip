// ListMLE (Plackett–Luce NLL) forward + closed-form backward over sampled pixel lists.
//
// Replaces, in one pass per list: prepare_fully_fledged_loss_input (pldepth/data/depth_utils.py:
// 39-61: gather pred[b, idx] with batch_dims=1), tfr ListMLELoss.compute_unreduced_loss (validity,
// sort-by-label, max-shift, reverse log-cumsum-exp; nll_loss.py:62) and the Keras
// SUM_OVER_BATCH_SIZE mean, plus the gradient d loss / d pred scattered back into the dense map
// (the gather's UnsortedSegmentSum).
//
// One wave64 per list; each lane owns EPL consecutive list elements (L <= 64*EPL). Keys are
// staged in LDS for the O(L) rank computation (lists arrive pre-sorted from the sampler, so the
// sort is usually the identity; ties keep "later element first", see oracle/listmle.py).
// HBM-bound: 8 B/element (idx, label) + 4 B gather + 4 B scatter.
#include <algorithm>

#include "common.h"

namespace pld {

constexpr float kLogEps = -23.025850929940457f;  // tf.math.log(1e-10) in float32

template <int EPL>
__global__ __launch_bounds__(256) void listmle_kernel(const float* __restrict__ pred,
                                                      const float* __restrict__ y_true, int B,
                                                      int HW, int R, int L, float inv_n,
                                                      float* __restrict__ nll_out,
                                                      float* __restrict__ dpred) {
  constexpr int WAVES = 4;
  constexpr int LMAX = 64 * EPL;
  __shared__ float s_key[WAVES][LMAX];
  __shared__ float s_val[WAVES][LMAX];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const long list = (long)blockIdx.x * WAVES + wave;
  const long nlists = (long)B * R;
  const bool active = list < nlists;  // wave-uniform; inactive waves still reach the barriers
  const int b = active ? (int)(list / R) : 0;
  if (!active) L = 0;
  const float* yt = y_true + (active ? list : 0) * (long)L * 2;
  const float* pb = pred + (long)b * HW;

  float s[EPL], lab[EPL];
  int idx[EPL];
  bool valid[EPL], inl[EPL];
  float minlab = INFINITY;
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int e = lane * EPL + q;
    inl[q] = e < L;
    idx[q] = -1;
    s[q] = 0.f;
    lab[q] = 0.f;
    valid[q] = false;
    if (inl[q]) {
      const float fi = yt[2 * e];
      lab[q] = yt[2 * e + 1];
      const int ii = (int)fi;  // tf.cast(float32 -> int32): truncation
      idx[q] = ii;
      s[q] = (ii >= 0 && ii < HW) ? pb[ii] : 0.f;  // TF GPU gather yields 0 out of range
      valid[q] = lab[q] >= 0.f;
      if (!valid[q]) lab[q] = 0.f;
      minlab = fminf(minlab, lab[q]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) minlab = fminf(minlab, __shfl_xor(minlab, o, 64));
  // sort scores: valid -> label, invalid -> min(label') - 1e-6 (float32)
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int e = lane * EPL + q;
    if (inl[q]) s_key[wave][e] = valid[q] ? lab[q] : (minlab - 1e-6f);
    if (!valid[q]) s[q] = kLogEps;
  }
  __syncthreads();
  int rank[EPL];
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int e = lane * EPL + q;
    int r = 0;
    if (inl[q]) {
      const float k = s_key[wave][e];
      for (int j = 0; j < L; ++j) {
        const float kj = s_key[wave][j];
        r += (kj > k) | ((kj == k) & (j > e));
      }
    }
    rank[q] = r;
  }
#pragma unroll
  for (int q = 0; q < EPL; ++q)
    if (inl[q]) s_val[wave][rank[q]] = s[q];
  __syncthreads();
  // sorted logits t_r, r = lane*EPL + q
  float t[EPL];
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int r = lane * EPL + q;
    t[q] = (r < L) ? s_val[wave][r] : -INFINITY;
    m = fmaxf(m, t[q]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float ex[EPL];
  float lsum = 0.f;
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int r = lane * EPL + q;
    ex[q] = (r < L) ? expf(t[q] - m) : 0.f;
    lsum += ex[q];
  }
  // suffix (reverse inclusive) sum over ranks: C_r = sum_{j>=r} ex_j
  // lanes above contribute their whole chunk sums: exclusive suffix scan across lanes
  // (exclusive scans are formed by shifting first, never by subtracting: the last ranks can
  // carry 1/C ~ 1e10 when invalid elements sit there, and a difference would cancel)
  float above = __shfl_down(lsum, 1, 64);
  if (lane == 63) above = 0.f;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float v = __shfl_down(above, o, 64);
    if (lane + o < 64) above += v;
  }  // sum of the chunks of lanes > lane
  float C[EPL];
  {
    float run = above;
#pragma unroll
    for (int q = EPL - 1; q >= 0; --q) {
      run += ex[q];
      C[q] = run;
    }
  }
  float part = 0.f, pinv = 0.f;
  float inv[EPL];
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int r = lane * EPL + q;
    if (r < L) {
      part += logf(C[q]) - (t[q] - m);
      inv[q] = 1.f / C[q];
    } else {
      inv[q] = 0.f;
    }
    pinv += inv[q];
  }
  const float nll = wave_sum(part);
  // prefix (inclusive) sum of 1/C over ranks
  float run = __shfl_up(pinv, 1, 64);
  if (lane == 0) run = 0.f;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float v = __shfl_up(run, o, 64);
    if (lane >= o) run += v;
  }  // sum of the chunks of lanes < lane
  __syncthreads();
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    const int r = lane * EPL + q;
    run += inv[q];
    if (r < L) s_val[wave][r] = ex[q] * run - 1.f;  // d nll / d t_r
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    if (inl[q] && valid[q] && idx[q] >= 0 && idx[q] < HW) {
      const float g = s_val[wave][rank[q]] * inv_n;
      atomicAdd(dpred + (long)b * HW + idx[q], g);
    }
  }
  if (active && lane == 0) nll_out[list] = nll;
}

// deterministic mean of the per-list nll (single block, fp64 accumulation)
__global__ __launch_bounds__(256) void mean_kernel(const float* __restrict__ x, long n,
                                                   float* __restrict__ out) {
  __shared__ double red[256];
  double acc = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) acc += (double)x[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] / (double)n);
}

// dpred = 0 ahead of the scatter. A kernel, not hipMemsetAsync: replayed from a hipGraph with
// this ROCm runtime's packet capture on, the memset node was not ordered before the scatter
// kernel that follows it (the atomics landed on a partly cleared buffer and replays drifted;
// tools/graph_bisect.py isolated this call, tools/graph_memset_repro.hip reproduces it with the
// runtime alone). Every node of the library's captured steps is now a kernel.
__global__ __launch_bounds__(256) void zero_kernel(float* __restrict__ p, long n) {
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long i = 4 * n4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    p[i] = 0.f;
}

}  // namespace pld

extern "C" int pld_listmle_fwd_bwd(const float* pred, const float* y_true, int B, int HW, int R,
                                   int L, float* nll, float* loss, float* dpred, int zero_dpred,
                                   void* stream) {
  using namespace pld;
  PLD_CHECK_ARG(pred && y_true && nll && loss && dpred, "pld_listmle_fwd_bwd: null pointer");
  PLD_CHECK_ARG(B > 0 && HW > 0 && R > 0 && L >= 1 && L <= 512,
                "pld_listmle_fwd_bwd: bad shape B=%d HW=%d R=%d L=%d (L must be 1..512)", B, HW,
                R, L);
  hipStream_t st = as_stream(stream);
  PLD_CHECK_ARG(!zero_dpred || aligned16(dpred), "pld_listmle_fwd_bwd: dpred must be 16-byte "
                "aligned");
  if (zero_dpred) {
    const long nz = (long)B * HW;
    zero_kernel<<<(unsigned)std::min<long>(cdiv(nz / 4 + 1, 256), 4096), 256, 0, st>>>(dpred, nz);
    int rc = check_launch("zero_kernel");
    if (rc) return rc;
  }
  const long n = (long)B * R;
  const float inv_n = (float)(1.0 / (double)n);
  dim3 grid(cdiv(n, 4)), block(256);
  if (L <= 64)
    listmle_kernel<1><<<grid, block, 0, st>>>(pred, y_true, B, HW, R, L, inv_n, nll, dpred);
  else if (L <= 128)
    listmle_kernel<2><<<grid, block, 0, st>>>(pred, y_true, B, HW, R, L, inv_n, nll, dpred);
  else if (L <= 256)
    listmle_kernel<4><<<grid, block, 0, st>>>(pred, y_true, B, HW, R, L, inv_n, nll, dpred);
  else
    listmle_kernel<8><<<grid, block, 0, st>>>(pred, y_true, B, HW, R, L, inv_n, nll, dpred);
  int rc = check_launch("listmle_kernel");
  if (rc) return rc;
  mean_kernel<<<1, 256, 0, st>>>(nll, n, loss);
  return check_launch("mean_kernel");
}

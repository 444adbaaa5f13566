// GPU ranking sampler: replaces the per-image numpy sampler the reference runs under
// tf.numpy_function (pldepth/data/providers/hourglass_provider.py:55-58 -> pldepth/data/sampling.py).
//
// Split into (a) draws and (b) a deterministic part, so (b) is tested bit-for-bit against the
// numpy restatement (oracle/sampler.py, itself pinned to the reference's golden vectors) by
// injecting the same draws:
//   compact : np.where(mask > 0) per image (row-major order), plus min/max of gt (Info strategy)
//   draw    : Philox4x32-10 keyed by (seed), counter (cand*L+slot, image, step) -> uniform index
//             in [0, nvalid) by 32x32->64 multiply-high (the reference: np.random.randint)
//   rank    : gather (flat index row*W+col as float32, gt), per-list descending sort (ties: later
//             slot first), strategy score in the reference's exact float types and association
//             (float32 sequential sum for Masked/Thresholded, float32 NumPy-pairwise sum + float64
//             penalties for Info), then per-image top-R by (score desc, candidate index desc).
// Compiled with -ffp-contract=off: no FMA contraction may change a rounding step.
#include <algorithm>

#include "common.h"

namespace pld {

// ------------------------------------------------------------------ compaction + min/max
// np.where(mask > 0) order (row-major flat index, sampling.py:135) for every image, plus the
// whole-image gt min/max of the Info strategy (sampling.py:223). Images are cut into segments of
// COMPACT_SEG pixels: pass 1 counts each segment's valid pixels (and its gt min/max), pass 2
// gives each segment its output offset (sum of the earlier segments' counts) and writes its
// indices in order with wave-ballot prefix sums. Reads are coalesced; 2 x B x S workgroups.
constexpr int COMPACT_THREADS = 1024;
constexpr int COMPACT_SEG = 16384;

__device__ __forceinline__ int block_sum_1024(int v, int* s_w) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) s_w[w] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int i = 0; i < COMPACT_THREADS / 64; ++i) t += s_w[i];
  return t;
}

__global__ __launch_bounds__(COMPACT_THREADS) void compact_count_kernel(
    const float* __restrict__ mask, int HW, const float* __restrict__ gt, int S,
    int* __restrict__ seg_cnt, float* __restrict__ seg_mm) {
  __shared__ int s_w[COMPACT_THREADS / 64];
  __shared__ float s_mn[COMPACT_THREADS / 64], s_mx[COMPACT_THREADS / 64];
  const int s = blockIdx.x, b = blockIdx.y;
  const int beg = s * COMPACT_SEG, end = min(HW, beg + COMPACT_SEG);
  const float* mb = mask + (long)b * HW;
  const float* gb = gt ? gt + (long)b * HW : nullptr;
  int cnt = 0;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = beg + threadIdx.x; i < end; i += COMPACT_THREADS) {
    cnt += mb[i] > 0.f;
    if (gb) {
      const float g = gb[i];
      mn = fminf(mn, g);
      mx = fmaxf(mx, g);
    }
  }
  const int tot = block_sum_1024(cnt, s_w);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  if (lane == 0) {
    s_mn[w] = mn;
    s_mx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < COMPACT_THREADS / 64; ++i) {
      mn = fminf(mn, s_mn[i]);
      mx = fmaxf(mx, s_mx[i]);
    }
    seg_cnt[b * S + s] = tot;
    seg_mm[2 * (b * S + s)] = mn;
    seg_mm[2 * (b * S + s) + 1] = mx;
  }
}

__global__ __launch_bounds__(COMPACT_THREADS) void compact_write_kernel(
    const float* __restrict__ mask, int HW, int S, const int* __restrict__ seg_cnt,
    const float* __restrict__ seg_mm, int* __restrict__ valid_idx, int* __restrict__ nvalid,
    float* __restrict__ gt_minmax) {
  __shared__ int s_w[COMPACT_THREADS / 64];
  const int s = blockIdx.x, b = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int off = 0;
  for (int i = 0; i < s; ++i) off += seg_cnt[b * S + i];
  if (s == 0 && threadIdx.x == 0) {
    int n = 0;
    float mn = INFINITY, mx = -INFINITY;
    for (int i = 0; i < S; ++i) {
      n += seg_cnt[b * S + i];
      mn = fminf(mn, seg_mm[2 * (b * S + i)]);
      mx = fmaxf(mx, seg_mm[2 * (b * S + i) + 1]);
    }
    nvalid[b] = n;
    if (gt_minmax) {
      gt_minmax[2 * b] = mn;
      gt_minmax[2 * b + 1] = mx;
    }
  }
  const int beg = s * COMPACT_SEG, end = min(HW, beg + COMPACT_SEG);
  const float* mb = mask + (long)b * HW;
  int* out = valid_idx + (long)b * HW;
  for (int base = beg; base < end; base += COMPACT_THREADS) {
    const int i = base + threadIdx.x;
    const bool f = i < end && mb[i] > 0.f;
    const unsigned long long bal = __ballot(f);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    __syncthreads();  // s_w reuse
    if (lane == 0) s_w[w] = __popcll(bal);
    __syncthreads();
    int wave_off = 0, total = 0;
#pragma unroll
    for (int k = 0; k < COMPACT_THREADS / 64; ++k) {
      const int c = s_w[k];
      wave_off += k < w ? c : 0;
      total += c;
    }
    if (f) out[off + wave_off + before] = i;
    off += total;
  }
}

// ------------------------------------------------------------------ Philox draws
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__global__ void draw_kernel(const int* __restrict__ nvalid, int B, int per_img, uint64_t seed,
                            uint64_t step_arg, const int64_t* __restrict__ step_dev,
                            int image_offset, int* __restrict__ draws) {
  const uint64_t step = step_dev ? (uint64_t)step_dev[0] : step_arg;
  const long total = (long)B * per_img;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int b = (int)(e / per_img);
    const uint32_t slot = (uint32_t)(e - (long)b * per_img);
    const uint4 r = philox4x32_10(
        make_uint4(slot, (uint32_t)(image_offset + b), (uint32_t)step, (uint32_t)(step >> 32)),
        make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const uint32_t n = (uint32_t)max(nvalid[b], 0);
    draws[e] = (int)(((uint64_t)r.x * n) >> 32);
  }
}

// ------------------------------------------------------------------ per-list sort + score
__device__ __forceinline__ int depth_relation32(float d1, float d2) {
  // pldepth/data/depth_utils.py:5-21 with tau = 0.03, float32 (NumPy 2 / NEP 50)
  const float eps = 1e-10f;
  const float r = __fdiv_rn(add_rn(d1, eps), add_rn(d2, eps));
  if (r >= 1.03f) return 1;
  if (r <= (float)(1.0 / 1.03)) return -1;  // float32(1/1.03), as NumPy casts the Python float
  return 0;
}

// NumPy float32 add.reduce of a contiguous array: 0 + pairwise_sum (oracle.sampler.pairwise_sum32)
__device__ float pairwise_sum32(const float* a, int n) {
  // iterative form of the recursion: the recursion only splits when n > 128
  if (n < 8) {
    float res = -0.0f;
    for (int i = 0; i < n; ++i) res = add_rn(res, a[i]);
    return res;
  }
  if (n <= 128) {
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] = add_rn(r[j], a[i + j]);
    float res = add_rn(add_rn(r[0], r[1]), add_rn(r[2], r[3]));
    res = add_rn(res, add_rn(add_rn(r[4], r[5]), add_rn(r[6], r[7])));
    for (; i < n; ++i) res = add_rn(res, a[i]);
    return res;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return add_rn(pairwise_sum32(a, n2), pairwise_sum32(a + n2, n - n2));
}

__device__ float pairwise_sum32_top(const float* a, int n) {
  return add_rn(0.0f, pairwise_sum32(a, n));
}

struct RankParams {
  const float* gt;
  const int* valid_idx;
  const int* nvalid;
  const float* gt_minmax;
  const int* draws;
  int B, H, W, L, n_cand, R_out, strategy;
  float* cand;     // [B][n_cand][L][2]
  double* score;   // [B][n_cand]
  float* out;      // [B][R_out][L][2]
};

template <int LMAX>
__global__ __launch_bounds__(256) void candidate_kernel(RankParams p) {
  const long total = (long)p.B * p.n_cand;
  const int L = p.L;
  const int HW = p.H * p.W;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int b = (int)(e / p.n_cand);
    const int* dr = p.draws + e * L;
    const int* vi = p.valid_idx + (long)b * HW;
    const float* gb = p.gt + (long)b * HW;
    const int nv = p.nvalid[b];
    float g[LMAX];
    int id[LMAX];
    for (int j = 0; j < L; ++j) {
      if (nv <= 0) {  // empty mask: nothing was compacted; a defined, all-invalid list (label
        id[j] = 0;    // -1: ListMLE's validity mask), never a read of the unwritten valid_idx
        g[j] = -1.0f;
        continue;
      }
      int d = dr[j];
      d = min(max(d, 0), nv - 1);
      const int pos = vi[d];
      id[j] = pos;
      g[j] = gb[pos];
    }
    // stable ascending insertion sort by g (then read reversed: descending, ties later-first)
    for (int i = 1; i < L; ++i) {
      const float kg = g[i];
      const int kid = id[i];
      int j = i - 1;
      while (j >= 0 && g[j] > kg) {
        g[j + 1] = g[j];
        id[j + 1] = id[j];
        --j;
      }
      g[j + 1] = kg;
      id[j + 1] = kid;
    }
    // descending copy in place (reverse)
    for (int i = 0, j = L - 1; i < j; ++i, --j) {
      const float tg = g[i]; g[i] = g[j]; g[j] = tg;
      const int ti = id[i]; id[i] = id[j]; id[j] = ti;
    }
    float* c = p.cand + e * L * 2;
    for (int j = 0; j < L; ++j) {
      c[2 * j] = (float)id[j];
      c[2 * j + 1] = g[j];
    }
    double sc = 0.0;
    if (p.strategy == PLD_SAMPLER_MASKED || p.strategy == PLD_SAMPLER_THRESH) {
      float acc = 0.0f;
      for (int j = 0; j + 1 < L; ++j) {
        if (p.strategy == PLD_SAMPLER_THRESH && depth_relation32(g[j], g[j + 1]) == 0)
          acc = add_rn(acc, -1000.0f);
        acc = add_rn(acc, fabsf(__fsub_rn(g[j], g[j + 1])));
      }
      sc = (double)acc;
    } else if (p.strategy == PLD_SAMPLER_INFO) {
      // expected = np.linspace(min+0.001, max, L+1)[1:] in float32
      const float start = add_rn(p.gt_minmax[2 * b], 0.001f);
      const float stop = p.gt_minmax[2 * b + 1];
      const float delta = __fsub_rn(stop, start);
      const float stepv = __fdiv_rn(delta, (float)L);
      float t[LMAX];
      for (int j = 0; j < L; ++j) {
        const float ev = (j == L - 1) ? stop : add_rn(mul_rn((float)(j + 1), stepv), start);
        const float d = __fsub_rn(g[j], ev);
        t[j] = __fdiv_rn(mul_rn(d, d), ev);
      }
      sc = -(double)pairwise_sum32_top(t, L);
      for (int j = 0; j + 1 < L; ++j)
        if (depth_relation32(g[j], g[j + 1]) == 0) sc = __dadd_rn(sc, -1000.0);
    }
    p.score[e] = sc;
  }
}

// 8 < L <= 64: one wavefront per candidate list, lane j holding draw j. The sort is a rank
// computation — position of j = #{k : g_k > g_j} + #{k : g_k == g_j, k > j}, exactly the
// stable-ascending-then-reversed order of candidate_kernel — and ds_permute moves each element to
// the lane of its position. Scores use the same fp32/fp64 operation order as candidate_kernel
// (NumPy's 8-accumulator pairwise sum for 8 <= L <= 128), computed redundantly by every lane.
__global__ __launch_bounds__(256) void candidate_wave_kernel(RankParams p) {
  const int lane = threadIdx.x & 63;
  const long total = (long)p.B * p.n_cand;
  const int L = p.L;
  const int HW = p.H * p.W;
  for (long e = (long)blockIdx.x * 4 + (threadIdx.x >> 6); e < total; e += (long)gridDim.x * 4) {
    const int b = (int)(e / p.n_cand);
    float g = 0.0f;
    int id = 0;
    if (lane < L) {
      const int nv = p.nvalid[b];
      if (nv > 0) {
        int d = p.draws[e * L + lane];
        d = min(max(d, 0), nv - 1);
        id = p.valid_idx[(long)b * HW + d];
        g = p.gt[(long)b * HW + id];
      } else {  // empty mask: defined all-invalid list (see candidate_kernel)
        g = -1.0f;
      }
    }
    int rank = 0;
    for (int k = 0; k < L; ++k) {  // wave-uniform trip count: every lane takes part in the shfl
      const float gk = __shfl(g, k, 64);
      rank += (gk > g) | ((gk == g) & (k > lane));
    }
    if (lane >= L) rank = lane;  // idle lanes keep their slot: the permutation stays 1:1
    const float gs = __int_as_float(__builtin_amdgcn_ds_permute(rank << 2, __float_as_int(g)));
    const int ids = __builtin_amdgcn_ds_permute(rank << 2, id);
    if (lane < L)
      reinterpret_cast<float2*>(p.cand + e * L * 2)[lane] = make_float2((float)ids, gs);
    double sc = 0.0;
    if (p.strategy == PLD_SAMPLER_MASKED || p.strategy == PLD_SAMPLER_THRESH) {
      float acc = 0.0f;
      float gj = __shfl(gs, 0, 64);
      for (int j = 0; j + 1 < L; ++j) {
        const float gj1 = __shfl(gs, j + 1, 64);
        if (p.strategy == PLD_SAMPLER_THRESH && depth_relation32(gj, gj1) == 0)
          acc = add_rn(acc, -1000.0f);
        acc = add_rn(acc, fabsf(__fsub_rn(gj, gj1)));
        gj = gj1;
      }
      sc = (double)acc;
    } else if (p.strategy == PLD_SAMPLER_INFO) {
      const float start = add_rn(p.gt_minmax[2 * b], 0.001f);
      const float stop = p.gt_minmax[2 * b + 1];
      const float stepv = __fdiv_rn(__fsub_rn(stop, start), (float)L);
      const float ev =
          (lane == L - 1) ? stop : add_rn(mul_rn((float)(lane + 1), stepv), start);
      const float dd = __fsub_rn(gs, ev);
      const float t = __fdiv_rn(mul_rn(dd, dd), ev);
      // pairwise_sum32, 8 <= n <= 128 branch
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = __shfl(t, j, 64);
      const int nfull = L - (L % 8);
      int i = 8;
      for (; i < nfull; i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = add_rn(r[j], __shfl(t, i + j, 64));
      float res = add_rn(add_rn(r[0], r[1]), add_rn(r[2], r[3]));
      res = add_rn(res, add_rn(add_rn(r[4], r[5]), add_rn(r[6], r[7])));
      for (; i < L; ++i) res = add_rn(res, __shfl(t, i, 64));
      sc = -(double)add_rn(0.0f, res);
      const float gn = __shfl(gs, min(lane + 1, 63), 64);
      const int nz = __popcll(__ballot(lane + 1 < L && depth_relation32(gs, gn) == 0));
      for (int k = 0; k < nz; ++k) sc = __dadd_rn(sc, -1000.0);
    }
    if (lane == 0) p.score[e] = sc;
  }
}

// per-image top-R, spread over (B, n / 256) workgroups: every workgroup stages the image's n
// scores in LDS and ranks 256 candidates against them, then copies the selected lists with all
// threads (coalesced). Same rank definition as select_kernel.
__global__ __launch_bounds__(256) void select_chunk_kernel(RankParams p) {
  extern __shared__ double s_score[];
  __shared__ int s_rank[256];
  const int b = blockIdx.x;
  const int n = p.n_cand;
  const double* sb = p.score + (long)b * n;
  for (int i = threadIdx.x; i < n; i += 256) s_score[i] = sb[i];
  __syncthreads();
  const int i = blockIdx.y * 256 + threadIdx.x;
  int rank = n;
  if (i < n) {
    const double si = s_score[i];
    int r0 = 0, r1 = 0;
    int j = 0;
    for (; j + 1 < n; j += 2) {
      const double s0 = s_score[j], s1 = s_score[j + 1];
      r0 += (s0 > si) | ((s0 == si) & (j > i));
      r1 += (s1 > si) | ((s1 == si) & (j + 1 > i));
    }
    if (j < n) r0 += (s_score[j] > si) | ((s_score[j] == si) & (j > i));
    rank = r0 + r1;
  }
  s_rank[threadIdx.x] = rank;
  __syncthreads();
  const int L2 = 2 * p.L;
  const int cnt = min(256, n - (int)blockIdx.y * 256);
  for (int q = threadIdx.x; q < cnt * L2; q += 256) {
    const int c = q / L2, k = q - c * L2;
    const int rk = s_rank[c];
    if (rk < p.R_out)
      p.out[((long)b * p.R_out + rk) * L2 + k] =
          p.cand[((long)b * n + blockIdx.y * 256 + c) * L2 + k];
  }
}

// per-image top-R: rank of candidate i = #{j : (score_j, j) > (score_i, i)} (lexicographic);
// the reference's argsort(scores)[::-1] order with ties broken toward the higher index
__global__ __launch_bounds__(1024) void select_kernel(RankParams p) {
  extern __shared__ double s_score[];
  const int b = blockIdx.x;
  const int n = p.n_cand;
  const double* sb = p.score + (long)b * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s_score[i] = sb[i];
  __syncthreads();
  const int L = p.L;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double si = s_score[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const double sj = s_score[j];
      rank += (sj > si) | ((sj == si) & (j > i));
    }
    if (rank < p.R_out) {
      const float* src = p.cand + ((long)b * n + i) * L * 2;
      float* dst = p.out + ((long)b * p.R_out + rank) * L * 2;
      for (int k = 0; k < 2 * L; ++k) dst[k] = src[k];
    }
  }
}

// pure strategy: the first floor(0.8R) candidates in draw order (no selection)
__global__ void copy_first_kernel(RankParams p) {
  const long per = (long)p.R_out * p.L * 2;
  const long total = (long)p.B * per;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const long b = e / per;
    const long r = e - b * per;
    p.out[e] = p.cand[b * (long)p.n_cand * p.L * 2 + r];
  }
}

static int factor_candidates(int R, int strategy) {
  switch (strategy) {
    case PLD_SAMPLER_PURE: return (int)(R * 0.8);
    case PLD_SAMPLER_MASKED:
    case PLD_SAMPLER_THRESH: return (int)(R * 1.5);
    case PLD_SAMPLER_INFO: return R * 5;
    default: return -1;
  }
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace pld

using namespace pld;

extern "C" int pld_sampler_candidates(int R, int strategy) { return factor_candidates(R, strategy); }

extern "C" size_t pld_sampler_workspace_size(int B, int H, int W, int R, int L, int strategy) {
  const int nc = factor_candidates(R, strategy);
  if (B <= 0 || nc <= 0 || L <= 0) return 0;
  return align_up(sizeof(float) * (size_t)B * nc * L * 2) + align_up(sizeof(double) * (size_t)B * nc);
}

extern "C" int pld_sampler_compact(const float* mask, int B, int H, int W, const float* gt,
                                   int* valid_idx, int* nvalid, float* gt_minmax, void* ws,
                                   void* stream) {
  PLD_CHECK_ARG(mask && valid_idx && nvalid && B > 0 && H > 0 && W > 0,
                "pld_sampler_compact: bad args");
  PLD_CHECK_ARG((long)H * W < (1 << 24), "pld_sampler_compact: H*W must stay below 2^24 "
                "(flat indices travel as float32)");
  const int HW = H * W;
  const int S = (int)cdiv(HW, COMPACT_SEG);
  PLD_CHECK_ARG(ws, "pld_sampler_compact: workspace required (pld_sampler_compact_workspace_size)");
  int* seg_cnt = (int*)ws;
  float* seg_mm = (float*)((char*)ws + align_up(sizeof(int) * (size_t)B * S));
  hipStream_t st = as_stream(stream);
  compact_count_kernel<<<dim3(S, B), COMPACT_THREADS, 0, st>>>(mask, HW, gt, S, seg_cnt, seg_mm);
  int rc = check_launch("compact_count_kernel");
  if (rc) return rc;
  compact_write_kernel<<<dim3(S, B), COMPACT_THREADS, 0, st>>>(mask, HW, S, seg_cnt, seg_mm,
                                                               valid_idx, nvalid, gt_minmax);
  return check_launch("compact_write_kernel");
}

extern "C" size_t pld_sampler_compact_workspace_size(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  const size_t S = cdiv((long)H * W, COMPACT_SEG);
  return align_up(sizeof(int) * B * S) + align_up(2 * sizeof(float) * B * S);
}

extern "C" int pld_sampler_draw(const int* nvalid, int B, int n_cand, int L, uint64_t seed,
                                uint64_t step, int image_offset, int* draws, void* stream) {
  PLD_CHECK_ARG(nvalid && draws && B > 0 && n_cand > 0 && L > 0, "pld_sampler_draw: bad args");
  const long total = (long)B * n_cand * L;
  draw_kernel<<<std::min<unsigned>(cdiv(total, 256), 4096), 256, 0, as_stream(stream)>>>(
      nvalid, B, n_cand * L, seed, step, nullptr, image_offset, draws);
  return check_launch("draw_kernel");
}

extern "C" int pld_sampler_draw_dev(const int* nvalid, int B, int n_cand, int L, uint64_t seed,
                                    const int64_t* step_dev, int image_offset, int* draws,
                                    void* stream) {
  PLD_CHECK_ARG(nvalid && draws && step_dev && B > 0 && n_cand > 0 && L > 0,
                "pld_sampler_draw_dev: bad args");
  const long total = (long)B * n_cand * L;
  draw_kernel<<<std::min<unsigned>(cdiv(total, 256), 4096), 256, 0, as_stream(stream)>>>(
      nvalid, B, n_cand * L, seed, 0, step_dev, image_offset, draws);
  return check_launch("draw_kernel");
}

extern "C" int pld_sampler_rank(const float* gt, const int* valid_idx, const int* nvalid,
                                const float* gt_minmax, const int* draws, int B, int H, int W,
                                int R, int L, int strategy, float* out, void* ws, void* stream) {
  PLD_CHECK_ARG(gt && valid_idx && nvalid && draws && out && ws && B > 0 && H > 0 && W > 0 &&
                    R > 0 && L > 0,
                "pld_sampler_rank: bad args");
  PLD_CHECK_ARG(L <= 512, "pld_sampler_rank: L=%d > 512", L);
  const int nc = factor_candidates(R, strategy);
  PLD_CHECK_ARG(nc > 0, "pld_sampler_rank: bad strategy %d", strategy);
  PLD_CHECK_ARG(strategy != PLD_SAMPLER_INFO || gt_minmax, "pld_sampler_rank: Info needs gt_minmax");
  RankParams p{};
  p.gt = gt;
  p.valid_idx = valid_idx;
  p.nvalid = nvalid;
  p.gt_minmax = gt_minmax;
  p.draws = draws;
  p.B = B; p.H = H; p.W = W; p.L = L;
  p.n_cand = nc;
  p.strategy = strategy;
  p.R_out = strategy == PLD_SAMPLER_PURE ? nc : R;
  p.cand = (float*)ws;
  p.score = (double*)((char*)ws + align_up(sizeof(float) * (size_t)B * nc * L * 2));
  p.out = out;
  hipStream_t st = as_stream(stream);
  const long total = (long)B * nc;
  const unsigned g = std::min<unsigned>(cdiv(total, 256), 8192);
  if (L <= 8) candidate_kernel<8><<<g, 256, 0, st>>>(p);
  else if (L <= 64)
    candidate_wave_kernel<<<std::min<unsigned>(cdiv(total, 4), 16384), 256, 0, st>>>(p);
  else candidate_kernel<512><<<g, 256, 0, st>>>(p);
  int rc = check_launch("candidate_kernel");
  if (rc) return rc;
  if (strategy == PLD_SAMPLER_PURE) {
    const long n = (long)B * p.R_out * L * 2;
    copy_first_kernel<<<std::min<unsigned>(cdiv(n, 256), 4096), 256, 0, st>>>(p);
    return check_launch("copy_first_kernel");
  }
  PLD_CHECK_ARG(sizeof(double) * (size_t)nc <= 150 * 1024,
                "pld_sampler_rank: %d candidates exceed the LDS selection buffer", nc);
  if (nc <= 1024) {
    select_kernel<<<B, 1024, sizeof(double) * nc, st>>>(p);
    return check_launch("select_kernel");
  }
  select_chunk_kernel<<<dim3(B, cdiv(nc, 256)), 256, sizeof(double) * nc, st>>>(p);
  return check_launch("select_chunk_kernel");
}

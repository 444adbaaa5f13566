// The bf16x3 implicit-GEMM tile kernel with LDS-DMA operand staging (FWD view: forward convs and
// dgrads). Round 5.
//
// Why (profiles/r05_x3_ablation.txt): conv_x3_kernel's producer waves — global loads into
// registers, the hi/lo split, the LDS stores — set its speed: with its MFMAs removed the dec1
// dgrad still takes 70 % of its time, with its loads removed 65 %. Here no wave stages through
// registers at all: every wave issues buffer_load ... lds (LDS-DMA) for its share of the next
// K-steps' A rows (fp32, full 128-byte lines) and B rows (the pre-split filter, bf16 hi / lo
// planes) into an S-slot LDS ring, S - 1 K-steps ahead of the MFMAs, and then computes: it reads
// its A fragments as fp32, splits them to bf16 hi / lo in registers between MFMAs, reads its B
// fragments as they are and issues the three products per pair (a_lo b_hi + a_hi b_lo + a_hi
// b_hi, fp32 accumulation: the same arithmetic as conv_x3_kernel, bit for bit).
//
// Synchronisation: one raw s_barrier per K-step. Before it each wave waits (counted vmcnt) for its
// own DMAs of the step about to be computed; after it, the slot read in the previous step is free
// and the wave issues the DMAs of step i + S - 1 into it. The last steps re-fetch the final step
// (a harmless copy into a free slot), so every iteration issues the same number of DMAs and the
// counted wait stays exact.
//
// LDS images (one slot): A [BM rows][8 x 16-byte chunks] fp32, chunk c of row r in slot
// c ^ ((r >> 1) & 7) (conflict-free for the fragment reads: each 16-lane group of a ds_read_b128
// reads 16 rows of one chunk); B hi / lo planes [BN rows][4 x 16-byte chunks] as conv_x3_kernel's
// (chunk_off). A DMA writes 1 KiB lane-linearly (8 A rows or 16 B rows): the swizzle goes on the
// per-lane SOURCE address.
#include "conv_x3_core.h"

namespace pld {
namespace x3 {

// One LDS-DMA wave-instruction: 16 bytes per lane from the buffer at byte offset `off` (OOB:
// zeros) to LDS [lds, lds + 1 KiB), lane-linear. Written as inline asm, not the builtin: for the
// builtin hipcc cannot tell the DMA's LDS bytes from the ones the fragment reads touch and waits
// vmcnt(0) before every ds_read, draining the whole ring each K-step. The waits are ours
// (wait_vm); M0 (the LDS base) is set and restored inside the statement.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned off) {
  const unsigned dst = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(r), "s"(__builtin_amdgcn_readfirstlane(dst))
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int WM, int WN, bool CAT, bool TI, int S, bool PC>
__global__ __launch_bounds__(WM * WN * 64 * (PC ? 2 : 1)) void conv_x3_dma_kernel(GemmConvParams p) {
  // PC: 4 more waves (4-7) only issue the DMAs; waves 0-3 only compute
  constexpr int NW = WM * WN;
  static_assert(NW == 4, "4 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  constexpr int A_BYTES = BM * 128, B_PLANE = BN * 64, SLOT = A_BYTES + 2 * B_PLANE;
  constexpr int GA = BM / 8 / NW;   // A DMAs per wave per K-step (8 rows each)
  constexpr int GB = BN / 8 / NW;   // B DMAs per wave per K-step (16 rows of one plane each)
  static_assert(GA >= 1 && GB >= 1 && (BM / 8) % NW == 0 && (BN / 8) % NW == 0, "DMA split");
  constexpr int G = GA + GB;
  static_assert(G * (S - 2 > 0 ? S - 2 : 0) <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) unsigned char smem[S * SLOT];

  const int wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = !PC || wave_id >= NW, computer = !PC || wave_id < NW;
  const int wave = PC ? wave_id % NW : wave_id;
  const int lane = threadIdx.x & 63;
  const int nmb = gridDim.x, nnb = gridDim.y;
  const int nwg = nmb * nnb * gridDim.z;
  const int wid = xcd_order(blockIdx.x + nmb * (blockIdx.y + nnb * blockIdx.z), nwg);
  const int nb = wid % nnb;
  const int mb = (wid / nnb) % nmb;
  const int zb = wid / (nnb * nmb);
  int kt_begin = 0, kt_end = p.kc_tap ? p.kc_tap * p.kh * p.kw : (p.K + BK - 1) / BK;
  if (p.ktiles_per_split > 0) {
    kt_begin = zb * p.ktiles_per_split;
    kt_end = min(kt_end, kt_begin + p.ktiles_per_split);
  }
  const int n_steps = kt_end - kt_begin;

  // ---- DMA source state. A: instruction i of this wave covers rows (wave GA + i) 8 + lane/8,
  // physical 16-byte slot lane % 8, i.e. logical chunk ca[i] (4 consecutive k) of that row.
  const int m0 = mb * BM, n0 = nb * BN;
  const int img_base = (int)p.dOH.div(p.dOW.div((uint32_t)m0));
  const long img_elems = (long)p.h * p.w;
  const __amdgpu_buffer_rsrc_t rs1 =
      make_rsrc(p.x1 + img_base * img_elems * p.c1, (p.n - img_base) * img_elems * p.c1 * 4);
  const __amdgpu_buffer_rsrc_t rs2 =
      CAT ? make_rsrc(p.x2 + img_base * img_elems * p.c2, (p.n - img_base) * img_elems * p.c2 * 4)
          : rs1;
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.bsplit, (long)p.N * p.K * 4);
  int a_base[GA], a_chunk[GA];
  unsigned a_taps[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = (wave * GA + i) * 8 + (lane >> 3);
    a_chunk[i] = (lane & 7) ^ ((r >> 1) & 7);
    const int m = m0 + r;
    const bool mok = m < p.M;
    const int mm = mok ? m : m0;
    const uint32_t q = p.dOW.div((uint32_t)mm);
    const int ox = mm - (int)q * p.ow;
    const uint32_t img = p.dOH.div(q);
    const int oy = (int)q - (int)img * p.oh;
    const int iy0 = oy * p.sh - p.pt, ix0 = ox * p.sw - p.pl;
    a_base[i] = (((int)img - img_base) * p.h + iy0) * p.w + ix0;
    unsigned t = 0;
    for (int ty = 0; ty < p.kh; ++ty)
      for (int tx = 0; tx < p.kw; ++tx)
        t |= (unsigned)(mok && (unsigned)(iy0 + ty) < (unsigned)p.h &&
                        (unsigned)(ix0 + tx) < (unsigned)p.w) << (ty * p.kw + tx);
    a_taps[i] = t;
  }
  // B: instruction j covers plane pl = jj / (BN/16), rows 16 (jj % (BN/16)) + lane/4 (jj = wave
  // GB + j), physical slot lane % 4 -> logical chunk (8 k) b_chunk[j]
  unsigned b_off[GB];
  bool b_ok[GB];
  int b_lds[GB], b_c8[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int jj = wave * GB + j;
    const int plane = jj / (BN / 16);
    const int r = 16 * (jj % (BN / 16)) + (lane >> 2);
    const int g = (((r >> 1) ^ (r >> 3)) & 1) | ((r >> 1) & 2);  // chunk_off's swizzle
    const int c = (lane & 3) ^ g;
    const int nn = n0 + r;
    b_ok[j] = nn < p.N;
    b_off[j] = (unsigned)(b_ok[j] ? nn : 0) * (unsigned)p.K * 4u + 32u * c + 16u * plane;
    b_lds[j] = A_BYTES + plane * B_PLANE + 16 * (jj % (BN / 16)) * 64;
    b_c8[j] = 8 * c;
  }

  // issue the DMAs of K-step kt (global index) into ring slot `slot`
  auto issue = [&](int kt, int slot) {
    unsigned char* base = smem + slot * SLOT;
    if constexpr (TI) {
      const int kq = (int)p.dTaps.div((uint32_t)kt);
      const int tap = kt - kq * p.kh * p.kw;
      const bool s2 = CAT && kq >= p.kc1;
      const int chb = (s2 ? kq - p.kc1 : kq) * BK;
      const int cs = s2 ? p.c2 : p.c1;
      const __amdgpu_buffer_rsrc_t rs = s2 ? rs2 : rs1;
      const int ty = (int)p.dKW.div((uint32_t)tap);
      const int toff = ty * p.w + (tap - ty * p.kw);
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int c = chb + 4 * a_chunk[i];
        const bool ok = c < cs && ((a_taps[i] >> tap) & 1u);
        dma16(rs, base + (wave * GA + i) * 1024, ok ? (unsigned)(((a_base[i] + toff) * cs + c) * 4)
                                                    : OOB);
      }
      const int kc = tap * p.C + (s2 ? p.c1 : 0) + chb;  // the step's first filter column
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const bool kcin = chb + b_c8[j] < cs;  // this lane's 8-k chunk inside the source
        dma16(rsb, base + b_lds[j], (b_ok[j] && kcin) ? b_off[j] + 4u * (unsigned)kc : OOB);
      }
    } else {
      const int k0 = kt * BK;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int k = k0 + 4 * a_chunk[i];
        const bool kin = k < p.K;
        const int kk = kin ? k : 0;
        const int tap = (int)p.dC.div((uint32_t)kk);
        const int ci = kk - tap * p.C;
        const int ty = (int)p.dKW.div((uint32_t)tap);
        const int toff = ty * p.w + (tap - ty * p.kw);
        const bool ok = kin && ((a_taps[i] >> tap) & 1u);
        dma16(rs1, base + (wave * GA + i) * 1024,
              ok ? (unsigned)(((a_base[i] + toff) * p.c1 + ci) * 4) : OOB);
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const bool kcin = k0 + b_c8[j] < p.K;
        dma16(rsb, base + b_lds[j], (b_ok[j] && kcin) ? b_off[j] + 4u * (unsigned)k0 : OOB);
      }
    }
  };

  // ---- compute state
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, l32 = lane & 31;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  auto compute = [&](int slot) {
    const unsigned char* A = smem + slot * SLOT;
    const unsigned char* B = A + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int r = wn * WTN + b * 32 + l32;
        bh[b] = lds_frag(B, r, 2 * s + h);
        bl[b] = lds_frag(B + B_PLANE, r, 2 * s + h);
      }
      float4 v[TM][2];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int r = wm * WTM + a * 32 + l32;
        const int sw = (r >> 1) & 7, c0 = 4 * s + 2 * h;
        v[a][0] = *reinterpret_cast<const float4*>(A + r * 128 + 16 * (c0 ^ sw));
        v[a][1] = *reinterpret_cast<const float4*>(A + r * 128 + 16 * ((c0 + 1) ^ sw));
      }
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        unsigned hi[4], lo[4];
        split2(v[a][0].x, v[a][0].y, hi[0], lo[0]);
        split2(v[a][0].z, v[a][0].w, hi[1], lo[1]);
        split2(v[a][1].x, v[a][1].y, hi[2], lo[2]);
        split2(v[a][1].z, v[a][1].w, hi[3], lo[3]);
        ah[a] = __builtin_bit_cast(bf16x8, u32x4{hi[0], hi[1], hi[2], hi[3]});
        al[a] = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], lo[2], lo[3]});
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    }
  };

  if (n_steps > 0) {
    const int last = kt_end - 1;
    if (loader) {
#pragma unroll
      for (int j = 0; j < S - 1; ++j) issue(min(kt_begin + j, last), j);
    }
    for (int i = 0; i < n_steps; ++i) {
      // this wave's DMAs of step i have landed (the S - 2 later steps may stay in flight); the
      // barrier publishes every wave's, and every wave is done reading step i - 1's slot
      if (loader) wait_vm<G * (S - 2)>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (loader) issue(min(kt_begin + i + S - 1, last), (i + S - 1) % S);
      if (computer) compute(i % S);
    }
  }
  // drain the re-fetch DMAs before the epilogue reuses the ring
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (!computer) return;
  const int m_w = m0 + wm * WTM, n_w = n0 + wn * WTN;
  if constexpr (4 * 32 * (WTN + 8) * 4 <= S * SLOT) {
    if (staged_ok(p)) {
      if (p.stats) acc_stats<TM, TN>(p, acc, m_w, n_w, lane);
      store_acc_staged<TM, TN>(p, acc, m_w, n_w, lane,
                               reinterpret_cast<float*>(smem) + wave * 32 * (WTN + 8));
      return;
    }
  }
  store_acc<TM, TN>(p, acc, m_w, n_w, lane, zb);
}

// ring depth per tile: the deepest ring (<= 4 slots) that fits 160 KiB with one workgroup per
// CU, or 2 slots (two workgroups per CU) when `two_per_cu` and a slot fits 40 KiB
template <int BM, int BN, int WM, int WN, int S, bool PC>
static void launch_dma_s(GemmConvParams& p, int splits, hipStream_t st) {
  dim3 grid(cdiv(p.M, BM), cdiv(p.N, BN), splits);
  const int T = PC ? 512 : 256;
  if (p.kc_tap) {
    if (p.c2) conv_x3_dma_kernel<BM, BN, WM, WN, true, true, S, PC><<<grid, T, 0, st>>>(p);
    else conv_x3_dma_kernel<BM, BN, WM, WN, false, true, S, PC><<<grid, T, 0, st>>>(p);
  } else {
    conv_x3_dma_kernel<BM, BN, WM, WN, false, false, S, PC><<<grid, T, 0, st>>>(p);
  }
}

template <int BM, int BN, int WM, int WN>
static void launch_dma(GemmConvParams& p, int splits, int depth, hipStream_t st) {
  // depth: ring slots; + 10: the producer/consumer form (4 loader + 4 compute waves)
  constexpr int SLOT = BM * 128 + BN * 128;
  constexpr int SMAX = (160 * 1024) / SLOT > 4 ? 4 : (160 * 1024) / SLOT;
  if (depth >= 10) {
    if constexpr (SMAX >= 3) {
      if (depth >= 13) return launch_dma_s<BM, BN, WM, WN, 3, true>(p, splits, st);
    }
    return launch_dma_s<BM, BN, WM, WN, 2, true>(p, splits, st);
  }
  if constexpr (SMAX >= 3) {
    if (depth >= 3) return launch_dma_s<BM, BN, WM, WN, 3, false>(p, splits, st);
  }
  launch_dma_s<BM, BN, WM, WN, 2, false>(p, splits, st);
}

// host side: the DMA kernel serves a grid schedule of the FWD view when the A operand can be
// fetched per 16-byte chunk by a wave-uniform descriptor (tap-inner order, or one source), the
// filter is pre-split and there is no input prologue. depth = ring slots (2..4).
bool dma_fwd_ok(const GemmConvParams& p) {
  return p.bsplit && !p.in_scale && (p.kc_tap || !p.c2) && p.K % 8 == 0 &&
         (p.kc_tap || p.C % 4 == 0);
}

void launch_fwd_dma(GemmConvParams& p, int splits, int cfg, int depth, hipStream_t st) {
  if (cfg == 3) launch_dma<128, 128, 2, 2>(p, splits, depth, st);
  else if (cfg == 9) launch_dma<128, 256, 2, 2>(p, splits, depth, st);
  else launch_fwd_grid(p, splits, cfg, st);
}

}  // namespace x3
}  // namespace pld

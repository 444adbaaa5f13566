// AddressSanitizer run of the C ABI's HOST code (SURVEY.md §5 "race detection / sanitizers"):
// every source of libpldepth_hip.so compiled host-only with -fsanitize=address (tools/asan/
// Makefile) and linked into this driver, which sweeps the entry points that run no kernel — the
// dispatch planners (workspace sizes, kernel family / name, schedule classes over every conv
// shape class the engines use, every schedule index and out-of-range ones), the fused-kernel
// eligibility helpers — and the argument checks of the compute entries (NULL / inconsistent
// arguments must come back as PLD_ERR_ARG with a message, before any device work). No GPU is
// needed; kernels are never launched. Exit 0 and "asan host check OK" on success.
#include <cstdio>
#include <cstring>
#include <vector>

#include "pldepth_hip.h"

extern "C" int pld__thin_ok(int K, int N);
extern "C" int pld__wide_ok(int K, int N);
extern "C" int pld__wide_stats_parts(long M, int K, int N);
extern "C" int pld__dw_tiled_ok(int k, int s, int c);

static int failures = 0;
#define EXPECT(cond)                                                       \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

struct Shape {
  int n, h, w, c1, c2, k, s, cout;
};

static pld_conv_args make(const Shape& sh, int math, int tile) {
  pld_conv_args a;
  std::memset(&a, 0, sizeof(a));
  static float dummy[16] __attribute__((aligned(16)));
  a.x1 = dummy;
  a.x2 = sh.c2 ? dummy : nullptr;
  a.c1 = sh.c1;
  a.c2 = sh.c2;
  a.n = sh.n;
  a.h = sh.h;
  a.w = sh.w;
  a.kh = a.kw = sh.k;
  a.sh = a.sw = sh.s;
  a.oh = (sh.h + sh.s - 1) / sh.s;
  a.ow = (sh.w + sh.s - 1) / sh.s;
  const int ph = (a.oh - 1) * sh.s + sh.k - sh.h;
  a.pad_t = ph > 0 ? ph / 2 : 0;
  a.pad_l = ph > 0 ? ph / 2 : 0;
  a.cout = sh.cout;
  a.tile = tile;
  a.math = math;
  return a;
}

int main() {
  EXPECT(pld_version() > 0);
  EXPECT(pld_last_error() != nullptr);

  // conv shape classes of ff_effnet / ff_redweb at 448^2 batch 32 and the unit-test sizes
  const std::vector<Shape> shapes = {
      {32, 448, 448, 3, 0, 3, 2, 32},     {32, 224, 224, 32, 0, 1, 1, 16},
      {32, 224, 224, 16, 0, 1, 1, 96},    {32, 112, 112, 24, 0, 1, 1, 144},
      {32, 56, 56, 40, 0, 1, 1, 240},     {32, 28, 28, 80, 0, 1, 1, 480},
      {32, 28, 28, 112, 0, 1, 1, 672},    {32, 14, 14, 192, 0, 1, 1, 1152},
      {32, 14, 14, 320, 0, 1, 1, 1280},   {32, 14, 14, 1280, 672, 3, 1, 672},
      {32, 28, 28, 672, 240, 3, 1, 240},  {32, 56, 56, 240, 144, 3, 1, 144},
      {32, 112, 112, 144, 32, 3, 1, 32},  {32, 224, 224, 32, 0, 3, 1, 1},
      {2, 64, 64, 3, 0, 7, 2, 64},        {2, 32, 32, 64, 0, 1, 2, 256},
      {2, 17, 9, 12, 0, 3, 1, 20},        {1, 5, 6, 48, 0, 1, 1, 64},
      {3, 7, 9, 80, 0, 1, 1, 480},        {1, 6, 5, 8, 0, 1, 1, 520},
  };
  for (int math = 0; math < 2; ++math) {
    const int ns = pld_conv_num_schedules(math);
    EXPECT(ns > 0);
    EXPECT(pld_conv_schedule_class(math, -1) == -1);
    EXPECT(pld_conv_schedule_class(math, ns) == -1);
    for (int i = 0; i < ns; ++i) EXPECT(pld_conv_schedule_class(math, i) >= 0);
    for (const Shape& sh : shapes)
      for (int tile = -1; tile <= ns + 1; ++tile) {
        pld_conv_args a = make(sh, math, tile);
        for (int mode = 0; mode < 3; ++mode) {
          const int kind = pld_conv_kernel_kind(&a, mode);
          const char* name = pld_conv_kernel_name(&a, mode);
          EXPECT(name != nullptr);
          EXPECT(kind < 0 || std::strlen(name) > 0);
        }
        (void)pld_conv2d_fwd_workspace_size(&a);
        (void)pld_conv2d_dgrad_workspace_size(&a);
        (void)pld_conv2d_wgrad_workspace_size(&a);
        (void)pld_conv2d_fwd_bn_stats_workspace_size(&a);
      }
  }
  EXPECT(pld_conv_kernel_kind(nullptr, 0) < 0);
  EXPECT(pld_conv2d_fwd_workspace_size(nullptr) == 0);

  for (int K = 0; K <= 256; K += 4)
    for (int N = 1; N <= 1400; N += 37) {
      (void)pld__thin_ok(K, N);
      if (pld__wide_ok(K, N)) EXPECT(pld__wide_stats_parts(401408, K, N) >= 1);
      (void)pld_pgemm_ok(K, N);
    }
  for (int k = 1; k <= 7; k += 2)
    for (int s = 1; s <= 2; ++s)
      for (int c = 1; c <= 1152; c += 13) {
        (void)pld__dw_tiled_ok(k, s, c);
        EXPECT(pld_dwconv_fwd_bn_stats_workspace_size(32, 112, 112, c, s) > 0);
      }
  for (int c = 1; c <= 1280; c += 31) {
    EXPECT(pld_channel_reduce_workspace_size(401408, c) > 0);
    (void)pld_se_workspace_size(32, 3136, c, 10);
    (void)pld_se_bwd_bn_full_workspace_size(32, 3136, c, 10);
    (void)pld_upconv_bwd_workspace_size(c);
    (void)pld_upconv_wgrad_workspace_size(c);
  }
  for (int strat = 0; strat < 4; ++strat)
    (void)pld_sampler_workspace_size(32, 448, 448, 100, 5, strat);

  // argument checks: rejected before any device work
  pld_conv_args a = make(shapes[3], 1, -1);
  EXPECT(pld_conv2d_fwd(&a, nullptr, nullptr, nullptr, 0, nullptr) != 0);
  EXPECT(pld_conv2d_dgrad(nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr) != 0);
  EXPECT(pld_conv2d_fwd_bn_stats(&a, nullptr, nullptr, nullptr, 1e-3f, 0.99f, nullptr, nullptr,
                                 nullptr, nullptr, nullptr, 0, nullptr) != 0);
  EXPECT(pld_filter_refresh(nullptr, 3, 3, 8, 8, nullptr, nullptr, nullptr, nullptr,
                            nullptr) != 0);
  EXPECT(pld_filter_split(nullptr, 4, 12, nullptr, nullptr) != 0);
  EXPECT(std::strlen(pld_last_error()) > 0);

  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("asan host check OK\n");
  return 0;
}

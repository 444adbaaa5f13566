// Instantiations of the bf16x3 tile kernel for weight gradients (conv_x3_core.h): tile grid
// (with split-K) and tile stream.
#include "conv_x3_core.h"

namespace pld {
namespace x3 {

void launch_wgrad_grid(GemmConvParams& p, int splits, int cfg, hipStream_t st) {
#define PLD_CALL(BM, BN, WM, WN) launch_cfg_grid<MODE_WGRAD, BM, BN, WM, WN>(p, splits, st)
  PLD_X3_DISPATCH(cfg, PLD_CALL)
#undef PLD_CALL
}

void launch_wgrad_stream(GemmConvParams& p, int cfg, int sk_grid, hipStream_t st) {
#define PLD_CALL(BM, BN, WM, WN) launch_cfg_stream<MODE_WGRAD, BM, BN, WM, WN>(p, sk_grid, st)
  PLD_X3_DISPATCH(cfg, PLD_CALL)
#undef PLD_CALL
}

}  // namespace x3
}  // namespace pld

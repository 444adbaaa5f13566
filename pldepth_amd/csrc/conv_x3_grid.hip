// Instantiations of the bf16x3 tile kernel on a tile grid (conv_x3_core.h): forward / dgrad.
#include "conv_x3_core.h"

namespace pld {
namespace x3 {

void launch_fwd_grid(GemmConvParams& p, int splits, int cfg, hipStream_t st) {
#define PLD_CALL(BM, BN, WM, WN) launch_cfg_grid<MODE_FWD, BM, BN, WM, WN>(p, splits, st)
  PLD_X3_DISPATCH(cfg, PLD_CALL)
#undef PLD_CALL
}

}  // namespace x3
}  // namespace pld

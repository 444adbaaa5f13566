// Instantiations of the bf16x3 tile kernel as a tile stream (conv_x3_core.h): forward / dgrad.
#include "conv_x3_core.h"

namespace pld {
namespace x3 {

void launch_fwd_stream(GemmConvParams& p, int cfg, int sk_grid, hipStream_t st) {
#define PLD_CALL(BM, BN, WM, WN) launch_cfg_stream<MODE_FWD, BM, BN, WM, WN>(p, sk_grid, st)
  PLD_X3_DISPATCH(cfg, PLD_CALL)
#undef PLD_CALL
}

}  // namespace x3
}  // namespace pld

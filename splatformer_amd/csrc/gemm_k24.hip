// gemm_kernel instantiations for operand mode MODE_GATHERS (multi-segment gathers, 64 x 128 tiles only: the
// test / reference path of sfx_linear with num_segments > 1)
#include "gemm_kernel.h"

namespace sfxg {

void launch_m2_w4(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st) {
  (void)cfg;
  launch<64, 128, 2, 4, MODE_GATHERS>(a, groups, vec, st);
}

}  // namespace sfxg

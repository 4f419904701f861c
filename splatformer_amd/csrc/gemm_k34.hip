// gemm_kernel instantiations for operand mode MODE_PAIR, 4-wave tiles (gemm.hip: dispatch_mode)
#include "gemm_kernel.h"

namespace sfxg {

void launch_m3_w4(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st) {
  constexpr int M = MODE_PAIR;
  switch (cfg) {
    case 0: launch<128, 128, 2, 4, M>(a, groups, vec, st); break;
    case 1: launch<128, 96, 4, 4, M>(a, groups, vec, st); break;
    case 2: launch<128, 64, 2, 4, M>(a, groups, vec, st); break;
    case 3: launch<64, 128, 2, 4, M>(a, groups, vec, st); break;
    default: launch<64, 64, 2, 4, M>(a, groups, vec, st); break;
  }
}

}  // namespace sfxg

// gemm_kernel instantiations for operand mode MODE_DENSE, 8-wave tiles (gemm.hip: dispatch_mode)
#include "gemm_kernel.h"

namespace sfxg {

void launch_m0_w8(int cfg, const GemmArgs& a, int groups, bool vec, hipStream_t st) {
  constexpr int M = MODE_DENSE;
  switch (cfg) {
    case 5: launch<256, 128, 4, 8, M>(a, groups, vec, st); break;
    default: launch<128, 256, 2, 8, M>(a, groups, vec, st); break;
  }
}

}  // namespace sfxg

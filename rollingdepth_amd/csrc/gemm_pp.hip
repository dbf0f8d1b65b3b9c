// 8-wave ping-pong GEMM engine (gemm_pp_kernel) instantiations; dispatch in gemm.hip.
#include "gemm_kernels.h"

namespace rdmi_gk {

template <int MODE>
static void pp_mode_launch(int wm, dim3 g, hipStream_t s, const GemmP& p) {
  if (wm == 4)
    hipLaunchKernelGGL((gemm_pp_kernel<MODE, 4, 4>), g, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_pp_kernel<MODE, 2, 4>), g, dim3(512), 0, s, p);
}

// dbg: the RDMI_GEMM_DBG diagnostic variants of the 256×256 dense tile (0 = the product kernels)
void launch_gemm_pp(int mode, int wm, int dbg, dim3 g, hipStream_t s, const GemmP& p) {
  if (dbg) {
    switch (dbg) {
      case 1: hipLaunchKernelGGL((gemm_pp_kernel<0, 2, 4, 1>), g, dim3(512), 0, s, p); return;
      case 5: hipLaunchKernelGGL((gemm_pp_kernel<0, 2, 4, 5>), g, dim3(512), 0, s, p); return;
      case 8: hipLaunchKernelGGL((gemm_pp_kernel<0, 2, 4, 8>), g, dim3(512), 0, s, p); return;
      default: hipLaunchKernelGGL((gemm_pp_kernel<0, 2, 4, 12>), g, dim3(512), 0, s, p); return;
    }
  }
  if (mode == 2)
    pp_mode_launch<2>(wm, g, s, p);
  else if (mode == 1)
    pp_mode_launch<1>(wm, g, s, p);
  else
    pp_mode_launch<0>(wm, g, s, p);
}

}  // namespace rdmi_gk

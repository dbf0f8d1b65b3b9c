// Classic 3-slot-ring implicit-GEMM engine (gemm_kernel) instantiations; dispatch in gemm.hip.
#include "gemm_kernels.h"

namespace rdmi_gk {

template <int MODE>
static void classic_mode(int bm, int bn, dim3 g, hipStream_t s, const GemmP& p) {
  if (bm == 256 && bn == 128)
    hipLaunchKernelGGL((gemm_kernel<256, 128, 4, 2, MODE>), g, dim3(512), 0, s, p);
  else if (bm == 128 && bn == 128)
    hipLaunchKernelGGL((gemm_kernel<128, 128, 2, 2, MODE>), g, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_kernel<256, 64, 8, 1, MODE>), g, dim3(512), 0, s, p);
}

void launch_gemm_classic(int mode, int bm, int bn, dim3 g, hipStream_t s, const GemmP& p) {
  if (mode == 2)
    classic_mode<2>(bm, bn, g, s, p);
  else if (mode == 1)
    classic_mode<1>(bm, bn, g, s, p);
  else
    classic_mode<0>(bm, bn, g, s, p);
}

}  // namespace rdmi_gk

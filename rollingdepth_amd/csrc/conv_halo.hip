// 8-wave halo conv (conv_halo_kernel) instantiations; dispatch in gemm.hip (rdmi_conv2d).
#include "gemm_kernels.h"

namespace rdmi_gk {

template <int MODE, int NPH, int WN>
static void halo_gn(bool gn, dim3 g, hipStream_t s, const GemmP& p) {
  if (gn)
    hipLaunchKernelGGL((conv_halo_kernel<MODE, NPH, WN, true>), g, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((conv_halo_kernel<MODE, NPH, WN, false>), g, dim3(512), 0, s, p);
}

// (mode, nph, wn): (1|2, 2, 4) and (1|2, 1, 2) with or without the GroupNorm input; (1|2, 4, 4)
// without
void launch_conv_halo(int mode, int nph, int wn, bool gn, dim3 g, hipStream_t s, const GemmP& p) {
  if (wn == 2) {
    if (mode == 2)
      halo_gn<2, 1, 2>(gn, g, s, p);
    else
      halo_gn<1, 1, 2>(gn, g, s, p);
  } else if (nph == 4) {
    if (mode == 2)
      hipLaunchKernelGGL((conv_halo_kernel<2, 4, 4, false>), g, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((conv_halo_kernel<1, 4, 4, false>), g, dim3(512), 0, s, p);
  } else {
    if (mode == 2)
      halo_gn<2, 2, 4>(gn, g, s, p);
    else
      halo_gn<1, 2, 4>(gn, g, s, p);
  }
}

}  // namespace rdmi_gk

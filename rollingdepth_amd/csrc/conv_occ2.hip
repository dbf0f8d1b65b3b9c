// Two-workgroups-per-CU engines: the 128-channel halo conv (conv_halo_occ2_kernel), its 32×32×16
// form (conv_halo32_kernel) and the dense GEMM (gemm_occ2_kernel); dispatch in gemm.hip.
#include "gemm_kernels.h"

namespace rdmi_gk {

template <int MODE>
static void occ2_mode_launch(bool gn, bool pipe, dim3 g, hipStream_t s, const GemmP& p) {
  if (gn && pipe)
    hipLaunchKernelGGL((conv_halo_occ2_kernel<MODE, true, true>), g, dim3(256), 0, s, p);
  else if (gn)
    hipLaunchKernelGGL((conv_halo_occ2_kernel<MODE, true, false>), g, dim3(256), 0, s, p);
  else if (pipe)
    hipLaunchKernelGGL((conv_halo_occ2_kernel<MODE, false, true>), g, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_halo_occ2_kernel<MODE, false, false>), g, dim3(256), 0, s, p);
}

void launch_conv_occ2(int mode, bool gn, bool pipe, dim3 g, hipStream_t s, const GemmP& p) {
  if (mode == 3) {  // phase-decomposed upsample (no GroupNorm input)
    if (pipe)
      hipLaunchKernelGGL((conv_halo_occ2_kernel<3, false, true>), g, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((conv_halo_occ2_kernel<3, false, false>), g, dim3(256), 0, s, p);
  } else if (mode == 2)
    occ2_mode_launch<2>(gn, pipe, g, s, p);
  else
    occ2_mode_launch<1>(gn, pipe, g, s, p);
}

void launch_conv_h32(bool gn, dim3 g, hipStream_t s, const GemmP& p) {
  if (gn)
    hipLaunchKernelGGL((conv_halo32_kernel<true>), g, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_halo32_kernel<false>), g, dim3(256), 0, s, p);
}

void launch_gemm_occ2(int bn, dim3 g, hipStream_t s, const GemmP& p) {
  // bn == 160 never carries GEGLU (launch_mode): its epilogue exists only for 64-column waves
  if (bn == 160 && !p.geglu)
    hipLaunchKernelGGL((gemm_occ2_kernel<0, 160>), g, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_occ2_kernel<0, 128>), g, dim3(256), 0, s, p);
}

}  // namespace rdmi_gk

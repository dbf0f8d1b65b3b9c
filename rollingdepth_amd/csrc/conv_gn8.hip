// conv_halo_gn8_kernel instantiations (the double-halo GroupNorm-input conv; dispatch in gemm.hip)
#include "gemm_kernels.h"

namespace rdmi_gk {

void launch_conv_gn8(bool silu, dim3 g, hipStream_t s, const GemmP& p) {
  if (silu)
    hipLaunchKernelGGL((conv_halo_gn8_kernel<true>), g, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_halo_gn8_kernel<false>), g, dim3(256), 0, s, p);
}

}  // namespace rdmi_gk

// Shared definitions for librdmi (RollingDepth snippet-denoise path on MI355X / gfx950).
// Conventions (include/rdmi.h): every entry point returns 0 or an RDMI_E_* / hipError_t code,
// never synchronises the device, never allocates, and records a thread-local message.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/rdmi.h"

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace rdmi {

void set_error(const char* fmt, ...);

// Check a launch; returns 0 or the HIP error code (message recorded).
int check_launch(const char* what);

inline int div_up(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace rdmi

#define RDMI_REQUIRE(cond, code, ...)       \
  do {                                       \
    if (!(cond)) {                           \
      rdmi::set_error(__VA_ARGS__);          \
      return (code);                         \
    }                                        \
  } while (0)

// x·σ(x) with the hardware exp2 and reciprocal (≈2 ulp f32; the f16 outputs it feeds round far
// coarser): 7 VALU ops instead of the ≈16 of an IEEE division.  exp2(+inf) = inf → rcp → 0 → −0
// for very negative x, as silu.
__device__ __forceinline__ float silu_f(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// GELU(erf) with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the f16 output's
// rounding): one rcp, one exp2 and 9 FMA-class ops, branch-free (ocml's erff branches per range).
__device__ __forceinline__ float gelu_erf_fast(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float pl = fmaf(1.061405429f, t, -1.453152027f);
  pl = fmaf(pl, t, 1.421413741f);
  pl = fmaf(pl, t, -0.284496736f);
  pl = fmaf(pl, t, 0.254829592f);
  pl *= t;
  const float e = __builtin_amdgcn_exp2f(-az * az * 1.4426950408889634f);
  const float erf_abs = fmaf(-pl, e, 1.0f);
  const float erf_z = __builtin_copysignf(erf_abs, z);
  return 0.5f * x * (1.0f + erf_z);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

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
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace rdmi {

void set_error(const char* fmt, ...);

// Check a launch; returns 0 or the HIP error code (message recorded).
int check_launch(const char* what);

// f32 engines behind rdmi_gemm / rdmi_conv2d (gemm_f32.hip), selected by args->dtype == RDMI_F32
int gemm_f32(const rdmi_gemm_args* a, void* stream);
int conv2d_f32(const rdmi_conv_args* a, void* stream);
// f32 flash attention behind rdmi_attention_fwd (attention_f32.hip)
int attention_fwd_f32(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk, long q_ld,
                      long k_ld, long v_ld, long o_ld, long q_bs, long k_bs, long v_bs, long o_bs, float scale,
                      int parts, void* stream);  // parts: 1 exact f32, 2 bf16x3, 3 bf16x6

inline int div_up(long a, long b) { return (int)((a + b - 1) / b); }

// XCD-aware remap (T1): dispatch id d runs on XCD d % 8; give each XCD a contiguous range of
// logical tiles so the n-tiles sharing one A row-panel share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int total) {
  if (total < 8) return bid;
  const int xcd = bid & 7, q = total >> 3, r = total & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// The same remap for a 3-D grid (attention: x = query block, y = head, z = batch), x fastest: the
// logical (x, y, z) of this workgroup.  Each XCD then runs consecutive query blocks of ONE (batch,
// head), so the K / V they all sweep is streamed into that XCD's L2 once instead of into every XCD's
// (in dispatch order the query blocks of a head are dealt round-robin to all 8 XCDs).
__device__ __forceinline__ void xcd_block3(int& x, int& y, int& z) {
  const int nx = gridDim.x, ny = gridDim.y;
  const int l = xcd_remap((blockIdx.z * ny + blockIdx.y) * nx + blockIdx.x, nx * ny * gridDim.z);
  x = l % nx;
  const int r = l / nx;
  y = r % ny;
  z = r / ny;
}

// logical tile → (m-tile, n-tile): groups of G m-tiles sweep all n-tiles with m fastest, so the
// tiles an XCD runs together share G A-panels and a few B-panels (L2 reuse in both operands)
__device__ __forceinline__ void tile_mn(int logical, int nbx, int nby, int G, int& mt, int& nt) {
  if (G <= 1) {
    mt = logical / nbx;
    nt = logical % nbx;
    return;
  }
  const int per = G * nbx;
  const int g = logical / per;
  const int first = g * G;
  const int gs = min(G, nby - first);
  const int r = logical - g * per;
  mt = first + r % gs;
  nt = r / gs;
}

// vmcnt(n) alone (gfx9 s_waitcnt encoding: vmcnt[3:0] | vmcnt[5:4]<<14, expcnt/lgkmcnt at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt_only() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}

// Two f32 values → their packed bf16 hi and lo parts (v_cvt_pk_bf16_f32, first operand in the low
// half; round-to-nearest-even both times): x = x_hi + x_lo + O(2^-18 |x|).  The f32 engines'
// bf16-split products (rdmi.h RDMI_F32_X3) are built from these.
__device__ __forceinline__ u32x2 split_bf16x2(float x0, float x1) {  // {hi, lo}
  unsigned hi, lo;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(hi) : "v"(x0), "v"(x1));
  const float r0 = x0 - __builtin_bit_cast(float, hi << 16), r1 = x1 - __builtin_bit_cast(float, hi & 0xffff0000u);
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(lo) : "v"(r0), "v"(r1));
  return u32x2{hi, lo};
}

// Two f32 values → packed bf16 hi, mid and lo parts (each remainder exact in f32, each part RNE):
// x = x_hi + x_mid + x_lo + O(2^-26 |x|) — the three-way split of the f32 engines' x6 products.
__device__ __forceinline__ void split3_bf16x2(float x0, float x1, unsigned& hi, unsigned& mid, unsigned& lo) {
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(hi) : "v"(x0), "v"(x1));
  const float r0 = x0 - __builtin_bit_cast(float, hi << 16), r1 = x1 - __builtin_bit_cast(float, hi & 0xffff0000u);
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(mid) : "v"(r0), "v"(r1));
  const float t0 = r0 - __builtin_bit_cast(float, mid << 16), t1 = r1 - __builtin_bit_cast(float, mid & 0xffff0000u);
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(lo) : "v"(t0), "v"(t1));
}

// 8 f32 values (a0 then a1) → bf16x8 hi and lo parts
__device__ __forceinline__ void split_bf16x8(const f32x4& a0, const f32x4& a1, bf16x8& hi, bf16x8& lo) {
  const u32x2 s0 = split_bf16x2(a0[0], a0[1]), s1 = split_bf16x2(a0[2], a0[3]);
  const u32x2 s2 = split_bf16x2(a1[0], a1[1]), s3 = split_bf16x2(a1[2], a1[3]);
  hi = __builtin_bit_cast(bf16x8, u32x4{s0[0], s1[0], s2[0], s3[0]});
  lo = __builtin_bit_cast(bf16x8, u32x4{s0[1], s1[1], s2[1], s3[1]});
}

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
// The polynomial's constant-addend steps as v_fmaak_f32 (the literal in the instruction; as fmaf,
// hipcc pre-loaded each constant with a v_mov for its accumulator form), and ½·x·(1 + erf) as
// x · fma(erf, ½, ½): ½·(1 + erf) rounds exactly as 1 + erf scaled by 2^-1, and ½·x is exact, so
// both forms round the same product — two ops instead of three.  Bitwise the previous GELU.
#define RDMI_FMAAK(a, b, k)                                                          \
  ([](float a_, float b_) {                                                          \
    float d_;                                                                        \
    asm("v_fmaak_f32 %0, %1, %2, " #k : "=v"(d_) : "v"(a_), "v"(b_));                \
    return d_;                                                                       \
  }((a), (b)))
__device__ __forceinline__ float gelu_erf_fast(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float pl = fmaf(1.061405429f, t, -1.453152027f);
  pl = RDMI_FMAAK(pl, t, 0x3fb5f0e3);   // + 1.421413741
  pl = RDMI_FMAAK(pl, t, 0xbe91a98e);   // − 0.284496736
  pl = RDMI_FMAAK(pl, t, 0x3e827906);   // + 0.254829592
  pl *= t;
  const float e = __builtin_amdgcn_exp2f(-az * az * 1.4426950408889634f);
  const float erf_abs = fmaf(-pl, e, 1.0f);
  const float erf_z = __builtin_copysignf(erf_abs, z);
  return x * fmaf(erf_z, 0.5f, 0.5f);
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

// 8-element vector load / store in either storage dtype (f16: one 16-B access; f32: two), values in
// f32 registers.  Lets one kernel template serve the f16 path and the paper preset's f32 path.
__device__ __forceinline__ void ld8(const f16* p, float (&v)[8]) {
  const f16x8 x = *(const f16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
}
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[4 + e] = b[e];
  }
}
__device__ __forceinline__ void st8(f16* p, const float (&v)[8]) {
  f16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (f16)v[e];
  *(f16x8*)p = o;
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
// the value a store of f in dtype T reads back as (the rounding the next op sees)
__device__ __forceinline__ float rt(f16*, float f) { return (float)(f16)f; }
__device__ __forceinline__ float rt(float*, float f) { return f; }

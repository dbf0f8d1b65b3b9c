// Decoder head: GroupNorm apply (+ SiLU) fused with the 3×3 convolution to ONE output channel
// (vae.decoder.conv_norm_out → conv_act → conv_out, vae.py:335-347, with the depth pipeline's mean
// over the three RGB outputs folded into the weights, rollingdepth_pipeline.py:737).
//
// A 1-channel 3×3 conv is HBM-bound, not MFMA-bound (2·9·C FLOPs per 2·C input bytes), and as an
// implicit GEMM it wastes the 16-wide MFMA N dimension and re-reads every input line 9×.  Here
// every input pixel is read once:
//   pass 1 (one thread per input pixel p): y = silu(a·x[p] + s) in f32 (a, s per image and channel
//           from the GroupNorm statistics), d[tap][p] = Σ_c y[c]·w[tap][c] for the 9 taps;
//   pass 2 (one thread per output pixel q): out[q] = bias + Σ_tap d[tap][q + offset(tap)], taps
//           outside the image contributing 0 (the conv's zero padding of the normalised input).
// HBM bytes per pixel: 2·C read + 9·4 written + 9·4 read (L2-served neighbours) + 2 written,
// against 4·C (GroupNorm apply) + 2·C + 2 for the separate apply → conv launches.
#include "common.h"

namespace {

constexpr int HT = 256;  // threads per workgroup

// pass 1: x [B][HW][C] f16, mr [B*G][2] {mean, rstd}, gamma/beta [C] f32, w [9][C] f32 → d [9][B*HW]
template <typename T>
__global__ __launch_bounds__(HT) void head_taps(const T* __restrict__ x, long HW, int C, int G,
                                                const float* __restrict__ mr, const float* __restrict__ gamma,
                                                const float* __restrict__ beta, const float* __restrict__ w,
                                                int silu, float* __restrict__ d, long P) {
  extern __shared__ float sm[];  // sc[C], sh[C], w[9][C]
  float* sc = sm;
  float* sh = sc + C;
  float* wl = sh + C;
  const int b = blockIdx.y;
  const int cpg = C / G;
  for (int c = threadIdx.x; c < C; c += HT) {
    const int g = c / cpg;
    const float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
    sc[c] = rstd * gamma[c];
    sh[c] = beta[c] - mean * sc[c];
  }
  for (int i = threadIdx.x; i < 9 * C; i += HT) wl[i] = w[i];
  __syncthreads();
  const long p = (long)blockIdx.x * HT + threadIdx.x;
  if (p >= HW) return;
  const T* xp = x + ((long)b * HW + p) * C;
  float acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = 0.f;
  for (int c0 = 0; c0 < C; c0 += 8) {
    float v[8];
    ld8(xp + c0, v);
    float y[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = fmaf(v[e], sc[c0 + e], sh[c0 + e]);
      y[e] = silu ? (sizeof(T) == 2 ? silu_f(f) : f / (1.0f + expf(-f))) : f;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[t] = fmaf(y[e], wl[t * C + c0 + e], acc[t]);
  }
  const long q = (long)b * HW + p;
#pragma unroll
  for (int t = 0; t < 9; ++t) d[t * P + q] = acc[t];
}

// pass 1, coalesced form (C = 8·LPP, LPP a power of two ≤ 64): LPP lanes share a pixel, each
// normalising and weighting 8 channels, so one wave load instruction reads 64/LPP whole pixel
// rows (the per-thread form above reads 64 rows 2·C bytes apart per instruction); the 9 tap sums
// are reduced across the LPP lanes in a fixed butterfly and written pixel-major, d[p][9].
// Sum over the LPP (≤ 16) lanes of a row group in the order of the xor butterfly (xor 1, 2, 4, 8): the
// partner value comes by DPP (quad_perm for 1 and 2, row_half_mirror / row_mirror for 4 and 8 — at
// those levels every lane of the partner group holds the same partial, so lane 7 − i / 15 − i gives
// the same operand as lane i ^ 4 / i ^ 8): bitwise the __shfl_xor form, without the LDS round trips
// of ds_bpermute.
template <int LPP>
__device__ __forceinline__ float group_sum(float v) {
  if (LPP > 1) v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  if (LPP > 2) v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  if (LPP > 4) v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  if (LPP > 8) v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

template <typename T, int LPP, bool SILU>
__global__ __launch_bounds__(HT) void head_taps_v(const T* __restrict__ x, long HW, int G,
                                                  const float* __restrict__ mr, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, const float* __restrict__ w,
                                                  float* __restrict__ d, long P, int ppb) {
  constexpr int C = 8 * LPP;
  const int b = blockIdx.y;
  const int cl = threadIdx.x % LPP;  // channel chunk of this lane
  const int c0 = cl * 8;
  const int cpg = C / G;
  float sc[8], sh[8], wt[9][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e, g = c / cpg;
    const float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
    sc[e] = rstd * gamma[c];
    sh[e] = beta[c] - mean * sc[e];
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t][e] = w[t * C + c];
  }
  const long pbeg = (long)blockIdx.x * ppb;
  const long pend = pbeg + ppb < HW ? pbeg + ppb : HW;
  for (long p = pbeg + threadIdx.x / LPP; p < pend; p += HT / LPP) {
    float v[8];
    ld8(x + ((long)b * HW + p) * C + c0, v);
    float acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = fmaf(v[e], sc[e], sh[e]);
      if constexpr (SILU) f = sizeof(T) == 2 ? silu_f(f) : f / (1.0f + expf(-f));
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[t] = fmaf(f, wt[t][e], acc[t]);
    }
    if constexpr (LPP <= 16) {
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[t] = group_sum<LPP>(acc[t]);
    } else {
#pragma unroll
      for (int o = 1; o < LPP; o <<= 1)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] += __shfl_xor(acc[t], o, 64);
    }
    float* dp = d + ((long)b * HW + p) * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if (t % LPP == cl) dp[t] = acc[t];  // tap t written by lane t mod LPP of the group
  }
}

// pass 1 at LPP = 16 (C = 128: the SD VAE decoder's head, the one the pipeline runs): head_taps_v's
// arithmetic, operation for operation (bitwise its taps), issued leaner — hipcc's form of it was
// vector-issue-bound at ≈230 instructions per pixel group:
//  * tap pairs (0,1) (2,3) (4,5) (6,7) as packed FMAs: v_pk_fma_f32 takes the channel's value from
//    one half of a register pair (op_sel) and does the two taps' FMAs, each rounding as v_fma_f32;
//  * the butterfly's DPP moves fused into the adds (v_add_f32_dpp: 36 instructions, not 72);
//  * the tap a lane writes picked by lane masks computed once (hipcc built a 9-way branch tree);
//  * the next pixel's 16 bytes loaded before this pixel's arithmetic;
//  * the taps written planar, d[t][B·HW], for head_gather (its 9 reads per output coalesced across
//    lanes; the pixel-major d[p][9] made each read touch 64 pixels 36 B apart) — the same sums in the
//    same order, so the same output bits.
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int LO>  // acc.xy += y[LO] * w.xy
__device__ __forceinline__ void pk_fma_lo(f32x2& acc, f32x2 y, f32x2 w) {
  if constexpr (LO == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(y), "v"(w));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(y), "v"(w));
}

// Σ over the 16 lanes of a row, xor-butterfly order (group_sum<16>), for nine values at once: nine
// independent adds per level, so one s_nop covers the DPP read-after-VALU-write hazard at entry.
__device__ __forceinline__ void group16_sum9(float& a0, float& a1, float& a2, float& a3, float& a4, float& a5,
                                             float& a6, float& a7, float& a8) {
#define RDMI_L9(CTL)                                                       \
  "v_add_f32_dpp %0, %0, %0 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %1, %1, %1 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %2, %2, %2 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %3, %3, %3 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %4, %4, %4 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %5, %5, %5 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %6, %6, %6 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %7, %7, %7 " CTL " row_mask:0xf bank_mask:0xf\n\t"        \
  "v_add_f32_dpp %8, %8, %8 " CTL " row_mask:0xf bank_mask:0xf\n\t"
  asm("s_nop 1\n\t" RDMI_L9("quad_perm:[1,0,3,2]") RDMI_L9("quad_perm:[2,3,0,1]") RDMI_L9("row_half_mirror")
          RDMI_L9("row_mirror")
      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+v"(a8));
#undef RDMI_L9
}

// 16 input bytes / 32 (f32) of one lane, loaded raw: the conversion waits for the load, so the
// prefetch of the next pixel holds the raw registers, not converted values.
template <typename T>
struct Raw8;
template <>
struct Raw8<f16> {
  f16x8 r;
  __device__ __forceinline__ void load(const f16* p) { r = *(const f16x8*)p; }
  __device__ __forceinline__ float operator[](int e) const { return (float)r[e]; }
};
template <>
struct Raw8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *(const f32x4*)p;
    b = *(const f32x4*)(p + 4);
  }
  __device__ __forceinline__ float operator[](int e) const { return e < 4 ? a[e] : b[e - 4]; }
};

template <typename T, bool SILU>
struct Head16 {
  float sc[8], sh[8];
  f32x2 wp[4][8];  // taps (2i, 2i+1) of channel c0 + e
  float w8[8];     // tap 8
  int cl;

  long P;  // planar tap stride: d[t][B·HW]
  __device__ __forceinline__ void pixel(const Raw8<T>& v, float* __restrict__ dq) const {
    f32x2 y[4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = fmaf(v[e], sc[e], sh[e]);
      if constexpr (SILU) f = sizeof(T) == 2 ? silu_f(f) : f / (1.0f + expf(-f));
      y[e >> 1][e & 1] = f;
    }
    f32x2 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = f32x2{0.f, 0.f};  // first step fma(y, w, 0) as head_taps_v's
    float a8 = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (e & 1)
          pk_fma_lo<1>(a[i], y[e >> 1], wp[i][e]);
        else
          pk_fma_lo<0>(a[i], y[e >> 1], wp[i][e]);
      }
      a8 = fmaf(y[e >> 1][e & 1], w8[e], a8);
    }
    float s0 = a[0].x, s1 = a[0].y, s2 = a[1].x, s3 = a[1].y, s4 = a[2].x, s5 = a[2].y, s6 = a[3].x, s7 = a[3].y;
    group16_sum9(s0, s1, s2, s3, s4, s5, s6, s7, a8);
    float o = s0;
    o = cl == 1 ? s1 : o;
    o = cl == 2 ? s2 : o;
    o = cl == 3 ? s3 : o;
    o = cl == 4 ? s4 : o;
    o = cl == 5 ? s5 : o;
    o = cl == 6 ? s6 : o;
    o = cl == 7 ? s7 : o;
    o = cl == 8 ? a8 : o;
    if (cl < 9) dq[cl * P] = o;  // tap cl written by lane cl of the group, planar (head_gather)
  }
};

template <typename T, bool SILU>
__global__ __launch_bounds__(HT) void head_taps_16(const T* __restrict__ x, long HW, int G,
                                                   const float* __restrict__ mr, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, const float* __restrict__ w,
                                                   float* __restrict__ d, long P, int ppb) {
  constexpr int C = 128, LPP = 16, S = HT / LPP;
  const int b = blockIdx.y;
  Head16<T, SILU> h;
  h.cl = threadIdx.x % LPP;
  const int c0 = h.cl * 8;
  const int cpg = C / G;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e, g = c / cpg;
    const float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
    h.sc[e] = rstd * gamma[c];
    h.sh[e] = beta[c] - mean * h.sc[e];
#pragma unroll
    for (int i = 0; i < 4; ++i) h.wp[i][e] = f32x2{w[(2 * i) * C + c], w[(2 * i + 1) * C + c]};
    h.w8[e] = w[8 * C + c];
  }
  const long pbeg = (long)blockIdx.x * ppb;
  const long pend = pbeg + ppb < HW ? pbeg + ppb : HW;
  long p = pbeg + threadIdx.x / LPP;
  if (p >= pend) return;
  const T* xb = x + (long)b * HW * C + c0;
  float* db = d + (long)b * HW;
  h.P = P;
  // two raw buffers in turn; the next pixel's load is unconditional (clamped to the last pixel) so
  // that the wait before each pixel's arithmetic counts only the older load
  Raw8<T> ra, rb;
  ra.load(xb + p * C);
  for (;;) {
    rb.load(xb + (p + S < pend ? p + S : pend - 1) * C);
    h.pixel(ra, db + p);
    p += S;
    if (p >= pend) break;
    ra.load(xb + (p + S < pend ? p + S : pend - 1) * C);
    h.pixel(rb, db + p);
    p += S;
    if (p >= pend) break;
  }
}

// pass 2 for the pixel-major taps: out[q] = bias + Σ_{dy,dx} d[q + (dy-1)·W + dx-1][3dy+dx]
template <typename T>
__global__ __launch_bounds__(HT) void head_gather_v(const float* __restrict__ d, int H, int W, long P, float bias,
                                                    T* __restrict__ out) {
  const long q = (long)blockIdx.x * HT + threadIdx.x;
  if (q >= P) return;
  const long HW = (long)H * W;
  const long b = q / HW;
  const int r = (int)(q - b * HW);
  const int h = r / W, wc = r - (r / W) * W;
  float s = bias;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int hh = h + dy - 1;
    if ((unsigned)hh >= (unsigned)H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int ww = wc + dx - 1;
      if ((unsigned)ww >= (unsigned)W) continue;
      s += d[(b * HW + (long)hh * W + ww) * 9 + 3 * dy + dx];
    }
  }
  out[q] = (T)s;
}

// pass 2: out[b][h][w] = bias + Σ_{dy,dx} d[3dy+dx][b][h+dy-1][w+dx-1] (zero outside the image)
template <typename T>
__global__ __launch_bounds__(HT) void head_gather(const float* __restrict__ d, int H, int W, long P, float bias,
                                                  T* __restrict__ out) {
  const long q = (long)blockIdx.x * HT + threadIdx.x;
  if (q >= P) return;
  const long HW = (long)H * W;
  const long b = q / HW;
  const int r = (int)(q - b * HW);
  const int h = r / W, wc = r - (r / W) * W;
  float s = bias;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int hh = h + dy - 1;
    if ((unsigned)hh >= (unsigned)H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int ww = wc + dx - 1;
      if ((unsigned)ww >= (unsigned)W) continue;
      s += d[(3 * dy + dx) * P + b * HW + (long)hh * W + ww];
    }
  }
  out[q] = (T)s;
}

template <typename T, typename U>
int head_launch(const void* x, int B, int H, int W, int C, int G, const float* mean_rstd, const float* gamma,
                const float* beta, int silu, const float* w, float bias, void* y, float* workspace, hipStream_t s) {
  const long HW = (long)H * W, P = (long)B * HW;
  const int lpp = C / 8;
  if (lpp == 16 || lpp == 32 || lpp == 64 || lpp == 8 || lpp == 4 || lpp == 2 || lpp == 1) {
    constexpr int PPB = 1024;  // pixels per workgroup
    dim3 g(rdmi::div_up(HW, PPB), B);
#define RDMI_HEAD(L)                                                                                             \
  case L:                                                                                                        \
    if (silu)                                                                                                    \
      hipLaunchKernelGGL((head_taps_v<T, L, true>), g, dim3(HT), 0, s, (const T*)x, HW, G, mean_rstd, gamma,    \
                         beta, w, workspace, P, PPB);                                                            \
    else                                                                                                         \
      hipLaunchKernelGGL((head_taps_v<T, L, false>), g, dim3(HT), 0, s, (const T*)x, HW, G, mean_rstd, gamma,   \
                         beta, w, workspace, P, PPB);                                                            \
    break;
    switch (lpp) {
      case 16: {
        if (silu)
          hipLaunchKernelGGL((head_taps_16<T, true>), g, dim3(HT), 0, s, (const T*)x, HW, G, mean_rstd, gamma, beta,
                             w, workspace, P, PPB);
        else
          hipLaunchKernelGGL((head_taps_16<T, false>), g, dim3(HT), 0, s, (const T*)x, HW, G, mean_rstd, gamma, beta,
                             w, workspace, P, PPB);
        int rc = rdmi::check_launch("conv3x3_to1_gn taps");
        if (rc) return rc;
        // planar taps: the gather's 9 reads per output are coalesced across lanes
        hipLaunchKernelGGL(head_gather<U>, dim3(rdmi::div_up(P, HT)), dim3(HT), 0, s, workspace, H, W, P, bias, (U*)y);
        return rdmi::check_launch("conv3x3_to1_gn gather");
      }
      RDMI_HEAD(1) RDMI_HEAD(2) RDMI_HEAD(4) RDMI_HEAD(8) RDMI_HEAD(32) RDMI_HEAD(64)
      default: break;
    }
#undef RDMI_HEAD
    int rc = rdmi::check_launch("conv3x3_to1_gn taps");
    if (rc) return rc;
    hipLaunchKernelGGL(head_gather_v<U>, dim3(rdmi::div_up(P, HT)), dim3(HT), 0, s, workspace, H, W, P, bias, (U*)y);
    return rdmi::check_launch("conv3x3_to1_gn gather");
  }
  const size_t lds = (size_t)11 * C * sizeof(float);
  hipLaunchKernelGGL(head_taps<T>, dim3(rdmi::div_up(HW, HT), B), dim3(HT), lds, s, (const T*)x, HW, C, G, mean_rstd,
                     gamma, beta, w, silu, workspace, P);
  int rc = rdmi::check_launch("conv3x3_to1_gn taps");
  if (rc) return rc;
  hipLaunchKernelGGL(head_gather<U>, dim3(rdmi::div_up(P, HT)), dim3(HT), 0, s, workspace, H, W, P, bias, (U*)y);
  return rdmi::check_launch("conv3x3_to1_gn gather");
}

}  // namespace

extern "C" long rdmi_conv3x3_to1_gn_workspace(int B, int H, int W) { return 9L * B * H * W; }

extern "C" int rdmi_conv3x3_to1_gn(const void* x, int dtype, int B, int H, int W, int C, int G, const float* mean_rstd,
                                   const float* gamma, const float* beta, int silu, const float* w, float bias,
                                   void* y, int y_dtype, float* workspace, void* stream) {
  RDMI_REQUIRE(x && mean_rstd && gamma && beta && w && y && workspace, RDMI_E_ARG, "conv3x3_to1_gn: null pointer");
  RDMI_REQUIRE(B > 0 && H > 0 && W > 0 && C % 8 == 0 && C > 0 && C <= 1024 && G > 0 && C % G == 0, RDMI_E_ARG,
               "conv3x3_to1_gn: bad sizes B=%d H=%d W=%d C=%d G=%d", B, H, W, C, G);
  RDMI_REQUIRE(((uintptr_t)x & 15) == 0, RDMI_E_ALIGN, "conv3x3_to1_gn: x not 16-byte aligned");
  RDMI_REQUIRE((dtype == RDMI_F16 || dtype == RDMI_F32) && (y_dtype == RDMI_F16 || y_dtype == RDMI_F32), RDMI_E_ARG,
               "conv3x3_to1_gn: dtype %d / y_dtype %d", dtype, y_dtype);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RDMI_F32)
    return y_dtype == RDMI_F32
               ? head_launch<float, float>(x, B, H, W, C, G, mean_rstd, gamma, beta, silu, w, bias, y, workspace, st)
               : head_launch<float, f16>(x, B, H, W, C, G, mean_rstd, gamma, beta, silu, w, bias, y, workspace, st);
  return y_dtype == RDMI_F32
             ? head_launch<f16, float>(x, B, H, W, C, G, mean_rstd, gamma, beta, silu, w, bias, y, workspace, st)
             : head_launch<f16, f16>(x, B, H, W, C, G, mean_rstd, gamma, beta, silu, w, bias, y, workspace, st);
}

// Frame ingest and resize: rollingdepth/video_io.py:38-137 (resize_max_res → torchvision resize with
// antialias=True on the decoded float frame, then (x / 255)·2 − 1) and the restore_res resize of
// rollingdepth_pipeline.py:155-173.  torchvision's tensor resize is
// F.interpolate(mode, align_corners=False, antialias=True) for BILINEAR / BICUBIC and
// F.interpolate(mode="nearest") for NEAREST; its antialiased path is separable — the width pass
// (into an f32 [N, C, H, Wo] intermediate) then the height pass — and only resamples a dimension
// whose size changes.  The tap ranges and weights below restate that kernel's arithmetic (ATen
// UpSampleKernel.cpp `_compute_indices_min_size_weights_aa`): scale = in / out in f32, center =
// scale·(i + 0.5) formed in f64 and rounded to f32, support = (interp/2)·max(scale, 1), taps
// [trunc(center − support + 0.5), trunc(center + support + 0.5)) clipped to the input, weights
// filter((j + xmin − center + 0.5)·invscale) normalised by their f32 sum; each output is the
// in-order f32 sum of tap·weight (products and sums rounded separately, no contraction).
// HBM-bound: one thread per output element, the taps computed in registers.
#include "common.h"

#include <type_traits>

namespace {

constexpr int MAXT = 40;  // taps per output: 2·ceil(support) + 1; the host caps scale (rdmi_resize)

__device__ __forceinline__ float filt(int mode, float x) {
  if (mode == RDMI_RESIZE_BILINEAR) {
    if (x < 0.f) x = -x;
    return x < 1.f ? (float)(1.0 - (double)x) : 0.f;
  }
  // bicubic, a = −0.5 (Keys), evaluated in f64 as the ATen filter's double literals make it
  const double a = -0.5, xd = fabs((double)x);
  if (xd < 1.0) return (float)(((a + 2.0) * xd - (a + 3.0)) * xd * xd + 1.0);
  if (xd < 2.0) return (float)((((xd - 5.0) * xd + 8.0) * xd - 4.0) * a);
  return 0.f;
}

// taps of output index i along a dimension in_size → out_size; returns the count, fills lo and w
__device__ __forceinline__ int taps(int mode, int i, int in_size, int out_size, int& lo, float* w) {
  const float scale = (float)in_size / (float)out_size;
  if (mode == RDMI_RESIZE_NEAREST) {  // ATen nearest_idx
    if (out_size == in_size) lo = i;
    else if (out_size == 2 * in_size) lo = i >> 1;
    else lo = min((int)floorf((float)i * scale), in_size - 1);
    w[0] = 1.f;
    return 1;
  }
  const float half = mode == RDMI_RESIZE_BICUBIC ? 2.f : 1.f;
  const float support = scale >= 1.f ? half * scale : half;
  const float center = (float)((double)scale * ((double)i + 0.5));
  const float invscale = scale >= 1.f ? (float)(1.0 / (double)scale) : 1.f;
  const int xmin = max((int)((double)(center - support) + 0.5), 0);
  const int xmax = min((int)((double)(center + support) + 0.5), in_size);
  const int n = min(xmax - xmin, MAXT);
  float total = 0.f;
  for (int j = 0; j < n; ++j) {
    const float d = (float)(j + xmin) - center;
    const float wj = filt(mode, (float)(((double)d + 0.5) * (double)invscale));
    w[j] = wj;
    total = __fadd_rn(total, wj);
  }
  if (total != 0.f)
    for (int j = 0; j < n; ++j) w[j] = __fdiv_rn(w[j], total);
  lo = xmin;
  return n;
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, long o) { return (float)p[o]; }

__device__ __forceinline__ float post(float v, int normalize) {
  return normalize ? __fsub_rn(__fmul_rn(__fdiv_rn(v, 255.f), 2.f), 1.f) : v;
}

// width pass: src element (n, c, y, x) at n·sn + c·sc + y·sy + x·sx → dst [N, C, H, Wo] (f32), or
// straight to the output (with the post-op) when the height does not change
template <typename T>
__global__ void resize_w_k(const T* __restrict__ x, long sn, long sc, long sy, long sx, int N, int C, int H, int W,
                           int Wo, int mode, int normalize, float* __restrict__ dst) {
  const long total = (long)N * C * H * Wo;
  for (long o = blockIdx.x * (long)blockDim.x + threadIdx.x; o < total; o += (long)gridDim.x * blockDim.x) {
    const int xo = (int)(o % Wo);
    const long r = o / Wo;
    const int y = (int)(r % H);
    const long nc = r / H;
    const int c = (int)(nc % C), n = (int)(nc / C);
    float w[MAXT];
    int lo;
    const int nt = taps(mode, xo, W, Wo, lo, w);
    const long base = n * sn + c * sc + y * sy;
    float acc = __fmul_rn(ld(x, base + (long)lo * sx), w[0]);
    for (int j = 1; j < nt; ++j) acc = __fadd_rn(acc, __fmul_rn(ld(x, base + (long)(lo + j) * sx), w[j]));
    dst[o] = post(acc, normalize);
  }
}

// height pass (or a plain copy when nothing is resampled: mode forced to nearest, identity taps)
template <typename T>
__global__ void resize_h_k(const T* __restrict__ x, long sn, long sc, long sy, long sx, int N, int C, int H, int Ho,
                           int Wo, int mode, int normalize, float* __restrict__ y) {
  const long total = (long)N * C * Ho * Wo;
  for (long o = blockIdx.x * (long)blockDim.x + threadIdx.x; o < total; o += (long)gridDim.x * blockDim.x) {
    const int xo = (int)(o % Wo);
    const long r = o / Wo;
    const int yo = (int)(r % Ho);
    const long nc = r / Ho;
    const int c = (int)(nc % C), n = (int)(nc / C);
    float w[MAXT];
    int lo;
    const int nt = taps(mode, yo, H, Ho, lo, w);
    const long base = n * sn + c * sc + xo * sx;
    float acc = __fmul_rn(ld(x, base + (long)lo * sy), w[0]);
    for (int j = 1; j < nt; ++j) acc = __fadd_rn(acc, __fmul_rn(ld(x, base + (long)(lo + j) * sy), w[j]));
    y[o] = post(acc, normalize);
  }
}

inline unsigned grid_for(long n) {
  long g = (n + 255) / 256;
  return (unsigned)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" size_t rdmi_resize_workspace(int N, int C, int H, int W, int Ho, int Wo) {
  return (H != Ho && W != Wo) ? (size_t)N * C * H * Wo * sizeof(float) : 0;
}

extern "C" int rdmi_resize(const void* x, int x_dtype, long sn, long sc, long sy, long sx, int N, int C, int H, int W,
                           int Ho, int Wo, int mode, int normalize, float* y, void* workspace, void* stream) {
  RDMI_REQUIRE(x && y && N > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, RDMI_E_ARG, "resize: bad sizes");
  RDMI_REQUIRE(x_dtype == RDMI_U8 || x_dtype == RDMI_F32, RDMI_E_UNSUPPORTED, "resize: input dtype u8 or f32");
  RDMI_REQUIRE(mode == RDMI_RESIZE_NEAREST || mode == RDMI_RESIZE_BILINEAR || mode == RDMI_RESIZE_BICUBIC,
               RDMI_E_UNSUPPORTED, "resize: mode NEAREST, BILINEAR or BICUBIC");
  // taps per output ≤ 2·support + 2 ≤ MAXT: downscale factor ≤ 9 (bicubic: 4.5)
  const float half = mode == RDMI_RESIZE_BICUBIC ? 2.f : 1.f;
  RDMI_REQUIRE(mode == RDMI_RESIZE_NEAREST ||
                   (2.f * half * fmaxf((float)W / Wo, 1.f) + 2.f <= MAXT && 2.f * half * fmaxf((float)H / Ho, 1.f) + 2.f <= MAXT),
               RDMI_E_UNSUPPORTED, "resize: downscale factor beyond the tap buffer");
  const bool rw = W != Wo, rh = H != Ho;
  RDMI_REQUIRE(!(rw && rh) || workspace, RDMI_E_ARG, "resize: workspace required (rdmi_resize_workspace)");
  hipStream_t st = (hipStream_t)stream;
  auto launch_w = [&](auto* xp, float* dst, int norm) {
    hipLaunchKernelGGL(resize_w_k<std::remove_const_t<std::remove_pointer_t<decltype(xp)>>>,
                       dim3(grid_for((long)N * C * H * Wo)), dim3(256), 0, st, xp, sn, sc, sy, sx, N, C, H, W, Wo, mode,
                       norm, dst);
  };
  auto launch_h = [&](auto* xp, long a, long b, long c, long d, int md, float* dst) {
    hipLaunchKernelGGL(resize_h_k<std::remove_const_t<std::remove_pointer_t<decltype(xp)>>>,
                       dim3(grid_for((long)N * C * Ho * Wo)), dim3(256), 0, st, xp, a, b, c, d, N, C, H, Ho, Wo, md,
                       normalize, dst);
  };
  const unsigned char* xu = (const unsigned char*)x;
  const float* xf = (const float*)x;
  if (rw && rh) {
    float* t = (float*)workspace;
    if (x_dtype == RDMI_U8) launch_w(xu, t, 0); else launch_w(xf, t, 0);
    launch_h(t, (long)C * H * Wo, (long)H * Wo, (long)Wo, 1L, mode, y);
  } else if (rw) {
    if (x_dtype == RDMI_U8) launch_w(xu, y, normalize); else launch_w(xf, y, normalize);
  } else {  // height only, or a copy (identity taps)
    const int md = rh ? mode : RDMI_RESIZE_NEAREST;
    if (x_dtype == RDMI_U8) launch_h(xu, sn, sc, sy, sx, md, y); else launch_h(xf, sn, sc, sy, sx, md, y);
  }
  return rdmi::check_launch("resize");
}

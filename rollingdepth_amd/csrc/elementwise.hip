// Layout conversion and small fused elementwise steps of the snippet path (all HBM-bound,
// grid-stride, 16-B vectors where the channel count allows).
#include "common.h"

namespace {

inline unsigned grid_for(long n, int per_block = 256) {
  long g = (n + per_block - 1) / per_block;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  return (unsigned)g;
}

template <typename TO>
__global__ void nchw_to_nhwc_k(const void* __restrict__ x, int x_f32, TO* __restrict__ y, int C, long HW, int Cpad,
                               long n, float scale, long bstride, long cstride) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    long pix = i / Cpad;
    int c = (int)(i - pix * Cpad);
    long b = pix / HW, p = pix - b * HW;
    float v = 0.f;
    if (c < C) {
      long src = b * bstride + c * cstride + p;
      v = x_f32 ? ((const float*)x)[src] : (float)((const f16*)x)[src];
      v *= scale;
    }
    y[i] = (TO)v;
  }
}

template <typename T>
__global__ void nhwc_to_nchw_k(const T* __restrict__ x, long ld, float* __restrict__ y, int C, long HW, long n,
                               float scale, float shift) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    long bc = i / HW, p = i - bc * HW;
    long b = bc / C;
    int c = (int)(bc - b * C);
    y[i] = (float)x[(b * HW + p) * ld + c] * scale + shift;
  }
}

// Ca, Cb in 16-B vectors (8 halves or 4 floats)
__global__ void concat_k(const f32x4* __restrict__ a, int AV, const f32x4* __restrict__ b, int BVv, f32x4* __restrict__ y,
                         long P) {
  const int CV = AV + BVv;
  long n = P * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    long p = i / CV;
    int cv = (int)(i - p * CV);
    y[i] = cv < AV ? a[p * AV + cv] : b[p * BVv + (cv - AV)];
  }
}

// nearest resize, PyTorch's index rule for an explicit output size: src = min(floor(dst·(in/out)), in−1)
// with the scale in f32 (F.interpolate(mode="nearest", size=...), as Upsample2D uses it)
__global__ void resize_nearest_k(const f32x4* __restrict__ x, int H, int W, int CV, f32x4* __restrict__ y, int Ho, int Wo,
                                 long n) {
  const float sy = (float)H / (float)Ho, sx = (float)W / (float)Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    const long px = i / CV;
    const int xo = (int)(px % Wo);
    const long r = px / Wo;
    const int yo = (int)(r % Ho);
    const long b = r / Ho;
    const int yi = min((int)floorf((float)yo * sy), H - 1), xi = min((int)floorf((float)xo * sx), W - 1);
    y[i] = x[((b * H + yi) * W + xi) * CV + cv];
  }
}

template <typename T>
__global__ void transpose_k(const T* __restrict__ src, T* __restrict__ dst, long rows, long cols, long sld,
                            long dld) {
  __shared__ T tile[64][65];
  const int b = blockIdx.z;
  const long r0 = blockIdx.y * 64L, c0 = blockIdx.x * 64L;
  src += (long)b * rows * sld;
  dst += (long)b * cols * dld;
  for (int i = threadIdx.y; i < 64; i += 4) {
    long r = r0 + i, c = c0 + threadIdx.x;
    if (r < rows && c < cols) tile[i][threadIdx.x] = src[r * sld + c];
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 64; i += 4) {
    long c = c0 + i, r = r0 + threadIdx.x;
    if (r < rows && c < cols) dst[c * dld + r] = tile[threadIdx.x][i];
  }
}

// out [count][HW][8]: rgb latent channels 0..3, depth latent 4..7
template <typename T>
__global__ void gather_unet_input_k(const T* __restrict__ rgb, long rgb_ld, const T* __restrict__ depth,
                                    long depth_ld, int bcast, const int* __restrict__ fidx, int count, long HW,
                                    T* __restrict__ out) {
  long n = (long)count * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int s = (int)(i / HW);
    long p = i - (long)s * HW;
    int f = fidx[s];
    const T* r = rgb + (long)f * rgb_ld + p * 8;
    const T* d = depth + (bcast ? 0 : (long)f * depth_ld) + p * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = (float)r[e];
      v[4 + e] = (float)d[e];
    }
    st8(out + i * 8, v);
  }
}

template <typename T>
__global__ void ddim_combine_k(const T* __restrict__ x, long ldx, const T* __restrict__ e, long lde,
                               T* __restrict__ y, long ldy, long P, int C, int Cpad, float ca, float cb, float sc,
                               long e_period) {
  long n = P * Cpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    long p = i / Cpad;
    int c = (int)(i - p * Cpad);
    long pe = e_period > 0 ? p % e_period : p;
    float v = 0.f;
    if (c < C) v = (ca * (float)x[p * ldx + c] + cb * (float)e[pe * lde + c]) * sc;
    y[p * ldy + c] = (T)v;
  }
}

// refine (rollingdepth_pipeline.py:586-629): new[f] = mean over the snippets s covering f
// (s = f - j*stride, slot j) of pred[s][j]; accumulated in f32 in snippet order.
template <typename T>
__global__ void snippet_average_k(const T* __restrict__ src, int n, int w, int stride, long P, int C, int ld,
                                  T* __restrict__ out) {
  const int f = blockIdx.y;
  const long tot = P * ld;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % ld);
    float v = 0.f;
    if (c < C) {
      // f64 sum of the ≤ w covering predictions: exact, so the sharded refine's per-rank sums
      // (snippet_accumulate_k, all-reduced in any order, snippet_finish_k) reproduce it bitwise
      double s = 0.0;
      int cnt = 0;
      for (int j = w - 1; j >= 0; --j) {  // snippet index ascending
        const int sn = f - j * stride;
        if (sn < 0 || sn >= n) continue;
        s += (double)(float)src[((long)sn * w + j) * tot + i];
        ++cnt;
      }
      v = cnt ? (float)(s / (double)cnt) : 0.f;
    }
    out[(long)f * tot + i] = (T)v;
  }
}

// sharded refine (rollingdepth_pipeline.py:586-629 split over ranks): the per-frame f32 sum over
// this rank's snippets k0 .. k0+nloc-1 (snippet index ascending, as snippet_average_k), for all N
// frames (zeros where no local snippet covers f) — all-reduced over ranks, then snippet_finish_k
template <typename T>
__global__ void snippet_accumulate_k(const T* __restrict__ src, int k0, int nloc, int w, int stride, long P, int C,
                                     int ld, double* __restrict__ sum) {
  const int f = blockIdx.y;
  const long tot = P * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const long p = i / C;
    const int c = (int)(i - p * C);
    double s = 0.0;
    for (int j = w - 1; j >= 0; --j) {
      const int sn = f - j * stride;
      if (sn < k0 || sn >= k0 + nloc) continue;
      s += (double)(float)src[((long)(sn - k0) * w + j) * P * ld + p * ld + c];
    }
    sum[(long)f * tot + i] = s;
  }
}

template <typename T>
__global__ void snippet_finish_k(const double* __restrict__ sum, int n, int w, int stride, long P, int C, int ld,
                                 T* __restrict__ out) {
  const int f = blockIdx.y;
  int cnt = 0;
  for (int j = 0; j < w; ++j) {
    const int sn = f - j * stride;
    cnt += (sn >= 0 && sn < n) ? 1 : 0;
  }
  const long tot = P * ld;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
    const long p = i / ld;
    const int c = (int)(i - p * ld);
    float v = 0.f;
    if (c < C && cnt) v = (float)(sum[((long)f * P + p) * C + c] / (double)cnt);
    out[(long)f * tot + i] = (T)v;
  }
}

// colorize_depth (src/util/colorize.py:12-66): per pixel, normalise by (min, max) in the depth's own
// dtype as numpy does ((d - mn) / (mx - mn), clip to [0, 1]), index a matplotlib colormap the way
// Colormap.__call__ does for floats (x·N, x == N → N−1, truncating int cast; NaN → the "bad" entry
// N + 2), and write the 8-bit RGB the reference gets from (lut·255).astype(uint8) (host-built table).
__device__ __forceinline__ float rnd(const f16*, float v) { return (float)(f16)v; }
__device__ __forceinline__ float rnd(const float*, float v) { return v; }

template <typename T>
__global__ void colorize_k(const T* __restrict__ d, long n, const T* __restrict__ mm, const unsigned char* __restrict__ lut,
                           int N, unsigned char* __restrict__ out, int* __restrict__ idx_out) {
  const float mn = (float)mm[0], rng = (float)mm[1];  // {min, max − min}, both as the caller's numpy computes them
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = (float)d[i];
    int idx;
    if (v != v) {
      idx = N + 2;
    } else {
      float x = rnd(d, __fdiv_rn(rnd(d, v - mn), rng));
      x = fminf(fmaxf(x, 0.f), 1.f);
      x = rnd(d, x * (float)N);
      if (x == (float)N) x = (float)(N - 1);
      idx = (int)x;
    }
    if (idx_out) {
      idx_out[i] = idx;
      continue;
    }
    out[3 * i] = lut[3 * idx];
    out[3 * i + 1] = lut[3 * idx + 1];
    out[3 * i + 2] = lut[3 * idx + 2];
  }
}

// 16-B vector loads (8 halves / 4 floats per lane and step), scalar tail; min/max are
// order-independent, so the result is exact whatever the split.
__global__ __launch_bounds__(256) void minmax_partial(const void* __restrict__ x, int xf32, long n,
                                                      float* __restrict__ part) {
  float mn = INFINITY, mx = -INFINITY;
  const long stride = (long)gridDim.x * blockDim.x;
  const long t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const bool al = ((uintptr_t)x & 15) == 0;
  const int per = xf32 ? 4 : 8;
  const long nvec = al ? n / per : 0;
  for (long i = t0; i < nvec; i += stride) {
    if (xf32) {
      const f32x4 v = ((const f32x4*)x)[i];
      mn = fminf(mn, fminf(fminf(v[0], v[1]), fminf(v[2], v[3])));
      mx = fmaxf(mx, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    } else {
      const f16x8 v = ((const f16x8*)x)[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mn = fminf(mn, (float)v[e]);
        mx = fmaxf(mx, (float)v[e]);
      }
    }
  }
  for (long i = nvec * per + t0; i < n; i += stride) {
    float v = xf32 ? ((const float*)x)[i] : (float)((const f16*)x)[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  __shared__ float r[2][4];
  if ((threadIdx.x & 63) == 0) {
    r[0][threadIdx.x >> 6] = mn;
    r[1][threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = fminf(fminf(r[0][0], r[0][1]), fminf(r[0][2], r[0][3]));
    part[2 * blockIdx.x + 1] = fmaxf(fmaxf(r[1][0], r[1][1]), fmaxf(r[1][2], r[1][3]));
  }
}

__global__ void minmax_final(const float* __restrict__ part, int nb, float* __restrict__ out) {
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nb; i += 64) {
    mn = fminf(mn, part[2 * i]);
    mx = fmaxf(mx, part[2 * i + 1]);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  if (threadIdx.x == 0) {
    out[0] = mn;
    out[1] = mx;
  }
}

// reference order (rollingdepth_pipeline.py:316-318): d -= min; d /= max(d); d = d*2 - 1
__global__ void renorm_k(float* __restrict__ x, long n, const float* __restrict__ mm) {
  const float mn = mm[0];
  const float rng = mm[1] - mn;  // max(d - min) == max - min exactly for the max element
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = x[i] - mn;
    v = v / rng;
    x[i] = v * 2.0f - 1.0f;
  }
}

}  // namespace

extern "C" int rdmi_nchw_to_nhwc(const void* x, int x_f32, void* y, int y_dtype, int B, int C, int H, int W, int Cpad,
                                 float scale, long x_bstride, long x_cstride, void* stream) {
  RDMI_REQUIRE(x && y && Cpad >= C, RDMI_E_ARG, "nchw_to_nhwc: bad args");
  long n = (long)B * H * W * Cpad;
  if (y_dtype == RDMI_F32)
    hipLaunchKernelGGL(nchw_to_nhwc_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, x_f32,
                       (float*)y, C, (long)H * W, Cpad, n, scale, x_bstride, x_cstride);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_k<f16>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, x_f32, (f16*)y,
                       C, (long)H * W, Cpad, n, scale, x_bstride, x_cstride);
  return rdmi::check_launch("nchw_to_nhwc");
}

extern "C" int rdmi_nhwc_to_nchw_f32(const void* x, int dtype, long ld, float* y, int B, int C, int H, int W,
                                     float scale, float shift, void* stream) {
  RDMI_REQUIRE(x && y && ld >= C, RDMI_E_ARG, "nhwc_to_nchw: bad args");
  long n = (long)B * C * H * W;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(nhwc_to_nchw_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const float*)x, ld,
                       y, C, (long)H * W, n, scale, shift);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_k<f16>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const f16*)x, ld, y,
                       C, (long)H * W, n, scale, shift);
  return rdmi::check_launch("nhwc_to_nchw");
}

extern "C" int rdmi_concat_channels(const void* a, int Ca, const void* b, int Cb, void* y, long P, int dtype,
                                    void* stream) {
  const int per = dtype == RDMI_F32 ? 4 : 8;  // elements per 16-B vector
  RDMI_REQUIRE(a && b && y && Ca % per == 0 && Cb % per == 0, RDMI_E_ALIGN,
               "concat: channels must be multiples of %d", per);
  long n = P * ((Ca + Cb) / per);
  hipLaunchKernelGGL(concat_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const f32x4*)a, Ca / per,
                     (const f32x4*)b, Cb / per, (f32x4*)y, P);
  return rdmi::check_launch("concat");
}

extern "C" int rdmi_resize_nearest(const void* x, int B, int H, int W, int C, void* y, int Ho, int Wo, int dtype,
                                   void* stream) {
  RDMI_REQUIRE(x && y && B > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0, RDMI_E_ARG, "resize_nearest: bad args");
  const int per = dtype == RDMI_F32 ? 4 : 8;
  RDMI_REQUIRE(C % per == 0, RDMI_E_ALIGN, "resize_nearest: C (%d) must be a multiple of %d", C, per);
  const long n = (long)B * Ho * Wo * (C / per);
  hipLaunchKernelGGL(resize_nearest_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const f32x4*)x, H, W,
                     C / per, (f32x4*)y, Ho, Wo, n);
  return rdmi::check_launch("resize_nearest");
}

extern "C" int rdmi_transpose(const void* src, void* dst, int batch, long rows, long cols, long src_ld, long dst_ld,
                              int dtype, void* stream) {
  RDMI_REQUIRE(src && dst && rows > 0 && cols > 0, RDMI_E_ARG, "transpose: bad args");
  dim3 g(rdmi::div_up(cols, 64), rdmi::div_up(rows, 64), batch);
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(transpose_k<float>, g, dim3(64, 4), 0, (hipStream_t)stream, (const float*)src, (float*)dst, rows,
                       cols, src_ld, dst_ld);
  else
    hipLaunchKernelGGL(transpose_k<f16>, g, dim3(64, 4), 0, (hipStream_t)stream, (const f16*)src, (f16*)dst, rows, cols,
                       src_ld, dst_ld);
  return rdmi::check_launch("transpose");
}

extern "C" int rdmi_gather_unet_input(const void* rgb, long rgb_frame_ld, const void* depth, long depth_frame_ld,
                                      int depth_bcast, const int* frame_idx, int count, long HW, void* out, int dtype,
                                      void* stream) {
  RDMI_REQUIRE(rgb && depth && frame_idx && out && count > 0, RDMI_E_ARG, "gather_unet_input: bad args");
  long n = (long)count * HW;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(gather_unet_input_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)rgb, rgb_frame_ld, (const float*)depth, depth_frame_ld, depth_bcast, frame_idx,
                       count, HW, (float*)out);
  else
    hipLaunchKernelGGL(gather_unet_input_k<f16>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const f16*)rgb,
                       rgb_frame_ld, (const f16*)depth, depth_frame_ld, depth_bcast, frame_idx, count, HW, (f16*)out);
  return rdmi::check_launch("gather_unet_input");
}

extern "C" int rdmi_ddim_combine(const void* x, long ld_x, const void* e, long ld_e, void* y, long ld_y, long P, int C,
                                 int Cpad, float ca, float cb, float out_scale, long e_period, int dtype, void* stream) {
  RDMI_REQUIRE(x && e && y && Cpad >= C, RDMI_E_ARG, "ddim_combine: bad args");
  long n = P * Cpad;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(ddim_combine_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       ld_x, (const float*)e, ld_e, (float*)y, ld_y, P, C, Cpad, ca, cb, out_scale, e_period);
  else
    hipLaunchKernelGGL(ddim_combine_k<f16>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const f16*)x, ld_x,
                       (const f16*)e, ld_e, (f16*)y, ld_y, P, C, Cpad, ca, cb, out_scale, e_period);
  return rdmi::check_launch("ddim_combine");
}

extern "C" int rdmi_minmax(const void* x, int x_f32, long n, float* minmax, float* workspace, void* stream) {
  RDMI_REQUIRE(x && minmax && workspace && n > 0, RDMI_E_ARG, "minmax: bad args");
  unsigned g = grid_for((n + 7) / 8);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(minmax_partial, dim3(g), dim3(256), 0, (hipStream_t)stream, x, x_f32, n, workspace);
  int rc = rdmi::check_launch("minmax_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(minmax_final, dim3(1), dim3(64), 0, (hipStream_t)stream, workspace, (int)g, minmax);
  return rdmi::check_launch("minmax_final");
}

extern "C" int rdmi_renormalize_f32(float* x, long n, const float* minmax, void* stream) {
  RDMI_REQUIRE(x && minmax && n > 0, RDMI_E_ARG, "renormalize: bad args");
  hipLaunchKernelGGL(renorm_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, minmax);
  return rdmi::check_launch("renormalize");
}

extern "C" int rdmi_snippet_average(const void* src, int n, int w, int stride, int N, long P, int C, int ld, void* out,
                                    int dtype, void* stream) {
  RDMI_REQUIRE(src && out && n > 0 && w > 0 && N > 0 && ld >= C, RDMI_E_ARG, "snippet_average: bad args");
  long tot = P * ld;
  long gx = (tot + 255) / 256;
  if (gx > 4096) gx = 4096;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(snippet_average_k<float>, dim3((unsigned)gx, N), dim3(256), 0, (hipStream_t)stream,
                       (const float*)src, n, w, stride, P, C, ld, (float*)out);
  else
    hipLaunchKernelGGL(snippet_average_k<f16>, dim3((unsigned)gx, N), dim3(256), 0, (hipStream_t)stream,
                       (const f16*)src, n, w, stride, P, C, ld, (f16*)out);
  return rdmi::check_launch("snippet_average");
}

extern "C" int rdmi_snippet_accumulate(const void* src, int dtype, int k0, int nloc, int w, int stride, int N, long P,
                                       int C, int ld, double* sum, void* stream) {
  RDMI_REQUIRE(sum && N > 0 && w > 0 && ld >= C && k0 >= 0 && nloc >= 0 && (nloc == 0 || src), RDMI_E_ARG,
               "snippet_accumulate: bad args");
  long gx = (P * C + 255) / 256;
  if (gx > 4096) gx = 4096;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(snippet_accumulate_k<float>, dim3((unsigned)gx, N), dim3(256), 0, (hipStream_t)stream,
                       (const float*)src, k0, nloc, w, stride, P, C, ld, sum);
  else
    hipLaunchKernelGGL(snippet_accumulate_k<f16>, dim3((unsigned)gx, N), dim3(256), 0, (hipStream_t)stream,
                       (const f16*)src, k0, nloc, w, stride, P, C, ld, sum);
  return rdmi::check_launch("snippet_accumulate");
}

extern "C" int rdmi_snippet_finish(const double* sum, int n, int w, int stride, int N, long P, int C, int ld, void* out,
                                   int dtype, void* stream) {
  RDMI_REQUIRE(sum && out && n > 0 && w > 0 && N > 0 && ld >= C, RDMI_E_ARG, "snippet_finish: bad args");
  long gx = (P * ld + 255) / 256;
  if (gx > 4096) gx = 4096;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(snippet_finish_k<float>, dim3((unsigned)gx, N), dim3(256), 0, (hipStream_t)stream, sum, n, w,
                       stride, P, C, ld, (float*)out);
  else
    hipLaunchKernelGGL(snippet_finish_k<f16>, dim3((unsigned)gx, N), dim3(256), 0, (hipStream_t)stream, sum, n, w,
                       stride, P, C, ld, (f16*)out);
  return rdmi::check_launch("snippet_finish");
}

extern "C" int rdmi_colorize(const void* depth, int dtype, long n, const void* minmax, const unsigned char* lut,
                             int lut_n, unsigned char* rgb, int* index, void* stream) {
  RDMI_REQUIRE(depth && minmax && n > 0 && lut_n > 0 && ((lut && rgb) || index), RDMI_E_ARG, "colorize: bad args");
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(colorize_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const float*)depth, n,
                       (const float*)minmax, lut, lut_n, rgb, index);
  else
    hipLaunchKernelGGL(colorize_k<f16>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const f16*)depth, n,
                       (const f16*)minmax, lut, lut_n, rgb, index);
  return rdmi::check_launch("colorize");
}

// GroupNorm (stats + apply[+SiLU]) and LayerNorm on NHWC / token-major f16 activations.
// All three are HBM-bound streaming passes: 16-B vector loads, f64 per-thread accumulation for
// the GroupNorm moments (no E[x²]−E[x]² cancellation at 10⁵-element groups), and a fixed
// reduction order so results are bitwise reproducible run to run.
#include "common.h"

namespace {

constexpr int GN_THREADS = 256;
constexpr int GN_MAX_SPLIT = 256;

// partial[b][split][g][2] (double sums).  A thread owns one 8-channel column and a row lane,
// streams its rows with four independent 16-B loads in flight and accumulates in f32 (at most a
// few hundred rows per thread); the per-group combination of the threads' sums is f64 in a fixed
// order.
template <typename T>
__global__ __launch_bounds__(GN_THREADS) void gn_partial(const T* __restrict__ x, long HW, int C, int G,
                                                         int split, double* __restrict__ part) {
  const int CV = C >> 3;
  const int b = blockIdx.y;
  const int sp = blockIdx.x;
  const long r0 = HW * sp / split, r1 = HW * (sp + 1) / split;
  const int RL = CV >= GN_THREADS ? 1 : GN_THREADS / CV;
  const int ncol = (CV + GN_THREADS - 1) / GN_THREADS;  // ≤ 2 (C ≤ 4096)
  const int t = threadIdx.x;
  __shared__ float red[2][8][2][GN_THREADS];  // [colset][elem][sum,sumsq][thread] = 32 KB
  const int cpg = C / G;
  const T* xb = x + (long)b * HW * C;
  for (int cs = 0; cs < 2; ++cs) {
    float s[8], ss[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = ss[e] = 0.f;
    int cv, rl;
    bool active;
    if (CV >= GN_THREADS) {
      cv = t + cs * GN_THREADS;
      rl = 0;
      active = cs < ncol && cv < CV;
    } else {
      cv = t % CV;
      rl = t / CV;
      active = cs == 0 && rl < RL;
    }
    if (active) {
      const T* xp = xb + cv * 8;
      long r = r0 + rl;
      for (; r + 3 * RL < r1; r += 4 * RL) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) ld8(xp + (r + u * RL) * C, v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = v[u][e];
            s[e] += f;
            ss[e] = fmaf(f, f, ss[e]);
          }
      }
      for (; r < r1; r += RL) {
        float v[8];
        ld8(xp + r * C, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = v[e];
          s[e] += f;
          ss[e] = fmaf(f, f, ss[e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[cs][e][0][t] = s[e];
      red[cs][e][1][t] = ss[e];
    }
  }
  __syncthreads();
  // one thread per group sums its (thread, element) entries in a fixed order
  for (int g = t; g < G; g += GN_THREADS) {
    double S = 0.0, SS = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      int cvv = c >> 3, e = c & 7;
      if (CV >= GN_THREADS) {
        int tt = cvv % GN_THREADS, cs = cvv / GN_THREADS;
        S += red[cs][e][0][tt];
        SS += red[cs][e][1][tt];
      } else {
        for (int rl = 0; rl < RL; ++rl) {
          int tt = rl * CV + cvv;
          S += red[0][e][0][tt];
          SS += red[0][e][1][tt];
        }
      }
    }
    double* o = part + (((long)b * split + sp) * G + g) * 2;
    o[0] = S;
    o[1] = SS;
  }
}

__global__ void gn_finalize(const double* __restrict__ part, int B, int G, int split, double n, float eps,
                            float* __restrict__ mean_rstd) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * G) return;
  int b = i / G, g = i % G;
  double S = 0.0, SS = 0.0;
  for (int sp = 0; sp < split; ++sp) {
    const double* o = part + (((long)b * split + sp) * G + g) * 2;
    S += o[0];
    SS += o[1];
  }
  double mean = S / n;
  double var = SS / n - mean * mean;
  if (var < 0) var = 0;
  mean_rstd[2 * i] = (float)mean;
  mean_rstd[2 * i + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// Statistics from producer-emitted 32-row × 4-channel moments: one workgroup per (group, image);
// thread t sums entries t, t+256, … of the group's [vec][block] range in f64, then a fixed-order
// tree reduction.  The per-image work (and so every rounding) does not depend on B.
__global__ __launch_bounds__(256) void gn_from_partials(const float* __restrict__ part, long ld, long HW, int C,
                                                        int G, float eps, float* __restrict__ mean_rstd) {
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int cpg = C / G;
  const int nv = cpg >> 2;
  const long nb = HW >> 5;
  const long total = nv * nb;
  const float* base = part + (long)(g * nv) * ld + (long)b * nb * 2;
  double S = 0.0, SS = 0.0;
  // 8 independent loads in flight per thread, summed in the same per-thread order as one at a time.
  // Element i = v·nb + k: one 32-bit division per 8 elements, the rest stepped (a 64-bit division
  // per element was most of this kernel's time — 25 µs a launch at the VAE's 768² shapes).
  constexpr int U = 8;
  const unsigned nbu = (unsigned)nb;
  // a step of 256 elements = dq whole rows of nb + dr: one compare per element whatever nb is
  const unsigned dq = 256u / nbu, dr = 256u % nbu;
  for (long i0 = t; i0 < total; i0 += 256 * U) {
    f32x2 e[U];
    unsigned v = (unsigned)i0 / nbu, k = (unsigned)i0 - v * nbu;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const long i = i0 + 256 * j;
      e[j] = i < total ? *(const f32x2*)(base + (long)v * ld + (long)k * 2) : f32x2{0.f, 0.f};
      k += dr;
      v += dq;
      if (k >= nbu) {
        k -= nbu;
        ++v;
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i0 + 256 * j < total) {
        S += (double)e[j][0];
        SS += (double)e[j][1];
      }
  }
  __shared__ double rs[256], rq[256];
  rs[t] = S;
  rq[t] = SS;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      rs[t] += rs[t + o];
      rq[t] += rq[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double n = (double)HW * cpg;
    const double mean = rs[0] / n;
    double var = rq[0] / n - mean * mean;
    if (var < 0) var = 0;
    const int i = b * G + g;
    mean_rstd[2 * i] = (float)mean;
    mean_rstd[2 * i + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// Streaming apply: each thread owns one 8-channel column (its 16 scale/shift values stay in
// registers) and walks rows; no per-element division, 16-B loads/stores.  SILU is a template
// argument (dispatched once per launch): as a runtime flag hipcc if-converts it, computing and
// discarding a SiLU per element of every non-SiLU apply.
template <typename T, bool SILU, int U>
__global__ __launch_bounds__(256) void gn_apply(const T* __restrict__ x, T* __restrict__ y, long HW, int C,
                                                int G, int rows_per_block, const float* __restrict__ mr,
                                                const float* __restrict__ gamma, const float* __restrict__ beta) {
  const int CV = C >> 3;
  const int cpg = C / G;
  const int b = blockIdx.y;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = r0 + rows_per_block < HW ? r0 + rows_per_block : HW;
  const int NT = blockDim.x;
  const int RL = CV >= NT ? 1 : NT / CV;
  const int t = threadIdx.x;
  const T* xb = x + (long)b * HW * C;
  T* yb = y + (long)b * HW * C;
  for (int cv0 = 0; cv0 < CV; cv0 += (CV >= NT ? NT : CV)) {
    int cv, rl;
    if (CV >= NT) {
      cv = cv0 + t;
      rl = 0;
      if (cv >= CV) break;
    } else {
      cv = t % CV;
      rl = t / CV;
      if (rl >= RL) break;
    }
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int c = cv * 8 + e;
      int g = c / cpg;
      float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
      sc[e] = rstd * gamma[c];
      sh[e] = beta[c] - mean * sc[e];
    }
    auto apply = [&](const float (&in)[8], long r) __attribute__((always_inline)) {
      float out[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float f = fmaf(in[e], sc[e], sh[e]);
        if constexpr (SILU) f = sizeof(T) == 2 ? silu_f(f) : f / (1.0f + expf(-f));
        out[e] = f;
      }
      st8(yb + r * C + cv * 8, out);
    };
    long r = r0 + rl;
    // U rows per trip, their loads issued together (U × 16 B in flight per thread instead of one row):
    // U = 4 moves 4.7-5.0 TB/s against 4.4-4.8 for one row (RDMI_GN_APPLY_U=1) and 4.5 for U = 8, bitwise
    // the same outputs (tools/gn_apply_probe.py, profiles/r05zk_gn_apply_probe2.log)
    for (; r + (U - 1) * RL < r1; r += U * RL) {
      float in[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) ld8(xb + (r + u * RL) * C + cv * 8, in[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) apply(in[u], r + u * RL);
    }
    for (; r < r1; r += RL) {
      float in[8];
      ld8(xb + r * C + cv * 8, in);
      apply(in, r);
    }
  }
}

// one wave per row; C ≤ 64*8*4 = 2048
// One wave per row, grid-stride over rows: the lane's columns are fixed, so gamma/beta live in
// registers (loaded once per wave, not per row), and the next row is loaded one row ahead.
template <typename T, int NV>  // 8-element vectors per lane: C ≤ 512·NV
__global__ __launch_bounds__(256) void layernorm_k(const T* __restrict__ x, T* __restrict__ y, long M, int C,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   float eps) {
  const int lane = threadIdx.x & 63;
  const int CV = C >> 3;
  float gr[NV][8], br[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int cv = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cv < CV ? cv * 8 + e : 0;
      gr[i][e] = gamma[c];
      br[i][e] = beta[c];
    }
  }
  const long stride = gridDim.x * 4L;
  long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  float vn[NV][8];
  auto load = [&](long r) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int cv = lane + 64 * i;
      if (r < M && cv < CV) ld8(x + r * C + cv * 8, vn[i]);
    }
  };
  load(row);
  for (; row < M; row += stride) {
    float v[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = vn[i][e];
    load(row + stride);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (lane + 64 * i < CV)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[i][e];
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (lane + 64 * i < CV)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[i][e] - mean;
          q += d * d;
        }
    const float rstd = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int cv = lane + 64 * i;
      if (cv < CV) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * gr[i][e] + br[i][e];
        st8(y + row * C + cv * 8, o);
      }
    }
  }
}

// Split count depends on HW only (not on B), so a sample's statistics are bitwise identical
// however many samples share the launch (snippet batching invariance).
int gn_split(int /*B*/, long HW, int C) {
  long s = (HW * C + 131071) / 131072;  // ~128 K elements per workgroup
  if (s > GN_MAX_SPLIT) s = GN_MAX_SPLIT;
  if (s > HW) s = HW;
  if (s < 1) s = 1;
  return (int)s;
}

}  // namespace

extern "C" long rdmi_groupnorm_workspace(int B, int G) { return (long)B * GN_MAX_SPLIT * G * 4; }

extern "C" int rdmi_groupnorm_stats(const void* x, int dtype, int B, long HW, int C, int G, float eps, float* mean_rstd,
                                    float* workspace, void* stream) {
  RDMI_REQUIRE(x && mean_rstd && workspace, RDMI_E_ARG, "groupnorm_stats: null pointer");
  RDMI_REQUIRE(C % 8 == 0 && G > 0 && C % G == 0 && C <= 4096 && B > 0 && HW > 0, RDMI_E_ARG,
               "groupnorm_stats: bad C=%d G=%d", C, G);
  RDMI_REQUIRE(((uintptr_t)workspace & 7) == 0, RDMI_E_ALIGN, "groupnorm_stats: workspace not 8-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  int split = gn_split(B, HW, C);
  double* part = (double*)workspace;
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(gn_partial<float>, dim3(split, B), dim3(GN_THREADS), 0, s, (const float*)x, HW, C, G, split, part);
  else
    hipLaunchKernelGGL(gn_partial<f16>, dim3(split, B), dim3(GN_THREADS), 0, s, (const f16*)x, HW, C, G, split, part);
  int rc = rdmi::check_launch("groupnorm_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(gn_finalize, dim3(rdmi::div_up(B * G, 256)), dim3(256), 0, s, part, B, G, split,
                     (double)HW * (C / G), eps, mean_rstd);
  return rdmi::check_launch("groupnorm_finalize");
}

extern "C" int rdmi_groupnorm_stats_partials(const float* part, long part_ld, int B, long HW, int C, int G,
                                             float eps, float* mean_rstd, void* stream) {
  RDMI_REQUIRE(part && mean_rstd, RDMI_E_ARG, "groupnorm_stats_partials: null pointer");
  RDMI_REQUIRE(G > 0 && C % G == 0 && (C / G) % 4 == 0 && HW % 32 == 0 && B > 0 && part_ld >= (long)B * HW / 16,
               RDMI_E_ARG, "groupnorm_stats_partials: needs (C/G) %% 4 == 0 and HW %% 32 == 0 (C=%d G=%d HW=%ld)", C, G,
               HW);
  hipLaunchKernelGGL(gn_from_partials, dim3(G, B), dim3(256), 0, (hipStream_t)stream, part, part_ld, HW, C, G, eps,
                     mean_rstd);
  return rdmi::check_launch("groupnorm_stats_partials");
}

namespace {

// Input-GroupNorm table of the fused halo conv (rdmi_conv_args.in_affine): the scale / shift of
// gn_apply, written per image and 64-channel block as [2][64].
__global__ __launch_bounds__(256) void gn_affine_k(const float* __restrict__ mr, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int B, int C, int G,
                                                   float* __restrict__ out) {
  const int cpg = C / G;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < (long)B * C; i += (long)gridDim.x * 256) {
    const int b = (int)(i / C), c = (int)(i - (long)b * C);
    const int g = c / cpg;
    const float mean = mr[2 * (b * G + g)], rstd = mr[2 * (b * G + g) + 1];
    const float sc = rstd * gamma[c];
    const float sh = beta[c] - mean * sc;
    float* o = out + ((long)b * (C >> 6) + (c >> 6)) * 128 + (c & 63);
    o[0] = sc;
    o[64] = sh;
  }
}

}  // namespace

extern "C" int rdmi_groupnorm_affine(const float* mean_rstd, const float* gamma, const float* beta, int B, int C,
                                     int G, float* out, void* stream) {
  RDMI_REQUIRE(mean_rstd && gamma && beta && out, RDMI_E_ARG, "groupnorm_affine: null pointer");
  RDMI_REQUIRE(B > 0 && C > 0 && C % 64 == 0 && G > 0 && C % G == 0, RDMI_E_ARG, "groupnorm_affine: bad B=%d C=%d G=%d",
               B, C, G);
  long n = (long)B * C;
  long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(gn_affine_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, mean_rstd, gamma, beta,
                     B, C, G, out);
  return rdmi::check_launch("groupnorm_affine");
}

extern "C" int rdmi_groupnorm_apply(const void* x, void* y, int dtype, int B, long HW, int C, int G, const float* mean_rstd,
                                    const float* gamma, const float* beta, int silu, void* stream) {
  RDMI_REQUIRE(x && y && mean_rstd && gamma && beta, RDMI_E_ARG, "groupnorm_apply: null pointer");
  RDMI_REQUIRE(C % 8 == 0 && C % G == 0, RDMI_E_ARG, "groupnorm_apply: bad C=%d G=%d", C, G);
  const int CV = C / 8;
  const int T = CV >= 256 ? 256 : (256 / CV) * CV;
  const int RL = CV >= T ? 1 : T / CV;
  // ~2048 workgroups over the whole tensor, at least RL rows (one pass of the row lanes) each
  long rpb = ((long)HW * B + 2047) / 2048;
  if (rpb < RL) rpb = RL;
  rpb = (rpb + RL - 1) / RL * RL;
  dim3 g((unsigned)((HW + rpb - 1) / rpb), B);
  hipStream_t st = (hipStream_t)stream;
  const char* ue = getenv("RDMI_GN_APPLY_U");
  const bool u1 = ue && ue[0] == '1';
#define RDMI_GN_APPLY(TT, S)                                                                                       \
  do {                                                                                                             \
    if (u1)                                                                                                        \
      hipLaunchKernelGGL((gn_apply<TT, S, 1>), g, dim3(T), 0, st, (const TT*)x, (TT*)y, HW, C, G, (int)rpb, mean_rstd, \
                         gamma, beta);                                                                             \
    else                                                                                                           \
      hipLaunchKernelGGL((gn_apply<TT, S, 4>), g, dim3(T), 0, st, (const TT*)x, (TT*)y, HW, C, G, (int)rpb, mean_rstd, \
                         gamma, beta);                                                                             \
  } while (0)
  if (dtype == RDMI_F32) {
    if (silu)
      RDMI_GN_APPLY(float, true);
    else
      RDMI_GN_APPLY(float, false);
  } else {
    if (silu)
      RDMI_GN_APPLY(f16, true);
    else
      RDMI_GN_APPLY(f16, false);
  }
#undef RDMI_GN_APPLY
  return rdmi::check_launch("groupnorm_apply");
}

template <typename T>
int layernorm_launch(const void* x, void* y, long M, int C, const float* gamma, const float* beta, float eps,
                     hipStream_t st) {
  long blocks = (M + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  const int nv = (C / 8 + 63) / 64;
  const T* xi = (const T*)x;
  T* yo = (T*)y;
  if (nv == 1)
    hipLaunchKernelGGL((layernorm_k<T, 1>), dim3((unsigned)blocks), dim3(256), 0, st, xi, yo, M, C, gamma, beta, eps);
  else if (nv == 2)
    hipLaunchKernelGGL((layernorm_k<T, 2>), dim3((unsigned)blocks), dim3(256), 0, st, xi, yo, M, C, gamma, beta, eps);
  else if (nv == 3)
    hipLaunchKernelGGL((layernorm_k<T, 3>), dim3((unsigned)blocks), dim3(256), 0, st, xi, yo, M, C, gamma, beta, eps);
  else
    hipLaunchKernelGGL((layernorm_k<T, 4>), dim3((unsigned)blocks), dim3(256), 0, st, xi, yo, M, C, gamma, beta, eps);
  return rdmi::check_launch("layernorm");
}

extern "C" int rdmi_layernorm(const void* x, void* y, int dtype, long M, int C, const float* gamma, const float* beta,
                              float eps, void* stream) {
  RDMI_REQUIRE(x && y && gamma && beta, RDMI_E_ARG, "layernorm: null pointer");
  RDMI_REQUIRE(C % 8 == 0 && C <= 2048 && M > 0, RDMI_E_ARG, "layernorm: bad C=%d", C);
  if (dtype == RDMI_F32) return layernorm_launch<float>(x, y, M, C, gamma, beta, eps, (hipStream_t)stream);
  return layernorm_launch<f16>(x, y, M, C, gamma, beta, eps, (hipStream_t)stream);
}

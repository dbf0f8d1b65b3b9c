// DepthAligner on device (rollingdepth/depth_aligner.py).
//
// The reference runs 2000 Adam iterations of per-snippet scale/shift optimisation through
// autograd, with three host syncs per iteration (loss.item(), summ.min/max, :213).  Here one
// iteration is three kernels with no host involvement:
//   frame_stats  — per frame f and subsampled pixel p, the mean over every covering (dilation,
//                  slot) of A = x·s + t and of 1/clip(A, 1e-3) (the M / M_depth / B scatter and
//                  the .sum(0)/B.sum(0) of :169-191, summed in the reference's row order), plus
//                  the per-frame L1 scales mean|T| (:197-198) and min/max for the loss history;
//   snippet_grad — per snippet the analytic gradient of the L1 + inverse-depth L1 loss
//                  (:200-203) w.r.t. its s and t (sign(A−T)/scale, the clip mask A ≥ 1e-3, the
//                  −1/clip² of pow(−1)), reduced in f64 in a fixed order (deterministic);
//   adam         — soft constraints λ2·mean(relu(1−s)²) + λ3·mean(t²) (:205-209) and
//                  torch.optim.Adam's single-tensor update in its exact f32 op order (lerp,
//                  mul+addcmul, sqrt/bc2_sqrt + eps, addcdiv), loss history row.
// merge        — merge_scaled_triplets (:231-262): per frame the mean over all covering slots of
//                s·x+t, rounded through the snippet dtype where the reference computes in it.
//
// Snippet lengths may differ per dilation (rollingdepth_pipeline.py:221-226).  The reference then
// scatters dilation i's slot j into row i·w_i + j of its [Σw, N, P] tensors M / M_depth / B
// (depth_aligner.py:169-188): rows of different dilations can coincide, and the later dilation's
// value overwrites the earlier one's at every frame both cover (B stays 1; the overwritten slot
// gets no gradient).  With one length for all dilations the rows are disjoint and the loops below
// reduce to the plain per-dilation, per-slot order.
#pragma clang fp contract(off)
#include <type_traits>

#include "common.h"

namespace {

constexpr int MAXD = 8;
constexpr int MAXR = 64;  // rows Σ w_d of the reference's M / M_depth / B tensors
// Pixel chunks per frame / per snippet: frame_stats and snippet_grad run N·PS and ntot·PS
// workgroups (one workgroup per frame or snippet alone left most of the 256 CUs idle and each
// latency-bound), partial sums combined in a fixed chunk order by the consumer (deterministic).
constexpr int PS = 8;

struct AlP {
  const float* x[MAXD];
  float* s[MAXD];
  float* t[MAXD];
  int n[MAXD], stride[MAXD], off[MAXD];  // off: first global snippet index of dilation d
  int w[MAXD], rb[MAXD];                 // snippet length, first row (d·w_d) of dilation d
  int nd, R, N;                          // R = Σ w_d rows
  long P;
  float lr, b1, b2, eps, lmda2, lmda3, dw, ls;
  // workspace views
  float *T, *Td;
  double* fpart;  // [N][PS][4]: Σ|T|, Σ|Td|, min T, max T over pixel chunk c of frame f
  double *gs, *gt, *l1, *l2;  // [ntot][PS]: per snippet and pixel chunk
  float *m, *v;  // Adam moments [2*Ntot] (s then t)
  const double* bct;  // [iters + 1][2]: Adam's bias corrections 1 − β1^step, 1 − β2^step (adam_bc_k)
  float* hist;
  int ntot;
};

__device__ __forceinline__ float mulrn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float addrn(float a, float b) { return __fadd_rn(a, b); }

template <int BS>
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  for (int i = 0; i < BS / 64; ++i) r += sh[i];
  return r;
}

__device__ __forceinline__ long chunk_lo(long P, int c) { return P * c / PS; }

// The (dilation, snippet) whose slot holds row r of frame f in the reference's scatter (the LAST
// dilation writing that position), or d = -1 when no dilation covers it.
__device__ __forceinline__ int row_owner(const AlP& p, int r, int f, int& k_out) {
  for (int d = p.nd - 1; d >= 0; --d) {
    const int j = r - p.rb[d];
    if (j < 0 || j >= p.w[d]) continue;
    const int k = f - j * p.stride[d];
    if (k < 0 || k >= p.n[d]) continue;
    k_out = k;
    return d;
  }
  return -1;
}

// Block sums of NV doubles at once, each in block_sum_d's order (the xor butterfly inside a wave,
// then the 4 wave partials in wave order): one LDS round instead of NV.  Result valid in thread 0.
template <int NV>
__device__ __forceinline__ void block_sums_d(double (&v)[NV]) {
  __shared__ double sh[NV][4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += __shfl_xor(v[i], o, 64);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) sh[i][threadIdx.x >> 6] = v[i];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      double r = 0.0;
      for (int w = 0; w < 4; ++w) r += sh[i][w];
      v[i] = r;
    }
}

// One (frame f, pixel chunk c) work unit of frame_stats; thread 0 returns the chunk's min/max of T.
__device__ __forceinline__ void frame_stats_body(const AlP& p, int f, int c, float& mn_out, float& mx_out) {
  // the slots covering frame f in row order (block-uniform): snippet row pointer, s, t — one row
  // per lane of wave 0 (R <= MAXR = 64), compacted in row order by a ballot
  __shared__ const float* ex[MAXR];
  __shared__ float es[MAXR], et[MAXR];
  __shared__ int ecnt;
  if (threadIdx.x < 64) {
    const int r = threadIdx.x;
    int k = 0;
    const int d = r < p.R ? row_owner(p, r, f, k) : -1;
    const unsigned long long m = __ballot(d >= 0);
    if (d >= 0) {
      const int slot = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      ex[slot] = p.x[d] + ((long)k * p.w[d] + (r - p.rb[d])) * p.P;
      es[slot] = p.s[d][k];
      et[slot] = p.t[d][k];
    }
    if (r == 0) ecnt = __popcll(m);
  }
  __syncthreads();
  const int cnt = ecnt;
  double sa = 0.0, sd = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  const long p1 = chunk_lo(p.P, c + 1);
  // UP pixels per thread per round, the covering slots' values loaded EB slots at a time: a round's
  // loads are issued together instead of one dependent round trip per (pixel, slot).  The same sums
  // in the same order (slots in row order per pixel, pixels in increasing order per thread).
  constexpr int UP = 4, EB = 4;
  for (long pb = chunk_lo(p.P, c) + threadIdx.x; pb < p1; pb += 256 * UP) {
    float sum[UP], sumd[UP];
#pragma unroll
    for (int u = 0; u < UP; ++u) sum[u] = sumd[u] = 0.f;
    for (int e0 = 0; e0 < cnt; e0 += EB) {
      float xv[EB][UP];
#pragma unroll
      for (int q = 0; q < EB; ++q) {
        const float* xr = ex[e0 + q < cnt ? e0 + q : cnt - 1];
#pragma unroll
        for (int u = 0; u < UP; ++u) {
          const long px = pb + 256L * u;
          xv[q][u] = (e0 + q < cnt && px < p1) ? xr[px] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < EB; ++q) {
        if (e0 + q >= cnt) break;
        const float se = es[e0 + q], te = et[e0 + q];
#pragma unroll
        for (int u = 0; u < UP; ++u) {
          float a = addrn(mulrn(xv[q][u], se), te);
          float ac = fmaxf(a, 1e-3f);
          sum[u] = addrn(sum[u], a);
          sumd[u] = addrn(sumd[u], 1.0f / ac);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const long px = pb + 256L * u;
      if (px >= p1) break;
      float T = 0.f, Td = 0.f;
      if (cnt) {
        T = sum[u] / (float)cnt;
        Td = sumd[u] / (float)cnt;
      }
      p.T[(long)f * p.P + px] = T;
      p.Td[(long)f * p.P + px] = Td;
      sa += fabs((double)T);
      sd += fabs((double)Td);
      mn = fminf(mn, T);
      mx = fmaxf(mx, T);
    }
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  __shared__ float r[2][4];
  if ((threadIdx.x & 63) == 0) {
    r[0][threadIdx.x >> 6] = mn;
    r[1][threadIdx.x >> 6] = mx;
  }
  double v[2] = {sa, sd};
  block_sums_d<2>(v);  // its barrier also publishes r
  if (threadIdx.x == 0) {
    double* o = p.fpart + ((long)f * PS + c) * 4;
    o[0] = v[0];
    o[1] = v[1];
    mn_out = fminf(fminf(r[0][0], r[0][1]), fminf(r[0][2], r[0][3]));
    mx_out = fmaxf(fmaxf(r[1][0], r[1][1]), fmaxf(r[1][2], r[1][3]));
  }
}

__global__ __launch_bounds__(256) void frame_stats(AlP p) {
  const int f = blockIdx.x, c = blockIdx.y;
  float mn, mx;
  frame_stats_body(p, f, c, mn, mx);
  if (threadIdx.x == 0) {
    double* o = p.fpart + ((long)f * PS + c) * 4;
    o[2] = mn;
    o[3] = mx;
  }
}

// per-frame L1 scales mean|T|, mean|Td| (:197-198) from the chunk partials, chunk order fixed
__device__ __forceinline__ void frame_scales(const AlP& p, int f, float& sc, float& scd) {
  double A = 0.0, D = 0.0;
  for (int c = 0; c < PS; ++c) {
    A += p.fpart[((long)f * PS + c) * 4];
    D += p.fpart[((long)f * PS + c) * 4 + 1];
  }
  sc = (float)(A / (double)p.P);
  scd = (float)(D / (double)p.P);
}

// One (global snippet gk, pixel chunk c) work unit of snippet_grad; the loss partials go to
// l1o[gk·PS + c], l2o[gk·PS + c].  COHERENT: the gradient partials are stored as agent-scope atomics
// (device-coherent, read by another workgroup in the same launch).
template <bool COHERENT>
__device__ __forceinline__ void snippet_grad_body(const AlP& p, int gk, int c, double* l1o, double* l2o) {
  const long p0 = chunk_lo(p.P, c), p1 = chunk_lo(p.P, c + 1);
  int d = 0;
  while (d + 1 < p.nd && gk >= p.off[d + 1]) ++d;
  const int k = gk - p.off[d];
  const float s = p.s[d][k], t = p.t[d][k];
  const float* x = p.x[d] + (long)k * p.w[d] * p.P;
  double gs = 0.0, gt = 0.0, l1 = 0.0, l2 = 0.0;
  for (int j = 0; j < p.w[d]; ++j) {
    const int f = k + j * p.stride[d];
    int kk = 0;
    if (row_owner(p, p.rb[d] + j, f, kk) != d) continue;  // overwritten by a later dilation's slot
    const float* Tf = p.T + (long)f * p.P;
    const float* Tdf = p.Td + (long)f * p.P;
    // UP pixels per thread per round: the round's operand loads and the frame's scale partials are
    // issued together; the same terms accumulate in the same order (pixels increasing per thread)
    constexpr int UP = 4;
    for (long pb = p0 + threadIdx.x; pb < p1; pb += 256 * UP) {
      float xa[UP], ta[UP], tda[UP];
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const long px = pb + 256L * u;
        const bool ok = px < p1;
        xa[u] = ok ? x[(long)j * p.P + px] : 0.f;
        ta[u] = ok ? Tf[px] : 0.f;
        tda[u] = ok ? Tdf[px] : 0.f;
      }
      float scf, scdf;
      frame_scales(p, f, scf, scdf);
      const float isc = 1.0f / scf, iscd = 1.0f / scdf;
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        if (pb + 256L * u >= p1) break;
        const float xv = xa[u];
        float a = addrn(mulrn(xv, s), t);
        float z = a - ta[u];
        float ac = fmaxf(a, 1e-3f);
        float ad = 1.0f / ac;
        float zd = ad - tda[u];
        float g1 = (z > 0.f ? 1.f : (z < 0.f ? -1.f : 0.f)) * isc;
        float g2 = 0.f;
        if (a >= 1e-3f) g2 = (zd > 0.f ? 1.f : (zd < 0.f ? -1.f : 0.f)) * iscd * (-1.0f / (ac * ac));
        double g = (double)g1 + (double)p.dw * (double)g2;
        gs += g * (double)xv;
        gt += g;
        l1 += fabs((double)z) * (double)isc;
        l2 += fabs((double)zd) * (double)iscd;
      }
    }
  }
  double v[4] = {gs, gt, l1, l2};
  block_sums_d<4>(v);
  gs = v[0], gt = v[1], l1 = v[2], l2 = v[3];
  if (threadIdx.x == 0) {
    const long o = (long)gk * PS + c;
    if (COHERENT) {
      __hip_atomic_store(&p.gs[o], gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&p.gt[o], gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      p.gs[o] = gs;
      p.gt[o] = gt;
    }
    l1o[o] = l1;
    l2o[o] = l2;
  }
}

__global__ __launch_bounds__(256) void snippet_grad(AlP p) {
  snippet_grad_body<false>(p, blockIdx.x, blockIdx.y, p.l1, p.l2);
}

// Loss-history row of iteration `step` (the closure's loss.item(), summ.min(), summ.max(), :213) from
// that iteration's loss partials l1/l2 [ntot·PS], chunk min/max mm(i) over N·PS chunks and the
// parameters BEFORE its update (sflat = [s | t] by global snippet index, or NULL: p.s / p.t).
template <typename MM>
__device__ __forceinline__ void hist_row(const AlP& p, int step, double denom, const double* l1, const double* l2,
                                         const float* sflat, MM mm) {
  __shared__ double sh[8];
  double L1 = 0.0, L2 = 0.0, soft = 0.0;
  for (int i = threadIdx.x; i < p.ntot * PS; i += 256) {
    L1 += l1[i];
    L2 += l2[i];
  }
  L1 = block_sum_d<256>(L1, sh);
  L2 = block_sum_d<256>(L2, sh);
  for (int d = 0; d < p.nd; ++d) {
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < p.n[d]; k += 256) {
      const float sv = sflat ? sflat[p.off[d] + k] : p.s[d][k];
      const float tv = sflat ? sflat[p.ntot + p.off[d] + k] : p.t[d][k];
      float r = fmaxf(0.f, 1.f - sv);
      a += (double)r * r;
      b += (double)tv * tv;
    }
    a = block_sum_d<256>(a, sh);
    b = block_sum_d<256>(b, sh);
    soft += p.lmda2 * a / p.n[d] + p.lmda3 * b / p.n[d];
  }
  float mn = INFINITY, mx = -INFINITY;
  for (long i = threadIdx.x; i < (long)p.N * PS; i += 256) {
    float lo, hi;
    mm(i, lo, hi);
    mn = fminf(mn, lo);
    mx = fmaxf(mx, hi);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  __shared__ float rmm[2][4];
  if ((threadIdx.x & 63) == 0) {
    rmm[0][threadIdx.x >> 6] = mn;
    rmm[1][threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    mn = fminf(fminf(rmm[0][0], rmm[0][1]), fminf(rmm[0][2], rmm[0][3]));
    mx = fmaxf(fmaxf(rmm[1][0], rmm[1][1]), fmaxf(rmm[1][2], rmm[1][3]));
    float* h = p.hist + 3L * (step - 1);
    h[0] = (float)(p.ls * (L1 / denom + p.dw * L2 / denom) + soft);
    h[1] = mn;
    h[2] = mx;
  }
  __syncthreads();
}

// torch.optim.Adam's update of parameter i (i < ntot: s of global snippet i, else t of i − ntot) at
// iteration `step`, its gradient = Σ_c of the chunk partials (chunk order fixed) · loss_scale/numel +
// the soft-constraint term.  Returns the parameter value before the update.
template <bool COHERENT>
__device__ __forceinline__ float adam_param(const AlP& p, int i, int step, double denom) {
  const double bc1 = p.bct[2 * step], bc2 = p.bct[2 * step + 1];
  const float step_size = (float)(p.lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const float lw = 1.0f - p.b1;   // lerp weight (1 - beta1)
  const float vw = 1.0f - p.b2;   // addcmul value (1 - beta2)
  const float gscale = (float)(p.ls / denom);
  const bool is_t = i >= p.ntot;
  const int gk = is_t ? i - p.ntot : i;
  int d = 0;
  while (d + 1 < p.nd && gk >= p.off[d + 1]) ++d;
  const int k = gk - p.off[d];
  float* prm = is_t ? &p.t[d][k] : &p.s[d][k];
  const float pv = *prm;
  const double* gp = (is_t ? p.gt : p.gs) + (long)gk * PS;
  double gsum = 0.0;
  for (int c = 0; c < PS; ++c)
    gsum += COHERENT ? __hip_atomic_load(gp + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : gp[c];
  float g = (float)(gsum * (double)gscale);
  const float nd = (float)p.n[d];
  if (!is_t) {
    float r = fmaxf(0.f, 1.f - pv);
    g = addrn(g, mulrn(mulrn(mulrn(p.lmda2, 2.0f), r), -1.0f) / nd);
  } else {
    g = addrn(g, mulrn(mulrn(p.lmda3, 2.0f), pv) / nd);
  }
  float m = p.m[i], v = p.v[i];
  const float diff = g - m;
  m = (lw < 0.5f) ? addrn(m, mulrn(lw, diff)) : g - mulrn(diff, 1.0f - lw);
  v = addrn(mulrn(v, p.b2), mulrn(mulrn(vw, g), g));
  const float den = addrn(sqrtf(v) / bc2s, p.eps);
  *prm = addrn(pv, mulrn(-step_size, m) / den);
  p.m[i] = m;
  p.v[i] = v;
  return pv;
}

__global__ __launch_bounds__(256) void adam_step(AlP p, int step, double denom) {
  // loss history (uses the parameters BEFORE this update, like the closure's loss)
  if (p.hist)
    hist_row(p, step, denom, p.l1, p.l2, nullptr, [&](long i, float& lo, float& hi) {
      lo = (float)p.fpart[i * 4 + 2];
      hi = (float)p.fpart[i * 4 + 3];
    });
  for (int i = threadIdx.x; i < 2 * p.ntot; i += 256) adam_param<false>(p, i, step, denom);
}

// snippet_grad with Adam fused in (the default loop: two launches per iteration).  The workgroup
// that finishes the LAST pixel chunk of snippet gk (a per-snippet arrival counter) applies Adam to
// s_gk and t_gk right there: their gradients need nothing else, and every reader of s_gk, t_gk in
// this launch is one of those chunks.  The hand-off is NOT a C++ release/acquire: the partials are
// relaxed agent-scope atomic stores, thread 0 waits for them with s_waitcnt vmcnt(0) (on gfx9 —
// this library is built for gfx950 only — vmcnt counts stores, and agent-scope atomics bypass the
// non-coherent caches, so they are visible device-wide once counted), then arrives with a relaxed
// fetch_add; the last arriver reads the partials as relaxed agent-scope atomic loads.  A true
// agent-scope release/acquire writes back / invalidates the XCD's whole L2 (1.6x slower loop).
// The loss history is deferred: the iteration's loss partials (hl), pre-update parameters (hst)
// and, in frame_stats, chunk min/max (hmm) go to per-iteration slots, and aligner_history turns
// each block of HBLK iterations into rows.  Same arithmetic in the same order as snippet_grad + adam_step: bitwise the
// same results (tests/test_aligner_gpu.py::test_aligner_fused_loop_bitwise).
__global__ __launch_bounds__(256) void snippet_grad_adam(AlP p, int it, long slot, double denom, unsigned* cnt,
                                                         double* hl, float* hst) {
  const long nps = (long)p.ntot * PS;
  const int gk = blockIdx.x;
  double* l1o = hl ? hl + slot * 2 * nps : p.l1;
  snippet_grad_body<true>(p, gk, blockIdx.y, l1o, l1o + nps);
  // Hand-off without cache maintenance (see above): the partials were stored as agent-scope atomics
  // by thread 0, which waits for their completion (vmcnt) before it arrives; the last arriver reads
  // them the same way.
  __shared__ unsigned last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(&cnt[gk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == PS - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < 2) {
    const int i = threadIdx.x ? p.ntot + gk : gk;
    const float pv = adam_param<true>(p, i, it, denom);
    if (hst) hst[slot * 2 * p.ntot + i] = pv;
  }
  if (threadIdx.x == 0) cnt[gk] = 0u;  // re-armed for the next iteration (next launch)
}

__global__ __launch_bounds__(256) void frame_stats_hist(AlP p, float* hmm) {
  const int f = blockIdx.x, c = blockIdx.y;
  float mn, mx;
  frame_stats_body(p, f, c, mn, mx);
  if (hmm && threadIdx.x == 0) {
    hmm[((long)f * PS + c) * 2] = mn;
    hmm[((long)f * PS + c) * 2 + 1] = mx;
  }
}

// History rows of the fused loop for iterations it0 .. it0+gridDim.x-1, one workgroup per iteration;
// their per-iteration slots are slots 0 .. gridDim.x-1 (the loop writes iteration it into slot
// (it − 1) mod HBLK and turns every block of HBLK iterations into rows before reusing the slots).
__global__ __launch_bounds__(256) void aligner_history(AlP p, double denom, const double* hl, const float* hmm,
                                                       const float* hst, int it0) {
  const int slot = blockIdx.x, it = it0 + blockIdx.x;
  const long nps = (long)p.ntot * PS, nfs = (long)p.N * PS;
  const double* l1 = hl + (long)slot * 2 * nps;
  const float* mm = hmm + (long)slot * nfs * 2;
  hist_row(p, it, denom, l1, l1 + nps, hst + (long)slot * 2 * p.ntot, [&](long i, float& lo, float& hi) {
    lo = mm[i * 2];
    hi = mm[i * 2 + 1];
  });
}

// ---------------------------------------------------------------------------------------------
// Persistent single-launch loop (opt-in, RDMI_ALIGNER_FUSED=2, where aligner_persist_upt fits).  The two-launch
// iteration spends ≈26 µs per iteration on two dependent kernels whose work is a few µs: each
// re-reads the snippets and the per-frame means from beyond the L2 and writes them back.  Here ONE
// workgroup per frame f runs all iterations: it loads the covering slots' subsampled pixels of f
// into registers once, and per iteration computes the means T, Td of f (frame_stats), the frame's
// L1 scales, and each covering slot's gradient partials Σ_px g·x, Σ_px g (snippet_grad) — all
// frame-local, because every term of a slot's gradient lives on that slot's frame.  The partials
// (2 doubles per (snippet, slot)) are published as agent-scope atomic stores, one grid barrier
// (arrival counter, bounded spin: a grid that is not co-resident fails with an error instead of
// hanging), then EVERY workgroup applies Adam to every parameter from the same partials in the same
// order — identical copies of s, t, m, v in each workgroup's LDS, no second exchange.  Per pixel the
// arithmetic is frame_stats / snippet_grad's, in the same f32 op order; the f64 sums group the same
// terms differently (per slot, then slots in order, instead of per pixel chunk), which changes an
// f64 sum by ~1e-16 relative — below the f32 rounding of the gradient except with probability
// ~1e-9 per value (tests/test_aligner_gpu.py::test_aligner_fused_loop_bitwise checks the results bitwise
// against the two- and three-launch loops).  Measured (tools/aligner_ab.py, STAMP build): with one
// workgroup per frame and 64-lane butterflies for the block sums, 56 vs 52 ms per 2 000 iterations — the
// 14-double gradient sum alone was ≈20k cycles of cross-lane shuffles; with two workgroups per frame (each
// the frame's means over all pixels, the gradient over half the pixel rounds) and the reduce-scatter sum
// (psums16), 48.9 vs 52.4 ms.  Opt-in: the whole aligner is ≈1 % of a fast-preset step.
constexpr int PT = 1024;      // threads per workgroup (one workgroup per frame)
constexpr int PCM = 6;        // covering slots per frame held in registers (the fast preset: 3 + 3)
constexpr int PMAXS = 1024;   // snippets (ntot) whose s, t, m, v live in LDS

struct PerP {
  int iters;
  int wmax;                   // max snippet length (partial slots per snippet)
  double denom;
  long spin_limit;
  double* part;               // [2][ntot][wmax][2] gradient partials (Σ g·x, Σ g), by iteration parity
  unsigned* bar;              // [0] arrival counter, [1] error flag
  double* hl;                 // [iters][N][2] per-frame loss partials (history), or NULL
  float* hmm;                 // [iters][N][2] per-frame min / max of T (history)
  float* hst;                 // [iters][2 ntot] parameters before each update (history)
};

// Sums of NV doubles over the 1024-thread block (xor butterfly per wave, then the 16 wave partials
// in wave order); every thread gets the results.
template <int NV>
__device__ __forceinline__ void psums(double (&v)[NV], double* sh /* [16 * NV + NV] */) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += __shfl_xor(v[i], o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) sh[w * NV + i] = v[i];
  __syncthreads();
  if (threadIdx.x < NV) {
    double r = 0.0;
    for (int k = 0; k < PT / 64; ++k) r += sh[k * NV + threadIdx.x];
    sh[(PT / 64) * NV + threadIdx.x] = r;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = sh[(PT / 64) * NV + i];
  __syncthreads();  // sh reusable
}

// Sums of 16 doubles over the 1024-thread block with a reduce-scatter butterfly: at lane offsets 32, 16, 8, 4
// each lane keeps half of its values and adds the partner's copy of that half (8 + 4 + 2 + 1 shuffles instead of
// 4 × 16), so lane 4i ends with value i's wave sum after two more levels; then the 16 wave sums in wave order.
// Every thread gets the results.  (A fixed order: deterministic; the grouping differs from psums.)
__device__ __forceinline__ void psums16(double (&v)[16], double* sh /* [16 * 16 + 16] */) {
  const int lane = threadIdx.x & 63;
  double a8[8], a4[4], a2[2], a1;
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8, b2 = lane & 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) a8[i] = (b5 ? v[i + 8] : v[i]) + __shfl_xor(b5 ? v[i] : v[i + 8], 32, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) a4[i] = (b4 ? a8[i + 4] : a8[i]) + __shfl_xor(b4 ? a8[i] : a8[i + 4], 16, 64);
#pragma unroll
  for (int i = 0; i < 2; ++i) a2[i] = (b3 ? a4[i + 2] : a4[i]) + __shfl_xor(b3 ? a4[i] : a4[i + 2], 8, 64);
  a1 = (b2 ? a2[1] : a2[0]) + __shfl_xor(b2 ? a2[0] : a2[1], 4, 64);
  a1 += __shfl_xor(a1, 2, 64);
  a1 += __shfl_xor(a1, 1, 64);
  const int w = threadIdx.x >> 6;
  if ((lane & 3) == 0) sh[w * 16 + (lane >> 2)] = a1;
  __syncthreads();
  if (threadIdx.x < 16) {
    double r = 0.0;
    for (int k = 0; k < PT / 64; ++k) r += sh[k * 16 + threadIdx.x];
    sh[(PT / 64) * 16 + threadIdx.x] = r;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = sh[(PT / 64) * 16 + i];
  __syncthreads();  // sh reusable
}

// Grid barrier of iteration `it` (all N workgroups arrive once per iteration on one monotonic counter).
// Thread 0's agent-scope partial stores are complete (vmcnt) before it arrives, as in snippet_grad_adam.
__device__ __forceinline__ bool pbarrier(const PerP& q, unsigned target) {
  __shared__ int ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(q.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int good = 1;
    long n = 0;
    while (__hip_atomic_load(q.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if ((++n & 1023) == 0 &&
          (n > q.spin_limit || __hip_atomic_load(q.bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
        __hip_atomic_store(q.bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

__device__ __forceinline__ unsigned long long al_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// STAMP = 1 (diagnostic, RDMI_ALIGNER_STAMPS=1): workgroup 0 prints its cycle sums per segment.
// snippet_grad's per-(pixel, slot) terms over the pixel rounds [U0, U1) of the persistent loop
template <int U0, int U1, int UPT>
__device__ __forceinline__ void persist_grad(const AlP& p, const float (&xv)[PCM][UPT], const float (&T)[UPT],
                                             const float (&Td)[UPT], const float* se, const float* te, int cnt,
                                             float isc, float iscd, long P, int tid, double (&g)[16]) {
#pragma unroll
  for (int e = 0; e < PCM; ++e) {
    if (e < cnt) {
#pragma unroll
      for (int u = U0; u < U1; ++u) {
        if (tid + (long)u * PT < P) {
          const float xvv = xv[e][u];
          float a = addrn(mulrn(xvv, se[e]), te[e]);
          float z = a - T[u];
          float ac = fmaxf(a, 1e-3f);
          float ad = 1.0f / ac;
          float zd = ad - Td[u];
          float g1 = (z > 0.f ? 1.f : (z < 0.f ? -1.f : 0.f)) * isc;
          float g2 = 0.f;
          if (a >= 1e-3f) g2 = (zd > 0.f ? 1.f : (zd < 0.f ? -1.f : 0.f)) * iscd * (-1.0f / (ac * ac));
          double gg = (double)g1 + (double)p.dw * (double)g2;
          g[2 * e] += gg * (double)xvv;
          g[2 * e + 1] += gg;
          g[2 * PCM] += fabs((double)z) * (double)isc;
          g[2 * PCM + 1] += fabs((double)zd) * (double)iscd;
        }
      }
    }
  }
}

// H workgroups per frame (blockIdx.y = hh): each computes the frame's means and scales over all its
// pixels (cheap) and the gradient partials of its 1/H of the pixel rounds (the costly part).
template <int UPT, int H, int STAMP = 0>
__global__ __launch_bounds__(PT, 1) void aligner_persist_k(AlP p, PerP q) {
  const int f = blockIdx.x, hh = blockIdx.y, tid = threadIdx.x;
  static_assert(UPT % H == 0, "pixel rounds split evenly");
  unsigned long long st[5] = {}, tp = 0;
  auto seg = [&](int i) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long t = al_stamp();
      if (i >= 0) st[i] += t - tp;
      tp = t;
    }
  };
  const int ntot = p.ntot, np = 2 * ntot;
  __shared__ float prm[2 * PMAXS], am[2 * PMAXS], av[2 * PMAXS];
  __shared__ int egk[PCM], ej[PCM], ecnt;
  __shared__ const float* ex[PCM];
  __shared__ double sh[(PT / 64 + 1) * 16];
  __shared__ float rmm[2][PT / 64];
  // parameters (global snippet order: s then t), Adam moments zero (torch.optim.Adam's initial state)
  for (int i = tid; i < np; i += PT) {
    const int gk = i < ntot ? i : i - ntot;
    int d = 0;
    while (d + 1 < p.nd && gk >= p.off[d + 1]) ++d;
    prm[i] = i < ntot ? p.s[d][gk - p.off[d]] : p.t[d][gk - p.off[d]];
    am[i] = 0.f;
    av[i] = 0.f;
  }
  // the slots covering frame f in row order (frame_stats_body's compaction)
  if (tid < 64) {
    const int r = tid;
    int k = 0;
    const int d = r < p.R ? row_owner(p, r, f, k) : -1;
    const unsigned long long m = __ballot(d >= 0);
    const int slot = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    if (d >= 0 && slot < PCM) {
      ex[slot] = p.x[d] + ((long)k * p.w[d] + (r - p.rb[d])) * p.P;
      egk[slot] = p.off[d] + k;
      ej[slot] = r - p.rb[d];
    }
    if (r == 0) ecnt = __popcll(m);
  }
  __syncthreads();
  const int cnt = ecnt;
  if (cnt > PCM) {  // the host checks this (aligner_persist_upt); never half-run
    if (tid == 0) __hip_atomic_store(q.bar + 1, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const long P = p.P;
  float xv[PCM][UPT];
#pragma unroll
  for (int e = 0; e < PCM; ++e)
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const long px = tid + (long)u * PT;
      xv[e][u] = (e < cnt && px < P) ? ex[e][px] : 0.f;
    }
  const float gscale = (float)(p.ls / q.denom);
  const float lw = 1.0f - p.b1, vw = 1.0f - p.b2;
  seg(-1);
  for (int it = 1; it <= q.iters; ++it) {
    const int buf = it & 1;
    // this iteration's s, t of the covering slots (LDS, read where used: registers are the limit)
    __shared__ float se[PCM], te[PCM];
    if (tid < cnt) {
      se[tid] = prm[egk[tid]];
      te[tid] = prm[ntot + egk[tid]];
    }
    __syncthreads();
    // ---- frame_stats: T, Td per pixel (slots in row order), Σ|T|, Σ|Td|, min / max T
    float T[UPT], Td[UPT];
    double v2[2] = {0.0, 0.0};
    float mn = INFINITY, mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      float sum = 0.f, sumd = 0.f;
#pragma unroll
      for (int e = 0; e < PCM; ++e) {
        if (e < cnt) {
          float a = addrn(mulrn(xv[e][u], se[e]), te[e]);
          float ac = fmaxf(a, 1e-3f);
          sum = addrn(sum, a);
          sumd = addrn(sumd, 1.0f / ac);
        }
      }
      T[u] = Td[u] = 0.f;
      if (cnt) {
        T[u] = sum / (float)cnt;
        Td[u] = sumd / (float)cnt;
      }
      if (tid + (long)u * PT < P) {
        v2[0] += fabs((double)T[u]);
        v2[1] += fabs((double)Td[u]);
        mn = fminf(mn, T[u]);
        mx = fmaxf(mx, T[u]);
      }
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    if ((tid & 63) == 0) {
      rmm[0][tid >> 6] = mn;
      rmm[1][tid >> 6] = mx;
    }
    psums<2>(v2, sh);  // its barriers also publish rmm
    seg(0);
    const float scf = (float)(v2[0] / (double)P), scdf = (float)(v2[1] / (double)P);
    const float isc = 1.0f / scf, iscd = 1.0f / scdf;
    // ---- snippet_grad: per covering slot Σ g·x, Σ g; the frame's loss partials
    double g[16];  // 2 per covering slot, the two loss partials at 2·PCM, 2·PCM + 1 (PCM ≤ 7), padding
    static_assert(2 * PCM + 2 <= 16, "psums16 holds 16 values");
#pragma unroll
    for (int i = 0; i < 16; ++i) g[i] = 0.0;
    // the pixel rounds [U0, U1) of this workgroup: a uniform branch between compile-time ranges (a per-round
    // predicate was if-converted by the compiler, every workgroup then computing every round)
    if (H == 1)
      persist_grad<0, UPT>(p, xv, T, Td, se, te, cnt, isc, iscd, P, tid, g);
    else if (hh == 0)
      persist_grad<0, UPT / H>(p, xv, T, Td, se, te, cnt, isc, iscd, P, tid, g);
    else
      persist_grad<UPT / H, UPT>(p, xv, T, Td, se, te, cnt, isc, iscd, P, tid, g);
    psums16(g, sh);
    seg(1);
    if (tid == 0) {
      double* pb = q.part + (long)buf * ntot * q.wmax * H * 2;
      for (int e = 0; e < cnt; ++e) {
        double* o = pb + (((long)egk[e] * q.wmax + ej[e]) * H + hh) * 2;
        __hip_atomic_store(o, g[2 * e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 1, g[2 * e + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (q.hl) {
        const long h = (long)(it - 1) * p.N + f;
        q.hl[2 * (h * H + hh)] = g[2 * PCM];
        q.hl[2 * (h * H + hh) + 1] = g[2 * PCM + 1];
        float lo = rmm[0][0], hi = rmm[1][0];
        for (int w = 1; w < PT / 64; ++w) {
          lo = fminf(lo, rmm[0][w]);
          hi = fmaxf(hi, rmm[1][w]);
        }
        q.hmm[2 * h] = lo;
        q.hmm[2 * h + 1] = hi;
      }
    }
    seg(2);
    if (!pbarrier(q, (unsigned)it * gridDim.x * gridDim.y)) {  // not co-resident / timed out: fail loudly (NaN s, t)
      if (f == 0 && hh == 0)
        for (int i = tid; i < np; i += PT) {
          const int gk = i < ntot ? i : i - ntot;
          int d = 0;
          while (d + 1 < p.nd && gk >= p.off[d + 1]) ++d;
          (i < ntot ? p.s[d] : p.t[d])[gk - p.off[d]] = __builtin_nanf("");
        }
      return;
    }
    // ---- Adam on every parameter (adam_param's f32 op order), the same in every workgroup
    seg(3);
    const double bc1 = p.bct[2 * it], bc2 = p.bct[2 * it + 1];
    const float step_size = (float)(p.lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    const double* pb = q.part + (long)buf * ntot * q.wmax * H * 2;
    for (int i = tid; i < np; i += PT) {
      const bool is_t = i >= ntot;
      const int gk = is_t ? i - ntot : i;
      int d = 0;
      while (d + 1 < p.nd && gk >= p.off[d + 1]) ++d;
      const int k = gk - p.off[d];
      double gsum = 0.0;
      for (int j = 0; j < p.w[d]; ++j) {
        int kk = 0;
        if (row_owner(p, p.rb[d] + j, k + j * p.stride[d], kk) != d) continue;  // overwritten slot: no term
#pragma unroll
        for (int h2 = 0; h2 < H; ++h2)
          gsum += __hip_atomic_load(pb + (((long)gk * q.wmax + j) * H + h2) * 2 + (is_t ? 1 : 0), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
      }
      const float pv = prm[i];
      float gf = (float)(gsum * (double)gscale);
      const float nd = (float)p.n[d];
      if (!is_t) {
        float r = fmaxf(0.f, 1.f - pv);
        gf = addrn(gf, mulrn(mulrn(mulrn(p.lmda2, 2.0f), r), -1.0f) / nd);
      } else {
        gf = addrn(gf, mulrn(mulrn(p.lmda3, 2.0f), pv) / nd);
      }
      float m = am[i], v = av[i];
      const float diff = gf - m;
      m = (lw < 0.5f) ? addrn(m, mulrn(lw, diff)) : gf - mulrn(diff, 1.0f - lw);
      v = addrn(mulrn(v, p.b2), mulrn(mulrn(vw, gf), gf));
      const float den = addrn(sqrtf(v) / bc2s, p.eps);
      prm[i] = addrn(pv, mulrn(-step_size, m) / den);
      am[i] = m;
      av[i] = v;
      if (q.hst && f == 0 && hh == 0) q.hst[(long)(it - 1) * np + i] = pv;
    }
    __syncthreads();
    seg(4);
  }
  if constexpr (STAMP) {
    if ((f == 0 || f == gridDim.x / 2) && hh == 0 && tid == 0)
      printf("aligner_persist wg %d cycles per iteration: stats %.0f grad %.0f publish %.0f barrier %.0f adam %.0f\n", f,
             (double)st[0] / q.iters, (double)st[1] / q.iters, (double)st[2] / q.iters, (double)st[3] / q.iters,
             (double)st[4] / q.iters);
  }
  if (f == 0 && hh == 0)
    for (int i = tid; i < np; i += PT) {
      const int gk = i < ntot ? i : i - ntot;
      int d = 0;
      while (d + 1 < p.nd && gk >= p.off[d + 1]) ++d;
      (i < ntot ? p.s[d] : p.t[d])[gk - p.off[d]] = prm[i];
    }
}

// History rows of the persistent loop: iteration it0 + blockIdx.x from its per-frame partials (hist_row
// with the loss summed over frames instead of over (snippet, pixel chunk) partials)
__global__ __launch_bounds__(256) void aligner_history_frames(AlP p, double denom, const double* hl, const float* hmm,
                                                              const float* hst, int H) {
  const int it = 1 + blockIdx.x;
  const long h0 = (long)(it - 1) * p.N;
  __shared__ double sh[8];
  double L1 = 0.0, L2 = 0.0, soft = 0.0;
  for (int i = threadIdx.x; i < p.N * H; i += 256) {
    L1 += hl[2 * (h0 * H + i)];
    L2 += hl[2 * (h0 * H + i) + 1];
  }
  L1 = block_sum_d<256>(L1, sh);
  L2 = block_sum_d<256>(L2, sh);
  const float* sflat = hst + (long)(it - 1) * 2 * p.ntot;
  for (int d = 0; d < p.nd; ++d) {
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < p.n[d]; k += 256) {
      const float sv = sflat[p.off[d] + k];
      const float tv = sflat[p.ntot + p.off[d] + k];
      float r = fmaxf(0.f, 1.f - sv);
      a += (double)r * r;
      b += (double)tv * tv;
    }
    a = block_sum_d<256>(a, sh);
    b = block_sum_d<256>(b, sh);
    soft += p.lmda2 * a / p.n[d] + p.lmda3 * b / p.n[d];
  }
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < p.N; i += 256) {
    mn = fminf(mn, hmm[2 * (h0 + i)]);
    mx = fmaxf(mx, hmm[2 * (h0 + i) + 1]);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  __shared__ float r2[2][4];
  if ((threadIdx.x & 63) == 0) {
    r2[0][threadIdx.x >> 6] = mn;
    r2[1][threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    mn = fminf(fminf(r2[0][0], r2[0][1]), fminf(r2[0][2], r2[0][3]));
    mx = fmaxf(fmaxf(r2[1][0], r2[1][1]), fmaxf(r2[1][2], r2[1][3]));
    float* h = p.hist + 3L * (it - 1);
    h[0] = (float)(p.ls * (L1 / denom + p.dw * L2 / denom) + soft);
    h[1] = mn;
    h[2] = mx;
  }
}

// Adam's bias corrections of every step, once per optimisation (the same double pow the update
// evaluated per parameter before: two double pows off each iteration's critical path)
__global__ void adam_bc_k(AlP p, int iters, double* bct) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= iters; i += gridDim.x * blockDim.x) {
    bct[2 * i] = 1.0 - pow((double)p.b1, (double)i);
    bct[2 * i + 1] = 1.0 - pow((double)p.b2, (double)i);
  }
}

__global__ void zero_f32(float* x, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] = 0.f;
}

struct MergeP {
  const void* x[MAXD];
  const float* s[MAXD];
  const float* t[MAXD];
  int n[MAXD], stride[MAXD], w[MAXD];
  int k0[MAXD], nloc[MAXD];  // rows of x[d] are global snippets k0[d] .. k0[d]+nloc[d]-1
  int nd, xf32;
  int sum_only;              // 1: write the per-frame f64 sum (sharded merge) to dsum, 0: the mean to out
  int f0;                    // first frame of out (out rows are frames f0 .. f0+gridDim.y-1)
  long HW;
  const float* shift;
  float* out;
  double* dsum;
};

// number of (dilation, slot) pairs covering frame f (the B.sum(0) of depth_aligner.py:190 / the
// length of the torch.cat of :258)
__device__ __forceinline__ int cover_count(const int* n, const int* stride, int nd, const int* w, int f) {
  int cnt = 0;
  for (int d = 0; d < nd; ++d)
    for (int j = 0; j < w[d]; ++j) {
      const int k = f - j * stride[d];
      cnt += (k >= 0 && k < n[d]) ? 1 : 0;
    }
  return cnt;
}

// The f32-arithmetic merges (x_f32 1 / 2) add the slots' f32 terms s·x + t in f64: the sum of a
// frame's few (≤ Σ w_d) f32 terms is exact whenever their exponents span ≤ ≈29 bits (all but rare
// rounding cases), so it does not depend on the order the terms are added in — the sharded merge (per-rank window sums, all-to-all, pieces added per frame, finish)
// gives bitwise the single-GPU result, and both round once, at the mean.  The f16-emulating mode 0
// (the reference's fp16 merge, RDMI_MERGE_F32=0) keeps its f32 running sum.
__global__ void merge_k(MergeP p) {
  const int f = p.f0 + blockIdx.y;
  const float sh = p.shift ? p.shift[0] : 0.f;
  for (long px = blockIdx.x * (long)blockDim.x + threadIdx.x; px < p.HW; px += (long)gridDim.x * blockDim.x) {
    float sum = 0.f;
    double dsum = 0.0;
    int cnt = 0;
    for (int d = 0; d < p.nd; ++d) {
      for (int j = p.w[d] - 1; j >= 0; --j) {  // boolean-mask order over [n_d, w]: k ascending
        int k = f - j * p.stride[d];
        if (k < p.k0[d] || k >= p.k0[d] + p.nloc[d]) continue;
        long off = ((long)(k - p.k0[d]) * p.w[d] + j) * p.HW + px;
        float a;
        if (p.xf32 == 1) {
          float xs = ((const float*)p.x[d])[off] - sh;
          a = addrn(mulrn(xs, p.s[d][k]), p.t[d][k]);
        } else if (p.xf32 == 2) {  // f16 snippets, f32 arithmetic (no intermediate f16 rounding)
          float xs = (float)((const f16*)p.x[d])[off] - sh;
          a = addrn(mulrn(xs, p.s[d][k]), p.t[d][k]);
        } else {
          f16 xs = (f16)((float)((const f16*)p.x[d])[off] - sh);
          f16 sc = (f16)p.s[d][k], tr = (f16)p.t[d][k];
          f16 prod = (f16)((float)xs * (float)sc);
          a = (float)(f16)((float)prod + (float)tr);
        }
        if (p.xf32)
          dsum += (double)a;
        else
          sum = addrn(sum, a);
        ++cnt;
      }
    }
    const long o = (long)blockIdx.y * p.HW + px;
    if (p.sum_only)
      p.dsum[o] = p.xf32 ? dsum : (double)sum;
    else
      p.out[o] = p.xf32 ? (cnt ? (float)(dsum / (double)cnt) : 0.f) : (cnt ? sum / (float)cnt : 0.f);
  }
}

// sharded merge with frame windows, second half: the received pieces — piece q holds the sums of
// frames pf0[q] .. pf0[q]+pnf[q]-1 from one source rank, pieces back to back in `recv` — added per
// frame in piece (= source rank) order, ÷ the frame's cover count.  Frames of this rank's chunk that
// no piece covers are 0 (no slot covers them: cover count 0).
constexpr int MAXPIECES = 64;
struct PiecesP {
  int pf0[MAXPIECES], pnf[MAXPIECES];
  long poff[MAXPIECES];
  int np;
};

__global__ void merge_finish_pieces_k(MergeP p, PiecesP q, const double* __restrict__ recv) {
  const int fl = blockIdx.y, f = p.f0 + fl;
  const int cnt = cover_count(p.n, p.stride, p.nd, p.w, f);
  for (long px = blockIdx.x * (long)blockDim.x + threadIdx.x; px < p.HW; px += (long)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int i = 0; i < q.np; ++i)
      if (f >= q.pf0[i] && f < q.pf0[i] + q.pnf[i]) s += recv[q.poff[i] + (long)(f - q.pf0[i]) * p.HW + px];
    p.out[(long)fl * p.HW + px] = cnt ? (float)(s / (double)cnt) : 0.f;
  }
}

struct PrepP {
  const void* x;
  int xf32;
  int n, w, H, W, border, factor, Hs, Ws;
  const float* shift;
  float* out;
};

__global__ void prepare_k(PrepP p) {
  const long P = (long)p.Hs * p.Ws;
  const long total = (long)p.n * p.w * P;
  const float sh = p.shift[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long img = i / P, q = i - img * P;
    int ys = (int)(q / p.Ws), xs = (int)(q - (long)ys * p.Ws);
    long src = img * p.H * p.W + (long)(p.border + ys * p.factor) * p.W + (p.border + xs * p.factor);
    float v;
    if (p.xf32)
      v = ((const float*)p.x)[src] - sh;
    else
      v = (float)(f16)((float)((const f16*)p.x)[src] - sh);
    p.out[i] = v;
  }
}

// Iterations per block of history slots: the fused loop keeps per-iteration loss partials for at
// most HBLK iterations, so the workspace does not grow with the iteration count (1500 frames with
// [1,10,25] at 2000 iterations would otherwise need 1.4 GB).
constexpr int HBLK = 128;

// RDMI_ALIGNER_FUSED (read per call: A/B and the bitwise tests): 0 the three-kernel loop, unset / 1 the
// two-launch loop (default), 2 the persistent loop where aligner_persist_upt fits (opt-in: bitwise the
// same results, 48.9 vs 52.4 ms per 2 000 iterations at the fast preset — DESIGN App. A)
int loop_mode() {
  const char* e = getenv("RDMI_ALIGNER_FUSED");
  return e && (e[0] == '0' || e[0] == '2') ? e[0] - '0' : 1;
}

// Workspace (floats): 4 double arrays (ntot·PS each), fpart (N·PS·4 doubles), T, Td (N·P each), m, v
// (2·ntot each), the per-snippet arrival counters (ntot, padded to 8 B), the bias-correction table
// ((iters + 1)·2 doubles); with a history, the
// fused loop's per-iteration slots for min(iters, HBLK) iterations: loss partials (2·ntot·PS
// doubles), chunk min/max (2·N·PS) and pre-update parameters (2·ntot).
long ws_floats(int N, long P, int ntot, int iters, bool hist, int wmax) {
  long f = 8L * ntot * PS + 8L * N * PS + 2L * N * P + 4L * ntot + ((ntot + 1) & ~1L) + 4L * (iters + 1);
  // the persistent loop (opt-in, loop_mode 2): partials (2 parities), barrier words, per-iteration history
  if (loop_mode() == 2) f += 16L * ntot * wmax + 2 + (hist ? 10L * iters * N + 2L * iters * ntot : 0);  // H <= 2
  const long slots = iters < HBLK ? iters : HBLK;
  if (hist) f += slots * (4L * ntot * PS + 2L * N * PS + 2L * ntot) + 2;
  return f + 64;
}


// pixels per thread of the persistent loop (0: it does not fit).  Its grid is one workgroup per frame,
// all resident at once (one per CU at most is needed), ≤ PCM covering slots per frame, ≤ PMAXS snippets.
int aligner_persist_upt(const AlP& p, int iters) {
  if (iters < 1 || p.ntot > PMAXS || p.P > 6L * PT) return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || p.N > cus)
    return 0;
  for (int f = 0; f < p.N; ++f) {  // covering slots of frame f (row_owner on the host)
    int c = 0;
    for (int r = 0; r < p.R; ++r)
      for (int d = p.nd - 1; d >= 0; --d) {
        const int j = r - p.rb[d];
        if (j < 0 || j >= p.w[d]) continue;
        const int k = f - j * p.stride[d];
        if (k < 0 || k >= p.n[d]) continue;
        ++c;
        break;
      }
    if (c > PCM) return 0;
  }
  const long u = (p.P + PT - 1) / PT;
  return u <= 2 ? 2 : u <= 4 ? 4 : 6;  // 6: 123 VGPRs at 16 waves per CU, no spill (8 spills)
}

}  // namespace

extern "C" long rdmi_aligner_workspace(const rdmi_aligner_args* a) {
  int ntot = 0;
  for (int d = 0; d < a->n_dil; ++d) ntot += a->n[d];
  int wmax = 1;
  for (int d = 0; d < a->n_dil; ++d) wmax = a->w[d] > wmax ? a->w[d] : wmax;
  return ws_floats(a->seq_len, a->P, ntot, a->iters, a->history != nullptr, wmax);
}

extern "C" int rdmi_aligner_optimize(const rdmi_aligner_args* a, void* stream) {
  RDMI_REQUIRE(a && a->workspace && a->n_dil >= 1 && a->n_dil <= MAXD && a->P > 0 && a->seq_len > 0,
               RDMI_E_ARG, "aligner_optimize: bad args");
  hipStream_t st = (hipStream_t)stream;
  AlP p{};
  p.nd = a->n_dil;
  p.N = a->seq_len;
  p.P = a->P;
  int ntot = 0;
  for (int d = 0; d < p.nd; ++d) {
    RDMI_REQUIRE(a->x[d] && a->s[d] && a->t[d] && a->n[d] > 0, RDMI_E_ARG, "aligner_optimize: dilation %d", d);
    p.x[d] = a->x[d];
    p.s[d] = a->s[d];
    p.t[d] = a->t[d];
    p.n[d] = a->n[d];
    p.stride[d] = a->stride[d];
    p.off[d] = ntot;
    ntot += a->n[d];
    RDMI_REQUIRE(a->w[d] >= 1, RDMI_E_ARG, "aligner_optimize: snippet length %d of dilation %d", a->w[d], d);
    p.w[d] = a->w[d];
    p.R += a->w[d];
  }
  RDMI_REQUIRE(p.R <= MAXR, RDMI_E_ARG, "aligner_optimize: %d rows (at most %d)", p.R, MAXR);
  for (int d = 0; d < p.nd; ++d) {
    p.rb[d] = d * p.w[d];  // the reference's torch.arange(i * w, (i + 1) * w), depth_aligner.py:182-188
    RDMI_REQUIRE(a->iters == 0 || p.rb[d] + p.w[d] <= p.R, RDMI_E_ARG,
                 "aligner_optimize: dilation %d rows %d..%d exceed the %d rows (the reference raises IndexError)", d,
                 p.rb[d], p.rb[d] + p.w[d] - 1, p.R);
  }
  p.ntot = ntot;
  p.lr = a->lr; p.b1 = a->beta1; p.b2 = a->beta2; p.eps = a->eps;
  p.lmda2 = a->lmda2; p.lmda3 = a->lmda3; p.dw = a->depth_w; p.ls = a->loss_scale;
  float* w = a->workspace;
  RDMI_REQUIRE(((uintptr_t)w & 7) == 0, RDMI_E_ALIGN, "aligner: workspace must be 8-byte aligned");
  double* dw = (double*)w;
  const long nps = (long)ntot * PS;
  p.gs = dw; p.gt = dw + nps; p.l1 = dw + 2 * nps; p.l2 = dw + 3 * nps;
  p.fpart = dw + 4 * nps;
  float* fw = (float*)(p.fpart + 4L * p.N * PS);
  p.T = fw; fw += (long)p.N * p.P;
  p.Td = fw; fw += (long)p.N * p.P;
  p.m = fw; fw += 2 * ntot;
  p.v = fw; fw += 2 * ntot;
  unsigned* cnt = (unsigned*)fw; fw += (ntot + 1) & ~1L;
  double* bct = (double*)fw; fw += 4L * (a->iters + 1);
  p.bct = bct;
  p.hist = a->history;
  const double denom = (double)p.R * p.N * (double)p.P;  // numel of the [Σw, N, P] loss tensor
  hipLaunchKernelGGL(zero_f32, dim3(16), dim3(256), 0, st, p.m, 4L * ntot + ((ntot + 1) & ~1L));  // m, v, cnt
  hipLaunchKernelGGL(adam_bc_k, dim3(8), dim3(256), 0, st, p, a->iters, bct);
  int rc = rdmi::check_launch("aligner_zero");
  if (rc) return rc;
  int wmax = 1;
  for (int d = 0; d < p.nd; ++d) wmax = p.w[d] > wmax ? p.w[d] : wmax;
  const int mode = loop_mode();
  PerP q{};
  q.iters = a->iters;
  q.wmax = wmax;
  q.denom = denom;
  q.spin_limit = 1L << 22;
  if (mode == 2) {  // the region ws_floats reserves for mode 2 only
    q.part = (double*)fw; fw += 16L * ntot * wmax;
    q.bar = (unsigned*)fw; fw += 2;
    if (p.hist) {
      q.hl = (double*)fw; fw += 8L * a->iters * p.N;
      q.hmm = fw; fw += 2L * a->iters * p.N;
      q.hst = fw; fw += 2L * a->iters * ntot;
    }
  }
  const int upt = mode == 2 ? aligner_persist_upt(p, a->iters) : 0;
  if (upt) {
    hipLaunchKernelGGL(zero_f32, dim3(1), dim3(64), 0, st, (float*)q.bar, 2L);  // arrival counter, error flag
    int cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int H = (upt % 2 == 0 && 2 * p.N <= cus && !getenv("RDMI_ALIGNER_PERSIST_H1")) ? 2 : 1;
    const dim3 g(p.N, H);
    const bool stamps = getenv("RDMI_ALIGNER_STAMPS") != nullptr;
    if (H == 2) {
      if (upt == 2)
        hipLaunchKernelGGL((aligner_persist_k<2, 2>), g, dim3(PT), 0, st, p, q);
      else if (upt == 4)
        hipLaunchKernelGGL((aligner_persist_k<4, 2>), g, dim3(PT), 0, st, p, q);
      else if (stamps)
        hipLaunchKernelGGL((aligner_persist_k<6, 2, 1>), g, dim3(PT), 0, st, p, q);
      else
        hipLaunchKernelGGL((aligner_persist_k<6, 2>), g, dim3(PT), 0, st, p, q);
    } else {
      if (upt == 2)
        hipLaunchKernelGGL((aligner_persist_k<2, 1>), g, dim3(PT), 0, st, p, q);
      else if (upt == 4)
        hipLaunchKernelGGL((aligner_persist_k<4, 1>), g, dim3(PT), 0, st, p, q);
      else if (stamps)
        hipLaunchKernelGGL((aligner_persist_k<6, 1, 1>), g, dim3(PT), 0, st, p, q);
      else
        hipLaunchKernelGGL((aligner_persist_k<6, 1>), g, dim3(PT), 0, st, p, q);
    }
    rc = rdmi::check_launch("aligner_persist");
    if (rc) return rc;
    if (p.hist) {
      hipLaunchKernelGGL(aligner_history_frames, dim3(a->iters), dim3(256), 0, st, p, denom, (const double*)q.hl,
                         (const float*)q.hmm, (const float*)q.hst, H);
      return rdmi::check_launch("aligner_history");
    }
    return 0;
  }
  if (mode != 0) {
    double* hl = nullptr;
    float *hmm = nullptr, *hst = nullptr;
    const long slots = a->iters < HBLK ? a->iters : HBLK;
    if (p.hist) {
      hl = (double*)fw;
      hmm = (float*)(hl + slots * 2 * nps);
      hst = hmm + slots * 2 * p.N * PS;
    }
    int it0 = 1;  // first iteration whose history slots are not yet turned into rows
    for (int it = 1; it <= a->iters; ++it) {
      const long slot = (it - 1) % HBLK;
      hipLaunchKernelGGL(frame_stats_hist, dim3(p.N, PS), dim3(256), 0, st, p,
                         hmm ? hmm + slot * 2 * p.N * PS : nullptr);
      hipLaunchKernelGGL(snippet_grad_adam, dim3(ntot, PS), dim3(256), 0, st, p, it, slot, denom, cnt, hl, hst);
      rc = rdmi::check_launch("aligner_iteration");
      if (rc) return rc;
      if (p.hist && (it - it0 + 1 == HBLK || it == a->iters)) {
        hipLaunchKernelGGL(aligner_history, dim3(it - it0 + 1), dim3(256), 0, st, p, denom, (const double*)hl,
                           (const float*)hmm, (const float*)hst, it0);
        rc = rdmi::check_launch("aligner_history");
        if (rc) return rc;
        it0 = it + 1;
      }
    }
    return 0;
  }
  for (int it = 1; it <= a->iters; ++it) {
    hipLaunchKernelGGL(frame_stats, dim3(p.N, PS), dim3(256), 0, st, p);
    hipLaunchKernelGGL(snippet_grad, dim3(ntot, PS), dim3(256), 0, st, p);
    hipLaunchKernelGGL(adam_step, dim3(1), dim3(256), 0, st, p, it, denom);
    rc = rdmi::check_launch("aligner_iteration");
    if (rc) return rc;
  }
  return 0;
}

extern "C" int rdmi_aligner_prepare(const void* x, int x_f32, int n, int w, int H, int W, int border, int factor,
                                    const float* shift, float* out, void* stream) {
  RDMI_REQUIRE(x && shift && out && H > 2 * border && W > 2 * border && factor > 0, RDMI_E_ARG,
               "aligner_prepare: bad args");
  PrepP p{x, x_f32, n, w, H, W, border, factor, (H - 2 * border + factor - 1) / factor,
          (W - 2 * border + factor - 1) / factor, shift, out};
  long total = (long)n * w * p.Hs * p.Ws;
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(prepare_k, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, p);
  return rdmi::check_launch("aligner_prepare");
}

static int merge_launch(int n_dil, const void* const* xf, int x_f32, const float* const* s, const float* const* t,
                        const int* n, const int* stride, const int* k0, const int* nloc, const int* w, int f0, int nf,
                        long HW, const float* shift, float* out, double* dsum, void* stream) {
  RDMI_REQUIRE(n_dil >= 1 && n_dil <= MAXD && (out || dsum) && HW > 0 && nf >= 0 && f0 >= 0, RDMI_E_ARG,
               "aligner_merge: bad args");
  MergeP p{};
  for (int d = 0; d < n_dil; ++d) {
    const int kk = k0 ? k0[d] : 0, nl = nloc ? nloc[d] : n[d];
    RDMI_REQUIRE(kk >= 0 && nl >= 0 && kk + nl <= n[d] && w[d] >= 1 && (nl == 0 || (xf[d] && s[d] && t[d])),
                 RDMI_E_ARG, "aligner_merge: dilation %d rows %d+%d of %d, length %d", d, kk, nl, n[d], w[d]);
    p.x[d] = xf[d];
    p.s[d] = s[d];
    p.t[d] = t[d];
    p.n[d] = n[d];
    p.stride[d] = stride[d];
    p.k0[d] = kk;
    p.nloc[d] = nl;
    p.w[d] = w[d];
  }
  p.nd = n_dil; p.xf32 = x_f32; p.HW = HW; p.shift = shift; p.out = out; p.dsum = dsum;
  p.sum_only = dsum != nullptr; p.f0 = f0;
  if (nf == 0) return 0;
  long gx = (HW + 255) / 256;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(merge_k, dim3((unsigned)gx, nf), dim3(256), 0, (hipStream_t)stream, p);
  return rdmi::check_launch("aligner_merge");
}

extern "C" int rdmi_aligner_merge(int n_dil, const void* const* xf, int x_f32, const float* const* s,
                                  const float* const* t, const int* n, const int* stride, const int* w, int seq_len, long HW,
                                  const float* shift, float* out, void* stream) {
  RDMI_REQUIRE(out, RDMI_E_ARG, "aligner_merge: null out");
  return merge_launch(n_dil, xf, x_f32, s, t, n, stride, nullptr, nullptr, w, 0, seq_len, HW, shift, out, nullptr,
                      stream);
}

extern "C" int rdmi_aligner_merge_partial_window(int n_dil, const void* const* xf, int x_f32, const float* const* s,
                                                 const float* const* t, const int* n, const int* stride, const int* k0,
                                                 const int* nloc, const int* w, int f0, int nf, long HW,
                                                 const float* shift, double* sum_out, void* stream) {
  RDMI_REQUIRE(k0 && nloc && sum_out, RDMI_E_ARG, "aligner_merge_partial_window: k0/nloc/sum_out required");
  return merge_launch(n_dil, xf, x_f32, s, t, n, stride, k0, nloc, w, f0, nf, HW, shift, nullptr, sum_out, stream);
}

extern "C" int rdmi_aligner_merge_finish_pieces(int n_dil, const int* n, const int* stride, const int* w, int f0,
                                                int nf, long HW, int npieces, const int* piece_f0,
                                                const int* piece_nf, const double* recv, float* out, void* stream) {
  RDMI_REQUIRE(n_dil >= 1 && n_dil <= MAXD && n && stride && w && (out || nf == 0) && HW > 0 && f0 >= 0 && nf >= 0 &&
                   npieces >= 0 && (npieces == 0 || (piece_f0 && piece_nf && recv)),
               RDMI_E_ARG, "aligner_merge_finish_pieces: bad args");
  if (nf == 0) return 0;
  MergeP p{};
  for (int d = 0; d < n_dil; ++d) {
    p.n[d] = n[d];
    p.stride[d] = stride[d];
    p.w[d] = w[d];
  }
  p.nd = n_dil; p.HW = HW;
  long off = 0;
  for (int i = 0; i < npieces; ++i) {
    RDMI_REQUIRE(piece_nf[i] >= 0 && piece_f0[i] >= f0 && piece_f0[i] + piece_nf[i] <= f0 + nf, RDMI_E_ARG,
                 "aligner_merge_finish_pieces: piece %d frames %d+%d outside %d+%d", i, piece_f0[i], piece_nf[i], f0, nf);
  }
  // The piece table travels in the kernel arguments (≤ MAXPIECES entries).  More pieces than that (one
  // per source rank and dilation: 3·W > 64 from W = 22 ranks on) are split by frame: each launch takes
  // a frame range and only the pieces that touch it, in their original (source-rank) order — every
  // frame still adds all of its pieces in that order within one thread, so the sums are those of a
  // single launch.  Only a single frame touched by more than MAXPIECES pieces is refused.
  auto touches = [&](int i, int a, int b) { return piece_nf[i] > 0 && piece_f0[i] < b && piece_f0[i] + piece_nf[i] > a; };
  long gx = (HW + 255) / 256;
  if (gx > 1024) gx = 1024;
  int fs = f0;
  while (fs < f0 + nf) {
    int fe = fs + 1, cnt = 0;
    for (int i = 0; i < npieces; ++i) cnt += touches(i, fs, fe);
    RDMI_REQUIRE(cnt <= MAXPIECES, RDMI_E_UNSUPPORTED,
                 "aligner_merge_finish_pieces: frame %d is covered by %d pieces (at most %d)", fs, cnt, MAXPIECES);
    while (fe < f0 + nf) {  // grow the range while its pieces still fit the table
      int c2 = 0;
      for (int i = 0; i < npieces; ++i) c2 += touches(i, fs, fe + 1);
      if (c2 > MAXPIECES) break;
      ++fe;
    }
    PiecesP q{};
    off = 0;
    for (int i = 0; i < npieces; ++i) {
      if (touches(i, fs, fe)) {
        q.pf0[q.np] = piece_f0[i];
        q.pnf[q.np] = piece_nf[i];
        q.poff[q.np] = off;
        ++q.np;
      }
      off += (long)piece_nf[i] * HW;
    }
    p.f0 = fs;
    p.out = out + (long)(fs - f0) * HW;
    hipLaunchKernelGGL(merge_finish_pieces_k, dim3((unsigned)gx, fe - fs), dim3(256), 0, (hipStream_t)stream, p, q, recv);
    if (int rc = rdmi::check_launch("aligner_merge_finish_pieces")) return rc;
    fs = fe;
  }
  return 0;
}

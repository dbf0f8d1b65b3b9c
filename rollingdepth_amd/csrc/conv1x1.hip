// Streaming 1×1 convolution for the VAE's narrow conv_shortcut layers (resnet.py:306-313: the 768²
// 256→128 shortcut of the decoder's last up block, the encoder's 384² 128→256): y = x·Wᵀ + b per pixel.
//
// These are HBM-bound GEMMs with a tiny weight (≤ 64 KiB) and a short K (≤ 256): on the 512×128
// ping-pong tiles they moved 3.5–4.5 TB/s (tools/conv1x1_probe.py), every tile paying its prologue and
// epilogue with nothing else in flight; here 4.8–5.3 TB/s (profiles/r05zh_conv1x1_probe*.log).  Here the weight is loaded into
// LDS once per workgroup and each wave streams 32-pixel strips straight into MFMA operand registers:
// a K-step's fragments of the next strip are loaded (global_load_dwordx4, no LDS staging) as soon as
// the current strip's MFMAs of that K-step have consumed the registers, so up to 16 KiB per wave is in
// flight beside the MFMAs and the epilogue.
//
// Bitwise the ping-pong engine's outputs: the same v_mfma_f32_16x16x32_f16 per (32-channel K-step,
// 16×16 block) with the weights as operand A and the pixels as operand B, the K-steps in ascending
// order from a zero accumulator, and the same epilogue, f16(fmaf(acc, alpha, bias)) by
// v_cvt_pk_f16_f32.  Output channels are permuted in LDS (fragment pair (2q, 2q+1), fragment row c ↔
// channel 32q + 8(c >> 2) + 4·(j & 1) + (c & 3)) so that a lane's accumulators of a fragment pair
// are 8 consecutive channels of one pixel: one 16-B store.
#include <algorithm>

#include "gemm_kernels.h"

namespace rdmi_gk {

template <int KS, int NF>
__global__ __launch_bounds__(256, 2) void conv1x1_stream_kernel(GemmP p) {
  constexpr int RF = 2, SR = 16 * RF;  // 16-pixel fragments per strip, pixels per strip
  constexpr int CIN = 32 * KS, COUT = 16 * NF;
  constexpr int ROWB = CIN * 2;  // bytes per LDS weight row (a multiple of 256: conflict-free with the swizzle)
  static_assert(KS >= 4 && KS <= 8 && NF % 2 == 0 && CIN * COUT <= 32768, "conv1x1 shape");
  __shared__ __attribute__((aligned(16))) unsigned char lw[COUT * ROWB + COUT * 4];
  float* const lbias = (float*)(lw + COUT * ROWB);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;

  // weights → LDS: row R = 16j + c holds output channel ch(R); its 16-B chunk q sits at chunk q ^ c, so
  // that the 16 rows of a fragment read hit 16 distinct 4-bank groups
  for (int u = tid; u < COUT * KS * 4; u += 256) {
    const int R = u / (KS * 4), q = u - R * (KS * 4);
    const int j = R >> 4, c = R & 15;
    const int ch = 32 * (j >> 1) + 8 * (c >> 2) + 4 * (j & 1) + (c & 3);
    *(f16x8*)(lw + R * ROWB + ((q ^ c) << 4)) = *(const f16x8*)(p.Wt + (long)ch * p.ldw + q * 8);
  }
  for (int c = tid; c < COUT; c += 256) lbias[c] = p.bias ? p.bias[c] : 0.f;
  __syncthreads();

  const long S = (p.M + SR - 1) / SR;  // strips
  const long nwv = (long)gridDim.x * 4;
  long s = (long)blockIdx.x * 4 + wid;
  if (s >= S) return;  // no barrier follows

  // operand B fragments of a strip: pixel 32s + 16rf + fr, channels 32ks + 8g .. +7.  One register set,
  // refilled as it is consumed: a K-step's fragments of the NEXT strip are loaded right after the
  // K-step's MFMAs, so they have the rest of this strip (the later K-steps and the epilogue) to land.
  f16x8 a[RF][KS];
  auto load = [&](long st, int rf, int ks) __attribute__((always_inline)) {
    const long row = st * SR + rf * 16 + fr;
    f16x8 z = {};
    a[rf][ks] = row < p.M ? *(const f16x8*)(p.A + row * p.lda + 8 * g + 32 * ks) : z;
  };
  auto wread = [&](int ks, int j) __attribute__((always_inline)) {
    return *(const f16x8*)(lw + (16 * j + fr) * ROWB + (((4 * ks + g) ^ fr) << 4));
  };
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) load(s, rf, ks);
  for (; s < S; s += nwv) {
    const long sn = s + nwv;
    const bool more = sn < S;
    f32x4 acc[RF][NF];
#pragma unroll
    for (int rf = 0; rf < RF; ++rf)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[rf][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // weight fragments (K-step ks, fragment j) read from LDS two steps ahead of their two MFMAs; the
    // sched_barrier per step keeps hipcc from hoisting all KS·NF reads (4 registers each) to the top
    constexpr int T = KS * NF;
    f16x8 wb[3];
#pragma unroll
    for (int t = 0; t < 2; ++t) wb[t] = wread(t / NF, t % NF);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int ks = t / NF, j = t % NF;
      if (t + 2 < T) wb[(t + 2) % 3] = wread((t + 2) / NF, (t + 2) % NF);
#pragma unroll
      for (int rf = 0; rf < RF; ++rf)
        acc[rf][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb[t % 3], a[rf][ks], acc[rf][j], 0, 0, 0);
      if (j == NF - 1 && more) {
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) load(sn, rf, ks);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const long row = s * SR + rf * 16 + fr;
      if (row < p.M) {
        f16* const crow = (f16*)p.C + row * p.ldc + 8 * g;
#pragma unroll
        for (int q = 0; q < NF / 2; ++q) {
          const f32x4 b0 = *(const f32x4*)(lbias + 32 * q + 8 * g), b1 = *(const f32x4*)(lbias + 32 * q + 8 * g + 4);
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = fmaf(acc[rf][2 * q][e], p.alpha, b0[e]);
            v[4 + e] = fmaf(acc[rf][2 * q + 1][e], p.alpha, b1[e]);
          }
          unsigned w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(w[e]) : "v"(v[2 * e]), "v"(v[2 * e + 1]));
          *(u32x4*)(crow + 32 * q) = u32x4{w[0], w[1], w[2], w[3]};
        }
      }
    }
  }
}

// (Cin, Cout) pairs with an instance; others return false (the caller keeps the GEMM engines)
// One 4-wave workgroup per CU (256 workgroups), each wave looping over strips: measured against two per
// CU (512) and 128-384 (tools/conv1x1_probe.py, profiles/r05zh_conv1x1_probe3.log: 5.3 vs 5.15 TB/s; uneven
// counts leave CUs idle); 64-pixel strips at one wave per SIMD (4-8 % slower, 2× slower where the
// accumulators spill) and nontemporal loads / stores (−10 %) were slower (r05zh_conv1x1_probe2/4.log).
// (Cin, Cout) pairs with an instance; others return false (the caller keeps the GEMM engines).
bool launch_conv1x1(const GemmP& p, int cin, int cout, hipStream_t st) {
  const long strips = (p.M + 31) / 32;
  const dim3 g((unsigned)std::min<long>((strips + 3) / 4, 256));
  if (cin == 256 && cout == 128)
    hipLaunchKernelGGL((conv1x1_stream_kernel<8, 8>), g, dim3(256), 0, st, p);
  else if (cin == 128 && cout == 256)
    hipLaunchKernelGGL((conv1x1_stream_kernel<4, 16>), g, dim3(256), 0, st, p);
  else if (cin == 128 && cout == 128)
    hipLaunchKernelGGL((conv1x1_stream_kernel<4, 8>), g, dim3(256), 0, st, p);
  else
    return false;
  return true;
}

}  // namespace rdmi_gk

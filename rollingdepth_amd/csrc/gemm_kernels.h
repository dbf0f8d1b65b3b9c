// Implicit-GEMM engine for the Linear layers and the convolutions of the UNet / VAE.
//
// One kernel template serves dense GEMM (Linear: A = activations [M, K]) and convolution
// (A = on-the-fly im2col of an NHWC f16 tensor, with optional nearest-×2 upsample folded into
// the address generator).  Tiles: BM×BN×32 per 256-thread workgroup, 2×2 waves, each wave
// (BM/2)×(BN/2) from v_mfma_f32_16x16x32_f16 (f32 accumulators), register-staged double-buffered
// LDS (global loads for tile k+1 in flight while tile k's MFMAs run, one barrier per K-step).
// Fused epilogues: alpha scale, per-column bias, per-(row group) bias (the ResnetBlock2D time
// embedding add, resnet.py:338-346), residual add (skip connections), GEGLU
// (activations.py:113-123), f16 or f32 output.
#pragma once
#include "common.h"

#include <utility>

namespace rdmi_gk {

constexpr int BK = 64;  // K per stage: 8 chunks of 8 halves (16 B) per tile row

struct GemmP {
  const f16* A; long lda, sA;
  const f16* Wt; long ldw, sW;
  void* C; long ldc, sC; int c_f32;
  const float* bias;
  const f16* R; long ldr, sR;
  const float* rowbias; int rpg; long rb_ld;
  float alpha;
  int M, N, K, Kvalid;
  int geglu, silu, vec;
  unsigned a_bytes, w_bytes;  // operand extents for the buffer descriptors (OOB lanes read 0)
  // convolution (A gathered from NHWC x)
  int IH, IW, Cin, Ho, Wo, kh, kw, stride, pt, pl, up, cin_vecs;
  int cmaj;  // weights / K order channel-block major (rdmi.h): K-tile = one tap of 64 channels
  float* gnp; long gn_ld;  // GroupNorm moments of the output (32 rows x 4 channels), or null
  int group_m;  // tile order inside an XCD's range: groups of group_m m-tiles, n-tiles within a group
  // GroupNorm (+SiLU) of the conv INPUT, applied as it is read (conv_halo_kernel<..., GN = true>)
  const float* gmr; const float* ggam; const float* gbet; int gG, gsilu;
  const float* gaff;  // optional [B][Cin/64][2][64] scale / shift table (rdmi_conv_args.in_affine)
  int cperm;       // halo convs: 32-channel output permutation for 16-B epilogue accesses (RDMI_CPERM)
  int conv_pipe;   // halo convs: software-pipelined fragment reads (RDMI_CONV_PIPE=0: all reads first, A/B)
  int halo_pref;   // conv_halo_occ2_kernel: L2 prefetch of the next channel block's halo (RDMI_HALO_PREF)
  int xprio;       // conv_halo_occ2_kernel: the GroupNorm halo transform at s_setprio 2 (default; RDMI_XFORM_PRIO=0 off)
  int eprio;       // conv_halo_occ2_kernel: the epilogue at s_setprio 2 (RDMI_EPI_PRIO=1, A/B)
  unsigned long long* stamps;  // STAMP builds only (tools/conv_stamp.hip): per-wave segment cycle sums
};

// In-kernel stamp (diagnostic builds, STAMP = 1; guide §7 'In-kernel stamps'): s_memtime with the
// lgkmcnt(0) it needs in one statement, fenced from the scheduler on both sides.
__device__ __forceinline__ unsigned long long gk_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// vmcnt(n) alone (gfx9 s_waitcnt encoding: vmcnt[3:0] | vmcnt[5:4]<<14, expcnt/lgkmcnt at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}

constexpr unsigned OOB = 0x80000000u;  // byte offset past every descriptor's extent → zeros

// GroupNorm(+SiLU)-transformed halo values → f16 with the conv's zero padding: out-of-image pixels
// (in = false) become 0.  Pairs rounded by one v_cvt_pk_f16_f32 (RNE, as the scalar conversions) and
// the padding applied to the packed word, only in waves that hold such a pixel: the same bits as
// `in ? (f16)f : 0` per element, 1.5 fewer VALU per element.
__device__ __forceinline__ f16x4 gn_pack4(const float* f, bool in) {
  unsigned w0, w1;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(w0) : "v"(f[0]), "v"(f[1]));
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(w1) : "v"(f[2]), "v"(f[3]));
  if (!__all(in)) {
    w0 = in ? w0 : 0u;
    w1 = in ? w1 : 0u;
  }
  return __builtin_bit_cast(f16x4, (__attribute__((ext_vector_type(2))) unsigned){w0, w1});
}

// GroupNorm of one f16 halo value (the low or high half of w): fmaf((float)v, sc, sh) as one
// v_fma_mix_f32 (the f16 operand converted exactly; written as asm so that hipcc does not SLP-pack the
// affine into v_pk_fma_f32, slower beside MFMAs).
template <bool HI>
__device__ __forceinline__ float gn_elem(unsigned w, float sc, float sh) {
  float f;
  if (HI)
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(f) : "v"(w), "v"(sc), "v"(sh));
  else
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(f) : "v"(w), "v"(sc), "v"(sh));
  return f;
}

// silu_f of four values: x · rcp(1 + exp2(x · −log2 e)), the same instructions as silu_f.  One asm
// block so that every v_exp / v_rcp result is read three instructions later (the trans-result
// forwarding hazard that hipcc pads for its own instructions does not see inside inline asm).
__device__ __forceinline__ void silu4(float (&f)[4]) {
  float t0, t1, t2, t3;
  asm("v_mul_f32 %0, 0xbfb8aa3b, %4\n\t"
      "v_mul_f32 %1, 0xbfb8aa3b, %5\n\t"
      "v_mul_f32 %2, 0xbfb8aa3b, %6\n\t"
      "v_mul_f32 %3, 0xbfb8aa3b, %7\n\t"
      "v_exp_f32 %0, %0\n\t"
      "v_exp_f32 %1, %1\n\t"
      "v_exp_f32 %2, %2\n\t"
      "v_exp_f32 %3, %3\n\t"
      "v_add_f32 %0, 1.0, %0\n\t"
      "v_add_f32 %1, 1.0, %1\n\t"
      "v_add_f32 %2, 1.0, %2\n\t"
      "v_add_f32 %3, 1.0, %3\n\t"
      "v_rcp_f32 %0, %0\n\t"
      "v_rcp_f32 %1, %1\n\t"
      "v_rcp_f32 %2, %2\n\t"
      "v_rcp_f32 %3, %3\n\t"
      "v_mul_f32 %0, %4, %0\n\t"
      "v_mul_f32 %1, %5, %1\n\t"
      "v_mul_f32 %2, %6, %2\n\t"
      "v_mul_f32 %3, %7, %3"
      : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
      : "v"(f[0]), "v"(f[1]), "v"(f[2]), "v"(f[3]));
  f[0] = t0;
  f[1] = t1;
  f[2] = t2;
  f[3] = t3;
}

// n (multiple of 4) halo values in place: GroupNorm (+SiLU), f16, zero padding where !in
template <int NW, bool SILU>
__device__ __forceinline__ void gn_xform_words(unsigned (&w)[NW], const float* sc, const float* sh, bool in) {
#pragma unroll
  for (int j = 0; j < NW; j += 2) {
    float f[4] = {gn_elem<false>(w[j], sc[2 * j], sh[2 * j]), gn_elem<true>(w[j], sc[2 * j + 1], sh[2 * j + 1]),
                  gn_elem<false>(w[j + 1], sc[2 * j + 2], sh[2 * j + 2]),
                  gn_elem<true>(w[j + 1], sc[2 * j + 3], sh[2 * j + 3])};
    if (SILU) silu4(f);
    const f16x4 o = gn_pack4(f, in);
    const auto u = __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o);
    w[j] = u[0];
    w[j + 1] = u[1];
  }
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned voff, f16* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, voff, 0, 0, 0);
}
// ... with a wave-uniform byte offset in the scalar soffset operand (a per-K-tile step that costs no
// VALU); lanes whose voff is OOB stay out of range.
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff, f16* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, voff, soff, 0, 0);
}

// Epilogue shared by both engines.  The MFMA ran as Dᵀ = W·Aᵀ, so a lane holds 4 CONSECUTIVE
// output channels n = fq*4 + r of one row m = lane&15: bias / time-embedding / residual are read
// and the result written as 4-element vectors (8-B f16 / 16-B f32), scalar only at a ragged N
// tail.  rows: the wave's output-row map (LinRows / PatchRows); nw: its first output column.
// Output-row maps of a wave's 16-row fragments i (lane row fr): consecutive rows of the GEMM M
// dimension, or the rows of a 16-pixel-wide spatial patch (conv_halo_kernel).  slot(i): the
// 32-row GroupNorm-moment slot of the fragment pair (i-1, i) (rdmi.h gn_part); every image's slots
// are the contiguous range [b·HW/32, (b+1)·HW/32) in both maps.
// Sum over the 16 lanes of a DPP row (the 16 rows of an MFMA fragment) with VALU DPP adds — the
// xor-1, xor-2 butterfly (quad_perm) then the 4- and 8-lane halves (row_half_mirror, row_mirror:
// every lane of a quad / half-row holds the same partial, so the mirror pairs add the same two
// operands as xor-4 / xor-8 would).  Replaces ds_bpermute shuffles (LDS round trips) in the
// GroupNorm-moment epilogue; the sum order is unchanged.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: xor 1
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: xor 2
  v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of the 8-lane half
  v += dpp_f<0x140>(v);  // row_mirror: the other half of the row
  return v;
}

// full(n): every row of the wave's n fragments exists; group(n, rpg): the one row-bias group
// (rows / rpg) all those rows fall in, or -1 when they straddle groups (wave-uniform).
struct LinRows {
  int mw, fr, M;
  __device__ int row(int i) const {
    const int m = mw + i * 16 + fr;
    return m < M ? m : -1;
  }
  __device__ long slot(int i) const { return (mw + (i - 1) * 16) >> 5; }
  __device__ bool full(int n) const { return mw + n * 16 <= M; }
  __device__ int group(int n, int rpg) const { return mw / rpg == (mw + n * 16 - 1) / rpg ? mw / rpg : -1; }
  __device__ int rstep() const { return 16; }  // row(i + 1) - row(i) where full()
};
struct PatchRows {  // patch rows y0 + rw + i (i = fragment), columns x0 + fr; Ho even, Wo % 16 == 0
  int b, Ho, Wo, y0, x0, rw, fr;
  __device__ int row(int i) const { return (b * Ho + y0 + rw + i) * Wo + x0 + fr; }
  __device__ long slot(int i) const { return (long)((b * Ho + y0 + rw + i - 1) >> 1) * (Wo >> 4) + (x0 >> 4); }
  __device__ bool full(int) const { return true; }
  __device__ int group(int, int rpg) const { return rpg == Ho * Wo ? b : -1; }  // conv: rpg = Ho·Wo
  __device__ int rstep() const { return Wo; }
};
// Output phase (a, c) of a ×2-upsampled conv computed on the source grid (conv_halo_occ2_kernel MODE 3):
// phase-grid patch rows y0 + rw + i, columns x0 + fr → output pixel (2y + a, 2x + c) of the
// Ho × Wo output.  Moment slots: image b's range [b·HoWo/32, (b+1)·HoWo/32) split into the four
// phases' sub-ranges of (Ho/2)(Wo/2)/32 slots, each laid out as PatchRows' on the phase grid.
struct PhaseRows {
  int b, Ho, Wo, y0, x0, rw, fr, a, c;
  __device__ int row(int i) const { return (b * Ho + 2 * (y0 + rw + i) + a) * Wo + 2 * (x0 + fr) + c; }
  __device__ long slot(int i) const {
    return (long)(b * 4 + 2 * a + c) * ((Ho >> 1) * (Wo >> 1) >> 5) + ((y0 + rw + i - 1) >> 1) * (Wo >> 5) + (x0 >> 4);
  }
  __device__ bool full(int) const { return true; }
  __device__ int group(int, int rpg) const { return rpg == Ho * Wo ? b : -1; }
  __device__ int rstep() const { return 2 * Wo; }
};

// 16-B epilogue accesses for the halo convs (p.cperm).  The weight rows are DMA'd into LDS in a
// permuted order (perm64 within each wave's 64-channel slab) so that MFMA fragments 2q and 2q+1
// of a lane hold 8 CONSECUTIVE output channels: fragment j, channel slot fq*4 + r lands on channel
// 32(j/2) + 8fq + 4(j%2) + r.  The epilogue then loads residuals and stores outputs as 16-B
// vectors (half the address-processing work of the 8-B per-fragment accesses); the K order per
// output element is unchanged, so the results are bitwise those of the unpermuted kernel.
__device__ __forceinline__ int perm64(int r) {
  const int j = r >> 4, c = r & 15;
  return 32 * (j >> 1) + 8 * (c >> 2) + 4 * (j & 1) + (c & 3);
}
__device__ __forceinline__ int col_base(bool perm, int nw, int j, int fq) {
  return perm ? nw + 32 * (j >> 1) + 8 * fq + 4 * (j & 1) : nw + j * 16 + fq * 4;
}

template <int RM, int RN, int WTN, bool SILU, class Rows>
__device__ __forceinline__ void store_tile_t(const GemmP& p, f32x4 (&acc)[RM][RN], const Rows& rows, int nw, int bz,
                                             int fr, int fq, bool perm) {
  const long cb = (long)bz * p.sC;
  const long rbz = (long)bz * p.sR;
  // Fast path for whole f16 tiles (every row exists, every 4-column group inside N, one row-bias
  // group): all operand loads (bias, row bias, residual) are issued before the first use, so the
  // wave waits for memory once instead of once per fragment.
  const int rbg = p.rowbias ? rows.group(RM, p.rpg) : 0;
  if (!p.geglu && !p.c_f32 && p.vec && rows.full(RM) && nw + RN * 16 <= p.N && rbg >= 0) {
    // bias and row-bias vectors loaded under one uniform branch each and combined only after the
    // residual loads are issued: a use inside the branch made hipcc wait (vmcnt(0)) once per column
    // fragment, four serialised round trips per tile with a row bias (the UNet resnets' time
    // embedding).  Same adds in the same order: bitwise the previous epilogue.
    f32x4 bb[RN], rbv[RN];
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < RN; ++j) bb[j] = *(const f32x4*)(p.bias + col_base(perm, nw, j, fq));
    } else {
#pragma unroll
      for (int j = 0; j < RN; ++j) bb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (p.rowbias) {
      const float* rbp = p.rowbias + (long)rbg * p.rb_ld;
#pragma unroll
      for (int j = 0; j < RN; ++j) rbv[j] = *(const f32x4*)(rbp + col_base(perm, nw, j, fq));
    }
    f16x4 rr[RM][RN];
    if (p.R) {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const f16* rrow = p.R + rbz + (long)rows.row(i) * p.ldr;
        if (perm && RN % 2 == 0) {
#pragma unroll
          for (int j = 0; j < RN; j += 2) {
            const f16x8 v = *(const f16x8*)(rrow + col_base(true, nw, j, fq));
            rr[i][j] = __builtin_shufflevector(v, v, 0, 1, 2, 3);
            rr[i][j + 1] = __builtin_shufflevector(v, v, 4, 5, 6, 7);
          }
        } else {
#pragma unroll
          for (int j = 0; j < RN; ++j) rr[i][j] = *(const f16x4*)(rrow + col_base(false, nw, j, fq));
        }
      }
    }
    f32x4 badd[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) badd[j] = p.rowbias ? bb[j] + rbv[j] : bb[j];
    float gs[RN], gq[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const long crow = cb + (long)rows.row(i) * p.ldc;
      f16x4 ov[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = col_base(perm, nw, j, fq);
        f16x4 o;
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] * p.alpha + badd[j][r];
          if (p.R) v += (float)rr[i][j][r];
          if constexpr (SILU) v = silu_f(v);
          o[r] = (f16)v;
          const float f = (float)o[r];
          s += f;
          q = fmaf(f, f, q);
        }
        ov[j] = o;
        if (!(perm && RN % 2 == 0)) *(f16x4*)((f16*)p.C + crow + n) = o;
        else if (j & 1)
          *(f16x8*)((f16*)p.C + crow + col_base(true, nw, j - 1, fq)) =
              __builtin_shufflevector(ov[j - 1], o, 0, 1, 2, 3, 4, 5, 6, 7);
        if (p.gnp) {  // as below: fixed butterfly over the 16 rows of the fragment pair
          if (!(i & 1)) {
            gs[j] = s;
            gq[j] = q;
          } else {
            s += gs[j];
            q += gq[j];
            s = row16_sum(s);
            q = row16_sum(q);
            if (fr == 0) {
              float* d = p.gnp + (long)(n >> 2) * p.gn_ld + rows.slot(i) * 2;
              d[0] = s;
              d[1] = q;
            }
          }
        }
      }
    }
    return;
  }
  if (!p.geglu) {
    static_assert(RM % 2 == 0, "GroupNorm moments pair 16-row tiles into 32-row blocks");
    float gs[RN], gq[RN];  // per column tile: moments of this lane's 4 outputs over a 32-row block
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = rows.row(i);
      const bool mok = m >= 0;
      const float* rbrow = p.rowbias && mok ? p.rowbias + (long)(m / p.rpg) * p.rb_ld : nullptr;
      const long crow = cb + (long)m * p.ldc;
      const long rrow = rbz + (long)m * p.ldr;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = col_base(perm, nw, j, fq);
        const bool ok = mok && n < p.N;
        float s = 0.f, q = 0.f;
        if (ok) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha;
          if (p.vec && n + 3 < p.N) {
            if (p.bias) {
              const f32x4 bb = *(const f32x4*)(p.bias + n);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += bb[r];
            }
            if (rbrow) {
              const f32x4 bb = *(const f32x4*)(rbrow + n);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += bb[r];
            }
            if (p.R) {
              const f16x4 rr = *(const f16x4*)(p.R + rrow + n);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += (float)rr[r];
            }
            if constexpr (SILU) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = silu_f(v[r]);
            }
            if (p.c_f32) {
              *(f32x4*)((float*)p.C + crow + n) = f32x4{v[0], v[1], v[2], v[3]};
            } else {
              f16x4 o;
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = (f16)v[r];
              *(f16x4*)((f16*)p.C + crow + n) = o;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float f = (float)o[r];
                s += f;
                q = fmaf(f, f, q);
              }
            }
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int nn = n + r;
              if (nn >= p.N) break;
              float x = v[r];
              if (p.bias) x += p.bias[nn];
              if (rbrow) x += rbrow[nn];
              if (p.R) x += (float)p.R[rrow + nn];
              if constexpr (SILU) x = silu_f(x);
              if (p.c_f32)
                ((float*)p.C)[crow + nn] = x;
              else
                ((f16*)p.C)[crow + nn] = (f16)x;
            }
          }
        }
        if (p.gnp) {  // host guarantees f16 output, N % 4 == 0, M % 32 == 0 (blocks whole)
          if (!(i & 1)) {
            gs[j] = s;
            gq[j] = q;
          } else {
            s += gs[j];
            q += gq[j];
            s = row16_sum(s);  // fixed butterfly over the 16 rows of the tile
            q = row16_sum(q);
            if (fr == 0 && ok) {
              float* d = p.gnp + (long)(n >> 2) * p.gn_ld + rows.slot(i) * 2;
              d[0] = s;
              d[1] = q;
            }
          }
        }
      }
    }
  } else if constexpr (WTN == 64) {
    // GEGLU: within each wave's WTN(=64)-column slab, columns [0,32) are the value half and
    // [32,64) the gate half of output columns slab*32 + [0,32) (N % 128 == 0: always vector).
    // (Launches with other wave widths never carry the GEGLU epilogue: launch_mode.)  The bias
    // vectors depend on the column only: loaded once, before the first use (p.C may alias p.bias
    // as far as the compiler knows, so it would otherwise reload them per fragment behind a wait).
    f32x4 bh[RN / 2], bg[RN / 2];
#pragma unroll
    for (int j = 0; j < RN / 2; ++j) {
      const int nh = nw + j * 16 + fq * 4;
      bh[j] = p.bias ? *(const f32x4*)(p.bias + nh) : f32x4{0.f, 0.f, 0.f, 0.f};
      bg[j] = p.bias ? *(const f32x4*)(p.bias + nh + WTN / 2) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = rows.row(i);
      if (m < 0) continue;
      const long crow = cb + (long)m * p.ldc;
#pragma unroll
      for (int j = 0; j < RN / 2; ++j) {
        const int no = nw / 2 + j * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float h = acc[i][j][r] * p.alpha + bh[j][r];
          const float g = acc[i][j + RN / 2][r] * p.alpha + bg[j][r];
          v[r] = h * gelu_erf_fast(g);  // no per-element flag: hipcc would branch on it per output
        }
        if (p.R) {  // one wave-uniform branch per 4 outputs (inside the loop hipcc branched per output)
          const f16* rp = p.R + rbz + (long)m * p.ldr + no;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)rp[r];
        }
        if (p.c_f32) {
          *(f32x4*)((float*)p.C + crow + no) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          f16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (f16)v[r];
          *(f16x4*)((f16*)p.C + crow + no) = o;
        }
      }
    }
  }
}


// x + (float)h and fmaf((float)h, (float)h, x), h the low / high f16 half of w: one v_fma_mix_f32 each
// (the f16 operand converted exactly, one rounding — bitwise the convert-then-add / -fma pair).
template <bool HI>
__device__ __forceinline__ float add_h(float x, unsigned w) {
  float f;
  if (HI)
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(f) : "v"(w), "v"(x));
  else
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(f) : "v"(w), "v"(x));
  return f;
}
template <bool HI>
__device__ __forceinline__ float sq_h(float x, unsigned w) {
  float f;
  if (HI)
    asm("v_fma_mix_f32 %0, %1, %1, %2 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "=v"(f) : "v"(w), "v"(x));
  else
    asm("v_fma_mix_f32 %0, %1, %1, %2 op_sel_hi:[1,1,0]" : "=v"(f) : "v"(w), "v"(x));
  return f;
}
// row16_sum of two values at once, each level one v_add_f32_dpp (v[perm] + v: the same sum as
// row16_sum's v + v[perm]); the s_nops are the VALU-write → DPP-read wait states, which hipcc does not
// pad inside inline asm.
__device__ __forceinline__ void row16_sum2(float& s, float& q) {
  asm("s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(s), "+v"(q));
}

// Specialised epilogue for the common case (whole f16 tile, one row-bias group, no SiLU / GEGLU):
// residual and GroupNorm moments are template arguments instead of flags tested per fragment
// (hipcc if-converted the residual add into an add + select per output and re-converted every
// output to f16 for the moments), the f16 operands enter the f32 sums through v_fma_mix_f32, the
// row sums are DPP adds, and the moment address is one per-lane base plus a wave-uniform offset.
// Same operations in the same order as store_tile_t's fast path: bitwise its outputs and moments.
// The 128-channel GroupNorm-input convs' epilogue is issue-bound beside the partner workgroup's MFMAs
// (tools/conv_stamp.hip: moments +10 k, residual +4.5 k cycles per wave before this).
template <int RM, int RN, bool PERM, bool RES, bool MOM, class Rows>
__device__ __forceinline__ void store_fast(const GemmP& p, f32x4 (&acc)[RM][RN], const Rows& rows, int nw, int bz,
                                           int fr, int fq, int rbg) {
  static_assert(!PERM || RN % 2 == 0, "16-B permuted accesses pair column fragments");
  static_assert(RM % 2 == 0, "GroupNorm moments pair 16-row tiles into 32-row blocks");
  using u32x2 = __attribute__((ext_vector_type(2))) unsigned;
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
  f32x4 bb[RN], rbv[RN];
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < RN; ++j) bb[j] = *(const f32x4*)(p.bias + col_base(PERM, nw, j, fq));
  } else {
#pragma unroll
    for (int j = 0; j < RN; ++j) bb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (p.rowbias) {
    const float* rbp = p.rowbias + (long)rbg * p.rb_ld;
#pragma unroll
    for (int j = 0; j < RN; ++j) rbv[j] = *(const f32x4*)(rbp + col_base(PERM, nw, j, fq));
  }
  u32x2 rr[RM][RN];
  if constexpr (RES) {
    // rows of a whole tile are row(0) + i·rstep(): one 64-bit product per tile, the step uniform
    const f16* const r0 = p.R + (long)bz * p.sR + (long)rows.row(0) * p.ldr;
    const long rst = (long)rows.rstep() * p.ldr;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const f16* rrow = r0 + i * rst;
      if constexpr (PERM) {
#pragma unroll
        for (int j = 0; j < RN; j += 2) {
          const u32x4 v = __builtin_bit_cast(u32x4, *(const f16x8*)(rrow + col_base(true, nw, j, fq)));
          rr[i][j] = u32x2{v[0], v[1]};
          rr[i][j + 1] = u32x2{v[2], v[3]};
        }
      } else {
#pragma unroll
        for (int j = 0; j < RN; ++j) rr[i][j] = __builtin_bit_cast(u32x2, *(const f16x4*)(rrow + col_base(false, nw, j, fq)));
      }
    }
  }
  f32x4 badd[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) badd[j] = p.rowbias ? bb[j] + rbv[j] : bb[j];
  // moments: this lane's channel group n >> 2 of column fragment j = lane part + j part
  float* const gb = MOM ? p.gnp + (long)((nw >> 2) + (PERM ? 2 * fq : fq)) * p.gn_ld : nullptr;
  f16* const c0 = (f16*)p.C + (long)bz * p.sC + (long)rows.row(0) * p.ldc;
  const long cst = (long)rows.rstep() * p.ldc;
  float gs[RN], gq[RN];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    f16* const crow = c0 + i * cst;
    u32x2 ow[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaf(acc[i][j][r], p.alpha, badd[j][r]);
      if constexpr (RES) {
        v[0] = add_h<false>(v[0], rr[i][j][0]);
        v[1] = add_h<true>(v[1], rr[i][j][0]);
        v[2] = add_h<false>(v[2], rr[i][j][1]);
        v[3] = add_h<true>(v[3], rr[i][j][1]);
      }
      unsigned w0, w1;
      asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(w0) : "v"(v[0]), "v"(v[1]));
      asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(w1) : "v"(v[2]), "v"(v[3]));
      ow[j] = u32x2{w0, w1};
      if constexpr (!PERM) {
        *(u32x2*)(crow + col_base(false, nw, j, fq)) = ow[j];
      } else if (j & 1) {
        *(u32x4*)(crow + col_base(true, nw, j - 1, fq)) = u32x4{ow[j - 1][0], ow[j - 1][1], w0, w1};
      }
      if constexpr (MOM) {
        float s = add_h<true>(add_h<false>(0.f, w0), w0);
        s = add_h<true>(add_h<false>(s, w1), w1);
        float q = sq_h<true>(sq_h<false>(0.f, w0), w0);
        q = sq_h<true>(sq_h<false>(q, w1), w1);
        if (!(i & 1)) {
          gs[j] = s;
          gq[j] = q;
        } else {
          s += gs[j];
          q += gq[j];
          row16_sum2(s, q);
          if (fr == 0) {
            const int sl = __builtin_amdgcn_readfirstlane((int)rows.slot(i));
            const long jo = (long)(PERM ? 8 * (j >> 1) + (j & 1) : 4 * j) * p.gn_ld + 2L * sl;
            *(__attribute__((ext_vector_type(2))) float*)(gb + jo) = {s, q};
          }
        }
      }
    }
  }
}

// The SiLU epilogue (TimestepEmbedding only) is a wave-uniform choice: dispatched here, outside the
// per-output code, so that no other GEMM / conv computes (and discards) a SiLU per output.  Whole
// f16 tiles without SiLU / GEGLU take store_fast, specialised on residual and moments; PSITE: the
// call site's usual 16-B permutation (the halo convs' p.cperm), the form store_fast is built for.
template <int RM, int RN, int WTN, bool PSITE = false, class Rows>
__device__ __forceinline__ void store_tile(const GemmP& p, f32x4 (&acc)[RM][RN], const Rows& rows, int nw, int bz,
                                           int fr, int fq, bool perm = false) {
  if (p.silu) {
    store_tile_t<RM, RN, WTN, true>(p, acc, rows, nw, bz, fr, fq, perm);
    return;
  }
  constexpr bool FP = PSITE && RN % 2 == 0;
  const int rbg = p.rowbias ? rows.group(RM, p.rpg) : 0;
  if (!p.geglu && !p.c_f32 && p.vec && rows.full(RM) && nw + RN * 16 <= p.N && rbg >= 0 && perm == FP) {
    if (p.R) {
      if (p.gnp)
        store_fast<RM, RN, FP, true, true>(p, acc, rows, nw, bz, fr, fq, rbg);
      else
        store_fast<RM, RN, FP, true, false>(p, acc, rows, nw, bz, fr, fq, rbg);
    } else if (p.gnp) {
      store_fast<RM, RN, FP, false, true>(p, acc, rows, nw, bz, fr, fq, rbg);
    } else {
      store_fast<RM, RN, FP, false, false>(p, acc, rows, nw, bz, fr, fq, rbg);
    }
    return;
  }
  store_tile_t<RM, RN, WTN, false>(p, acc, rows, nw, bz, fr, fq, perm);
}

using rdmi::tile_mn;
using rdmi::xcd_remap;

// MODE 0: dense A [M, K] (Linear, 1×1 conv); MODE 1: implicit im2col of NHWC x for a 3×3 conv
// (any stride/padding); MODE 2: 3×3 conv reading x through a nearest ×2 upsample.
// Operands reach LDS by LDS-DMA (buffer_load_dwordx4 … lds: no VGPR staging, no ds_write) into a
// 3-slot ring of [rows][64-half] tiles, two K-steps in flight, one barrier per K-step.  Padding,
// ragged M/N/K and the implicit zero padding of the conv all become out-of-range buffer offsets,
// which the descriptor's range check turns into zero chunks (no select, no zero buffer).  Each
// 1-KiB DMA instruction fills 8 rows lane-linearly; the 16-B chunk swizzle (phys = logical ^
// (row & 7)) is applied on the per-lane SOURCE offset and on the fragment read (guide rule 21),
// so ds_read_b128 fragment reads are conflict-free.
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_kernel(GemmP p) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AV = BM / 8 / NW;  // 1-KiB DMA instructions per wave per stage (A)
  constexpr int BV = BN / 8 / NW;
  constexpr int LPS = AV + BV;     // DMA instructions per wave per stage
  constexpr int SLOT = (BM + BN) * BK;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile/waves mismatch");
  __shared__ __attribute__((aligned(16))) f16 lds[3 * SLOT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nbx = gridDim.x;
  const int logical = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
  int mt_, nt_;
  tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  const int n0 = nt_ * BN;
  const int m0 = mt_ * BM;
  const int bz = blockIdx.z;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (long)bz * p.sA), (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.Wt + (long)bz * p.sW), (short)0, (int)p.w_bytes, 0x00020000);

  // lane → (row within its 8-row DMA group, logical chunk): phys chunk = lane & 7
  const int lrow = lane >> 3;
  const int chunk = (lane & 7) ^ lrow;
  // per A row: element offset of the tap-(0,0) input pixel (MODE 1), or of the row (MODE 0);
  // rows past M get hb = INT_MIN/2 so every bounds check fails
  int arow[AV], ahb[AV], awb[AV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int m = m0 + (i * NW + wid) * 8 + lrow;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    if (MODE != 0) {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw;
      const int r = mm - b * hw;
      const int ho = r / p.Wo;
      const int wo = r - ho * p.Wo;
      const int hb = ho * p.stride - p.pt;
      ahb[i] = ok ? hb : -(1 << 28);  // rows past M fail every bounds check
      awb[i] = wo * p.stride - p.pl;
      arow[i] = MODE == 1 ? (b * p.IH + hb) * p.IW * p.Cin + awb[i] * p.Cin  // may be < 0: only used when valid
                          : b * p.IH * p.IW * p.Cin;
    } else {
      ahb[i] = ok ? 0 : -1;
      awb[i] = 0;
      arow[i] = mm * (int)p.lda;
    }
  }
  int brow[BV];
#pragma unroll
  for (int i = 0; i < BV; ++i) {
    const int n = n0 + (i * NW + wid) * 8 + lrow;
    brow[i] = n < p.N ? n * (int)p.ldw : -1;
  }
  // A chunk → (tap, channel vector).  Tap-major K: chunk g of the K-tile is g-th vector of
  // [tap][Cin]; channel-block major: 32-channel half h = chunk>>2 of the K-tile is block
  // (cb, tap) = divmod(2u + h, 9) and its vector cb*4 + (chunk&3).
  int tap = 0, cv = chunk;
  if (MODE != 0) {
    if (p.cmaj) {  // K-tile u = tap u % 9 of the 64-channel block u / 9
      tap = 0;
      cv = chunk;
    } else {
      tap = chunk / p.cin_vecs;
      cv = chunk - tap * p.cin_vecs;
    }
  }
  const int Hl = p.IH << (MODE == 2 ? 1 : 0), Wl = p.IW << (MODE == 2 ? 1 : 0);

  // issue the DMA of K-step `ks` into ring slot `slot`
  auto issue = [&](int ks, int slot) {
    const int kk = ks * BK + chunk * 8;
    const bool kok = kk < p.Kvalid;
    f16* la = lds + slot * SLOT;
    f16* lb = la + BM * BK;
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        const bool ok = ahb[i] == 0 && kok;
        dma16(ra_, ok ? (unsigned)(arow[i] + kk) * 2u : OOB, la + (i * NW + wid) * 8 * BK);
      }
    } else {
      const int dy = (tap * 11) >> 5;  // tap / 3 for tap < 9 (3×3 kernels only)
      const int dx = tap - 3 * dy;
      const int tapoff = (dy * p.IW + dx) * p.Cin + cv * 8;
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        const int hi = ahb[i] + dy, wi = awb[i] + dx;
        const bool ok = kok && (unsigned)hi < (unsigned)Hl && (unsigned)wi < (unsigned)Wl;
        int off;
        if (MODE == 1)
          off = arow[i] + tapoff;
        else
          off = arow[i] + ((hi >> 1) * p.IW + (wi >> 1)) * p.Cin + cv * 8;
        dma16(ra_, ok ? (unsigned)off * 2u : OOB, la + (i * NW + wid) * 8 * BK);
      }
      if (p.cmaj) {
        if (++tap == 9) {
          tap = 0;
          cv += 8;
        }
      } else {
        cv += 8;
        while (cv >= p.cin_vecs) {
          cv -= p.cin_vecs;
          ++tap;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const bool ok = brow[i] >= 0 && kok;
      dma16(rw_, ok ? (unsigned)(brow[i] + kk) * 2u : OOB, lb + (i * NW + wid) * 8 * BK);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  issue(0, 0);
  issue(1, 1);  // (a zero-chunk DMA when nk == 1: exactly LPS younger DMAs at every wait)
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt<LPS>();  // this wave's DMA for step kt has landed (step kt+1 still in flight)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA for kt landed; every wave done with kt-1
    asm volatile("" ::: "memory");
    // branch-free: past the last K-step the DMA reads the zero chunk into a drained slot
    issue(kt + 2, (kt + 2) % 3);
    const f16* la = lds + (kt % 3) * SLOT + (wm * WTM) * BK;
    const f16* lb = lds + (kt % 3) * SLOT + BM * BK + (wn * WTN) * BK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int lc = 4 * s + fq;
      f16x8 af[RM], bf[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = i * 16 + fr;  // (wm*WTM) is a multiple of 8: same swizzle phase
        af[i] = *(const f16x8*)(la + row * BK + ((lc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = j * 16 + fr;
        bf[j] = *(const f16x8*)(lb + row * BK + ((lc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
  }
  wait_vmcnt<0>();  // drain the trailing zero-chunk DMAs before the workgroup can retire

  store_tile<RM, RN, WTN>(p, acc, LinRows{m0 + wm * WTM, fr, p.M}, n0 + wn * WTN, bz, fr, fq);
}

// ---------------------------------------------------------------------------------------------
// Ping-pong engine for the large launches (the VAE / UNet convolutions, big Linear layers).
// Tile BM×BN = (WM·128)×(WN·RN·16) with 8 waves as WM × WN (WM·WN = 8), each wave a 128×(16·RN)
// output sub-tile (8×RN 16×16 f32 accumulators): 256×256 (WM 2, RN 4) and 512×128 (WM 4, RN 4:
// the VAE's 128-channel convs).  (RN 5 — 256×320 for the UNet's 320-multiples — needs more than
// the 256 registers of a 2-wave/SIMD kernel: hipcc moves the accumulators to scratch.)  K advances in
// 64-wide K-tiles (one full 128-B line per operand row) through a 2-slot LDS ring filled by
// LDS-DMA.  Each K-tile is four phases of 4·RN MFMAs per wave:  p0 = (A rows 0-63 of the wave,
// k 0-31), p1 = (rows 0-63, k 32-63), p2 = (rows 64-127, k 0-31), p3 = (rows 64-127, k 32-63);
// the B fragments of both k halves are read in p0/p1 and stay in registers for p2/p3.  The two
// wave groups (waves 0-3 and 4-7: one wave per SIMD each) run one barrier apart, so on every SIMD
// one wave issues its MFMAs while the other issues its ds_reads, address arithmetic and LDS-DMA
// for a later K-tile (guide §5 "256² 8-phase template": ping-pong, s_setprio around the MFMAs,
// counted vmcnt, raw s_barrier).
// Every load section first issues its fragment reads, then its share of the DMA (per wave and
// K-tile: NA pieces of A rows 0-63 of every wave row (A0), NA of rows 64-127 (A1), NB of B; one
// piece = one 1-KiB instruction), ahead of their first read by 3-6 phases:
//   LOAD(4u)  : A0b(u+1)                 LOAD(4u+1): wait A1(u), A1(u+1)
//   LOAD(4u+2): B0(u+2)                  LOAD(4u+3): wait B(u+1)+A0(u+1), B1(u+2), A0a(u+2)
// with LOAD(q) the load section of phase q = 4·(K-tile) + p, A0 = A0a (first A0A pieces) + A0b,
// B = B0 (first NB0 pieces) + B1.  RAW: each wave's wait sits in the load section before the
// first read of the data, which is followed by a barrier that every reader (either group) passes
// first.  WAR: B(u) and A0(u) are last read in LOAD(4u+1), which ends with s_waitcnt lgkmcnt(0)
// before its barrier, so their regions are free from the next phase on in either group (the
// groups are one barrier apart): B0(u+2) lands there in LOAD(4u+2), B1(u+2)/A0a(u+2) in
// LOAD(4u+3), A0b(u+2) in LOAD(4u+4); A1(u+2) overwrites A1(u), last read in LOAD(4u+3), in
// LOAD(4u+5).  Past the last K-tile the DMAs read zero chunks (out-of-range offsets) so the vmcnt
// arithmetic stays uniform.
// LDS row images are 128 B (64 halves); 16-B chunk c of row r is stored at c ^ (r & 7) (source
// side of the DMA, guide rule 21), which makes the 16×16×32 fragment reads conflict-free on the
// ds_read_b128 lane groups, and lets every 8-lane group of a DMA read one whole 128-B line.
// Conv (MODE 1/2) needs the channel-block-major K order with 64-channel blocks (p.cmaj): K-tile u
// is tap u % 9 of channels 64·(u / 9) .. +63.
// DBG (ablation builds only, RDMI_GEMM_DBG): bit0 no main-loop DMA, bit1 no barriers in the loop,
// bit2 no ds_reads in the loop, bit3 no MFMAs.  Results are garbage; timings isolate the costs.
template <int MODE, int WM, int RN, int DBG = 0>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmP p) {
  constexpr int WN = 8 / WM;
  constexpr int BM = WM * 128, BN = WN * RN * 16, BKP = 64;
  constexpr int RM = 8;
  constexpr int NA = WM;                 // A pieces per half per wave
  constexpr int NB = BN / 64;            // B pieces per wave
  constexpr int A0A = NA > 2 ? NA / 2 : 0;  // A0 pieces issued one phase early (LOAD(4u+3))
  constexpr int NB0 = NB > 2 ? 2 : 1;
  constexpr int SLOT = (BM + BN) * BKP;  // halves
  static_assert(WM * WN == 8 && 2 * SLOT * 2 <= 163840, "tile does not fit");
  __shared__ __attribute__((aligned(16))) f16 lds[2 * SLOT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wids = __builtin_amdgcn_readfirstlane(wid);  // DMA LDS destinations in SGPRs (M0)
  const int grp = wid >> 2;
  const int wm = wid / WN, wn = wid % WN;
  const int nbx = gridDim.x;
  const int logical = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
  int mt_, nt_;
  tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  const int n0 = nt_ * BN;
  const int m0 = mt_ * BM;
  const int bz = blockIdx.z;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (long)bz * p.sA), (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.Wt + (long)bz * p.sW), (short)0, (int)p.w_bytes, 0x00020000);

  // DMA lane geometry: one 1-KiB instruction = 8 rows × 128 B; lane → (row lrow, phys chunk lane&7)
  const int lrow = lane >> 3;
  const int chunk = (lane & 7) ^ lrow;  // logical chunk fetched (piece rows start at multiples of 8)
  // A pieces of this wave: half h, t = wid + 8e → tile rows (t>>3)*128 + h*64 + (t&7)*8 + lrow
  int arow[2][NA], ahb[2][NA], awb[2][NA];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < NA; ++e) {
      const int t = wid + 8 * e;
      const int m = m0 + (t >> 3) * 128 + h * 64 + (t & 7) * 8 + lrow;
      const bool ok = m < p.M;
      const int mm = ok ? m : 0;
      if (MODE != 0) {
        const int hw = p.Ho * p.Wo;
        const int b = mm / hw;
        const int r = mm - b * hw;
        const int ho = r / p.Wo;
        const int wo = r - ho * p.Wo;
        const int hb = ho * p.stride - p.pt;
        ahb[h][e] = ok ? hb : -(1 << 28);
        awb[h][e] = wo * p.stride - p.pl;
        arow[h][e] = MODE == 1 ? (b * p.IH + hb) * p.IW * p.Cin + awb[h][e] * p.Cin : b * p.IH * p.IW * p.Cin;
      } else {
        ahb[h][e] = ok ? 0 : -1;
        awb[h][e] = 0;
        arow[h][e] = mm * (int)p.lda;
      }
    }
  unsigned bvo[NB];  // weight byte offsets of this lane's rows at K-tile 0 (the K step goes in soffset), or OOB
#pragma unroll
  for (int e = 0; e < NB; ++e) {
    const int n = n0 + (wid + 8 * e) * 8 + lrow;
    bvo[e] = n < p.N ? (unsigned)(n * (int)p.ldw + chunk * 8) * 2u : OOB;
  }
  unsigned avo[2][NA];  // MODE 0: the same for the A rows
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < NA; ++e) avo[h][e] = ahb[h][e] == 0 ? (unsigned)(arow[h][e] + chunk * 8) * 2u : OOB;
  const int Hl = p.IH << (MODE == 2 ? 1 : 0), Wl = p.IW << (MODE == 2 ? 1 : 0);

  // A pieces e in [e0, e1) of half h, K-tile u
  auto issueA = [&](int h, int u, int e0, int e1) {
    f16* la = lds + (u & 1) * SLOT;
    if (MODE == 0) {
      const bool kok = u * BKP + chunk * 8 < p.Kvalid;  // lane-dependent only in a ragged last K-tile
#pragma unroll
      for (int e = 0; e < NA; ++e) {
        if (e < e0 || e >= e1) continue;
        const int t = wids + 8 * e;
        dma16s(ra_, kok ? avo[h][e] : OOB, u * BKP * 2, la + ((t >> 3) * 128 + h * 64 + (t & 7) * 8) * BKP);
      }
    } else {
      const int cb = u / 9;  // wave-uniform
      const int tap = u - cb * 9;
      const int dy = (tap * 11) >> 5, dx = tap - 3 * dy;
      const bool kok = cb * 64 < p.Cin;
      const int cofs = cb * 64 + chunk * 8;
      const int tapoff = (dy * p.IW + dx) * p.Cin + cofs;
#pragma unroll
      for (int e = 0; e < NA; ++e) {
        if (e < e0 || e >= e1) continue;
        const int t = wids + 8 * e;
        const int hi = ahb[h][e] + dy, wi = awb[h][e] + dx;
        const bool ok = kok && (unsigned)hi < (unsigned)Hl && (unsigned)wi < (unsigned)Wl;
        int off;
        if (MODE == 1)
          off = arow[h][e] + tapoff;
        else
          off = arow[h][e] + ((hi >> 1) * p.IW + (wi >> 1)) * p.Cin + cofs;
        dma16(ra_, ok ? (unsigned)off * 2u : OOB, la + ((t >> 3) * 128 + h * 64 + (t & 7) * 8) * BKP);
      }
    }
  };
  // B pieces e in [e0, e1) of K-tile u
  auto issueB = [&](int u, int e0, int e1) {
    const bool kok = u * BKP + chunk * 8 < p.Kvalid;
    f16* lb = lds + (u & 1) * SLOT + BM * BKP;
#pragma unroll
    for (int e = 0; e < NB; ++e) {
      if (e < e0 || e >= e1) continue;
      dma16s(rw_, kok ? bvo[e] : OOB, u * BKP * 2, lb + (wids + 8 * e) * 8 * BKP);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BKP - 1) / BKP;
  const int fr = lane & 15, fq = lane >> 4;
  // fragment offsets (halves) of this lane's row fr for the two k halves: chunk (4kh + fq) ^ (fr & 7)
  const int off0 = fr * BKP + ((fq ^ (fr & 7)) << 3);
  const int off1 = fr * BKP + (((4 + fq) ^ (fr & 7)) << 3);

  // prologue: the steady-state issue sequence up to iteration 0; then B(0) and A0(0) landed
  issueB(0, 0, NB);
  issueA(0, 0, 0, NA);
  issueA(1, 0, 0, NA);
  issueB(1, 0, NB);
  issueA(0, 1, 0, A0A);
  wait_vmcnt<NA + NB + A0A>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();  // K-tile 0 (B, A0) visible to every wave
  if (grp == 1 && !(DBG & 2)) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
  asm volatile("" ::: "memory");

  f16x8 af[4] = {}, bf[2][RN] = {};
  for (int u = 0; u < nk; ++u) {
    const f16* la = lds + (u & 1) * SLOT + (wm * 128) * BKP;
    const f16* lb = lds + (u & 1) * SLOT + BM * BKP + (wn * RN * 16) * BKP;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int h = ph >> 1, kh = ph & 1;
      // ---- LOAD(4u + ph): this phase's fragment reads first (their latency hides under the DMA
      // issue that follows), then the waits / DMA for later K-tiles
      if (!(DBG & 4)) {
        const int off = kh ? off1 : off0;
        if (h == 0) {
#pragma unroll
          for (int j = 0; j < RN; ++j) bf[kh][j] = *(const f16x8*)(lb + j * 16 * BKP + off);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *(const f16x8*)(la + (h * 64 + i * 16) * BKP + off);
      } else {
#pragma unroll
        for (int j = 0; j < RN; ++j) asm volatile("" : "+v"(bf[kh][j]));
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(af[i]));
      }
      if (!(DBG & 1)) {
        if (ph == 0) {
          issueA(0, u + 1, A0A, NA);  // A0b(u+1)
        } else if (ph == 1) {
          wait_vmcnt<NA + NB>();  // A1(u) landed (B(u+1), A0(u+1) in flight)
          issueA(1, u + 1, 0, NA);
        } else if (ph == 2) {
          issueB(u + 2, 0, NB0);
        } else {
          wait_vmcnt<NA + NB0>();  // B(u+1), A0(u+1) landed (A1(u+1), B0(u+2) in flight)
          issueB(u + 2, NB0, NB);
          issueA(0, u + 2, 0, A0A);
        }
      }
      // the last reads of B and A0 (p1) retire before the barrier: B0(u+2) re-fills B(u)'s region
      // in the next load section (either group)
      if (ph == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("" ::: "memory");
      if (!(DBG & 2)) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ---- MFMA(4u + ph)
      __builtin_amdgcn_s_setprio(1);
      if (!(DBG & 8)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[h * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[kh][j], af[i], acc[h * 4 + i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < RN; ++j) asm volatile("" ::"v"(bf[kh][j]));
      }
      __builtin_amdgcn_s_setprio(0);
      asm volatile("" ::: "memory");
      if (!(DBG & 2)) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if (grp == 0 && !(DBG & 2)) __builtin_amdgcn_s_barrier();  // match group 1's extra barrier
  wait_vmcnt<0>();  // drain the trailing zero-chunk DMAs before the workgroup can retire

  store_tile<RM, RN, RN * 16>(p, acc, LinRows{m0 + wm * 128, fr, p.M}, n0 + wn * RN * 16, bz, fr, fq);
}

// Halo ("direct") 3×3 convolution, stride 1, pad 1 (MODE 1), or through a nearest ×2 upsample
// (MODE 2), for Cin % 64 == 0 and output sizes that tile into 16×16 patches.
// The implicit GEMM above re-reads every input line for each of the 9 taps (9 A K-tiles per
// 64-channel block, served by L2): its per-CU L2→LDS stream, not the MFMAs, sets its speed.  Here
// a workgroup owns a 16×16 output-pixel patch × 256 output channels; per 64-channel block it loads
// the 18×18-pixel input halo ONCE into LDS (40.5 KiB, one LDS-DMA pass) and reads the A fragments
// of all 9 taps from it at shifted pixel positions; only the weights stream per tap (32 KiB).  Per
// 64-channel block the workgroup moves 41 + 9·32 KiB instead of 9·(32 + 32) KiB (−43 %).
// Structure: the 8-wave ping-pong of gemm_pp_kernel (2 M × 4 N waves, 128 pixels = 8 patch rows ×
// 16 columns by 64 channels per wave, four phases of 16 MFMAs per K-tile, groups one barrier
// apart); K-tile u = (channel block u / 9, tap u % 9) in the cmaj64 weight order.
// LDS: two halo buffers (41 pieces of 8 pixels: 324 used; of the 48 piece slots of 8 waves × 6,
// slots ≥ 41 are not loaded) + a 2-slot weight ring = 146 KiB (+ 8 KiB GroupNorm table).
// DMA per wave: per K-tile 4 weight pieces (B0 in LOAD(4u+2), B1 in LOAD(4u+3), for K-tile u+2);
// per channel block cb, the 6 halo pieces of block cb+1 in LOAD(4u) of taps 1..6.
// Waits (LOAD(4u+3)): B(u+1) landed — vmcnt(2), or vmcnt(3) when a halo piece was issued in
// LOAD(4u); on tap 7 that wait also covers all of halo(cb+1), first read at tap 0 of block cb+1.
// WAR: B(u+2) overwrites B(u), last read in LOAD(4u+1), which ends with lgkmcnt(0) (as in
// gemm_pp_kernel); halo(cb+1) overwrites halo(cb-1), last read in the final K-tile of block cb-1,
// ≥ 5 phases before tap 1 of block cb.
// Halo LDS image: pixel hp = r·18 + c of the halo at 128 B, 16-B chunk k stored at k ^ (hp & 7)
// (source-side swizzle): the 16 consecutive pixels of a fragment read are conflict-free for any
// tap shift.  Halo pixels outside the image read as zeros (out-of-range buffer offsets) = padding.
// NPH = phases per K-tile: 4 (16 MFMAs per phase, as gemm_pp_kernel) or 2 (32 MFMAs per phase:
// both k halves of a row half; half the barriers, twice the work between them).  With NPH = 2 the
// weights of K-tile u+2 are issued whole in LOAD(2u+1) after waiting for B(u+1) (vmcnt 0, or 1
// with a halo piece in flight), B(u) having been last read in LOAD(2u), which ends with lgkmcnt(0).
// WN = waves along N: 4 (256 output channels, waves of 8 patch rows × 64 channels) or 2 (128
// output channels, waves of 4 patch rows × 64 channels; NPH = 1: one phase of 32 MFMAs per K-tile
// and a 3-slot weight ring, since B(u) is read until the end of K-tile u: B(u+2) goes into the
// slot of B(u-1) in LOAD(u), after the halo piece, and the wait for B(u+1) follows it (vmcnt 2,
// or 3 with a halo piece); every load section ends with lgkmcnt(0)).
// GN: the input is the raw tensor under a GroupNorm (+SiLU) (ResnetBlock2D norm1/norm2 → conv1/
// conv2, resnet.py:326-352): each wave normalises the halo pieces it loaded, in place in LDS, with
// the per-channel scale/shift of its image (table in LDS, built in the prologue from mean/rstd,
// gamma, beta; the same f32 formula as rdmi_groupnorm_apply, so the result is identical to the
// unfused pair).  Piece e of halo(cb+1), issued in tap e+1, has landed by the wait of tap e+2 and
// is normalised inside the wave's own MFMA segments — channels 0-3 in phase 1 of tap e+2, 4-7 in
// phase 0 of tap e+3 (NPH 1: all in tap e+2) — as VALU work between its MFMAs, which the matrix
// pipe runs concurrently (normalising in the load segments instead, as extra work on the critical
// path, cost as much as the separate apply pass it replaces: tools/kbench.py gnconv).  The segment
// ends with lgkmcnt(0); the last write (tap 8 phase 0) is ≥ 2 barriers before the first read of
// block cb+1 by the group running one barrier ahead.  Halo pixels outside the image stay zero (the conv's zero padding is
// applied after the norm).  Halo(0) is normalised in the prologue.
// STAMP = 1 (diagnostic build only, tools/conv_stamp.hip): per-wave cycle sums — 0 prologue, 1 load
// sections (fragment reads, DMA issue, waits), 2 barrier before the MFMAs, 3 MFMA issue, 4 GroupNorm
// transform, 5 barrier after, 6 epilogue, 7 total — written to p.stamps.
template <int MODE, int NPH, int WN, bool GN, int STAMP = 0>
__global__ __launch_bounds__(512, 1) void conv_halo_kernel(GemmP p) {
  unsigned long long st_acc[8] = {}, st_prev = 0, st_start = 0;
  auto seg = [&](int i) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long t = gk_stamp();
      st_acc[i] += t - st_prev;
      st_prev = t;
    }
  };
  if constexpr (STAMP) st_start = st_prev = gk_stamp();
  constexpr int NT = 9;                    // taps per channel block
  constexpr int WM = 8 / WN;
  constexpr int BN = WN * 64, BKP = 64, RM = 16 / WM, RN = 4;
  constexpr int NRG = NPH == 4 ? 2 : NPH;  // row groups of a wave (one per phase group)
  constexpr int RPG = RM / NRG;            // patch rows per row group
  constexpr int NKH = NPH == 4 ? 1 : 2;    // k halves per phase
  constexpr int NB = BN / 64;              // weight pieces per wave per K-tile
  constexpr int NBS = NPH == 1 ? 3 : 2;    // weight ring slots
  constexpr int HWD = 18, HPIX = HWD * HWD;
  constexpr int HPW = 6;                   // halo piece slots per wave per channel block (48 >= 41)
  constexpr int HPC = 41;                  // pieces holding halo pixels (41·8 = 328 >= 324)
  constexpr int HALO = HPC * 8 * BKP;      // halves per halo buffer (41 KiB)
  constexpr int BSLOT = BN * BKP;          // halves per weight slot
  constexpr int GNT = GN ? 1024 : 0;       // GroupNorm scale/shift table: sc[1024], sh[1024] floats
  static_assert(RPG == 4 && (NPH != 1 || WN == 2) && (WN != 2 || NPH == 1) && (!GN || NPH != 4),
                "unsupported halo variant");
  __shared__ __attribute__((aligned(16))) f16 lds[2 * HALO + NBS * BSLOT + 4 * GNT];
  float* const gnt = (float*)(lds + 2 * HALO + NBS * BSLOT);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int grp = wid >> 2;
  const int wm = wid / WN, wn = wid % WN;
  const int nbx = gridDim.x;
  const int logical = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
  int mt_, nt_;
  tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  const int n0 = nt_ * BN;
  const int pxn = p.Wo >> 4, pyn = p.Ho >> 4;
  const int px = mt_ % pxn;
  const int py = (mt_ / pxn) % pyn;
  const int b = mt_ / (pxn * pyn);
  const int y0 = py * 16, x0 = px * 16;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.Wt, (short)0, (int)p.w_bytes, 0x00020000);

  const int lrow = lane >> 3;
  const int chunk = (lane & 7) ^ lrow;  // logical chunk fetched: piece pixels start at multiples of 8
  const int Hl = p.IH << (MODE == 2 ? 1 : 0), Wl = p.IW << (MODE == 2 ? 1 : 0);
  // halo pieces of this wave: t = wid + 8e → halo pixels hp = 8t + lrow (hp < 324 used)
  unsigned hvo[HPW];  // byte offsets at channel block 0 (the block step goes in soffset), or OOB
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    const int hp = (wid + 8 * e) * 8 + lrow;
    const int hr = hp / HWD, hc = hp - hr * HWD;
    const int yy = y0 - 1 + hr, xx = x0 - 1 + hc;
    const bool ok = hp < HPIX && (unsigned)yy < (unsigned)Hl && (unsigned)xx < (unsigned)Wl;
    const int sy = MODE == 2 ? yy >> 1 : yy, sx = MODE == 2 ? xx >> 1 : xx;
    hvo[e] = ok ? (unsigned)(((b * p.IH + sy) * p.IW + sx) * p.Cin + chunk * 8) * 2u : OOB;
  }
  unsigned bvo[NB];  // weight byte offsets at K-tile 0 (the K step goes in soffset), or OOB
#pragma unroll
  for (int e = 0; e < NB; ++e) {
    const int rt = (wid + 8 * e) * 8 + lrow;  // LDS row of the tile
    const int n = n0 + (p.cperm ? (rt & ~63) + perm64(rt & 63) : rt);
    bvo[e] = n < p.N ? (unsigned)(n * (int)p.ldw + chunk * 8) * 2u : OOB;
  }
  const int ncb = p.Cin >> 6;
  const int wids = __builtin_amdgcn_readfirstlane(wid);
  auto hv = [&](int e) { return wids + 8 * e < HPC; };  // piece slot e of this wave holds halo pixels
  auto issueHalo = [&](int cb, int e) {  // past the last block: zero-fill DMAs (the wait counts stay fixed)
    f16* lh = lds + (cb & 1) * HALO + (wids + 8 * e) * 8 * BKP;
    const bool ok = cb < ncb;  // wave-uniform
    dma16s(ra_, ok ? hvo[e] : OOB, ok ? cb * 128 : 0, lh);
  };
  auto issueB = [&](int u, int e0, int e1) {  // Kvalid % 64 == 0 (9 or 4 taps of Cin % 64 == 0)
    f16* lb = lds + 2 * HALO + (u % NBS) * BSLOT;
    const bool kok = u * BKP < p.Kvalid;  // wave-uniform
#pragma unroll
    for (int e = e0; e < e1; ++e) dma16s(rw_, kok ? bvo[e] : OOB, kok ? u * BKP * 2 : 0, lb + (wids + 8 * e) * 8 * BKP);
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = ncb * NT;
  const int fr = lane & 15, fq = lane >> 4;
  const int off0 = fr * BKP + ((fq ^ (fr & 7)) << 3);
  const int off1 = fr * BKP + (((4 + fq) ^ (fr & 7)) << 3);

  // in-place GroupNorm (+SiLU) of half hf (4 channels) of this wave's piece e of halo(cbn): lane
  // data = 8 channels of logical chunk `chunk` of one halo pixel (the DMA wrote lane L's 16 B at
  // piece + 16·L)
  auto xform = [&](int cbn, int e, int hf) {
    f16* lh = lds + (cbn & 1) * HALO + (wid + 8 * e) * 8 * BKP + lane * 8 + hf * 4;
    const float* ts = gnt + cbn * 64 + chunk * 8 + hf * 4;
    const f32x4 sc = *(const f32x4*)ts, sh = *(const f32x4*)(ts + GNT);
    unsigned w[2];
    *(f16x4*)w = *(const f16x4*)lh;
    const bool in = hvo[e] != OOB;
    const float scv[4] = {sc[0], sc[1], sc[2], sc[3]}, shv[4] = {sh[0], sh[1], sh[2], sh[3]};
    if (p.gsilu)  // the SiLU flag dispatched once per piece, not tested per element
      gn_xform_words<2, true>(w, scv, shv, in);
    else
      gn_xform_words<2, false>(w, scv, shv, in);
    *(f16x4*)lh = *(const f16x4*)w;
  };

  // prologue: halo(0) and the weights of K-tiles 0 and 1; wait for halo(0) + B(0)
#pragma unroll
  for (int e = 0; e < HPW; ++e)
    if (hv(e)) issueHalo(0, e);
  issueB(0, 0, NB);
  float gmean[2] = {0.f, 0.f}, grstd[2] = {0.f, 0.f}, ggam[2] = {0.f, 0.f}, gbet[2] = {0.f, 0.f};
  if constexpr (GN) {  // mean/rstd, gamma, beta of image b's channels (loads overlap the DMA latency)
    const int cpg = p.Cin / p.gG;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;
      if (c < p.Cin) {
        const int g = c / cpg;
        gmean[r] = p.gmr[2 * (b * p.gG + g)];
        grstd[r] = p.gmr[2 * (b * p.gG + g) + 1];
        ggam[r] = p.ggam[c];
        gbet[r] = p.gbet[c];
      }
    }
  }
  issueB(1, 0, NB);
  wait_vmcnt<NB>();
  if constexpr (GN) {  // scale/shift table (the formula of rdmi_groupnorm_apply)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float sc = grstd[r] * ggam[r];
      gnt[tid + 512 * r] = sc;
      gnt[GNT + tid + 512 * r] = gbet[r] - gmean[r] * sc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int e = 0; e < HPW; ++e)
      if (hv(e)) {
        xform(0, e, 0);
        xform(0, e, 1);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
  asm volatile("" ::: "memory");

  const int wms = __builtin_amdgcn_readfirstlane(wm);
  f16x8 af[NKH][4] = {}, bf[2][RN] = {};
  seg(0);
  for (int u = 0; u < nk; ++u) {
    const int cb = u / NT;  // wave-uniform
    const int tap = u - cb * NT;
    const int dy = (tap * 11) >> 5, dx = tap - 3 * dy;
    const f16* lb = lds + 2 * HALO + (u % NBS) * BSLOT + (wn * 64) * BKP;
    const bool halo_now = tap >= 1 && tap <= HPW && hv(tap - 1);
    // halo pixel of fragment row r = RM·wm + 4·rg + i, lane fr: hp = (r + dy)·18 + dx + fr, whose
    // swizzle term hp & 7 = (fr + dx + 2(i + dy)) & 7 does not depend on wm or rg (RM·18, 72 ≡ 0 mod 8)
    const int xb = fr + dx + 2 * dy;
    // A fragment (kh, rg, i): halo row wms·RM + 4·rg + i + dy, pixel dx + fr, chunk (kh·4 + fq) ^ ((xb + 2i) & 7):
    // four lane byte offsets per K-tile; row group rg by DS immediate, kh = 1 as the offset ^ 64
    const unsigned abase = (unsigned)((cb & 1) * HALO * 2 + ((wms * RM + dy) * HWD + dx + fr) * BKP * 2);
    unsigned aoff[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) aoff[r] = abase + (unsigned)((fq ^ ((xb + 2 * r) & 7)) << 4);
#pragma unroll
    for (int ph = 0; ph < NPH; ++ph) {
      const int rg = NPH == 4 ? ph >> 1 : ph;
      // ---- LOAD(NPH·u + ph): [normalise a landed halo piece], fragment reads, then waits / DMA
      // piece normalised in this phase's MFMA segment (NPH 2: half 0 of piece tap-2 in phase 1,
      // half 1 of piece tap-3 in phase 0; NPH 1: both halves of piece tap-2)
      const int xe = NPH == 2 && ph == 0 ? tap - 3 : tap - 2;
      const bool xf = GN && xe >= 0 && xe < HPW && cb + 1 < ncb && hv(xe);
#pragma unroll
      for (int q = 0; q < NKH; ++q) {
        const int kh = NPH == 4 ? (ph & 1) : q;
        if (rg == 0) {
          const int off = kh ? off1 : off0;
#pragma unroll
          for (int j = 0; j < RN; ++j) bf[kh][j] = *(const f16x8*)(lb + j * 16 * BKP + off);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[q][i] = *(const f16x8*)((const char*)lds + (kh ? aoff[i] ^ 64u : aoff[i]) + (rg * 4 + i) * HWD * BKP * 2);
      }
      if (NPH == 4) {
        if (ph == 0) {
          if (halo_now) issueHalo(cb + 1, tap - 1);
        } else if (ph == 2) {
          issueB(u + 2, 0, 2);
        } else if (ph == 3) {
          if (halo_now)
            wait_vmcnt<3>();  // B(u+1) landed (this tap's halo piece and B0(u+2) in flight)
          else
            wait_vmcnt<2>();  // B(u+1) (and on tap 7 all of halo(cb+1)) landed (B0(u+2) in flight)
          issueB(u + 2, 2, 4);
        }
        if (ph == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      } else if (NPH == 2) {
        if (ph == 0) {
          if (halo_now) issueHalo(cb + 1, tap - 1);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // B(u) read for the last time
        } else {
          if (halo_now)
            wait_vmcnt<1>();  // B(u+1) landed (this tap's halo piece in flight)
          else
            wait_vmcnt<0>();  // B(u+1) (and on tap 7 all of halo(cb+1)) landed
          issueB(u + 2, 0, NB);
        }
      } else {
        if (halo_now) issueHalo(cb + 1, tap - 1);
        issueB(u + 2, 0, NB);  // into the slot of B(u-1), read for the last time in LOAD(u-1)
        if (halo_now)
          wait_vmcnt<NB + 1>();  // B(u+1) landed (halo piece, B(u+2) in flight)
        else
          wait_vmcnt<NB>();  // B(u+1) (and on tap 7 all of halo(cb+1)) landed (B(u+2) in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      seg(1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      seg(2);
      // ---- MFMA(NPH·u + ph)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int q = 0; q < NKH; ++q) {
        const int kh = NPH == 4 ? (ph & 1) : q;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[rg * 4 + i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[kh][j], af[q][i], acc[rg * 4 + i][j], 0, 0, 0);
      }
      seg(3);
      if (xf) {  // after this wave's MFMAs (interleaved between them, or with its operands read
                 // in the load segment, it measured slower: tools/kbench.py gnconv)
        if (NPH == 1 || ph == 1) xform(cb + 1, xe, 0);
        if (NPH == 1 || ph == 0) xform(cb + 1, xe, 1);
      }
      __builtin_amdgcn_s_setprio(0);
      if (xf) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // normalised values written
      seg(4);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      seg(5);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // match group 1's extra barrier
  wait_vmcnt<0>();  // drain the trailing zero-chunk DMAs before the workgroup can retire
  seg(5);

  store_tile<RM, RN, 64, true>(p, acc, PatchRows{b, p.Ho, p.Wo, y0, x0, wm * RM, fr}, n0 + wn * 64, 0, fr, fq, p.cperm);
  if constexpr (STAMP) {
    wait_vmcnt<0>();
    seg(6);
    st_acc[7] = st_prev - st_start;
    if (lane == 0) {
      unsigned long long* o = p.stamps + (((long)blockIdx.y * gridDim.x + blockIdx.x) * 8 + wid) * 8;
      for (int i = 0; i < 8; ++i) o[i] = st_acc[i];
    }
  }
}

// Issue-order pins for conv_halo_occ2_kernel's pipelined K-tile (sched_group_barrier needs
// constant operands): group ST = [its DS reads: A(ST+PD), and the second k half's B fragments at
// ST = BPRE] then its RN MFMAs.
template <int RN, int PD, int NS, int BPRE, int ST>
__device__ __forceinline__ void occ2_sched_one() {
  constexpr int nr = (ST == BPRE ? RN : 0) + (ST + PD < NS ? 1 : 0);
  if constexpr (nr > 0) __builtin_amdgcn_sched_group_barrier(0x100, nr, 0);
  __builtin_amdgcn_sched_group_barrier(0x008, RN, 0);
}
template <int RN, int PD, int NS, int BPRE, int... S>
__device__ __forceinline__ void occ2_sched(std::integer_sequence<int, S...>) {
  (occ2_sched_one<RN, PD, NS, BPRE, S>(), ...);
}

// Two-workgroups-per-CU halo conv for 128-channel output tiles (the VAE's 768² convs).  With
// 128 output channels and Cin = 128 a tile has only 18 K-tiles, so the 8-wave single-workgroup
// variant above pays its prologue and epilogue un-overlapped on every tile (≈7 µs of ≈27 µs:
// tools/kbench.py sweep) and its 64×64 wave tiles read 0.5 KiB of LDS per MFMA.  Here a 4-wave
// workgroup owns a 16×16 patch × 128 channels with 128-pixel × 64-channel wave tiles (0.375 KiB
// per MFMA, as the 256-channel variant) and ≤ 80 KiB of LDS (one 41-KiB halo buffer, a 2-slot
// 16-KiB weight ring, the GroupNorm table), so two workgroups share each CU and one's epilogue,
// prologue and halo refills run under the other's MFMAs — occupancy, not an intra-workgroup
// ping-pong, hides the latencies.  Per K-tile: wait for the own weight DMA of this K-tile
// (issued one K-tile earlier) and the own fragment reads of the previous one, one barrier, issue
// the next K-tile's weights into the other slot (last read in the previous K-tile), then 24
// fragment reads and 64 MFMAs.  At a channel block's first tap the halo is refilled in place:
// barrier (all reads of the previous block's halo done), DMA, wait, [GroupNorm+SiLU of the own
// pieces], barrier.
// MODE 3: nearest ×2 upsample + 3×3 conv as four 2×2 convs on the source grid, one per output
// phase (a, c) = (y & 1, x & 1): the 3×3 taps that land on the same source pixel (rows {0 | 1, 2}
// for a = 0, {0, 1 | 2} for a = 1, columns likewise) act through one merged weight, stored as an
// f16 hi + lo pair (hi = f16(Σ w), lo = f16(Σ w − hi), Σ in f32: rdmi.h rdmi_conv_args.w_up2), so
// each product x·hi, x·lo is exact in the f32 accumulator and the result is the 9-tap conv's up to
// f32 accumulation order.  Per 64-channel block 7 K-tiles: the 4 hi taps (dy, dx) ∈ {0, 1}², then
// the lo parts of the 3 taps that merge 2 or 4 weights (the phase's single-weight tap (a, c) is
// exact in f16 and has no lo part) — 7/9 of MODE 2's MFMA work.  A tile is 16×16 pixels of one
// phase grid (Ho/2 × Wo/2); its 17×17 source halo (origin (y0 − 1 + a, x0 − 1 + c)) sits in the
// 18×18 halo buffer; weights p.Wt + phase·N·ldw.
// STAMP = 1 (diagnostic build only, tools/conv_stamp.hip): per-wave cycle sums of the segments —
// 0 prologue, 1 K-tile wait + barrier, 2 fragment reads + MFMA issue, 3 halo refill (barrier, DMA,
// wait, GroupNorm transform, barrier), 4 epilogue, 5 total — written to p.stamps.
template <int MODE, bool GN, bool PIPE, int STAMP = 0>
__global__ __launch_bounds__(256, 2) void conv_halo_occ2_kernel(GemmP p) {
  unsigned long long st_acc[6] = {}, st_prev = 0, st_start = 0;
  auto seg = [&](int i) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long t = gk_stamp();
      st_acc[i] += t - st_prev;
      st_prev = t;
    }
  };
  if constexpr (STAMP) st_start = st_prev = gk_stamp();
  constexpr int BN = 128, BKP = 64, RM = 8, RN = 4;
  constexpr int HWD = 18, HPIX = HWD * HWD;
  constexpr int HPC = 41;                  // pieces of 8 halo pixels (41·8 = 328 >= 324)
  constexpr int HPW = 11;                  // piece slots per wave (4 × 11 = 44 >= 41)
  constexpr int HALO = HPC * 8 * BKP;      // halves (41 KiB)
  constexpr int BSLOT = BN * BKP;          // halves (16 KiB)
  constexpr int NB = 4;                    // weight pieces per wave per K-tile (16 / 4 waves)
  constexpr int GNT = GN ? 256 : 0;        // sc[256], sh[256] floats (Cin <= 256)
  constexpr int PREF = 4 * 2 * 64 * 2;     // halves: the halo prefetch's landing area (4 waves × 2 × 64 dwords)
  __shared__ __attribute__((aligned(16))) f16 lds[HALO + 2 * BSLOT + 4 * GNT + PREF];
  float* const gnt = (float*)(lds + HALO + 2 * BSLOT);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int wids = __builtin_amdgcn_readfirstlane(wid);
  const int nbx = gridDim.x;
  int mt_, nt_;
  if (p.group_m < 0 && nbx > 1 && 8 % nbx == 0 && gridDim.y % (8 / nbx) == 0) {
    // n-tile per XCD (RDMI_CONV_NXCD=1, A/B): dispatch id d runs on XCD d % 8; XCD x computes only
    // n-tile x % nbx (8 / nbx XCDs share one, taking every (8 / nbx)-th m-tile), so its L2 holds one
    // n-tile's weights (1.2 MB for the 512-channel convs) instead of all of them.  Same tiles.
    const int bid = blockIdx.y * nbx + blockIdx.x, xcd = bid & 7;
    nt_ = xcd % nbx;
    mt_ = (bid >> 3) * (8 / nbx) + xcd / nbx;
  } else {
    const int logical = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
    tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  }
  const int n0 = nt_ * BN;
  constexpr int NT = MODE == 3 ? 7 : 9;  // K-tiles (taps) per channel block
  // MODE 3: m-tile = (image, phase, 16×16 tile of the Ho/2 × Wo/2 phase grid)
  const int pxn = p.Wo >> (MODE == 3 ? 5 : 4), pyn = p.Ho >> (MODE == 3 ? 5 : 4);
  const int px = mt_ % pxn;
  const int py = (mt_ / pxn) % pyn;
  const int phs = MODE == 3 ? (mt_ / (pxn * pyn)) & 3 : 0;
  const int b = mt_ / (pxn * pyn * (MODE == 3 ? 4 : 1));
  const int pa = phs >> 1, pc = phs & 1;
  const int y0 = py * 16, x0 = px * 16;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.Wt, (short)0, (int)p.w_bytes, 0x00020000);

  const int lrow = lane >> 3;
  const int chunk = (lane & 7) ^ lrow;
  const int Hl = p.IH << (MODE == 2 ? 1 : 0), Wl = p.IW << (MODE == 2 ? 1 : 0);
  unsigned hvo[HPW];  // piece t = wid + 4e: halo pixels 8t + lrow — byte offset at channel block 0, or OOB
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    const int hp = (wid + 4 * e) * 8 + lrow;
    const int hr = hp / HWD, hc = hp - hr * HWD;
    const int yy = y0 - 1 + pa + hr, xx = x0 - 1 + pc + hc;
    const bool ok = hp < HPIX && (unsigned)yy < (unsigned)Hl && (unsigned)xx < (unsigned)Wl;
    const int sy = MODE == 2 ? yy >> 1 : yy, sx = MODE == 2 ? xx >> 1 : xx;
    hvo[e] = ok ? (unsigned)(((b * p.IH + sy) * p.IW + sx) * p.Cin + chunk * 8) * 2u : OOB;
  }
  // Halo L2 prefetch (p.halo_pref, opt-in A/B): one dword of every 128-B line of the NEXT channel block's
  // halo pieces this wave refills — lane l of instruction j covers pixel (j·64 + l) & 7 of piece
  // wid + 4·((j·64 + l) >> 3) — loaded by LDS-DMA into a scratch area nothing reads, so that the refill's
  // DMA finds the lines in L2 instead of HBM.  Arithmetic unchanged (bitwise the plain kernel).
  unsigned pvo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = j * 64 + lane, e = idx >> 3;
    const int hp = (wid + 4 * e) * 8 + (idx & 7);
    const int hr = hp / HWD, hc = hp - hr * HWD;
    const int yy = y0 - 1 + pa + hr, xx = x0 - 1 + pc + hc;
    const bool ok = e < HPW && wid + 4 * e < HPC && hp < HPIX && (unsigned)yy < (unsigned)Hl && (unsigned)xx < (unsigned)Wl;
    const int sy = MODE == 2 ? yy >> 1 : yy, sx = MODE == 2 ? xx >> 1 : xx;
    pvo[j] = ok ? (unsigned)(((b * p.IH + sy) * p.IW + sx) * p.Cin) * 2u : OOB;
  }
  auto prefetchHalo = [&](int cb) {
    f16* lp = lds + HALO + 2 * BSLOT + 4 * GNT + wids * 256;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (__attribute__((address_space(3))) void*)(lp + j * 128), 4,
                                               pvo[j], cb * 128, 0, 0);
  };
  unsigned bvo[NB];  // weight DMA byte offsets of this lane's rows at K-tile 0 (the K step goes in soffset)
#pragma unroll
  for (int e = 0; e < NB; ++e) {
    const int rt = (wid + 4 * e) * 8 + lrow;  // LDS row of the tile
    const int n = n0 + (p.cperm ? (rt & ~63) + perm64(rt & 63) : rt);
    bvo[e] = n < p.N ? (unsigned)((phs * p.N + n) * (int)p.ldw + chunk * 8) * 2u : OOB;
  }
  const int ncb = p.Cin >> 6;
  auto hv = [&](int e) { return wids + 4 * e < HPC; };
  auto issueHalo = [&](int cb) {
#pragma unroll
    for (int e = 0; e < HPW; ++e)
      if (hv(e)) {
        f16* lh = lds + (wids + 4 * e) * 8 * BKP;
        dma16s(ra_, hvo[e], cb * 128, lh);
      }
  };
  auto issueB = [&](int u) {  // Kvalid % 64 == 0 (halo convs: 9 or 4 taps of Cin % 64 == 0)
    f16* lb = lds + HALO + (u & 1) * BSLOT;
#pragma unroll
    for (int e = 0; e < NB; ++e) dma16s(rw_, bvo[e], u * BKP * 2, lb + (wids + 4 * e) * 8 * BKP);
  };
  // The lane's 8 scales / shifts of channel block cb: from the global table p.gaff (any Cin; the four
  // 16-B loads issued with the halo DMA, so the refill's vmcnt wait covers them), else from the LDS
  // table the prologue built (Cin ≤ 256).  Same values either way.
  f32x4 aff[4];
  auto loadAff = [&](int cb) {
    if (p.gaff) {
      const float* ta = p.gaff + ((long)b * ncb + cb) * 128 + chunk * 8;
      aff[0] = *(const f32x4*)ta;
      aff[1] = *(const f32x4*)(ta + 4);
      aff[2] = *(const f32x4*)(ta + 64);
      aff[3] = *(const f32x4*)(ta + 68);
    }
  };
  // in-place GroupNorm (+SiLU) of this wave's landed pieces of the halo of channel block cb
  auto xformHalo = [&](int cb) {
    if (!p.gaff) {
      const float* ts = gnt + cb * 64 + chunk * 8;
      aff[0] = *(const f32x4*)ts;
      aff[1] = *(const f32x4*)(ts + 4);
      aff[2] = *(const f32x4*)(ts + GNT);
      aff[3] = *(const f32x4*)(ts + GNT + 4);
    }
    const float sc[8] = {aff[0][0], aff[0][1], aff[0][2], aff[0][3], aff[1][0], aff[1][1], aff[1][2], aff[1][3]};
    const float sh[8] = {aff[2][0], aff[2][1], aff[2][2], aff[2][3], aff[3][0], aff[3][1], aff[3][2], aff[3][3]};
    // each piece's 16 B read one piece ahead of its arithmetic, so the read's LDS latency runs under the
    // previous piece's transform instead of in front of it (same values, same writes: bitwise the
    // read-then-transform loop).  Piece 0 (wid < 4 < HPC) exists in every wave.
    unsigned wn[4];
    *(f16x8*)wn = *(const f16x8*)(lds + wid * 8 * BKP + lane * 8);
#pragma unroll
    for (int e = 0; e < HPW; ++e)
      if (hv(e)) {
        f16* lh = lds + (wid + 4 * e) * 8 * BKP + lane * 8;
        unsigned w[4] = {wn[0], wn[1], wn[2], wn[3]};
        if (e + 1 < HPW && hv(e + 1)) *(f16x8*)wn = *(const f16x8*)(lh + 4 * 8 * BKP);
        const bool in = hvo[e] != OOB;
        if (p.gsilu)  // the SiLU flag dispatched once per piece (see gn_elem)
          gn_xform_words<4, true>(w, sc, sh, in);
        else
          gn_xform_words<4, false>(w, sc, sh, in);
        *(f16x8*)lh = *(const f16x8*)w;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = ncb * NT;
  const int fr = lane & 15, fq = lane >> 4;
  const int off0 = fr * BKP + ((fq ^ (fr & 7)) << 3);
  const int off1 = fr * BKP + (((4 + fq) ^ (fr & 7)) << 3);

  // prologue: halo(0), B(0) [, GroupNorm scale/shift of image b]
  issueHalo(0);
  issueB(0);
  if constexpr (GN) loadAff(0);
  if (GN && !p.gaff) {
    const int c = tid;
    float mean = 0.f, rstd = 0.f, gm = 0.f, bt = 0.f;
    if (c < p.Cin) {
      const int g = c / (p.Cin / p.gG);
      mean = p.gmr[2 * (b * p.gG + g)];
      rstd = p.gmr[2 * (b * p.gG + g) + 1];
      gm = p.ggam[c];
      bt = p.gbet[c];
    }
    const float sc = rstd * gm;
    gnt[c] = sc;
    gnt[GNT + c] = bt - mean * sc;
  }
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (GN) {
    if (p.xprio) __builtin_amdgcn_s_setprio(2);
    xformHalo(0);
    if (p.xprio) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("" ::: "memory");

  const int wms = __builtin_amdgcn_readfirstlane(wm);
  const bool live = n0 + (wids & 1) * 64 < p.N;  // wave-uniform
  seg(0);
  for (int u = 0; u < nk; ++u) {
    const int cb = u / NT;
    const int tap = u - cb * NT;
    // MODE 3: K-tiles 0-3 the hi parts of taps t = 2dy + dx, 4-6 the lo parts of the taps t ≠ phase
    const int t4 = tap < 4 ? tap : tap - 4 + (tap - 4 >= phs ? 1 : 0);
    const int dy = MODE == 3 ? t4 >> 1 : (tap * 11) >> 5, dx = MODE == 3 ? t4 & 1 : tap - 3 * dy;
    const bool pf = p.halo_pref && cb + 1 < ncb && NT > 2;  // wave-uniform
    if (u > 0) seg(2);
    if (u > 0) {
      if (tap == 0) {  // refill the halo with channel block cb
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave is past its reads of halo(cb-1)
        asm volatile("" ::: "memory");
        issueHalo(cb);
        if constexpr (GN) loadAff(cb);
        wait_vmcnt<0>();  // B(u) and the halo pieces of this wave (and its scale / shift loads)
        if constexpr (GN) {
          if (p.xprio) __builtin_amdgcn_s_setprio(2);
          xformHalo(cb);
          if (p.xprio) __builtin_amdgcn_s_setprio(0);
        }
      } else {
        // B(u), issued one K-tile ago — and, at tap 2 with a prefetch in flight (issued after B(u) at
        // tap 1), everything but the prefetch's two loads (loads complete in issue order)
        if (pf && tap == 2)
          wait_vmcnt<2>();
        else
          wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of B(u-1) done (slot reuse)
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (tap == 0) seg(3); else seg(1);
    }
    if (u + 1 < nk) issueB(u + 1);
    if (pf && tap == 1) prefetchHalo(cb + 1);
    const f16* lb = lds + HALO + (u & 1) * BSLOT + (wn * 64) * BKP;
    const int xb = fr + dx + 2 * dy;
    // A fragment (kh, i): halo row wms·RM + i + dy, pixel dx + fr, 16-B chunk (kh·4 + fq) ^ ((xb + 2i) & 7).
    // The swizzle has period 4 in i and kh = 1 flips chunk bit 2, so four lane byte offsets per K-tile
    // serve all 16 reads: rows i and i + 4 differ by a DS immediate, kh = 1 is the offset ^ 64.
    const unsigned abase = (unsigned)(((wms * RM + dy) * HWD + dx + fr) * BKP * 2);
    unsigned aoff[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) aoff[r] = abase + (unsigned)((fq ^ ((xb + 2 * r) & 7)) << 4);
    auto readA = [&](int kh, int i) {
      const unsigned a = kh ? (aoff[i & 3] ^ 64u) : aoff[i & 3];
      return *(const f16x8*)((const char*)lds + a + i * HWD * BKP * 2);
    };
    // a wave whose 64 columns all lie past N (the ragged last 128-channel tile of a Cout = 320 conv)
    // issues no fragment reads or MFMAs: its SIMD's matrix pipe goes to the co-resident workgroup
    if (live) {
      if constexpr (PIPE) {
        // Software-pipelined fragment reads over the K-tile's 16 MFMA groups s = (kh, i): A(s+2) is
        // read while group s's 4 MFMAs issue, the second k half's B fragments 3 groups ahead of their
        // first use (≈44 live fragment registers instead of 96: with the f32 accumulators the
        // all-reads-first form ran out of registers, and the compiler then serialised every A read
        // behind lgkmcnt(0) in front of its MFMAs).  The sched_group_barrier sequence pins the issue
        // order (the scheduler otherwise sinks each read to just before its use).
        constexpr int NS = 2 * RM, PD = 2, BPRE = RM - 3;
        f16x8 bfr[2][RN], ar[PD + 1];
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[0][j] = *(const f16x8*)(lb + j * 16 * BKP + off0);
#pragma unroll
        for (int q = 0; q < PD; ++q) ar[q] = readA(q / RM, q % RM);
#pragma unroll
        for (int st = 0; st < NS; ++st) {
          if (st == BPRE) {
#pragma unroll
            for (int j = 0; j < RN; ++j) bfr[1][j] = *(const f16x8*)(lb + j * 16 * BKP + off1);
          }
          if (st + PD < NS) ar[(st + PD) % (PD + 1)] = readA((st + PD) / RM, (st + PD) % RM);
          const int kh = st / RM, i = st % RM;
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfr[kh][j], ar[st % (PD + 1)], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, RN + PD, 0);
        occ2_sched<RN, PD, NS, BPRE>(std::make_integer_sequence<int, NS>{});
      } else {
        f16x8 af[2][RM], bf[2][RN];
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const int off = kh ? off1 : off0;
#pragma unroll
          for (int j = 0; j < RN; ++j) bf[kh][j] = *(const f16x8*)(lb + j * 16 * BKP + off);
#pragma unroll
          for (int i = 0; i < RM; ++i) af[kh][i] = readA(kh, i);
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[kh][j], af[kh][i], acc[i][j], 0, 0, 0);
      }
    }
  }
  seg(2);
  if (live) {
    if (p.eprio) __builtin_amdgcn_s_setprio(2);  // RDMI_EPI_PRIO (A/B): the epilogue above the partner's MFMAs
    if constexpr (MODE == 3)
      store_tile<RM, RN, 64, true>(p, acc, PhaseRows{b, p.Ho, p.Wo, y0, x0, wm * RM, fr, pa, pc}, n0 + wn * 64, 0, fr,
                                   fq, p.cperm);
    else
      store_tile<RM, RN, 64, true>(p, acc, PatchRows{b, p.Ho, p.Wo, y0, x0, wm * RM, fr}, n0 + wn * 64, 0, fr, fq,
                                   p.cperm);
  }
  if constexpr (STAMP) {
    wait_vmcnt<0>();
    seg(4);
    st_acc[5] = st_prev - st_start;
    if (lane == 0) {
      unsigned long long* o = p.stamps + (((long)blockIdx.y * gridDim.x + blockIdx.x) * 4 + wid) * 8;
      for (int i = 0; i < 6; ++i) o[i] = st_acc[i];
      o[6] = st_start;
      o[7] = st_prev;
    }
  }
}

// Halo conv with 32×32×16 MFMAs for 128-channel output tiles (the VAE's 768² / 384² convs with
// Cout % 128 == 0 — in the pipeline the 128-channel decoder / encoder convs, GroupNorm input
// included).  The two-workgroups-per-CU structure of conv_halo_occ2_kernel, re-cut for vector-issue
// headroom: those convs are bound by the SIMD's vector-instruction issue, not by the matrix pipe
// (SQ PMC, profiles/r02_pmc_conv_summary.txt: 4.2k–7.1k VALU per wave against 1 152 16×16×32 MFMAs,
// each of which holds the vector issue for 8 of its 16 cycles).  Here
//  * v_mfma_f32_32x32x16_f16 (8 of 32 cycles held): half the issue cost per FLOP of the MFMAs;
//  * a 32×8 output patch (a 32-pixel fragment = one patch row), so that with the 16-B chunks of each
//    halo pixel swizzled by its COLUMN, (col >> 1) & 7, every fragment read is conflict-free and its
//    address is a per-lane register chosen by (tap dx, k-step) plus a compile-time immediate: the
//    nine taps of a channel block are unrolled and the K loop carries no address arithmetic;
//  * weight rows permuted within each 32-row block (perm32) so that a lane's 16 accumulator entries
//    are 16 consecutive output channels (two 16-B stores / residual loads per fragment).
// Workgroup = 4 waves: wm = wid >> 1 → patch rows 4wm..4wm+3, wn = wid & 1 → channels 64wn..+63;
// wave tile 4 fragments (rows) × 2 fragments (32 channels) of 32×32.  LDS: the 10×34 halo of one
// 64-channel block (43 KiB), a 2-slot weight ring (2 × 16 KiB), the GroupNorm table (2 KiB).
// K order per output (channel block, tap, 16-k steps) as the other halo engines; the MFMA's own
// 16-k reduction differs from the 32-k one of 16×16×32, so results match them to f32 rounding, not
// bitwise.  Moments: per (fragment, 4-channel group) the lane's 4 channels, then the 32 pixels of
// the fragment (rows of 16 lanes by DPP, the two rows by row_bcast:15).
__device__ __forceinline__ int perm32(int m) { return ((m >> 2) & 1) * 16 + (m >> 3) * 4 + (m & 3); }

template <int NKS>
__device__ __forceinline__ void h32_sched() {
  __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (ks + 1 < NKS) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
  }
}

template <bool GN>
__global__ __launch_bounds__(256, 2) void conv_halo32_kernel(GemmP p) {
  constexpr int BN = 128, BKP = 64;
  constexpr int HR = 10, HC = 34, HPIX = HR * HC;  // halo of a 32×8 patch
  constexpr int HPC = 43;                          // 8-pixel pieces (344 >= 340)
  constexpr int HPW = 11;                          // piece slots per wave (44 >= 43)
  constexpr int HALO = HPC * 8 * BKP;              // halves
  constexpr int BSLOT = BN * BKP;                  // halves
  constexpr int NB = 4;                            // weight pieces per wave per K-tile
  constexpr int GNT = GN ? 256 : 0;
  __shared__ __attribute__((aligned(16))) f16 lds[HALO + 2 * BSLOT + 4 * GNT];
  float* const gnt = (float*)(lds + HALO + 2 * BSLOT);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int wids = __builtin_amdgcn_readfirstlane(wid);
  const int nbx = gridDim.x;
  const int logical = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
  int mt_, nt_;
  tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  const int n0 = nt_ * BN;
  const int pxn = p.Wo >> 5, pyn = p.Ho >> 3;
  const int px = mt_ % pxn;
  const int py = (mt_ / pxn) % pyn;
  const int b = mt_ / (pxn * pyn);
  const int y0 = py * 8, x0 = px * 32;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.Wt, (short)0, (int)p.w_bytes, 0x00020000);

  // DMA geometry: a 1-KiB piece = 8 pixel slots (or weight rows) × 8 physical 16-B chunks, lane L
  // writing slot L >> 3, physical chunk L & 7, i.e. logical chunk (L & 7) ^ swizzle(slot)
  const int lrow = lane >> 3, pc = lane & 7;
  unsigned hoff[HPW];  // byte offset of this lane's 16 B of halo piece e in channel block 0, or OOB
  // logical chunk of this lane in piece e (GroupNorm channels 8·lc .. +8 of the block)
  auto hlc = [&](int e) __attribute__((always_inline)) {
    const int hp = (wid + 4 * e) * 8 + lrow;
    return pc ^ (((hp - (hp / HC) * HC) >> 1) & 7);
  };
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    const int hp = (wid + 4 * e) * 8 + lrow;
    const int hr = hp / HC, hc = hp - hr * HC;
    const int yy = y0 - 1 + hr, xx = x0 - 1 + hc;
    const bool ok = hp < HPIX && (unsigned)yy < (unsigned)p.IH && (unsigned)xx < (unsigned)p.IW;
    hoff[e] = ok ? (unsigned)((((b * p.IH + yy) * p.IW + xx) * p.Cin + hlc(e) * 8) * 2) : OOB;
  }
  unsigned boff[NB];
#pragma unroll
  for (int e = 0; e < NB; ++e) {
    const int rt = (wid + 4 * e) * 8 + lrow;  // LDS row of the weight tile
    const int n = n0 + (rt & ~31) + perm32(rt & 31);
    const int lc = pc ^ ((rt >> 1) & 7);
    boff[e] = n < p.N ? (unsigned)((n * (int)p.ldw + lc * 8) * 2) : OOB;
  }
  const int ncb = p.Cin >> 6;
  auto hv = [&](int e) { return wids + 4 * e < HPC; };
  auto issueHalo = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < HPW; ++e)
      if (hv(e))
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (__attribute__((address_space(3))) void*)(lds + (wid + 4 * e) * 8 * BKP),
                                                 16, hoff[e], cb * 128, 0, 0);
  };
  auto issueB = [&](int u) __attribute__((always_inline)) {
    f16* lb = lds + HALO + (u & 1) * BSLOT;
#pragma unroll
    for (int e = 0; e < NB; ++e)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw_, (__attribute__((address_space(3))) void*)(lb + (wid + 4 * e) * 8 * BKP),
                                               16, boff[e], u * 128, 0, 0);
  };
  unsigned inmask = 0;  // bit e: this lane's pixel of halo piece e lies inside the image
#pragma unroll
  for (int e = 0; e < HPW; ++e) inmask |= (hoff[e] != OOB ? 1u : 0u) << e;
  // in-place GroupNorm (+SiLU) of this wave's landed pieces (always_inline: called from every tap-0
  // K-tile instantiation, hipcc otherwise outlined it and passed the captures through 464 B of scratch
  // per lane — the 2.2× GroupNorm slowdown of round 5, profiles/r05b_h32_ab.log): the instructions of
  // conv_halo_occ2_kernel's transform (gn_xform_words: v_fma_mix affine, silu4, packed RNE
  // conversion, padding only in waves holding out-of-image pixels) — bitwise the unfused
  // gn_apply; the lane's logical chunk (and so its 8 scale / shift values) changes per piece here
  auto xformHalo = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < HPW; ++e)
      if (hv(e)) {
        f16* lh = lds + (wid + 4 * e) * 8 * BKP + lane * 8;
        const float* ts = gnt + cb * 64 + hlc(e) * 8;
        const f32x4 s0 = *(const f32x4*)ts, s1 = *(const f32x4*)(ts + 4);
        const f32x4 h0 = *(const f32x4*)(ts + GNT), h1 = *(const f32x4*)(ts + GNT + 4);
        const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
        const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        unsigned w[4];
        *(f16x8*)w = *(const f16x8*)lh;
        const bool in = (inmask >> e) & 1;
        if (p.gsilu)
          gn_xform_words<4, true>(w, sc, sh, in);
        else
          gn_xform_words<4, false>(w, sc, sh, in);
        *(f16x8*)lh = *(const f16x8*)w;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // fragment addresses (bytes from lds): pixel j = lane & 31 of a fragment row, k-step ks reads
  // logical chunk 2ks + hh of halo slot (row 4wm + pb + dy, column j + dx), physical chunk
  // logical ^ (((j + dx) >> 1) & 7); weights: row 64wn + 32chb + j, physical chunk
  // logical ^ ((row >> 1) & 7) (32chb does not change (row >> 1) & 7)
  const int j = lane & 31, hh = lane >> 5;
  const unsigned lds0 = (unsigned)(uintptr_t)LDS_PTR(f16, lds);
  unsigned poff[3][4], woff[4];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      poff[dx][ks] = lds0 + (unsigned)(((4 * wm * HC + j + dx) * BKP + (((2 * ks + hh) ^ (((j + dx) >> 1) & 7)) << 3)) * 2);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int row = 64 * wn + j;
    woff[ks] = lds0 + (unsigned)((HALO + row * BKP + (((2 * ks + hh) ^ ((row >> 1) & 7)) << 3)) * 2);
  }

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][c][r] = 0.f;

  // prologue: halo(0), B(0) [, GroupNorm scale/shift of image b]
  issueHalo(0);
  issueB(0);
  if constexpr (GN) {
    const int c = tid;
    float mean = 0.f, rstd = 0.f, gm = 0.f, bt = 0.f;
    if (c < p.Cin) {
      const int g = c / (p.Cin / p.gG);
      mean = p.gmr[2 * (b * p.gG + g)];
      rstd = p.gmr[2 * (b * p.gG + g) + 1];
      gm = p.ggam[c];
      bt = p.gbet[c];
    }
    const float sc = rstd * gm;
    gnt[c] = sc;
    gnt[GNT + c] = bt - mean * sc;
  }
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (GN) {
    xformHalo(0);
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("" ::: "memory");

  // one K-tile: tap TAP of channel block cb, weights in slot PAR
  auto ktile = [&](auto TAPc, auto PARc, int cb) __attribute__((always_inline)) {
    constexpr int TAP = decltype(TAPc)::value, PAR = decltype(PARc)::value;
    constexpr int dy = TAP / 3, dx = TAP % 3;
    const int u = cb * 9 + TAP;
    if (u > 0) {
      if (TAP == 0) {  // refill the halo with channel block cb
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave is past its reads of halo(cb-1)
        asm volatile("" ::: "memory");
        issueHalo(cb);
        wait_vmcnt<0>();  // B(u) and this wave's halo pieces
        if constexpr (GN) xformHalo(cb);
      } else {
        wait_vmcnt<0>();  // B(u), issued one K-tile ago
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of B(u-1) done (slot reuse)
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (u + 1 < 9 * ncb) issueB(u + 1);
    f16x8 af[2][2], bf[2][4];
    auto rd = [&](int ks, int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
        af[buf][c] = *(const f16x8*)LDS_PTR(f16, (uintptr_t)(woff[ks] + (PAR * BSLOT + c * 32 * BKP) * 2));
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
        bf[buf][pb] = *(const f16x8*)LDS_PTR(f16, (uintptr_t)(poff[dx][ks] + ((pb + dy) * HC * BKP) * 2));
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks + 1 < 4) rd(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc[pb][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[ks & 1][c], bf[ks & 1][pb], acc[pb][c], 0, 0, 0);
    }
    h32_sched<4>();
  };
  auto block = [&](auto PAR0, int cb) __attribute__((always_inline)) {  // the nine taps of channel block cb, slot parity alternating
    constexpr int P0 = decltype(PAR0)::value;
    ktile(std::integral_constant<int, 0>{}, std::integral_constant<int, P0>{}, cb);
    ktile(std::integral_constant<int, 1>{}, std::integral_constant<int, P0 ^ 1>{}, cb);
    ktile(std::integral_constant<int, 2>{}, std::integral_constant<int, P0>{}, cb);
    ktile(std::integral_constant<int, 3>{}, std::integral_constant<int, P0 ^ 1>{}, cb);
    ktile(std::integral_constant<int, 4>{}, std::integral_constant<int, P0>{}, cb);
    ktile(std::integral_constant<int, 5>{}, std::integral_constant<int, P0 ^ 1>{}, cb);
    ktile(std::integral_constant<int, 6>{}, std::integral_constant<int, P0>{}, cb);
    ktile(std::integral_constant<int, 7>{}, std::integral_constant<int, P0 ^ 1>{}, cb);
    ktile(std::integral_constant<int, 8>{}, std::integral_constant<int, P0>{}, cb);
  };
  for (int cb = 0; cb < ncb; cb += 2) {  // ncb even (h32_ok): K-tile u = 9cb + tap uses slot u & 1
    block(std::integral_constant<int, 0>{}, cb);
    block(std::integral_constant<int, 1>{}, cb + 1);
  }
  wait_vmcnt<0>();  // drain trailing DMAs before the workgroup can retire

  // ---- epilogue: fragment (pb, c) = pixels (y0 + 4wm + pb, x0 + j), channels nb .. nb + 15.
  // The optional parts are wave-uniform: one instantiation per (residual, SiLU) so that neither is
  // if-converted into every output.
  const long rbg = p.rowbias ? (long)b * p.rb_ld : 0;  // conv row bias: one group per image
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
  // Specialised epilogue (no SiLU), as store_fast: the residual's f16 halves and the moments' f16
  // outputs enter the f32 sums through v_fma_mix_f32, the moment row sums are DPP adds (the same
  // operations in the same order as the generic form below: bitwise its outputs and moments).
  auto epi_fast = [&](auto RESc, auto MOMc) {
    constexpr bool RES = decltype(RESc)::value, MOM = decltype(MOMc)::value;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int nb = n0 + 64 * wn + 32 * c + 16 * hh;
      f32x4 badd[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        badd[q] = p.bias ? *(const f32x4*)(p.bias + nb + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
        if (p.rowbias) badd[q] += *(const f32x4*)(p.rowbias + rbg + nb + 4 * q);
      }
      const long m0 = (long)(b * p.Ho + y0 + 4 * wm) * p.Wo + x0 + j;
      u32x4 rr[4][2];
      if constexpr (RES) {
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          const f16* rrow = p.R + (m0 + (long)pb * p.Wo) * p.ldr + nb;
          rr[pb][0] = *(const u32x4*)rrow;
          rr[pb][1] = *(const u32x4*)(rrow + 8);
        }
      }
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        unsigned ow[8];
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          float v0 = fmaf(acc[pb][c][2 * h], p.alpha, badd[h >> 1][(2 * h) & 3]);
          float v1 = fmaf(acc[pb][c][2 * h + 1], p.alpha, badd[h >> 1][(2 * h + 1) & 3]);
          if constexpr (RES) {
            v0 = add_h<false>(v0, rr[pb][h >> 2][h & 3]);
            v1 = add_h<true>(v1, rr[pb][h >> 2][h & 3]);
          }
          asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(ow[h]) : "v"(v0), "v"(v1));
        }
        f16* crow = (f16*)p.C + (m0 + (long)pb * p.Wo) * p.ldc + nb;
        *(u32x4*)crow = u32x4{ow[0], ow[1], ow[2], ow[3]};
        *(u32x4*)(crow + 8) = u32x4{ow[4], ow[5], ow[6], ow[7]};
        if constexpr (MOM) {  // slot (4-channel group, the 32 pixels of this fragment row)
          const long slot = ((long)(b * p.Ho + y0 + 4 * wm + pb) * p.Wo + x0) >> 5;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float s = add_h<true>(add_h<false>(0.f, ow[2 * g]), ow[2 * g]);
            s = add_h<true>(add_h<false>(s, ow[2 * g + 1]), ow[2 * g + 1]);
            float q = sq_h<true>(sq_h<false>(0.f, ow[2 * g]), ow[2 * g]);
            q = sq_h<true>(sq_h<false>(q, ow[2 * g + 1]), ow[2 * g + 1]);
            row16_sum2(s, q);
            s += dpp_f<0x142>(s);  // row_bcast:15 — rows 1 and 3 add the sums of rows 0 and 2
            q += dpp_f<0x142>(q);
            if ((lane & 31) == 16) {
              float* d = p.gnp + (long)((nb + 4 * g) >> 2) * p.gn_ld + slot * 2;
              *(__attribute__((ext_vector_type(2))) float*)d = {s, q};
            }
          }
        }
      }
    }
  };
  auto epilogue = [&](auto RESc, auto SILUc) {
    constexpr bool RES = decltype(RESc)::value, SILU = decltype(SILUc)::value;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int nb = n0 + 64 * wn + 32 * c + 16 * hh;
      f32x4 badd[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        badd[q] = p.bias ? *(const f32x4*)(p.bias + nb + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
        if (p.rowbias) badd[q] += *(const f32x4*)(p.rowbias + rbg + nb + 4 * q);
      }
      f16x8 rr[4][2];
      if constexpr (RES) {
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          const long m = (long)(b * p.Ho + y0 + 4 * wm + pb) * p.Wo + x0 + j;
          const f16* rrow = p.R + m * p.ldr + nb;
          rr[pb][0] = *(const f16x8*)rrow;
          rr[pb][1] = *(const f16x8*)(rrow + 8);
        }
      }
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const long m = (long)(b * p.Ho + y0 + 4 * wm + pb) * p.Wo + x0 + j;
        f16x8 ov[2];
        float gs[4], gq[4];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float v = acc[pb][c][i] * p.alpha + badd[i >> 2][i & 3];
          if constexpr (RES) v += (float)rr[pb][i >> 3][i & 7];
          if constexpr (SILU) v = silu_f(v);
          const f16 o = (f16)v;
          ov[i >> 3][i & 7] = o;
          const float f = (float)o;
          if ((i & 3) == 0) {
            gs[i >> 2] = f;
            gq[i >> 2] = f * f;
          } else {
            gs[i >> 2] += f;
            gq[i >> 2] = fmaf(f, f, gq[i >> 2]);
          }
        }
        f16* crow = (f16*)p.C + m * p.ldc + nb;
        *(f16x8*)crow = ov[0];
        *(f16x8*)(crow + 8) = ov[1];
        if (p.gnp) {  // slot (4-channel group, 32 pixels of this fragment row)
          const long slot = ((long)(b * p.Ho + y0 + 4 * wm + pb) * p.Wo + x0) >> 5;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float s = row16_sum(gs[g]), q = row16_sum(gq[g]);
            s += dpp_f<0x142>(s);  // row_bcast:15 — rows 1 and 3 add the sums of rows 0 and 2
            q += dpp_f<0x142>(q);
            if ((lane & 31) == 16) {
              float* d = p.gnp + (long)((nb + 4 * g) >> 2) * p.gn_ld + slot * 2;
              d[0] = s;
              d[1] = q;
            }
          }
        }
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (p.silu) {
    if (p.R) epilogue(T_{}, T_{}); else epilogue(F_{}, T_{});
  } else if (p.R) {
    if (p.gnp) epi_fast(T_{}, T_{}); else epi_fast(T_{}, F_{});
  } else {
    if (p.gnp) epi_fast(F_{}, T_{}); else epi_fast(F_{}, F_{});
  }
}

// Two-workgroups-per-CU dense GEMM (the UNet's single-batch Linears).  A 256×256
// ping-pong tile over K = 320 runs only 5 K-tiles between a DMA prologue and a 128-KiB epilogue
// that one workgroup per CU cannot overlap, and such GEMMs move as many bytes (A in, C out) as
// they compute: their bound is the stream, not the MFMAs.  Here 4-wave workgroups own 128×128
// tiles (64×64 per wave) in a 64-KiB 2-slot LDS ring, two per CU, so one workgroup's epilogue
// stores and next prologue run under the other's K loop.  Per K-tile as conv_halo_occ2_kernel:
// wait for the own DMA of this K-tile (issued one K-tile earlier) and the own fragment reads of
// the previous one, one barrier, issue the next K-tile into the other slot, 16 fragment reads,
// 32 MFMAs.  LDS rows are 128 B with 16-B chunk c of row r at c ^ (r & 7) (as gemm_pp_kernel).
// BN = 160 (N % 160 == 0: the L0 N = 320 / 960 Linears): 64×80 per wave, a 72-KiB ring — two column
// tiles of N = 320 instead of two and a half-dead third, so A is read twice, not three times, and no
// workgroup slot holds dead waves.  Same MFMA operands and order per output: bitwise the BN = 128 tile.
template <int V = 0, int BN = 128>
__global__ __launch_bounds__(256, 2) void gemm_occ2_kernel(GemmP p) {
  constexpr int BM = 128, BKP = 64, RM = 4, RN = BN / 32, WN = BN / 2;
  constexpr int NA = 4, NB = BN / 32;      // 1-KiB DMA pieces per wave per K-tile (BM / 8 and BN / 8 over 4 waves)
  constexpr int SLOT = (BM + BN) * BKP;    // halves (32 / 36 KiB)
  __shared__ __attribute__((aligned(16))) f16 lds[2 * SLOT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wids = __builtin_amdgcn_readfirstlane(wid);  // DMA LDS destinations in SGPRs (M0)
  const int wm = wid >> 1, wn = wid & 1;
  const int nbx = gridDim.x;
  const int logical = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
  int mt_, nt_;
  tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  const int n0 = nt_ * BN, m0 = mt_ * BM;
  const int bz = blockIdx.z;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (long)bz * p.sA), (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.Wt + (long)bz * p.sW), (short)0, (int)p.w_bytes, 0x00020000);

  const int lrow = lane >> 3;
  const int chunk = (lane & 7) ^ lrow;
  unsigned avo[NA], bvo[NB];  // byte offsets of this lane's rows at K-tile 0 (the K step goes in soffset), or OOB
#pragma unroll
  for (int e = 0; e < NA; ++e) {
    const int m = m0 + (wid + 4 * e) * 8 + lrow;
    avo[e] = m < p.M ? (unsigned)(m * (int)p.lda + chunk * 8) * 2u : OOB;
  }
#pragma unroll
  for (int e = 0; e < NB; ++e) {
    const int n = n0 + (wid + 4 * e) * 8 + lrow;
    bvo[e] = n < p.N ? (unsigned)(n * (int)p.ldw + chunk * 8) * 2u : OOB;
  }
  auto issue = [&](int u) {
    const bool kok = u * BKP + chunk * 8 < p.Kvalid;  // lane-dependent only in a ragged last K-tile
    f16* la = lds + (u & 1) * SLOT;
    f16* lb = la + BM * BKP;
#pragma unroll
    for (int e = 0; e < NA; ++e) dma16s(ra_, kok ? avo[e] : OOB, u * BKP * 2, la + (wids + 4 * e) * 8 * BKP);
#pragma unroll
    for (int e = 0; e < NB; ++e) dma16s(rw_, kok ? bvo[e] : OOB, u * BKP * 2, lb + (wids + 4 * e) * 8 * BKP);
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BKP - 1) / BKP;
  const int fr = lane & 15, fq = lane >> 4;
  const int off0 = fr * BKP + ((fq ^ (fr & 7)) << 3);
  const int off1 = fr * BKP + (((4 + fq) ^ (fr & 7)) << 3);

  const bool live = n0 + (wids & 1) * WN < p.N;  // wave-uniform
  issue(0);
  wait_vmcnt<0>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int u = 0; u < nk; ++u) {
    if (u > 0) {
      wait_vmcnt<0>();  // this K-tile, issued one K-tile ago
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the slot issue() refills
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (u + 1 < nk) issue(u + 1);
    if (!live) continue;  // columns all past N (the ragged last tile of N = 320 / 960): no reads, no MFMAs
    const f16* la = lds + (u & 1) * SLOT + (wm * 64) * BKP;
    const f16* lb = lds + (u & 1) * SLOT + BM * BKP + (wn * WN) * BKP;
    f16x8 af[2][RM], bf[2][RN];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int off = kh ? off1 : off0;
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[kh][j] = *(const f16x8*)(lb + j * 16 * BKP + off);
#pragma unroll
      for (int i = 0; i < RM; ++i) af[kh][i] = *(const f16x8*)(la + i * 16 * BKP + off);
    }
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[kh][j], af[kh][i], acc[i][j], 0, 0, 0);
  }
  if (live) store_tile<RM, RN, WN>(p, acc, LinRows{m0 + wm * 64, fr, p.M}, n0 + wn * WN, bz, fr, fq);
}

// Launchers, one translation unit per engine family (gemm_classic.hip, gemm_pp.hip, conv_halo.hip,
// conv_occ2.hip) so that the engines compile in parallel; the dispatch (gemm.hip) calls these.
void launch_gemm_classic(int mode, int bm, int bn, dim3 g, hipStream_t s, const GemmP& p);
void launch_gemm_pp(int mode, int wm, int dbg, dim3 g, hipStream_t s, const GemmP& p);
void launch_gemm_occ2(int bn, dim3 g, hipStream_t s, const GemmP& p);
void launch_conv_halo(int mode, int nph, int wn, bool gn, dim3 g, hipStream_t s, const GemmP& p);
void launch_conv_occ2(int mode, bool gn, bool pipe, dim3 g, hipStream_t s, const GemmP& p);
void launch_conv_h32(bool gn, dim3 g, hipStream_t s, const GemmP& p);
bool launch_conv1x1(const GemmP& p, int cin, int cout, hipStream_t st);  // false: no instance

}  // namespace rdmi_gk

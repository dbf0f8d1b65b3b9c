// f32 implicit-GEMM engine: the paper preset's fp32 arithmetic (run_video.py:444-449, dtype fp32)
// for the same Linear / conv call sites as gemm.hip (rdmi_gemm / rdmi_conv2d with dtype RDMI_F32).
//
// gfx950 has no xf32: f32 inputs run on v_mfma_f32_16x16x4_f32 (exact f32 products, an f32 fmaf
// chain per output; 64 FLOP/clk/SIMD = 157 TF, 1/16 of the f16 rate — MI355X_MICROARCH.md).  Each
// 128×128 output tile is one 256-thread workgroup of 2×2 waves (64×64 per wave, 4×4 fragments of
// 16×16).  K advances in 32-float K-tiles — one full 128-B line per operand row, the same byte
// geometry as the f16 engine's 64-half K-tiles — through a 3-slot LDS ring filled by
// buffer-load-to-LDS DMA (no VGPR staging, two K-tiles in flight, one barrier per K-tile); ragged
// M / N / K and the conv's implicit zero padding are out-of-range buffer offsets (zeros).  16-B
// chunk c of LDS row r sits at c ^ swz(r) (swizzled on the DMA source side; swz below).
// Fragment reads: lane quarter q (lane >> 4) supplies k = 8q + s at MFMA step s (s = 0..7 per
// K-tile) for BOTH operands, so a lane reads its 8 k values as two 16-B chunks (2q, 2q+1) per
// fragment instead of eight 4-B reads; the sum over k is the same set of products.
// The MFMA runs as Dᵀ = W·Aᵀ, so a lane holds 4 consecutive output channels of one output row
// (the f16 engine's epilogue geometry): bias / residual / output move as 16-B vectors.
//
// X3 (dtype RDMI_F32_X3): the same engine with the products on the bf16 MFMA, 16× the f32 rate.
// Every f32 operand is split into two bf16 parts, x = x_hi + x_lo + O(2^-17 |x|) (x_hi = bf16(x),
// x_lo = bf16(x − x_hi); the weights once at load, the activations as their fragments leave LDS),
// and a·w is formed as a_hi·w_hi + a_hi·w_lo + a_lo·w_hi with f32 accumulation: three
// v_mfma_f32_16x16x32_bf16 per 32-deep K step in place of eight v_mfma_f32_16x16x4_f32.  The dropped
// a_lo·w_lo and the two splits leave ≈2^-16 relative error per product (about 2^-24 for exact f32,
// 2^-11 for the TF32 that cuDNN's fp32 convolutions use by default on the reference's Ampere GPU).
// The weight rows hold, per 32-deep K-tile, 32 bf16 hi then 32 bf16 lo values — 128 B, the byte
// geometry of the f32 engine's K-tile, so the DMA and its swizzle are unchanged.
//
// X6 (dtype RDMI_F32_X6, round 5): three-way splits, x = x_hi + x_mid + x_lo + O(2^-26 |x|), and the six
// products whose parts' orders sum to ≤ 2 (a_hi·w_hi, a_hi·w_mid, a_mid·w_hi, a_mid·w_mid, a_lo·w_hi,
// a_hi·w_lo): a few 2^-24 per product — f32's own product rounding, the reference's exact-fp32 Linear
// precision — in six bf16 MFMAs per 32-deep K step (≈0.4 of the exact engine's matrix time).  The
// weight rows hold, per K-tile, [32 hi | 32 mid | 32 lo | 32 zero] bf16 = 256 B: two 128-B LDS rows per
// output channel (the same DMA geometry), and the tile is 64 × 128 so that two workgroups still share
// a CU (2 slots × (64 + 2·128) rows × 128 B = 80 KiB).
#include "common.h"

namespace {

constexpr int BKF = 32;  // K per stage (floats)

struct GemmF32P {
  const float* A; long lda, sA;
  const float* Wt; long ldw, sW;
  float* C; long ldc, sC;
  const float* bias;
  const float* R; long ldr, sR;
  const float* rowbias; int rpg; long rb_ld;
  float alpha;
  int M, N, K, Kvalid;
  int geglu, silu, vec;
  unsigned a_bytes, w_bytes;
  int IH, IW, Cin, Ho, Wo, stride, pt, pl, cin_vecs;
  int group_m;
};

constexpr unsigned OOB = 0x80000000u;

// LDS image of a 128-B row r (32 floats / 64 bf16): 16-B chunk c at position c ^ swz(r & 15) (round 5).
// The fragment reads of the 16x16 MFMA layouts — lane quarter q reads chunk 2q + h (f32 operands) or
// q, 4 + q (bf16 parts) of rows fr = lane & 15 — are then conflict-free for ds_read_b128's lane groups
// ({0-3, 12-15, 20-27}, ...); the former c ^ (r & 7) put the f32 reads 2-way on the same banks.
__device__ __forceinline__ int swz(int r) { return ((r >> 1) & 1) ^ (((r >> 2) & 1) << 2) ^ (((r >> 3) & 1) * 6); }

__device__ __forceinline__ void dma16f(__amdgpu_buffer_rsrc_t r, unsigned voff, float* l, int soff = 0) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, voff, soff, 0, 0);
}

// Epilogue: fragment (i, j) of a lane = output row mw + 16i + fr, channels nw + 16j + 4fq .. +3.
template <int RM, int RN>
__device__ __forceinline__ void store_tile_f32(const GemmF32P& p, f32x4 (&acc)[RM][RN], int mw, int nw, int bz,
                                               int fr, int fq) {
  const long cb = (long)bz * p.sC;
  const long rbz = (long)bz * p.sR;
  if (!p.geglu) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = mw + i * 16 + fr;
      if (m >= p.M) continue;
      const float* rbrow = p.rowbias ? p.rowbias + (long)(m / p.rpg) * p.rb_ld : nullptr;
      const long crow = cb + (long)m * p.ldc;
      const long rrow = rbz + (long)m * p.ldr;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = nw + j * 16 + fq * 4;
        if (n >= p.N) continue;
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
            const f32x4 rr = *(const f32x4*)(p.R + rrow + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += rr[r];
          }
          if (p.silu) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] / (1.0f + expf(-v[r]));
          }
          *(f32x4*)(p.C + crow + n) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = n + r;
            if (nn >= p.N) break;
            float x = v[r];
            if (p.bias) x += p.bias[nn];
            if (rbrow) x += rbrow[nn];
            if (p.R) x += p.R[rrow + nn];
            if (p.silu) x = x / (1.0f + expf(-x));
            p.C[crow + nn] = x;
          }
        }
      }
    }
  } else {
    // GEGLU: within each 64-column slab of a wave, columns [0,32) are the value half and [32,64) the
    // gate half of output columns slab·32 + [0,32) (N % 128 == 0, weights row-interleaved).
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = mw + i * 16 + fr;
      if (m >= p.M) continue;
      const long crow = cb + (long)m * p.ldc;
#pragma unroll
      for (int sl = 0; sl < RN / 4; ++sl)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int j = 4 * sl + jj;
          const int nh = nw + 64 * sl + jj * 16 + fq * 4;
          const int no = nw / 2 + 32 * sl + jj * 16 + fq * 4;
          const f32x4 bh = p.bias ? *(const f32x4*)(p.bias + nh) : f32x4{0.f, 0.f, 0.f, 0.f};
          const f32x4 bg = p.bias ? *(const f32x4*)(p.bias + nh + 32) : f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float h = acc[i][j][r] * p.alpha + bh[r];
            const float g = acc[i][j + 2][r] * p.alpha + bg[r];
            o[r] = h * gelu_erf(g);
            if (p.R) o[r] += p.R[rbz + (long)m * p.ldr + no + r];
          }
          *(f32x4*)(p.C + crow + no) = o;
        }
    }
  }
}

// MODE 0: dense A [M, K]; MODE 1: implicit im2col of an NHWC f32 tensor for a 3×3 conv (any stride /
// padding, K order [tap][Cin]); MODE 2: the 3×3 conv reading x through a nearest ×2 upsample.
// X3: bf16-split products (header).
// NS: LDS ring slots — 3 (96 KiB: one workgroup per CU, two K-tiles in flight) or 2 (64 KiB: two
// workgroups per CU, one K-tile in flight; the co-resident workgroup covers the DMA latency).
// NP: 1 exact f32 products, 2 bf16x3 (X3), 3 bf16x6 (X6).
template <int MODE, int NP, int NS>
__global__ __launch_bounds__(256, NS == 2 ? 2 : 1) void gemm_f32_kernel(GemmF32P p) {
  constexpr bool X3 = NP == 2;
  // wave tiles: X3 32 × 128 (each wave splits only its own A rows: no A fragment is split twice in a
  // workgroup), exact / X6 2 × 2 waves of BM/2 × 64
  constexpr int WGN = NP == 2 ? 1 : 2;  // waves along N
  constexpr int BM = NP == 3 ? 64 : 128, BN = 128, NW = 4, WTM = BM * WGN / NW, WTN = BN / WGN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int BH = NP == 3 ? 2 : 1;  // 128 B of LDS per weight row and K-tile (X6: one 256-B row)
  constexpr int AV = BM / 8 / NW, BV = BH * BN / 8 / NW;  // 1-KiB DMA instructions per wave per K-tile
  constexpr int WROW = BH * BKF;                           // floats per LDS weight row
  constexpr int LPS = AV + BV;
  constexpr int SLOT = (BM + BH * BN) * BKF;  // floats
  __shared__ __attribute__((aligned(16))) float lds[NS * SLOT];  // 96 / 64 / 80 KiB

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int nbx = gridDim.x;
  const int logical = rdmi::xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * gridDim.y);
  int mt_, nt_;
  rdmi::tile_mn(logical, nbx, gridDim.y, p.group_m, mt_, nt_);
  const int n0 = nt_ * BN, m0 = mt_ * BM;
  const int bz = blockIdx.z;
  const __amdgpu_buffer_rsrc_t ra_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (long)bz * p.sA), (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.Wt + (long)bz * p.sW), (short)0, (int)p.w_bytes, 0x00020000);

  const int lrow = lane >> 3;
  // DMA instruction i of this wave fills 8 rows (i·NW + wid)·8 + lrow of 128 B; a lane fetches the
  // logical 4-float chunk that lands at position lane & 7 of its row under the swizzle
  int arow[AV], ahb[AV], awb[AV], achk[AV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int rt = (i * NW + wid) * 8 + lrow;
    achk[i] = (lane & 7) ^ swz(rt & 15);
    const int m = m0 + rt;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    if (MODE != 0) {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw;
      const int r = mm - b * hw;
      const int ho = r / p.Wo;
      const int wo = r - ho * p.Wo;
      const int hb = ho * p.stride - p.pt;
      ahb[i] = ok ? hb : -(1 << 28);
      awb[i] = wo * p.stride - p.pl;
      arow[i] = MODE == 1 ? (b * p.IH + hb) * p.IW * p.Cin + awb[i] * p.Cin : b * p.IH * p.IW * p.Cin;
    } else {
      ahb[i] = ok ? 0 : -1;
      awb[i] = 0;
      arow[i] = mm * (int)p.lda;
    }
  }
  // weights: 128-B rows as A; X6: 256-B rows (hi | mid | lo | zero per K-tile), instruction i filling
  // rows (i·NW + wid)·4 + (lane >> 4), chunk c at position c ^ (row & 15)
  int brow[BV], bchk[BV];
#pragma unroll
  for (int i = 0; i < BV; ++i) {
    const int q = NP == 3 ? (i * NW + wid) * 4 + (lane >> 4) : (i * NW + wid) * 8 + lrow;
    bchk[i] = NP == 3 ? (lane & 15) ^ (q & 15) : (lane & 7) ^ swz(q & 15);
    const int n = n0 + q;
    brow[i] = n < p.N ? n * (int)p.ldw : -1;
  }
  const int Hl = p.IH << (MODE == 2 ? 1 : 0), Wl = p.IW << (MODE == 2 ? 1 : 0);
  const int wids = __builtin_amdgcn_readfirstlane(wid);
  // Fast addressing (round 5): when a K-tile never straddles a tap (dense A, or Cin % 32 == 0) and
  // lies inside Kvalid, a lane's A offset depends on the K-tile only through a wave-uniform step —
  // the channel offset within the tap, or ks·BKF — which goes in the buffer instruction's scalar
  // soffset; the per-lane row offsets (with the padding test) are recomputed only when the tap
  // changes.  Out-of-range lanes keep an OOB voffset, still out of range after the soffset.
  const bool fast = MODE == 0 || (p.cin_vecs % 8 == 0);
  unsigned aoff[AV];
  int atap = -1;
  auto tap_offsets = [&](int t) {
    const int dy = (t * 11) >> 5;  // t / 3 for t < 9
    const int dx = t - 3 * dy;
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      if (MODE == 0) {
        aoff[i] = ahb[i] == 0 ? (unsigned)(arow[i] + achk[i] * 4) * 4u : OOB;
      } else {
        const int hi = ahb[i] + dy, wi = awb[i] + dx;
        const bool ok = (unsigned)hi < (unsigned)Hl && (unsigned)wi < (unsigned)Wl;
        const int off = MODE == 1 ? arow[i] + (dy * p.IW + dx) * p.Cin + achk[i] * 4
                                  : arow[i] + ((hi >> 1) * p.IW + (wi >> 1)) * p.Cin + achk[i] * 4;
        aoff[i] = ok ? (unsigned)off * 4u : OOB;
      }
    }
  };
  unsigned boff[BV];
#pragma unroll
  for (int i = 0; i < BV; ++i) boff[i] = brow[i] >= 0 ? (unsigned)(brow[i] + bchk[i] * 4) * 4u : OOB;

  auto issue = [&](int ks, int slot) {
    float* la = lds + slot * SLOT;
    float* lb = la + BM * BKF;
    const bool whole = (ks + 1) * BKF <= p.Kvalid;  // wave-uniform
    if (fast && whole) {
      // K-tile ks: tap t0 = ks·BKF / Cin (uniform), channel step c0 within it
      const int k0 = ks * BKF;
      int t0 = 0, c0 = k0;
      if (MODE != 0) {
        t0 = k0 / p.Cin;
        c0 = k0 - t0 * p.Cin;
      }
      if (t0 != atap) {  // wave-uniform
        tap_offsets(t0);
        atap = t0;
      }
#pragma unroll
      for (int i = 0; i < AV; ++i) dma16f(ra_, aoff[i], la + (i * NW + wids) * 8 * BKF, c0 * 4);
    } else if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        const int kk = ks * BKF + achk[i] * 4;
        const bool ok = ahb[i] == 0 && kk < p.Kvalid;
        dma16f(ra_, ok ? (unsigned)(arow[i] + kk) * 4u : OOB, la + (i * NW + wids) * 8 * BKF);
      }
    } else {
      // general implicit im2col: this lane's (tap, channel chunk) of K-tile ks
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        const int kk = ks * BKF + achk[i] * 4;
        const bool kok = kk < p.Kvalid;
        const int tl = kk / p.Cin;  // per lane
        const int cl = kk - tl * p.Cin;
        const int dy = (tl * 11) >> 5, dx = tl - 3 * dy;
        const int hi = ahb[i] + dy, wi = awb[i] + dx;
        const bool ok = kok && (unsigned)hi < (unsigned)Hl && (unsigned)wi < (unsigned)Wl;
        const int off = MODE == 1 ? arow[i] + (dy * p.IW + dx) * p.Cin + cl
                                  : arow[i] + ((hi >> 1) * p.IW + (wi >> 1)) * p.Cin + cl;
        dma16f(ra_, ok ? (unsigned)off * 4u : OOB, la + (i * NW + wids) * 8 * BKF);
      }
    }
    // W: X3 / X6 K-tiles are always whole (split parts, zero padded past K); exact f32 rows end at K
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const bool wok = NP > 1 || ks * BKF + bchk[i] * 4 < p.Kvalid;
      dma16f(rw_, wok ? boff[i] : OOB, lb + (i * NW + wids) * 8 * BKF, ks * WROW * 4);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BKF - 1) / BKF;
  issue(0, 0);
  if (NS == 3) issue(1, 1);
  const int fr = lane & 15, fq = lane >> 4;
  const int gfr = swz(fr);  // swizzle of every fragment row of this lane (rows ≡ fr mod 16)
  for (int kt = 0; kt < nk; ++kt) {
    if (NS == 3)
      rdmi::wait_vmcnt_only<LPS>();  // K-tile kt landed (kt+1 in flight)
    else
      rdmi::wait_vmcnt_only<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(kt + NS - 1, (kt + NS - 1) % NS);  // into the slot read last in K-tile kt-1
    const float* la = lds + (kt % NS) * SLOT + (wm * WTM) * BKF;
    const float* lb = lds + (kt % NS) * SLOT + BM * BKF + (wn * WTN) * WROW;
    if constexpr (NP == 3) {
      // lane quarter fq holds k = 8fq .. 8fq+7: A as f32 chunks 2fq, 2fq+1 split three ways; W as bf16
      // chunks fq (hi), 4+fq (mid) and 8+fq (lo) of its 256-B row
      bf16x8 as[RM][3], bs[RN][3];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = i * 16 + fr;
        const f32x4 a0 = *(const f32x4*)(la + row * BKF + (((2 * fq) ^ gfr) << 2));
        const f32x4 a1 = *(const f32x4*)(la + row * BKF + (((2 * fq + 1) ^ gfr) << 2));
        unsigned h[4], m[4], l[4];
        rdmi::split3_bf16x2(a0[0], a0[1], h[0], m[0], l[0]);
        rdmi::split3_bf16x2(a0[2], a0[3], h[1], m[1], l[1]);
        rdmi::split3_bf16x2(a1[0], a1[1], h[2], m[2], l[2]);
        rdmi::split3_bf16x2(a1[2], a1[3], h[3], m[3], l[3]);
        as[i][0] = __builtin_bit_cast(bf16x8, u32x4{h[0], h[1], h[2], h[3]});
        as[i][1] = __builtin_bit_cast(bf16x8, u32x4{m[0], m[1], m[2], m[3]});
        as[i][2] = __builtin_bit_cast(bf16x8, u32x4{l[0], l[1], l[2], l[3]});
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const float* wr = lb + (j * 16 + fr) * WROW;  // row ≡ fr mod 16
        bs[j][0] = *(const bf16x8*)(wr + ((fq ^ fr) << 2));
        bs[j][1] = *(const bf16x8*)(wr + (((4 + fq) ^ fr) << 2));
        bs[j][2] = *(const bf16x8*)(wr + (((8 + fq) ^ fr) << 2));
      }
      // (weight part, activation part), largest first
      constexpr int wpart[6] = {0, 0, 1, 1, 0, 2}, apart[6] = {0, 1, 0, 1, 2, 0};
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int t = 0; t < 6; ++t)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bs[j][wpart[t]], as[i][apart[t]], acc[i][j], 0, 0, 0);
      continue;
    }
    if constexpr (X3) {
      // lane quarter fq holds k = 8fq .. 8fq+7 of its row in both operands (the bf16 16x16x32 layout):
      // A as f32 chunks 2fq, 2fq+1 (split here), W as bf16 chunks fq (hi) and 4+fq (lo)
      bf16x8 ah[RM], al[RM], bh[RN], bl[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = i * 16 + fr;
        const f32x4 a0 = *(const f32x4*)(la + row * BKF + (((2 * fq) ^ gfr) << 2));
        const f32x4 a1 = *(const f32x4*)(la + row * BKF + (((2 * fq + 1) ^ gfr) << 2));
        rdmi::split_bf16x8(a0, a1, ah[i], al[i]);
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = j * 16 + fr;
        bh[j] = *(const bf16x8*)(lb + row * BKF + ((fq ^ gfr) << 2));
        bl[j] = *(const bf16x8*)(lb + row * BKF + (((4 + fq) ^ gfr) << 2));
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al[i], acc[i][j], 0, 0, 0);
        }
      continue;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lc = 2 * fq + h;  // logical chunk: k = 8·fq + 4h + (0..3)
      f32x4 af[RM], bf[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int row = i * 16 + fr;
        af[i] = *(const f32x4*)(la + row * BKF + ((lc ^ gfr) << 2));
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int row = j * 16 + fr;
        bf[j] = *(const f32x4*)(lb + row * BKF + ((lc ^ gfr) << 2));
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[j][s], af[i][s], acc[i][j], 0, 0, 0);
    }
  }
  rdmi::wait_vmcnt_only<0>();
  store_tile_f32<RM, RN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, bz, fr, fq);
}

bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

bool vec_ok(const GemmF32P& p) {
  bool ok = p.ldc % 4 == 0 && p.sC % 4 == 0 && al16(p.C);
  if (p.R) ok = ok && p.ldr % 4 == 0 && p.sR % 4 == 0 && al16(p.R);
  if (p.bias) ok = ok && al16(p.bias);
  if (p.rowbias) ok = ok && al16(p.rowbias) && p.rb_ld % 4 == 0;
  return ok;
}

int launch_f32(GemmF32P p, int batch, hipStream_t s, int mode, int np) {
  const char* gm = getenv("RDMI_GEMM_GROUP");
  p.group_m = gm ? atoi(gm) : 8;
  const bool x3 = np == 2;
  dim3 g(rdmi::div_up(p.N, 128), rdmi::div_up(p.M, np == 3 ? 64 : 128), batch);
  // RDMI_F32_SLOTS (read per launch, A/B): unset / 2 = two workgroups per CU with a 2-slot ring (the
  // default: +30-40 % for the bf16-split products, +12-15 % exact, bitwise the same —
  // profiles/r03k_f32_slots_ab.log), 3 = one workgroup per CU with a 3-slot ring
  const char* se = getenv("RDMI_F32_SLOTS");
  const bool ns2 = !(se && se[0] == '3');
#define RDMI_F32_LAUNCH(M)                                                                     \
  if (np == 3)                                                                                 \
    hipLaunchKernelGGL((gemm_f32_kernel<M, 3, 2>), g, dim3(256), 0, s, p);                    \
  else if (x3 && ns2)                                                                          \
    hipLaunchKernelGGL((gemm_f32_kernel<M, 2, 2>), g, dim3(256), 0, s, p);                    \
  else if (x3)                                                                                 \
    hipLaunchKernelGGL((gemm_f32_kernel<M, 2, 3>), g, dim3(256), 0, s, p);                    \
  else if (ns2)                                                                                \
    hipLaunchKernelGGL((gemm_f32_kernel<M, 1, 2>), g, dim3(256), 0, s, p);                    \
  else                                                                                         \
    hipLaunchKernelGGL((gemm_f32_kernel<M, 1, 3>), g, dim3(256), 0, s, p);
  if (mode == 2) {
    RDMI_F32_LAUNCH(2)
  } else if (mode == 1) {
    RDMI_F32_LAUNCH(1)
  } else {
    RDMI_F32_LAUNCH(0)
  }
#undef RDMI_F32_LAUNCH
  return rdmi::check_launch(np == 3 ? "gemm_f32x6" : x3 ? "gemm_f32x3" : "gemm_f32");
}

}  // namespace

namespace rdmi {

int gemm_f32(const rdmi_gemm_args* a, void* stream) {
  const int np = a->dtype == RDMI_F32_X6 ? 3 : a->dtype == RDMI_F32_X3 ? 2 : 1;
  const bool x3 = np > 1;
  // X3 / X6: W is the bf16 split layout, ldw in bf16 elements (2 / 4 per f32 K position)
  const long ldw = x3 ? a->ldw / 2 : a->ldw;
  RDMI_REQUIRE(!x3 || (a->ldw % 64 == 0), RDMI_E_ALIGN, "gemm f32x3/x6: ldw (%ld bf16) must be a multiple of 64", a->ldw);
  const int Kt = (a->K + BKF - 1) / BKF * BKF;
  const long kw = np == 3 ? 2L * Kt : x3 ? Kt : a->K;  // floats of a weight row that the K-tiles read
  RDMI_REQUIRE(a->K % 4 == 0 && a->lda % 4 == 0 && ldw % 4 == 0 && ldw >= kw, RDMI_E_ALIGN,
               "gemm f32: K (%d), lda (%ld), ldw (%ld) must be multiples of 4 (ldw >= K)", a->K, a->lda, ldw);
  RDMI_REQUIRE(al16(a->A) && al16(a->W) && a->strideA % 4 == 0 && a->strideW % 4 == 0, RDMI_E_ALIGN,
               "gemm f32: A/W not 16-byte aligned");
  RDMI_REQUIRE(a->epilogue != RDMI_EPI_GEGLU || a->N % 128 == 0, RDMI_E_ARG, "gemm f32: GEGLU needs N %% 128 == 0");
  RDMI_REQUIRE(!a->rowbias || a->rows_per_group > 0, RDMI_E_ARG, "gemm f32: rowbias needs rows_per_group");
  RDMI_REQUIRE(!a->gn_part, RDMI_E_UNSUPPORTED, "gemm f32: no GroupNorm moments (the groupnorm pass computes them)");
  RDMI_REQUIRE((long)a->M * a->lda < (1L << 29) && (long)a->N * ldw < (1L << 29), RDMI_E_ARG,
               "gemm f32: operand exceeds 2^29 elements (2 GiB) per batch");
  GemmF32P p{};
  p.A = (const float*)a->A; p.lda = a->lda; p.sA = a->strideA;
  p.Wt = (const float*)a->W; p.ldw = ldw; p.sW = x3 ? a->strideW / 2 : a->strideW;
  p.C = (float*)a->C; p.ldc = a->ldc; p.sC = a->strideC;
  p.bias = a->bias; p.R = (const float*)a->residual; p.ldr = a->ldr; p.sR = a->strideR;
  p.rowbias = a->rowbias; p.rpg = a->rows_per_group > 0 ? a->rows_per_group : 1; p.rb_ld = a->rowbias_ld;
  p.alpha = a->alpha;
  p.M = a->M; p.N = a->N; p.K = (a->K + BKF - 1) / BKF * BKF; p.Kvalid = a->K;
  p.geglu = a->epilogue == RDMI_EPI_GEGLU;
  p.silu = a->epilogue == RDMI_EPI_SILU;
  p.vec = vec_ok(p);
  RDMI_REQUIRE(!p.geglu || p.vec, RDMI_E_ALIGN, "gemm f32: GEGLU output needs 4-element aligned rows");
  p.a_bytes = (unsigned)(((long)(a->M - 1) * a->lda + a->K) * 4);
  p.w_bytes = (unsigned)(((long)(a->N - 1) * ldw + kw) * 4);
  return launch_f32(p, a->batch, (hipStream_t)stream, 0, np);
}

int conv2d_f32(const rdmi_conv_args* a, void* stream) {
  // Kp counts f32 K positions (the bf16 rows are 2·Kp long for X3, 4·Kp for X6)
  const int np = a->dtype == RDMI_F32_X6 ? 3 : a->dtype == RDMI_F32_X3 ? 2 : 1;
  const bool x3 = np > 1;
  RDMI_REQUIRE(a->Cin % 4 == 0, RDMI_E_ALIGN, "conv2d f32: Cin (%d) must be a multiple of 4", a->Cin);
  const int K = a->kh * a->kw * a->Cin;
  RDMI_REQUIRE(a->Kp >= K && a->Kp % (x3 ? 32 : 4) == 0, RDMI_E_ARG, "conv2d f32: Kp (%d) must be >= %d, a multiple of %d",
               a->Kp, K, x3 ? 32 : 4);
  RDMI_REQUIRE(al16(a->x) && al16(a->w), RDMI_E_ALIGN, "conv2d f32: x/w not 16-byte aligned");
  RDMI_REQUIRE((long)a->B * a->H * a->W * a->Cin < (1L << 29) && (long)a->Cout * a->Kp < (1L << 29), RDMI_E_ARG,
               "conv2d f32: input exceeds 2^29 elements (2 GiB; split the batch)");
  RDMI_REQUIRE(!a->in_mean_rstd, RDMI_E_UNSUPPORTED, "conv2d f32: no fused input GroupNorm");
  RDMI_REQUIRE(!a->gn_part, RDMI_E_UNSUPPORTED, "conv2d f32: no GroupNorm moments");
  GemmF32P p{};
  p.A = (const float*)a->x; p.Wt = (const float*)a->w; p.ldw = np == 3 ? 2L * a->Kp : a->Kp;
  p.C = (float*)a->y; p.ldc = a->y_ld > 0 ? a->y_ld : a->Cout;
  p.bias = a->bias; p.R = (const float*)a->residual; p.ldr = a->res_ld > 0 ? a->res_ld : a->Cout;
  p.rowbias = a->rowbias; p.rpg = a->Ho * a->Wo; p.rb_ld = a->rowbias_ld;
  p.alpha = a->alpha;
  p.M = a->B * a->Ho * a->Wo; p.N = a->Cout; p.K = (a->Kp + BKF - 1) / BKF * BKF; p.Kvalid = K;
  p.IH = a->H; p.IW = a->W; p.Cin = a->Cin; p.Ho = a->Ho; p.Wo = a->Wo;
  p.stride = a->stride; p.pt = a->pad_top; p.pl = a->pad_left; p.cin_vecs = a->Cin / 4;
  const bool dense = a->kh == 1 && a->kw == 1 && a->stride == 1 && a->pad_top == 0 && a->pad_left == 0 && !a->upsample &&
                     a->Ho == a->H && a->Wo == a->W;
  if (dense) p.lda = a->Cin;
  RDMI_REQUIRE(dense || (a->kh == 3 && a->kw == 3), RDMI_E_UNSUPPORTED, "conv2d f32: only 3x3 and dense 1x1 kernels");
  RDMI_REQUIRE(!a->upsample || a->stride == 1, RDMI_E_UNSUPPORTED, "conv2d f32: upsample needs stride 1");
  p.vec = vec_ok(p);
  p.a_bytes = (unsigned)((long)a->B * a->H * a->W * a->Cin * 4);
  p.w_bytes = (unsigned)((long)a->Cout * p.ldw * 4);
  return launch_f32(p, 1, (hipStream_t)stream, dense ? 0 : (a->upsample ? 2 : 1), np);
}

}  // namespace rdmi

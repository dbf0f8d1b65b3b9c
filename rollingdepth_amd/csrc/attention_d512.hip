// Single-head flash attention for head dim 512: the VAE mid-block attention of the SD VAE
// (unet_2d_blocks.py:680-697, AttnProcessor2_0's 4-D path: one head, d = C = 512, S = h·w tokens —
// 9 216 at 768²), replacing f32 scores GEMM → row softmax → PV GEMM (which streams 340 MB of f32
// scores per frame through HBM twice) with one pass over K / Vᵀ.
//
// Workgroup = 8 waves × 16 queries (128 queries of one image), one workgroup per CU (128 KiB of
// LDS: two stages of a 32-key K tile [32 keys][512] and its Vᵀ tile [512][32 keys]); every wave
// is independent apart from the shared tiles (one barrier per tile, for the stage reuse):
//   Sᵀ = K·Qᵀ with v_mfma_f32_16x16x32_f16: the wave's Q fragments (16 queries × 512) live in
//     registers for the whole sweep; A-row i of key block kb reads key κ = 8(i >> 2) + 4kb +
//     (i & 3), so that the accumulator entries of a lane (rows 4hq + r of blocks 0 and 1) are the 8
//     CONSECUTIVE keys 8hq + 0..7 — the f16 P feeds the PV MFMA as its B operand straight from
//     registers (no LDS round trip, no cross-lane move);
//   online softmax in the exp2 domain per lane (one query per lane; the row reduction is
//     lane-local plus two lane-xor exchanges), the running max m̃ set on the first tile and re-set —
//     with the O / l rescale — only when a tile's row sum would leave the f16 range of P (> 2^15);
//   Oᵀ += Vᵀ·Pᵀ: 32 d-blocks of 16 rows, one 32-key k-step; 128 f32 accumulators per lane.
// LDS images: 16-B chunk swizzles (kswz / vswz below) applied on the DMA source offsets.  Keys
// past Sk read as zeros (K beyond the buffer; Vᵀ zero-padded to a multiple of 32 by the caller)
// and are masked to −inf.
#include "common.h"

namespace {

constexpr int D5 = 512;
constexpr int NW5 = 8;           // waves per workgroup (two per SIMD)
constexpr int QB5 = 16 * NW5;    // queries per workgroup (16 per wave)
constexpr int KT5 = 32;          // keys per tile
constexpr int KTILE = KT5 * D5;  // halves per K (or Vᵀ) tile
constexpr int STAGE = 2 * KTILE;
constexpr int PPW = 32 / NW5;    // 1-KiB DMA pieces per wave per tile, per tensor

// 16-B chunk swizzles of the LDS tiles, conflict-free for the ds_read_b128 lane groups
// {0–3,12–15,20–27}, {4–11,16–19,28–31} (+32) of the fragment reads: K row k (64 chunks), the
// low 4 bits of the chunk XORed with (k & 3) | ((k >> 3) & 3) << 2 — the rows a group reads,
// κ = 8(j >> 2) + 4kb + (j & 3), then cover all 16 bank groups; Vᵀ row d (4 chunks) XORed with
// 3·((d >> 3) & 1).
__device__ __forceinline__ int kswz(int k) { return (k & 3) | (((k >> 3) & 3) << 2); }
__device__ __forceinline__ int vswz(int d) { return ((d >> 3) & 1) * 3; }

struct Attn512P {
  const f16* q; const f16* k; const f16* vt; f16* o;
  int Sq, Sk, Skp;
  long q_ld, k_ld, vt_ld, o_ld, q_bs, k_bs, vt_bs, o_bs;
  float c;  // scale · log2(e)
  int* flags;  // [B][ceil(Sq / 128)]: set by the 32-query pass where its fixed m̃ failed (see below)
};

__global__ __launch_bounds__(64 * NW5, 1) void attn_fwd_d512(Attn512P p) {
  __shared__ __attribute__((aligned(16))) f16 lds5[2 * STAGE];  // 2 stages × [K tile | Vᵀ tile] (128 KiB)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int hq = lane >> 4;   // lane quarter
  const int j16 = lane & 15;
  // dispatch order (query block fastest): every XCD takes part in every image.  The XCD-local order of
  // the d = 64 kernel (rdmi::xcd_block3: one image per XCD) measured 2-4 % slower here, bitwise equal
  // (profiles/r06a_attn_xcd_ab.log; an image's 19 MB of K / Vᵀ exceeds one XCD's 4 MB L2 either way)
  const int qblk = blockIdx.x, b = blockIdx.y;
  const int q = qblk * QB5 + wid * 16 + j16;
  // as the fix-up pass behind attn_fwd_d512_w4: only the 128-query blocks that pass flagged
  if (p.flags && p.flags[b * gridDim.x + qblk] == 0) return;

  const f16* Q = p.q + (long)b * p.q_bs;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.k + (long)b * p.k_bs), (short)0, (int)(((long)(p.Sk - 1) * p.k_ld + D5) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.vt + (long)b * p.vt_bs), (short)0, (int)(((long)(D5 - 1) * p.vt_ld + p.Skp) * 2), 0x00020000);

  // Q fragments (the B operand of Sᵀ = K·Qᵀ, 16×16×32): lane holds Q[q][32ks + 8hq .. +8]
  f16x8 qf[16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    f16x8 z = {};
    qf[ks] = q < p.Sq ? *(const f16x8*)(Q + (long)q * p.q_ld + ks * 32 + hq * 8) : z;
  }

  // DMA geometry.  K: piece e of this wave = key row kr = PPW·wid + e (1 KiB), lane L writes
  // physical chunk L ← logical chunk L ^ kswz(kr).  Vᵀ: piece pp = PPW·wid + e = rows 16pp +
  // (L >> 2), physical chunk L & 3 ← logical (L & 3) ^ vswz(d).
  unsigned koff[PPW], voff[PPW];
#pragma unroll
  for (int e = 0; e < PPW; ++e) {
    const int kr = PPW * wid + e;
    koff[e] = (unsigned)((kr * p.k_ld + ((lane ^ kswz(kr)) << 3)) * 2);
    const int d = 16 * (PPW * wid + e) + (lane >> 2);
    voff[e] = (unsigned)((d * p.vt_ld + (((lane & 3) ^ vswz(d)) << 3)) * 2);
  }
  auto issue = [&](int t) {
    f16* st = lds5 + (t & 1) * STAGE;
#pragma unroll
    for (int e = 0; e < PPW; ++e) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(st + (PPW * wid + e) * 512),
                                               16, koff[e], t * KT5 * (int)p.k_ld * 2, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(st + KTILE + (PPW * wid + e) * 512),
                                               16, voff[e], t * KT5 * 2, 0, 0);
    }
  };

  // Fragment addresses (bytes).  Sᵀ = K·Qᵀ for key block kb (16 keys): A-row i = j16 reads key
  // κ = 8(i >> 2) + 4kb + (i & 3), so that the accumulator entries r of a lane (rows 4hq + r) of
  // blocks kb = 0, 1 are the 8 CONSECUTIVE keys 8hq + 4kb + r — the lane's own f16 P is then the
  // PV B fragment for k-slots 8hq .. 8hq + 7.  K row κ, logical chunk 4ks + hq at
  // (4ks + hq) ^ kswz(κ) = 16(ks >> 2) + ((4(ks & 3) + hq) ^ kswz(κ)).  Vᵀ operand row d = 16db +
  // j16, chunk hq at hq ^ vswz(d) = hq ^ vswz(j16); 16db rows (1 KiB) an immediate.
  const unsigned base0 = (unsigned)(uintptr_t)LDS_PTR(f16, lds5);
  unsigned kaddr[2][4], vaddr;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int kap = 8 * (j16 >> 2) + 4 * kb + (j16 & 3);
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) kaddr[kb][b4] = (unsigned)(kap * 1024 + (((4 * b4 + hq) ^ kswz(kap)) << 4));
  }
  vaddr = (unsigned)(KTILE * 2 + j16 * 64 + ((hq ^ vswz(j16)) << 4));

  f32x4 o[32];  // Oᵀ blocks: d-block db (16 rows) × this wave's 16 queries
#pragma unroll
  for (int db = 0; db < 32; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mt = 0.f, l = 0.f;  // m̃ (in units of score·c) and this query's row sum

  const int nt = p.Skp / KT5;
  issue(0);
  for (int t = 0; t < nt; ++t) {
    __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));  // vmcnt(0) alone: this wave's pieces of tile t landed
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces landed; tile t-1 fully read
    asm volatile("" ::: "memory");
    if (t + 1 < nt) issue(t + 1);
    const unsigned st = base0 + (unsigned)((t & 1) * STAGE * 2);

    // ---- Sᵀ = K · Qᵀ: two 16-key blocks, 16 k-steps of 32
    f32x4 s[2] = {};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const f16x8 kf = *(const f16x8*)LDS_PTR(f16, (uintptr_t)(st + kaddr[kb][ks & 3] + (ks >> 2) * 256));
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[ks], s[kb], 0, 0, 0);
      }
    // ---- softmax: entry r of block kb = key 8hq + 4kb + r of the tile
    const int kb0 = t * KT5;
    if (kb0 + KT5 > p.Sk) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kb0 + 8 * hq + 4 * kb + r >= p.Sk) s[kb][r] = -INFINITY;
    }
    float pv[8];
    float rs = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pv[e] = __builtin_amdgcn_exp2f(fmaf(s[e >> 2][e & 3], p.c, -mt));
      rs += pv[e];
    }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    if (t == 0 || __any(!(rs <= 32768.f))) {
      float mx = -INFINITY;
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = fmaxf(mx, s[e >> 2][e & 3] * p.c);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = t == 0 ? mx : fmaxf(mt, mx);
      if (t == 0 || mnew > mt) {
        const float alpha = t == 0 ? 0.f : __builtin_amdgcn_exp2f(mt - mnew);
        l *= alpha;
        if (t != 0) {
#pragma unroll
          for (int db = 0; db < 32; ++db) o[db] *= alpha;
        }
        mt = mnew;
      }
      rs = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pv[e] = __builtin_amdgcn_exp2f(fmaf(s[e >> 2][e & 3], p.c, -mt));
        rs += pv[e];
      }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
    }
    l += rs;
    f16x8 pf;
#pragma unroll
    for (int e = 0; e < 8; ++e) pf[e] = (f16)pv[e];
    // ---- Oᵀ += Vᵀ · Pᵀ (32 d-blocks of 16 rows, one k-step of 32 keys)
#pragma unroll
    for (int db = 0; db < 32; ++db) {
      const f16x8 vf = *(const f16x8*)LDS_PTR(f16, (uintptr_t)(st + vaddr + db * 1024));
      o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf, o[db], 0, 0, 0);
    }
  }
  // ---- O[q][d] = Oᵀ[d][q] / l: lane holds d = 16db + 4hq + r for its query
  if (q < p.Sq) {
    const float inv = 1.f / l;
    f16* O = p.o + (long)b * p.o_bs + (long)q * p.o_ld;
#pragma unroll
    for (int db = 0; db < 32; ++db) {
      f16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (f16)(o[db][r] * inv);
      *(f16x4*)(O + 16 * db + 4 * hq) = w;
    }
  }
}


// Variant: 4 waves × 32 queries (one wave per SIMD, 512 registers per wave) with
// v_mfma_f32_32x32x16_f16 — every K / Vᵀ fragment read from LDS feeds twice the MFMA work of the
// 16-query form (whose LDS traffic, 1 KiB per 16-cycle MFMA per wave, caps it near half the MFMA
// rate), the 32×512 f32 Oᵀ accumulator in the AGPRs.  K operand row i = 8j + 4hh + r reads key
// κ = 16(j >> 1) + 8hh + 4(j & 1) + r so that a lane's accumulator entries for PV k-step s are the
// consecutive keys 16s + 8hh + 0..7.  Fragment reads are pinned two MFMAs ahead
// (sched_group_barrier) so that the compiler does not hoist the whole tile's reads.
// No VALU may touch O inside the loop (an in-place `o *= alpha` moves the 256 accumulators out of
// the AGPRs: 354 spilled registers), so m̃ is fixed by the first tile; a wave whose later tile
// would overflow the f16 P marks its 128-query block in p.flags and skips its store, and the
// 16-query kernel (which rescales) re-runs exactly the marked blocks.  Measured 693 TF/s against
// the 16-query kernel's 816 (B = 75, S = 9216): with one wave per SIMD nothing overlaps a wave's
// own QKᵀ → softmax → PV chain — kept opt-in (RDMI_D512_W4=1, kernels.attention_d512).
__device__ __forceinline__ int kswz32(int k) { return k & 15; }
__device__ __forceinline__ int vswz32(int d) { return (d >> 2) & 3; }

template <int N>
__device__ __forceinline__ void w4_sched() {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
}

__global__ __launch_bounds__(256, 1) void attn_fwd_d512_w4(Attn512P p) {
  __shared__ __attribute__((aligned(16))) f16 lds5[2 * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int hh = lane >> 5;
  const int j32 = lane & 31;
  const int qblk = blockIdx.x, b = blockIdx.y;
  const int q = qblk * 128 + wid * 32 + j32;

  const f16* Q = p.q + (long)b * p.q_bs;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.k + (long)b * p.k_bs), (short)0, (int)(((long)(p.Sk - 1) * p.k_ld + D5) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.vt + (long)b * p.vt_bs), (short)0, (int)(((long)(D5 - 1) * p.vt_ld + p.Skp) * 2), 0x00020000);

  f16x8 qf[32];
#pragma unroll
  for (int ks = 0; ks < 32; ++ks) {
    f16x8 z = {};
    qf[ks] = q < p.Sq ? *(const f16x8*)(Q + (long)q * p.q_ld + ks * 16 + hh * 8) : z;
  }
  unsigned koff[8], voff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kr = 8 * wid + e;
    koff[e] = (unsigned)((kr * p.k_ld + ((lane ^ kswz32(kr)) << 3)) * 2);
    const int d = 16 * (8 * wid + e) + (lane >> 2);
    voff[e] = (unsigned)((d * p.vt_ld + (((lane & 3) ^ vswz32(d)) << 3)) * 2);
  }
  auto issue = [&](int t) {
    f16* st = lds5 + (t & 1) * STAGE;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(st + (8 * wid + e) * 512),
                                               16, koff[e], t * KT5 * (int)p.k_ld * 2, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(st + KTILE + (8 * wid + e) * 512),
                                               16, voff[e], t * KT5 * 2, 0, 0);
    }
  };
  const int jj = j32 >> 3, hk = (j32 >> 2) & 1, rr = j32 & 3;
  const int kap = 16 * (jj >> 1) + 8 * hk + 4 * (jj & 1) + rr;
  const unsigned base0 = (unsigned)(uintptr_t)LDS_PTR(f16, lds5);
  unsigned kaddr[8], vaddr[2];
#pragma unroll
  for (int bks = 0; bks < 8; ++bks) kaddr[bks] = (unsigned)(kap * 1024 + (((2 * bks + hh) ^ kswz32(kap)) << 4));
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) vaddr[s2] = (unsigned)(KTILE * 2 + j32 * 64 + (((2 * s2 + hh) ^ vswz32(j32)) << 4));

  f32x16 o[16];
#pragma unroll
  for (int db = 0; db < 16; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float mt = 0.f, l = 0.f;
  bool bad = false;
  const int nt = p.Skp / KT5;
  issue(0);
  for (int t = 0; t < nt; ++t) {
    __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < nt) issue(t + 1);
    const unsigned st = base0 + (unsigned)((t & 1) * STAGE * 2);
    f32x16 s = {};
#pragma unroll
    for (int ks = 0; ks < 32; ++ks) {
      const f16x8 kf = *(const f16x8*)LDS_PTR(f16, (uintptr_t)(st + kaddr[ks & 7] + (ks >> 3) * 256));
      s = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[ks], s, 0, 0, 0);
    }
    w4_sched<32>();
    const int kb0 = t * KT5;
    if (kb0 + KT5 > p.Sk) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int jx = e >> 2;
        if (kb0 + 16 * (jx >> 1) + 8 * hh + 4 * (jx & 1) + (e & 3) >= p.Sk) s[e] = -INFINITY;
      }
    }
    if (t == 0) {
      float mx = -INFINITY;
#pragma unroll
      for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s[e] * p.c);
      mt = fmaxf(mx, __shfl_xor(mx, 32, 64));
    }
    float pv[16];
    float rs = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      pv[e] = __builtin_amdgcn_exp2f(fmaf(s[e], p.c, -mt));
      rs += pv[e];
    }
    rs += __shfl_xor(rs, 32, 64);
    // m̃ is fixed after the first tile: a later tile whose row sum leaves the f16 range of P
    // (or overflows) marks the block for the fix-up pass instead of rescaling O here
    bad |= __any(!(rs <= 32768.f));
    l += rs;
    f16x8 pf[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) pf[e >> 3][e & 7] = (f16)pv[e];
#pragma unroll
    for (int db = 0; db < 16; ++db)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const f16x8 vf = *(const f16x8*)LDS_PTR(f16, (uintptr_t)(st + vaddr[s2] + db * 2048));
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[s2], o[db], 0, 0, 0);
      }
    w4_sched<32>();
  }
  // block flag = OR over the four waves (all tiles are consumed: the LDS stages are free)
  int* badw = (int*)lds5;
  __syncthreads();
  if (lane == 0) badw[wid] = bad;
  __syncthreads();
  if (tid == 0) p.flags[b * gridDim.x + qblk] = badw[0] | badw[1] | badw[2] | badw[3];
  if (q < p.Sq && !bad) {
    const float inv = 1.f / l;
    f16* O = p.o + (long)b * p.o_bs + (long)q * p.o_ld;
#pragma unroll
    for (int db = 0; db < 16; ++db)
#pragma unroll
      for (int jx = 0; jx < 4; ++jx) {
        f16x4 w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = (f16)(o[db][4 * jx + r] * inv);
        *(f16x4*)(O + 32 * db + 8 * jx + 4 * hh) = w;
      }
  }
}

}  // namespace

extern "C" int rdmi_attention_d512(const void* q, const void* k, const void* vt, void* o, int B, int Sq, int Sk, int Skp,
                                   long q_ld, long k_ld, long vt_ld, long o_ld, long q_bs, long k_bs, long vt_bs,
                                   long o_bs, float scale, int* flags, void* stream) {
  RDMI_REQUIRE(q && k && vt && o, RDMI_E_ARG, "attention_d512: null pointer");
  RDMI_REQUIRE(B > 0 && Sq > 0 && Sk > 0 && Skp >= Sk && Skp % 32 == 0 && vt_ld >= Skp, RDMI_E_ARG,
               "attention_d512: bad sizes (Skp %% 32 == 0, Skp >= Sk, vt_ld >= Skp)");
  RDMI_REQUIRE(q_ld % 8 == 0 && k_ld % 8 == 0 && vt_ld % 8 == 0 && o_ld % 4 == 0 &&
                   (((uintptr_t)q | (uintptr_t)k | (uintptr_t)vt) & 15) == 0 && ((uintptr_t)o & 7) == 0,
               RDMI_E_ALIGN, "attention_d512: strides / pointers not aligned");
  RDMI_REQUIRE((long)(Sk - 1) * k_ld + D5 < (1L << 30) && (long)(D5 - 1) * vt_ld + Skp < (1L << 30), RDMI_E_ARG,
               "attention_d512: K / Vᵀ exceed the 2 GiB buffer range");
  Attn512P p{(const f16*)q, (const f16*)k, (const f16*)vt, (f16*)o, Sq, Sk, Skp, q_ld, k_ld, vt_ld, o_ld,
             q_bs, k_bs, vt_bs, o_bs, scale * 1.4426950408889634f, flags};
  // flags given: the 32-query pass, then the 16-query kernel as its fix-up over the flagged blocks
  // only (the same 128-query blocks; unflagged workgroups return on their first load)
  const dim3 grid(rdmi::div_up(Sq, QB5), B);
  if (flags) {
    hipLaunchKernelGGL(attn_fwd_d512_w4, grid, dim3(256), 0, (hipStream_t)stream, p);
    if (int e = rdmi::check_launch("attention_d512 (32-query pass)")) return e;
  }
  hipLaunchKernelGGL(attn_fwd_d512, grid, dim3(64 * NW5), 0, (hipStream_t)stream, p);
  return rdmi::check_launch("attention_d512");
}

// Cross-frame attention kernels.
//
// attn_fwd_d64: flash-style fused softmax(q kᵀ·scale) v for head_dim 64 on gfx950.
//   Workgroup = 8 waves × 32 queries (256 queries) of one (batch, head); 128-key K/V tiles arrive
//   by LDS-DMA into a 5-slot ring (K XOR-swizzled per 16-B chunk through the source address); the
//   two halves of the workgroup run staggered by one barrier (MFMA block ∥ softmax block).
//   Per wave and tile: Sᵀ = K·Qᵀ with v_mfma_f32_32x32x16_f16 (Q fragments live in registers for
//   the whole sweep), so each lane owns one query's scores ("swapped QKᵀ": the row max/sum is
//   lane-local plus one lane^32 exchange); Oᵀ = Vᵀ·Pᵀ with the P accumulator re-used directly
//   as the B operand (keys in the MFMA's permuted k order) and V read from LDS with
//   ds_read_b64_tr_b16 (hardware transpose).  Online softmax in exp2 domain with the running max
//   entering the QKᵀ MFMA chain as its initial accumulator (details at the kernel).
// attn_smallkv: attention of every query token against ≤ 16 shared keys (the UNet's
//   cross-attention to the 2-token empty-text context) — a streaming kernel, no MFMA.
// softmax_rows: f32 scores → f16 probabilities, for the d=C single-head VAE attention that is
//   run as GEMM → softmax → GEMM.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace {

struct AttnP {
  const f16* q; const f16* k; const f16* v; f16* o;
  int H, Sq, Sk;
  long q_ld, k_ld, v_ld, o_ld, q_bs, k_bs, v_bs, o_bs;
  float sl2;  // scale * log2(e)
  unsigned long long* stamps;  // STAMP builds only (tools/attn_stamp.hip): per-wave segment cycle sums
  int sprio;                   // attn_fwd_d64: the softmax block at s_setprio 2 (RDMI_ATTN_SPRIO, A/B)
};

// In-kernel stamp (diagnostic builds, STAMP = 1; guide §7 'In-kernel stamps'): s_memtime with the
// lgkmcnt(0) it needs in one statement, fenced from the scheduler on both sides.
__device__ __forceinline__ unsigned long long attn_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

constexpr int NWV = 8;        // waves per workgroup
constexpr int QB = 32 * NWV;  // queries per workgroup (32 per wave)
constexpr int KB = 128;       // keys per tile
constexpr int NKB = KB / 32;  // 32-key MFMA blocks per tile
constexpr int DPW = KB / 8 / NWV;  // 8-row DMA instructions per wave per tile, per tensor
constexpr int TILE = KB * 64; // halves per K (or V) tile

template <int N>
__device__ __forceinline__ void attn_wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}

// K/V tiles arrive by LDS-DMA (buffer_load_dwordx4 … lds) into a 5-slot ring (no VGPR staging,
// no ds_write): each wave moves 8 key rows of K and of V per tile.  K's 16-B chunks are
// XOR-swizzled by (key & 7) through the per-lane source offset; V stays row-major for the
// transposed reads.  Keys past Sk fall outside the buffer descriptors' range and read as zeros.
//
// Softmax VALU budget.  Q is prescaled by scale·log2(e) once, and the running row maximum m̃ enters
// the Sᵀ = K·Qᵀ MFMA chain as its initial accumulator (-m̃ in all 16 entries of a lane: in the swapped
// layout a lane's accumulator entries all belong to its one query), so the chain delivers
// S' = scores − m̃ directly and each score costs only exp2, half a cvt_pk and half a packed f16 add
// (the row sum is a pairwise v_pk_add_f16 tree over the f16 P the PV MFMA consumes).  The
// rescale is rare: m̃ is set exactly on the first tile and re-set — with the O/l rescale — only
// when a tile's row sum over this lane's 64 keys exceeds 2^15 (the f16 range of P), i.e. when
// the row max grew by more than ≈9 (log2 units); otherwise P stays bounded by 2^15 and f16 P keeps
// its relative precision.  (Earlier form: m̃ as a 65th head dimension, K' = [K | 1], Q' = [Q | -m̃],
// one extra MFMA per 32-key block: 3 % slower than the accumulator init; f32 v_add row sums: 4 %
// slower than the f16 tree — tools/kbench.py attn, RDMI_ATTN_F32SUM=1 selects the f32 sums.)

// MFMA/VALU overlap.  Per tile t a wave runs an MFMA block M(t) = {Oᵀ += Vᵀ·P(t-1)ᵀ; S'(t) =
// K(t)·Qᵀ − m̃} (32 MFMAs) and a VALU block S(t) = {softmax of S'(t) → P(t); DMA}, separated by
// barriers.  Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave is in its MFMA
// block while its partner is in its VALU block (guide §5.5 T16 / MI355X_MICROARCH "Two waves per
// SIMD").  With interval i between barriers, group g runs M(t) in interval 2t+g and S(t) in
// 2t+1+g; K(t) is read in M(t), V(t) in M(t+1), so slot t is busy until interval 2t+3.
// DMA(t) is issued in S(t-3) and each wave waits for it in S(t-2) (before the barrier that
// precedes M(t) in both groups); it overwrites tile t-5, whose last read (M(t-4), group 1) ended
// in interval 2t-7 < 2t-5.
constexpr int NSLOT = 5;

// Measured alternatives (tools/kbench.py, L0 shape, same process): issuing the DMA in the MFMA
// block instead of the softmax block −4 %; packed v_pk_add_f32 row sums −11 %; no priority flips
// (MFMA block pinned by sched_barrier) or a static s_setprio 1 for waves 4-7 instead: within ±2 %
// run-to-run (profiles/r01_attn_prio_ab.log); one row-sum partial per key block (4 independent
// add chains instead of one) −11 %.
// STAMP = 1 (diagnostic build only): per-wave cycle sums of the segments — 0 MFMA block, 1 its
// barrier, 2 softmax block, 3 DMA wait + barrier, 4 prologue, 5 epilogue — written to p.stamps.
template <bool F16SUM, int STAMP = 0>
__global__ __launch_bounds__(64 * NWV, 1) void attn_fwd_d64(AttnP p) {
  unsigned long long st_acc[6] = {}, st_prev = 0;
  auto seg = [&](int i) {
    if constexpr (STAMP) {
      const unsigned long long t = attn_stamp();
      st_acc[i] += t - st_prev;
      st_prev = t;
    }
  };
  if constexpr (STAMP) st_prev = attn_stamp();
  __shared__ __attribute__((aligned(16))) f16 lds[NSLOT * 2 * TILE];  // 160 KB: slot s = [K | V]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int grp = wid >> 2;
  const int hh = lane >> 5;  // lane half
  const int c = lane & 31;
  int qblk, head, b;
  rdmi::xcd_block3(qblk, head, b);
  const int qi = qblk * QB + wid * 32 + c;

  const f16* Q = p.q + (long)b * p.q_bs + head * 64;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.k + (long)b * p.k_bs + head * 64), (short)0, (int)(((long)(p.Sk - 1) * p.k_ld + 64) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.v + (long)b * p.v_bs + head * 64), (short)0, (int)(((long)(p.Sk - 1) * p.v_ld + 64) * 2), 0x00020000);

  // Q as the B operand of Sᵀ = K·Qᵀ: lane holds Q[qi][16ks + 8hh + 0..7] · scale·log2(e)
  // (the product Q·scale·log2 e is formed in f32 and rounded to f16 once)
  f16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    f16x8 z = {};
    const f16x8 qr = qi < p.Sq ? *(const f16x8*)(Q + (long)qi * p.q_ld + ks * 16 + hh * 8) : z;
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[ks][e] = (f16)((float)qr[e] * p.sl2);
  }
  // the 65th dimension: A = ones column (k index 0 of the lanes < 32), B = -m̃ (same slot)
  // -m̃ enters as the chain's initial accumulator (rows are lane-local in the swapped layout, so all
  // 16 accumulator entries of a lane carry its query's -m̃)
  f32x16 negm = {};

  // DMA lane geometry: 8 rows x 8 chunks per 1-KiB instruction; row = (i*NWV + wid)*8 + drow.
  // LDS images (bank-conflict-free for the fragment reads, checked with SQ_LDS_BANK_CONFLICT):
  //   K: phys chunk = logical ^ ((row >> 1) & 7)   (ds_read_b128 of 16 distinct rows / group)
  //   V: phys chunk = logical ^ (((row >> 1) & 1) << 2)   (tr reads of 4 rows x 64 B / half-wave)
  const int drow = lane >> 3;
  unsigned koff[DPW], voff[DPW];
#pragma unroll
  for (int i = 0; i < DPW; ++i) {
    const int row = (i * NWV + wid) * 8 + drow;
    const int kchunk = (lane & 7) ^ ((row >> 1) & 7);
    const int vchunk = (lane & 7) ^ (((row >> 1) & 1) << 2);
    koff[i] = (unsigned)(row * p.k_ld + kchunk * 8) * 2u;
    voff[i] = (unsigned)(row * p.v_ld + vchunk * 8) * 2u;
  }
  const unsigned kstep = (unsigned)(KB * p.k_ld * 2), vstep = (unsigned)(KB * p.v_ld * 2);
  const int wids = __builtin_amdgcn_readfirstlane(wid);  // provably uniform: the LDS-DMA destinations in SGPRs
  auto issue = [&](int kt) {
    const int slot = kt % NSLOT;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      f16* ks_ = lds + slot * 2 * TILE + (i * NWV + wids) * 8 * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)ks_, 16,
                                               koff[i] + (unsigned)kt * kstep, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(ks_ + TILE), 16,
                                               voff[i] + (unsigned)kt * vstep, 0, 0, 0);
    }
  };

  f32x16 o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float mt = 0.f, l = 0.f;  // m̃ (an f16 value, held in f32) and this lane's half of the row sum

  const int nt = (p.Sk + KB - 1) / KB;
  // tr-read lane geometry (16-lane groups)
  const int gi = lane >> 4, li = lane & 15;
  const int tr_key = 4 * (gi >> 1) + (li >> 2);
  const int tr_col = 16 * (gi & 1) + 4 * (li & 3);
  f16x8 pf[2 * NKB] = {};

  // Oᵀ += Vᵀ · Pᵀ for the tile in slot `slot` (KB/16 k-steps of 16 keys, 2 d-blocks of 32).
  // The transposed V reads are inline asm: with the ds_read_tr builtin hipcc assumes the read may
  // alias the in-flight LDS-DMA and drains vmcnt(0) before it, which serialises the K/V prefetch.
  // Reads run two k-steps ahead of the MFMAs, each consumer behind a counted lgkmcnt.
  auto pv = [&](int slot) {
    const unsigned vbase = (unsigned)(uintptr_t)LDS_PTR(f16, lds + slot * 2 * TILE + TILE);
    unsigned vaddr[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      // row = 16st + tr_key (+8): (row >> 1) & 1 == (tr_key >> 1) & 1 for both reads
      const int col = d * 32 + tr_col;
      const int pc = ((col >> 3) ^ (((tr_key >> 1) & 1) << 2)) << 3 | (col & 7);
      vaddr[d] = vbase + (unsigned)((tr_key * 64 + pc) * 2);
    }
    i16x4 vr[3][4];  // [stage][d*2 + lo/hi]
    auto rd = [&](int st, int buf) {
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vr[buf][2 * d]) : "v"(vaddr[d]), "i"(st * 16 * 64 * 2));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"
                     : "=v"(vr[buf][2 * d + 1]) : "v"(vaddr[d]), "i"((st * 16 + 8) * 64 * 2));
      }
    };
    rd(0, 0);
    rd(1, 1);
#pragma unroll
    for (int st = 0; st < 2 * NKB; ++st) {
      const int buf = st % 3;
      if (st + 1 < 2 * NKB)
        asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");  // stage st landed (st+1 in flight)
      else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // the destinations count as written here, not at the issuing asm (guide §5.7 item 1 form ii):
      // no compiler copy of them can be placed between the read and the wait
      asm volatile("" : "+v"(vr[buf][0]), "+v"(vr[buf][1]), "+v"(vr[buf][2]), "+v"(vr[buf][3]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const f16x8 vf = __builtin_bit_cast(
            f16x8, __builtin_shufflevector(vr[buf][2 * d], vr[buf][2 * d + 1], 0, 1, 2, 3, 4, 5, 6, 7));
        o[d] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[st], o[d], 0, 0, 0);
      }
      if (st + 2 < 2 * NKB) rd(st + 2, (st + 2) % 3);
    }
  };

  // Row sum of this lane's 64 probabilities as the MFMA will see them (the f16 P): a pairwise tree
  // of packed f16 adds (31 v_pk_add_f16 instead of 64 v_add_f32 on the softmax's VALU critical
  // path).  Partial sums stay ≤ the 2^15 rescale bound (an overflow to inf triggers the rescale).
  auto psum = [&]() -> float {
    f16x8 a0 = pf[0] + pf[1], a1 = pf[2] + pf[3], a2 = pf[4] + pf[5], a3 = pf[6] + pf[7];
    a0 += a1;
    a2 += a3;
    a0 += a2;
    f16x4 b = __builtin_shufflevector(a0, a0, 0, 1, 2, 3) + __builtin_shufflevector(a0, a0, 4, 5, 6, 7);
    f16x2 c2 = __builtin_shufflevector(b, b, 0, 1) + __builtin_shufflevector(b, b, 2, 3);
    return (float)c2[0] + (float)c2[1];
  };

  // prologue: DMA(0..2) issued ("S(-3..-1)"), DMA(0) and DMA(1) waited ("S(-2), S(-1)")
  issue(0);
  issue(1);
  issue(2);
  attn_wait_vmcnt<2 * DPW>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
  asm volatile("" ::: "memory");
  seg(4);

  for (int kt = 0; kt < nt; ++kt) {
    // ================= M(kt): PV of the previous tile, S' of this tile.  The s_setprio pair keeps
    // hipcc from moving the block's MFMAs across the barriers (guide §5.5 T5).
    __builtin_amdgcn_s_setprio(1);
    if (kt > 0) pv((kt - 1) % NSLOT);
    const f16* ks_ = lds + (kt % NSLOT) * 2 * TILE;
    f32x16 s[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      const int key = kb * 32 + c;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = 2 * ks + hh;
        f16x8 kf = *(const f16x8*)(ks_ + key * 64 + ((ch ^ ((key >> 1) & 7)) << 3));
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[ks], ks ? s[kb] : negm, 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    seg(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    seg(1);
    // ================= S(kt): softmax → P(kt); wait DMA(kt+2)
    if (p.sprio) __builtin_amdgcn_s_setprio(2);
    issue(kt + 3);  // past the end: zero rows into a drained slot
    // ---- mask (last tile only; lane owns query c, keys (r&3)+8(r>>2)+4hh of each block)
    const int kbase = kt * KB;
    if (kbase + KB > p.Sk) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kbase + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key >= p.Sk) s[kb][r] = -INFINITY;
        }
    }
    // ---- P = exp2(S'), row sum
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[kb][r]);  // v_exp_f32, no denorm fixup
        if (!F16SUM) rs += e;
        pf[kb * 2 + (r >> 3)][r & 7] = (f16)e;
      }
    if (F16SUM) rs = psum();
    // ---- (re)set m̃: always on the first tile, else only when P would leave the f16 range
    if (kt == 0 || __any(!(rs <= 32768.f))) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (kt != 0) mx = fmaxf(mx, 0.f);               // never lower m̃ (l >= 1 stays true)
      const float mnew = (float)(f16)(mt + mx);       // next m̃, an f16 value
      const float delta = mnew - mt;                  // exact: both are f16 values
      const float alpha = __builtin_amdgcn_exp2f(-delta);
      l *= alpha;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      mt = mnew;
#pragma unroll
      for (int r = 0; r < 16; ++r) negm[r] = -mnew;
      rs = 0.f;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[kb][r] - delta);
          if (!F16SUM) rs += e;
          pf[kb * 2 + (r >> 3)][r & 7] = (f16)e;
        }
      if (F16SUM) rs = psum();
    }
    l += rs;
    if (p.sprio) __builtin_amdgcn_s_setprio(0);
    seg(2);
    attn_wait_vmcnt<2 * DPW>();  // DMA(kt+2) landed (DMA(kt+3) in flight)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    seg(3);
  }
  // ================= M(nt): PV of the last tile
  pv((nt - 1) % NSLOT);
  if (grp == 0) __builtin_amdgcn_s_barrier();  // match group 1's extra barrier
  attn_wait_vmcnt<0>();  // drain trailing zero-row DMAs before the workgroup retires
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = 1.f / lt;
  if (qi < p.Sq) {
    f16* O = p.o + (long)b * p.o_bs + (long)qi * p.o_ld + head * 64;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (f16)(o[d][4 * g + e] * inv);
        *(f16x4*)(O + d * 32 + 8 * g + 4 * hh) = w;
      }
  }
  if constexpr (STAMP) {
    seg(5);
    if (lane == 0) {
      unsigned long long* o = p.stamps + ((((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * NWV + wid) * 6;
      for (int i = 0; i < 6; ++i) o[i] = st_acc[i];
    }
  }
}

// attn_fwd_d64_pipe: the same arithmetic as attn_fwd_d64, restructured for ONE wave per SIMD.
//
// Why (tools/attn_stamp.hip, profiles/r03h_attn_stamp.log): in attn_fwd_d64 the two waves of a SIMD
// alternate an MFMA block (32 MFMAs = 1 024 matrix cycles) with a softmax block, and both blocks
// measure ≈1 500 cycles per 128-key tile: the SIMD's one vector-issue port serves the softmax wave's
// ≈850 issue cycles of exp / cvt / add AND the MFMA wave's issue holds (8 of every 32 cycles), so
// the matrix pipe idles ≈35 % of the time.  Here each wave owns its SIMD and interleaves its own
// softmax with its own MFMAs (software pipeline; guide §5.5 T15, Appendix B 'Fused attention
// prefill', 4-wave structure).  A wave holds 64 queries as two 32-query blocks q0, q1 that share
// every K and V fragment; per 32-key sub-tile u the MFMA stream is
//     PV_q0(u) | QK_q0(u+1) | PV_q1(u) | QK_q1(u+1)        (4 MFMAs each)
// and the softmax of S_q1(u) runs beside the first two segments, that of S_q0(u+1) beside the last
// two, each followed by its block's m̃ / rescale decision — so every 32-cycle MFMA gap carries ≈4
// vector instructions (2 exponentials), and only one 16-register S per block is live.  A workgroup
// = 4 waves = 256 queries; K/V in 64-key tiles by LDS-DMA into a 4-slot ring, one barrier per tile.
// Same exponent / rounding order per query as attn_fwd_d64; the packed-f16 row sum is taken per 32
// keys instead of per 64 (results equal to f16 rounding of P sums).
namespace pp {
constexpr int NW = 4;              // waves per workgroup (one per SIMD)
constexpr int QB = 64 * NW;        // queries per workgroup (64 per wave)
constexpr int TK = 64;             // keys per K/V tile (DMA and barrier granule): 2 sub-tiles of 32
constexpr int NSL = 4;             // tile slots in the LDS ring
constexpr int TH = TK * 64;        // halves per K (or V) tile (8 KiB)
constexpr int DPW = TK / 8 / NW;   // 8-row DMA pieces per wave per tile per tensor (2)
}  // namespace pp

// NEGM (the dispatched form, round 5): −m̃ enters each QKᵀ chain as its initial accumulator, as in
// attn_fwd_d64, instead of a fifth k-step (kone × qm below): 16 of 18 MFMAs per sub-tile → 16 of 16,
// bitwise the same results, 3 % faster at L0 / L1 (profiles/r05zp_pipe_kb.log; 5 registers spill at two
// workgroups per CU, and one workgroup per CU is 25 % slower).
template <int STAMP = 0, bool NEGM = false>
__global__ __launch_bounds__(64 * pp::NW, 2) void attn_fwd_d64_pipe(AttnP p) {
  constexpr int NW = pp::NW, QB = pp::QB, TK = pp::TK, NSL = pp::NSL, TH = pp::TH, DPW = pp::DPW;
  __shared__ __attribute__((aligned(16))) f16 lds[NSL * 2 * TH];  // 64 KiB: slot s = [K | V]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int hh = lane >> 5;
  const int c = lane & 31;
  int qblk, head, b;
  rdmi::xcd_block3(qblk, head, b);
  const int q0 = qblk * QB + wid * 64;  // query block qb of this wave: q0 + 32 qb + c

  const f16* Q = p.q + (long)b * p.q_bs + head * 64;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.k + (long)b * p.k_bs + head * 64), (short)0, (int)(((long)(p.Sk - 1) * p.k_ld + 64) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.v + (long)b * p.v_bs + head * 64), (short)0, (int)(((long)(p.Sk - 1) * p.v_ld + 64) * 2), 0x00020000);

  // Q·scale·log2(e) as the B operand of Sᵀ = K·Qᵀ (rounded to f16 once), per query block
  f16x8 qf[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qi = q0 + 32 * qb + c;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f16x8 z = {};
      const f16x8 qr = qi < p.Sq ? *(const f16x8*)(Q + (long)qi * p.q_ld + ks * 16 + hh * 8) : z;
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[qb][ks][e] = (f16)((float)qr[e] * p.sl2);
    }
  }

  // DMA lane geometry (as attn_fwd_d64): row = (i·NW + wid)·8 + drow of the 64-key tile
  const int drow = lane >> 3;
  unsigned koff[DPW], voff[DPW];
#pragma unroll
  for (int i = 0; i < DPW; ++i) {
    const int row = (i * NW + wid) * 8 + drow;
    const int kchunk = (lane & 7) ^ ((row >> 1) & 7);
    const int vchunk = (lane & 7) ^ (((row >> 1) & 1) << 2);
    koff[i] = (unsigned)(row * p.k_ld + kchunk * 8) * 2u;
    voff[i] = (unsigned)(row * p.v_ld + vchunk * 8) * 2u;
  }
  const unsigned kstep = (unsigned)(TK * p.k_ld * 2), vstep = (unsigned)(TK * p.v_ld * 2);
  auto issue = [&](int kt) __attribute__((always_inline)) {  // past the end: zero rows (descriptor range)
    const int slot = kt % NSL;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      f16* ks_ = lds + slot * 2 * TH + (i * NW + wid) * 8 * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)ks_, 16,
                                               koff[i] + (unsigned)kt * kstep, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(ks_ + TH), 16,
                                               voff[i] + (unsigned)kt * vstep, 0, 0, 0);
    }
  };

  // fragment addresses (bytes): K row c of a 32-key sub-tile, chunk 2ks + hh swizzled by
  // (row >> 1) & 7 = (c >> 1) & 7 (sub-tile row offsets are multiples of 16); Vᵀ by transposed
  // reads of rows 16st + tr_key (+8), chunk swizzle (tr_key >> 1) & 1 — immediates per sub-tile
  const unsigned lbase = (unsigned)(uintptr_t)LDS_PTR(f16, lds);
  unsigned kaddr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) kaddr[ks] = (unsigned)((c * 64 + (((2 * ks + hh) ^ ((c >> 1) & 7)) << 3)) * 2);
  const int gi = lane >> 4, li = lane & 15;
  const int tr_key = 4 * (gi >> 1) + (li >> 2);
  const int tr_col = 16 * (gi & 1) + 4 * (li & 3);
  unsigned vaddr[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const int col = d * 32 + tr_col;
    const int pc = ((col >> 3) ^ (((tr_key >> 1) & 1) << 2)) << 3 | (col & 7);
    vaddr[d] = (unsigned)((TH + tr_key * 64 + pc) * 2);
  }
  auto sub_base = [&](int u) __attribute__((always_inline)) {
    return lbase + (unsigned)(((u >> 1) % NSL) * 2 * TH * 2 + (u & 1) * 32 * 64 * 2);
  };

  const int nt = (p.Sk + TK - 1) / TK;
  const int nsub = (p.Sk + 31) / 32;  // sub-tiles holding keys

  f32x16 o[2][2];  // [qb][d-block]: Oᵀ accumulators
  // −m̃ enters the QKᵀ chain as a fifth k-step K' = [1 0 …], Q' = [−m̃ 0 …] (m̃ is an f16 value, so the
  // product is exact), issued FIRST on a zero accumulator: the chain then starts from exactly −m̃ in
  // every entry, as attn_fwd_d64's initial accumulator does, without 16 live registers per block
  // (and without the copies of them into each chain's accumulator)
  f16x8 kone = {}, qm[2] = {};
  if (hh == 0) kone[0] = (f16)1.0f;
  f32x16 nm[2] = {};  // NEGM: −m̃ as the chain's initial accumulator (16 registers per block, no fifth MFMA)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[qb][d][r] = 0.f;
  }
  float mt[2] = {0.f, 0.f}, l[2] = {0.f, 0.f};
  f16x8 kf[4];         // K fragments of the next sub-tile (shared by both blocks)
  i16x4 vr[2][2][2];   // Vᵀ fragments of the current sub-tile [st][d][lo/hi] (shared by both blocks)
  f32x16 s[2];         // S' of each block's current sub-tile
  f16x8 pf[2][2];      // P of each block's current sub-tile [qb][16-key step]
  float e[16];         // exponentials of the block being normalised

  // Vᵀ reads as asm (hipcc drains the in-flight LDS-DMA, vmcnt(0), in front of a ds_read_tr builtin),
  // counted by hand; K reads as plain loads, whose lgkmcnt hipcc places before each consumer (its
  // counts ignore the asm reads issued before them, so they over-wait, never under-wait).  The V
  // reads carry a "memory" clobber so the K loads stay behind them: lgkmcnt(4) then means "V landed".
  auto kread = [&](int u) __attribute__((always_inline)) {
    const f16* kb = lds + ((u >> 1) % NSL) * 2 * TH + (u & 1) * 32 * 64;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[ks] = *(const f16x8*)(kb + kaddr[ks] / 2);
  };
  auto vread = [&](int u) __attribute__((always_inline)) {
    const unsigned vb = sub_base(u);
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"
                     : "=v"(vr[st][d][0]) : "v"(vb + vaddr[d]), "i"(st * 16 * 64 * 2) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"
                     : "=v"(vr[st][d][1]) : "v"(vb + vaddr[d]), "i"((st * 16 + 8) * 64 * 2) : "memory");
      }
  };
  // the destinations count as written at the wait (guide §5.7 item 1 form ii)
  auto vwait = [&](bool k_behind) __attribute__((always_inline)) {
    if (k_behind)
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1]), "+v"(vr[1][0][0]),
                 "+v"(vr[1][0][1]), "+v"(vr[1][1][0]), "+v"(vr[1][1][1]));
  };
  // S'_qb = K·Qᵀ − m̃ (five chained MFMAs, the −m̃ step first)
  auto qk = [&](int qb) __attribute__((always_inline)) {
    if constexpr (NEGM) {
      s[qb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[0], qf[qb][0], nm[qb], 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < 4; ++ks) s[qb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[ks], qf[qb][ks], s[qb], 0, 0, 0);
    } else {
      const f32x16 zero = {};
      s[qb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kone, qm[qb], zero, 0, 0, 0);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s[qb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[ks], qf[qb][ks], s[qb], 0, 0, 0);
    }
  };
  // Oᵀ_qb += Vᵀ·P_qbᵀ (two 16-key steps × two 32-row d-blocks)
  auto pv = [&](int qb) __attribute__((always_inline)) {
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const f16x8 vf =
            __builtin_bit_cast(f16x8, __builtin_shufflevector(vr[st][d][0], vr[st][d][1], 0, 1, 2, 3, 4, 5, 6, 7));
        o[qb][d] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[qb][st], o[qb][d], 0, 0, 0);
      }
  };
  // keys past Sk masked (guarded form: the sub-tile straddling the end)
  auto mask = [&](int qb, int u, bool guarded) __attribute__((always_inline)) {
    if (guarded && 32 * u + 32 > p.Sk) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (32 * u + (r & 3) + 8 * (r >> 2) + 4 * hh >= p.Sk) s[qb][r] = -INFINITY;
    }
  };
  auto exps = [&](int qb, int lo, int hi) __attribute__((always_inline)) {
#pragma unroll
    for (int r = lo; r < hi; ++r) e[r] = __builtin_amdgcn_exp2f(s[qb][r]);  // v_exp_f32, no denorm fixup
  };
  // f16 P (the PV B operand) and its packed-f16 row sum over this lane's 16 keys
  auto pack_sum = [&](int qb) __attribute__((always_inline)) -> float {
#pragma unroll
    for (int r = 0; r < 16; ++r) pf[qb][r >> 3][r & 7] = (f16)e[r];
    const f16x8 a = pf[qb][0] + pf[qb][1];
    const f16x4 b4 = __builtin_shufflevector(a, a, 0, 1, 2, 3) + __builtin_shufflevector(a, a, 4, 5, 6, 7);
    const f16x2 c2 = __builtin_shufflevector(b4, b4, 0, 1) + __builtin_shufflevector(b4, b4, 2, 3);
    return (float)c2[0] + (float)c2[1];
  };
  // block qb's m̃: set on the first sub-tile, re-set (O_qb, l_qb rescaled, P recomputed) when its P
  // would leave the f16 range.  O_qb holds PV of sub-tiles < u only; QK_qb(u+1) is issued after.
  auto decide = [&](int qb, float rs, bool first) __attribute__((always_inline)) {
    if (__builtin_expect(first || __any(!(rs <= 32768.f)), 0)) {
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[qb][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (!first) mx = fmaxf(mx, 0.f);            // never lower m̃ (l >= 1 stays true)
      const float mnew = (float)(f16)(mt[qb] + mx);  // next m̃, an f16 value
      const float delta = mnew - mt[qb];            // exact: both are f16 values
      const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-delta);
      l[qb] *= alpha;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[qb][d][r] *= alpha;
      mt[qb] = mnew;
      if constexpr (NEGM) {
#pragma unroll
        for (int r = 0; r < 16; ++r) nm[qb][r] = -mnew;
      } else if (hh == 0) {
        qm[qb][0] = (f16)(-mnew);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) s[qb][r] -= delta;
      exps(qb, 0, 16);
      rs = pack_sum(qb);
    }
    l[qb] += rs;
  };

  // prologue: DMA(0..2); tiles 0 and 1 landed; S'_q0(0), S'_q1(0); softmax + m̃ of block 0
  issue(0);
  issue(1);
  issue(2);
  attn_wait_vmcnt<2 * DPW>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  kread(0);
  qk(0);
  qk(1);
  mask(0, 0, true);
  exps(0, 0, 16);
  decide(0, pack_sum(0), true);

  // period u, two halves, each one basic block in the steady state:
  //   A: [V(u), K(u+1) reads; 8 exps of S'_q1(u)] | PV_q0(u), QK_q0(u+1) ∥ the rest of softmax_q1(u)
  //   decide q1
  //   B: PV_q1(u), QK_q1(u+1) ∥ softmax_q0(u+1)
  //   decide q0
  // Tile barrier at the head of odd periods, before K of sub-tile u+1 (tile kt+1) is read: tile kt+1
  // landed for every wave, and the slot of tile kt-1 (read for the last time in period u-2) free for
  // DMA(kt+3).  Issue order inside each half pinned by sched_group_barrier (MFMA 0x8, VALU 0x2).
  auto period = [&](int u, auto guarded, auto parity) __attribute__((always_inline)) {
    constexpr bool G = decltype(guarded)::value;
    constexpr int PAR = decltype(parity)::value;  // 0 / 1: u's parity known; 2: read from u
    const bool nx = !G || u + 1 < nsub;
    if (PAR == 1 || (PAR == 2 && (u & 1))) {
      attn_wait_vmcnt<2 * DPW>();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue((u >> 1) + 3);
    }
    vread(u);
    if (nx) kread(u + 1);
    mask(1, u, G);
    exps(1, 0, 8);
    __builtin_amdgcn_sched_barrier(0);
    vwait(nx);
    pv(0);
    exps(1, 8, 16);
    if (nx) qk(0);
    const float rs1 = pack_sum(1);
    if constexpr (!G) {
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      }
    }
    decide(1, rs1, G && u == 0);
    pv(1);
    if (nx) {
      qk(1);
      mask(0, u + 1, G);
      exps(0, 0, 16);
      const float rs0 = pack_sum(0);
      if constexpr (!G) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#pragma unroll
        for (int i = 0; i < 7; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      }
      decide(0, rs0, false);
    }
  };
  // steady state while sub-tile u+1 is whole; the guarded form for the first two and the last sub-tiles
  const int nst = p.Sk / 32 - 1;
  int u = 0;
  for (; u < 2 && u < nsub; ++u) period(u, std::true_type{}, std::integral_constant<int, 2>{});  // first of q1
  for (; u + 1 < nst; u += 2) {
    period(u, std::false_type{}, std::integral_constant<int, 0>{});
    period(u + 1, std::false_type{}, std::integral_constant<int, 1>{});
  }
  for (; u < nsub; ++u) period(u, std::true_type{}, std::integral_constant<int, 2>{});
  attn_wait_vmcnt<0>();  // drain trailing zero-row DMAs before the workgroup retires
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qi = q0 + 32 * qb + c;
    const float lt = l[qb] + __shfl_xor(l[qb], 32, 64);
    const float inv = 1.f / lt;
    if (qi < p.Sq) {
      f16* O = p.o + (long)b * p.o_bs + (long)qi * p.o_ld + head * 64;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f16x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = (f16)(o[qb][d][4 * g + e] * inv);
          *(f16x4*)(O + d * 32 + 8 * g + 4 * hh) = w;
        }
    }
  }
}

// one thread per (token, head); D == 64, L ≤ 16
template <typename T>
__global__ __launch_bounds__(256) void attn_smallkv(const T* __restrict__ q, const T* __restrict__ k,
                                                    const T* __restrict__ v, T* __restrict__ o, int H, int Sq,
                                                    int L, long q_ld, long o_ld, long q_bs, long o_bs, long kv_bs,
                                                    float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* kl = (T*)smem;              // [L][H*64]
  T* vl = kl + L * H * 64;
  const int b = blockIdx.y;
  const int HD = H * 64;
  for (int i = threadIdx.x; i < L * HD * (int)sizeof(T) / 16; i += blockDim.x) {
    ((f32x4*)kl)[i] = ((const f32x4*)(k + (long)b * kv_bs))[i];
    ((f32x4*)vl)[i] = ((const f32x4*)(v + (long)b * kv_bs))[i];
  }
  __syncthreads();
  long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)Sq * H) return;
  int tok = (int)(idx / H), h = (int)(idx % H);
  const T* qr = q + (long)b * q_bs + (long)tok * q_ld + h * 64;
  float qv[64];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float t[8];
    ld8(qr + 8 * i, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[8 * i + e] = t[e];
  }
  float sc[16];
  float mx = -INFINITY;
  for (int j = 0; j < L; ++j) {
    const T* kr = kl + j * HD + h * 64;
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) a += qv[d] * (float)kr[d];
    sc[j] = a * scale;
    mx = fmaxf(mx, sc[j]);
  }
  float den = 0.f;
  for (int j = 0; j < L; ++j) {
    sc[j] = sizeof(T) == 2 ? __expf(sc[j] - mx) : expf(sc[j] - mx);
    den += sc[j];
  }
  float inv = 1.f / den;
  float acc[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) acc[d] = 0.f;
  for (int j = 0; j < L; ++j) {
    const T* vr = vl + j * HD + h * 64;
    float w = sc[j] * inv;
#pragma unroll
    for (int d = 0; d < 64; ++d) acc[d] += w * (float)vr[d];
  }
  T* orow = o + (long)b * o_bs + (long)tok * o_ld + h * 64;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = acc[8 * i + e];
    st8(orow + 8 * i, t);
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void softmax_rows_k(const float* __restrict__ s, TO* __restrict__ pout, long cols,
                                                      long p_ld, float scale) {
  const long row = blockIdx.x;
  const float* sr = s + row * cols;
  __shared__ float red[4];
  float mx = -INFINITY;
  for (long c = threadIdx.x; c < cols; c += 256) mx = fmaxf(mx, sr[c]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (long c = threadIdx.x; c < cols; c += 256)
    sum += sizeof(TO) == 2 ? __expf((sr[c] - mx) * scale) : expf((sr[c] - mx) * scale);
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  sum = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / sum;
  TO* pr = pout + row * p_ld;
  for (long c = threadIdx.x; c < cols; c += 256)
    pr[c] = (TO)((sizeof(TO) == 2 ? __expf((sr[c] - mx) * scale) : expf((sr[c] - mx) * scale)) * inv);
  for (long c = cols + threadIdx.x; c < p_ld; c += 256) pr[c] = (TO)0.f;  // K padding of the PV GEMM
}

// Single-pass row softmax: the row (≤ 1024·NV floats) is read once into registers as float4s,
// max and sum are block reductions, and the probabilities are written from registers — one HBM
// read of the f32 scores instead of three (the scores of a 96² VAE attention are 36 KiB rows
// that the L2 does not hold across three passes with every CU streaming).
template <int NV>
__global__ __launch_bounds__(256) void softmax_rows_reg_k(const float* __restrict__ s, f16* __restrict__ pout, long cols,
                                                          long p_ld, float scale) {
  const long row = blockIdx.x;
  const f32x4* sr = (const f32x4*)(s + row * cols);
  const int nv = (int)(cols >> 2);
  __shared__ float red[4];
  f32x4 v[NV];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + 256 * i;
    v[i] = c < nv ? sr[c] : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    mx = fmaxf(mx, fmaxf(fmaxf(v[i][0], v[i][1]), fmaxf(v[i][2], v[i][3])));
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[i][e] = __expf((v[i][e] - mx) * scale);
      sum += v[i][e];
    }
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  sum = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / sum;
  f16* pr = pout + row * p_ld;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + 256 * i;
    if (c < nv) {
      f16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (f16)(v[i][e] * inv);
      *(f16x4*)(pr + 4 * c) = o;
    }
  }
  for (long c = cols + threadIdx.x; c < p_ld; c += 256) pr[c] = (f16)0.f;  // K padding of the PV GEMM
}

// attn2 block against a TWO-token context (the empty-text embedding BOS+EOS), collapsed by exact
// algebra (attention_processor.py:2172-2276 with Sk = 2; attention.py:480-492 norm2 + residual):
// softmax over two keys is σ(s1 − s0), so per head h
//   o_h = V0_h + σ(n2·w_h) (V1_h − V0_h),  w_h = scale · Wq_hᵀ (K1_h − K0_h)
// and after to_out: out = t + c + Σ_h σ(n2·w_h) u_h,  u_h = Wo_h (V1_h − V0_h),  c = Wo V0 + bo,
// with n2 = LayerNorm(t) (norm2, rounded to f16 as the unfused LN output).  One wave per token
// row: LN moments (same order as layernorm_k), H dot products against w (LDS), the sigmoid
// weights, the output row — one read and one write of the row instead of LN + q GEMM + attention
// + out GEMM (five row passes).  w, u, c are folded once per context (unet.Transformer).
// HC > 0: H = HC at compile time — the H head dot products are formed first and their wave sums
// run level by level together (H independent reduction chains in flight instead of H serial ones), then
// the sigmoids and the output accumulation in head order: the same operations on every value as the
// HC = 0 loop, bitwise its output.  With the reductions below, 25-snippet L0 / L1 launches 476–497 →
// 431 µs / 414 → 315 µs (profiles/r04ak_pair_dpp_ab.log); L0 stays vector-issue-bound (40 of 64 lanes
// hold columns at C = 320).
// wave_sum's xor butterfly (32, 16, 8, 4, 2, 1: the same pairs, the same operand per add, so the
// same bits) without the LDS crossbar: xor 32 / 16 as v_permlane32_swap / v_permlane16_swap of the
// value with a copy of itself (the two results sum to v_i + v_partner in every lane), xor 8 as DPP
// row_ror:8, xor 4 as row_ror:4 or row_ror:12 by lane bit 2 (b2 = (lane >> 2) & 1), xor 2 / 1 as
// quad_perm — no ds_bpermute and no lgkmcnt wait in the chain (bitwise: tests/test_kernels_gpu.py
// test_cross_attn_pair against the per-head shuffle loop).  The swaps are inline asm: hipcc folded the
// builtins' swap of a value with itself into an identity (r0 + r1 = 2v); the s_nops cover the
// VALU-write → permlane-read and permlane-write → VALU-read hazards.
template <bool X32>
__device__ __forceinline__ float swap_sum(float v) {
  float a = v, b = v;
  if constexpr (X32)
    asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  else
    asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  return a + b;
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int HC>
__device__ __forceinline__ void wave_sum_n(float (&d)[HC], bool b2) {
#pragma unroll
  for (int h = 0; h < HC; ++h) d[h] = swap_sum<true>(d[h]);
#pragma unroll
  for (int h = 0; h < HC; ++h) d[h] = swap_sum<false>(d[h]);
#pragma unroll
  for (int h = 0; h < HC; ++h) d[h] = d[h] + dppf<0x128>(d[h]);
#pragma unroll
  for (int h = 0; h < HC; ++h) {
    const float p4 = dppf<0x124>(d[h]), p12 = dppf<0x12C>(d[h]);  // both read by every lane, then a select
    d[h] = d[h] + (b2 ? p4 : p12);
  }
#pragma unroll
  for (int h = 0; h < HC; ++h) d[h] = d[h] + dppf<0x4E>(d[h]);
#pragma unroll
  for (int h = 0; h < HC; ++h) d[h] = d[h] + dppf<0xB1>(d[h]);
}

template <int NV, int HC = 0>  // f16x8 vectors per lane: C ≤ 512·NV
__global__ __launch_bounds__(256) void attn2_pair_k(const f16* __restrict__ x, f16* __restrict__ y, long M, int C,
                                                    int H, const float* __restrict__ g, const float* __restrict__ b,
                                                    float eps, const float* __restrict__ wd,
                                                    const float* __restrict__ u, const float* __restrict__ c0) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // w [H][C] | u [H][C]
  for (int i = threadIdx.x; i < H * C / 4; i += 256) {
    ((f32x4*)sm)[i] = ((const f32x4*)wd)[i];
    ((f32x4*)sm)[H * C / 4 + i] = ((const f32x4*)u)[i];
  }
  __syncthreads();
  const float* ws = sm;
  const float* us = sm + H * C;
  const int lane = threadIdx.x & 63;
  const bool b2 = (lane >> 2) & 1;
  const int CV = C >> 3;
  // this lane's columns are fixed: LN affine and the constant row c stay in registers
  float gr[NV][8], br[NV][8], cr[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int cv = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int cc = cv < CV ? cv * 8 + e : 0;
      gr[i][e] = g[cc];
      br[i][e] = b[cc];
      cr[i][e] = c0[cc];
    }
  }
  const long stride = gridDim.x * 4L;
  long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  f16x8 vn[NV];  // next row, loaded one row ahead
  auto load = [&](long r) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int cv = lane + 64 * i;
      if (r < M && cv < CV) vn[i] = *(const f16x8*)(x + r * C + cv * 8);
    }
  };
  load(row);
  for (; row < M; row += stride) {
    f16x8 v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = vn[i];
    load(row + stride);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (lane + 64 * i < CV)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)v[i][e];
    float sr[1] = {s};
    if constexpr (HC > 0) wave_sum_n<1>(sr, b2); else sr[0] = wave_sum(s);
    const float mean = sr[0] / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (lane + 64 * i < CV)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = (float)v[i][e] - mean;
          q += d * d;
        }
    float qr[1] = {q};
    if constexpr (HC > 0) wave_sum_n<1>(qr, b2); else qr[0] = wave_sum(q);
    const float rstd = rsqrtf(qr[0] / C + eps);
    float n[NV][8], o[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        n[i][e] = lane + 64 * i < CV ? (float)(f16)(((float)v[i][e] - mean) * rstd * gr[i][e] + br[i][e]) : 0.f;
        o[i][e] = 0.f;
      }
    if constexpr (HC > 0) {
      float d[HC];
#pragma unroll
      for (int h = 0; h < HC; ++h) {
        d[h] = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int cv = lane + 64 * i;
          if (cv < CV) {
            const f32x4 w0 = *(const f32x4*)(ws + h * C + cv * 8), w1 = *(const f32x4*)(ws + h * C + cv * 8 + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) d[h] = fmaf(n[i][e], w0[e], fmaf(n[i][4 + e], w1[e], d[h]));
          }
        }
      }
      wave_sum_n<HC>(d, b2);
#pragma unroll
      for (int h = 0; h < HC; ++h) {
        const float ph = 1.0f / (1.0f + __expf(-d[h]));
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int cv = lane + 64 * i;
          if (cv < CV) {
            const f32x4 u0 = *(const f32x4*)(us + h * C + cv * 8), u1 = *(const f32x4*)(us + h * C + cv * 8 + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              o[i][e] = fmaf(ph, u0[e], o[i][e]);
              o[i][4 + e] = fmaf(ph, u1[e], o[i][4 + e]);
            }
          }
        }
      }
    }
    for (int h = 0; h < (HC > 0 ? 0 : H); ++h) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int cv = lane + 64 * i;
        if (cv < CV) {
          const f32x4 w0 = *(const f32x4*)(ws + h * C + cv * 8), w1 = *(const f32x4*)(ws + h * C + cv * 8 + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) d = fmaf(n[i][e], w0[e], fmaf(n[i][4 + e], w1[e], d));
        }
      }
      d = wave_sum(d);
      const float ph = 1.0f / (1.0f + __expf(-d));
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int cv = lane + 64 * i;
        if (cv < CV) {
          const f32x4 u0 = *(const f32x4*)(us + h * C + cv * 8), u1 = *(const f32x4*)(us + h * C + cv * 8 + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[i][e] = fmaf(ph, u0[e], o[i][e]);
            o[i][4 + e] = fmaf(ph, u1[e], o[i][4 + e]);
          }
        }
      }
    }
    f16* yr = y + row * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int cv = lane + 64 * i;
      if (cv < CV) {
        f16x8 r;
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = (f16)((float)v[i][e] + (cr[i][e] + o[i][e]));
        *(f16x8*)(yr + cv * 8) = r;
      }
    }
  }
}

}  // namespace

extern "C" int rdmi_attention_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                                  int D, long q_ld, long k_ld, long v_ld, long o_ld, long q_bs, long k_bs, long v_bs,
                                  long o_bs, float scale, int dtype, void* stream) {
  RDMI_REQUIRE(q && k && v && o, RDMI_E_ARG, "attention_fwd: null pointer");
  RDMI_REQUIRE(D == 64, RDMI_E_UNSUPPORTED, "attention_fwd: head_dim %d unsupported (64 only)", D);
  RDMI_REQUIRE(B > 0 && H > 0 && Sq > 0 && Sk > 0, RDMI_E_ARG, "attention_fwd: bad sizes");
  if (dtype == RDMI_F32 || dtype == RDMI_F32_X3 || dtype == RDMI_F32_X6)
    return rdmi::attention_fwd_f32(q, k, v, o, B, H, Sq, Sk, q_ld, k_ld, v_ld, o_ld, q_bs, k_bs, v_bs, o_bs, scale,
                                   dtype == RDMI_F32_X3 ? 2 : dtype == RDMI_F32_X6 ? 3 : 1, stream);
  RDMI_REQUIRE(q_ld % 8 == 0 && k_ld % 8 == 0 && v_ld % 8 == 0 && o_ld % 4 == 0 && (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v) & 15) == 0,
               RDMI_E_ALIGN, "attention_fwd: strides/pointers must be 16-byte aligned");
  AttnP p{(const f16*)q, (const f16*)k, (const f16*)v, (f16*)o, H, Sq, Sk, q_ld, k_ld, v_ld, o_ld, q_bs, k_bs, v_bs, o_bs,
          scale * 1.4426950408889634f, nullptr};
  const char* sp = getenv("RDMI_ATTN_SPRIO");  // read per launch (A/B)
  p.sprio = sp && sp[0] == '1';
  dim3 g(rdmi::div_up(Sq, QB), H, B);
  static const bool f32sum = [] { const char* e = getenv("RDMI_ATTN_F32SUM"); return e && e[0] == '1'; }();
  const char* pe = getenv("RDMI_ATTN_PIPE");  // read per launch (A/B): 1 = the one-wave-per-SIMD pipeline
  if (pe && pe[0] == '1' && !f32sum) {
    hipLaunchKernelGGL((attn_fwd_d64_pipe<0, true>), dim3(rdmi::div_up(Sq, pp::QB), H, B), dim3(64 * pp::NW), 0,
                       (hipStream_t)stream, p);
    return rdmi::check_launch("attention_fwd");
  }
  if (!f32sum)
    hipLaunchKernelGGL(attn_fwd_d64<true>, g, dim3(64 * NWV), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(attn_fwd_d64<false>, g, dim3(64 * NWV), 0, (hipStream_t)stream, p);
  return rdmi::check_launch("attention_fwd");
}

extern "C" int rdmi_attention_smallkv(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int L,
                                      int D, long q_ld, long o_ld, long q_bs, long o_bs, long kv_bs, float scale,
                                      int dtype, void* stream) {
  RDMI_REQUIRE(q && k && v && o, RDMI_E_ARG, "attention_smallkv: null pointer");
  RDMI_REQUIRE(D == 64 && L >= 1 && L <= 16, RDMI_E_UNSUPPORTED, "attention_smallkv: D=%d L=%d unsupported", D, L);
  const size_t esz = dtype == RDMI_F32 ? 4 : 2;
  size_t lds = (size_t)2 * L * H * 64 * esz;
  RDMI_REQUIRE(lds <= 64 * 1024, RDMI_E_UNSUPPORTED, "attention_smallkv: K/V too large for LDS");
  dim3 g(rdmi::div_up((long)Sq * H, 256), B);
  if (dtype == RDMI_F32)
    hipLaunchKernelGGL(attn_smallkv<float>, g, dim3(256), lds, (hipStream_t)stream, (const float*)q, (const float*)k,
                       (const float*)v, (float*)o, H, Sq, L, q_ld, o_ld, q_bs, o_bs, kv_bs, scale);
  else
    hipLaunchKernelGGL(attn_smallkv<f16>, g, dim3(256), lds, (hipStream_t)stream, (const f16*)q, (const f16*)k,
                       (const f16*)v, (f16*)o, H, Sq, L, q_ld, o_ld, q_bs, o_bs, kv_bs, scale);
  return rdmi::check_launch("attention_smallkv");
}

extern "C" int rdmi_softmax_rows(const float* s, void* p, long rows, long cols, long p_ld, float scale, int p_dtype,
                                 void* stream) {
  RDMI_REQUIRE(s && p && rows > 0 && cols > 0 && p_ld >= cols, RDMI_E_ARG, "softmax_rows: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (p_dtype == RDMI_F32) {
    hipLaunchKernelGGL(softmax_rows_k<float>, dim3((unsigned)rows), dim3(256), 0, st, s, (float*)p, cols, p_ld, scale);
    return rdmi::check_launch("softmax_rows");
  }
  const bool vec = cols % 4 == 0 && p_ld % 4 == 0 && ((uintptr_t)s & 15) == 0 && ((uintptr_t)p & 7) == 0;
  const long nv = (cols / 4 + 255) / 256;  // float4s per thread
  if (vec && nv <= 4)
    hipLaunchKernelGGL(softmax_rows_reg_k<4>, dim3((unsigned)rows), dim3(256), 0, st, s, (f16*)p, cols, p_ld, scale);
  else if (vec && nv <= 16)
    hipLaunchKernelGGL(softmax_rows_reg_k<16>, dim3((unsigned)rows), dim3(256), 0, st, s, (f16*)p, cols, p_ld, scale);
  else
    hipLaunchKernelGGL(softmax_rows_k<f16>, dim3((unsigned)rows), dim3(256), 0, st, s, (f16*)p, cols, p_ld, scale);
  return rdmi::check_launch("softmax_rows");
}

extern "C" int rdmi_cross_attn_pair(const void* x, void* y, long M, int C, int H, const float* ln_gamma,
                                    const float* ln_beta, float eps, const float* w, const float* u, const float* c,
                                    void* stream) {
  RDMI_REQUIRE(x && y && ln_gamma && ln_beta && w && u && c && M > 0 && H > 0, RDMI_E_ARG, "cross_attn_pair: bad args");
  RDMI_REQUIRE(C % 8 == 0 && C <= 64 * 8 * 3, RDMI_E_UNSUPPORTED, "cross_attn_pair: C=%d unsupported", C);
  RDMI_REQUIRE((((uintptr_t)x | (uintptr_t)y | (uintptr_t)w | (uintptr_t)u) & 15) == 0, RDMI_E_ALIGN,
               "cross_attn_pair: pointers must be 16-byte aligned");
  const size_t lds = (size_t)2 * H * C * sizeof(float);
  RDMI_REQUIRE(lds <= 64 * 1024 && H <= 16, RDMI_E_UNSUPPORTED, "cross_attn_pair: H=%d, H*C=%d unsupported", H, H * C);
  long blocks = (M + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  const int nv = (C / 8 + 63) / 64;
#define RDMI_PAIR(NVV, HCC) \
  hipLaunchKernelGGL((attn2_pair_k<NVV, HCC>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, \
                     (const f16*)x, (f16*)y, M, C, H, ln_gamma, ln_beta, eps, w, u, c)
  // the SD2 UNet's L0 / L1 blocks (5 / 10 heads) with the heads unrolled (RDMI_PAIR_HC=0: the loop, A/B)
  const char* ehc = getenv("RDMI_PAIR_HC");
  const bool hc = !(ehc && ehc[0] == '0');
  if (nv == 1 && H == 5 && hc)
    RDMI_PAIR(1, 5);
  else if (nv == 2 && H == 10 && hc)
    RDMI_PAIR(2, 10);
  else if (nv == 1)
    RDMI_PAIR(1, 0);
  else if (nv == 2)
    RDMI_PAIR(2, 0);
  else
    RDMI_PAIR(3, 0);
#undef RDMI_PAIR
  return rdmi::check_launch("cross_attn_pair");
}

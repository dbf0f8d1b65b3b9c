// Cross-frame attention kernels.
//
// attn_fwd_d64: flash-style fused softmax(q kᵀ·scale) v for head_dim 64 on gfx950.
//   Workgroup = 8 waves × 32 queries (256 queries) of one (batch, head); 128-key K/V tiles arrive
//   by LDS-DMA into a 3-slot ring (two tiles in flight; K XOR-swizzled per 16-B chunk through the
//   source address).
//   Per wave and tile: Sᵀ = K·Qᵀ with v_mfma_f32_32x32x16_f16 (Q fragments live in registers for
//   the whole sweep), so each lane owns one query's scores ("swapped QKᵀ": the row max/sum is
//   lane-local plus one lane^32 exchange); Oᵀ = Vᵀ·Pᵀ with the P accumulator re-used directly
//   as the B operand (keys in the MFMA's permuted k order) and V read from LDS with
//   ds_read_b64_tr_b16 (hardware transpose).  Online softmax in exp2 domain, f32 throughout; the
//   O rescale is skipped (exactly) on tiles where no lane's running max moved.
// attn_smallkv: attention of every query token against ≤ 16 shared keys (the UNet's
//   cross-attention to the 2-token empty-text context) — a streaming kernel, no MFMA.
// softmax_rows: f32 scores → f16 probabilities, for the d=C single-head VAE attention that is
//   run as GEMM → softmax → GEMM.
#include "common.h"

namespace {

struct AttnP {
  const f16* q; const f16* k; const f16* v; f16* o;
  int H, Sq, Sk;
  long q_ld, k_ld, v_ld, o_ld, q_bs, k_bs, v_bs, o_bs;
  float sl2;  // scale * log2(e)
};

constexpr int NWV = 8;        // waves per workgroup
constexpr int QB = 32 * NWV;  // queries per workgroup (32 per wave)
constexpr int KB = 128;       // keys per tile
constexpr int NKB = KB / 32;  // 32-key MFMA blocks per tile
constexpr int DPW = KB / 8 / NWV;  // 8-row DMA instructions per wave per tile, per tensor
constexpr int TILE = KB * 64; // halves per K (or V) tile

__device__ f16x8 g_attn_zero16;

template <int N>
__device__ __forceinline__ void attn_wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}

// K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4) into a 3-slot ring (no VGPR staging,
// no ds_write): each wave moves 8 key rows of K and of V per tile.  K's 16-B chunks are
// XOR-swizzled by (key & 7) through the per-lane source address; V stays row-major for the
// transposed reads.
__global__ __launch_bounds__(64 * NWV, 1) void attn_fwd_d64(AttnP p) {
  __shared__ __attribute__((aligned(16))) f16 lds[3 * 2 * TILE];  // 96 KB: slot s = [K | V]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int hh = lane >> 5;  // lane half
  const int c = lane & 31;
  const int head = blockIdx.y;
  const int b = blockIdx.z;
  const int qi = blockIdx.x * QB + wid * 32 + c;

  const f16* Q = p.q + (long)b * p.q_bs + head * 64;
  const f16* K = p.k + (long)b * p.k_bs + head * 64;
  const f16* V = p.v + (long)b * p.v_bs + head * 64;

  // Q as the B operand of Sᵀ = K·Qᵀ: lane holds Q[qi][16ks + 8hh + 0..7]
  f16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    f16x8 z = {};
    qf[ks] = qi < p.Sq ? *(const f16x8*)(Q + (long)qi * p.q_ld + ks * 16 + hh * 8) : z;
  }

  // DMA lane geometry: 8 rows x 8 chunks per 1-KiB instruction; row = wid*8 + drow.
  // LDS images (bank-conflict-free for the fragment reads, checked with SQ_LDS_BANK_CONFLICT):
  //   K: phys chunk = logical ^ ((row >> 1) & 7)   (ds_read_b128 of 16 distinct rows / group)
  //   V: phys chunk = logical ^ (((row >> 1) & 1) << 2)   (tr reads of 4 rows x 64 B / half-wave)
  const int drow = lane >> 3;
  const f16* zero = (const f16*)&g_attn_zero16;
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int row = (i * NWV + wid) * 8 + drow;  // (row >> 1) & 7 depends on drow and wid only
      const int kchunk = (lane & 7) ^ ((row >> 1) & 7);
      const int vchunk = (lane & 7) ^ (((row >> 1) & 1) << 2);
      const int key = kt * KB + row;
      const bool ok = key < p.Sk;
      f16* ks_ = lds + slot * 2 * TILE + (i * NWV + wid) * 8 * 64;
      __builtin_amdgcn_global_load_lds(ok ? (const void*)(K + (long)key * p.k_ld + kchunk * 8) : (const void*)zero,
                                       (__attribute__((address_space(3))) void*)ks_, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(ok ? (const void*)(V + (long)key * p.v_ld + vchunk * 8) : (const void*)zero,
                                       (__attribute__((address_space(3))) void*)(ks_ + TILE), 16, 0, 0);
    }
  };

  f32x16 o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  const int nt = (p.Sk + KB - 1) / KB;
  // tr-read lane geometry (16-lane groups)
  const int gi = lane >> 4, li = lane & 15;
  const int tr_key = 4 * (gi >> 1) + (li >> 2);
  const int tr_col = 16 * (gi & 1) + 4 * (li & 3);
  issue(0, 0);
  issue(1, 1);  // zero rows when nt == 1: keeps exactly 2·DPW younger DMAs in flight at every wait

  for (int kt = 0; kt < nt; ++kt) {
    attn_wait_vmcnt<2 * DPW>();  // this wave's DMAs of tile kt landed (tile kt+1 in flight)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of kt landed; every wave done with kt-1
    asm volatile("" ::: "memory");
    issue(kt + 2, (kt + 2) % 3);   // past the end: zero rows into the drained slot
    const f16* ks_ = lds + (kt % 3) * 2 * TILE;
    const f16* vs_ = ks_ + TILE;
    // ---- Sᵀ = K · Qᵀ for NKB key blocks of 32
    f32x16 s[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
      const int key = kb * 32 + c;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = 2 * ks + hh;
        f16x8 kf = *(const f16x8*)(ks_ + key * 64 + ((ch ^ ((key >> 1) & 7)) << 3));
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[ks], s[kb], 0, 0, 0);
      }
    }
    // ---- mask + online softmax (lane owns query c, keys (r&3)+8(r>>2)+4hh of each block)
    const int kbase = kt * KB;
    float mx = -INFINITY;
    if (kbase + KB <= p.Sk) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
    } else {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int key = kbase + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key >= p.Sk) s[kb][r] = -INFINITY;
          mx = fmaxf(mx, s[kb][r]);
        }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    // exact T13: rescale O only when some lane's running max moved (alpha == 1 otherwise)
    if (__any(mn > m)) {
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * p.sl2);
      l *= alpha;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      m = mn;
    }
    const float msc = m * p.sl2;
    float rs = 0.f;
    f16x8 pf[2 * NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float e = __builtin_amdgcn_exp2f(fmaf(s[kb][r], p.sl2, -msc));  // v_exp_f32, no denorm fixup
        rs += e;
        pf[kb * 2 + (r >> 3)][r & 7] = (f16)e;
      }
    l += rs;
    // ---- Oᵀ += Vᵀ · Pᵀ (KB/16 k-steps of 16 keys, 2 d-blocks of 32)
#pragma unroll
    for (int st = 0; st < 2 * NKB; ++st) {
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        // row = 16st + tr_key (+8): (row >> 1) & 1 == (tr_key >> 1) & 1 for both reads
        const int col = d * 32 + tr_col;
        const int pc = ((col >> 3) ^ (((tr_key >> 1) & 1) << 2)) << 3 | (col & 7);
        const f16* base = vs_ + (16 * st + tr_key) * 64 + pc;
        i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(i16x4, base));
        i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(i16x4, base + 8 * 64));
        const f16x8 vf = __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        o[d] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[st], o[d], 0, 0, 0);
      }
    }
  }
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
}

// one thread per (token, head); D == 64, L ≤ 16
__global__ __launch_bounds__(256) void attn_smallkv(const f16* __restrict__ q, const f16* __restrict__ k,
                                                    const f16* __restrict__ v, f16* __restrict__ o, int H, int Sq,
                                                    int L, long q_ld, long o_ld, long q_bs, long o_bs, long kv_bs,
                                                    float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f16* kl = (f16*)smem;              // [L][H*64]
  f16* vl = kl + L * H * 64;
  const int b = blockIdx.y;
  const int HD = H * 64;
  for (int i = threadIdx.x; i < L * HD / 8; i += blockDim.x) {
    ((f16x8*)kl)[i] = ((const f16x8*)(k + (long)b * kv_bs))[i];
    ((f16x8*)vl)[i] = ((const f16x8*)(v + (long)b * kv_bs))[i];
  }
  __syncthreads();
  long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)Sq * H) return;
  int tok = (int)(idx / H), h = (int)(idx % H);
  const f16* qr = q + (long)b * q_bs + (long)tok * q_ld + h * 64;
  float qv[64];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f16x8 t = *(const f16x8*)(qr + 8 * i);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[8 * i + e] = (float)t[e];
  }
  float sc[16];
  float mx = -INFINITY;
  for (int j = 0; j < L; ++j) {
    const f16* kr = kl + j * HD + h * 64;
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) a += qv[d] * (float)kr[d];
    sc[j] = a * scale;
    mx = fmaxf(mx, sc[j]);
  }
  float den = 0.f;
  for (int j = 0; j < L; ++j) {
    sc[j] = __expf(sc[j] - mx);
    den += sc[j];
  }
  float inv = 1.f / den;
  float acc[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) acc[d] = 0.f;
  for (int j = 0; j < L; ++j) {
    const f16* vr = vl + j * HD + h * 64;
    float w = sc[j] * inv;
#pragma unroll
    for (int d = 0; d < 64; ++d) acc[d] += w * (float)vr[d];
  }
  f16* orow = o + (long)b * o_bs + (long)tok * o_ld + h * 64;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f16x8 t;
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = (f16)acc[8 * i + e];
    *(f16x8*)(orow + 8 * i) = t;
  }
}

__global__ __launch_bounds__(256) void softmax_rows_k(const float* __restrict__ s, f16* __restrict__ pout, long cols,
                                                      float scale) {
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
  for (long c = threadIdx.x; c < cols; c += 256) sum += __expf((sr[c] - mx) * scale);
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  sum = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / sum;
  f16* pr = pout + row * cols;
  for (long c = threadIdx.x; c < cols; c += 256) pr[c] = (f16)(__expf((sr[c] - mx) * scale) * inv);
}

}  // namespace

extern "C" int rdmi_attention_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                                  int D, long q_ld, long k_ld, long v_ld, long o_ld, long q_bs, long k_bs, long v_bs,
                                  long o_bs, float scale, void* stream) {
  RDMI_REQUIRE(q && k && v && o, RDMI_E_ARG, "attention_fwd: null pointer");
  RDMI_REQUIRE(D == 64, RDMI_E_UNSUPPORTED, "attention_fwd: head_dim %d unsupported (64 only)", D);
  RDMI_REQUIRE(B > 0 && H > 0 && Sq > 0 && Sk > 0, RDMI_E_ARG, "attention_fwd: bad sizes");
  RDMI_REQUIRE(q_ld % 8 == 0 && k_ld % 8 == 0 && v_ld % 8 == 0 && o_ld % 4 == 0 && (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v) & 15) == 0,
               RDMI_E_ALIGN, "attention_fwd: strides/pointers must be 16-byte aligned");
  AttnP p{(const f16*)q, (const f16*)k, (const f16*)v, (f16*)o, H, Sq, Sk, q_ld, k_ld, v_ld, o_ld, q_bs, k_bs, v_bs, o_bs,
          scale * 1.4426950408889634f};
  dim3 g(rdmi::div_up(Sq, QB), H, B);
  hipLaunchKernelGGL(attn_fwd_d64, g, dim3(64 * NWV), 0, (hipStream_t)stream, p);
  return rdmi::check_launch("attention_fwd");
}

extern "C" int rdmi_attention_smallkv(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int L,
                                      int D, long q_ld, long o_ld, long q_bs, long o_bs, long kv_bs, float scale,
                                      void* stream) {
  RDMI_REQUIRE(q && k && v && o, RDMI_E_ARG, "attention_smallkv: null pointer");
  RDMI_REQUIRE(D == 64 && L >= 1 && L <= 16, RDMI_E_UNSUPPORTED, "attention_smallkv: D=%d L=%d unsupported", D, L);
  size_t lds = (size_t)2 * L * H * 64 * sizeof(f16);
  RDMI_REQUIRE(lds <= 64 * 1024, RDMI_E_UNSUPPORTED, "attention_smallkv: K/V too large for LDS");
  dim3 g(rdmi::div_up((long)Sq * H, 256), B);
  hipLaunchKernelGGL(attn_smallkv, g, dim3(256), lds, (hipStream_t)stream, (const f16*)q, (const f16*)k, (const f16*)v,
                     (f16*)o, H, Sq, L, q_ld, o_ld, q_bs, o_bs, kv_bs, scale);
  return rdmi::check_launch("attention_smallkv");
}

extern "C" int rdmi_softmax_rows(const float* s, void* p, long rows, long cols, float scale, void* stream) {
  RDMI_REQUIRE(s && p && rows > 0 && cols > 0, RDMI_E_ARG, "softmax_rows: bad args");
  hipLaunchKernelGGL(softmax_rows_k, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, s, (f16*)p, cols, scale);
  return rdmi::check_launch("softmax_rows");
}

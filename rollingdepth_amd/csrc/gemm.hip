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
#include "common.h"

namespace {

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
  int geglu, silu;
  // convolution (A gathered from NHWC x)
  int IH, IW, Cin, Ho, Wo, kh, kw, stride, pt, pl, up, cin_vecs;
};

// MODE 0: dense A [M, K] (Linear, 1×1 conv); MODE 1: implicit im2col of NHWC x (kh×kw conv).
// LDS tiles are [rows][64] halves with the 16-B chunk index XOR-swizzled by (row & 7)
// (conflict-spread ds_read_b128 fragment reads, cdna_hip_programming.md §5.5 T2).
template <int BM, int BN, int MODE>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmP p) {
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AV = BM / 32;  // 16-B A vectors per thread per stage (8 chunks x BM rows / 256)
  constexpr int BV = BN / 32;
  __shared__ __attribute__((aligned(16))) f16 lds[2][(BM + BN) * BK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // XCD-aware remap (T1): dispatch id d runs on XCD d % 8; give each XCD a contiguous range of
  // logical tiles so the n-tiles sharing one A row-panel share that XCD's L2.
  const int nbx = gridDim.x, nby = gridDim.y;
  const int total = nbx * nby;
  const int bid = blockIdx.y * nbx + blockIdx.x;
  int logical = bid;
  if (total >= 8) {
    const int xcd = bid & 7, q = total >> 3, r = total & 7;
    logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int n0 = (logical % nbx) * BN;
  const int m0 = (logical / nbx) * BM;
  const int bz = blockIdx.z;
  const f16* A = p.A + (long)bz * p.sA;
  const f16* Wt = p.Wt + (long)bz * p.sW;

  const int chunk = tid & 7;
  const int rbase = tid >> 3;
  bool arow_ok[AV];
  long abase[AV];
  int ahb[AV], awb[AV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    const int m = m0 + rbase + 32 * i;
    arow_ok[i] = m < p.M;
    const int mm = arow_ok[i] ? m : 0;
    if (MODE == 1) {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw;
      const int r = mm - b * hw;
      const int ho = r / p.Wo;
      const int wo = r - ho * p.Wo;
      ahb[i] = ho * p.stride - p.pt;
      awb[i] = wo * p.stride - p.pl;
      abase[i] = (long)b * p.IH * p.IW * p.Cin;
    } else {
      abase[i] = (long)mm * p.lda;
      ahb[i] = awb[i] = 0;
    }
  }
  // incremental (tap, channel-vector) of this thread's chunk: k-vector index = k0/8 + chunk
  int tap = 0, cv = chunk;
  if (MODE == 1) {
    tap = chunk / p.cin_vecs;
    cv = chunk - tap * p.cin_vecs;
  }
  const int Hl = p.IH << p.up, Wl = p.IW << p.up;

  auto loadA = [&](int k0, f16x8 (&ra)[AV]) {
    const int kk = k0 + chunk * 8;
    const bool kok = kk < p.Kvalid;
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        f16x8 v = {};
        if (arow_ok[i] && kok) v = *(const f16x8*)(A + abase[i] + kk);
        ra[i] = v;
      }
    } else {
      int dy, dx;
      if (p.kw == 3) {
        dy = (tap * 11) >> 5;  // tap / 3 for tap < 9
        dx = tap - 3 * dy;
      } else {
        dy = tap / p.kw;
        dx = tap - dy * p.kw;
      }
      const long coff = (long)cv * 8;
#pragma unroll
      for (int i = 0; i < AV; ++i) {
        f16x8 v = {};
        int hi = ahb[i] + dy, wi = awb[i] + dx;
        if (arow_ok[i] && kok && hi >= 0 && hi < Hl && wi >= 0 && wi < Wl) {
          hi >>= p.up;
          wi >>= p.up;
          v = *(const f16x8*)(A + abase[i] + ((long)hi * p.IW + wi) * p.Cin + coff);
        }
        ra[i] = v;
      }
    }
  };
  auto advance = [&]() {
    if (MODE == 1) {
      cv += 8;
      while (cv >= p.cin_vecs) {
        cv -= p.cin_vecs;
        ++tap;
      }
    }
  };
  auto loadB = [&](int k0, f16x8 (&rb)[BV]) {
    const int kk = k0 + chunk * 8;
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int n = n0 + rbase + 32 * i;
      f16x8 v = {};
      if (n < p.N && kk < p.Kvalid) v = *(const f16x8*)(Wt + (long)n * p.ldw + kk);
      rb[i] = v;
    }
  };
  auto store = [&](int buf, const f16x8 (&ra)[AV], const f16x8 (&rb)[BV]) {
    f16* la = lds[buf];
    f16* lb = lds[buf] + BM * BK;
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int row = rbase + 32 * i;
      *(f16x8*)(la + row * BK + ((chunk ^ (row & 7)) << 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int row = rbase + 32 * i;
      *(f16x8*)(lb + row * BK + ((chunk ^ (row & 7)) << 3)) = rb[i];
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f16x8 ra[AV], rb[BV];
  const int nk = (p.K + BK - 1) / BK;
  loadA(0, ra);
  loadB(0, rb);
  advance();
  store(0, ra, rb);
  __syncthreads();
  int cur = 0;
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      loadA((kt + 1) * BK, ra);
      loadB((kt + 1) * BK, rb);
      advance();
    }
    const f16* la = lds[cur] + (wm * WTM) * BK;
    const f16* lb = lds[cur] + BM * BK + (wn * WTN) * BK;
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(cur ^ 1, ra, rb);
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + r
  const long cb = (long)bz * p.sC;
  const long rbz = (long)bz * p.sR;
  if (!p.geglu) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
        if (m >= p.M) continue;
        const float* rbrow = p.rowbias ? p.rowbias + (long)(m / p.rpg) * p.rb_ld : nullptr;
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          int n = n0 + wn * WTN + j * 16 + fr;
          if (n >= p.N) continue;
          float v = acc[i][j][r] * p.alpha;
          if (p.bias) v += p.bias[n];
          if (rbrow) v += rbrow[n];
          if (p.R) v += (float)p.R[rbz + (long)m * p.ldr + n];
          if (p.silu) v = silu_f(v);
          if (p.c_f32)
            ((float*)p.C)[cb + (long)m * p.ldc + n] = v;
          else
            ((f16*)p.C)[cb + (long)m * p.ldc + n] = (f16)v;
        }
      }
    }
  } else {
    // GEGLU: within each wave's WTN(=64)-column slab, columns [0,32) are the value half and
    // [32,64) the gate half of output columns slab*32 + [0,32).
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < RN / 2; ++j) {
          int nh = n0 + wn * WTN + j * 16 + fr;
          int ng = nh + WTN / 2;
          int no = (n0 + wn * WTN) / 2 + j * 16 + fr;
          float h = acc[i][j][r] * p.alpha + (p.bias ? p.bias[nh] : 0.f);
          float g = acc[i][j + RN / 2][r] * p.alpha + (p.bias ? p.bias[ng] : 0.f);
          float v = h * gelu_erf(g);
          if (p.R) v += (float)p.R[rbz + (long)m * p.ldr + no];
          if (p.c_f32)
            ((float*)p.C)[cb + (long)m * p.ldc + no] = v;
          else
            ((f16*)p.C)[cb + (long)m * p.ldc + no] = (f16)v;
        }
      }
    }
  }
}

template <int MODE>
void launch_mode(const GemmP& p, int batch, hipStream_t s, bool force128) {
  if (force128 || p.N % 128 == 0 || p.N > 512) {
    dim3 g(rdmi::div_up(p.N, 128), rdmi::div_up(p.M, 128), batch);
    hipLaunchKernelGGL((gemm_kernel<128, 128, MODE>), g, dim3(256), 0, s, p);
  } else {
    dim3 g(rdmi::div_up(p.N, 64), rdmi::div_up(p.M, 256), batch);
    hipLaunchKernelGGL((gemm_kernel<256, 64, MODE>), g, dim3(256), 0, s, p);
  }
}

int launch(const GemmP& p, int batch, hipStream_t s, bool force128, bool conv) {
  if (conv)
    launch_mode<1>(p, batch, s, force128);
  else
    launch_mode<0>(p, batch, s, force128);
  return rdmi::check_launch("gemm");
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int rdmi_gemm(const rdmi_gemm_args* a, void* stream) {
  RDMI_REQUIRE(a && a->A && a->W && a->C, RDMI_E_ARG, "gemm: null pointer");
  RDMI_REQUIRE(a->M > 0 && a->N > 0 && a->K > 0 && a->batch > 0, RDMI_E_ARG, "gemm: bad sizes M=%d N=%d K=%d", a->M, a->N, a->K);
  RDMI_REQUIRE(a->K % 8 == 0 && a->lda % 8 == 0 && a->ldw % 8 == 0 && a->ldw >= a->K,
               RDMI_E_ALIGN, "gemm: K (%d), lda (%ld) must be multiples of 8 and ldw (%ld) >= K", a->K, a->lda, a->ldw);
  RDMI_REQUIRE(al16(a->A) && al16(a->W) && a->strideA % 8 == 0 && a->strideW % 8 == 0, RDMI_E_ALIGN, "gemm: A/W not 16-byte aligned");
  RDMI_REQUIRE(a->epilogue != RDMI_EPI_GEGLU || a->N % 128 == 0, RDMI_E_ARG, "gemm: GEGLU needs N %% 128 == 0");
  RDMI_REQUIRE(!a->rowbias || a->rows_per_group > 0, RDMI_E_ARG, "gemm: rowbias needs rows_per_group");
  GemmP p{};
  p.A = (const f16*)a->A; p.lda = a->lda; p.sA = a->strideA;
  p.Wt = (const f16*)a->W; p.ldw = a->ldw; p.sW = a->strideW;
  p.C = a->C; p.ldc = a->ldc; p.sC = a->strideC; p.c_f32 = a->c_f32;
  p.bias = a->bias; p.R = (const f16*)a->residual; p.ldr = a->ldr; p.sR = a->strideR;
  p.rowbias = a->rowbias; p.rpg = a->rows_per_group > 0 ? a->rows_per_group : 1; p.rb_ld = a->rowbias_ld;
  p.alpha = a->alpha;
  p.M = a->M; p.N = a->N; p.K = (a->K + BK - 1) / BK * BK; p.Kvalid = a->K;
  p.geglu = a->epilogue == RDMI_EPI_GEGLU;
  p.silu = a->epilogue == RDMI_EPI_SILU;
  return launch(p, a->batch, (hipStream_t)stream, p.geglu, false);
}

extern "C" int rdmi_conv2d(const rdmi_conv_args* a, void* stream) {
  RDMI_REQUIRE(a && a->x && a->w && a->y, RDMI_E_ARG, "conv2d: null pointer");
  RDMI_REQUIRE(a->Cin % 8 == 0, RDMI_E_ALIGN, "conv2d: Cin (%d) must be a multiple of 8", a->Cin);
  RDMI_REQUIRE(a->B > 0 && a->H > 0 && a->W > 0 && a->Cout > 0 && a->Ho > 0 && a->Wo > 0, RDMI_E_ARG, "conv2d: bad sizes");
  const int K = a->kh * a->kw * a->Cin;
  RDMI_REQUIRE(a->Kp >= K && a->Kp % 8 == 0, RDMI_E_ARG, "conv2d: Kp (%d) must be >= %d and a multiple of 8", a->Kp, K);
  RDMI_REQUIRE(al16(a->x) && al16(a->w), RDMI_E_ALIGN, "conv2d: x/w not 16-byte aligned");
  GemmP p{};
  p.A = (const f16*)a->x; p.Wt = (const f16*)a->w; p.ldw = a->Kp;
  p.C = a->y; p.ldc = a->y_ld > 0 ? a->y_ld : a->Cout;
  p.bias = a->bias; p.R = (const f16*)a->residual; p.ldr = a->res_ld > 0 ? a->res_ld : a->Cout;
  p.rowbias = a->rowbias; p.rpg = a->Ho * a->Wo; p.rb_ld = a->rowbias_ld;
  p.alpha = a->alpha;
  p.M = a->B * a->Ho * a->Wo; p.N = a->Cout; p.K = a->Kp; p.Kvalid = K;
  p.IH = a->H; p.IW = a->W; p.Cin = a->Cin; p.Ho = a->Ho; p.Wo = a->Wo;
  p.kh = a->kh; p.kw = a->kw; p.stride = a->stride; p.pt = a->pad_top; p.pl = a->pad_left;
  p.up = a->upsample ? 1 : 0; p.cin_vecs = a->Cin / 8;
  // a 1×1, stride-1, unpadded conv on NHWC is a dense GEMM over pixels (conv_shortcut, quant convs)
  const bool dense = a->kh == 1 && a->kw == 1 && a->stride == 1 && a->pad_top == 0 && a->pad_left == 0 && !a->upsample &&
                     a->Ho == a->H && a->Wo == a->W;
  if (dense) p.lda = a->Cin;
  return launch(p, 1, (hipStream_t)stream, false, !dense);
}

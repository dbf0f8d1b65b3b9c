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

constexpr int BK = 32;
constexpr int LDSK = BK + 8;  // padded LDS row (80 B) against ds_read_b128 bank conflicts

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
  int conv, IH, IW, Cin, Ho, Wo, kh, kw, stride, pt, pl, up, cin_vecs;
};

template <int BM, int BN>
__global__ __launch_bounds__(256) void gemm_kernel(GemmP p) {
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AV = BM * 4 / 256;  // 16-B A vectors per thread per K-step
  constexpr int BV = BN * 4 / 256;
  __shared__ __attribute__((aligned(16))) f16 lds[2][(BM + BN) * LDSK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;
  const int bz = blockIdx.z;
  const f16* A = p.A + (long)bz * p.sA;
  const f16* Wt = p.Wt + (long)bz * p.sW;

  const int chunk = tid & 3;
  // per-row precompute for the A gather
  int arow_ok[AV];
  long abase[AV];
  int aho[AV], awo[AV];
#pragma unroll
  for (int i = 0; i < AV; ++i) {
    int m = m0 + (tid >> 2) + 64 * i;
    arow_ok[i] = m < p.M;
    int mm = arow_ok[i] ? m : 0;
    if (p.conv) {
      int hw = p.Ho * p.Wo;
      int b = mm / hw;
      int r = mm - b * hw;
      aho[i] = r / p.Wo;
      awo[i] = r - aho[i] * p.Wo;
      abase[i] = (long)b * p.IH * p.IW * p.Cin;
    } else {
      abase[i] = (long)mm * p.lda;
      aho[i] = awo[i] = 0;
    }
  }

  auto loadA = [&](int k0, f16x8 (&ra)[AV]) {
    const int kk = k0 + chunk * 8;
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      f16x8 v = {};
      if (arow_ok[i] && kk < p.Kvalid) {
        if (!p.conv) {
          v = *(const f16x8*)(A + abase[i] + kk);
        } else {
          int kv = kk >> 3;
          int tap = kv / p.cin_vecs;
          int cv = kv - tap * p.cin_vecs;
          int dy = tap / p.kw;
          int dx = tap - dy * p.kw;
          int hi = aho[i] * p.stride - p.pt + dy;
          int wi = awo[i] * p.stride - p.pl + dx;
          int Hl = p.IH << p.up, Wl = p.IW << p.up;
          if (hi >= 0 && hi < Hl && wi >= 0 && wi < Wl) {
            hi >>= p.up;
            wi >>= p.up;
            v = *(const f16x8*)(A + abase[i] + ((long)hi * p.IW + wi) * p.Cin + cv * 8);
          }
        }
      }
      ra[i] = v;
    }
  };
  auto loadB = [&](int k0, f16x8 (&rb)[BV]) {
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      int n = n0 + (tid >> 2) + 64 * i;
      f16x8 v = {};
      if (n < p.N && k0 + chunk * 8 < p.Kvalid) v = *(const f16x8*)(Wt + (long)n * p.ldw + k0 + chunk * 8);
      rb[i] = v;
    }
  };
  auto store = [&](int buf, const f16x8 (&ra)[AV], const f16x8 (&rb)[BV]) {
    f16* la = lds[buf];
    f16* lb = lds[buf] + BM * LDSK;
#pragma unroll
    for (int i = 0; i < AV; ++i) *(f16x8*)(la + ((tid >> 2) + 64 * i) * LDSK + chunk * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BV; ++i) *(f16x8*)(lb + ((tid >> 2) + 64 * i) * LDSK + chunk * 8) = rb[i];
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f16x8 ra[AV], rb[BV];
  const int nk = p.K / BK;
  loadA(0, ra);
  loadB(0, rb);
  store(0, ra, rb);
  __syncthreads();
  int cur = 0;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      loadA((kt + 1) * BK, ra);
      loadB((kt + 1) * BK, rb);
    }
    const f16* la = lds[cur] + (wm * WTM) * LDSK;
    const f16* lb = lds[cur] + BM * LDSK + (wn * WTN) * LDSK;
    f16x8 af[RM], bf[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = *(const f16x8*)(la + (i * 16 + fr) * LDSK + fk);
#pragma unroll
    for (int j = 0; j < RN; ++j) bf[j] = *(const f16x8*)(lb + (j * 16 + fr) * LDSK + fk);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
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
        int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
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
        int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
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

int launch(const GemmP& p, int batch, hipStream_t s, bool force128) {
  if (force128 || p.N % 128 == 0) {
    dim3 g(rdmi::div_up(p.N, 128), rdmi::div_up(p.M, 128), batch);
    hipLaunchKernelGGL((gemm_kernel<128, 128>), g, dim3(256), 0, s, p);
  } else {
    dim3 g(rdmi::div_up(p.N, 64), rdmi::div_up(p.M, 256), batch);
    hipLaunchKernelGGL((gemm_kernel<256, 64>), g, dim3(256), 0, s, p);
  }
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
  p.M = a->M; p.N = a->N; p.K = (a->K + 31) / 32 * 32; p.Kvalid = a->K;
  p.geglu = a->epilogue == RDMI_EPI_GEGLU;
  p.silu = a->epilogue == RDMI_EPI_SILU;
  return launch(p, a->batch, (hipStream_t)stream, p.geglu);
}

extern "C" int rdmi_conv2d(const rdmi_conv_args* a, void* stream) {
  RDMI_REQUIRE(a && a->x && a->w && a->y, RDMI_E_ARG, "conv2d: null pointer");
  RDMI_REQUIRE(a->Cin % 8 == 0, RDMI_E_ALIGN, "conv2d: Cin (%d) must be a multiple of 8", a->Cin);
  RDMI_REQUIRE(a->B > 0 && a->H > 0 && a->W > 0 && a->Cout > 0 && a->Ho > 0 && a->Wo > 0, RDMI_E_ARG, "conv2d: bad sizes");
  const int K = a->kh * a->kw * a->Cin;
  RDMI_REQUIRE(a->Kp >= K && a->Kp % 32 == 0, RDMI_E_ARG, "conv2d: Kp (%d) must be >= %d and a multiple of 32", a->Kp, K);
  RDMI_REQUIRE(al16(a->x) && al16(a->w), RDMI_E_ALIGN, "conv2d: x/w not 16-byte aligned");
  GemmP p{};
  p.A = (const f16*)a->x; p.Wt = (const f16*)a->w; p.ldw = a->Kp;
  p.C = a->y; p.ldc = a->y_ld > 0 ? a->y_ld : a->Cout;
  p.bias = a->bias; p.R = (const f16*)a->residual; p.ldr = a->res_ld > 0 ? a->res_ld : a->Cout;
  p.rowbias = a->rowbias; p.rpg = a->Ho * a->Wo; p.rb_ld = a->rowbias_ld;
  p.alpha = a->alpha;
  p.M = a->B * a->Ho * a->Wo; p.N = a->Cout; p.K = a->Kp; p.Kvalid = K;
  p.conv = 1; p.IH = a->H; p.IW = a->W; p.Cin = a->Cin; p.Ho = a->Ho; p.Wo = a->Wo;
  p.kh = a->kh; p.kw = a->kw; p.stride = a->stride; p.pt = a->pad_top; p.pl = a->pad_left;
  p.up = a->upsample ? 1 : 0; p.cin_vecs = a->Cin / 8;
  return launch(p, 1, (hipStream_t)stream, false);
}

// Implicit-GEMM engine: host-side dispatch (engine choice per launch shape, argument checks).
// The kernels are in gemm_kernels.h; each engine family is instantiated in its own translation
// unit (gemm_classic.hip, gemm_pp.hip, conv_halo.hip, conv_occ2.hip).
#include "gemm_kernels.h"

#include <stdlib.h>

namespace {

using namespace rdmi_gk;


// Two-workgroups-per-CU GEMM engine (RDMI_GEMM_OCC2, read per launch for A/B: 0 off, 2 every
// dense GEMM, unset/1 = the measured policy in launch_mode)
int occ2_mode() {
  const char* e = getenv("RDMI_GEMM_OCC2");
  return e ? atoi(e) : 1;
}

// Engine choice.  RDMI_GEMM_PP (read per launch; for tests and A/B measurements): 0 = classic
// engine only, 2 = a ping-pong tile whenever the shape allows one, unset/1 = by estimated cost.
int pp_mode() {
  const char* e = getenv("RDMI_GEMM_PP");
  return e ? atoi(e) : 1;
}

// Relative cost of a launch on an engine: rounds of one tile per CU × tile area ÷ measured
// efficiency (tools/kbench.py on MI355X: the 256×256 ping-pong tile ≈ 1.3× the classic 256×128
// engine per tile area, the 512×128 one ≈ 1.0×).
double tile_cost(long tiles, int bm, int bn, double eff) {
  return (double)((tiles + 255) / 256) * bm * bn / eff;
}

template <int MODE, int WM, int RN>
void launch_pp(const GemmP& p, int batch, hipStream_t s) {
  constexpr int BM = WM * 128, BN = (8 / WM) * RN * 16;
  dim3 g(p.N / BN, rdmi::div_up(p.M, BM), batch);
  static_assert(RN == 4, "ping-pong tiles use RN = 4");
  launch_gemm_pp(MODE, WM, 0, g, s, p);
}

template <int MODE>
void launch_mode(const GemmP& p, int batch, hipStream_t s, bool force128) {
  if (MODE == 0) {
    // measured policy (tools/gemm_policy_ab.py at the pipeline's shapes, profiles/r02_gemm_policy_ab.log,
    // after the epilogue fix): the two-workgroups-per-CU engine wins on the UNet's single-batch
    // Linears whose N has no 128-wide ping-pong tile (L0: N = 320 / 960, +17…24 %); with one
    // (N % 128 == 0: L1 N = 640 / 1920, L2 N = 1280 at K = 5120) the 512×128 / 256×256 ping-pong
    // tiles win by 3…17 %; it loses on the GEGLU projections and the batched VAE attention GEMMs
    const int oc = occ2_mode();
    const bool pick = !p.geglu && batch == 1 && !p.c_f32 && p.N <= 1920 && p.N % 128 != 0;
    if (oc == 2 || (oc == 1 && pick)) {
      // 160-column tiles where N allows (RDMI_GEMM_BN160=0: 128 only, for A/B).  GEGLU stays on
      // 128-column tiles: its epilogue exists only for 64-column waves (store_tile_t)
      const char* e160 = getenv("RDMI_GEMM_BN160");
      const int bn = (p.N % 160 == 0 && !p.geglu && !(e160 && e160[0] == '0')) ? 160 : 128;
      dim3 g(rdmi::div_up(p.N, bn), rdmi::div_up(p.M, 128), batch);
      launch_gemm_occ2(bn, g, s, p);
      return;
    }
  }
  const int pp = pp_mode();
  // ping-pong candidates (N must be a multiple of the tile width; conv needs 64-channel blocks)
  if (pp != 0 && (MODE == 0 || p.cmaj)) {
    const char* dbg = MODE == 0 ? getenv("RDMI_GEMM_DBG") : nullptr;
    if (dbg && p.N % 256 == 0) {
      dim3 g(p.N / 256, rdmi::div_up(p.M, 256), batch);
      const int dv = atoi(dbg);
      if (dv == 1 || dv == 5 || dv == 8 || dv == 12) {
        launch_gemm_pp(0, 2, dv, g, s, p);
        return;
      }
    }
    const long mt256 = rdmi::div_up(p.M, 256), mt512 = rdmi::div_up(p.M, 512);
    const long ct = rdmi::div_up(p.N, 128);
    const double classic = tile_cost(mt256 * ct * batch, 256, 128, 1.0);
    double best = pp == 2 ? 1e300 : classic;
    int pick = 0;
    if (p.N % 256 == 0) {
      const double c = tile_cost(mt256 * (p.N / 256) * batch, 256, 256, 1.3);
      if (c < best) best = c, pick = 1;
    }
    if (p.N % 128 == 0) {
      // measured 1.06–1.11× the classic engine per area at the L1 Linears and the VAE 1×1 conv
      // (profiles/r02_gemm_policy_ab.log, after the epilogue fix)
      const double c = tile_cost(mt512 * (p.N / 128) * batch, 512, 128, 1.1);
      if (c < best) best = c, pick = 3;
    }
    switch (pick) {
      case 1: launch_pp<MODE, 2, 4>(p, batch, s); return;
      case 3: launch_pp<MODE, 4, 4>(p, batch, s); return;
      default: break;
    }
  }
  const long mt256 = (p.M + 255) / 256;
  if (force128 || p.N % 128 == 0 || p.N > 512) {
    if (mt256 * ((p.N + 127) / 128) * batch >= 512) {  // enough tiles to fill the chip with 256-row tiles
      dim3 g(rdmi::div_up(p.N, 128), rdmi::div_up(p.M, 256), batch);
      launch_gemm_classic(MODE, 256, 128, g, s, p);
    } else {
      dim3 g(rdmi::div_up(p.N, 128), rdmi::div_up(p.M, 128), batch);
      launch_gemm_classic(MODE, 128, 128, g, s, p);
    }
  } else {
    dim3 g(rdmi::div_up(p.N, 64), rdmi::div_up(p.M, 256), batch);
    launch_gemm_classic(MODE, 256, 64, g, s, p);
  }
}

int launch(GemmP p, int batch, hipStream_t s, bool force128, int mode) {
  const char* gm = getenv("RDMI_GEMM_GROUP");
  p.group_m = gm ? atoi(gm) : 8;  // measured: 8 m-tiles per group (tools/abl.sh, 8192³: +7 %)
  if (mode == 2)
    launch_mode<2>(p, batch, s, force128);
  else if (mode == 1)
    launch_mode<1>(p, batch, s, force128);
  else
    launch_mode<0>(p, batch, s, force128);
  return rdmi::check_launch("gemm");
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// 4-wide epilogue vectors need 4-element-aligned rows and pointers
bool vec_ok(const GemmP& p) {
  const uintptr_t csz = p.c_f32 ? 16 : 8;
  bool ok = p.ldc % 4 == 0 && p.sC % 4 == 0 && ((uintptr_t)p.C % csz) == 0;
  if (p.R) ok = ok && p.ldr % 4 == 0 && p.sR % 4 == 0 && ((uintptr_t)p.R & 7) == 0;
  if (p.bias) ok = ok && ((uintptr_t)p.bias & 15) == 0;
  if (p.rowbias) ok = ok && ((uintptr_t)p.rowbias & 15) == 0 && p.rb_ld % 4 == 0;
  return ok;
}

// Halo engine (RDMI_CONV_HALO, read per launch for A/B measurements: 0 disables it, 1 = the
// 4-phase 256-wide variant where one exists, 2 = the 256-wide 8-wave ping-pong for Cout % 256 == 0,
// 4 = the 8-wave variant for 128 output channels instead of the two-workgroups-per-CU one,
// unset/3 = default: the two-workgroups-per-CU variant for every Cout % 128 == 0 conv except a
// GroupNorm input wider than its 256-channel table.  Measured after the round-3 K-loop VALU cuts
// (tools/kbench.py conv, profiles/r03x_kbench.log): +4–9 % on the VAE 512-channel 96² and upsample
// convs, +6 % on the 384² GroupNorm conv, +1 % on the bench (r03x_halo_ab.log); bitwise the same
// results as the 256-wide form (same K-tile order and MFMA operands per output, r03y_bits_diff.txt).
int halo_mode() {
  const char* he = getenv("RDMI_CONV_HALO");
  return he ? atoi(he) : 3;
}

// 3×3 s1 p1 (optionally through the ×2 upsample), 64-channel blocks, 16×16 output patches,
// Cout % 64 == 0 (a ragged last 128-channel tile in the two-workgroups-per-CU variant).
bool halo_eligible(const rdmi_conv_args* a, int hmode) {
  return hmode != 0 && a->kh == 3 && a->kw == 3 && a->Cin % 64 == 0 && a->stride == 1 && a->pad_top == 1 &&
         a->pad_left == 1 && a->Ho % 16 == 0 && a->Wo % 16 == 0 && a->Cout % 64 == 0 &&
         a->Ho == (a->upsample ? 2 * a->H : a->H) && a->Wo == (a->upsample ? 2 * a->W : a->W);
}

// input GroupNorm: groups divide Cin; without in_affine the LDS scale/shift table holds ≤ 1024
// channels (≤ 256 in the two-workgroups-per-CU variant, the only one for Cout % 256 != 0 other than
// 128); with in_affine (the table in global memory, read per channel block) any Cin — only
// conv_halo_occ2_kernel reads that table, so rdmi_conv2d sends every in_affine conv to it whatever
// RDMI_CONV_HALO selects (the 256-wide and 8-wave engines keep their fixed 1024-entry LDS table); the
// opt-in 32×32×16 engine takes GroupNorm only for Cin ≤ 256, from the LDS table it builds itself
bool in_gn_ok(const rdmi_conv_args* a) {
  const int cmax = a->in_affine ? (1 << 30) : (a->Cout % 256 == 0 || a->Cout == 128) ? 1024 : 256;
  return a->in_groups > 0 && a->Cin <= cmax && a->Cin % a->in_groups == 0;
}

// conv_halo32_kernel: no upsample, Cout % 128 == 0, Cin % 128 == 0 (channel blocks in pairs), 32×8
// patches, 16-B epilogue accesses, input GroupNorm table ≤ 256 channels.  Opt-in (RDMI_CONV_H32=1):
// measured against conv_halo_occ2_kernel on the 768² 128-channel conv (tools/conv_ab.py,
// tools/pmc_conv_ab.sh, profiles/r02_pmc_conv_ab.txt) it cuts VALU per wave 3.4k → 1.5k and lifts
// MFMA-busy 0.60 → 0.63, but the chip is power-limited there (1.43–1.71 GHz under these loads) and
// the clock drops by as much: −2…+4 % plain, −4…−6 % with the GroupNorm input + residual.
bool h32_ok(const rdmi_conv_args* a, const GemmP& p, bool gn) {
  const char* e = getenv("RDMI_CONV_H32");
  if (!e || e[0] != '1') return false;
  return !a->upsample && a->Cout % 128 == 0 && a->Cin % 128 == 0 && a->Ho % 8 == 0 && a->Wo % 32 == 0 && p.vec && !p.c_f32 &&
         ((uintptr_t)p.C & 15) == 0 && p.ldc % 8 == 0 && (!p.R || (((uintptr_t)p.R & 15) == 0 && p.ldr % 8 == 0)) &&
         (!p.bias || ((uintptr_t)p.bias & 15) == 0) && (!gn || a->Cin <= 256);
}

// Streaming 1×1 conv (conv1x1.hip) for a dense 1×1 conv with a plain bias epilogue; RDMI_CONV1X1=0
// keeps the GEMM engines (A/B; bitwise the same outputs)
bool conv1x1_ok(const GemmP& p) {
  const char* e = getenv("RDMI_CONV1X1");
  if (e && e[0] == '0') return false;
  return !p.R && !p.rowbias && !p.gnp && p.vec && ((uintptr_t)p.C & 15) == 0 && p.ldc % 8 == 0 && p.ldw % 8 == 0 &&
         (!p.bias || ((uintptr_t)p.bias & 15) == 0);
}

}  // namespace

extern "C" int rdmi_conv2d_in_gn_supported(const rdmi_conv_args* a) {
  return a && a->dtype == RDMI_F16 && halo_eligible(a, halo_mode()) && in_gn_ok(a) ? 1 : 0;
}

extern "C" int rdmi_gemm(const rdmi_gemm_args* a, void* stream) {
  RDMI_REQUIRE(a && a->A && a->W && a->C, RDMI_E_ARG, "gemm: null pointer");
  RDMI_REQUIRE(a->M > 0 && a->N > 0 && a->K > 0 && a->batch > 0, RDMI_E_ARG, "gemm: bad sizes M=%d N=%d K=%d", a->M, a->N, a->K);
  RDMI_REQUIRE(a->dtype == RDMI_F16 || a->dtype == RDMI_F32 || a->dtype == RDMI_F32_X3 || a->dtype == RDMI_F32_X6,
               RDMI_E_UNSUPPORTED, "gemm: dtype %d", a->dtype);
  if (a->dtype != RDMI_F16) return rdmi::gemm_f32(a, stream);
  RDMI_REQUIRE(a->K % 8 == 0 && a->lda % 8 == 0 && a->ldw % 8 == 0 && a->ldw >= a->K,
               RDMI_E_ALIGN, "gemm: K (%d), lda (%ld) must be multiples of 8 and ldw (%ld) >= K", a->K, a->lda, a->ldw);
  RDMI_REQUIRE(al16(a->A) && al16(a->W) && a->strideA % 8 == 0 && a->strideW % 8 == 0, RDMI_E_ALIGN, "gemm: A/W not 16-byte aligned");
  RDMI_REQUIRE(a->epilogue != RDMI_EPI_GEGLU || a->N % 128 == 0, RDMI_E_ARG, "gemm: GEGLU needs N %% 128 == 0");
  RDMI_REQUIRE(!a->rowbias || a->rows_per_group > 0, RDMI_E_ARG, "gemm: rowbias needs rows_per_group");
  RDMI_REQUIRE((long)a->M * a->lda < (1L << 30) && (long)a->N * a->ldw < (1L << 30), RDMI_E_ARG,
               "gemm: operand exceeds 2^30 elements (2 GiB) per batch");
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
  p.vec = vec_ok(p);
  RDMI_REQUIRE(!p.geglu || p.vec, RDMI_E_ALIGN, "gemm: GEGLU output needs 4-element aligned rows");
  p.gnp = a->gn_part; p.gn_ld = a->gn_ld;
  RDMI_REQUIRE(!p.gnp || (a->batch == 1 && !p.c_f32 && !p.geglu && p.vec && a->N % 4 == 0 && a->M % 32 == 0 &&
                          ((uintptr_t)p.gnp & 7) == 0 && p.gn_ld >= 2L * (a->M / 32)),
               RDMI_E_ARG, "gemm: GroupNorm moments need batch 1, f16 vector output, N %% 4 == 0, M %% 32 == 0");
  p.a_bytes = (unsigned)(((long)(a->M - 1) * a->lda + a->K) * 2);
  p.w_bytes = (unsigned)(((long)(a->N - 1) * a->ldw + a->K) * 2);
  return launch(p, a->batch, (hipStream_t)stream, p.geglu, 0);
}

extern "C" int rdmi_conv2d(const rdmi_conv_args* a, void* stream) {
  RDMI_REQUIRE(a && a->x && a->w && a->y, RDMI_E_ARG, "conv2d: null pointer");
  RDMI_REQUIRE(a->B > 0 && a->H > 0 && a->W > 0 && a->Cout > 0 && a->Ho > 0 && a->Wo > 0, RDMI_E_ARG, "conv2d: bad sizes");
  RDMI_REQUIRE(a->dtype == RDMI_F16 || a->dtype == RDMI_F32 || a->dtype == RDMI_F32_X3 || a->dtype == RDMI_F32_X6,
               RDMI_E_UNSUPPORTED, "conv2d: dtype %d", a->dtype);
  if (a->dtype != RDMI_F16) return rdmi::conv2d_f32(a, stream);
  RDMI_REQUIRE(a->Cin % 8 == 0, RDMI_E_ALIGN, "conv2d: Cin (%d) must be a multiple of 8", a->Cin);
  const int K = a->kh * a->kw * a->Cin;
  RDMI_REQUIRE(a->Kp >= K && a->Kp % 8 == 0, RDMI_E_ARG, "conv2d: Kp (%d) must be >= %d and a multiple of 8", a->Kp, K);
  RDMI_REQUIRE(al16(a->x) && al16(a->w), RDMI_E_ALIGN, "conv2d: x/w not 16-byte aligned");
  RDMI_REQUIRE((long)a->B * a->H * a->W * a->Cin < (1L << 30) && (long)a->Cout * a->Kp < (1L << 30), RDMI_E_ARG,
               "conv2d: input exceeds 2^30 elements (2 GiB; split the batch)");
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
  p.cmaj = a->kh * a->kw > 1 && a->Cin % 64 == 0;
  // a 1×1, stride-1, unpadded conv on NHWC is a dense GEMM over pixels (conv_shortcut, quant convs)
  const bool dense = a->kh == 1 && a->kw == 1 && a->stride == 1 && a->pad_top == 0 && a->pad_left == 0 && !a->upsample &&
                     a->Ho == a->H && a->Wo == a->W;
  if (dense) p.lda = a->Cin;
  RDMI_REQUIRE(dense || (a->kh == 3 && a->kw == 3), RDMI_E_UNSUPPORTED, "conv2d: only 3x3 and dense 1x1 kernels");
  RDMI_REQUIRE(!a->upsample || a->stride == 1, RDMI_E_UNSUPPORTED, "conv2d: upsample needs stride 1");
  p.vec = vec_ok(p);
  p.gnp = a->gn_part; p.gn_ld = a->gn_ld;
  RDMI_REQUIRE(!p.gnp || (p.vec && a->Cout % 4 == 0 && p.M % 32 == 0 && ((uintptr_t)p.gnp & 7) == 0 &&
                          p.gn_ld >= 2L * (p.M / 32)),
               RDMI_E_ARG, "conv2d: GroupNorm moments need vector output, Cout %% 4 == 0, B*Ho*Wo %% 32 == 0");
  p.a_bytes = (unsigned)((long)a->B * a->H * a->W * a->Cin * 2);
  p.w_bytes = (unsigned)((long)a->Cout * a->Kp * 2);
  const int hmode = halo_mode();
  RDMI_REQUIRE(!a->in_mean_rstd || (a->in_gamma && a->in_beta), RDMI_E_ARG, "conv2d: input GroupNorm needs gamma and beta");
  RDMI_REQUIRE(!a->in_mean_rstd || (halo_eligible(a, hmode) && in_gn_ok(a)), RDMI_E_UNSUPPORTED,
               "conv2d: input GroupNorm not supported for this shape (rdmi_conv2d_in_gn_supported)");
  if (halo_eligible(a, hmode)) {
    const char* gm = getenv("RDMI_GEMM_GROUP");
    p.group_m = gm ? atoi(gm) : 8;
    const char* nx = getenv("RDMI_CONV_NXCD");  // n-tile per XCD in the two-workgroups-per-CU engine (A/B)
    if (nx && nx[0] == '1') p.group_m = -1;
    const char* cpp = getenv("RDMI_CONV_PIPE");
    p.conv_pipe = !cpp || cpp[0] != '0';
    const char* hpf = getenv("RDMI_HALO_PREF");  // opt-in A/B: L2 prefetch of the next channel block's halo
    p.halo_pref = hpf && hpf[0] == '1';
    // the GroupNorm halo transform at s_setprio 2 (its refill is the workgroup's critical path; the partner's
    // MFMA issue waits): bitwise the same, pipeline −0.3 % in 5 of 5 interleaved rounds
    // (profiles/r06zc_xprio_pipe_ab.log); RDMI_XFORM_PRIO=0 restores the flat priority (A/B)
    const char* xp = getenv("RDMI_XFORM_PRIO");
    p.xprio = !(xp && xp[0] == '0');
    const char* ep = getenv("RDMI_EPI_PRIO");  // opt-in A/B: the halo conv's epilogue at s_setprio 2
    p.eprio = ep && ep[0] == '1';
    const char* cp = getenv("RDMI_CPERM");
    p.cperm = (!cp || cp[0] != '0') && p.vec && ((uintptr_t)p.C & 15) == 0 && p.ldc % 8 == 0 &&
              (!p.R || (((uintptr_t)p.R & 15) == 0 && p.ldr % 8 == 0));
    p.gmr = a->in_mean_rstd; p.ggam = a->in_gamma; p.gbet = a->in_beta; p.gG = a->in_groups; p.gsilu = a->in_silu;
    p.gaff = a->in_mean_rstd ? a->in_affine : nullptr;
    RDMI_REQUIRE(!p.gaff || ((uintptr_t)p.gaff & 15) == 0, RDMI_E_ALIGN, "conv2d: in_affine not 16-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    const unsigned patches = (unsigned)((a->Ho / 16) * (a->Wo / 16) * a->B);
    const bool gn = p.gmr != nullptr;
    if (a->upsample && a->w_up2 && !gn && a->Ho % 32 == 0 && a->Wo % 32 == 0 && al16(a->w_up2)) {
      // phase-decomposed ×2 upsample conv: 4 hi + 3 lo taps per phase (conv_halo_occ2_kernel MODE 3)
      p.Wt = (const f16*)a->w_up2; p.ldw = 7L * a->Cin; p.K = p.Kvalid = 7 * a->Cin;
      p.w_bytes = (unsigned)(4L * a->Cout * p.ldw * 2);
      launch_conv_occ2(3, false, p.conv_pipe != 0, dim3((a->Cout + 127) / 128, patches, 1), st, p);
    } else if (a->Cout % 256 == 0 && !p.gaff && !(hmode == 3 && (!gn || a->Cin <= 256))) {
      dim3 g(a->Cout / 256, patches, 1);
      const bool ph2 = hmode != 1 || gn;  // 2 phases per K-tile: +5-8 % over 4 (tools/kbench.py)
      if (a->upsample) {
        launch_conv_halo(2, ph2 ? 2 : 4, 4, ph2 && gn, g, st, p);
      } else {
        launch_conv_halo(1, ph2 ? 2 : 4, 4, ph2 && gn, g, st, p);
      }
    } else if (a->Cout == 128 && !p.gaff && (hmode == 4 || (gn && a->Cin > 256))) {  // the 8-wave 128-channel variant
      dim3 g(1, patches, 1);
      launch_conv_halo(a->upsample ? 2 : 1, 1, 2, gn, g, st, p);
    } else if (h32_ok(a, p, gn)) {  // 32×32×16 MFMA form on 32×8 patches (GN: Cin ≤ 256, its own LDS table)
      dim3 g(a->Cout / 128, (unsigned)((a->Ho / 8) * (a->Wo / 32) * a->B), 1);
      launch_conv_h32(gn, g, st, p);
    } else {  // two workgroups per CU (RDMI_CONV_HALO=3: also for Cout % 256 == 0)
      dim3 g((a->Cout + 127) / 128, patches, 1);
      launch_conv_occ2(a->upsample ? 2 : 1, gn, p.conv_pipe != 0, g, st, p);
    }
    return rdmi::check_launch("conv2d halo");
  }
  if (dense && conv1x1_ok(p) && launch_conv1x1(p, a->Cin, a->Cout, (hipStream_t)stream))
    return rdmi::check_launch("conv2d 1x1");
  return launch(p, 1, (hipStream_t)stream, false, dense ? 0 : (a->upsample ? 2 : 1));
}


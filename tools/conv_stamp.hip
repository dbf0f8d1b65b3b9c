// Diagnostic: where conv_halo_occ2_kernel's cycles go, by segment (guide cdna_hip_programming.md §7
// 'In-kernel stamps').  Builds the kernel from rollingdepth_amd/csrc/gemm_kernels.h with STAMP = 1 (the
// product library never instantiates it) and runs it on random data at the pipeline's heaviest
// 128-channel shape: 768² 128 → 128, B images, GroupNorm+SiLU input, residual and GroupNorm moments
// out (the VAE ResnetBlock2D conv2).  Read the SHARES, not the stamped build's run time.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/conv_stamp.hip -o tools/conv_stamp
//   ./tools/conv_stamp [B] [HW] [gn res moments: 0/1 each] [Cin] [Cout] [residual row stride] [gaff 0/1]
// Cout = 128: conv_halo_occ2_kernel; Cout % 256 == 0: conv_halo_kernel<1, 2, 4, GN> (8 waves, ping-pong).
// gaff = 1: the GroupNorm scale / shift from the per-(image, channel block) table in global memory
// (rdmi_conv_args.in_affine, the pipeline's default), any Cout on conv_halo_occ2_kernel — the dispatch
// rdmi_conv2d makes for every in_affine conv.
#include "../rollingdepth_amd/csrc/gemm_kernels.h"

#include <algorithm>
#include <vector>

using namespace rdmi_gk;

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                               \
    }                                                         \
  } while (0)

__global__ void fill_h(f16* x, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    const float u = ((h & 255) + ((h >> 8) & 255) + ((h >> 16) & 255) + (h >> 24)) / 255.f - 2.f;
    x[i] = (f16)(u * scale);
  }
}
__global__ void fill_f(float* x, long n, float a, float b) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = (i & 1) ? b : a;
}

template <int ST>
void launch(dim3 g, const GemmP& p, bool wide) {
  if (wide) {
    if (p.gmr)
      hipLaunchKernelGGL((conv_halo_kernel<1, 2, 4, true, ST>), g, dim3(512), 0, 0, p);
    else
      hipLaunchKernelGGL((conv_halo_kernel<1, 2, 4, false, ST>), g, dim3(512), 0, 0, p);
  } else if (p.gmr) {
    hipLaunchKernelGGL((conv_halo_occ2_kernel<1, true, true, ST>), g, dim3(256), 0, 0, p);
  } else {
    hipLaunchKernelGGL((conv_halo_occ2_kernel<1, false, true, ST>), g, dim3(256), 0, 0, p);
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8, HW = argc > 2 ? atoi(argv[2]) : 768;
  const bool gn = argc > 3 ? atoi(argv[3]) : 1, res = argc > 4 ? atoi(argv[4]) : 1, mom = argc > 5 ? atoi(argv[5]) : 1;
  const int Cin = argc > 6 ? atoi(argv[6]) : 128, Cout = argc > 7 ? atoi(argv[7]) : 128, Kp = 9 * Cin, G = 32;
  const int rld = argc > 8 ? atoi(argv[8]) : Cout;  // residual row stride (0: every row reads one cached row)
  const bool gaff = gn && argc > 9 && atoi(argv[9]) != 0;
  const bool wide = Cout % 256 == 0 && !gaff;
  const int WPG = wide ? 8 : 4;  // waves per workgroup
  const long M = (long)B * HW * HW;
  f16 *x, *w, *y, *r;
  float *gmr, *gam, *bet, *gnp;
  CK(hipMalloc(&x, M * Cin * 2)); CK(hipMalloc(&w, (long)Cout * Kp * 2));
  CK(hipMalloc(&y, M * Cout * 2)); CK(hipMalloc(&r, M * Cout * 2));
  CK(hipMalloc(&gmr, B * G * 2 * 4)); CK(hipMalloc(&gam, Cin * 4)); CK(hipMalloc(&bet, Cin * 4));
  const long gn_ld = 2 * (M / 32);
  CK(hipMalloc(&gnp, (Cout / 4) * gn_ld * 4));
  hipLaunchKernelGGL(fill_h, dim3(4096), dim3(256), 0, 0, x, M * Cin, 1u, 1.0f);
  hipLaunchKernelGGL(fill_h, dim3(4096), dim3(256), 0, 0, w, (long)Cout * Kp, 2u, 0.03f);
  hipLaunchKernelGGL(fill_h, dim3(4096), dim3(256), 0, 0, r, M * Cout, 3u, 1.0f);
  hipLaunchKernelGGL(fill_f, dim3(64), dim3(256), 0, 0, gmr, (long)B * G * 2, 0.1f, 1.2f);
  hipLaunchKernelGGL(fill_f, dim3(1), dim3(256), 0, 0, gam, (long)Cin, 1.0f, 0.9f);
  hipLaunchKernelGGL(fill_f, dim3(1), dim3(256), 0, 0, bet, (long)Cin, 0.05f, -0.05f);
  GemmP p{};
  p.A = x; p.Wt = w; p.ldw = Kp; p.C = y; p.ldc = Cout; p.alpha = 1.f;
  p.R = res ? r : nullptr; p.ldr = rld; p.rpg = HW * HW;
  p.M = (int)M; p.N = Cout; p.K = Kp; p.Kvalid = Kp;
  p.IH = HW; p.IW = HW; p.Cin = Cin; p.Ho = HW; p.Wo = HW; p.kh = 3; p.kw = 3; p.stride = 1; p.pt = 1; p.pl = 1;
  p.cin_vecs = Cin / 8; p.cmaj = 1; p.vec = 1;
  p.gnp = mom ? gnp : nullptr; p.gn_ld = gn_ld;
  p.a_bytes = (unsigned)(M * Cin * 2); p.w_bytes = (unsigned)((long)Cout * Kp * 2);
  p.group_m = 8; p.cperm = 1; p.conv_pipe = 1;
  if (gn) { p.gmr = gmr; p.ggam = gam; p.gbet = bet; p.gG = G; p.gsilu = 1; }
  if (gaff) {  // [B][Cin/64][64 scales | 64 shifts]
    float* tab;
    const long nt = (long)B * (Cin / 64) * 128;
    CK(hipMalloc(&tab, nt * 4));
    hipLaunchKernelGGL(fill_f, dim3(64), dim3(256), 0, 0, tab, nt, 0.9f, 0.05f);
    p.gaff = tab;
  }
  const dim3 g(wide ? Cout / 256 : (Cout + 127) / 128, (unsigned)((HW / 16) * (HW / 16) * B), 1);
  const long nw = (long)g.x * g.y * WPG;
  unsigned long long* st;
  CK(hipMalloc(&st, nw * 8 * 8));
  p.stamps = st;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double fl = 2.0 * M * Cout * Kp;
  printf("conv 3x3 %d->%d %dx%d B=%d gn=%d%s res=%d moments=%d: %u workgroups, %.1f GFLOP\n", Cin, Cout, HW, HW, B,
         gn, gaff ? " (in_affine table)" : "", res, mom, g.x * g.y, fl / 1e9);
  for (int variant = 0; variant < 2; ++variant) {
    float best = 1e30f;
    for (int rep = 0; rep < 8; ++rep) {
      CK(hipEventRecord(e0, 0));
      if (variant == 0) launch<0>(g, p, wide); else launch<1>(g, p, wide);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    CK(hipGetLastError());
    std::vector<unsigned short> yh(M * Cout);
    CK(hipMemcpy(yh.data(), y, M * Cout * 2, hipMemcpyDeviceToHost));
    unsigned long long hsh = 1469598103934665603ull;  // FNV-1a of the output bits (A/B: bitwise equality)
    for (unsigned short v : yh) hsh = (hsh ^ v) * 1099511628211ull;
    printf("%s: %.3f ms  %.1f TF/s  output fnv %016llx\n", variant ? "stamped" : "product", best, fl / best / 1e9, hsh);
  }
  std::vector<unsigned long long> h(nw * 8);
  CK(hipMemcpy(h.data(), st, nw * 8 * 8, hipMemcpyDeviceToHost));
  const char* occ2_names[6] = {"prologue", "K-tile wait+barrier", "reads+MFMA issue", "halo refill", "epilogue", "total"};
  const char* wide_names[8] = {"prologue", "load sections", "barrier before MFMA", "MFMA issue", "GroupNorm transform",
                               "barrier after", "epilogue", "total"};
  const int ns = wide ? 8 : 6, tot = ns - 1;
  double sum[8] = {};
  for (long i = 0; i < nw; ++i)
    for (int s = 0; s < ns; ++s) sum[s] += (double)h[i * 8 + s];
  printf("per wave (mean s_memtime ticks, %ld waves):\n", nw);
  for (int s = 0; s < ns; ++s)
    printf("  %-22s %10.0f  %5.1f %%\n", wide ? wide_names[s] : occ2_names[s], sum[s] / nw, 100.0 * sum[s] / sum[tot]);
  printf("  (one wave's MFMA work: %d K-tiles x 64 16x16x32 MFMAs x 16 cycles = %d cycles)\n", Kp / 64, Kp / 64 * 1024);
  return 0;
}

// Diagnostic: where attn_fwd_d64's cycles go, by segment (guide cdna_hip_programming.md §7 'In-kernel
// stamps').  Builds the kernel from rollingdepth_amd/csrc/attention.hip with STAMP = 1 (the product
// library never instantiates it) and runs it on random data at the pipeline's L0 shape.  Read the
// SHARES, not the stamped build's run time (its stamps fence overlaps the real kernel has).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/attn_stamp.hip -o tools/attn_stamp
//   ./tools/attn_stamp [B] [S]
#include "../rollingdepth_amd/csrc/attention.hip"

#include <vector>

namespace rdmi {
void set_error(const char*, ...) {}
int check_launch(const char*) { return (int)hipGetLastError(); }
int attention_fwd_f32(const void*, const void*, const void*, void*, int, int, int, int, long, long, long, long, long,
                      long, long, long, float, bool, void*) {
  return -1;
}
}  // namespace rdmi

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

__global__ void fill_k(f16* x, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    // approx N(0,1) from the sum of 4 uniform bytes
    float u = ((h & 255) + ((h >> 8) & 255) + ((h >> 16) & 255) + (h >> 24)) / 255.f - 2.f;
    x[i] = (f16)(u * 1.7f);
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8, S = argc > 2 ? atoi(argv[2]) : 27648, H = 5, D = 64;
  const long n = (long)B * S * H * D;
  f16 *q, *k, *v, *o;
  CK(hipMalloc(&q, n * 2)); CK(hipMalloc(&k, n * 2)); CK(hipMalloc(&v, n * 2)); CK(hipMalloc(&o, n * 2));
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, q, n, 1u);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, k, n, 2u);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, v, n, 3u);
  const long ld = (long)H * D, bs = (long)S * ld;
  AttnP p{q, k, v, o, H, S, S, ld, ld, ld, ld, bs, bs, bs, bs, 0.125f * 1.4426950408889634f, nullptr};
  dim3 g(rdmi::div_up(S, QB), H, B);
  const long nw = (long)g.x * g.y * g.z * NWV;
  unsigned long long* st;
  CK(hipMalloc(&st, nw * 6 * 8));
  p.stamps = st;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double fl = 4.0 * S * (double)S * D * H * B;
  for (int variant = 0; variant < 2; ++variant) {
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(e0, 0));
      if (variant == 0)
        hipLaunchKernelGGL((attn_fwd_d64<true, 0>), g, dim3(64 * NWV), 0, 0, p);
      else
        hipLaunchKernelGGL((attn_fwd_d64<true, 1>), g, dim3(64 * NWV), 0, 0, p);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%s build: %.3f ms  %.1f TF/s (B=%d H=%d S=%d)\n", variant ? "STAMP" : "plain", best, fl / best / 1e9, B, H, S);
  }
  // the one-wave-per-SIMD pipeline (attn_fwd_d64_pipe): timing and max |Δ| against attn_fwd_d64
  {
    f16* o2;
    CK(hipMalloc(&o2, n * 2));
    AttnP p2 = p;
    p2.o = o2;
    dim3 g2(rdmi::div_up(S, pp::QB), H, B);
    // extra dynamic LDS forces one workgroup per CU (one wave per SIMD) for the A/B
    const size_t xl = getenv("PIPE_1WG") ? 80 * 1024 : 0;
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((attn_fwd_d64_pipe<0>), g2, dim3(64 * pp::NW), xl, 0, p2);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    hipLaunchKernelGGL((attn_fwd_d64<true, 0>), g, dim3(64 * NWV), 0, 0, p);
    CK(hipDeviceSynchronize());
    std::vector<f16> a(n), c2(n);
    CK(hipMemcpy(a.data(), o, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c2.data(), o2, n * 2, hipMemcpyDeviceToHost));
    double md = 0, ma = 0;
    long bad = 0;
    for (long i = 0; i < n; ++i) {
      const double x = (double)(float)a[i], y = (double)(float)c2[i];
      if (!(y == y)) ++bad;
      md = fmax(md, fabs(x - y));
      ma = fmax(ma, fabs(x));
    }
    printf("pipe%s build: %.3f ms  %.1f TF/s   max |pipe - d64| %.3e (max |O| %.3f, non-finite %ld)\n", xl ? "(1wg)" : "", best,
           fl / best / 1e9, md, ma, bad);
  }
  std::vector<unsigned long long> h(nw * 6);
  CK(hipMemcpy(h.data(), st, nw * 6 * 8, hipMemcpyDeviceToHost));
  const char* names[6] = {"MFMA block (PV t-1, QK t)", "barrier after MFMA block", "softmax block", "DMA wait + barrier",
                          "prologue", "epilogue"};
  for (int grp = 0; grp < 2; ++grp) {
    double sum[6] = {}, tot = 0;
    long cnt = 0;
    for (long w = 0; w < nw; ++w) {
      if (((w % NWV) >> 2) != grp) continue;
      for (int i = 0; i < 6; ++i) sum[i] += (double)h[w * 6 + i];
      ++cnt;
    }
    for (int i = 0; i < 6; ++i) tot += sum[i];
    const int nt = (S + KB - 1) / KB;
    printf("waves %d-%d (%ld waves, %d tiles each): %.0f cycles per wave\n", 4 * grp, 4 * grp + 3, cnt, nt, tot / cnt);
    for (int i = 0; i < 6; ++i)
      printf("  %-28s %10.0f cyc/wave  %6.1f cyc/tile  %5.1f %%\n", names[i], sum[i] / cnt, sum[i] / cnt / nt,
             100.0 * sum[i] / tot);
  }
  return 0;
}

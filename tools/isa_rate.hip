// Issue-rate probe for the softmax's VALU instructions on gfx950 (one wave per SIMD, 16 independent
// instructions per unrolled group, s_memtime around the loop): cycles per wave-instruction.
//   hipcc -O3 --offload-arch=gfx950 tools/isa_rate.hip -o tools/isa_rate && ./tools/isa_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP16(X) X X X X X X X X X X X X X X X X

template <int OP>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc, int iters) {
  float a0 = threadIdx.x * 1e-3f - 1.f, a1 = a0 * 0.5f, a2 = a0 * 0.25f, a3 = a0 * 0.125f;
  float a4 = a0 + 0.1f, a5 = a1 + 0.1f, a6 = a2 + 0.1f, a7 = a3 + 0.1f;
  long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; ++i) {
    if (OP == 0) {  // v_exp_f32
      asm volatile(REP16("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    } else if (OP == 1) {  // v_exp_f16 (low half)
      asm volatile(REP16("v_exp_f16 %0, %0\n v_exp_f16 %1, %1\n v_exp_f16 %2, %2\n v_exp_f16 %3, %3\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    } else if (OP == 2) {  // v_exp_f16 SDWA into the high half
      asm volatile(REP16(
                       "v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
                       "v_exp_f16_sdwa %1, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
                       "v_exp_f16_sdwa %2, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
                       "v_exp_f16_sdwa %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    } else if (OP == 3) {  // v_cvt_pk_f16_f32
      asm volatile(REP16("v_cvt_pk_f16_f32 %0, %4, %5\n v_cvt_pk_f16_f32 %1, %5, %6\n"
                         "v_cvt_pk_f16_f32 %2, %6, %7\n v_cvt_pk_f16_f32 %3, %7, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    } else if (OP == 4) {  // v_pk_add_f16
      asm volatile(REP16("v_pk_add_f16 %0, %0, %4\n v_pk_add_f16 %1, %1, %5\n v_pk_add_f16 %2, %2, %6\n"
                         "v_pk_add_f16 %3, %3, %7\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    } else if (OP == 5) {  // v_add_f32
      asm volatile(REP16("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %5\n v_add_f32 %2, %2, %6\n"
                         "v_add_f32 %3, %3, %7\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    } else if (OP == 7) {  // v_pk_fma_f16 (two f16 FMAs per lane: a polynomial exp2 would be built of these)
      asm volatile(REP16("v_pk_fma_f16 %0, %0, %4, %5\n v_pk_fma_f16 %1, %1, %5, %6\n v_pk_fma_f16 %2, %2, %6, %7\n"
                         "v_pk_fma_f16 %3, %3, %7, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    } else if (OP == 8) {  // v_fma_f32
      asm volatile(REP16("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %5, %6\n v_fma_f32 %2, %2, %6, %7\n"
                         "v_fma_f32 %3, %3, %7, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    } else if (OP == 9) {  // v_exp_f32 / v_add_f32 alternating on independent registers: do they overlap?
      asm volatile(REP16("v_exp_f32 %0, %0\n v_add_f32 %1, %1, %4\n v_exp_f32 %2, %2\n v_add_f32 %3, %3, %5\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5));
    } else if (OP == 10) {  // v_pk_fma_f32 (packed f32 pairs: 64-bit register pairs)
      double d0 = a0, d1 = a1, d2 = a2, d3 = a3, e0 = a4, e1 = a5;
      asm volatile(REP16("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %5, %4\n v_pk_fma_f32 %2, %2, %4, %5\n"
                         "v_pk_fma_f32 %3, %3, %5, %4\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(e0), "v"(e1));
      a0 = (float)(d0 + d1);
      a1 = (float)(d2 + d3);
    } else if (OP == 11) {  // v_exp_f32 / v_pk_fma_f16 alternating on independent registers
      asm volatile(REP16("v_exp_f32 %0, %0\n v_pk_fma_f16 %1, %1, %4, %5\n v_exp_f32 %2, %2\n v_pk_fma_f16 %3, %3, %5, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(a5));
    } else if (OP == 6) {  // v_exp_f16 lo + SDWA hi pairs (the packed-P form)
      asm volatile(REP16("v_exp_f16 %0, %4\n v_exp_f16_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n"
                         "v_exp_f16 %1, %5\n v_exp_f16_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n")
                   : "+v"(a0), "+v"(a1) : "v"(a4), "v"(a5));
    }
  }
  long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(const char* name, float* out, long long* cyc, int blocks) {
  const int iters = 2000;
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  long long h[1024];
  hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks; ++i) s += (double)h[i];
  const double per = s / blocks / (iters * 64.0);
  printf("%-28s %6.2f cycles per wave-instruction (s_memtime ticks)\n", name, per);
}

int main() {
  float* out;
  long long* cyc;
  const int blocks = 256;  // 4 waves per CU = one per SIMD
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipMalloc(&cyc, 1024 * sizeof(long long));
  run<0>("v_exp_f32", out, cyc, blocks);
  run<1>("v_exp_f16", out, cyc, blocks);
  run<2>("v_exp_f16_sdwa (hi)", out, cyc, blocks);
  run<6>("v_exp_f16 lo + sdwa hi", out, cyc, blocks);
  run<3>("v_cvt_pk_f16_f32", out, cyc, blocks);
  run<4>("v_pk_add_f16", out, cyc, blocks);
  run<5>("v_add_f32", out, cyc, blocks);
  run<8>("v_fma_f32", out, cyc, blocks);
  run<7>("v_pk_fma_f16", out, cyc, blocks);
  run<10>("v_pk_fma_f32", out, cyc, blocks);
  run<9>("v_exp_f32 + v_add_f32 alt", out, cyc, blocks);
  run<11>("v_exp_f32 + v_pk_fma_f16 alt", out, cyc, blocks);
  return 0;
}

/* rdmi.h — C ABI of librdmi.so, the MI355X (gfx950) HIP kernels of RollingDepth's
 * snippet-denoise hot path.
 *
 * The reference (yizuo417/RollingDepth) has no native code and no FFI: its hot path is implicit
 * PyTorch library kernels issued from Python.  Each entry point below
 * replaces one such implicit op (or a fused group of them) and names the reference call site it
 * stands in for.  The Python host package `rollingdepth_amd` binds these through ctypes
 * (INTEGRATION.md shows the binding a maintainer of the reference would add).
 *
 * Conventions:
 *  - plain pointers (device memory owned by the caller), sizes and strides in ELEMENTS, and a
 *    hipStream_t passed as `void*` (0 = the null stream);
 *  - activations are NHWC / token-major [B, S, C]; f16 storage with f32 accumulation unless a
 *    parameter says otherwise; norm affine parameters and biases are f32;
 *  - every call returns 0 or an error code (RDMI_E_* for bad arguments, else the hipError_t of
 *    the launch); rdmi_last_error() returns a thread-local message; nothing synchronises the
 *    device, allocates, frees, or retains a pointer after return, so every call is graph-capturable.
 */
#ifndef RDMI_H
#define RDMI_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RDMI_OK 0
#define RDMI_E_ARG 1001         /* bad shape / stride / null pointer */
#define RDMI_E_ALIGN 1002       /* pointer or leading dimension not 16-byte aligned */
#define RDMI_E_UNSUPPORTED 1003 /* configuration this build does not implement */

/* storage dtype codes of the `dtype` arguments (f32 is the paper preset's arithmetic, run_video.py:444-449) */
#define RDMI_F16 0
#define RDMI_F32 1
#define RDMI_U8 2 /* decoded video frames (rdmi_resize input) */
/* rdmi_gemm / rdmi_conv2d only: f32 activations and output, weights pre-split into bf16 hi/lo parts,
 * products a_hi·w_hi + a_hi·w_lo + a_lo·w_hi on the bf16 MFMA with f32 accumulation (≈2^-16 relative
 * error per product; the paper preset's fast f32 engine, RDMI_F32_X3=1 in rollingdepth_amd) */
#define RDMI_F32_X3 3
/* rdmi_attention_fwd (round 5): f32 q/k/v/o and softmax, both products on the bf16 MFMA over a three-way
 * bf16 split of each f32 operand (hi + mid + lo, six partial products kept): a few 2^-24 relative per
 * product — f32's own product rounding, the reference's exact-fp32 SDPA precision — at ≈0.4 of the
 * exact f32-input MFMA's matrix time */
#define RDMI_F32_X6 4

/* rdmi_resize modes: torchvision InterpolationMode NEAREST / BILINEAR / BICUBIC */
#define RDMI_RESIZE_NEAREST 0
#define RDMI_RESIZE_BILINEAR 1
#define RDMI_RESIZE_BICUBIC 2

#define RDMI_EPI_NONE 0
#define RDMI_EPI_GEGLU 1 /* out[:, n] = (h + b_h) * gelu_erf(g + b_g), weights row-interleaved */
#define RDMI_EPI_SILU 2  /* out = silu(acc·alpha + bias ...) (TimestepEmbedding act, embeddings.py:543) */

/* ---------------------------------------------------------------------------------------
 * Library
 */
const char* rdmi_last_error(void);
int rdmi_version(void);

/* ---------------------------------------------------------------------------------------
 * GEMM (Linear layers): C[b] = alpha * A[b] · W[b]ᵀ (+ bias[n]) (+ rowbias[m / rows_per_group][n])
 *                                                     (+ residual[b][m][n])
 * A [M, K] f16 (lda), W [N, K] f16 (ldw ≥ K), K % 8 == 0, C f16 or f32 (ldc).
 * Replaces torch.nn.Linear / F.linear in Attention.to_q/k/v/to_out
 * (diffusers/models/attention_processor.py:2226-2261), FeedForward/GEGLU
 * (diffusers/models/attention.py:1116, activations.py:113-123), Transformer2DModel.proj_in/out
 * (transformers/transformer_2d.py:485-533) and TimestepEmbedding (embeddings.py:543).
 */
typedef struct rdmi_gemm_args {
  const void* A; long lda; long strideA;
  const void* W; long ldw; long strideW;
  void* C; long ldc; long strideC; int c_f32;
  const float* bias;
  const void* residual; long ldr; long strideR;
  const float* rowbias; int rows_per_group; long rowbias_ld;
  float alpha;
  int M, N, K, batch;
  int epilogue;
  /* optional GroupNorm moments of the f16 output (batch == 1, f16 C, N % 4 == 0, M % 32 == 0):
   * gn_part[v * gn_ld + 2*r + {0,1}] = (Σ, Σ²) over output rows 32r..32r+31 and channels
   * 4v..4v+3, summed in a fixed order (rdmi_groupnorm_stats_partials consumes them).  NULL: off. */
  float* gn_part; long gn_ld;
  /* storage dtype of A, W, C and residual: RDMI_F16 (f16 MFMA, f32 accumulate; C f32 when c_f32) or
   * RDMI_F32 (the paper preset: f32-input MFMA v_mfma_f32_16x16x4_f32, exact f32 products, C / residual
   * f32; K % 4 == 0; no GroupNorm moments) or RDMI_F32_X3 (as RDMI_F32, W the bf16 split layout:
   * row n holds, per 32-deep K-tile t, bf16(w[n, 32t..32t+31]) then bf16(w − that), so ldw / strideW
   * count bf16 elements, ldw % 64 == 0 and ldw ≥ 2·ceil(K/32)·32) */
  int dtype;
} rdmi_gemm_args;
int rdmi_gemm(const rdmi_gemm_args* args, void* stream);

/* ---------------------------------------------------------------------------------------
 * Convolution as implicit GEMM on NHWC f16 (MFMA 16x16x32 f16, f32 accumulate).
 * y[b, ho, wo, co] = alpha * Σ w[co, dy, dx, ci] x[b, ho*s - pt + dy, wo*s - pl + dx, ci]
 *                    (+ bias[co]) (+ rowbias[b * rowbias_ld + co]) (+ residual[b, ho, wo, co])
 * `upsample`=1 reads x through a nearest ×2 upsample (Upsample2D, upsampling.py:141-190) without
 * materialising it.  Cin % 8 == 0 (pad channels).  Weight layout, zero padded to Kp % 32 == 0:
 *   kh*kw > 1 and Cin % 64 == 0: [Cout][Cin/64][kh][kw][64] (channel-block major: one K-tile of 64
 *     is one tap of a 64-channel block, i.e. one full 128-B line per output pixel, and the taps of
 *     a block are adjacent in K, so the implicit-im2col re-reads of a block hit L2);
 *   otherwise:                    [Cout][kh][kw][Cin].
 * Replaces the cuDNN conv2d of ResnetBlock2D.conv1/conv2/conv_shortcut (resnet.py:320-373),
 * Downsample2D (downsampling.py:132-148, including the VAE's F.pad(0,1,0,1) via pad_top/left=0
 * with the extra row/column read as zero), Upsample2D.conv, conv_in/conv_out of the UNet and VAE.
 */
typedef struct rdmi_conv_args {
  const void* x; const void* w; void* y;
  const float* bias; const void* residual; const float* rowbias;
  int B, H, W, Cin, Cout, kh, kw, stride, pad_top, pad_left, upsample, Ho, Wo, Kp;
  long y_ld; long res_ld; float alpha; long rowbias_ld; /* 0: one row shared by all images */
  float* gn_part; long gn_ld; /* GroupNorm moments of y, laid out as in rdmi_gemm_args; rows = B·Ho·Wo */
  /* GroupNorm (+SiLU) of the INPUT applied as x is read (the norm1/norm2 → conv1/conv2 pairs of
   * ResnetBlock2D, resnet.py:326-352): the conv sees silu?(x·sc + sh) with sc = rstd·gamma[c],
   * sh = beta[c] − mean·sc per image b (in_mean_rstd as rdmi_groupnorm_stats writes it), the
   * padding still zero; the same values rdmi_groupnorm_apply writes.  NULL in_mean_rstd: off.
   * Shapes that support it: rdmi_conv2d_in_gn_supported (otherwise RDMI_E_UNSUPPORTED). */
  const float* in_mean_rstd; const float* in_gamma; const float* in_beta; int in_groups, in_silu;
  /* RDMI_F16 or RDMI_F32 (x, w, y, residual).  f32 weights are always [Cout][kh][kw][Cin] (tap-major,
   * Kp % 32 == 0), Cin % 4 == 0, no input GroupNorm and no GroupNorm moments.  RDMI_F32_X3: f32 x, y,
   * residual; w in the bf16 split layout that rdmi_gemm_args describes, rows of 2·Kp bf16 (Kp still counts f32 K). */
  int dtype;
  /* Optional, upsample = 1 only: the same conv's weights for the phase-decomposed form — the ×2
   * nearest upsample + 3×3 conv computed as four 2×2 convs on the source grid, one per output
   * phase (a, c) = (y & 1, x & 1), the 3×3 taps that read the same source pixel merged
   * (rows {0 | 1,2} for a = 0, {0,1 | 2} for a = 1; columns likewise).  A merged weight Σw (sum in
   * f32 of 2 or 4 f16 taps) is stored as hi = f16(Σw) and lo = f16(Σw − hi), so every product is
   * exact in the f32 accumulator: the result is the 9-tap conv's up to f32 accumulation order (and
   * lo's f16 rounding where Σw − hi is subnormal or wider than 11 bits), in 7/9 of the MFMA work.
   * Layout [4 phases (2a + c)][Cout][Cin/64][7][64] f16 (row stride 7·Cin): per 64-channel block
   * the hi parts of taps (dy, dx) = (0,0), (0,1), (1,0), (1,1), then the lo parts of those taps other
   * than (a, c) (a single 3×3 weight, exact in f16), in the same order.  Used where the halo engine
   * runs the conv (f16, Cin % 64 == 0, Ho % 32 == 0, Wo % 32 == 0, no input GroupNorm); elsewhere
   * `w` is used.  NULL: off. */
  const void* w_up2;
  /* Optional with in_mean_rstd (round 5): the input GroupNorm's per-channel scale / shift as
   * rdmi_groupnorm_affine writes them, [B][Cin/64][2][64] f32 — per image and 64-channel block the 64
   * scales sc = rstd·gamma[c], then the 64 shifts sh = beta[c] − mean·sc.  With it the
   * two-workgroups-per-CU halo engine fuses the norm for any Cin % 64 == 0 (each wave loads the block's
   * 8 + 8 values of its lanes with the halo refill); without it only for Cin ≤ 256 (the table built in
   * LDS).  The values are the ones the kernel would compute itself: bitwise the same results. */
  const float* in_affine;
} rdmi_conv_args;
int rdmi_conv2d(const rdmi_conv_args* args, void* stream);
/* 1 if rdmi_conv2d fuses an input GroupNorm for this shape (in_groups set; pointers not read) */
int rdmi_conv2d_in_gn_supported(const rdmi_conv_args* args);

/* ---------------------------------------------------------------------------------------
 * GroupNorm on NHWC f16 / f32 (dtype RDMI_F16 / RDMI_F32): statistics then apply (optionally fused SiLU).
 * Replaces F.group_norm (+ SiLU) of ResnetBlock2D.norm1/norm2 (resnet.py:326,351),
 * Transformer2DModel.norm (transformer_2d.py:175-177), conv_norm_out of UNet/VAE, and the VAE
 * mid-block Attention.group_norm (attention_processor.py:2221-2222).
 * stats: mean_rstd[b*G + g] = {mean, rstd}; workspace ≥ rdmi_groupnorm_workspace(B, G) floats.
 */
long rdmi_groupnorm_workspace(int B, int G);
int rdmi_groupnorm_stats(const void* x, int dtype, int B, long HW, int C, int G, float eps,
                         float* mean_rstd, float* workspace, void* stream);
/* Statistics from the 32-row × 4-channel moments a producing GEMM/conv emitted (gn_part): for
 * image b (rows b·HW .. b·HW+HW-1, HW % 32 == 0) and group g ((C/G) % 4 == 0), an f64 sum over the
 * group's partials in a fixed order — independent of how many images share the tensor. */
int rdmi_groupnorm_stats_partials(const float* part, long part_ld, int B, long HW, int C, int G, float eps,
                                  float* mean_rstd, void* stream);
/* Input-GroupNorm scale / shift table for rdmi_conv_args.in_affine: out [B][C/64][2][64] f32, per image b
 * and 64-channel block the scales rstd·gamma[c] then the shifts beta[c] − mean·(rstd·gamma[c]) — the f32
 * arithmetic of rdmi_groupnorm_apply (mean_rstd as rdmi_groupnorm_stats writes it; C % 64 == 0). */
int rdmi_groupnorm_affine(const float* mean_rstd, const float* gamma, const float* beta, int B, int C, int G,
                          float* out, void* stream);
int rdmi_groupnorm_apply(const void* x, void* y, int dtype, int B, long HW, int C, int G,
                         const float* mean_rstd, const float* gamma, const float* beta, int silu,
                         void* stream);

/* GroupNorm apply (+ SiLU when silu = 1) fused with a 3×3, stride-1, pad-1 convolution to ONE output
 * channel: y[b, h, w] = bias + Σ_{dy,dx,c} w[3dy+dx][c] · n(x)[b, h+dy-1, w+dx-1, c], n = the
 * normalised (+SiLU) input, zero outside the image.  x [B][H][W][C] in `dtype` (RDMI_F16 / RDMI_F32),
 * y [B][H][W] in `y_dtype` (RDMI_F16 / RDMI_F32: the f16 pipeline keeps its decoded depth in f32, so
 * the f16 rounding of the depth map does not reach the aligner and the min/max renormalisation),
 * w [9][C] f32, workspace ≥ rdmi_conv3x3_to1_gn_workspace(B, H, W) floats.  Replaces the decoder's
 * conv_norm_out → conv_act → conv_out (vae.py:335-347) followed by the depth pipeline's mean over
 * the RGB outputs (rollingdepth_pipeline.py:737), which is linear and folded into w / bias. */
long rdmi_conv3x3_to1_gn_workspace(int B, int H, int W);
int rdmi_conv3x3_to1_gn(const void* x, int dtype, int B, int H, int W, int C, int G, const float* mean_rstd,
                        const float* gamma, const float* beta, int silu, const float* w, float bias,
                        void* y, int y_dtype, float* workspace, void* stream);

/* LayerNorm over the last dim (BasicTransformerBlock.norm1/2/3, attention.py:445,495,522). */
int rdmi_layernorm(const void* x, void* y, int dtype, long M, int C, const float* gamma, const float* beta,
                   float eps, void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused multi-head attention forward, softmax(q kᵀ · scale) v, non-causal, no mask, D = 64; dtype
 * RDMI_F16 (f16 MFMA, f32 softmax), RDMI_F32 (f32-input MFMA, f32 softmax; the paper preset) or
 * RDMI_F32_X3 (f32 q/k/v/o and softmax, both products as bf16-split triples on the bf16 MFMA) or
 * RDMI_F32_X6 (the same with three-part splits and six products: f32-equivalent products).
 * Token-major q/k/v/o with row strides (ld*) and batch strides (bs*), head h at column h*D.
 * With the num_view fold done by the caller's strides (one "batch" = one snippet of n frames,
 * S = n·h·w), this is the cross-frame self-attention of the modified AttnProcessor2_0
 * (attention_processor.py:2208-2266) / XFormersAttnProcessor (:1989-2050).
 */
int rdmi_attention_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq,
                       int Sk, int D, long q_ld, long k_ld, long v_ld, long o_ld, long q_bs,
                       long k_bs, long v_bs, long o_bs, float scale, int dtype, void* stream);

/* Attention against a short key set (L ≤ 16 keys, e.g. the 2-token empty-text context of the
 * UNet cross-attention attn2, attention.py:508-516); k/v [Bkv][L][H*D] contiguous, Bkv ∈ {1, B}. */
int rdmi_attention_smallkv(const void* q, const void* k, const void* v, void* o, int B, int H,
                           int Sq, int L, int D, long q_ld, long o_ld, long q_bs, long o_bs,
                           long kv_bs, float scale, int dtype, void* stream);

/* BasicTransformerBlock's norm2 → attn2 → +residual against a TWO-token shared context
 * (attention.py:480-492, attention_processor.py:2172-2276 with Sk = 2), collapsed by exact algebra:
 * y = x + c + Σ_h σ(LN(x)·w_h) u_h with w = scale·Wq_hᵀ(K1−K0)_h and u_h = Wo_h(V1−V0)_h
 * ([H, C] f32 each, 16-B aligned), c = Wo·V0 + bo ([C] f32).  x, y: [M, C] f16 rows (C ≤ 1536,
 * 2·H·C·4 B ≤ 64 KiB).  Replaces LN + q GEMM + rdmi_attention_smallkv + out GEMM for that case. */
int rdmi_cross_attn_pair(const void* x, void* y, long M, int C, int H, const float* ln_gamma,
                         const float* ln_beta, float eps, const float* w, const float* u, const float* c,
                         void* stream);

/* Row softmax: p[r, :] = softmax(scale * s[r, :]) (f32 in, p_dtype out: RDMI_F16 / RDMI_F32).  Used with two rdmi_gemm
 * calls for the single-head d=C VAE mid-block attention (unet_2d_blocks.py:680-697). */
/* p[r·p_ld + c] = softmax_c(scale·s[r·cols + c]) for c < cols, 0 for cols ≤ c < p_ld (so a PV GEMM
 * can run on K = p_ld, a multiple of 8, when the key count is not). */
int rdmi_softmax_rows(const float* s, void* p, long rows, long cols, long p_ld, float scale, int p_dtype,
                      void* stream);

/* ---------------------------------------------------------------------------------------
 * Layout / elementwise helpers (f16 NHWC unless stated)
 */
/* NCHW (f32 if x_f32 else f16, batch/channel strides in elements; x_cstride = 0 replicates one
 * channel, e.g. the depth → 3-channel repeat before re-encoding, rollingdepth_pipeline.py:327)
 * → NHWC in y_dtype (RDMI_F16 / RDMI_F32) with channel padding to Cpad (zeros), y = x*scale */
int rdmi_nchw_to_nhwc(const void* x, int x_f32, void* y, int y_dtype, int B, int C, int H, int W, int Cpad,
                      float scale, long x_bstride, long x_cstride, void* stream);
/* NHWC in dtype (ld = channel stride) → NCHW f32, first C channels, y = x*scale + shift */
int rdmi_nhwc_to_nchw_f32(const void* x, int dtype, long ld, float* y, int B, int C, int H, int W,
                          float scale, float shift, void* stream);
/* The helpers below take the storage dtype (RDMI_F16 / RDMI_F32) of every activation operand. */
/* y[p, 0:Ca] = a[p, :], y[p, Ca:Ca+Cb] = b[p, :]  (torch.cat dim=1 of CrossAttn/UpBlock skips);
 * Ca, Cb multiples of one 16-B vector (8 f16 / 4 f32) */
int rdmi_concat_channels(const void* a, int Ca, const void* b, int Cb, void* y, long P, int dtype, void* stream);
/* NHWC f16 nearest resize to an explicit size: y[b,yo,xo] = x[b, ⌊yo·H/Ho⌋, ⌊xo·W/Wo⌋] (f32 scale,
 * clamped) — F.interpolate(size=…, mode="nearest") of Upsample2D when the UNet forwards an
 * upsample size (latent not a multiple of 2^levels; unet_2d_condition.py forward_upsample_size,
 * upsampling.py:167-178).  C % 8 == 0. */
int rdmi_resize_nearest(const void* x, int B, int H, int W, int C, void* y, int Ho, int Wo, int dtype,
                        void* stream);
/* 2-D transpose per batch: dst[b][c][r] = src[b][r][c] */
int rdmi_transpose(const void* src, void* dst, int batch, long rows, long cols, long src_ld,
                   long dst_ld, int dtype, void* stream);
/* Build the 8-channel UNet input of single_step (rollingdepth_pipeline.py:646-651):
 * out[i, p, 0:4] = rgb[frame_idx[i], p, 0:4], out[i, p, 4:8] = depth[dsel(i), p, 0:4]
 * (depth_ld: frame stride of `depth` in elements; depth_bcast=1 uses depth frame 0 for all). */
int rdmi_gather_unet_input(const void* rgb, long rgb_frame_ld, const void* depth,
                           long depth_frame_ld, int depth_bcast, const int* frame_idx, int count,
                           long HW, void* out, int dtype, void* stream);
/* DDIM step (eta = 0) / add_noise as the affine map they reduce to (scheduling_ddim.py:402-448,
 * :471-495): y = (ca·x + cb·e) * out_scale; x, e: [P] pixel rows with strides, y [P, ld_y]
 * channels 0..C-1, channels C..Cpad-1 of y zeroed; e_period > 0 broadcasts e over pixel rows
 * (the shared init noise of every frame, :282-288). */
int rdmi_ddim_combine(const void* x, long ld_x, const void* e, long ld_e, void* y, long ld_y,
                      long P, int C, int Cpad, float ca, float cb, float out_scale, long e_period,
                      int dtype, void* stream);
/* Refine averaging (rollingdepth_pipeline.py:586-629): out[f] = mean over the snippets s = f − j·stride
 * (0 ≤ s < n) of src[s][j]; src [n][w][P][ld], out [N][P][ld] f16 (channels ≥ C zeroed).  The sum is
 * taken in f64: exact for f16 terms (hence independent of the order of addition); for f32 terms
 * order-independent except when the terms' exponents span more than ≈29 bits (rare). */
int rdmi_snippet_average(const void* src, int n, int w, int stride, int N, long P, int C, int ld,
                         void* out, int dtype, void* stream);
/* Depth colourisation (src/util/colorize.py:12-93, the CLI's visualisation): rgb [n][3] u8 =
 * lut[idx(d)] with idx as matplotlib's Colormap.__call__ computes it for the normalised depth
 * ((d - minmax[0]) / (minmax[1] - minmax[0]) clipped to [0, 1], evaluated in the depth's dtype),
 * lut [(lut_n + 3)][3] = (colormap table · 255) as uint8 incl. the under / over / bad entries.  minmax =
 * {min, max − min} in the depth's dtype (the range as the reference's numpy forms it).  index != NULL:
 * write the table index per pixel instead (lut / rgb unused). */
int rdmi_colorize(const void* depth, int dtype, long n, const void* minmax, const unsigned char* lut, int lut_n,
                  unsigned char* rgb, int* index, void* stream);
/* Sharded refine averaging (the loop above split over ranks): sum [N][P][C] f64 =
 * per frame the sum over THIS rank's snippets k0 .. k0+nloc-1 (src [nloc][w][P][ld], dtype RDMI_F16 /
 * RDMI_F32), zero where none covers the frame; after an all-reduce SUM over ranks,
 * rdmi_snippet_finish divides by the frame's cover count over all n snippets → out [N][P][ld]
 * (channels ≥ C zeroed).  The f64 sums are exact for f16 terms, so every world size and every
 * all-reduce order reproduces rdmi_snippet_average bitwise; with f32 terms the same holds except in rare
 * rounding cases (terms whose exponents span more than ≈29 bits). */
int rdmi_snippet_accumulate(const void* src, int dtype, int k0, int nloc, int w, int stride, int N, long P, int C,
                            int ld, double* sum, void* stream);
int rdmi_snippet_finish(const double* sum, int n, int w, int stride, int N, long P, int C, int ld, void* out,
                        int dtype, void* stream);
/* Global min/max of an f16 or f32 buffer → minmax[2] f32 (workspace ≥ 2*1024 floats)
 * (the `min([snippet.min() ...])` of depth_aligner.py:78 and the min/max of :316-317). */
int rdmi_minmax(const void* x, int x_f32, long n, float* minmax, float* workspace, void* stream);
/* In place: x = (x - mn) / (mx - mn) * 2 - 1 with mn,mx read from device (re-normalise, :316-318) */
int rdmi_renormalize_f32(float* x, long n, const float* minmax, void* stream);

/* ---------------------------------------------------------------------------------------
 * DepthAligner (rollingdepth/depth_aligner.py) — co-alignment of dilated snippets.
 * Snippet layout: one f32 buffer per dilation, x_d [n_d][w_d][P] (border-cropped, stride-subsampled,
 * min-shifted; depth_aligner.py:78-92).  Parameters s_d, t_d are f32 [n_d].  Snippet lengths w_d may
 * differ per dilation (rollingdepth_pipeline.py:221-226): the loss then follows the reference's
 * scatter of dilation i's slot j into row i·w_i + j of [Σw, N, P] (depth_aligner.py:169-188) —
 * coinciding rows are overwritten by the later dilation, and a layout whose rows run past Σw
 * (the reference's IndexError) is rejected with RDMI_E_ARG.
 */
typedef struct rdmi_aligner_args {
  int n_dil;                 /* number of dilations (≤ 8) */
  const float* x[8];         /* subsampled snippets per dilation [n_d][w_d][P] */
  float* s[8]; float* t[8];  /* scales / translations [n_d] (in: init, out: result) */
  int n[8]; int stride[8];   /* snippets per dilation, frame stride (dilation) */
  int w[8];                  /* snippet length per dilation (Σ w_d ≤ 64) */
  int seq_len; long P;
  float lr, beta1, beta2, eps, lmda2, lmda3, depth_w, loss_scale;
  int iters;
  float* history;            /* [iters][3] (loss, min summ, max summ) or NULL */
  float* workspace;          /* ≥ rdmi_aligner_workspace(...) floats */
} rdmi_aligner_args;
long rdmi_aligner_workspace(const rdmi_aligner_args* a);
/* Adam loop of DepthAligner.optimize (:123-229) fully on device, no host sync. */
int rdmi_aligner_optimize(const rdmi_aligner_args* a, void* stream);
/* Border crop + stride subsample + min shift of one dilation's decoded snippets
 * x [n][w][H][W] (f16/f32) → out [n][w][P] f32 with out = dtype(x - shift[0]) (:78-92). */
int rdmi_aligner_prepare(const void* x, int x_f32, int n, int w, int H, int W, int border,
                         int factor, const float* shift, float* out, void* stream);
/* merge_scaled_triplets (:231-262): full-resolution snippets per dilation xf_d [n_d][w_d][HW]
 * (w: snippet length per dilation)
 * (x_f32 = 1: f32 snippets; 0: f16 snippets in the reference's f16 arithmetic; 2: f16 snippets with
 * the shift and s·x+t in f32 — no intermediate f16 rounding; the min shift read from shift[0] is
 * applied first),
 * s/t f32 → out [seq_len][HW] f32 (s·x+t rounded through the snippet dtype exactly where the
 * reference computes in it; the per-frame mean is accumulated in f32). */
int rdmi_aligner_merge(int n_dil, const void* const* xf, int x_f32, const float* const* s,
                       const float* const* t, const int* n, const int* stride, const int* w, int seq_len,
                       long HW, const float* shift, float* out, void* stream);

/* Sharded merge over frame windows: each rank sums s·x+t of ITS full-resolution
 * snippets — rows k0[d] .. k0[d]+nloc[d]-1 of dilation d, xf_d [nloc_d][w_d][HW] — over only frames
 * f0 .. f0+nf-1 (the window its snippets cover) into sum_out [nf][HW] f64 (the per-slot arithmetic of
 * rdmi_aligner_merge, zero where no local slot covers a frame), sends every other rank the rows of that
 * rank's frame chunk (an all-to-all of uneven row counts), and rdmi_aligner_merge_finish_pieces adds the
 * received pieces per frame in source-rank order and divides by the frame's cover count over all n[d]
 * snippets: piece q = frames piece_f0[q] .. piece_f0[q]+piece_nf[q]-1 of one source, pieces stored back
 * to back in recv [Σ piece_nf][HW] f64, all inside this rank's frames f0 .. f0+nf-1 → out [nf][HW] f32.
 * Any piece count (the launch is split by frame range where more than 64 pieces arrive; a single frame
 * touched by more than 64 pieces → RDMI_E_UNSUPPORTED).  With f32 arithmetic (x_f32 1 / 2) the f64 sums
 * reproduce rdmi_aligner_merge bitwise in practice (exact while a frame's terms span ≤ ≈29 exponent bits). */
int rdmi_aligner_merge_partial_window(int n_dil, const void* const* xf, int x_f32, const float* const* s,
                                      const float* const* t, const int* n, const int* stride, const int* k0,
                                      const int* nloc, const int* w, int f0, int nf, long HW, const float* shift,
                                      double* sum_out, void* stream);
int rdmi_aligner_merge_finish_pieces(int n_dil, const int* n, const int* stride, const int* w, int f0, int nf, long HW,
                                     int npieces, const int* piece_f0, const int* piece_nf, const double* recv,
                                     float* out, void* stream);

/* Single-head flash attention for head dim 512 (f16): the VAE mid-block attention
 * (unet_2d_blocks.py:680-697 through AttnProcessor2_0's 4-D path, attention_processor.py:2172-2276 —
 * one head, d = C = 512) as one pass over K / Vᵀ instead of f32 scores → softmax → PV.
 * q [B][Sq][512] (row stride q_ld), k [B][Sk][512] (k_ld), vt = Vᵀ [B][512][Skp] (row stride vt_ld ≥
 * Skp, Skp = Sk rounded up to 32, columns Sk..Skp-1 zero), o [B][Sq][512] (o_ld); batch strides in
 * elements; o = softmax(q kᵀ · scale) v with f32 accumulation and f32 softmax statistics.
 * flags: int workspace of B·ceil(Sq / 128) entries (no initialisation needed) enabling the
 * 32-query-per-wave pass with a fixed running max and a fix-up pass over the blocks it flags; NULL
 * runs the 16-query kernel (running max with rescale) alone.  Same result either way. */
int rdmi_attention_d512(const void* q, const void* k, const void* vt, void* o, int B, int Sq, int Sk, int Skp,
                        long q_ld, long k_ld, long vt_ld, long o_ld, long q_bs, long k_bs, long vt_bs, long o_bs,
                        float scale, int* flags, void* stream);

/* ---------------------------------------------------------------------------------------
 * Frame ingest / resize.  Replaces load_video_frames' per-frame resize_max_res + normalisation
 * (rollingdepth/video_io.py:38-67, 104-123: torchvision resize(antialias=True) of the decoded
 * float frame, then (x / 255)·2 − 1) and __call__'s restore_res resizes
 * (rollingdepth_pipeline.py:155-173).  x element (n, c, y, x) at x + n·sn + c·sc + y·sy + x·sx
 * (elements) of dtype RDMI_U8 (decoded rgb24 frames, e.g. sn = H·W·3, sc = 1, sy = W·3, sx = 3) or
 * RDMI_F32; y f32 [N, C, Ho, Wo] contiguous.  mode RDMI_RESIZE_*: the antialiased separable
 * filter of F.interpolate(antialias=True) for BILINEAR / BICUBIC (width pass, then height pass;
 * a dimension whose size does not change is not resampled), ATen nearest indexing for NEAREST.
 * normalize != 0: y = (v / 255)·2 − 1.  Downscale factor ≤ 9 (bicubic ≤ 4.5).  workspace ≥
 * rdmi_resize_workspace(...) bytes (f32 intermediate when both dimensions change).
 */
size_t rdmi_resize_workspace(int N, int C, int H, int W, int Ho, int Wo);
int rdmi_resize(const void* x, int x_dtype, long sn, long sc, long sy, long sx, int N, int C, int H, int W, int Ho,
                int Wo, int mode, int normalize, float* y, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RDMI_H */

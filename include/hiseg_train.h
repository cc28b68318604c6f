/*
 * hiseg_train.h — C ABI of libhiseg's TRAINING kernels (backward passes, train-mode
 * BatchNorm, dropout, the refined hierarchical loss and the AdamW update) for the
 * ROI-hierarchical path of PINTO0309/human-instance-segmentation.  Conventions as in hiseg.h:
 * caller-owned device pointers, NHWC activations with 16-B channel padding, stream-ordered,
 * no host synchronisation, 0 / negative hiseg_status return.
 *
 * The reference trains with PyTorch autograd (train_advanced.py:680-762: autocast forward,
 * scaled backward, clip_grad_norm_, AdamW); every entry below replaces the backward (or the
 * train-mode forward) of one op class on that path, cited per function.
 */
#ifndef HISEG_TRAIN_H_
#define HISEG_TRAIN_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ----------------------------------------------------------------------------------------
 * Convolution weight gradient (nn.Conv2d / nn.ConvTranspose2d backward w.r.t. weight and
 * bias; autograd of every conv site listed at hiseg_conv2d_fwd).
 * `fwd` describes the FORWARD conv exactly as passed to hiseg_conv2d_fwd (sources, geometry,
 * Cout = GEMM columns, convT); only its input-side fields are read.  `dy` is the gradient of
 * the forward GEMM output (NHWC, dtype fwd->dtype, channel stride dy_cstride, offset dy_coff;
 * for convT the full-resolution output).  Computes, for one split s of the output pixels,
 *   ws[s][j][k] = sum_{p in split s} dy[p][j] * X[p][k]       (k < Ktot = KH*KW*(Ca+Cb))
 *   ws[s][j][Ktot] = sum_{p in split s} dy[p][j]                (if want_bias)
 * as f32, j < Cg = round_up(Cout, 16), k < Kg (hiseg_conv2d_wgrad_dims).  MFMA bf16 / f32.
 * -------------------------------------------------------------------------------------- */
int hiseg_conv2d_wgrad_dims(const hiseg_conv2d_desc* fwd, int want_bias, int* Cg, int* Kg, int* splits);
int hiseg_conv2d_wgrad(const hiseg_conv2d_desc* fwd, const void* dy, int dy_cstride, int dy_coff,
                       int want_bias, float* ws, int splits, hiseg_stream_t stream);
/* Which kernel computed each weight gradient since the last reset: counts[5] indexed by
 * HISEG_WGRAD_PATH_* (wide 256x256 tile, transposed-read tile, generic bf16 fallback, f32, halo tile).
 * hiseg_wgrad_last_path: the path of this thread's last hiseg_conv2d_wgrad (-1 before any). */
#define HISEG_WGRAD_PATH_WIDE 0
#define HISEG_WGRAD_PATH_TR 1
#define HISEG_WGRAD_PATH_GENERIC 2
#define HISEG_WGRAD_PATH_F32 3
#define HISEG_WGRAD_PATH_HWC 4
int hiseg_wgrad_path_stats(long long* counts, int reset);
int hiseg_wgrad_last_path(void);

/* Sum the split partials and scatter into the reference parameter layouts (f32):
 *   conv : gw[co][ci][ky][kx]  ([Cout][Cin][KH][KW], Cin = ca_real + cb_real), gb[co]
 *   convT: gw[ci][co][dy][dx]  ([Cin][Cout/4][2][2]),                          gb[co] (sum of the 4 sub-pixel columns)
 * ca/cb are the padded source channel counts of the packed K layout.  accumulate != 0 adds
 * to gw/gb (gradient accumulation), else overwrites.  gb may be null. */
typedef struct hiseg_wgrad_map {
  int Cout, KH, KW, ca, ca_real, cb, cb_real, convT, Cg, Kg, want_bias;
} hiseg_wgrad_map;
int hiseg_conv2d_wgrad_reduce(const float* ws, int splits, const hiseg_wgrad_map* map, float* gw, float* gb,
                              int accumulate, hiseg_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Weight packing after every optimiser step, all layers in one launch.  Each table entry
 * (device memory) packs one f32 parameter in the reference layout into the implicit-GEMM
 * operand of the forward conv (mode 0: conv, 2: convT) or of its data-gradient conv
 * (mode 1: conv -> flipped taps, Cin/Cout swapped; mode 3: convT -> 2x2/s2 conv).
 * mode | HISEG_PACK_FRAG (modes 0 and 1 of 3x3 layers whose K channel count is a multiple of 64): the same
 * [rows][K_pad] matrix written in MFMA A-fragment order (hiseg.ops.frag_pack: [rows/16][K/64 channel blocks]
 * [tap][2][64 lanes][8], the weight_frag operand of hiseg_conv2d_desc).
 * -------------------------------------------------------------------------------------- */
#define HISEG_PACK_FRAG 8
/* mode HISEG_PACK_BIAS: dst (f32, total entries) [i] = src[i % Cout] -- a conv bias into its epilogue shift
 * (ConvTranspose: total = 4 * Cout, one copy per sub-pixel column block); rows = 1, K_pad = total. */
#define HISEG_PACK_BIAS 4
typedef struct hiseg_pack_entry {
  const float* src; void* dst; int dtype; int mode;
  int Cout, Cin_real, KH, KW;   /* reference dims (convT: Cin_real = in, Cout = out channels)  */
  int ca, ca_real, cb, cb_real; /* padded / real channel split of the forward K layout         */
  int rows, K_pad;              /* packed [rows][K_pad]                                       */
  int cop;                      /* dgrad modes: padded channel count of the output gradient   */
  int total;                    /* rows * K_pad                                               */
} hiseg_pack_entry;
int hiseg_pack_weights(const hiseg_pack_entry* table_dev, int n, int max_total, hiseg_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Train-mode BatchNorm2d (advanced/normalization_comparison.py:181-182; nn.BatchNorm2d
 * eps 1e-5, momentum 0.1): batch statistics over N*H*W, running-stat update with the
 * unbiased variance, then y = act(z*scale + shift [+ residual]) * chan_mul[n][c].
 * -------------------------------------------------------------------------------------- */
/* Upper bound on the pixel splits of the statistics / backward-reduce kernels: size `partial`
 * buffers by it.  The split count actually used depends on P (adaptive, >= 32 pixels per split);
 * hiseg_bn_stats writes, and hiseg_bn_finalize merges, exactly that count for the same P, so a
 * caller must not fill `partial` itself and hand it to hiseg_bn_finalize. */
int hiseg_bn_partials(void);
int hiseg_bn_stats(int dtype, const void* z, long long P, int C, int cstride, int coff, float* partial,
                   hiseg_stream_t stream);
/* partial [splits(P)][3][C], as written by hiseg_bn_stats for the same P -> mean/invstd [C], scale/shift [C] (fold of gamma/beta), running update. */
int hiseg_bn_finalize(const float* partial, int C, long long P, const float* gamma, const float* beta, float eps,
                      float momentum, float* running_mean, float* running_var, float* mean, float* invstd,
                      float* scale, float* shift, hiseg_stream_t stream);
/* The same merge over an explicit split count: the partials a conv epilogue wrote
 * (hiseg_conv2d_desc.stats_partial, S = hiseg_conv2d_stats_tiles).  `partial` is scratch the merge consumes: with
 * more than 256 splits, groups of 64 are pre-merged in place (row 64 g holds group g's merge afterwards). */
int hiseg_bn_finalize_n(float* partial, int S, int C, long long P, const float* gamma, const float* beta,
                        float eps, float momentum, float* running_mean, float* running_var, float* mean,
                        float* invstd, float* scale, float* shift, hiseg_stream_t stream);
typedef struct hiseg_bn_apply_desc {
  int dtype; long long P; int HW; int C;
  const void* z; int z_cstride, z_coff;
  const float* scale; const float* shift;
  const void* residual; int r_cstride, r_coff;
  int act;
  const float* chan_mul;          /* [N][C] or null (Dropout2d mask, 0 or 1/(1-p)) */
  void* y; int y_cstride, y_coff;
  float act_beta;                 /* Swish beta (act == HISEG_ACT_SWISH) */
  int per_sample;                 /* scale / shift are [N][C] per-sample tables (LayerNorm2d), n = p / HW */
} hiseg_bn_apply_desc;
int hiseg_bn_apply(const hiseg_bn_apply_desc* d, hiseg_stream_t stream);

/* Backward.  g = dy * chan_mul * act'(y) (ReLU: y > 0; sigmoid: y(1-y); SiLU: from the pre-activation
 * xhat*gamma + beta; none: 1), xhat = (z - mean)*invstd:
 *   reduce : dgamma[c] (+)= sum g*xhat, dbeta[c] (+)= sum g ; partial [splits][2][C]
 *   apply  : dz = gamma*invstd*(g - sum(g)/P - xhat*sum(g*xhat)/P)     (to dz, dtype)
 *            dres (+)= g  (the residual input's gradient, if dres != null; accumulate flag)
 * dconv_bias (+)= sum dz (analytically ~0; conv bias before BN) if non-null. */
typedef struct hiseg_bn_bwd_desc {
  int dtype; long long P; int HW; int C;
  const void* dy; int dy_cstride, dy_coff;
  const void* y; int y_cstride, y_coff;
  const void* z; int z_cstride, z_coff;
  const float* chan_mul;
  int act;
  const float* mean; const float* invstd; const float* gamma;
  float* partial;
  float* dgamma; float* dbeta; float* dconv_bias; int accumulate_params;
  void* dz; int dz_cstride, dz_coff;
  void* dres; int dres_cstride, dres_coff; int dres_accumulate;
  const float* beta;              /* BN shift; needed for act = SiLU (pre-activation = xhat*gamma + beta) */
  /* optional, act = ReLU without dres: the forward's folded affine (hiseg_bn_finalize scale / shift); the
   * ReLU mask is then recomputed from z as z*scale + shift > 0 -- exactly the forward's expression -- and
   * y is not read (one activation stream less in each pass) */
  const float* fwd_scale; const float* fwd_shift;
  float act_beta;                 /* Swish beta */
  /* the forward's residual input (optional): with fwd_scale / fwd_shift the activation derivative is taken at
   * the forward's pre-activation z*fwd_scale + fwd_shift + residual -- required for GELU / Swish / SiLU / ReLU
   * after a residual add; GELU and Swish always need fwd_scale / fwd_shift */
  const void* residual; int r_cstride, r_coff;
  /* round 5, optional: > 0 -- `partial` already holds [partial_splits][3][C] sums of g, g*xhat, xhat written by
   * the data-gradient conv's epilogue (hiseg_conv2d_desc.bnb_partial); the reduction pass is skipped.  `partial`
   * then needs (partial_splits + ceil(partial_splits / 64) + 1) * 3 * C floats. */
  int partial_splits;
} hiseg_bn_bwd_desc;
int hiseg_bn_bwd(const hiseg_bn_bwd_desc* d, hiseg_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Train-mode LayerNorm2d (model.py:18-38, normalization_type 'layernorm2d' of
 * advanced/normalization_comparison.py:159-206): per sample n, mean and biased variance of the
 * conv output z over (C, H, W), eps 1e-5; no running statistics.
 *   hiseg_ln_fwd_stats: mean/invstd [N] and the folded per-sample tables scale/shift [N][C]
 *     (scale = w_c * invstd_n, shift = b_c - mean_n * scale); the output is then
 *     hiseg_bn_apply with per_sample = 1 (+ residual, act, Dropout2d mask).
 *   hiseg_ln_bwd: g = dy * chan_mul * act'(z*scale + shift [+ residual]), xhat = (z - mean_n)*invstd_n,
 *     dz = invstd_n * (w_c g - a_n - xhat b_n) with a_n = mean over (C,H,W) of w_c g and
 *     b_n = mean of w_c g xhat; dw (+)= sum g xhat, db (+)= sum g, dconv_bias (+)= sum dz,
 *     dres (+)= g.
 * ws: hiseg_ln_ws(N, HW, C) floats, 16-B aligned (shared by the two calls of one layer).
 * -------------------------------------------------------------------------------------- */
long long hiseg_ln_ws(int N, int HW, int C);
int hiseg_ln_fwd_stats(int dtype, const void* z, int N, int HW, int C, int cstride, int coff, const float* gamma,
                       const float* beta, float eps, float* ws, float* mean, float* invstd, float* scale, float* shift,
                       hiseg_stream_t stream);
typedef struct hiseg_ln_bwd_desc {
  int dtype; int N, HW, C;
  const void* dy; int dy_cstride, dy_coff;
  const void* z; int z_cstride, z_coff;
  const void* residual; int r_cstride, r_coff;
  const float* chan_mul;          /* [N][C] or null */
  int act; float act_beta;
  const float* mean; const float* invstd;   /* [N] */
  const float* scale; const float* shift;   /* [N][C] forward tables */
  const float* gamma;
  float* dgamma; float* dbeta; float* dconv_bias; int accumulate_params;
  void* dz; int dz_cstride, dz_coff;
  void* dres; int dres_cstride, dres_coff; int dres_accumulate;
  float* ws;
} hiseg_ln_bwd_desc;
int hiseg_ln_bwd(const hiseg_ln_bwd_desc* d, hiseg_stream_t stream);

/* Dropout2d mask (nn.Dropout2d in refinement.py:484,486,519,525,540): per (n, c) 0 with
 * probability p else 1/(1-p), from a counter-based hash of (seed, n*C + c). */
int hiseg_dropout2d_mask(int N, int C, float p, unsigned long long seed, float* out, hiseg_stream_t stream);
/* The same mask from a device-resident seed base (seed = (*seed_base * 0x9E3779B1 + offset) mod 2^48), and the
 * one-thread kernel that advances the base: a step captured into a HIP graph draws fresh masks per replay. */
int hiseg_dropout2d_mask_dev(int N, int C, float p, const unsigned long long* seed_base, unsigned long long offset,
                             float* out, hiseg_stream_t stream);
int hiseg_seed_advance(unsigned long long* seed_base, hiseg_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Element-wise backward helpers (NHWC views, dtype = compute dtype, f32 math).
 *   relu_bwd : dz = dy * chan_mul * (y > 0)                       (activation without BN)
 *   sigmoid_bwd: dz = dy * s * (1 - s)
 *   gate_fwd : out = a * g                                          (fg_gate / bottleneck gate)
 *   gate_bwd : da (+)= dy * g ;  dzg = dy * a * g * (1 - g)         (g = sigmoid output)
 *   add      : dst += src
 * -------------------------------------------------------------------------------------- */
typedef struct hiseg_ew_view { void* p; int cstride, coff; } hiseg_ew_view;
int hiseg_relu_bwd(int dtype, long long P, int HW, int C, hiseg_ew_view dy, hiseg_ew_view y, const float* chan_mul,
                   hiseg_ew_view dz, hiseg_stream_t stream);
int hiseg_sigmoid_bwd(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view s, hiseg_ew_view dz,
                      hiseg_stream_t stream);
int hiseg_gate_fwd(int dtype, long long P, int C, hiseg_ew_view a, hiseg_ew_view g, hiseg_ew_view out,
                   hiseg_stream_t stream);
int hiseg_gate_bwd(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view a, hiseg_ew_view g,
                   hiseg_ew_view da, int da_accumulate, hiseg_ew_view dzg, hiseg_stream_t stream);
/* dz (dtype, += if accumulate) = dy * act'(y) with dy, y f32 views (the 1/2-channel f32 heads:
 * contour sigmoid, distance map, EnhancedUNet's f32 logits). act: NONE or SIGMOID (y = output). */
int hiseg_act_bwd_cvt(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view y, int act, hiseg_ew_view dz,
                      int accumulate, hiseg_stream_t stream);
int hiseg_add_inplace(int dtype, long long P, int C, hiseg_ew_view dst, hiseg_ew_view src, hiseg_stream_t stream);
/* dz (+= if accumulate) = dy * act'(z) at the pre-activation z (compute dtype views): the backward of an
 * activation applied without normalisation (GELU / Swish(act_beta) / SiLU after a plain conv). */
int hiseg_act_bwd_pre(int dtype, long long P, int C, hiseg_ew_view dy, hiseg_ew_view z, int act, float act_beta,
                      hiseg_ew_view dz, int accumulate, hiseg_stream_t stream);

/* MaxPool2d(2) backward (EnhancedUNet, hierarchical_segmentation_unet.py:366,384): dx (+)= dy
 * routed to the first maximum of each 2x2 window (PyTorch's tie rule). */
int hiseg_maxpool2x2_bwd(int dtype, const void* x, int N, int H, int W, int C, const void* dy, void* dx,
                         int accumulate, hiseg_stream_t stream);

/* F.interpolate(bilinear, align_corners=False) backward for the aux heads' up-sampling
 * (refinement.py:775-800): NCHW f32 planes, dx = adjoint of resize (h,w) -> (H,W). */
int hiseg_resize_bilinear_bwd(const float* dy, int NC, int h, int w, int H, int W, float* dx, hiseg_stream_t stream);

/* EfficientNet MBConv training (timm InvertedResidual / DepthwiseSeparableConv, smp encoder stages unfrozen by
 * train_distillation_staged.py's progressive schedule).  Depthwise conv: NHWC with cstride == C, weights in
 * the parameter layout [C][K*K] f32; fwd writes the raw conv (train-mode BN follows); bwd_data writes or
 * accumulates dx; bwd_weight ACCUMULATES into dw (f32 [C][K*K]) through ws (hiseg_dw_bwd_weight_ws floats). */
int hiseg_dw_train_fwd(int dtype, const void* x, int N, int H, int W, int C, int K, int stride, const float* w,
                       void* out, int Ho, int Wo, hiseg_stream_t stream);
int hiseg_dw_bwd_data(int dtype, const void* dy, int N, int H, int W, int C, int K, int stride, const float* w,
                      int Ho, int Wo, void* dx, int accumulate, hiseg_stream_t stream);
long long hiseg_dw_bwd_weight_ws(int dtype, int N, int Ho, int Wo, int C, int K);   /* floats (pixel splits x C x K*K) */
int hiseg_dw_bwd_weight(int dtype, const void* x, const void* dy, int N, int H, int W, int C, int K, int stride,
                        int Ho, int Wo, float* ws, float* dw, hiseg_stream_t stream);

/* timm SqueezeExcite in training: gate = sigmoid(W2 act(W1 gap(x) + b1) + b2), out = x * gate (materialised:
 * the projection conv's input).  fwd keeps gap [N][C], hpre [N][Cr], gate [N][C]; bwd from d(out) writes dx
 * and ACCUMULATES dW1 [Cr][C], db1, dW2 [C][Cr], db2.  ws: hiseg_se_train_ws floats. */
long long hiseg_se_train_ws(int N, int C, int Cr);
int hiseg_se_train_fwd(int dtype, const void* x, int N, int HW, int C, const float* w1, const float* b1, int Cr,
                       const float* w2, const float* b2, int act, float* ws, float* gap, float* hpre, float* gate,
                       void* out, hiseg_stream_t stream);
int hiseg_se_train_bwd(int dtype, const void* x, int N, int HW, int C, const float* w1, int Cr, const float* w2,
                       int act, const float* gap, const float* hpre, const float* gate, const void* dout, void* dx,
                       float* ws, float* dw1, float* db1, float* dw2, float* db2, hiseg_stream_t stream);

/* Backward of the nearest x2 upsample the UNet decoder fuses into its conv1 loader (smp DecoderBlock,
 * F.interpolate(scale_factor=2, mode="nearest")): dx[n][y][x][c] (+)= sum of the 2x2 children
 * dy[n][2y+i][2x+j][c].  dy is the full-resolution gradient view (N x 2h x 2w), dx the (h x w) one. */
int hiseg_upsample2x_bwd(int dtype, long long N, int h, int w, int C, hiseg_ew_view dy, hiseg_ew_view dx,
                         int accumulate, hiseg_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Optimiser step over a flat f32 parameter space (all trainable parameters of the model are
 * views into one buffer, their gradients into another): torch.nn.utils.clip_grad_norm_ +
 * torch.optim.AdamW (train_advanced.py:733-740 clip 1.0; :1111-1143 AdamW lr 1e-4, wd 0.01).
 *   hiseg_grad_norm_partials: partial[b] = sum of g^2 over block b's slice (b < hiseg_optim_blocks())
 *   hiseg_adamw_step: total = sqrt(sum partial) (written to norm_out by block 0 if non-null);
 *     coef = min(1, max_norm / (total + 1e-6)) if max_norm > 0 (grads scaled in place, as
 *     clip_grad_norm_ does); then AdamW with bias corrections bc1 = 1-beta1^t, bc2 = 1-beta2^t.
 * -------------------------------------------------------------------------------------- */
int hiseg_optim_blocks(void);
int hiseg_grad_norm_partials(const float* g, long long n, float* partial, hiseg_stream_t stream);
int hiseg_adamw_step(float* p, float* g, float* m, float* v, long long n, float lr, float beta1, float beta2, float eps,
                     float weight_decay, float bc1, float bc2, const float* partial, float max_norm, float* norm_out,
                     hiseg_stream_t stream);
/* The same step with the non-finite guard and the step count on the device (no host sync):
 *   the reference never applies a step whose gradients are not finite -- GradScaler.step skips it on the
 *   AMP path (train_advanced.py:751-762), the fp32 path skips a NaN loss / NaN gradients (:814-832).  If
 *   total = sqrt(sum partial) is NaN or Inf, p, g, m, v are left untouched, the step count is not
 *   advanced and *skipped is incremented; otherwise t = steps[parity] + 1 drives the bias corrections
 *   (computed in double as torch.optim.AdamW does) and steps[parity ^ 1] receives the new count
 *   (steps[parity] otherwise) -- two slots: every block reads slot `parity` while block 0 writes the
 *   other -- and a one-thread commit launch then copies it back into slot `parity`, so the count always
 *   lives in slot `parity` and a fixed parity (0) serves every call: the step can be captured into a HIP
 *   graph and replayed.  norm_out (optional) receives total. */
int hiseg_adamw_step_guarded(float* p, float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                             float eps, float weight_decay, const float* partial, float max_norm, float* norm_out,
                             int* steps, int parity, int* skipped, hiseg_stream_t stream);
/* The guarded step with a step count per parameter segment, as torch.optim.AdamW keeps one per parameter
 * (parameters added to the optimizer later -- progressive unfreezing, train_distillation_staged.py:1531-1552 --
 * start at t = 0 while the others continue).  seg_start[0..nseg] (int64, device) cuts [0, n) into nseg <=
 * hiseg_adamw_max_segments() runs of parameters that share a count; steps is [2][nseg] int32 (slot
 * parity * nseg + s holds segment s's count, the other row is the staging row of the commit, as above).  A
 * non-finite total skips the whole step (no segment advances).  Inf-only gradients are skipped here on purpose,
 * although the reference's fp32 path (train_advanced.py:815-832) checks only for NaN.  The update follows
 * torch.optim.AdamW's multi-tensor arithmetic op for op (p *= decay; m = lerp(m, g, 1 - beta1); v = v beta2 +
 * (1 - beta2) g g; p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)), with one_minus_beta1/2 and decay = 1 - lr
 * weight_decay rounded from double on the host as torch's Python scalars are. */
int hiseg_adamw_max_segments(void);
int hiseg_adamw_step_segmented(float* p, float* g, float* m, float* v, long long n, float lr, float beta1,
                               float beta2, float one_minus_beta1, float one_minus_beta2, float decay, float eps,
                               const float* partial, float max_norm, float* norm_out, const long long* seg_start,
                               int nseg, int* steps, int parity, int* skipped, hiseg_stream_t stream);
/* The segmented step with the learning rate and the decoupled decay factor on the device: lr_decay[0] = lr,
 * lr_decay[1] = 1 - lr * weight_decay (rounded from double on the host), read by the kernel at run time, so a HIP
 * graph that captured the step follows a learning-rate schedule (CosineAnnealingLR, train_advanced.py:1126-1131,
 * stepped per epoch at :1633) by a device write before its replay, without a re-capture. */
int hiseg_adamw_step_segmented_dev(float* p, float* g, float* m, float* v, long long n, const float* lr_decay,
                                   float beta1, float beta2, float one_minus_beta1, float one_minus_beta2, float eps,
                                   const float* partial, float max_norm, float* norm_out, const long long* seg_start,
                                   int nseg, int* steps, int parity, int* skipped, hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif  /* HISEG_TRAIN_H_ */

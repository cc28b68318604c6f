/*
 * hiseg.h — C ABI of libhiseg, the MI355X (gfx950) kernels behind the ROI-hierarchical
 * instance-segmentation hot path of PINTO0309/human-instance-segmentation.
 *
 * The reference has no FFI of its own: its "operator API" for this path is the set of
 * PyTorch ops the nn.Modules call.  Every entry point below replaces
 * one op class of that path; the reference call site it replaces is cited per function.
 * Reference paths are relative to the reference repository root.
 *
 * Conventions
 *   - Activations are NHWC ("pixels" x "channels"), channel dimension padded to a multiple
 *     of 8 elements (bf16) / 4 elements (f32) so every pixel row is a whole number of 16-B
 *     chunks.  A tensor view is (base pointer, channel stride, channel offset).
 *   - All pointers are device pointers owned by the caller (the library never allocates).
 *   - Every call is asynchronous on `stream` (a hipStream_t passed as void*), performs no
 *     host<->device synchronisation and no host read of device data; graph-capturable.
 *   - Every call returns 0 (HISEG_OK) or a negative hiseg_status; the text of the last error
 *     of the calling thread is returned by hiseg_last_error_string().
 */
#ifndef HISEG_H_
#define HISEG_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef void* hiseg_stream_t; /* hipStream_t */

enum hiseg_dtype { HISEG_F32 = 0, HISEG_BF16 = 1 };

/* Activations (advanced/activation_utils.py:71-101): GELU is nn.GELU's exact erf form,
 * SWISH is x * sigmoid(beta * x) with beta taken from the caller's act_beta (SILU == SWISH, beta 1). */
enum hiseg_act { HISEG_ACT_NONE = 0, HISEG_ACT_RELU = 1, HISEG_ACT_SIGMOID = 2, HISEG_ACT_SILU = 3,
                 HISEG_ACT_GELU = 4, HISEG_ACT_SWISH = 5 };

enum hiseg_status {
  HISEG_OK = 0,
  HISEG_ERR_BAD_ARG = -1,     /* null pointer / negative size / unsupported enum      */
  HISEG_ERR_BAD_SHAPE = -2,   /* shape or alignment contract violated                 */
  HISEG_ERR_BAD_DTYPE = -3,   /* dtype combination not built                          */
  HISEG_ERR_LAUNCH = -4       /* hipLaunchKernel / hipGetLastError reported a failure */
};

/* Library identification. */
int hiseg_version(void);
const char* hiseg_last_error_string(void);
/* 1 if the library's code object contains gfx950 kernels (always true for this build). */
int hiseg_built_for_gfx950(void);
/* Test utility (tests/, tools/): fill the LDS of every CU with a 32-bit pattern -- 160 KB workgroups, `rounds`
 * times the CU count of them -- so that a kernel which reads LDS it did not write in its own dispatch (stale data
 * left by an earlier kernel: LDS is not cleared between dispatches) sees the pattern (e.g. a NaN). */
int hiseg_debug_fill_lds(unsigned pattern, int rounds, hiseg_stream_t stream);
/* Test utility: counts of the kernel choices that depended on where a layer's two sources lie in memory, since the
 * last reset -- `declined`: a kernel refused the layer for its placement (another kernel took it); `far`: a kernel
 * took it through one buffer resource per source.  Either pointer may be NULL; reset != 0 zeroes both after reading. */
int hiseg_placement_stats(long long* declined, long long* far, int reset);

/* A HIP stream whose kernels run only on the CUs whose bits are set in mask[0..nwords) (hipExtStreamCreateWithCUMask),
 * for the serving schedule's full-image UNet stream (hiseg.StreamPipelinedExport(cu_mask=...)); destroy with
 * hiseg_stream_destroy. */
int hiseg_stream_create_cu_mask(const unsigned* mask, int nwords, hiseg_stream_t* out);
int hiseg_stream_destroy(hiseg_stream_t s);

/* ----------------------------------------------------------------------------------------
 * Dynamic RoIAlign forward.
 * Replaces DynamicRoIAlign.forward (src/human_edge_detection/dynamic_roi_align.py:56-171):
 * endpoint-inclusive linspace grid (:110-134), [-1,1] normalisation (:139-146),
 * index_select + grid_sample(bilinear, zeros, align_corners=aligned) (:156-169).
 * Reads `feat` as NCHW f32 [B, C, H, W] (the reference's input layout); `rois` f32 [N, 5]
 * = [batch_idx, x1, y1, x2, y2] in [0,1].  Output pixel (n, i, j) of channel c goes to
 *   NHWC:  out[((n*oh + i)*ow + j)*o_cstride + o_coff + c]   (o_nchw == 0, dtype out_dtype)
 *   NCHW:  out[((n*Cout + c)*oh + i)*ow + j]                  (o_nchw == 1, f32 only)
 * If `aff_w` is non-null the sampled source is channel 0 of `feat` mapped per output
 * channel c as aff_w[c]*v + aff_b[c] BEFORE interpolation (this is the trainable 1->2
 * output_conv of PreTrainedPeopleSegmentationUNetWrapper, hierarchical_segmentation_unet.py
 * :1963-1971,1990, fused into the gather), Cout = n_aff; otherwise Cout = C.
 * Channels [Cout, zero_to) of an NHWC output are written with zeros (channel padding).
 * A batch index outside [0, B) yields zeros (the reference raises in index_select).
 * -------------------------------------------------------------------------------------- */
typedef struct hiseg_roi_align_desc {
  const float* feat; int B, C, H, W;
  const float* rois; int N;
  int oh, ow;
  float scale_h, scale_w;   /* DynamicRoIAlign.spatial_scale_h / _w                      */
  int aligned;              /* DynamicRoIAlign.aligned                                   */
  const float* aff_w; const float* aff_b; int n_aff;
  void* out; int out_dtype; int o_cstride; int o_coff; int o_nchw; int zero_to;
} hiseg_roi_align_desc;
int hiseg_roi_align_fwd(const hiseg_roi_align_desc* d, hiseg_stream_t stream);

/* ----------------------------------------------------------------------------------------
 * Implicit-GEMM convolution forward on MFMA (bf16 in / f32 accumulate, or exact f32).
 * Replaces nn.Conv2d (+ the following eval-mode nn.BatchNorm2d, activation, residual add,
 * attention multiply) at every conv site of the path: ResidualBlock
 * (advanced/hierarchical_segmentation_refinement.py:31-55, hierarchical_segmentation_unet.py
 * :35-58), rgb_feature_extractor (advanced/hierarchical_segmentation_rgb.py:657-673),
 * feature_combiner (:695, concat of :760 fused through the two-source loader),
 * EnhancedUNet (hierarchical_segmentation_unet.py:277-417), fg_gate / target branch /
 * contour / distance heads (hierarchical_segmentation_refinement.py:255-344,479-545) and the
 * smp UNet decoder (nearest x2 upsample + skip concat fused through src A up-factor 2).
 * With convT == 1 it is nn.ConvTranspose2d(k=2, s=2) (hierarchical_segmentation_unet.py:353
 * -355, refinement.py:502,515): a 1x1 GEMM over input pixels whose 4*Cout columns (q-major,
 * q = 2*dy+dx) are scattered to output pixel (2y+dy, 2x+dx).
 *
 * GEMM view: rows = output pixels (N*Ho*Wo), cols = Cout, K = KH*KW*(Ca+Cb).
 * Weights packed [Cout_pad][K_pad] with K index (ky*KW + kx)*(Ca+Cb) + ci.
 * Epilogue, per (pixel, co):  v = acc*scale[co] + shift[co]; v += residual; v = act(v);
 *                             v *= mul;  out = v;  out2 = v (optional duplicate store).
 * Input channel ci < Ca is read from src A (spatial (H/a_up, W/a_up), nearest), otherwise
 * channel ci-Ca from src B (spatial (H, W)).  If in_scale is set, src-A channel ci of image
 * n is multiplied by in_scale[n*Ca + ci] while loading (squeeze-excite gate fusion).
 * dtype applies to src A/B, weights, residual, mul, out2; out uses out_dtype.
 * -------------------------------------------------------------------------------------- */
typedef struct hiseg_conv2d_desc {
  int dtype, out_dtype;
  int N, H, W;              /* conv input grid (after src-A upsampling)                   */
  int Ho, Wo;               /* conv output grid (GEMM rows); for convT: Ho == H, Wo == W  */
  int KH, KW, stride, pad;
  const void* srcA; int a_cstride, a_coff, Ca, a_up;
  const void* srcB; int b_cstride, b_coff, Cb;
  const float* in_scale;
  const void* weight; int Cout, Cout_pad, K_pad;   /* Cout = GEMM cols (4*C for convT)    */
  const float* scale; const float* shift;          /* length >= Cout (GEMM cols)          */
  int act;
  const void* residual; int r_cstride, r_coff;
  const void* mul; int m_cstride, m_coff;
  void* out; int o_cstride, o_coff;
  void* out2; int o2_cstride, o2_coff;
  int convT;
  /* Optional second copy of the weights in MFMA-fragment order ([Cout_pad/16][nK][2][64][8],
   * nK = K_pad/64 K blocks in channel-block-major / tap-minor order) used by the 3x3 halo
   * kernel that streams weights straight into registers; null disables that kernel. */
  const void* weight_frag;
  float act_beta;           /* Swish beta (act == HISEG_ACT_SWISH); ignored otherwise        */
  /* Optional caller workspace (device memory, stream-ordered like the operands): the automatic
   * choice splits the K loop of a small-grid 1x1 layer -- or of a 3x3 layer over images of <= 256
   * pixels with K >= 1536 -- over workgroups when it holds at least hiseg_conv2d_workspace_bytes(d)
   * bytes; null keeps every layer unsplit.  The plan depends on the layer and the per-image grid only;
   * whether to pass a workspace for a 3x3 layer is the caller's choice (it pays for small batches). */
  void* workspace; long long workspace_bytes;
  /* Optional (train mode, the conv feeding a BatchNorm2d): when non-null the automatic choice writes the
   * BatchNorm batch-statistics partials of its bf16 output here -- [S][3][Cout] f32 (count, mean, M2
   * per channel over split s: a pixel tile's share of one wave), S = hiseg_conv2d_stats_tiles(d) --
   * for hiseg_bn_finalize_n
   * (advanced/normalization_comparison.py:181-182); the call fails when that is 0. */
  float* stats_partial;
  /* Optional (round 5, train mode, a data-gradient conv that alone writes the output gradient of a
   * conv -> BatchNorm2d -> ReLU / identity layer): when bnb_partial is non-null the automatic choice also
   * writes that BatchNorm's backward reduction from its epilogue -- per split s (S as
   * hiseg_conv2d_stats_tiles) and output channel c, over the split's pixels: sum g, sum g * xhat, sum xhat
   * with g = out * act'(bnb_z * bnb_scale + bnb_shift) (bnb_act HISEG_ACT_RELU; HISEG_ACT_NONE: g = out)
   * and xhat = (bnb_z - bnb_mean) * bnb_invstd -- into bnb_partial [S][3][Cout] for hiseg_bn_bwd
   * (hiseg_bn_bwd_desc.partial_splits = S); bnb_z is the BatchNorm's input (bf16, Cout channels), the
   * four tables its forward's folded affine and batch statistics.  Needs no activation / residual of its
   * own; the call fails when the layer has no such kernel. */
  float* bnb_partial; const void* bnb_z; int bnb_z_cstride, bnb_z_coff;
  const float* bnb_scale; const float* bnb_shift; const float* bnb_mean; const float* bnb_invstd; int bnb_act;
} hiseg_conv2d_desc;
int hiseg_conv2d_fwd(const hiseg_conv2d_desc* d, hiseg_stream_t stream);
/* sizeof of every descriptor struct of the C ABI, in the order roi_align_desc, conv2d_desc, wgrad_map, pack_entry,
 * bn_apply_desc, bn_bwd_desc, ln_bwd_desc, ew_view, ubf_desc, ubf_grads, loss_cfg, distill_cfg, roi_target_desc
 * (the first n of them into out); returns their count.  Bindings check their struct layouts against it. */
int hiseg_struct_sizes(long long* out, int n);
/* Workspace bytes hiseg_conv2d_fwd's automatic choice would use for this layer (0: none). */
long long hiseg_conv2d_workspace_bytes(const hiseg_conv2d_desc* d);
/* Splits S of the BatchNorm statistics partials the automatic choice fuses into this layer's
 * epilogue when d->stats_partial is set (bf16 3x3 halo-kernel layers with no activation / residual),
 * 0 when it does not (the caller then runs hiseg_bn_stats over the output). */
int hiseg_conv2d_stats_tiles(const hiseg_conv2d_desc* d);
/* Tuning/test entry: variant -1 forces the generic kernel, 0 = automatic choice (as
 * hiseg_conv2d_fwd), k > 0 selects pipelined-kernel configuration k when the layer qualifies
 * (99: the split-K generic kernel; it needs the workspace and fails when the layer does not split). */
int hiseg_conv2d_fwd_variant(const hiseg_conv2d_desc* d, int variant, hiseg_stream_t stream);

/* MaxPool2d(2) on NHWC (hierarchical_segmentation_unet.py:331-332,391).
 * in [N, H, W, C] (cstride == C), out [N, H/2, W/2, C]. */
int hiseg_maxpool2x2_fwd(int dtype, const void* in, int N, int H, int W, int C, void* out,
                         hiseg_stream_t stream);

/* SpatialAttentionModule (advanced/attention_modules.py:67-113): mean/max over C,
 * 7x7 conv 2->1 (no bias), sigmoid, x * map.  `w7` is the f32 [2][k][k] kernel.
 * `stats` is caller workspace of N*H*W*2 floats, `att` of N*H*W floats. */
int hiseg_attn_spatial_fwd(int dtype, const void* x, int N, int H, int W, int C, const float* w7,
                           int k, float* stats, float* att, void* out, hiseg_stream_t stream);

/* Global average pool + two 1x1 convs + sigmoid gate, shared by ChannelAttentionModule
 * (advanced/attention_modules.py:10-64: no bias, act = the module activation) and the
 * EfficientNet SqueezeExcite of the smp encoder (bias, SiLU).  x NHWC [N, HW, C] (cstride C).
 * w1 f32 [Cr][C], b1 [Cr] or null, w2 [C][Cr], b2 [C] or null.  Writes gate[N][C] (f32).
 * `partial` is workspace of N*splits*C floats (splits = hiseg_gap_splits(HW)), consumed. */
int hiseg_gap_splits(int HW);
int hiseg_se_gate_fwd(int dtype, const void* x, int N, int HW, int C, const float* w1,
                      const float* b1, int Cr, const float* w2, const float* b2, int act, float act_beta,
                      float* partial, float* gate, hiseg_stream_t stream);

/* y[n, p, c] = x[n, p, c] * gate[n, c]  (attention_modules.py:64). */
int hiseg_channel_scale_fwd(int dtype, const void* x, int N, int HW, int C, const float* gate,
                            void* out, hiseg_stream_t stream);

/* Depthwise KxK conv (stride s, pad K/2, no bias) + folded BN + activation on NHWC — the
 * conv_dw of the EfficientNet DepthwiseSeparable / InvertedResidual blocks of the smp
 * encoder (hierarchical_segmentation_unet.py:1770-1774 -> timm). w f32 [K*K][C]. */
int hiseg_dwconv_fwd(int dtype, const void* in, int N, int H, int W, int C, int K, int stride,
                     const float* w, const float* scale, const float* shift, int act, void* out,
                     int Ho, int Wo, hiseg_stream_t stream);
/* The same depthwise conv fused with the SqueezeExcite global average pool that consumes its output
 * (timm MBConv: conv_dw -> bn -> act -> se): gap_partial [N][parts][C] f32 receives per-tile channel
 * sums of the output (parts = hiseg_dw_gap_parts(dtype, N, Ho, Wo, C, K, stride): the kernel that takes the
 * layer fixes it); hiseg_se_gate_partials_fwd turns them into the gate [N][C] without re-reading the
 * activation.  hiseg_dw_gap_tiles(N, Ho, Wo) is the strip-range count of the register-gather kernel (the
 * layers hiseg_dw_gap_parts does not give to the LDS-tiled kernel). */
int hiseg_dw_gap_tiles(int N, int Ho, int Wo);
int hiseg_dw_gap_parts(int dtype, int N, int Ho, int Wo, int C, int K, int stride);
int hiseg_dwconv_gap_fwd(int dtype, const void* in, int N, int H, int W, int C, int K, int stride,
                         const float* w, const float* scale, const float* shift, int act, void* out,
                         int Ho, int Wo, float* gap_partial, hiseg_stream_t stream);
/* partial is consumed: after the pooled sums are read it holds intermediate values (the hidden units' partial
 * products).  Two launches when every 64-channel block's partial columns can hold Cr values, else three. */
int hiseg_se_gate_partials_fwd(float* partial, int splits, int N, int HW, int C, const float* w1,
                               const float* b1, int Cr, const float* w2, const float* b2, int act,
                               float* gate, hiseg_stream_t stream);

/* Image prologue of PreTrainedPeopleSegmentationUNet.normalize_input
 * (hierarchical_segmentation_unet.py:1885-1890) fused with NCHW f32 -> NHWC(dtype, C padded
 * to cpad) conversion.  The reference's host-synchronising `if x.max() > 1: x /= 255` is a
 * device-side flag: hiseg_image_max_fwd writes max(x) to *maxbuf (one float, caller
 * zero-initialises nothing: the call resets it), the normalize kernel reads it. */
int hiseg_image_max_fwd(const float* x, long long n, float* maxbuf, hiseg_stream_t stream);
int hiseg_input_norm_fwd(int dtype, const float* x, int B, int C, int H, int W, const float* maxbuf,
                         const float* mean, const float* std, void* out, int cpad,
                         hiseg_stream_t stream);

/* Hierarchical combine of ExtendedHierarchicalSegmentationHeadUNetV2.forward
 * (advanced/hierarchical_segmentation_refinement.py:559-596) fused with the whole
 * upsample_bg_fg branch (:501-506: ConvTranspose2d 2->32 k2s2, BN, act, 1x1 32->2) and the
 * final 1x1 128->2 of the target branch (:521).
 *   low  : f32 NHWC [N, h, w, 2]       bg_fg_logits_low
 *   tfeat: dtype NHWC [N, 2h, 2w, Ct]  target-branch features before its last 1x1 (cstride Ct)
 *   ut_w [2][32][2][2], ut_scale/ut_shift [32] (convT bias + BN folded; [N][32] per-sample
 *   tables when ut_per_sample), ut_act / ut_beta the branch activation, u1_w [2][32], u1_b[2]
 *   t_w [2][Ct], t_b [2]
 * Outputs (f32 NCHW): logits [N,3,2h,2w]; optional bgfg [N,2,2h,2w], tn [N,2,2h,2w]. */
int hiseg_hier_combine_fwd(int dtype, const float* low, int N, int h, int w, const void* tfeat,
                           int Ct, const float* ut_w, const float* ut_scale, const float* ut_shift,
                           int ut_act, float ut_beta, int ut_per_sample, const float* u1_w,
                           const float* u1_b, const float* t_w, const float* t_b, float* logits,
                           float* bgfg, float* tn, hiseg_stream_t stream);
/* upsample_bg_fg with LayerNorm2d (normalization_type 'layernorm2d', model.py:18-38): per-sample
 * statistics of z = ConvTranspose2d(low) (+ bias) over (32, 2h, 2w) -> mean/invstd [N] (optional)
 * and the folded tables scale/shift [N][32]: act(z * scale + shift) -- or, with fold_bias = 1, the
 * tables for the bias-free ConvTranspose sum that hiseg_hier_combine_fwd takes with
 * ut_per_sample = 1. */
int hiseg_ubf_ln_tables(const float* low, int N, int h, int w, const float* ut_w, const float* ut_b,
                        const float* gamma, const float* beta, float eps, int fold_bias, float* mean,
                        float* invstd, float* scale, float* shift, hiseg_stream_t stream);

/* NHWC(dtype, cstride, coff) -> NCHW f32 copy of C channels (aux outputs of the reference's
 * forward dict are NCHW f32). */
int hiseg_nhwc_to_nchw_fwd(int dtype, const void* in, int N, int H, int W, int C, int cstride,
                           int coff, float* out, hiseg_stream_t stream);
/* NCHW f32 -> NHWC(dtype) with channel padding (zeros in [C, cpad)). */
int hiseg_nchw_to_nhwc_fwd(int dtype, const float* in, int N, int C, int H, int W, void* out,
                           int cpad, hiseg_stream_t stream);

/* Exported inference contract (src/human_edge_detection/export_onnx_advanced.py:360-392):
 * instance = (argmax_c logits == 1) as f32 {0,1} [N,1,mh,mw];  binary = softmax over the two
 * output_conv channels of the UNet logit u, channel 0 = softmax([w0*u+b0, w1*u+b1])[0],
 * [B,1,H,W] f32.  Optional MaskDilationModule (export_hierarchical_instance_peopleseg_onnx.py
 * :85-141) with `dilation` > 0 is applied to the logits first (in place on a copy). */
int hiseg_instance_masks_fwd(const float* logits, int N, int mh, int mw, int dilation,
                             float* instance, hiseg_stream_t stream);
int hiseg_binary_masks_fwd(int dtype, const void* u, int u_cstride, int B, int H, int W,
                           const float* oc_w, const float* oc_b, float* binary,
                           hiseg_stream_t stream);

/* Bilinear resize, align_corners=False (F.interpolate as used for the contour / distance aux
 * maps, advanced/hierarchical_segmentation_refinement.py:775-800).  NCHW f32, NC planes. */
int hiseg_resize_bilinear_fwd(const float* in, int NC, int H, int W, float* out, int Ho, int Wo,
                              hiseg_stream_t stream);

/* DistanceTransformDecoder mask (refinement.py:342): out = sigmoid((x - *threshold) * 10);
 * `threshold` is a device pointer (the learnable parameter), n elements. */
int hiseg_distance_mask_fwd(const float* x, long long n, const float* threshold, float* out,
                            hiseg_stream_t stream);

/* 1x1 conv 1 -> 2 of PreTrainedPeopleSegmentationUNetWrapper.output_conv
 * (hierarchical_segmentation_unet.py:1963-1971,1990): u [B,1,H,W] -> out [B,2,H,W], f32. */
int hiseg_output_conv_fwd(const float* u, int B, int H, int W, const float* w, const float* b, float* out,
                          hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HISEG_H_ */

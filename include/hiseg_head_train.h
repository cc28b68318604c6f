/*
 * hiseg_head_train.h — training entry points of libhiseg for the refined hierarchical head's
 * non-convolution ops and the pretrained-UNet output_conv (train forward with saved state,
 * and backward).  Conventions as in hiseg.h / hiseg_train.h.
 */
#ifndef HISEG_HEAD_TRAIN_H_
#define HISEG_HEAD_TRAIN_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* SpatialAttentionModule (advanced/attention_modules.py:67-113) followed by the head's
 * Dropout2d (refinement.py:519): out = x * sigmoid(conv7x7([mean_c x, max_c x])) * chan_mul.
 * Saves stats [P][2], argmax [P] (first max channel, the gradient route of torch.max) and
 * att [P] for the backward.  x: dense NHWC (cstride == C). */
int hiseg_attn_spatial_train_fwd(int dtype, const void* x, int N, int H, int W, int C, const float* w7, int k,
                                 const float* chan_mul, float* stats, int* argmax, float* att, void* out,
                                 hiseg_stream_t stream);
/* f32 workspace size (elements) of hiseg_attn_spatial_bwd */
int hiseg_attn_spatial_ws(int N, int H, int W, int k);
/* dx = d out/dx (written); dw7 += d out/d w7. */
int hiseg_attn_spatial_bwd(int dtype, const void* x, int N, int H, int W, int C, const float* w7, int k,
                           const float* chan_mul, const float* stats, const int* argmax, const float* att,
                           const void* dout, void* dx, float* ws, float* dw7, hiseg_stream_t stream);

/* ChannelAttentionModule (attention_modules.py:10-64, fc1/fc2 without bias) followed by the
 * head's Dropout2d (refinement.py:525): out = x * sigmoid(W2 act(W1 gap(x))) * chan_mul.
 * Saves gap [N][C], hpre [N][Cr] (pre-activation), gate [N][C]. */
int hiseg_attn_channel_ws(int N, int C, int Cr);
int hiseg_attn_channel_train_fwd(int dtype, const void* x, int N, int HW, int C, const float* w1, int Cr,
                                 const float* w2, int act, float act_beta, const float* chan_mul, float* ws, float* gap,
                                 float* hpre, float* gate, void* out, hiseg_stream_t stream);
/* dx written; dw1 [Cr][C] += ..., dw2 [C][Cr] += ... */
int hiseg_attn_channel_bwd(int dtype, const void* x, int N, int HW, int C, const float* w1, int Cr, const float* w2,
                           int act, float act_beta, const float* chan_mul, const float* gap, const float* hpre,
                           const float* gate, const void* dout, void* dx, float* ws, float* dw1, float* dw2,
                           hiseg_stream_t stream);

/* upsample_bg_fg [ConvTranspose2d(2,32,2,s2), BatchNorm2d(32) train, ReLU, Conv2d(32,2,1)],
 * softmax, the target branch's last Conv2d(Ct,2,1) and the hierarchical combine
 * (refinement.py:501-506, 527-531, 559-596):
 *   logits[:,0] = b0, logits[:,1] = b1 + t0*p_fg, logits[:,2] = b1 + t1*p_fg, p_fg = softmax(b)[1]
 * low: f32 [N][h][w][2] (EnhancedUNet output); tfeat: [N][2h][2w][Ct] compute dtype;
 * logits/bgfg/tn: NCHW f32 [N][3|2|2][2h][2w].  The train forward computes the BN batch
 * statistics of the ConvTranspose output into mean/invstd/scale/shift (caller buffers of 32)
 * and updates the running statistics -- or, with layernorm = 1, the per-sample LayerNorm2d
 * statistics (buffers of N and N*32, running_mean/var unused). */
typedef struct hiseg_ubf_desc {
  int dtype;
  const float* low; int N, h, w;
  const float* ut_w; const float* ut_b;
  const float* gamma; const float* beta;
  float* mean; float* invstd; float* scale; float* shift;
  const float* u1_w; const float* u1_b;
  const void* tfeat; int Ct; const float* t_w; const float* t_b;
  float* logits; float* bgfg; float* tn;
  int act; float act_beta;        /* branch activation (refinement.py:503): ReLU in every preset */
  int layernorm;                  /* 0: BatchNorm2d(32) train (mean/invstd/scale/shift [32], running update);
                                   * 1: LayerNorm2d (model.py:18-38): mean/invstd [N], scale/shift [N][32] */
} hiseg_ubf_desc;
typedef struct hiseg_ubf_grads {
  float* dut_w; float* dut_b; float* dgamma; float* dbeta; float* du1_w; float* du1_b;   /* accumulated */
} hiseg_ubf_grads;
int hiseg_ubf_ws(int N);
int hiseg_ubf_train_fwd(const hiseg_ubf_desc* d, float eps, float momentum, float* running_mean, float* running_var,
                        float* ws, hiseg_stream_t stream);
/* dlogits: NCHW f32 gradient of logits; dbgfg_ext / dtn_ext: extra gradients of the bgfg / tn
 * outputs (the loss's auxiliary terms) or null.  Writes dtn_out [P][2] (gradient of the target
 * logits, consumed by hiseg_pw2_bwd), dlow [N][h][w][2] f32; db_buf [P][2] scratch. */
int hiseg_ubf_train_bwd(const hiseg_ubf_desc* d, const float* dlogits, const float* dbgfg_ext, const float* dtn_ext,
                        float* db_buf, float* dtn_out, float* dlow, float* ws, const hiseg_ubf_grads* g,
                        hiseg_stream_t stream);

/* Backward of the target branch's last Conv2d(Ct, 2, 1) (refinement.py:527): dt [P][Ct] written
 * (compute dtype), dw [2][Ct] += , db [2] += . */
int hiseg_pw2_ws(int Ct);
int hiseg_pw2_bwd(int dtype, const void* tfeat, long long P, int Ct, const float* dtn, const float* w, void* dt,
                  float* ws, float* dw, float* db, hiseg_stream_t stream);

/* DynamicRoIAlign backward into the trainable output_conv (hierarchical_segmentation_unet.py
 * :1963-1971 feeding dynamic_roi_align.py:56-171): with roi logits r_c = interp(w_c*u + b_c),
 *   dw_c += sum g_c * interp(u),  db_c += sum g_c * interp(1)   (taps outside the map are 0).
 * g: the RoIAlign output gradient, NHWC [N][oh][ow] with channel stride g_cstride, offset
 * g_coff, dtype g_dtype; u: f32 [B][1][H][W]. */
int hiseg_roi_align_ws(int N);
int hiseg_roi_align_bwd_affine(const hiseg_roi_align_desc* d, const void* g, int g_dtype, int g_cstride, int g_coff,
                               float* ws, float* dw, float* db, hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif  /* HISEG_HEAD_TRAIN_H_ */

/*
 * hiseg_distill.h — UNet knowledge-distillation loss on the GPU
 * (advanced/unet_decoder_distillation.py:338-663, UNetDistillationLoss.forward, and the gradient of its
 * total w.r.t. the student logits).  Conventions as in hiseg.h.
 *
 * Inputs NCHW f32 [B][1][H][W]: student and teacher logits, targets (binary masks, f32) or null.
 * The loss state the reference keeps on the host (temperature, alpha, task weight, adaptive flags,
 * performance ratio) is passed by value; every per-element term and reduction runs on the device:
 *   kl   = clamp(mean(pt (log(pt+e) - log(ps+e)) + (1-pt)(log(1-pt+e) - log(1-ps+e))), 0, 5),
 *          ps/pt = clamp(sigmoid(clamp(x, -10, 10) / T), e, 1-e), e = 1e-5
 *   mse  = mean((s - t)^2)
 *   bce  = BCEWithLogits(s, y, pos_weight) (mean),  dice = 1 - mean_b (2 I_b + 1e-5) / (P_b + Y_b + 1e-5)
 *   task = 0.7 bce + 0.3 dice (or bce),  distill = kw kl + (1-kw) mse,  kw = min(alpha_eff, 0.1)
 *   total = tw task + (1-tw) distill  (targets) | distill (no targets)
 * Non-finite totals take the reference's fallbacks (:650-659): the task loss (targets, task not NaN), else the
 * MSE term (not NaN), else a constant 1.0 with a zero gradient; the gradient is that of the value returned.
 * loss_dict values that are NaN are reported as 0 (:571-590); clamps keep NaN (torch.clamp).
 */
#ifndef HISEG_DISTILL_H_
#define HISEG_DISTILL_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hiseg_distill_cfg {
  float temperature;
  float kl_weight;        /* min(alpha_eff, 0.1) */
  float task_weight;      /* tw (effective) */
  float pos_weight;       /* sqrt((1 - fg_ratio) / fg_ratio) */
  int distill_terms;      /* 0: kl and mse are skipped (reported 0) -- eliminated / disabled distillation */
  int distill_in_total;   /* 0: distillation_loss = 0 in the total (alpha == 0 with adaptive, or tw >= 0.99) */
  int use_dice;
  int has_target;
  /* optional device f32[4] {temperature, kl_weight, task_weight, pos_weight}: when non-null the kernels read these
   * four at run time instead of the fields above (a captured distillation step follows the per-epoch temperature
   * schedule, train_distillation_staged.py:1597-1610, without a re-capture); the host fields still pass the checks */
  const float* dev_scalars;
} hiseg_distill_cfg;

enum { HISEG_DISTILL_TOTAL = 0, HISEG_DISTILL_KL, HISEG_DISTILL_MSE, HISEG_DISTILL_BCE, HISEG_DISTILL_DICE,
       HISEG_DISTILL_NOUT };

/* f32 workspace elements for B samples of H x W */
long long hiseg_distill_ws(int B, int H, int W);
/* out: HISEG_DISTILL_NOUT f32 on the device (total, kl, mse, bce, dice). */
int hiseg_distill_loss_fwd(const hiseg_distill_cfg* cfg, int B, int H, int W, const float* student,
                           const float* teacher, const float* target, float* ws, float* out, hiseg_stream_t stream);
/* dstudent = grad_out[0] * d total / d student (NCHW f32), from the coefficients left in ws. */
int hiseg_distill_loss_bwd(const hiseg_distill_cfg* cfg, int B, int H, int W, const float* student,
                           const float* teacher, const float* target, const float* ws, const float* grad_out,
                           float* dstudent, hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif  /* HISEG_DISTILL_H_ */

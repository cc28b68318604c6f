/*
 * hiseg_loss.h — RefinedHierarchicalLoss on the GPU (advanced/hierarchical_segmentation_refinement.py
 * :807-1068 over advanced/hierarchical_segmentation.py:150-395 and losses.py:9-88), forward and
 * backward, with the dynamic class-weight EMA state kept on the device (no host round trip;
 * the reference reads it back with .item() every call).  Conventions as in hiseg.h.
 *
 * Inputs are NCHW f32: pred [N][3][H][W], bgfg [N][2][H][W], tn [N][2][H][W],
 * cont [N][1][H][W] (the contour branch's sigmoid output), dist [N][1][H][W]; targets int64
 * [N][H][W] with classes {0,1,2}.
 */
#ifndef HISEG_LOSS_H_
#define HISEG_LOSS_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hiseg_loss_cfg {
  float bg_weight, fg_weight, target_weight, consistency_weight, dice_weight, ce_weight;
  float boundary_aware_weight, contour_weight /* resolution-adjusted, refinement.py:951-963 */, distance_weight;
  int use_dynamic_weights, use_boundary_aware, use_contour, use_distance;
  int contour_ks;   /* dilation kernel 2*edge_width-1 (1 = none), refinement.py:1018-1038 */
} hiseg_loss_cfg;

/* Outputs (f32, device, HISEG_LOSS_NOUT + 1 values) of hiseg_loss_fwd, index constants; element
 * [HISEG_LOSS_NOUT] is the base HierarchicalLoss total (the reference's loss_dict['total_loss']). */
enum {
  HISEG_LOSS_TOTAL = 0, HISEG_LOSS_BGFG, HISEG_LOSS_TN, HISEG_LOSS_FINAL, HISEG_LOSS_CONS, HISEG_LOSS_DICE,
  HISEG_LOSS_BA, HISEG_LOSS_CONTOUR, HISEG_LOSS_DIST, HISEG_LOSS_ACC, HISEG_LOSS_IOU, HISEG_LOSS_W_BG,
  HISEG_LOSS_W_FG, HISEG_LOSS_W_T, HISEG_LOSS_W_NT, HISEG_LOSS_NOUT
};

/* Device state: double[8] = ema_bg, ema_fg, ema_t, ema_nt, tn_initialised, last_t, last_nt, calls;
 * initialise with hiseg_loss_state_init. */
int hiseg_loss_state_init(double* state, hiseg_stream_t stream);
/* f32 workspace elements for N ROIs of H x W */
long long hiseg_loss_ws(int N, int H, int W);
int hiseg_loss_fwd(const hiseg_loss_cfg* cfg, int N, int H, int W, const float* pred, const float* bgfg,
                   const float* tn, const float* cont, const float* dist, const long long* targets, double* state,
                   float* ws, float* out, hiseg_stream_t stream);
/* hiseg_loss_fwd in two phases, for data-parallel training: _begin rasterises the per-pixel targets and
 * writes this batch's 4 class pixel counts (bg, fg, target, non-target; double[4], optional) -- the caller
 * all-reduces them over the ranks -- and _end updates the dynamic class weights' EMA from `counts` (null:
 * this batch's own counts, i.e. hiseg_loss_fwd) before the loss terms (hierarchical_segmentation.py:227-255,
 * 286-309: the weights come from the counts of the whole batch, which under data parallelism spans the
 * ranks).  Same ws for both phases and for hiseg_loss_bwd. */
int hiseg_loss_fwd_begin(const hiseg_loss_cfg* cfg, int N, int H, int W, const long long* targets, float* ws,
                         double* counts, hiseg_stream_t stream);
int hiseg_loss_fwd_end(const hiseg_loss_cfg* cfg, int N, int H, int W, const float* pred, const float* bgfg,
                       const float* tn, const float* cont, const float* dist, const long long* targets,
                       const double* counts, double* state, float* ws, float* out, hiseg_stream_t stream);
/* Gradients (written, NCHW f32, same shapes) of grad_out[0] * total; any output may be null. Uses the
 * coefficients hiseg_loss_fwd left in ws. */
int hiseg_loss_bwd(const hiseg_loss_cfg* cfg, int N, int H, int W, const float* pred, const float* bgfg,
                   const float* tn, const float* cont, const float* dist, const long long* targets, const float* ws,
                   const float* grad_out, float* dpred, float* dbgfg, float* dtn, float* dcont, float* ddist,
                   hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif  /* HISEG_LOSS_H_ */

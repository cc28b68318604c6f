/*
 * hiseg_metrics.h — validation metrics of the ROI masks on the GPU (train_utils.py:109-402, evaluate_model;
 * the per-sample IoU and confusion loops of :279-318 over calculate_iou :14-22 and
 * calculate_confusion_matrix :25-47).  Conventions as in hiseg.h.
 *
 * The reference moves the predicted classes to the host and counts them with one boolean reduction (and
 * one .item()) per (sample, class) and per (sample, target, prediction) pair.  Every metric it reports is
 * a function of one small per-sample histogram, so one HBM pass builds that histogram for all samples:
 *
 *   conf[n][t][p] += #{ pixels of sample n with target row t and predicted column p }
 *
 * rows    t = target value for 0 <= target < C;  t = C for target >= C;  t = C+1 for target < 0
 * columns p = predicted class (argmax over the C logits: first maximum, NaN counts as the maximum,
 *             as torch.argmax), or for class-label input p = label for 0 <= label < C, p = C otherwise
 *
 * so that the IoUs (pred == c vs target == c), the 3x3 confusion matrix, the background-vs-target matrix
 * (target == 1 vs pred == 1, every other target value counting as background) and the target-vs-nontarget
 * matrix over target > 0 are all exact sums of conf entries.
 */
#ifndef HISEG_METRICS_H_
#define HISEG_METRICS_H_

#include "hiseg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Accumulates into conf (uint64, [N][C+2][C+1], zeroed by the caller for a fresh count).
 *   logits       [N][C][HW] (NCHW) of dtype HISEG_F32 or HISEG_BF16, or null when pred_labels is given
 *   pred_labels  int64 [N][HW] predicted class ids (used when logits is null)
 *   target       int64 [N][HW]
 * 2 <= C <= 4.  Reads 4*C (f32) + 8 bytes per pixel once; no host synchronisation. */
int hiseg_seg_confusion(const void* logits, int dtype, const long long* pred_labels, const long long* target,
                        int N, int C, long long HW, unsigned long long* conf, hiseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif

"""Validation-metrics CPU restatement -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

numpy restatement of the metric part of evaluate_model (src/human_edge_detection/train_utils.py:109-402):
per-sample IoU per class (calculate_iou :14-22, loop :302-313), the 3x3 confusion matrix
(calculate_confusion_matrix :25-47, :279-280), the background-vs-target and target-vs-nontarget
matrices (:282-300), detection rates (calculate_detection_metrics :85-106) and the derived accuracies
(:325-372).  It follows the reference's own per-sample formulation (boolean masks per sample and class),
not the histogram the GPU path reduces to, so the two are independent.

Pinned to tests/golden/metrics.npz: the reference's evaluate_model itself run in the build container
on recorded logits / masks (tests/golden/gen_metrics_golden.py).
"""
from __future__ import annotations

from typing import Dict, Iterable, Tuple

import numpy as np


def calculate_iou(pred: np.ndarray, target: np.ndarray) -> float:
    """train_utils.py:14-22 (boolean masks; float32 sums and division as torch)."""
    inter = np.float32(np.logical_and(pred, target).sum())
    union = np.float32(np.logical_or(pred, target).sum())
    if union == 0:
        return 1.0 if inter == 0 else 0.0
    return float(np.float32(inter / union))


def calculate_detection_metrics(ious, thresholds=(0.5, 0.7)) -> Dict[str, float]:
    """train_utils.py:85-106."""
    if not ious:
        return {f"detection_rate_{t}": 0.0 for t in thresholds}
    a = np.array(ious)
    return {f"detection_rate_{t}": (a > t).mean() for t in thresholds}


def evaluate_metrics(batches: Iterable[Tuple[np.ndarray, np.ndarray]], num_classes: int = 3) -> Dict[str, object]:
    """batches: (logits [N,C,H,W] float, masks [N,H,W] int).  Returns the metric keys of evaluate_model
    (iou_class_*, target_iou, miou, detection rates, accuracies, the three confusion matrices)."""
    class_ious = {c: [] for c in range(num_classes)}
    target_ious = []
    conf_total = np.zeros((num_classes, num_classes), np.int64)
    conf_bt = np.zeros((2, 2), np.int64)
    conf_tn = np.zeros((2, 2), np.int64)
    for logits, masks in batches:
        pred = np.argmax(logits, axis=1)                                     # :277
        pf, tf = pred.reshape(-1), masks.reshape(-1)
        for t in range(num_classes):                                          # :43-45
            for p in range(num_classes):
                conf_total[t, p] += np.sum((tf == t) & (pf == p))
        pbt, tbt = (pred == 1).astype(np.int64), (masks == 1).astype(np.int64)   # :286-287
        for i in range(pred.shape[0]):
            for t in range(2):
                for p in range(2):
                    conf_bt[t, p] += np.sum((tbt[i] == t) & (pbt[i] == p))
            fg = masks[i] > 0                                                 # :296
            if fg.any():
                ptn = (pred[i] == 2).astype(np.int64)[fg]
                ttn = (masks[i] == 2).astype(np.int64)[fg]
                for t in range(2):
                    for p in range(2):
                        conf_tn[t, p] += np.sum((ttn == t) & (ptn == p))
        for c in range(num_classes):                                          # :303-313
            for i in range(pred.shape[0]):
                iou = calculate_iou(pred[i] == c, masks[i] == c)
                class_ious[c].append(iou)
                if c == 1:
                    target_ious.append(iou)
    m: Dict[str, object] = {}
    for c in range(num_classes):                                              # :325-330
        m[f"iou_class_{c}"] = sum(class_ious[c]) / len(class_ious[c]) if class_ious[c] else 0.0
    m["target_iou"] = sum(target_ious) / len(target_ious) if target_ious else 0.0
    m["miou"] = m["target_iou"]
    m.update(calculate_detection_metrics(target_ious))
    if conf_total.sum() > 0:                                                  # :346-347
        m["overall_accuracy"] = np.diag(conf_total).sum() / conf_total.sum()
    if conf_bt.sum() > 0:                                                     # :350-370
        tp, fp, fn = conf_bt[1, 1], conf_bt[0, 1], conf_bt[1, 0]
        m["target_precision"] = tp / (tp + fp) if tp + fp > 0 else 0.0
        m["target_recall"] = tp / (tp + fn) if tp + fn > 0 else 0.0
        pr, rc = m["target_precision"], m["target_recall"]
        m["target_f1"] = 2 * (pr * rc) / (pr + rc) if pr + rc > 0 else 0.0
    if conf_tn.sum() > 0:                                                     # :373-376
        m["instance_separation_accuracy"] = np.diag(conf_tn).sum() / conf_tn.sum()
    m["conf_matrix_total"] = conf_total
    m["conf_matrix_bg_target"] = conf_bt
    m["conf_matrix_target_nontarget"] = conf_tn
    return m

"""Validation metrics on the GPU (src/human_edge_detection/train_utils.py:14-106 helpers, :109-402
evaluate_model).

Same names, arguments and returned keys as the reference.  The reference moves the predicted classes to
the host and reduces one boolean mask (plus one ``.item()``) per (sample, class) and per confusion cell;
here one HIP pass (``hiseg_seg_confusion``, include/hiseg_metrics.h) builds a per-sample
(target row, predicted column) histogram on the device -- argmax fused -- and every reported number is an
exact integer sum of its cells.  The loss values are kept on the device as well, so the evaluation loop
does not synchronise per batch: the histograms and loss values come to the host in one copy each after
the last batch, where the reference's float arithmetic (float32 IoU division, Python sums in the same
order, numpy ratios) is reproduced exactly.
"""
from __future__ import annotations

import warnings
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L
from .losses import LazyLossDict


def _hdtype(dt: torch.dtype) -> int:
    from .ops import hdtype
    return hdtype(dt)


def seg_confusion(pred: torch.Tensor, target: torch.Tensor, num_classes: int = 3,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-sample histogram int64 [N, C+2, C+1] (rows: target 0..C-1, >=C, <0; columns: predicted class
    0..C-1, other).  ``pred``: logits [N, C, H, W] (f32/bf16; argmax = first maximum, NaN maximal, as
    torch.argmax) or class labels [N, H, W] (integer).  Accumulates into ``out`` when given."""
    if not (pred.is_cuda and target.is_cuda):
        raise RuntimeError("hiseg metrics run on the GPU only (got a CPU tensor)")
    C = num_classes
    N = target.shape[0]
    HW = target.numel() // N if N else 0
    if out is None:
        out = torch.zeros(N, C + 2, C + 1, dtype=torch.int64, device=target.device)
    if N == 0 or HW == 0:
        return out
    tg = target.to(torch.int64).contiguous()
    lib = L.lib()
    if pred.dim() == target.dim() + 1:       # logits
        if pred.shape[1] != C or pred.shape[0] != N or pred[0, 0].numel() != HW:
            raise ValueError(f"seg_confusion: logits {tuple(pred.shape)} vs target {tuple(target.shape)}")
        if pred.dtype not in (torch.float32, torch.bfloat16):
            pred = pred.float()
        lg = pred.contiguous()
        L.check(lib.hiseg_seg_confusion(lg.data_ptr(), _hdtype(lg.dtype), None, tg.data_ptr(), N, C, HW,
                                        out.data_ptr(), L.stream_ptr()), "seg_confusion")
    else:
        if tuple(pred.shape) != tuple(target.shape):
            raise ValueError(f"seg_confusion: labels {tuple(pred.shape)} vs target {tuple(target.shape)}")
        lb = pred.to(torch.int64).contiguous()
        L.check(lib.hiseg_seg_confusion(None, 0, lb.data_ptr(), tg.data_ptr(), N, C, HW, out.data_ptr(),
                                        L.stream_ptr()), "seg_confusion")
    return out


def calculate_confusion_matrix(pred: torch.Tensor, target: torch.Tensor, num_classes: int = 3) -> torch.Tensor:
    """train_utils.py:25-47: int64 [C, C] counts of (target == t) & (pred == p) over all pixels (device)."""
    conf = seg_confusion(pred.reshape(pred.shape[0], -1) if pred.dim() > 1 else pred.reshape(1, -1),
                         target.reshape(target.shape[0], -1) if target.dim() > 1 else target.reshape(1, -1),
                         num_classes)
    return conf[:, :num_classes, :num_classes].sum(0)


def calculate_iou(pred: torch.Tensor, target: torch.Tensor) -> float:
    """train_utils.py:14-22 for two boolean masks (one 2-class histogram on the device)."""
    conf = seg_confusion(pred.reshape(1, -1).to(torch.int64), target.reshape(1, -1).to(torch.int64), 2)[0]
    c = conf.cpu().numpy()
    inter = int(c[1, 1])
    union = int(c[:, 1].sum() + c[1, :].sum()) - inter
    return _iou(inter, union)


def calculate_detection_metrics(ious: list, thresholds: Sequence[float] = (0.5, 0.7)) -> dict:
    """train_utils.py:85-106 (host arithmetic on the per-sample IoUs)."""
    if not ious:
        return {f"detection_rate_{t}": 0.0 for t in thresholds}
    a = np.array(ious)
    return {f"detection_rate_{t}": (a > t).mean() for t in thresholds}


def _iou(inter: int, union: int) -> float:
    # float32 sums and division, as (intersection / union).item() on float tensors
    if union == 0:
        return 1.0 if inter == 0 else 0.0
    return float(np.float32(inter) / np.float32(union))


class SegmentationMetrics:
    """Device-side accumulator of evaluate_model's mask metrics (train_utils.py:150-158, 276-318, 320-402).

    ``update(pred_logits, masks)`` launches one histogram kernel and never synchronises; ``compute()``
    copies the histograms once and returns the reference's keys: iou_class_{c}, target_iou, miou,
    detection_rate_{0.5,0.7}, overall_accuracy, target_precision/recall/f1,
    instance_separation_accuracy and the three confusion matrices (numpy int64)."""

    def __init__(self, num_classes: int = 3):
        if num_classes != 3:
            raise ValueError("evaluate_model's metrics are defined for the 3-class hierarchy (bg/target/non-target)")
        self.C = num_classes
        self._confs: List[torch.Tensor] = []

    def reset(self):
        self._confs.clear()

    def update(self, pred: torch.Tensor, masks: torch.Tensor) -> None:
        self._confs.append(seg_confusion(pred.detach(), masks, self.C))

    def histograms(self) -> np.ndarray:
        if not self._confs:
            return np.zeros((0, self.C + 2, self.C + 1), np.int64)
        return torch.cat(self._confs).cpu().numpy()

    def compute(self) -> Dict[str, object]:
        return metrics_from_histograms(self.histograms(), self.C)


def metrics_from_histograms(h: np.ndarray, C: int = 3) -> Dict[str, object]:
    """The reference's metric arithmetic (train_utils.py:320-402) from per-sample histograms [S, C+2, C+1]
    in evaluation order (batch-major, then sample)."""
    m: Dict[str, object] = {}
    inter = np.stack([h[:, c, c] for c in range(C)], 1)          # [S, C]
    n_pred = h.sum(1)[:, :C]                                      # pred == c over every target value
    n_tgt = h.sum(2)[:, :C]                                       # target == c over every prediction
    union = n_pred + n_tgt - inter
    class_ious = [[_iou(int(i), int(u)) for i, u in zip(inter[:, c], union[:, c])] for c in range(C)]
    for c in range(C):
        m[f"iou_class_{c}"] = sum(class_ious[c]) / len(class_ious[c]) if class_ious[c] else 0.0
    target_ious = class_ious[1]
    m["target_iou"] = sum(target_ious) / len(target_ious) if target_ious else 0.0
    m["miou"] = m["target_iou"]
    m.update(calculate_detection_metrics(target_ious))
    tot = h.sum(0)                                                # [C+2, C+1]
    conf_total = tot[:C, :C].copy()
    all_px = tot.sum()
    bt11 = tot[1, 1]
    bt10 = tot[1, :].sum() - bt11
    bt01 = tot[:, 1].sum() - bt11
    conf_bt = np.array([[all_px - bt11 - bt10 - bt01, bt01], [bt10, bt11]], np.int64)
    fg_rows = [r for r in range(1, C + 1) if r != 2]              # target > 0 and != 2 (incl. >= C)
    tn11 = tot[2, 2]
    tn10 = tot[2, :].sum() - tn11
    tn01 = sum(tot[r, 2] for r in fg_rows)
    tn00 = sum(tot[r, :].sum() - tot[r, 2] for r in fg_rows)
    conf_tn = np.array([[tn00, tn01], [tn10, tn11]], np.int64)
    if conf_total.sum() > 0:
        m["overall_accuracy"] = np.diag(conf_total).sum() / conf_total.sum()
    if conf_bt.sum() > 0:
        tp, fp, fn = conf_bt[1, 1], conf_bt[0, 1], conf_bt[1, 0]
        m["target_precision"] = tp / (tp + fp) if tp + fp > 0 else 0.0
        m["target_recall"] = tp / (tp + fn) if tp + fn > 0 else 0.0
        pr, rc = m["target_precision"], m["target_recall"]
        m["target_f1"] = 2 * (pr * rc) / (pr + rc) if pr + rc > 0 else 0.0
    if conf_tn.sum() > 0:
        m["instance_separation_accuracy"] = np.diag(conf_tn).sum() / conf_tn.sum()
    m["conf_matrix_total"] = conf_total
    m["conf_matrix_bg_target"] = conf_bt
    m["conf_matrix_target_nontarget"] = conf_tn
    return m


def _value(v) -> float:
    return v.item() if isinstance(v, torch.Tensor) else v


def evaluate_model(model, dataloader, loss_fn, device: str, feature_extractor: Optional[object] = None,
                   config: Optional[object] = None, epoch: Optional[int] = None,
                   output_dir: Optional[object] = None) -> Dict[str, object]:
    """train_utils.py:109-402 for the RGB hierarchical model: ``model(images, rois) -> (logits, aux)``,
    ``loss_fn(logits, masks, aux) -> (loss, loss_dict)``; batches are dicts with 'image', 'roi_boxes',
    'roi_masks'.  Returns the reference's keys.  No host synchronisation inside the loop."""
    if config is not None:
        mc = getattr(config, "model", None)
        if getattr(getattr(config, "distillation", None), "enabled", False) or not (
                getattr(mc, "use_rgb_hierarchical", False) or getattr(mc, "use_hierarchical", False)):
            raise NotImplementedError("hiseg.evaluate_model covers the RGB hierarchical model (SURVEY.md §8a)")
    if feature_extractor is not None:
        raise NotImplementedError("feature_extractor (base models) is outside the RGB hierarchical path")
    model.eval()
    acc = SegmentationMetrics(3)
    losses: List[torch.Tensor] = []
    dicts = []
    with torch.no_grad():
        for batch in dataloader:
            images = batch["image"].to(device)
            rois = batch["roi_boxes"].to(device)
            masks = batch["roi_masks"].to(device)
            predictions = model(images, rois)
            if isinstance(predictions, tuple):
                logits, aux = predictions
                loss, loss_dict = loss_fn(logits, masks, aux)
            else:
                logits = predictions
                loss, loss_dict = loss_fn(logits, masks, {})
            losses.append(loss.detach().reshape(()))
            dicts.append(loss_dict)
            acc.update(logits, masks)
    if not losses:
        raise ZeroDivisionError("evaluate_model: empty dataloader (the reference divides by num_batches = 0)")
    # one transfer for the totals and one for every lazily held loss dict
    totals = [float(x) for x in torch.stack([t.to(losses[0].device).float() for t in losses]).cpu().tolist()]
    lazy = [d for d in dicts if isinstance(d, LazyLossDict) and d._vals is None]
    if lazy:
        host = torch.stack([d._out.detach() for d in lazy]).cpu().tolist()
        for d, h in zip(lazy, host):
            d._materialise(h)
    n = len(losses)
    total_loss = total_ce = total_dice = 0.0
    aux_fg_bg = aux_acc = aux_iou = 0.0
    active = boundary = contour = distance = 0.0
    for t, d in zip(totals, dicts):                                  # :245-264, in batch order
        total_loss += t
        total_ce += _value(d.get("ce_loss", d.get("base_ce_loss", 0)))
        total_dice += _value(d.get("dice_loss", d.get("base_dice_loss", 0)))
        aux_fg_bg += d.get("aux_fg_bg_loss", 0)
        aux_acc += d.get("aux_fg_accuracy", 0)
        aux_iou += d.get("aux_fg_iou", 0)
        active += d.get("active_contour", 0)
        boundary += d.get("boundary_aware", 0)
        contour += d.get("contour", 0)
        distance += d.get("distance_transform", 0)
    metrics: Dict[str, object] = {"total_loss": total_loss / n, "ce_loss": total_ce / n, "dice_loss": total_dice / n}
    if aux_fg_bg > 0:
        metrics["aux_fg_bg_loss"] = aux_fg_bg / n
        metrics["aux_fg_accuracy"] = aux_acc / n
        metrics["aux_fg_iou"] = aux_iou / n
    if active > 0:
        metrics["active_contour"] = active / n
    if boundary > 0:
        metrics["boundary_aware"] = boundary / n
    if contour > 0:
        metrics["contour"] = contour / n
    if distance > 0:
        metrics["distance_transform"] = distance / n
    metrics.update(acc.compute())
    if output_dir is not None and epoch is not None:
        warnings.warn("hiseg.evaluate_model does not plot confusion matrices (matplotlib/seaborn figures); "
                      "the matrices are returned in the metrics dict")
    return metrics

"""Golden vectors of the reference's validation metrics (src/human_edge_detection/train_utils.py:109-402).

Run in the build container only (the reference is at /root/reference and never leaves it):
    python tests/golden/gen_metrics_golden.py
Runs the reference's own evaluate_model on recorded batches: a stand-in model returns the recorded
logits for each batch (with an empty aux dict) and a stand-in loss returns recorded loss values, so
the metric and loss-averaging code of evaluate_model runs unchanged.  train_utils imports seaborn
(plotting only; absent from this image): a stand-in module is installed for the import; no plot is
drawn (output_dir=None).
Writes tests/golden/metrics.npz: per batch the logits, masks and loss values, and every metric value
evaluate_model returns (scalars and the three confusion matrices).
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
from src.human_edge_detection.train_utils import evaluate_model  # noqa: E402

LOSS_KEYS = ["ce_loss", "dice_loss", "aux_fg_bg_loss", "aux_fg_accuracy", "aux_fg_iou", "boundary_aware",
             "contour", "distance_transform"]


def make_batches(seed: int):
    """Three batches of different ROI counts / mask sizes.  Logits are quantised to 1/4 so that exact
    ties occur (argmax takes the first maximum); one pixel is NaN; masks are ellipses (class 1), offset
    ellipses (class 2) plus a few out-of-range values (255, -1) the reference counts as 'not class c'."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for n, h, w in ((4, 24, 20), (3, 16, 12), (5, 32, 24)):
        logits = torch.round(torch.randn(n, 3, h, w, generator=g) * 4) / 4
        yy, xx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
        r = torch.rand(n, 4, generator=g) * 0.4 + 0.3
        m1 = (yy[None] / r[:, 0, None, None]) ** 2 + (xx[None] / r[:, 1, None, None]) ** 2 < 1
        m2 = ((yy[None] - 0.5) / r[:, 2, None, None]) ** 2 + ((xx[None] + 0.4) / r[:, 3, None, None]) ** 2 < 0.5
        masks = torch.zeros(n, h, w, dtype=torch.int64)
        masks[m1] = 1
        masks[m2 & ~m1] = 2
        # bias the logits toward the target so that IoUs spread over [0, 1]
        logits += torch.nn.functional.one_hot(masks, 3).permute(0, 3, 1, 2).float() * 1.5
        noise = torch.rand(n, h, w, generator=g)
        masks[noise < 0.01] = 255
        masks[(noise >= 0.01) & (noise < 0.015)] = -1
        out.append([logits, masks])
    # sample with no class-1 target and no class-1 prediction: IoU 1.0 (union == 0); all-background sample
    out[0][1][1] = 0
    out[0][0][1, 1] = -5.0
    out[1][1][2] = 0
    out[0][0][0, 2, 3, 4] = float("nan")
    return out


class _Replay(nn.Module):
    def __init__(self, logits):
        super().__init__()
        self.logits = list(logits)
        self.k = 0

    def forward(self, images, rois):
        x = self.logits[self.k]
        self.k += 1
        return x, {}


class _ReplayLoss:
    def __init__(self, vals):
        self.vals = list(vals)
        self.k = 0

    def __call__(self, logits, masks, aux):
        total, d = self.vals[self.k]
        self.k += 1
        return torch.tensor(total), dict(d)


def main():
    batches = make_batches(7)
    rng = np.random.default_rng(3)
    loss_vals = []
    for _ in batches:
        d = {k: float(np.float32(rng.uniform(0.01, 2.0))) for k in LOSS_KEYS}
        loss_vals.append((float(np.float32(rng.uniform(0.5, 3.0))), d))
    ns = types.SimpleNamespace
    config = ns(model=ns(use_rgb_hierarchical=True, use_hierarchical=False), multiscale=ns(enabled=False),
                cascade=ns(enabled=False), distance_loss=ns(enabled=False), distillation=ns(enabled=False))
    loader = [{"image": torch.zeros(m.shape[0], 3, 8, 8), "roi_boxes": torch.zeros(m.shape[0], 5), "roi_masks": m}
              for _, m in batches]
    metrics = evaluate_model(_Replay([b[0] for b in batches]), loader, _ReplayLoss(loss_vals), "cpu", config=config)
    arrays = {}
    for i, (lg, m) in enumerate(batches):
        arrays[f"b{i}_logits"] = lg.numpy().astype(np.float32)
        arrays[f"b{i}_masks"] = m.numpy()
        arrays[f"b{i}_loss_total"] = np.float64(loss_vals[i][0])
        arrays[f"b{i}_loss_terms"] = np.array([loss_vals[i][1][k] for k in LOSS_KEYS], np.float64)
    arrays["num_batches"] = np.int64(len(batches))
    arrays["loss_keys"] = np.array(LOSS_KEYS)
    keys = sorted(metrics)
    arrays["metric_keys"] = np.array(keys)
    for k in keys:
        arrays[f"m_{k}"] = np.asarray(metrics[k], dtype=np.int64 if k.startswith("conf_") else np.float64)
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), **arrays)
    print({k: (v if not isinstance(v, np.ndarray) else v.tolist()) for k, v in metrics.items()})


if __name__ == "__main__":
    main()

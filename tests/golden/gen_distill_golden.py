"""Golden vectors of the reference's UNetDistillationLoss (advanced/unet_decoder_distillation.py:338-663).

Run in the build container only (imports the reference from /root/reference through gen_golden.py's
segmentation_models_pytorch stand-in; the loss itself never touches smp):
    python tests/golden/gen_distill_golden.py
Writes tests/golden/distill_loss.npz: per case the seeded inputs' recipe (seed, shape), the loss
state (temperature, alpha, task weight, adaptive flags, performance ratio), the total loss, the five
loss-dict values and d(total)/d(student logits).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402,F401  (installs the smp stand-in and the reference path)
from src.human_edge_detection.advanced.unet_decoder_distillation import UNetDistillationLoss  # noqa: E402

KEYS = ["total_loss", "kl_loss", "mse_loss", "bce_loss", "dice_loss"]


def distill_inputs(seed: int, b: int, h: int, w: int):
    """Student / teacher logits (N(0, 4^2): some beyond the +-10 clamp) and ellipse-ish binary masks."""
    g = torch.Generator().manual_seed(seed)
    s = torch.randn(b, 1, h, w, generator=g) * 4.0
    t = torch.randn(b, 1, h, w, generator=g) * 4.0
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
    r = torch.rand(b, 2, generator=g) * 0.4 + 0.3
    m = ((yy[None] / r[:, 0, None, None]) ** 2 + (xx[None] / r[:, 1, None, None]) ** 2 < 1).float()[:, None]
    return s, t, m


# (name, seed, shape, ctor kwargs, schedule ops, use targets)
CASES = [
    ("dist_default", 1, (2, 24, 32), dict(temperature=1.0, alpha=0.05, task_weight=0.7), [], True),
    ("dist_t4", 2, (3, 16, 20), dict(temperature=4.0, alpha=0.3, task_weight=0.3), [], True),
    ("dist_cos_sched", 3, (2, 32, 32), dict(temperature=4.0, alpha=0.3, task_weight=0.7),
     [("temp", 12, 50, 1.0, "cosine")], True),
    ("dist_lin_sched", 4, (2, 16, 16), dict(temperature=4.0, alpha=0.3, task_weight=0.7),
     [("temp", 30, 50, 1.0, "linear")], True),
    ("dist_student_better", 5, (2, 16, 24), dict(temperature=2.0, alpha=0.3, task_weight=0.7),
     [("alpha", 0.81, 0.80, 0.0, 30.0, 0.03)], True),
    ("dist_eliminated", 6, (2, 16, 24), dict(temperature=2.0, alpha=0.3, task_weight=0.7),
     [("alpha", 0.90, 0.80, 0.0, 30.0, 0.03)], True),
    ("dist_no_target", 7, (2, 16, 16), dict(temperature=3.0, alpha=0.3, task_weight=0.7), [], False),
    ("finetune", 8, (2, 16, 16), dict(temperature=1.0, alpha=0.0, task_weight=1.0, adaptive_distillation=False), [],
     True),
    ("no_dice", 9, (2, 16, 16), dict(temperature=2.0, alpha=0.2, task_weight=0.5, use_dice_loss=False), [], True),
]

# Non-finite inputs: the reference's fallbacks (:560-568 KL -> L1, :650-659 total -> task loss, else MSE, else a
# constant 1.0 without a gradient).  (name, seed, shape, ctor kwargs, use targets, [(tensor, flat index, value)])
POISON_CASES = [
    ("nan_teacher", 21, (2, 16, 16), dict(temperature=4.0, alpha=0.05, task_weight=0.7), True,
     [("t", 5, float("nan")), ("t", 300, float("nan"))]),
    ("inf_teacher", 22, (2, 16, 16), dict(temperature=4.0, alpha=0.05, task_weight=0.7), True,
     [("t", 17, float("inf")), ("t", 400, float("-inf"))]),
    ("nan_student", 23, (2, 16, 16), dict(temperature=4.0, alpha=0.05, task_weight=0.7), True,
     [("s", 9, float("nan"))]),
    ("nan_teacher_no_target", 24, (2, 16, 16), dict(temperature=3.0, alpha=0.3, task_weight=0.7), False,
     [("t", 33, float("nan"))]),
    ("inf_teacher_no_target", 25, (2, 16, 16), dict(temperature=3.0, alpha=0.3, task_weight=0.7), False,
     [("t", 44, float("inf"))]),
    ("nan_teacher_finetune", 26, (2, 16, 16), dict(temperature=1.0, alpha=0.0, task_weight=1.0,
                                                   adaptive_distillation=False), True, [("t", 7, float("nan"))]),
]


def main():
    out = {"keys": np.array(KEYS)}
    names = []
    for name, seed, (b, h, w), kw, ops, with_t in CASES:
        fn = UNetDistillationLoss(**kw)
        for op in ops:
            if op[0] == "temp":
                fn.update_temperature(op[1], op[2], final_temperature=op[3], schedule_type=op[4])
            else:
                fn.update_distillation_weight(op[1], op[2], min_alpha=op[3], amplification_factor=op[4],
                                              zero_distillation_threshold=op[5])
        s, t, m = distill_inputs(seed, b, h, w)
        s.requires_grad_(True)
        loss, d = fn(s, t, m if with_t else None)
        loss.backward()
        names.append(name)
        out[f"{name}_meta"] = np.array([seed, b, h, w, int(with_t)], dtype=np.int64)
        out[f"{name}_state"] = np.array([fn.temperature, fn.alpha, fn.task_weight, float(fn.adaptive_distillation),
                                         float(fn.distillation_eliminated), fn.performance_ratio,
                                         float(fn.use_dice_loss), fn.initial_alpha, fn.initial_task_weight],
                                        dtype=np.float64)
        out[f"{name}_ctor"] = np.array([kw.get("temperature", 3.0), kw.get("alpha", 0.5), kw.get("task_weight", 0.3),
                                        float(kw.get("use_dice_loss", True)),
                                        float(kw.get("adaptive_distillation", True))], dtype=np.float64)
        out[f"{name}_loss"] = np.array(float(loss))
        out[f"{name}_dict"] = np.array([float(d.get(k, np.nan)) for k in KEYS])
        out[f"{name}_grad"] = s.grad.numpy().astype(np.float32)
        print(name, float(loss), {k: round(float(v), 5) for k, v in d.items()})
    for name, seed, (b, h, w), kw, with_t, poison in POISON_CASES:
        fn = UNetDistillationLoss(**kw)
        s, t, m = distill_inputs(seed, b, h, w)
        for which, idx, val in poison:
            (s if which == "s" else t).view(-1)[idx] = val
        s.requires_grad_(True)
        loss, d = fn(s, t, m if with_t else None)
        if loss.requires_grad and loss.grad_fn is not None:
            loss.backward()
        grad = s.grad if s.grad is not None else torch.zeros_like(s)
        names.append(name)
        out[f"{name}_meta"] = np.array([seed, b, h, w, int(with_t)], dtype=np.int64)
        out[f"{name}_state"] = np.array([fn.temperature, fn.alpha, fn.task_weight, float(fn.adaptive_distillation),
                                         float(fn.distillation_eliminated), fn.performance_ratio,
                                         float(fn.use_dice_loss), fn.initial_alpha, fn.initial_task_weight],
                                        dtype=np.float64)
        out[f"{name}_ctor"] = np.array([kw.get("temperature", 3.0), kw.get("alpha", 0.5), kw.get("task_weight", 0.3),
                                        float(kw.get("use_dice_loss", True)),
                                        float(kw.get("adaptive_distillation", True))], dtype=np.float64)
        out[f"{name}_poison"] = np.array([[0 if wh == "s" else 1, idx, val] for wh, idx, val in poison],
                                         dtype=np.float64)
        out[f"{name}_loss"] = np.array(float(loss))
        out[f"{name}_dict"] = np.array([float(d.get(k, np.nan)) for k in KEYS])
        out[f"{name}_grad"] = grad.detach().numpy().astype(np.float32)
        print(name, float(loss), {k: round(float(v), 5) for k, v in d.items()})
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "distill_loss.npz"), **out)


if __name__ == "__main__":
    main()

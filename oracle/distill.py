"""Distillation-path CPU restatement -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

* UNetDistillationLoss.forward (advanced/unet_decoder_distillation.py:510-663) with its host state
  (temperature, alpha, task weight, adaptive flags, performance ratio; :338-469) as plain floats,
  differentiable w.r.t. the student logits through torch autograd on the CPU;
* the distillation training step of train_distillation_staged.py:256-366 for the student smp-UNet
  (oracle.rgb_model.effunet_logits inside oracle.train.train_mode(): batch-statistics BatchNorm on every
  layer of the student, frozen encoder stages excluded from the gradient).

Pinned to tests/golden/distill_loss.npz (the reference's own loss run in the build container,
tests/golden/gen_distill_golden.py).  The EfficientNet-UNet arithmetic is the same restatement as the
inference oracle (smp/timm absent: parity of that sub-network unpinned, see oracle/rgb_model.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def distill_loss(student, teacher, target, temperature, alpha, task_weight, adaptive=True, eliminated=False,
                 performance_ratio=1.0, use_dice=True, fg_ratio=0.162):
    """Returns (total, {total_loss, kl_loss, mse_loss, bce_loss, dice_loss}) as the reference's forward."""
    d = {}
    disabled = (adaptive and alpha == 0.0) or task_weight >= 0.99 or eliminated
    if disabled:                                                       # :529-535
        kl = student.new_zeros(())
        mse = student.new_zeros(())
        d["kl_loss"] = d["mse_loss"] = 0.0
    else:                                                              # :536-568
        eps = 1e-5
        ps = torch.sigmoid(torch.clamp(student, -10, 10) / temperature).clamp(eps, 1 - eps)
        pt = torch.sigmoid(torch.clamp(teacher, -10, 10) / temperature).clamp(eps, 1 - eps)
        t1 = pt * (torch.log(pt + eps) - torch.log(ps + eps))
        t2 = (1 - pt) * (torch.log(1 - pt + eps) - torch.log(1 - ps + eps))
        kl = (t1 + t2).mean()
        if not torch.isfinite(kl):                                     # :560-564
            kl = torch.abs(pt - ps).mean() * 0.1
        kl = torch.clamp(kl, 0.0, 5.0)
        mse = F.mse_loss(student, teacher)
        d["kl_loss"], d["mse_loss"] = _nz(kl), _nz(mse)
    if target is not None:                                             # :571-600
        pw = torch.tensor([math.sqrt((1.0 - fg_ratio) / fg_ratio)], dtype=student.dtype)
        bce = F.binary_cross_entropy_with_logits(student, target.to(student.dtype), pos_weight=pw)
        d["bce_loss"] = _nz(bce)
        if use_dice:                                                   # :471-508
            p = torch.sigmoid(student).reshape(student.shape[0], -1)
            y = target.to(student.dtype).reshape(student.shape[0], -1)
            coeff = (2 * (p * y).sum(1) + 1e-5) / (p.sum(1) + y.sum(1) + 1e-5)
            dice = 1.0 - coeff.mean()
            d["dice_loss"] = _nz(dice)
            task = 0.7 * bce + 0.3 * dice
        else:
            d["dice_loss"] = 0.0
            task = bce
    else:
        d["bce_loss"] = d["dice_loss"] = 0.0
        task = None
    if (adaptive and alpha == 0.0) or task_weight >= 0.99:             # :602-615
        dist = student.new_zeros(())
    else:
        eff = alpha * max(0.1, 2.0 - performance_ratio) if adaptive and performance_ratio > 1.0 else alpha
        kw = min(eff, 0.1)
        dist = kw * kl + (1 - kw) * mse
    total = task_weight * task + (1 - task_weight) * dist if task is not None else dist   # :617-628
    if not torch.isfinite(total):                                      # :650-659
        if task is not None and not torch.isnan(task):
            total = task
        elif not torch.isnan(mse):
            total = mse
        else:
            total = student.new_tensor(1.0)   # a constant: no gradient reaches the student
    d["total_loss"] = float(total.detach())
    return total, d


def _nz(v):
    """loss_dict value: .item(), NaN reported as 0.0 (:567, :571, :585, :590)."""
    x = float(v.detach())
    return 0.0 if x != x else x


def temperature_at(initial, final, epoch, total_epochs, schedule="linear"):
    """update_temperature (:366-408)."""
    if total_epochs <= 1:
        return final
    progress = epoch / (total_epochs - 1)
    if schedule == "linear":
        return initial + (final - initial) * progress
    if schedule == "cosine":
        return final + (initial - final) * 0.5 * (1 + math.cos(math.pi * progress))
    if schedule == "exponential":
        return initial * math.exp(math.log(final / initial) * progress)
    return initial


def unfreeze_schedule(total_epochs, start=10, rate=5, max_blocks=7):
    """DistillationUNetWrapper.get_progressive_unfreeze_schedule (:276-302)."""
    return {e: 0 if e < start else min(1 + (e - start) // rate, max_blocks) for e in range(total_epochs)}


def np_inputs(seed, b, h, w):
    """The golden script's input recipe (tests/golden/gen_distill_golden.py: distill_inputs)."""
    g = torch.Generator().manual_seed(seed)
    s = torch.randn(b, 1, h, w, generator=g) * 4.0
    t = torch.randn(b, 1, h, w, generator=g) * 4.0
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
    r = torch.rand(b, 2, generator=g) * 0.4 + 0.3
    m = ((yy[None] / r[:, 0, None, None]) ** 2 + (xx[None] / r[:, 1, None, None]) ** 2 < 1).float()[:, None]
    return s, t, m

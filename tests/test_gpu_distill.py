"""Distillation path on the GPU: the UNetDistillationLoss kernels (include/hiseg_distill.h) against the
reference's golden vectors, and the student training step against the CPU oracle."""
import numpy as np
import pytest
import torch

from helpers import load
from test_oracle_distill import G, KEYS, NAMES, case_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _loss_fn(name):
    import hiseg
    ct = G[f"{name}_ctor"]
    fn = hiseg.UNetDistillationLoss(temperature=float(ct[0]), alpha=float(ct[1]), task_weight=float(ct[2]),
                                    use_dice_loss=bool(ct[3]), adaptive_distillation=bool(ct[4]))
    st = G[f"{name}_state"]
    fn.temperature, fn.alpha, fn.task_weight = float(st[0]), float(st[1]), float(st[2])
    fn.distillation_eliminated, fn.performance_ratio = bool(st[4]), float(st[5])
    return fn


@pytest.mark.parametrize("name", NAMES)
def test_distill_loss_kernel_matches_reference_golden(name):
    s, t, m, _ = case_inputs(name)
    fn = _loss_fn(name)
    sd = s.to(DEV).requires_grad_(True)
    total, d = fn(sd, t.to(DEV), m.to(DEV) if m is not None else None)
    total.backward()
    assert total.item() == pytest.approx(float(G[f"{name}_loss"]), rel=1e-5, abs=1e-6)
    for k, v in zip(KEYS, G[f"{name}_dict"]):
        assert d[k] == pytest.approx(float(v), rel=1e-4, abs=1e-6), k
    ref = torch.from_numpy(G[f"{name}_grad"])
    assert (sd.grad.cpu() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-9


def test_distill_schedule_methods_match_reference_state():
    import hiseg
    fn = hiseg.UNetDistillationLoss(temperature=4.0, alpha=0.3, task_weight=0.7)
    fn.update_temperature(12, 50, final_temperature=1.0, schedule_type="cosine")
    assert fn.temperature == pytest.approx(float(G["dist_cos_sched_state"][0]))
    fn = hiseg.UNetDistillationLoss(temperature=2.0, alpha=0.3, task_weight=0.7)
    fn.update_distillation_weight(0.81, 0.80, min_alpha=0.0, amplification_factor=30.0,
                                  zero_distillation_threshold=0.03)
    st = G["dist_student_better_state"]
    assert (fn.alpha, fn.task_weight, fn.performance_ratio) == pytest.approx((st[1], st[2], st[5]))
    fn.update_distillation_weight(0.90, 0.80, amplification_factor=30.0)
    assert fn.distillation_eliminated and fn.alpha == 0.0 and fn.task_weight == 1.0

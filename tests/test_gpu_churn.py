"""Allocator-churn regression tests for the C3 train step and the C5 distillation step (the B0
step's is tests/test_gpu_train.py::test_train_step_independent_of_allocator_churn_between_forward_and_backward).

Every buffer a backward reads must stay alive until that backward ran (hiseg._lib.Desc holds what its pointer fields
point at; closures hold the rest).  Between the forward and the backward the caching allocator's free blocks of
every size class are taken, filled with NaN and released again: a backward reading a released block then reads
NaN.  Bar: bit-identical parameter gradients with and without the churn.  tools/churn_control.py is the negative
control (the same tests with the holds undone)."""
import pytest
import torch

import filler

pytestmark = pytest.mark.gpu
DEV = "cuda"


def churn():
    """Take, poison and release blocks of every size class the caching allocator holds (512 B .. 64 MiB)."""
    held = []
    n = 128
    while n <= (16 << 20):
        held += [torch.full((n,), float("nan"), device=DEV) for _ in range(24 if n < (1 << 20) else 4)]
        n *= 2
    torch.cuda.synchronize()
    del held


def _grads(fwd_loss, state_of, n_runs=2):
    out = []
    for poisoned in (False, True)[:n_runs]:
        torch.manual_seed(0)
        loss, model = fwd_loss()
        if poisoned:
            churn()
        loss.backward()
        torch.cuda.synchronize()
        out.append(state_of(model).flat.grad.clone())
    return out


def test_c3_train_step_independent_of_allocator_churn():
    """C3 (B1-enhanced preset: EnhancedUNet base 72, ROI 80x60), bf16, Dropout2d on."""
    import hiseg
    from helpers import configs, hiseg_kwargs
    kw = hiseg_kwargs(dict(configs()["b1"]["model_kwargs"]))
    images = torch.from_numpy(filler.uniform(41, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(42, 2, 1)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(43, 2, *kw["mask_size"])).to(DEV)

    def fwd_loss():
        m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**kw))
        hiseg.set_compute_dtype(m, torch.bfloat16)
        m = m.to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
        loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                                use_distance_transform=True, boundary_aware_weight=0.1,
                                                contour_loss_weight=0.1, distance_loss_weight=0.1)
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        return loss, m
    g = _grads(fwd_loss, lambda m: m.__dict__["_hiseg_train"])
    assert torch.isfinite(g[0]).all()
    assert torch.equal(g[0], g[1])


def test_c5_distillation_step_independent_of_allocator_churn():
    """C5 (B7 teacher, B0 student with its last encoder stages unfrozen: the MBConv / depthwise / SE backward on
    the tape), bf16."""
    import hiseg
    from oracle import distill as OD
    x = torch.from_numpy(filler.normal(51, (2, 3, 64, 96))).to(DEV)
    msk = OD.np_inputs(52, 2, 64, 96)[2].to(DEV)

    def fwd_loss():
        model, loss_fn = hiseg.create_unet_distillation_model("timm-efficientnet-b0", "timm-efficientnet-b7",
                                                              teacher_checkpoint="absent.pth", device="cpu",
                                                              progressive_unfreeze=True)
        filler.fill_module(model.student, seed=11)
        filler.fill_module(model.teacher, seed=12)
        model.unfreeze_encoder_blocks(2)
        hiseg.set_compute_dtype(model, torch.bfloat16)
        model = model.to(DEV).train()
        loss_fn.temperature = 4.0
        s, t = model(x)
        loss, _ = loss_fn(s, t, msk)
        return loss, model
    g = _grads(fwd_loss, lambda m: m.student.__dict__["_hiseg_train"])
    assert torch.isfinite(g[0]).all()
    assert torch.equal(g[0], g[1])

"""Parity at the reference's own plumbing workload and against float64.

* C1 (BASELINE.json configs[0]): 1 image 3x480x640 (torch.rand, seed 0), the four fixed ROIs, B0-std,
  eval, f32, RoIAlign scale (480, 640) -- validate_rgb_hierarchical_simple.py:23-33 restated as a synthetic forward.
  Logits at the north-star 1e-4 against the oracle; instance masks exact.
* U4: PreTrainedPeopleSegmentationUNet.train (hierarchical_segmentation_unet.py:1892-1899) keeps the frozen smp net in
  eval: a model.train() forward leaves every UNet BatchNorm buffer untouched, and its full-image logits equal the
  eval-mode oracle (unet.py:1869-1879 freezing; 1e-4).
* One f32 train step against the oracle run in float64: per-tensor relative errors of hiseg's f32 step and of the
  oracle's own f32 step, both against float64.  Against float64 the kernels' rounding is the only error source; the
  bar is that hiseg's f32 step is about as accurate as PyTorch's f32 CPU step (gradient medians / p90 at most 2x,
  logits at most 3x), which the printed table shows stage by stage and tensor by tensor.  (Round 4: this test found
  hiseg's RoIAlign coordinates FMA-contracted -- 1e-5 on the ROI patches, 1.4e-3 on the logits -- now bit-identical
  to the oracle's f32 arithmetic.)
"""
import statistics

import numpy as np
import pytest
import torch
import torch.nn as nn

import filler
from helpers import configs, hiseg_kwargs

pytestmark = pytest.mark.gpu
DEV = "cuda"
C1_ROIS = [[0, 0.10, 0.10, 0.40, 0.90], [0, 0.35, 0.15, 0.60, 0.95], [0, 0.55, 0.05, 0.80, 0.70],
           [0, 0.70, 0.30, 0.95, 0.99]]


def _rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _b0(dt=torch.float32, drop_zero=False):
    import hiseg
    kw = hiseg_kwargs(dict(configs()["b0"]["model_kwargs"]))
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**kw))
    if drop_zero:
        for mod in m.modules():
            if isinstance(mod, (nn.Dropout, nn.Dropout2d)):
                mod.p = 0.0
    hiseg.set_compute_dtype(m, dt)
    return m, kw


def test_c1_plumbing_workload_f32_matches_oracle():
    from oracle import rgb_model as O
    model, kw = _b0()
    sd = O.np_state(model)
    model = model.to(DEV).eval()
    images = torch.rand(1, 3, 480, 640, generator=torch.Generator().manual_seed(0))
    rois = torch.tensor(C1_ROIS, dtype=torch.float32)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 480, 640
    import hiseg
    with torch.no_grad():
        logits, aux = model(images.to(DEV), rois.to(DEV))
        inst, binary = hiseg.RGBHierarchicalExportWrapper(model)(images.to(DEV), rois.to(DEV))
        ref, ref_aux, ref_u = O.rgb_model(sd, images, rois, O.cfg_from_kwargs(kw), (480, 640), "b0")
    torch.cuda.synchronize()
    assert logits.shape == ref.shape == (4, 3, 128, 96)
    assert _rel(aux["full_image_logits"].cpu(), ref_aux["full_image_logits"]) < 1e-4
    assert _rel(logits.cpu(), ref) < 1e-4
    ref_inst = O.instance_masks(ref)
    diff = (inst.cpu() != ref_inst)
    if diff.any():   # name the pixels and the oracle's argmax margin there
        top2 = ref.topk(2, dim=1).values
        margin = (top2[:, 0] - top2[:, 1])[diff[:, 0]]
        pytest.fail(f"{int(diff.sum())} instance-mask pixels differ; oracle margins there {margin[:8].tolist()}")
    assert (binary.cpu() - O.binary_masks(sd, ref_u)).abs().max().item() < 1e-4


def test_u4_train_mode_keeps_the_frozen_unet_in_eval():
    from oracle import rgb_model as O
    model, kw = _b0(drop_zero=True)
    sd = O.np_state(model)
    model = model.to(DEV)
    model.train()
    # unet.py:1892-1899: PreTrainedPeopleSegmentationUNet itself follows train(); its smp net (.model) stays in eval
    assert model.training and model.pretrained_unet.training and model.pretrained_unet.model.training
    unet = model.pretrained_unet.model.model
    assert not unet.training and not any(m.training for m in unet.modules())
    bufs = {k: v.detach().clone() for k, v in unet.state_dict().items() if "running" in k or "num_batches" in k}
    assert bufs
    images = torch.from_numpy(filler.uniform(501, (2, 3, 96, 128)))
    rois = torch.from_numpy(filler.box_rois(502, 2, 2))
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 96, 128
    logits, aux = model(images.to(DEV), rois.to(DEV))        # the train-mode forward, UNet computed (no override)
    import hiseg
    loss, _ = hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)(
        logits, torch.from_numpy(filler.ellipse_targets(503, 4, 128, 96)).to(DEV), aux)
    loss.backward()
    torch.cuda.synchronize()
    for k, v in unet.state_dict().items():
        if k in bufs:
            assert torch.equal(v, bufs[k]), f"{k} changed in a train-mode step"
    assert all(p.grad is None or not p.grad.any() for p in unet.parameters())
    with torch.no_grad():
        _, ref_aux, _ = O.rgb_model(sd, images, rois, O.cfg_from_kwargs(kw), (96, 128), "b0")   # eval-mode oracle
    assert _rel(aux["full_image_logits"].detach().cpu(), ref_aux["full_image_logits"]) < 1e-4


def test_f32_train_step_against_float64_oracle():
    import hiseg
    from oracle import rgb_model as O
    from oracle import train as OT
    from hiseg import train_engine as TE
    m, kw = _b0(drop_zero=True)
    cfg = O.cfg_from_kwargs(kw)
    images = torch.from_numpy(filler.uniform(61, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(62, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]])
    tgt = torch.from_numpy(filler.ellipse_targets(63, 3, *cfg["mask_hw"]))
    ref = {}
    for dt in (torch.float32, torch.float64):
        sd = OT.params_of(m)
        sd = {k: (v.detach().to(dt).requires_grad_(v.requires_grad) if v.is_floating_point() else v)
              for k, v in sd.items()}
        lg, aux = OT.forward_train(sd, images.to(dt), rois, u.to(dt), cfg, (96, 128))
        loss, _ = OT.RefinedHierarchicalLoss()(lg, tgt, aux)
        loss.backward()
        ref[dt] = (lg.detach(), float(loss), {k: v.grad for k, v in sd.items() if v.requires_grad and v.grad is not None},
                   {k: v.detach() for k, v in aux.items() if torch.is_tensor(v)})
    mm = m.to(DEV).train()
    for x in (mm.roi_align_mask, mm.roi_align_rgb):
        x.spatial_scale_h, x.spatial_scale_w = 96, 128
    logits, aux = TE.train_forward(mm, images.to(DEV), rois.to(DEV), u_override=u.to(DEV))
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    loss, _ = loss_fn(logits, tgt.to(DEV), aux)
    loss.backward()
    torch.cuda.synchronize()
    l64, loss64, g64, a64 = ref[torch.float64]
    l32, loss32, g32, a32 = ref[torch.float32]
    # where along the forward the f32 error enters: every intermediate both sides expose, vs float64
    stages = "\n".join(f"  {_rel(aux[k].detach().float().cpu(), a64[k]):.3e}  {_rel(a32[k], a64[k]):.3e}  aux[{k}]"
                        for k in a64 if k in aux and torch.is_tensor(aux[k]) and tuple(aux[k].shape) == tuple(a64[k].shape))
    e_log_h, e_log_o = _rel(logits.detach().cpu(), l64), _rel(l32, l64)
    e_loss_h, e_loss_o = abs(loss.item() - loss64) / abs(loss64), abs(loss32 - loss64) / abs(loss64)
    scale = statistics.median(float(g.norm()) for g in g64.values())
    rows = []
    params = dict(mm.named_parameters())
    for k, g in g64.items():
        if float(g.norm()) < 1e-6 * scale:   # analytically zero (a conv bias feeding a batch-statistics BN)
            continue
        gh = params[k].grad.detach().double().cpu()
        n = float(g.norm())
        rows.append((float((gh - g).norm()) / n, float((g32[k].double() - g).norm()) / n, k))
    med_h, med_o = statistics.median(r[0] for r in rows), statistics.median(r[1] for r in rows)
    p90_h = float(np.percentile([r[0] for r in rows], 90))
    p90_o = float(np.percentile([r[1] for r in rows], 90))
    table = "\n".join(f"  {h:.3e}  {o:.3e}  {k}" for h, o, k in sorted(rows, reverse=True)[:30])
    summary = (f"vs float64 -- logits: hiseg f32 {e_log_h:.3e}, oracle f32 {e_log_o:.3e}; loss {e_loss_h:.3e} / "
               f"{e_loss_o:.3e}; gradients ({len(rows)} tensors) median {med_h:.3e} / {med_o:.3e}, p90 {p90_h:.3e} / "
               f"{p90_o:.3e}\n  hiseg      oracle-f32  forward stage\n{stages}\n"
               f"  hiseg      oracle-f32  tensor (largest hiseg errors)\n{table}")
    print(summary)
    # logits within 3x of PyTorch's own f32 error (measured 2.5x: 1.5e-4 vs 6.0e-5; the MFMA f32 conv sums its
    # K = 9 x 256 products in one chain per accumulator where oneDNN blocks them, and train-mode BN over 3 ROIs
    # amplifies the difference ~20x from the shared features to the logits -- the table below shows both growing
    # stage by stage at the same rate)
    assert e_log_h < max(3 * e_log_o, 1e-6), summary
    assert e_loss_h < max(2 * e_loss_o, 1e-6), summary
    assert med_h < 2 * med_o and p90_h < 2 * p90_o, summary

"""Golden vectors for the TRAINING path, produced by running the REFERENCE on CPU (build container only).

    python tests/golden/gen_train_golden.py

Writes tests/golden/train_loss.npz and tests/golden/train_step_b0.npz (data only: inputs are
regenerated from seeds by the tests, weights from tests/golden/filler.py).

* train_loss.npz — RefinedHierarchicalLoss (advanced/hierarchical_segmentation_refinement.py:807-984,
  built with the train_advanced.py:551-568 weights) on seeded random predictions / aux outputs and
  SURVEY §8d ellipse targets: loss value, every loss-dict entry and the gradients w.r.t. the four
  differentiable inputs, for several mask sizes (contour edge width 1 / 3 / 3), a no-foreground
  batch and three consecutive calls (EMA class weights, :227-255,286-309).
* train_step_b0.npz — the B0-std model (smp UNet output injected, see gen_golden.py) in train mode
  with every Dropout p = 0 (RNG streams cannot match): forward, loss, backward, then
  clip_grad_norm_(1.0) + torch.optim.AdamW(lr 1e-4, wd 0.01) (train_advanced.py:733-740,1111-1143)
  and a second forward.  Per parameter: sum of squares and a strided sample of the gradient, the
  updated value sample; BatchNorm running statistics after the step.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the smp stand-in, imports the reference)
import filler  # noqa: E402

from src.human_edge_detection.advanced.hierarchical_segmentation_refinement import RefinedHierarchicalLoss  # noqa: E402

LOSS_KW = dict(bg_weight=1.5, fg_weight=1.5, target_weight=1.2, consistency_weight=0.3, use_dynamic_weights=True,
               dice_weight=1.0, ce_weight=1.0, active_contour_weight=0.1, boundary_aware_weight=0.1,
               contour_loss_weight=0.1, distance_loss_weight=0.1, use_active_contour_loss=False,
               use_boundary_aware_loss=True, use_contour_detection=True, use_distance_transform=True)
DICT_KEYS = ["bg_fg_loss", "target_nontarget_loss", "final_loss", "consistency_loss", "total_loss", "ce_loss",
             "dice_loss", "aux_fg_bg_loss", "aux_fg_accuracy", "aux_fg_iou", "bg_weight", "fg_weight",
             "target_weight", "nontarget_weight", "boundary_aware", "contour", "contour_weight",
             "distance_transform"]


def loss_inputs(seed, n, mh, mw):
    """Seeded predictions: logits/bg_fg/tn ~ 2*N(0,1), contours = sigmoid(N(0,1)) (the branch ends in a
    Sigmoid), distance_map ~ U(0,1)."""
    pred = torch.from_numpy(filler.normal(seed, (n, 3, mh, mw)) * 2.0)
    bgfg = torch.from_numpy(filler.normal(seed + 1, (n, 2, mh, mw)) * 2.0)
    tn = torch.from_numpy(filler.normal(seed + 2, (n, 2, mh, mw)) * 2.0)
    cont = torch.sigmoid(torch.from_numpy(filler.normal(seed + 3, (n, 1, mh, mw))))
    dist = torch.from_numpy(filler.uniform(seed + 4, (n, 1, mh, mw)))
    return pred, bgfg, tn, cont, dist


def gen_loss():
    out = {}
    cases = [("a", 11, 3, 32, 24, "ellipse"), ("b", 21, 2, 128, 96, "ellipse"), ("c", 31, 1, 160, 120, "ellipse"),
             ("d", 41, 2, 32, 24, "bg"), ("e", 51, 2, 32, 24, "fg_only")]
    for name, seed, n, mh, mw, kind in cases:
        loss_fn = RefinedHierarchicalLoss(**LOSS_KW)
        calls = 3 if name == "a" else 1
        for call in range(calls):
            s = seed + 100 * call
            ins = [t.clone().requires_grad_(True) for t in loss_inputs(s, n, mh, mw)]
            if kind == "ellipse":
                tgt = torch.from_numpy(filler.ellipse_targets(s + 5, n, mh, mw))
            elif kind == "bg":
                tgt = torch.zeros(n, mh, mw, dtype=torch.int64)
            else:
                tgt = torch.from_numpy(filler.ellipse_targets(s + 5, n, mh, mw)).clamp(min=1)
            aux = {"bg_fg_logits": ins[1], "target_nontarget_logits": ins[2], "contours": ins[3], "distance_map": ins[4]}
            loss, d = loss_fn(ins[0], tgt, aux)
            loss.backward()
            key = f"{name}{call}"
            out[f"{key}_meta"] = np.array([seed + 100 * call, n, mh, mw], dtype=np.int64)
            out[f"{key}_kind"] = np.array(kind)
            out[f"{key}_loss"] = loss.detach()
            out[f"{key}_dict"] = np.array([float(d.get(k, np.nan)) for k in DICT_KEYS], dtype=np.float64)
            for i, g in enumerate(["pred", "bgfg", "tn", "cont", "dist"]):
                gr = ins[i].grad
                out[f"{key}_grad_{g}"] = gr if gr is not None else np.zeros(0, np.float32)  # empty = no gradient
    out["dict_keys"] = np.array(DICT_KEYS)
    G.save("train_loss", **out)


def sample(t: torch.Tensor, k: int = 64) -> torch.Tensor:
    f = t.detach().reshape(-1)
    step = max(1, f.numel() // k)
    return f[::step][:k].clone()


def gen_step(kw):
    torch.manual_seed(0)
    model = G.build_ref_model(kw).train()
    for m in model.modules():
        if isinstance(m, (torch.nn.Dropout, torch.nn.Dropout2d)):
            m.p = 0.0
    images = torch.from_numpy(filler.uniform(61, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(62, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]], dtype=torch.float32)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale, m.spatial_scale_h, m.spatial_scale_w = (96, 128), 96, 128
    mh, mw = G.tup(kw["mask_size"])
    tgt = torch.from_numpy(filler.ellipse_targets(63, 3, mh, mw))
    G._InjectedUnet.injected = u
    loss_fn = RefinedHierarchicalLoss(**LOSS_KW)
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4, weight_decay=0.01)
    opt.zero_grad()
    logits, aux = model(images, rois)
    loss, d = loss_fn(logits, tgt, aux)
    loss.backward()
    out = {"logits_sample": sample(logits, 4096), "logits_chmean": logits.detach().mean(dim=(0, 2, 3)),
           "loss": loss.detach(), "dict": np.array([float(d.get(k, np.nan)) for k in DICT_KEYS])}
    names, sq, gs, nograd = [], [], [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        if p.grad is None:
            nograd.append(name)
            continue
        names.append(name)
        sq.append(float((p.grad.double() ** 2).sum()))
        gs.append(sample(p.grad).numpy())
    out["grad_names"] = np.array(names)
    out["grad_sumsq"] = np.array(sq)
    out["grad_sample"] = np.stack([np.pad(g, (0, 64 - g.size)) for g in gs])
    out["grad_sample_len"] = np.array([g.size for g in gs])
    out["nograd_names"] = np.array(nograd)
    oc = model.pretrained_unet.output_conv
    out["output_conv_wgrad"], out["output_conv_bgrad"] = oc.weight.grad, oc.bias.grad
    total = torch.nn.utils.clip_grad_norm_([p for p in model.parameters() if p.requires_grad], 1.0)
    opt.step()
    out["total_norm"] = total.detach()
    out["param_after_sample"] = np.stack([np.pad(sample(dict(model.named_parameters())[n]).numpy(), (0, 64 - L))
                                          for n, L in zip(names, out["grad_sample_len"])])
    rs = {}
    for name, b in model.named_buffers():
        if "running_" in name:
            rs[name] = sample(b).numpy()
    out["bn_names"] = np.array(list(rs.keys()))
    out["bn_running_sample"] = np.stack([np.pad(v, (0, 64 - v.size)) for v in rs.values()])
    out["bn_running_len"] = np.array([v.size for v in rs.values()])
    logits2, aux2 = model(images, rois)
    loss2, _ = loss_fn(logits2, tgt, aux2)
    out["loss2"] = loss2.detach()
    out["logits2_sample"] = sample(logits2, 4096)
    G.save("train_step_b0", **out)


def gen_blocks():
    """Train-mode blocks (tight tolerances: shallow, well conditioned): ResidualBlock(64), the attention
    modules (attention_modules.py:10-113) and EnhancedUNet(256, 64, depth 3); output, input gradient,
    parameter-gradient sum of squares + samples for a seeded upstream gradient."""
    from src.human_edge_detection.advanced.attention_modules import ChannelAttentionModule, SpatialAttentionModule
    out = {}
    mods = {
        "res": (G.R.ResidualBlock(64, "batchnorm", 8, "relu", 1.0), (4, 64, 12, 10)),
        "sa": (SpatialAttentionModule(kernel_size=7), (3, 32, 10, 8)),
        "ca": (ChannelAttentionModule(128, reduction_ratio=8, activation_function="relu"), (3, 128, 12, 8)),
        "unet": (G.U.EnhancedUNet(256, base_channels=64, depth=3, normalization_type="batchnorm",
                                  normalization_groups=8, activation_function="relu"), (4, 256, 16, 12)),
    }
    for i, (key, (m, shape)) in enumerate(mods.items()):
        m = filler.fill_module(m).train()
        x = torch.from_numpy(filler.normal(71 + i, shape)).requires_grad_(True)
        y = m(x)
        gy = torch.from_numpy(filler.normal(81 + i, tuple(y.shape)))
        (y * gy).sum().backward()
        out[f"{key}_y"] = y.detach()
        out[f"{key}_gx"] = x.grad
        names = [n for n, p in m.named_parameters()]
        out[f"{key}_names"] = np.array(names)
        out[f"{key}_sumsq"] = np.array([float((p.grad.double() ** 2).sum()) for _, p in m.named_parameters()])
        out[f"{key}_sample"] = np.stack([np.pad(sample(p.grad).numpy(), (0, 64 - sample(p.grad).numel()))
                                         for _, p in m.named_parameters()])
    G.save("train_blocks", **out)


if __name__ == "__main__":
    import json
    cfgs = json.load(open(os.path.join(HERE, "configs.json")))
    gen_loss()
    gen_blocks()
    gen_step(cfgs["b0"]["model_kwargs"])

"""Training-path CPU restatement — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

* train-mode forward of the RGB hierarchical ROI path (BatchNorm with batch statistics and
  running-stat updates, normalization_comparison.py:181-182; Dropout given explicit masks or
  disabled), differentiable w.r.t. the parameters via torch autograd on the CPU;
* RefinedHierarchicalLoss (advanced/hierarchical_segmentation_refinement.py:807-1068) over
  HierarchicalLoss (advanced/hierarchical_segmentation.py:150-395) and DiceLoss (losses.py:9-88),
  with the EMA class-weight state of the reference (host floats);
* one reference optimiser step: clip_grad_norm_(1.0) + torch.optim.AdamW(lr, wd=0.01)
  (train_advanced.py:733-740, 1111-1143) — torch's own optimiser is the reference's dependency.

Pinned to tests/golden/train_loss.npz and train_step_b0.npz (reference run in the build container,
tests/golden/gen_train_golden.py).
"""
from __future__ import annotations

import contextlib
import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import rgb_model as RM
from .roi_align import linspace01

_STATE = {"train": False, "linspace": "scalar"}


def use_torch_linspace(flag: bool = True):
    """RoIAlign grid from torch.linspace (the reference's own call, dynamic_roi_align.py:110-111) instead of
    the scalar two-sided formula the kernel uses.  torch's CPU linspace rounds the last ulp by host SIMD
    width, which train-mode BatchNorm amplifies to ~1e-3; golden tests (same host as the reference run)
    use it to pin the oracle exactly, GPU parity tests keep the scalar grid of the kernel."""
    _STATE["linspace"] = "torch" if flag else "scalar"


@contextlib.contextmanager
def train_mode():
    """Within the block, oracle BatchNorm uses batch statistics and updates the running buffers in
    place (momentum 0.1, unbiased running variance), and RoIAlign is differentiable."""
    old = _STATE["train"]
    _STATE["train"] = True
    try:
        yield
    finally:
        _STATE["train"] = old


def is_train() -> bool:
    return _STATE["train"]


def bn_train(sd, p, x, eps=1e-5):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        True, 0.1, eps)


def roi_align_torch(feat: torch.Tensor, rois: torch.Tensor, oh: int, ow: int, scale_h, scale_w, aligned=True):
    """DynamicRoIAlign (dynamic_roi_align.py:56-171) as differentiable torch ops: the same sample
    coordinates as oracle/roi_align.py (float32), bilinear with zero padding as an explicit 4-tap gather."""
    B, C, H, W = feat.shape
    r = rois.detach().float()
    b = torch.trunc(r[:, 0]).long()
    x1, y1 = r[:, 1] * np.float32(scale_w), r[:, 2] * np.float32(scale_h)
    x2, y2 = r[:, 3] * np.float32(scale_w), r[:, 4] * np.float32(scale_h)
    if _STATE["linspace"] == "torch":
        gx, gy = torch.linspace(0, 1, ow), torch.linspace(0, 1, oh)
    else:
        gx, gy = torch.from_numpy(linspace01(ow)), torch.from_numpy(linspace01(oh))
    fx = x1[:, None] + gx[None, :] * (x2 - x1)[:, None]
    fy = y1[:, None] + gy[None, :] * (y2 - y1)[:, None]

    def unnorm(f, size):
        if aligned:
            n = (f / np.float32(size - 1)) * 2 - 1
            return (n + 1) * np.float32((size - 1) / 2)
        n = (f / np.float32(size)) * 2 - 1
        return (n + 1) * np.float32(size / 2) - np.float32(0.5)

    ix, iy = unnorm(fx, W), unnorm(fy, H)                       # [N, ow], [N, oh]
    x0, y0 = torch.floor(ix), torch.floor(iy)
    wx1, wy1 = ix - x0, iy - y0
    wx0, wy0 = 1 - wx1, 1 - wy1
    x0, y0 = x0.long(), y0.long()
    out = []
    for n in range(r.shape[0]):
        if not (0 <= int(b[n]) < B):
            out.append(feat.new_zeros(C, oh, ow))
            continue
        fm = feat[int(b[n])]
        acc = 0
        for yy, wy in ((y0[n], wy0[n]), (y0[n] + 1, wy1[n])):
            for xx, wx in ((x0[n], wx0[n]), (x0[n] + 1, wx1[n])):
                ok = ((yy >= 0) & (yy < H))[:, None] & ((xx >= 0) & (xx < W))[None, :]
                v = fm[:, yy.clamp(0, H - 1)][:, :, xx.clamp(0, W - 1)]
                acc = acc + v * (wy[:, None] * wx[None, :] * ok)[None]
        out.append(acc)
    return torch.stack(out)


# ---------------------------------------------------------------------------------------- loss
def _ce(logits, target, weight=None, reduction="mean"):
    if weight is not None:   # (float64 oracle runs: the class weights follow the logits' dtype)
        weight = weight.to(logits.dtype)
    return F.cross_entropy(logits, target, weight=weight, reduction=reduction)


class RefinedHierarchicalLoss:
    """Restatement of RefinedHierarchicalLoss with the train_advanced.py:551-568 weights."""

    def __init__(self, bg_weight=1.5, fg_weight=1.5, target_weight=1.2, consistency_weight=0.3, use_dynamic_weights=True,
                 dice_weight=1.0, ce_weight=1.0, boundary_aware_weight=0.1, contour_loss_weight=0.1,
                 distance_loss_weight=0.1, use_boundary_aware_loss=True, use_contour_detection=True,
                 use_distance_transform=True, base_mask_size=(64, 48)):
        self.bg_weight, self.fg_weight, self.target_weight = bg_weight, fg_weight, target_weight
        self.consistency_weight, self.dyn = consistency_weight, use_dynamic_weights
        self.dice_weight, self.ce_weight = dice_weight, ce_weight
        self.ba_w, self.c_w, self.d_w = boundary_aware_weight, contour_loss_weight, distance_loss_weight
        self.use_ba, self.use_c, self.use_d = use_boundary_aware_loss, use_contour_detection, use_distance_transform
        self.base_res = base_mask_size[0] * base_mask_size[1]
        self.ema = {"bg": 1.0, "fg": 1.0}          # hierarchical_segmentation.py:184-188
        self.ema_tn = None                          # created on first use (:286-296)
        self.last = {"bg": 1.0, "fg": 1.0, "t": 1.0, "nt": 1.0}

    def __call__(self, pred, target, aux):
        # ---- HierarchicalLoss.forward (hierarchical_segmentation.py:201-395)
        fg = (target > 0).long()
        bg_cnt, fg_cnt = (target == 0).float().sum(), fg.float().sum()
        tot = bg_cnt + fg_cnt
        if self.dyn:
            bw = (tot / (2 * bg_cnt.clamp(min=1))).clamp(0.5, 3.0)
            fw = (tot / (2 * fg_cnt.clamp(min=1)) * self.target_weight).clamp(0.5, 3.0)
            self.ema["bg"] = 0.9 * self.ema["bg"] + 0.1 * bw.item()
            self.ema["fg"] = 0.9 * self.ema["fg"] + 0.1 * fw.item()
            self.last["bg"], self.last["fg"] = self.ema["bg"], self.ema["fg"]
            w = torch.tensor([self.ema["bg"], self.ema["fg"]])
        else:
            self.last["bg"], self.last["fg"] = 1.0, self.target_weight
            w = torch.tensor([1.0, self.target_weight])
        bgfg_loss = _ce(aux["bg_fg_logits"], fg, w)
        tn_loss = torch.tensor(0.0)
        if fg.any():
            tn_t = (target == 2).long()
            t_cnt, nt_cnt = ((target == 1) & (fg > 0)).float().sum(), ((target == 2) & (fg > 0)).float().sum()
            ftot = t_cnt + nt_cnt
            if ftot > 0:
                if self.dyn:
                    tw = (ftot / (2 * t_cnt.clamp(min=1))).clamp(0.5, 3.0)
                    ntw = (ftot / (2 * nt_cnt.clamp(min=1))).clamp(0.5, 3.0)
                    if self.ema_tn is None:
                        self.ema_tn = [tw.item(), ntw.item()]
                    else:
                        self.ema_tn = [0.9 * self.ema_tn[0] + 0.1 * tw.item(), 0.9 * self.ema_tn[1] + 0.1 * ntw.item()]
                    cw = torch.tensor(self.ema_tn)
                    self.last["t"], self.last["nt"] = self.ema_tn
                else:
                    cw = torch.tensor([1.0, 1.0])
                    self.last["t"], self.last["nt"] = 1.0, 1.0
                l = _ce(aux["target_nontarget_logits"], tn_t, cw, "none")
                tn_loss = (l * fg.float()).sum() / fg.float().sum().clamp(min=1)
        final = _ce(pred, target)
        pb = F.softmax(aux["bg_fg_logits"], dim=1)
        pf = F.softmax(pred, dim=1)
        cons = F.mse_loss(pb[:, 1], pf[:, 1] + pf[:, 2])
        oh1 = (target == 1).float()
        inter = (pf[:, 1] * oh1).sum(dim=(1, 2))
        dice = (1 - (2 * inter + 1e-6) / (pf[:, 1].sum(dim=(1, 2)) + oh1.sum(dim=(1, 2)) + 1e-6)).mean()
        total = (self.bg_weight * bgfg_loss + self.fg_weight * tn_loss + self.ce_weight * final
                 + self.dice_weight * dice + self.consistency_weight * cons)
        with torch.no_grad():
            pr = aux["bg_fg_logits"].argmax(dim=1)
            acc = (pr == fg).float().mean().item()
            fp, ft = (pr == 1).float(), fg.float()
            iou = ((fp * ft).sum() / (fp + ft).clamp(max=1).sum().clamp(min=1)).item()
        d = {"bg_fg_loss": bgfg_loss.item(), "target_nontarget_loss": tn_loss.item(), "final_loss": final.item(),
             "consistency_loss": cons.item(), "total_loss": total.item(), "ce_loss": final.item(),
             "dice_loss": dice.item(), "aux_fg_bg_loss": bgfg_loss.item(), "aux_fg_accuracy": acc,
             "aux_fg_iou": iou, "bg_weight": self.last["bg"], "fg_weight": self.last["fg"],
             "target_weight": self.last["t"], "nontarget_weight": self.last["nt"]}
        # ---- refinement terms (refinement.py:930-984)
        if self.use_ba:
            ba = boundary_aware_loss(pred, target).clamp(max=10.0)
            total = total + self.ba_w * ba
            d["boundary_aware"] = ba.item()
        if self.use_c and "contours" in aux:
            cl = F.binary_cross_entropy_with_logits(aux["contours"], contour_targets(target)).clamp(max=10.0)
            H, W = target.shape[1:]
            wgt = max(0.001, min(self.c_w * float(np.sqrt(self.base_res / (H * W))), 0.5))
            total = total + wgt * cl
            d["contour"], d["contour_weight"] = cl.item(), wgt
        if self.use_d and "distance_map" in aux:
            dl = F.l1_loss(aux["distance_map"], distance_targets(target)).clamp(max=10.0)
            total = total + self.d_w * dl
            d["distance_transform"] = dl.item()
        return total, d


def boundary_aware_loss(pred, target, boundary_width=3, boundary_weight=2.0):
    """refinement.py:389-431 (called with boundary_weight=2.0 at :932-936)."""
    C = pred.shape[1]
    oh = F.one_hot(target, C).permute(0, 3, 1, 2).float()
    k = boundary_width
    dil = F.max_pool2d(oh, k, 1, k // 2)
    ero = 1 - F.max_pool2d(1 - oh, k, 1, k // 2)
    boundary = (dil - ero).sum(dim=1) > 0
    w = torch.ones_like(target, dtype=torch.float32)
    w[boundary] = boundary_weight
    return (_ce(pred, target, reduction="none") * w).mean()


def contour_targets(masks):
    """refinement.py:986-1040."""
    B, H, W = masks.shape
    t = (masks == 1).float()[:, None]
    dy = F.pad((t[:, :, 1:] - t[:, :, :-1]).abs(), (0, 0, 0, 1), mode="replicate")
    dx = F.pad((t[:, :, :, 1:] - t[:, :, :, :-1]).abs(), (0, 1, 0, 0), mode="replicate")
    c = torch.max(dy, dx)
    ew = max(1, int(np.sqrt(H * W / 3072) * 1.5))
    if ew > 1:
        ks = 2 * ew - 1
        c = (F.conv2d(c, torch.ones(1, 1, ks, ks) / (ks * ks), padding=ks // 2) > 0.1).float()
    return c


def distance_targets(masks):
    """refinement.py:1042-1068."""
    d = (masks == 1).float()[:, None]
    for _ in range(5):
        d = d + (1 - d) * F.max_pool2d(d, 3, 1, 1) * 0.5
    return d


# ---------------------------------------------------------------------------------------- model step
def params_of(module) -> Dict[str, torch.Tensor]:
    """state_dict copy with trainable parameters as leaf tensors requiring grad (frozen UNet excluded)."""
    sd = {k: v.detach().float().cpu().clone() for k, v in module.state_dict().items()}
    train_names = {n for n, p in module.named_parameters() if p.requires_grad}
    for n in train_names:
        sd[n].requires_grad_(True)
    return sd


def forward_train(sd, images, rois, u, cfg, scale_hw):
    """Train-mode forward of the ROI path from the UNet logit map (rgb.py:729-774)."""
    with train_mode():
        return RM.rgb_model_from_unet(sd, images, rois, u, cfg, scale_hw)


def adamw_step(params, grads, state, lr=1e-4, wd=0.01, betas=(0.9, 0.999), eps=1e-8, max_norm: Optional[float] = 1.0):
    """clip_grad_norm_ + torch.optim.AdamW step (train_advanced.py:733-740,1111-1143), in place."""
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads)).float()
    if max_norm is not None:
        coef = min(1.0, max_norm / (total.item() + 1e-6))
        grads = [g * coef for g in grads]
    state["step"] = state.get("step", 0) + 1
    t = state["step"]
    for i, (p, g) in enumerate(zip(params, grads)):
        m = state.setdefault(("m", i), torch.zeros_like(p))
        v = state.setdefault(("v", i), torch.zeros_like(p))
        with torch.no_grad():
            p.mul_(1 - lr * wd)
            m.mul_(betas[0]).add_(g, alpha=1 - betas[0])
            v.mul_(betas[1]).addcmul_(g, g, value=1 - betas[1])
            bc1, bc2 = 1 - betas[0] ** t, 1 - betas[1] ** t
            denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
            p.addcdiv_(m, denom, value=-lr / bc1)
    return total

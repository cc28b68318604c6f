"""Float32 CPU restatement of the RGB hierarchical path — TEST INFRASTRUCTURE ONLY.

Functional form over a state_dict (keys exactly as the reference's modules), torch CPU ops.
Citations are file:line in the reference (PINTO0309/human-instance-segmentation).
Eval-mode semantics by default (BatchNorm with running statistics, Dropout2d as identity);\noracle/train.py switches BatchNorm/RoIAlign to training semantics (Dropout stays identity: p = 0 in tests).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .roi_align import roi_align as _roi_align_np

SD = Dict[str, torch.Tensor]


# ---------------------------------------------------------------------------------------- primitives
def conv(sd: SD, p: str, x, stride=1, pad=None):
    w = sd[p + ".weight"]
    b = sd.get(p + ".bias")
    if pad is None:
        pad = w.shape[-1] // 2
    return F.conv2d(x, w, b, stride=stride, padding=pad)


def layernorm2d(sd: SD, p: str, x, eps=1e-5):
    """LayerNorm2d (src/human_edge_detection/model.py:18-38): per-sample mean / biased variance over
    (C, H, W), weight / bias [1, C, 1, 1].  Same in train and eval (no running statistics)."""
    mean = x.mean(dim=(1, 2, 3), keepdim=True)
    var = x.var(dim=(1, 2, 3), keepdim=True, unbiased=False)
    return (x - mean) / torch.sqrt(var + eps) * sd[p + ".weight"] + sd[p + ".bias"]


def bn(sd: SD, p: str, x, eps=1e-5):
    """The normalisation layer of get_normalization_layer (advanced/normalization_comparison.py:159-206):
    nn.BatchNorm2d (:181-182) with running statistics (eval), or batch statistics + running-stat update
    inside oracle.train.train_mode(); 'layernorm2d' (no running statistics in the state) -> layernorm2d."""
    if p + ".running_mean" not in sd:
        return layernorm2d(sd, p, x, eps)
    from . import train as _T
    if _T.is_train():
        return _T.bn_train(sd, p, x, eps)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, eps)


def act(x, kind: str, beta: float = 1.0):
    """advanced/activation_utils.py:71-101.  kind may carry Swish's beta as 'swish:<beta>' (cfg_from_kwargs)."""
    if ":" in kind:
        kind, b = kind.split(":")
        beta = float(b)
    if kind == "relu":
        return F.relu(x)
    if kind == "silu" or (kind == "swish" and beta == 1.0):
        return F.silu(x)
    if kind == "swish":
        return x * torch.sigmoid(beta * x)
    if kind == "gelu":
        return F.gelu(x)
    raise ValueError(kind)


def plain(a: str) -> str:
    """The activation of get_activation_function in unet.py:13-32 / rgb.py:21-40: 'swish' -> nn.SiLU
    (Swish's beta dropped), unlike activation_utils.get_activation used by the refinement modules."""
    return a.split(":")[0]


def residual(sd: SD, p: str, x, a: str):
    """ResidualBlock: refinement.py:46-55 (== unet.py:52-58 for eval)."""
    h = act(bn(sd, p + ".norm1", conv(sd, p + ".conv1", x)), a)
    h = bn(sd, p + ".norm2", conv(sd, p + ".conv2", h))
    return act(h + x, a)


def roi_align(feat: torch.Tensor, rois: torch.Tensor, oh: int, ow: int, scale_h, scale_w, aligned=True):
    """dynamic_roi_align.py:56-171 (numpy restatement in oracle/roi_align.py; differentiable torch
    form oracle.train.roi_align_torch inside train_mode())."""
    from . import train as _T
    if _T.is_train():
        return _T.roi_align_torch(feat, rois, oh, ow, scale_h, scale_w, aligned)
    out = _roi_align_np(feat.detach().numpy(), rois.detach().numpy(), oh, ow, scale_h, scale_w, aligned)
    return torch.from_numpy(out)


# ---------------------------------------------------------------------------------------- ROI path
def rgb_feature_extractor(sd: SD, p: str, x, a: str):
    """advanced/hierarchical_segmentation_rgb.py:657-673 (stand-alone activations from rgb.py:21-40,
    the residual blocks are refinement.py's with get_activation)."""
    x = act(bn(sd, p + ".1", conv(sd, p + ".0", x)), plain(a))
    x = residual(sd, p + ".3", x, a)
    x = act(bn(sd, p + ".5", conv(sd, p + ".4", x)), plain(a))
    x = residual(sd, p + ".7", x, a)
    x = act(bn(sd, p + ".9", conv(sd, p + ".8", x)), plain(a))
    x = residual(sd, p + ".11", x, a)
    return act(bn(sd, p + ".13", conv(sd, p + ".12", x)), plain(a))


def enhanced_unet(sd: SD, p: str, x, depth: int, a: str):
    """EnhancedUNet.forward, advanced/hierarchical_segmentation_unet.py:375-417 (every activation from
    unet.py's get_activation_function)."""
    a = plain(a)
    feats = []
    for i in range(depth):
        e = f"{p}.encoders.{i}"
        if i == 0:
            x = act(bn(sd, e + ".1", conv(sd, e + ".0", x)), a)
            x = residual(sd, e + ".3", x, a)
            x = residual(sd, e + ".4", x, a)
        else:
            x = residual(sd, e + ".0", x, a)
            x = residual(sd, e + ".1", x, a)
            x = act(bn(sd, e + ".3", conv(sd, e + ".2", x)), a)
        feats.append(x)
        if i < depth - 1:
            x = F.max_pool2d(x, 2)
    b = p + ".bottleneck"
    t = residual(sd, b + ".0", x, a)
    t = residual(sd, b + ".1", t, a)
    t = act(bn(sd, b + ".3", conv(sd, b + ".2", t)), a)
    att = torch.sigmoid(conv(sd, b + ".5", t))
    x = conv(sd, p + ".bottleneck_conv", x) * att
    for i in range(depth - 1):
        w = sd[f"{p}.upconvs.{i}.weight"]
        x = F.conv_transpose2d(x, w, sd[f"{p}.upconvs.{i}.bias"], stride=2)
        skip = feats[depth - 2 - i]
        x = F.interpolate(x, size=skip.shape[2:], mode="bilinear", align_corners=False)
        x = torch.cat([x, skip], dim=1)
        d = f"{p}.decoders.{i}"
        x = act(bn(sd, d + ".1", conv(sd, d + ".0", x)), a)
        x = residual(sd, d + ".3", x, a)
        x = residual(sd, d + ".4", x, a)
    f = p + ".final"
    x = act(bn(sd, f + ".1", conv(sd, f + ".0", x)), a)
    return conv(sd, f + ".3", x)


def channel_attention(sd: SD, p: str, x, a: str):
    """ChannelAttentionModule, advanced/attention_modules.py:45-64."""
    g = F.adaptive_avg_pool2d(x, 1)
    g = act(F.conv2d(g, sd[p + ".fc1.weight"]), a)
    g = torch.sigmoid(F.conv2d(g, sd[p + ".fc2.weight"]))
    return x * g


def spatial_attention(sd: SD, p: str, x):
    """SpatialAttentionModule, advanced/attention_modules.py:92-113."""
    s = torch.cat([x.mean(dim=1, keepdim=True), x.max(dim=1, keepdim=True)[0]], dim=1)
    w = sd[p + ".conv.weight"]
    return x * torch.sigmoid(F.conv2d(s, w, padding=w.shape[-1] // 2))


def hier_head(sd: SD, p: str, x, cfg: dict) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """RefinedHierarchicalSegmentationHead.forward (refinement.py:734-804) over
    ExtendedHierarchicalSegmentationHeadUNetV2.forward (refinement.py:550-606)."""
    a = cfg["activation_function"]
    mh, mw = cfg["mask_hw"]
    bh = p + ".base_head"
    s = act(bn(sd, bh + ".shared_features.1", conv(sd, bh + ".shared_features.0", x)), a)
    s = residual(sd, bh + ".shared_features.4", s, a)
    s = residual(sd, bh + ".shared_features.6", s, a)
    low = enhanced_unet(sd, bh + ".bg_vs_fg_unet", s, cfg["hierarchical_depth"], a)
    u = bh + ".upsample_bg_fg"
    bgfg = F.conv_transpose2d(low, sd[u + ".0.weight"], sd[u + ".0.bias"], stride=2)
    bgfg = conv(sd, u + ".3", act(bn(sd, u + ".1", bgfg), a))
    if bgfg.shape[2:] != (mh, mw):
        bgfg = F.interpolate(bgfg, size=(mh, mw), mode="bilinear", align_corners=False)
    p_fg = F.softmax(bgfg, dim=1)[:, 1]
    g = bh + ".fg_gate"
    fa = act(conv(sd, g + ".0", low), a)
    fa = act(conv(sd, g + ".3", fa), a)
    fa = torch.sigmoid(conv(sd, g + ".5", fa))
    t = s * fa
    tb = bh + ".target_vs_nontarget_branch"
    if cfg["use_attention_module"]:
        t = residual(sd, tb + ".0", t, a)
        t = spatial_attention(sd, tb + ".1", t)
        t = F.conv_transpose2d(t, sd[tb + ".3.weight"], sd[tb + ".3.bias"], stride=2)
        t = act(bn(sd, tb + ".4", t), a)
        t = channel_attention(sd, tb + ".6", t, a)
        t = residual(sd, tb + ".8", t, a)
        tn = conv(sd, tb + ".9", t)
    else:
        t = residual(sd, tb + ".0", t, a)
        t = F.conv_transpose2d(t, sd[tb + ".2.weight"], sd[tb + ".2.bias"], stride=2)
        t = act(bn(sd, tb + ".3", t), a)
        t = residual(sd, tb + ".6", t, a)
        tn = conv(sd, tb + ".7", t)
    if tn.shape[2:] != (mh, mw):
        tn = F.interpolate(tn, size=(mh, mw), mode="bilinear", align_corners=False)
    logits = torch.stack([bgfg[:, 0], bgfg[:, 1] + tn[:, 0] * p_fg, bgfg[:, 1] + tn[:, 1] * p_fg], dim=1)
    aux = {"bg_fg_logits": bgfg, "bg_fg_logits_low": low, "target_nontarget_logits": tn, "fg_attention": fa,
           "shared_features": s}
    if cfg.get("use_contour_detection"):
        c = p + ".contour_branch.contour_branch"
        h = act(bn(sd, c + ".1", conv(sd, c + ".0", s)), a)
        h = act(bn(sd, c + ".4", conv(sd, c + ".3", h)), a)
        h = torch.sigmoid(conv(sd, c + ".6", h))
        aux["contours"] = F.interpolate(h, size=(mh, mw), mode="bilinear", align_corners=False) \
            if h.shape[2:] != (mh, mw) else h
    if cfg.get("use_distance_transform"):
        d = p + ".distance_decoder"
        h = act(bn(sd, d + ".distance_head.1", conv(sd, d + ".distance_head.0", s)), a)
        h = residual(sd, d + ".distance_head.3", h, a)
        dmap = conv(sd, d + ".distance_head.4", h)
        dmask = torch.sigmoid((dmap - sd[d + ".threshold"]) * 10)
        if dmap.shape[2:] != (mh, mw):
            dmask = F.interpolate(dmask, size=(mh, mw), mode="bilinear", align_corners=False)
            dmap = F.interpolate(dmap, size=(mh, mw), mode="bilinear", align_corners=False)
        aux["distance_mask"], aux["distance_map"] = dmask, dmap
    return logits, aux


def rgb_model_from_unet(sd: SD, images, rois, u, cfg: dict, scale_hw) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet.forward (rgb.py:729-774) given the
    UNet logit map u [B,1,H,W] (the smp.Unet output of unet.py:1914)."""
    a = cfg["activation_function"]
    rh, rw = cfg["roi_hw"]
    two = conv(sd, "pretrained_unet.output_conv", u)           # unet.py:1990
    roi_feat = roi_align(two, rois, rh, rw, scale_hw[0], scale_hw[1], True)
    roi_rgb = roi_align(images, rois, rh, rw, scale_hw[0], scale_hw[1], True)
    feats = rgb_feature_extractor(sd, "rgb_feature_extractor", roi_rgb, a)
    comb = conv(sd, "feature_combiner", torch.cat([feats, roi_feat], dim=1))
    logits, aux = hier_head(sd, "segmentation_head", comb, cfg)
    aux.update(full_image_logits=two, roi_features=roi_feat, roi_patches=roi_rgb)
    return logits, aux


def cfg_from_kwargs(kw: dict) -> dict:
    """Normalise create_rgb_hierarchical_model kwargs (rgb.py:925-1027) for the oracle."""
    def hw(v):
        return (int(v[0]), int(v[1])) if isinstance(v, (list, tuple)) else (int(v), int(v))
    c = dict(kw)
    c["roi_hw"], c["mask_hw"] = hw(kw["roi_size"]), hw(kw["mask_size"])
    if c.get("activation_function") == "swish" and float(c.get("activation_beta", 1.0)) != 1.0:
        c["activation_function"] = f"swish:{float(c['activation_beta'])}"
    return c


# ---------------------------------------------------------------------------------------- EfficientNet-UNet
# Restated timm EfficientNet arch string / smp Unet (third-party; absent from the image): PARITY UNPINNED.
_ARCH = [("ds", 1, 3, 1, 1, 16), ("ir", 2, 3, 2, 6, 24), ("ir", 2, 5, 2, 6, 40), ("ir", 3, 3, 2, 6, 80),
         ("ir", 3, 5, 1, 6, 112), ("ir", 4, 5, 2, 6, 192), ("ir", 1, 3, 1, 6, 320)]
_MULT = {"b0": (1.0, 1.0), "b1": (1.0, 1.1), "b2": (1.1, 1.2), "b3": (1.2, 1.4), "b4": (1.4, 1.8),
         "b5": (1.6, 2.2), "b6": (1.8, 2.6), "b7": (2.0, 3.1)}


def _div8(v: float) -> int:
    n = max(8, int(v + 4) // 8 * 8)
    return n + 8 if n < 0.9 * v else n


def _se(sd: SD, p: str, x):
    g = x.mean(dim=(2, 3), keepdim=True)
    g = F.silu(conv(sd, p + ".conv_reduce", g))
    return x * torch.sigmoid(conv(sd, p + ".conv_expand", g))


def _dw(sd: SD, p: str, x, stride):
    w = sd[p + ".weight"]
    return F.conv2d(x, w, None, stride=stride, padding=w.shape[-1] // 2, groups=w.shape[0])


def effunet_logits(sd: SD, p: str, x_norm, variant: str):
    """smp.Unet('timm-efficientnet-<variant>') forward on normalised input -> [B,1,H,W]."""
    wm, dm = _MULT[variant]
    e = p + ".encoder"
    x = F.silu(bn(sd, e + ".bn1", conv(sd, e + ".conv_stem", x_norm, stride=2, pad=1)))
    feats = [x]
    cin = _div8(32 * wm)
    for si, (bt, reps, k, s, ex, c) in enumerate(_ARCH):
        cout = _div8(c * wm)
        for r in range(int(math.ceil(reps * dm))):
            stride = s if r == 0 else 1
            b = f"{e}.blocks.{si}.{r}"
            skip = stride == 1 and cin == cout
            if bt == "ds":
                h = F.silu(bn(sd, b + ".bn1", _dw(sd, b + ".conv_dw", x, stride)))
                h = _se(sd, b + ".se", h)
                h = bn(sd, b + ".bn2", conv(sd, b + ".conv_pw", h))
            else:
                h = F.silu(bn(sd, b + ".bn1", conv(sd, b + ".conv_pw", x)))
                h = F.silu(bn(sd, b + ".bn2", _dw(sd, b + ".conv_dw", h, stride)))
                h = _se(sd, b + ".se", h)
                h = bn(sd, b + ".bn3", conv(sd, b + ".conv_pwl", h))
            x = h + x if skip else h
            cin = cout
        if si + 1 in (2, 3, 5, 7):
            feats.append(x)
    skips = feats[-2::-1]
    x = feats[-1]
    i = 0
    while f"{p}.decoder.blocks.{i}.conv1.0.weight" in sd:
        d = f"{p}.decoder.blocks.{i}"
        x = F.interpolate(x, scale_factor=2, mode="nearest")
        if i < len(skips):
            x = torch.cat([x, skips[i]], dim=1)
        x = F.relu(bn(sd, d + ".conv1.1", conv(sd, d + ".conv1.0", x)))
        x = F.relu(bn(sd, d + ".conv2.1", conv(sd, d + ".conv2.0", x)))
        i += 1
    return conv(sd, p + ".segmentation_head.0", x)


def pretrained_unet_logits(sd: SD, images, variant: str):
    """PreTrainedPeopleSegmentationUNet.forward (unet.py:1885-1916)."""
    x = images
    if x.max() > 1.0:
        x = x / 255.0
    x = (x - sd["pretrained_unet.model.norm_mean"]) / sd["pretrained_unet.model.norm_std"]
    return effunet_logits(sd, "pretrained_unet.model.model", x, variant)


def rgb_model(sd: SD, images, rois, cfg: dict, scale_hw, variant: str):
    u = pretrained_unet_logits(sd, images, variant)
    logits, aux = rgb_model_from_unet(sd, images, rois, u, cfg, scale_hw)
    return logits, aux, u


def instance_masks(logits: torch.Tensor, dilation: int = 0) -> torch.Tensor:
    """export_onnx_advanced.py:360-364 (+ MaskDilationModule, export_hierarchical_instance_peopleseg_onnx.py:85-141)."""
    if dilation > 0:
        probs = F.softmax(logits, dim=1)[:, 1:2]
        dil = F.max_pool2d(probs, 2 * dilation + 1, stride=1, padding=dilation)
        logits = logits.clone()
        logits[:, 1:2] = torch.where((dil - probs) > 0.1, logits[:, 1:2] + 2.0, logits[:, 1:2])
    cls = torch.argmax(logits, dim=1, keepdim=True)
    return (cls == 1).float()


def binary_masks(sd: SD, u: torch.Tensor) -> torch.Tensor:
    """export_onnx_advanced.py:374-387: softmax(output_conv(u))[:, 0:1]."""
    return F.softmax(conv(sd, "pretrained_unet.output_conv", u), dim=1)[:, 0:1]


def np_state(module) -> SD:
    return {k: v.detach().float().cpu() for k, v in module.state_dict().items()}


__all__ = ["roi_align", "residual", "enhanced_unet", "hier_head", "rgb_model_from_unet", "rgb_model",
           "effunet_logits", "pretrained_unet_logits", "instance_masks", "binary_masks", "cfg_from_kwargs",
           "np_state", "np"]

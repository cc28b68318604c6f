"""Standard-op ONNX lowering of the two composite hiseg ops (``hiseg::unet_logit``, ``hiseg::rgb_head``).

The reference deploys its model as an ONNX file of standard operators (export_onnx_advanced.py:338-457, opset 16,
consumed by onnxruntime in test_hierarchical_instance_peopleseg_onnx.py:170-196).  hiseg's traced modules emit
custom ops at the reference's module boundaries (export.py); for ``torch.onnx.export`` each op needs a symbolic
function.  The four leaf ops (RoIAlign, output conv, instance / binary masks) already lower to standard operators;
this module lowers the two composite ones the same way, so the exported graph runs in any ONNX runtime:

* ``unet_logit``: PreTrainedPeopleSegmentationUNet.forward (hierarchical_segmentation_unet.py:1885-1916) -- the
  data-dependent /255 (ReduceMax > 1 -> Where), the mean / std normalisation, the smp EfficientNet-UNet
  (stem, MBConv / depthwise-separable blocks with squeeze-excite, nearest x2 decoder with skip concats,
  3x3 segmentation head; restated from timm / smp, see effunet.py).
* ``rgb_head``: HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet.forward from the UNet logit on
  (hierarchical_segmentation_rgb.py:729-774): output conv, both RoIAligns (export._onnx_roi_align: GridSample),
  the RGB feature extractor, the 258 -> 256 combiner, and the refined hierarchical head
  (hierarchical_segmentation_refinement.py:550-606, 734-804) with every aux output the spec lists.

Every emitter walks the module skeleton the op's JSON spec rebuilds (export._skeleton: structure only, no
weights) and takes each parameter from the op's state inputs by its state_dict name, so the weights stay graph
inputs / initialisers exactly as in the reference's export.  BatchNorm is emitted in inference form
(BatchNormalization); the reference's exporter script folds it into an affine afterwards
(export_hierarchical_instance_peopleseg_onnx.py:474-480), which any ONNX optimiser does the same way.

``g`` is anything with ``op(name, *inputs, **attributes)`` in the TorchScript exporter's attribute convention
(``axis_i``, ``mode_s``, ``value_t`` ...): the exporter's graph context, or tests/test_export.py's eager
interpreter, which checks these graphs against the CPU oracle.
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
import torch.nn as nn

from . import effunet as EU
from . import layers as LY


class Emitter:
    """ONNX node emission over one module skeleton and its named state values."""

    def __init__(self, g, root: nn.Module, values: Dict[str, object]):
        self.g = g
        self.values = values
        self.names = {id(m): n for n, m in root.named_modules()}

    # -- constants and parameters
    def const(self, v, dtype=torch.float32):
        return self.g.op("Constant", value_t=torch.tensor(v, dtype=dtype))

    def p(self, m: nn.Module, attr: str):
        n = self.names[id(m)]
        return self.values[f"{n}.{attr}" if n else attr]

    def op(self, name, *xs, **at):
        return self.g.op(name, *xs, **at)

    # -- layers
    def conv(self, m: nn.Conv2d, x):
        kh, kw = m.kernel_size
        ins = [x, self.p(m, "weight")] + ([self.p(m, "bias")] if m.bias is not None else [])
        return self.op("Conv", *ins, kernel_shape_i=[kh, kw], strides_i=list(m.stride),
                       pads_i=[m.padding[0], m.padding[1], m.padding[0], m.padding[1]], group_i=m.groups,
                       dilations_i=list(m.dilation))

    def conv_t(self, m: nn.ConvTranspose2d, x):
        kh, kw = m.kernel_size
        return self.op("ConvTranspose", x, self.p(m, "weight"), self.p(m, "bias"), kernel_shape_i=[kh, kw],
                       strides_i=list(m.stride), pads_i=[0, 0, 0, 0])

    def norm(self, m: nn.Module, x):
        if isinstance(m, nn.BatchNorm2d):   # eval: running statistics (normalization_comparison.py:181-182)
            return self.op("BatchNormalization", x, self.p(m, "weight"), self.p(m, "bias"), self.p(m, "running_mean"),
                           self.p(m, "running_var"), epsilon_f=float(m.eps))
        if isinstance(m, LY.LayerNorm2d):   # model.py:18-38: per sample over (C, H, W), biased variance
            mean = self.op("ReduceMean", x, axes_i=[1, 2, 3], keepdims_i=1)
            d = self.op("Sub", x, mean)
            var = self.op("ReduceMean", self.op("Mul", d, d), axes_i=[1, 2, 3], keepdims_i=1)
            xn = self.op("Div", d, self.op("Sqrt", self.op("Add", var, self.const(float(m.eps)))))
            return self.op("Add", self.op("Mul", xn, self.p(m, "weight")), self.p(m, "bias"))
        raise NotImplementedError(f"ONNX lowering: normalisation {type(m).__name__}")

    def sigmoid(self, x):
        return self.op("Sigmoid", x)

    def act(self, m: nn.Module, x):
        """activation_utils.py:71-101 / unet.py:13-32 by module type (SiLU and Swish as x * sigmoid(beta x); GELU in
        its exact erf form -- opset 17 has neither as an operator)."""
        if isinstance(m, nn.ReLU):
            return self.op("Relu", x)
        if isinstance(m, nn.SiLU):
            return self.op("Mul", x, self.sigmoid(x))
        if isinstance(m, LY.Swish):
            bx = x if float(m.beta) == 1.0 else self.op("Mul", x, self.const(float(m.beta)))
            return self.op("Mul", x, self.sigmoid(bx))
        if isinstance(m, nn.GELU):
            e = self.op("Erf", self.op("Mul", x, self.const(1.0 / math.sqrt(2.0))))
            return self.op("Mul", self.op("Mul", x, self.const(0.5)), self.op("Add", e, self.const(1.0)))
        if isinstance(m, nn.Sigmoid):
            return self.sigmoid(x)
        if isinstance(m, (nn.Identity, nn.Dropout, nn.Dropout2d)):
            return x
        raise NotImplementedError(f"ONNX lowering: activation {type(m).__name__}")

    def cna(self, conv, norm, act, x):
        return self.act(act, self.norm(norm, self.conv(conv, x)))

    def residual(self, blk: LY.ResidualBlock, x):
        """ResidualBlock (refinement.py:46-55, unet.py:52-58): act(norm2(conv2(act(norm1(conv1 x)))) + x)."""
        a1 = getattr(blk, "activation1", None) or blk.activation
        a2 = getattr(blk, "activation2", None) or blk.activation
        h = self.cna(blk.conv1, blk.norm1, a1, x)
        h = self.norm(blk.norm2, self.conv(blk.conv2, h))
        return self.act(a2, self.op("Add", h, x))

    def channel_slice(self, x, a: int, b: int):
        return self.op("Slice", x, self.const([a], torch.int64), self.const([b], torch.int64),
                       self.const([1], torch.int64))

    def resize_to(self, x, hw, mode="linear"):
        """F.interpolate(size=hw, bilinear, align_corners=False) -- pytorch_half_pixel."""
        nc = self.op("Slice", self.op("Shape", x), self.const([0], torch.int64), self.const([2], torch.int64),
                     self.const([0], torch.int64))
        sizes = self.op("Concat", nc, self.const([int(hw[0]), int(hw[1])], torch.int64), axis_i=0)
        return self.op("Resize", x, self.const([], torch.float32), self.const([], torch.float32), sizes,
                       mode_s=mode, coordinate_transformation_mode_s="pytorch_half_pixel")

    def up2_nearest(self, x):
        """F.interpolate(scale_factor=2, mode='nearest') (smp DecoderBlock)."""
        return self.op("Resize", x, self.const([], torch.float32), self.const([1.0, 1.0, 2.0, 2.0]), mode_s="nearest",
                       coordinate_transformation_mode_s="asymmetric", nearest_mode_s="floor")

    def maxpool2(self, x):
        return self.op("MaxPool", x, kernel_shape_i=[2, 2], pads_i=[0, 0, 0, 0], strides_i=[2, 2])


# ------------------------------------------------------------------------------------ EfficientNet-UNet
def _se(e: Emitter, se: EU.SqueezeExcite, x):
    s = e.op("GlobalAveragePool", x)
    s = e.act(se.act1, e.conv(se.conv_reduce, s))
    return e.op("Mul", x, e.sigmoid(e.conv(se.conv_expand, s)))


def _silu(e: Emitter, x):
    return e.op("Mul", x, e.sigmoid(x))


def emit_effunet(e: Emitter, net: EU.EfficientNetUnet, x):
    """smp.Unet('timm-efficientnet-bX') on the normalised input -> [B, 1, H, W] (effunet.py; timm
    _gen_efficientnet, smp UnetDecoder / SegmentationHead)."""
    enc = net.encoder
    x = _silu(e, e.norm(enc.bn1, e.conv(enc.conv_stem, x)))
    feats = [x]
    for si, stage in enumerate(enc.blocks):
        for b in stage:
            if isinstance(b, EU.DepthwiseSeparableConv):
                h = _silu(e, e.norm(b.bn1, e.conv(b.conv_dw, x)))
                h = _se(e, b.se, h)
                h = e.norm(b.bn2, e.conv(b.conv_pw, h))
            else:
                h = _silu(e, e.norm(b.bn1, e.conv(b.conv_pw, x)))
                h = _silu(e, e.norm(b.bn2, e.conv(b.conv_dw, h)))
                h = _se(e, b.se, h)
                h = e.norm(b.bn3, e.conv(b.conv_pwl, h))
            x = e.op("Add", h, x) if b.has_skip else h
        if si + 1 in EU.STAGE_IDXS + (len(enc.blocks),):
            feats.append(x)
    skips = feats[-2::-1]
    x = feats[-1]
    for i, blk in enumerate(net.decoder.blocks):
        x = e.up2_nearest(x)
        if i < len(skips):
            x = e.op("Concat", x, skips[i], axis_i=1)
        x = e.cna(blk.conv1[0], blk.conv1[1], blk.conv1[2], x)
        x = e.cna(blk.conv2[0], blk.conv2[1], blk.conv2[2], x)
    return e.conv(net.segmentation_head[0], x)


def emit_unet_logit(g, pre: nn.Module, values: Dict[str, object], images):
    """PreTrainedPeopleSegmentationUNet.forward (unet.py:1885-1916): if images.max() > 1: /255; (x - mean) / std;
    the smp network."""
    e = Emitter(g, pre, values)
    big = e.op("Greater", e.op("ReduceMax", images, keepdims_i=0), e.const(1.0))
    x = e.op("Where", big, e.op("Div", images, e.const(255.0)), images)
    x = e.op("Div", e.op("Sub", x, values["norm_mean"]), values["norm_std"])
    return emit_effunet(e, pre.model, x)


# ------------------------------------------------------------------------------------ the ROI path
def _enhanced_unet(e: Emitter, u: LY.EnhancedUNet, x, hw):
    """EnhancedUNet.forward (hierarchical_segmentation_unet.py:375-417) on an input of spatial size hw."""
    lv = [tuple(hw)]   # spatial size per encoder level (MaxPool2d(2) floors)
    for _ in range(u.depth - 1):
        lv.append((lv[-1][0] // 2, lv[-1][1] // 2))
    feats = []
    for i, enc in enumerate(u.encoders):
        if i == 0:
            x = e.cna(enc[0], enc[1], enc[2], x)
            x = e.residual(enc[3], x)
            x = e.residual(enc[4], x)
        else:
            x = e.residual(enc[0], x)
            x = e.residual(enc[1], x)
            x = e.cna(enc[2], enc[3], enc[4], x)
        feats.append(x)
        if i < u.depth - 1:
            x = e.maxpool2(x)
    b = u.bottleneck
    t = e.residual(b[0], x)
    t = e.residual(b[1], t)
    t = e.cna(b[2], b[3], b[4], t)
    att = e.sigmoid(e.conv(b[5], t))
    x = e.op("Mul", e.conv(u.bottleneck_conv, x), att)
    for i, (up, dec) in enumerate(zip(u.upconvs, u.decoders)):
        x = e.conv_t(up, x)
        lo, hi = lv[u.depth - 1 - i], lv[u.depth - 2 - i]
        skip = feats[u.depth - 2 - i]
        if (2 * lo[0], 2 * lo[1]) != hi:   # bilinear resize to the skip (:408; identity at the configured sizes)
            x = e.resize_to(x, hi)
        x = e.op("Concat", x, skip, axis_i=1)
        x = e.cna(dec[0], dec[1], dec[2], x)
        x = e.residual(dec[3], x)
        x = e.residual(dec[4], x)
    f = u.final
    return e.conv(f[3], e.cna(f[0], f[1], f[2], x))


def _spatial_attention(e: Emitter, m: LY.SpatialAttentionModule, x):
    s = e.op("Concat", e.op("ReduceMean", x, axes_i=[1], keepdims_i=1), e.op("ReduceMax", x, axes_i=[1], keepdims_i=1),
             axis_i=1)
    return e.op("Mul", x, e.sigmoid(e.conv(m.conv, s)))


def _channel_attention(e: Emitter, m: LY.ChannelAttentionModule, x):
    s = e.op("GlobalAveragePool", x)
    s = e.act(m.activation, e.conv(m.fc1, s))
    return e.op("Mul", x, e.sigmoid(e.conv(m.fc2, s)))


def emit_rgb_head(g, model: nn.Module, values: Dict[str, object], images, u, rois, scale_hw, outs: List[str]):
    """rgb.py:729-774 from the UNet logit u on; returns the tensors named in ``outs`` (export.rgb_out_templates)."""
    from .export import _onnx_roi_align
    e = Emitter(g, model, values)
    (rh, rw), (mh, mw) = model.roi_size, model.mask_size
    sh, sw = float(scale_hw[0]), float(scale_hw[1])
    two = e.conv(model.pretrained_unet.output_conv, u)                                # unet.py:1990
    roi_feat = _onnx_roi_align(g, two, rois, rh, rw, sh, sw, True)                   # rgb.py:749
    roi_rgb = _onnx_roi_align(g, images, rois, rh, rw, sh, sw, True)                 # rgb.py:752
    fx = model.rgb_feature_extractor                                                 # rgb.py:657-673
    x = e.cna(fx[0], fx[1], fx[2], roi_rgb)
    x = e.residual(fx[3], x)
    x = e.cna(fx[4], fx[5], fx[6], x)
    x = e.residual(fx[7], x)
    x = e.cna(fx[8], fx[9], fx[10], x)
    x = e.residual(fx[11], x)
    x = e.cna(fx[12], fx[13], fx[14], x)
    comb = e.conv(model.feature_combiner, e.op("Concat", x, roi_feat, axis_i=1))      # rgb.py:758-762

    head = model.segmentation_head
    bh = head.base_head
    sf = bh.shared_features                                                        # refinement.py:479-487
    s = e.cna(sf[0], sf[1], sf[2], comb)
    s = e.residual(sf[4], s)
    s = e.residual(sf[6], s)
    low = _enhanced_unet(e, bh.bg_vs_fg_unet, s, (rh, rw))
    ub = bh.upsample_bg_fg                                                         # refinement.py:501-506
    bgfg = e.conv(ub[3], e.act(ub[2], e.norm(ub[1], e.conv_t(ub[0], low))))
    if (2 * rh, 2 * rw) != (mh, mw):
        bgfg = e.resize_to(bgfg, (mh, mw))
    p_fg = e.channel_slice(e.op("Softmax", bgfg, axis_i=1), 1, 2)                   # refinement.py:559-567
    fg = bh.fg_gate                                                                # refinement.py:537-545
    fa = e.act(fg[1], e.conv(fg[0], low))
    fa = e.act(fg[4], e.conv(fg[3], fa))
    fa = e.sigmoid(e.conv(fg[5], fa))
    t = e.op("Mul", s, fa)
    tb = bh.target_vs_nontarget_branch                                             # refinement.py:509-523
    if bh.use_attention_module:
        t = e.residual(tb[0], t)
        t = _spatial_attention(e, tb[1], t)
        t = e.act(tb[5], e.norm(tb[4], e.conv_t(tb[3], t)))
        t = _channel_attention(e, tb[6], t)
        t = e.residual(tb[8], t)
        tn = e.conv(tb[9], t)
    else:
        t = e.residual(tb[0], t)
        t = e.act(tb[4], e.norm(tb[3], e.conv_t(tb[2], t)))
        t = e.residual(tb[6], t)
        tn = e.conv(tb[7], t)
    if (2 * rh, 2 * rw) != (mh, mw):
        tn = e.resize_to(tn, (mh, mw))
    # hierarchical combine (refinement.py:588-596): [bg0, bg1 + tn0 p_fg, bg1 + tn1 p_fg]
    b0, b1 = e.channel_slice(bgfg, 0, 1), e.channel_slice(bgfg, 1, 2)
    l1 = e.op("Add", b1, e.op("Mul", e.channel_slice(tn, 0, 1), p_fg))
    l2 = e.op("Add", b1, e.op("Mul", e.channel_slice(tn, 1, 2), p_fg))
    d = {"logits": e.op("Concat", b0, l1, l2, axis_i=1), "bg_fg_logits": bgfg, "bg_fg_logits_low": low,
         "target_nontarget_logits": tn, "fg_attention": fa, "shared_features": s, "full_image_logits": two,
         "roi_features": roi_feat, "roi_patches": roi_rgb}
    if head.use_contour_detection and "contours" in outs:                          # refinement.py:255-295, 775-785
        cb = head.contour_branch.contour_branch
        c = e.cna(cb[0], cb[1], cb[2], s)
        c = e.cna(cb[3], cb[4], cb[5], c)
        c = e.sigmoid(e.conv(cb[6], c))
        d["contours"] = e.resize_to(c, (mh, mw)) if (rh, rw) != (mh, mw) else c
    if head.use_distance_transform and ("distance_map" in outs or "distance_mask" in outs):   # :298-344, 786-800
        dd = head.distance_decoder
        dh = dd.distance_head
        h = e.cna(dh[0], dh[1], dh[2], s)
        h = e.residual(dh[3], h)
        dmap = e.conv(dh[4], h)
        dmask = e.sigmoid(e.op("Mul", e.op("Sub", dmap, e.p(dd, "threshold")), e.const(10.0)))
        if (rh, rw) != (mh, mw):
            dmask, dmap = e.resize_to(dmask, (mh, mw)), e.resize_to(dmap, (mh, mw))
        d["distance_mask"], d["distance_map"] = dmask, dmap
    return [d[n] for n in outs]

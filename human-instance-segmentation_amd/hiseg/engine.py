"""Execution of the RGB hierarchical path on libhiseg kernels.

The modules in :mod:`hiseg.model` / :mod:`hiseg.layers` / :mod:`hiseg.effunet` only hold
parameters.  This module walks them in the reference's forward order and issues one
libhiseg call per fused layer:

* every Conv2d(+BatchNorm2d eval)(+activation)(+residual add)(+gate multiply) is ONE
  implicit-GEMM launch (hiseg_conv2d_fwd) with BN/bias folded into a per-channel affine;
* concatenations (feature_combiner input, EnhancedUNet / smp decoder skips) never exist in
  memory: the conv loader reads its K range from two sources (and upsamples source A ×2 for
  the smp decoder);
* the trainable 1→2 output_conv of the pretrained-UNet wrapper is fused into the RoIAlign
  gather, the whole upsample_bg_fg branch and the target branch's last 1×1 into the
  hierarchical combine kernel.

Packed weights ("plans") are cached per model, compute dtype and device and rebuilt when
any parameter or buffer changes (tensor version counters).  Activations are NHWC.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .effunet import DepthwiseSeparableConv, InvertedResidual
from .layers import LayerNorm2d, Swish
from .ops import Act, round_up

ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_SILU = L.ACT_NONE, L.ACT_RELU, L.ACT_SIGMOID, L.ACT_SILU
ACT_GELU, ACT_SWISH = L.ACT_GELU, L.ACT_SWISH


# ------------------------------------------------------------------------------------ plans
def act_code(m: nn.Module) -> int:
    """The hiseg activation code of an activation module (advanced/activation_utils.py:71-101).
    Swish(beta != 1) returns an L.ActCode carrying beta."""
    if isinstance(m, nn.ReLU):
        return ACT_RELU
    if isinstance(m, nn.SiLU):
        return ACT_SILU
    if isinstance(m, Swish):
        return ACT_SILU if float(m.beta) == 1.0 else L.ActCode(ACT_SWISH, float(m.beta))
    if isinstance(m, nn.GELU):
        if getattr(m, "approximate", "none") != "none":
            raise NotImplementedError("tanh-approximate GELU is not in the reference's activation factory")
        return ACT_GELU
    if isinstance(m, nn.Sigmoid):
        return ACT_SIGMOID
    if isinstance(m, nn.Identity):
        return ACT_NONE
    raise NotImplementedError(f"activation {type(m).__name__} is not in the reference's activation factory")


def _bn(m: Optional[nn.Module]):
    if m is None:
        return None
    if isinstance(m, nn.BatchNorm2d):
        if m.training:
            raise NotImplementedError("batch-statistics BatchNorm (train mode) is not on the hiseg inference path")
        return m
    if isinstance(m, LayerNorm2d):
        raise AssertionError("LayerNorm2d has per-sample statistics and cannot be folded into a conv plan (use cna)")
    raise NotImplementedError(f"normalisation {type(m).__name__}")


def _signature(tensors):
    return tuple((t.data_ptr(), t._version) for t in tensors if t is not None)


def _bn_tensors(bn):
    if bn is None:
        return ()
    return (getattr(bn, "weight", None), getattr(bn, "bias", None), getattr(bn, "running_mean", None),
            getattr(bn, "running_var", None))


class Ctx:
    """Per-forward context: compute dtype, device and the model's plan cache.

    Every plan records the (storage, version) of the tensors it was packed from and is rebuilt only when one
    of them changed -- so a training step that updates some parameters (or train-mode BN running statistics)
    re-packs just those layers, not the whole model (the frozen encoder of the distillation student, the
    teacher)."""

    def __init__(self, root: nn.Module, dtype: torch.dtype, device: torch.device):
        if dtype not in (torch.float32, torch.bfloat16):
            raise TypeError(f"hiseg compute dtype must be float32 or bfloat16, got {dtype}")
        self.dtype, self.device = dtype, device
        cache = root.__dict__.get("_hiseg_plans")
        if cache is None or cache["dtype"] != dtype or cache["device"] != device:
            cache = {"dtype": dtype, "device": device, "plans": {}}
            root.__dict__["_hiseg_plans"] = cache
        self.plans: Dict = cache["plans"]

    def _get(self, key, build, deps=()):
        sig = _signature(deps)
        ent = self.plans.get(key)
        if ent is None or ent[0] != sig:
            ent = (sig, build())
            self.plans[key] = ent
        return ent[1]

    def conv(self, conv: nn.Conv2d, bn=None, act: int = ACT_NONE, split=None) -> ops.ConvPlan:
        def build():
            assert conv.groups == 1 and conv.dilation in ((1, 1), 1)
            assert conv.kernel_size[0] == conv.kernel_size[1] and conv.stride[0] == conv.stride[1]
            return ops.pack_conv(conv.weight, conv.bias, _bn(bn), act, self.dtype, self.device,
                                 stride=conv.stride[0], pad=conv.padding[0], split=split)
        return self._get(("conv", id(conv), act, split), build, (conv.weight, conv.bias) + _bn_tensors(bn))

    def convT(self, conv: nn.ConvTranspose2d, bn=None, act: int = ACT_NONE) -> ops.ConvPlan:
        def build():
            assert conv.kernel_size == (2, 2) and conv.stride == (2, 2) and conv.padding == (0, 0)
            return ops.pack_convT2x2(conv.weight, conv.bias, _bn(bn), act, self.dtype, self.device)
        return self._get(("convT", id(conv), act), build, (conv.weight, conv.bias) + _bn_tensors(bn))

    def f32(self, t: torch.Tensor, shape=None) -> torch.Tensor:
        def build():
            v = t.detach().to(device=self.device, dtype=torch.float32).contiguous()
            return v.view(shape) if shape is not None else v
        return self._get(("f32", id(t), shape), build, (t,))

    def affine(self, key, cout, bias, bn):
        def build():
            s, h = ops.fold_affine(cout, bias, _bn(bn), self.device)
            return s.contiguous(), h.contiguous()
        return self._get(("aff", key), build, (bias,) + _bn_tensors(bn))

    def dw(self, conv: nn.Conv2d, bn):
        def build():
            c, _, k, _ = conv.weight.shape
            w = conv.weight.detach().float().to(self.device).view(c, k * k).t().contiguous()
            s, h = ops.fold_affine(c, conv.bias, _bn(bn), self.device)
            return w, s.contiguous(), h.contiguous(), k, conv.stride[0]
        return self._get(("dw", id(conv)), build, (conv.weight, conv.bias) + _bn_tensors(bn))


def cna(E: Ctx, conv: nn.Module, norm: Optional[nn.Module], act: int, x: Act, xb: Optional[Act] = None, *,
        split=None, residual: Optional[Act] = None, out: Optional[Act] = None, convT: bool = False) -> Act:
    """conv -> norm -> (+ residual) -> act.  Eval BatchNorm (or no norm) folds into the conv launch;
    LayerNorm2d (model.py:18-38) needs the conv output's per-sample statistics first: raw conv (+ bias),
    then ops.layernorm2d (statistics + one apply pass with residual and activation)."""
    if isinstance(norm, LayerNorm2d):
        plan = E.convT(conv, None, ACT_NONE) if convT else E.conv(conv, None, ACT_NONE, split=split)
        z = ops.conv2d(plan, x, xb)
        C = z.C
        return ops.layernorm2d(z, E.f32(norm.weight, (C,)), E.f32(norm.bias, (C,)), norm.eps, act,
                               residual=residual, out=out)
    plan = E.convT(conv, norm, act) if convT else E.conv(conv, norm, act, split=split)
    return ops.conv2d(plan, x, xb, residual=residual, out=out)


def _check_input(x: torch.Tensor, what: str):
    if not x.is_cuda:
        raise RuntimeError(f"{what}: hiseg runs on the GPU only (got a CPU tensor); there is no CPU fallback")


# ------------------------------------------------------------------------------------ blocks
def residual_block(E: Ctx, blk: nn.Module, x: Act, out: Optional[Act] = None) -> Act:
    """ResidualBlock (refinement.py:31-55 / unet.py:35-58): two fused launches."""
    a1 = act_code(blk.activation1 if hasattr(blk, "activation1") else blk.activation)
    a2 = act_code(blk.activation2 if hasattr(blk, "activation2") else blk.activation)
    h = cna(E, blk.conv1, blk.norm1, a1, x)
    return cna(E, blk.conv2, blk.norm2, a2, h, residual=x, out=out)


def rgb_feature_extractor(E: Ctx, seq: nn.Sequential, x: Act) -> Act:
    """hierarchical_segmentation_rgb.py:657-673."""
    h = cna(E, seq[0], seq[1], act_code(seq[2]), x)
    h = residual_block(E, seq[3], h)
    h = cna(E, seq[4], seq[5], act_code(seq[6]), h)
    h = residual_block(E, seq[7], h)
    h = cna(E, seq[8], seq[9], act_code(seq[10]), h)
    h = residual_block(E, seq[11], h)
    return cna(E, seq[12], seq[13], act_code(seq[14]), h)


def enhanced_unet(E: Ctx, u: nn.Module, x: Act) -> Tuple[Act, Act]:
    """EnhancedUNet.forward (hierarchical_segmentation_unet.py:375-417).

    Returns the 2-channel logits twice: f32 [N,h,w,2] (combine input) and compute-dtype
    channel-padded (fg_gate input), both written by the same final launch.
    """
    d = u.depth
    if x.H % (1 << (d - 1)) or x.W % (1 << (d - 1)):
        raise NotImplementedError(
            f"ROI size {x.H}x{x.W} is not divisible by 2^{d - 1}: the reference's bilinear resize of the up-conv "
            "output (unet.py:408) is then not the identity; not supported on the hiseg path")
    feats = []
    for i in range(d):
        enc = u.encoders[i]
        if i == 0:
            x = cna(E, enc[0], enc[1], act_code(enc[2]), x)
            x = residual_block(E, enc[3], x)
            x = residual_block(E, enc[4], x)
        else:
            x = residual_block(E, enc[0], x)
            x = residual_block(E, enc[1], x)
            x = cna(E, enc[2], enc[3], act_code(enc[4]), x)
        feats.append(x)
        if i < d - 1:
            x = ops.maxpool2x2(x)
    b = u.bottleneck
    a = residual_block(E, b[0], x)
    a = residual_block(E, b[1], a)
    a = cna(E, b[2], b[3], act_code(b[4]), a)
    att = ops.conv2d(E.conv(b[5], None, ACT_SIGMOID), a)
    x = ops.conv2d(E.conv(u.bottleneck_conv), x, mul=att)
    for i in range(d - 1):
        up = ops.conv2d(E.convT(u.upconvs[i]), x)
        skip = feats[d - 2 - i]
        dec = u.decoders[i]
        x = cna(E, dec[0], dec[1], act_code(dec[2]), up, skip, split=(up.C, skip.C))
        x = residual_block(E, dec[3], x)
        x = residual_block(E, dec[4], x)
    f = u.final
    h = cna(E, f[0], f[1], act_code(f[2]), x)
    low = Act.new(h.N, h.H, h.W, 2, torch.float32, E.device, cpad=2, zero=False)
    low_t = Act.new(h.N, h.H, h.W, 2, E.dtype, E.device)
    ops.conv2d(E.conv(f[3]), h, out=low, out2=low_t)
    return low, low_t


def hier_head(E: Ctx, head: nn.Module, feat: Act, aux: str) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """RefinedHierarchicalSegmentationHead.forward (refinement.py:734-804) over
    ExtendedHierarchicalSegmentationHeadUNetV2.forward (:550-606)."""
    bh = head.base_head
    sf = bh.shared_features
    s = cna(E, sf[0], sf[1], act_code(sf[2]), feat)
    s = residual_block(E, sf[4], s)
    s = residual_block(E, sf[6], s)
    low, low_t = enhanced_unet(E, bh.bg_vs_fg_unet, s)
    fg = bh.fg_gate
    g = cna(E, fg[0], None, act_code(fg[1]), low_t)
    g = cna(E, fg[3], None, act_code(fg[4]), g)
    gated = ops.conv2d(E.conv(fg[5], None, ACT_SIGMOID), g, mul=s)
    tb = bh.target_vs_nontarget_branch
    if bh.use_attention_module:
        t = residual_block(E, tb[0], gated)
        t = ops.attn_spatial(t, E.f32(tb[1].conv.weight))
        t = cna(E, tb[3], tb[4], act_code(tb[5]), t, convT=True)
        ca = tb[6]
        gate = ops.se_gate(t, E.f32(ca.fc1.weight, (ca.fc1.out_channels, ca.fc1.in_channels)), None,
                           E.f32(ca.fc2.weight, (ca.fc2.out_channels, ca.fc2.in_channels)), None,
                           act_code(ca.activation))
        t = ops.channel_scale(t, gate)
        t = residual_block(E, tb[8], t)
        last = tb[9]
    else:
        t = residual_block(E, tb[0], gated)
        t = cna(E, tb[2], tb[3], act_code(tb[4]), t, convT=True)
        t = residual_block(E, tb[6], t)
        last = tb[7]
    mh, mw = bh.mask_height, bh.mask_width
    if (t.H, t.W) != (mh, mw) or (2 * low.H, 2 * low.W) != (mh, mw):
        raise NotImplementedError(f"mask size {mh}x{mw} must be 2x the ROI size {low.H}x{low.W} on the hiseg path")
    up = bh.upsample_bg_fg
    per_sample = isinstance(up[1], LayerNorm2d)
    if per_sample:   # LayerNorm2d over the ConvTranspose output: per-ROI tables [N][32]
        ut_s = torch.empty(low.N * 32, dtype=torch.float32, device=E.device)
        ut_h = torch.empty_like(ut_s)
        L.check(L.lib().hiseg_ubf_ln_tables(low.t.data_ptr(), low.N, low.H, low.W, E.f32(up[0].weight).data_ptr(),
                                            E.f32(up[0].bias).data_ptr(), E.f32(up[1].weight, (32,)).data_ptr(),
                                            E.f32(up[1].bias, (32,)).data_ptr(), float(up[1].eps), 1, None, None,
                                            ut_s.data_ptr(), ut_h.data_ptr(), L.stream_ptr()), "ubf_ln_tables")
    else:
        ut_s, ut_h = E.affine(("ut", id(up[0])), up[0].out_channels, up[0].bias, up[1])
    want = aux == "full"
    logits, bgfg, tn = ops.hier_combine(
        low.t, low.N, low.H, low.W, t, E.f32(up[0].weight), ut_s, ut_h, act_code(up[2]),
        E.f32(up[3].weight, (2, up[3].in_channels)), E.f32(up[3].bias),
        E.f32(last.weight, (2, last.in_channels)), E.f32(last.bias), want, per_sample=per_sample)
    auxd: Dict[str, torch.Tensor] = {}
    if not want:
        return logits, auxd
    fg_att = ops.conv2d(E.conv(fg[5], None, ACT_SIGMOID), g)
    auxd.update({
        "bg_fg_logits": bgfg, "bg_fg_logits_low": low.to_nchw(), "target_nontarget_logits": tn,
        "fg_attention": fg_att.to_nchw(), "shared_features": s.to_nchw(),
    })
    lib = L.lib()
    if head.use_contour_detection:
        cb = head.contour_branch.contour_branch
        c = cna(E, cb[0], cb[1], act_code(cb[2]), s)
        c = cna(E, cb[3], cb[4], act_code(cb[5]), c)
        cm = Act.new(c.N, c.H, c.W, 1, torch.float32, E.device, cpad=1, zero=False)
        ops.conv2d(E.conv(cb[6], None, ACT_SIGMOID), c, out=cm)
        auxd["contours"] = _resize(cm.t.view(c.N, 1, c.H, c.W), mh, mw, lib)
    if head.use_distance_transform:
        dd = head.distance_decoder
        dh = dd.distance_head
        dx = cna(E, dh[0], dh[1], act_code(dh[2]), s)
        dx = residual_block(E, dh[3], dx)
        dm = Act.new(dx.N, dx.H, dx.W, 1, torch.float32, E.device, cpad=1, zero=False)
        ops.conv2d(E.conv(dh[4]), dx, out=dm)
        dmap = dm.t.view(dx.N, 1, dx.H, dx.W)
        dmask = torch.empty_like(dmap)
        L.check(lib.hiseg_distance_mask_fwd(dmap.data_ptr(), dmap.numel(), E.f32(dd.threshold).data_ptr(),
                                            dmask.data_ptr(), L.stream_ptr()), "distance_mask")
        auxd["distance_mask"] = _resize(dmask, mh, mw, lib)
        auxd["distance_map"] = _resize(dmap, mh, mw, lib)
    return logits, auxd


def _resize(x: torch.Tensor, H: int, W: int, lib) -> torch.Tensor:
    N, C, h, w = x.shape
    if (h, w) == (H, W):
        return x
    out = torch.empty(N, C, H, W, dtype=torch.float32, device=x.device)
    L.check(lib.hiseg_resize_bilinear_fwd(x.data_ptr(), N * C, h, w, out.data_ptr(), H, W, L.stream_ptr()),
            "resize_bilinear")
    return out


# ------------------------------------------------------------------------------------ full-image UNet
def _se(E: Ctx, se: nn.Module, h: Act) -> torch.Tensor:
    rd, c = se.conv_reduce.out_channels, se.conv_reduce.in_channels
    return ops.se_gate(h, E.f32(se.conv_reduce.weight, (rd, c)), E.f32(se.conv_reduce.bias),
                       E.f32(se.conv_expand.weight, (c, rd)), E.f32(se.conv_expand.bias), ACT_SILU)


def _dw(E: Ctx, conv: nn.Conv2d, bn, x: Act, act: int) -> Act:
    w, s, h, k, stride = E.dw(conv, bn)
    return ops.dwconv(x, w, s, h, k, stride, act)


def _dw_se(E: Ctx, conv: nn.Conv2d, bn, se: nn.Module, x: Act) -> Tuple[Act, torch.Tensor]:
    """conv_dw + BN + SiLU with the SE global pool fused into it, then the SE MLP -> gate [N, C]."""
    w, s, h, k, stride = E.dw(conv, bn)
    rd, c = se.conv_reduce.out_channels, se.conv_reduce.in_channels
    return ops.dwconv_se_gate(x, w, s, h, k, stride, ACT_SILU, E.f32(se.conv_reduce.weight, (rd, c)),
                              E.f32(se.conv_reduce.bias), E.f32(se.conv_expand.weight, (c, rd)),
                              E.f32(se.conv_expand.bias), ACT_SILU)


def mbconv(E: Ctx, blk: nn.Module, x: Act, out_cpad: Optional[int] = None) -> Act:
    """timm DepthwiseSeparableConv / InvertedResidual (eval): the SE pool is fused into the depthwise conv,
    the SE gate is applied inside the projection conv's loader (in_scale), the skip add in its epilogue.
    ``out_cpad``: channel stride of the block output (zero pad channels)."""
    if isinstance(blk, DepthwiseSeparableConv):
        h, g = _dw_se(E, blk.conv_dw, blk.bn1, blk.se, x)
        return ops.conv2d(E.conv(blk.conv_pw, blk.bn2), h, in_scale=g, residual=x if blk.has_skip else None,
                          out_cpad=out_cpad)
    if isinstance(blk, InvertedResidual):
        h = ops.conv2d(E.conv(blk.conv_pw, blk.bn1, ACT_SILU), x)
        h, g = _dw_se(E, blk.conv_dw, blk.bn2, blk.se, h)
        return ops.conv2d(E.conv(blk.conv_pwl, blk.bn3), h, in_scale=g, residual=x if blk.has_skip else None,
                          out_cpad=out_cpad)
    raise TypeError(type(blk))


def _block_out_channels(blk: nn.Module) -> int:
    return (blk.conv_pw if isinstance(blk, DepthwiseSeparableConv) else blk.conv_pwl).out_channels


def _drain(gen):
    """Run a forward generator (below) to its end and return its value."""
    while True:
        try:
            next(gen)
        except StopIteration as e:
            return e.value


def unet_logit(E: Ctx, pre: nn.Module, images: torch.Tensor) -> torch.Tensor:
    """PreTrainedPeopleSegmentationUNet.forward (unet.py:1901-1916): normalise, smp.Unet -> u [B,1,H,W] f32."""
    return _drain(unet_logit_iter(E, pre, images))


def unet_logit_iter(E: Ctx, pre: nn.Module, images: torch.Tensor):
    """unet_logit as a generator: yields after each encoder block / decoder block (the serving schedule's chunks,
    hiseg.model.StreamPipelinedExport(gate=True)), returns u."""
    B, _, H, W = images.shape
    if H % 32 or W % 32:
        raise NotImplementedError(f"image size {H}x{W} must be a multiple of 32 for the EfficientNet-UNet")
    x = ops.input_norm(images, E.f32(pre.norm_mean, (3,)), E.f32(pre.norm_std, (3,)), E.dtype)
    return (yield from effunet_forward_iter(E, pre.model, x))


def effunet_forward(E: Ctx, net: nn.Module, x: Act) -> torch.Tensor:
    """smp.Unet('timm-efficientnet-bX') forward (eval) on an NHWC input -> logits [B,1,H,W] f32."""
    return _drain(effunet_forward_iter(E, net, x))


def effunet_forward_iter(E: Ctx, net: nn.Module, x: Act):
    """effunet_forward as a generator: yields after the stem, each MBConv block and each decoder block."""
    B, H, W = x.N, x.H, x.W
    enc = net.encoder
    x = ops.conv2d(E.conv(enc.conv_stem, enc.bn1, ACT_SILU), x)
    feats = [x]
    yield
    for si, stage in enumerate(enc.blocks):
        for bi, blk in enumerate(stage):
            # the skip features of decoder blocks 0-2 (stage 2 / 3 / 5 outputs: 24 / 40 / 112 channels for B0-B1,
            # 48 / 80 / 224 for B7) are stored with a 64-multiple channel stride, zero pad channels, so those
            # blocks' conv1 (upsampled x ++ skip) takes the halo-tiled kernels instead of the generic one; the next
            # stage reads the padded map through its channel stride
            cpad = None
            if E.dtype == torch.bfloat16 and si + 1 in (2, 3, 5) and bi == len(stage) - 1:
                c = _block_out_channels(blk)
                cpad = round_up(c, 64) if c % 64 else None
            x = mbconv(E, blk, x, out_cpad=cpad)
            yield
        if si + 1 in (2, 3, 5, 7):
            feats.append(x)
    skips = feats[-2::-1]
    x = feats[-1]
    for i, blk in enumerate(net.decoder.blocks):
        skip = skips[i] if i < len(skips) else None
        split = (x.C, skip.C, skip.cstride) if skip is not None else None
        x = ops.conv2d(E.conv(blk.conv1[0], blk.conv1[1], ACT_RELU, split=split), x, skip, a_up=2)
        x = ops.conv2d(E.conv(blk.conv2[0], blk.conv2[1], ACT_RELU), x)
        yield
    u = Act.new(B, H, W, 1, torch.float32, E.device, cpad=1, zero=False)
    ops.conv2d(E.conv(net.segmentation_head[0]), x, out=u)
    return u.t.view(B, 1, H, W)


# ------------------------------------------------------------------------------------ entry points
def _root_dtype(m: nn.Module) -> torch.dtype:
    return getattr(m, "hiseg_dtype", torch.float32)


def unet_logits_nchw(pre: nn.Module, x: torch.Tensor) -> torch.Tensor:
    _check_input(x, "PreTrainedPeopleSegmentationUNet")
    E = Ctx(pre, _root_dtype(pre), x.device)
    return unet_logit(E, pre, x)


def _output_conv(E: Ctx, oc: nn.Conv2d, u: torch.Tensor) -> torch.Tensor:
    B, _, H, W = u.shape
    out = torch.empty(B, 2, H, W, dtype=torch.float32, device=u.device)
    L.check(L.lib().hiseg_output_conv_fwd(u.data_ptr(), B, H, W, E.f32(oc.weight, (2,)).data_ptr(),
                                          E.f32(oc.bias).data_ptr(), out.data_ptr(), L.stream_ptr()), "output_conv")
    return out


def unet_two_channel_nchw(wrapper: nn.Module, x: torch.Tensor) -> torch.Tensor:
    _check_input(x, "PreTrainedPeopleSegmentationUNetWrapper")
    E = Ctx(wrapper, _root_dtype(wrapper), x.device)
    return _output_conv(E, wrapper.output_conv, unet_logit(E, wrapper.model, x))


def roi_align_nchw(m: nn.Module, feat: torch.Tensor, rois: torch.Tensor, oh, ow) -> torch.Tensor:
    _check_input(feat, "DynamicRoIAlign")
    oh = int(oh.item()) if torch.is_tensor(oh) else int(oh[0] if isinstance(oh, (list, tuple)) else oh)
    ow = int(ow.item()) if torch.is_tensor(ow) else int(ow[0] if isinstance(ow, (list, tuple)) else ow)
    feat = feat.contiguous().float()
    out = torch.empty(rois.shape[0], feat.shape[1], oh, ow, dtype=torch.float32, device=feat.device)
    ops.roi_align(feat, rois.to(feat.device), oh, ow, m.spatial_scale_h, m.spatial_scale_w, m.aligned,
                  nchw_out=out)
    return out


def rgb_model_forward(model: nn.Module, images: torch.Tensor, rois: torch.Tensor, aux: str = "full",
                      unet_logit_override: Optional[torch.Tensor] = None):
    """HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet.forward (rgb.py:729-774).

    ``unet_logit_override`` (tests only) substitutes the smp.Unet output u [B,1,H,W], the way the
    golden vectors were produced from the reference.
    """
    _check_input(images, "HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet")
    if model.training:
        raise NotImplementedError("hiseg executes the inference (eval-mode) forward; call model.eval()")
    dev = images.device
    E = Ctx(model, _root_dtype(model), dev)
    images = images.contiguous().float()
    rois = rois.to(device=dev, dtype=torch.float32).contiguous()
    N = rois.shape[0]
    rh, rw = model.roi_size
    wrapper = model.pretrained_unet
    if unet_logit_override is not None:
        u = unet_logit_override.to(device=dev, dtype=torch.float32).contiguous()
    else:
        u = unet_logit(E, wrapper.model, images)
    oc = wrapper.output_conv
    ma, mr = model.roi_align_mask, model.roi_align_rgb
    roi_logits = Act.new(N, rh, rw, 2, E.dtype, dev, zero=False)
    ops.roi_align(u, rois, rh, rw, ma.spatial_scale_h, ma.spatial_scale_w, ma.aligned, out=roi_logits,
                  aff_w=E.f32(oc.weight, (2,)), aff_b=E.f32(oc.bias), zero_to=roi_logits.cstride)
    rgb = Act.new(N, rh, rw, 3, E.dtype, dev, zero=False)
    ops.roi_align(images, rois, rh, rw, mr.spatial_scale_h, mr.spatial_scale_w, mr.aligned, out=rgb,
                  zero_to=rgb.cstride)
    feats = rgb_feature_extractor(E, model.rgb_feature_extractor, rgb)
    comb = ops.conv2d(E.conv(model.feature_combiner, split=(feats.C, 2)), feats, roi_logits)
    logits, auxd = hier_head(E, model.segmentation_head, comb, aux)
    if aux == "full":
        auxd["full_image_logits"] = _output_conv(E, oc, u)
        rf = torch.empty(N, 2, rh, rw, dtype=torch.float32, device=dev)
        ops.roi_align(u, rois, rh, rw, ma.spatial_scale_h, ma.spatial_scale_w, ma.aligned, nchw_out=rf,
                      aff_w=E.f32(oc.weight, (2,)), aff_b=E.f32(oc.bias))
        auxd["roi_features"] = rf
        rp = torch.empty(N, 3, rh, rw, dtype=torch.float32, device=dev)
        ops.roi_align(images, rois, rh, rw, mr.spatial_scale_h, mr.spatial_scale_w, mr.aligned, nchw_out=rp)
        auxd["roi_patches"] = rp
    else:
        auxd["unet_logit"] = u
    return logits, auxd


def export_forward(model: nn.Module, images: torch.Tensor, rois: torch.Tensor, dilation: int = 0):
    """Exported contract: (instance_masks [N,1,mh,mw], binary_masks [B,1,H,W])."""
    logits, auxd = rgb_model_forward(model, images, rois, aux="none")
    E = Ctx(model, _root_dtype(model), images.device)
    oc = model.pretrained_unet.output_conv
    inst = ops.instance_masks(logits, dilation)
    binary = ops.binary_masks(auxd["unet_logit"], E.f32(oc.weight, (2,)), E.f32(oc.bias))
    return inst, binary


def export_unet_phase(model: nn.Module, images: torch.Tensor):
    """First half of the exported contract: full-image UNet logit u and binary_masks."""
    return _drain(export_unet_phase_iter(model, images))


def export_unet_phase_iter(model: nn.Module, images: torch.Tensor):
    """export_unet_phase as a generator (yields between UNet blocks), returns (u, binary_masks)."""
    _check_input(images, "RGBHierarchicalExportWrapper")
    E = Ctx(model, _root_dtype(model), images.device)
    u = yield from unet_logit_iter(E, model.pretrained_unet.model, images.contiguous().float())
    oc = model.pretrained_unet.output_conv
    return u, ops.binary_masks(u, E.f32(oc.weight, (2,)), E.f32(oc.bias))


def export_head_phase(model: nn.Module, images: torch.Tensor, rois: torch.Tensor, u: torch.Tensor, dilation: int = 0):
    """Second half: RoIAlign + ROI head from u -> instance_masks."""
    logits, _ = rgb_model_forward(model, images, rois, aux="none", unet_logit_override=u)
    return ops.instance_masks(logits, dilation)


# ------------------------------------------------------------------------------------ sub-module forwards (NCHW f32)
def _root_for(m: nn.Module):
    return m


def residual_block_nchw(blk: nn.Module, x: torch.Tensor) -> torch.Tensor:
    _check_input(x, "ResidualBlock")
    E = Ctx(blk, _root_dtype(blk), x.device)
    return residual_block(E, blk, Act.from_nchw(x, E.dtype)).to_nchw()


def enhanced_unet_nchw(u: nn.Module, x: torch.Tensor) -> torch.Tensor:
    _check_input(x, "EnhancedUNet")
    E = Ctx(u, _root_dtype(u), x.device)
    low, _ = enhanced_unet(E, u, Act.from_nchw(x, E.dtype))
    return low.to_nchw()


def head_nchw(head: nn.Module, x: torch.Tensor):
    _check_input(x, "RefinedHierarchicalSegmentationHead")
    E = Ctx(head, _root_dtype(head), x.device)
    return hier_head(E, head, Act.from_nchw(x, E.dtype), "full")

"""Train-mode execution of the smp-UNet student of the distillation path on libhiseg.

The reference trains ``smp.Unet('timm-efficientnet-b0')`` in train mode (train_distillation_staged.py
:256-366 with ``model.student.train()``): every BatchNorm of the student -- the frozen encoder's
included -- normalises with batch statistics and updates its running buffers, while only the decoder
(``unet.decoder``) and, after progressive unfreezing, the deepest encoder stages receive gradients.

Here the encoder runs as a forward-only chain of raw convolutions (the inference kernels with no BN
folded: stem conv, 1x1 expand/project convs, depthwise convs, SE gate fused into the projection
loader) each followed by the train-mode BatchNorm kernels of hiseg.train_engine (batch statistics,
running-stat update, SiLU / residual in the apply pass).  The decoder blocks (nearest-x2 upsample
fused into conv1's loader, skip concatenation as the conv's second source, conv-BN-ReLU x 2) and the
segmentation head record a tape exactly like the ROI path (hiseg.train_engine) and run the
hand-written backward: BN backward, transposed-read MFMA weight gradients, and the data gradient
through the upsample (dgrad conv at full resolution + 2x2 sum, hiseg_upsample2x_bwd).  Encoder stages
unfrozen by the progressive schedule (a suffix of ``encoder.blocks``) run on the tape too: 1x1 expand /
project convs through the train engine, depthwise convs and SqueezeExcite through their own backward
kernels (include/hiseg_train.h: hiseg_dw_*, hiseg_se_train_*), BN-SiLU backward from the pre-activation,
and the decoder routes gradients into the skip features those stages produce.  The whole
student is one autograd node; its parameter gradients land in the flat gradient buffer.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.nn as nn

from . import _lib as L
from . import engine as EG
from . import ops
from . import train_engine as TE
from .effunet import DepthwiseSeparableConv, InvertedResidual
from .ops import Act, hdtype, round_up

ACT_NONE, ACT_RELU, ACT_SILU = L.ACT_NONE, L.ACT_RELU, L.ACT_SILU


# ======================================================================================= frozen encoder
def _bn(T: TE.Tape, bn: nn.BatchNorm2d, z: Act, act: int, residual: Optional[Act] = None) -> Act:
    y, _ = TE.bn_forward(T, bn, z, act=act, residual=residual)
    return y


def _mbconv(E: EG.Ctx, T: TE.Tape, blk: nn.Module, x: Act) -> Act:
    """timm DepthwiseSeparableConv / InvertedResidual in train mode (forward only: frozen stage)."""
    res = x if blk.has_skip else None
    if isinstance(blk, DepthwiseSeparableConv):
        h = _bn(T, blk.bn1, EG._dw(E, blk.conv_dw, None, x, ACT_NONE), ACT_SILU)
        g = EG._se(E, blk.se, h)
        return _bn(T, blk.bn2, ops.conv2d(E.conv(blk.conv_pw), h, in_scale=g), ACT_NONE, res)
    if isinstance(blk, InvertedResidual):
        h = _bn(T, blk.bn1, ops.conv2d(E.conv(blk.conv_pw), x), ACT_SILU)
        h = _bn(T, blk.bn2, EG._dw(E, blk.conv_dw, None, h, ACT_NONE), ACT_SILU)
        g = EG._se(E, blk.se, h)
        return _bn(T, blk.bn3, ops.conv2d(E.conv(blk.conv_pwl), h, in_scale=g), ACT_NONE, res)
    raise TypeError(type(blk))


# ======================================================================================= unfrozen encoder stages
def dw_bn_silu(T: TE.Tape, conv: nn.Conv2d, bn: nn.BatchNorm2d, x: Act, need_dx: bool) -> Act:
    """conv_dw (groups = C, bias-free) -> BN(train) -> SiLU with the hand-written depthwise backward."""
    S, lib = T.S, L.lib()
    c, _, k, _ = conv.weight.shape
    st = conv.stride[0]
    assert x.C == c and x.cstride == c and x.coff == 0
    Ho, Wo = (x.H + 2 * (k // 2) - k) // st + 1, (x.W + 2 * (k // 2) - k) // st + 1
    dev = x.t.device
    z = Act.new(x.N, Ho, Wo, c, x.dtype, dev, zero=False)
    fast = x.dtype == torch.bfloat16 and _fast_dw()
    if fast:
        # the inference depthwise kernels (LDS-tiled / register-quad, hiseg_dwconv_fwd) with a unit affine and no
        # activation: the raw conv the train-mode BN normalises.  Their weight layout is [K*K][C]: the parameter is
        # transposed once per step (it changes every step).
        one, zero = _unit_affine(S, c, dev)
        wt = conv.weight.detach().reshape(c, k * k).t().contiguous()
        TE._chk(lib.hiseg_dwconv_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, c, k, st, wt.data_ptr(), one.data_ptr(),
                                     zero.data_ptr(), ACT_NONE, z.ptr(), Ho, Wo, TE._stream()), "dwconv(train)")
    else:
        TE._chk(lib.hiseg_dw_train_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, c, k, st, conv.weight.data_ptr(),
                                       z.ptr(), Ho, Wo, TE._stream()), "dw_train_fwd")
    y, bst = TE.bn_forward(T, bn, z, act=ACT_SILU)

    def back():
        dz = Act.new(z.N, z.H, z.W, c, z.dtype, dev, zero=False)
        TE.bn_backward(T, bn, z, y, bst, dz, act=ACT_SILU)
        if conv.weight.requires_grad:
            ws = torch.empty(int(lib.hiseg_dw_bwd_weight_ws(hdtype(x.dtype), x.N, Ho, Wo, c, k)), dtype=torch.float32,
                             device=dev)
            TE._chk(lib.hiseg_dw_bwd_weight(hdtype(x.dtype), x.ptr(), dz.ptr(), x.N, x.H, x.W, c, k, st, Ho, Wo,
                                            ws.data_ptr(), S.grad(conv.weight).data_ptr(), TE._stream()),
                    "dw_bwd_weight")
        if need_dx:
            gx, acc = T.grad(x)
            if fast and st == 1 and not acc:
                # stride 1: the data gradient is the same depthwise conv of dz with the kernel rotated by 180 degrees
                one, zero = _unit_affine(S, c, dev)
                wf = conv.weight.detach().reshape(c, k, k).flip(1, 2).reshape(c, k * k).t().contiguous()
                TE._chk(lib.hiseg_dwconv_fwd(hdtype(x.dtype), dz.ptr(), x.N, x.H, x.W, c, k, 1, wf.data_ptr(),
                                             one.data_ptr(), zero.data_ptr(), ACT_NONE, gx.ptr(), x.H, x.W,
                                             TE._stream()), "dwconv(train dgrad)")
            else:
                TE._chk(lib.hiseg_dw_bwd_data(hdtype(x.dtype), dz.ptr(), x.N, x.H, x.W, c, k, st,
                                              conv.weight.data_ptr(), Ho, Wo, gx.ptr(), int(acc), TE._stream()),
                        "dw_bwd_data")
            T.mark(x)
    T.push(back)
    return y


def _fast_dw() -> bool:
    """HISEG_TRAIN_DW_FAST=0: the training depthwise forward / stride-1 data gradient on the plain train kernels
    (hiseg_dw_train_fwd / hiseg_dw_bwd_data) instead of the inference kernels (A/B timing; read per call)."""
    import os
    return os.environ.get("HISEG_TRAIN_DW_FAST", "1") != "0"


def _unit_affine(S, c: int, dev) -> tuple:
    key = ("unit_affine", c, dev)
    v = S.cached.get(key)
    if v is None:
        v = S.cached[key] = (torch.ones(c, dtype=torch.float32, device=dev), torch.zeros(c, dtype=torch.float32,
                                                                                            device=dev))
    return v


def se_train(T: TE.Tape, se: nn.Module, h: Act) -> Act:
    """timm SqueezeExcite in training; returns the gated activation h * gate (the projection conv's input)."""
    S, lib = T.S, L.lib()
    assert h.coff == 0 and h.cstride == h.C
    N, C, HW = h.N, h.C, h.H * h.W
    rd = se.conv_reduce.out_channels
    dev = h.t.device
    gap = torch.empty(N * C, dtype=torch.float32, device=dev)
    hpre = torch.empty(N * rd, dtype=torch.float32, device=dev)
    gate = torch.empty(N * C, dtype=torch.float32, device=dev)
    ws = torch.empty(int(lib.hiseg_se_train_ws(N, C, rd)), dtype=torch.float32, device=dev)
    out = Act.new(h.N, h.H, h.W, C, h.dtype, dev, zero=False)
    w1, b1, w2, b2 = se.conv_reduce.weight, se.conv_reduce.bias, se.conv_expand.weight, se.conv_expand.bias
    TE._chk(lib.hiseg_se_train_fwd(hdtype(h.dtype), h.ptr(), N, HW, C, w1.data_ptr(), b1.data_ptr(), rd, w2.data_ptr(),
                                   b2.data_ptr(), ACT_SILU, ws.data_ptr(), gap.data_ptr(), hpre.data_ptr(),
                                   gate.data_ptr(), out.ptr(), TE._stream()), "se_train_fwd")

    def back():
        gout = T.grad_in(out)
        gh, acc = T.grad(h)
        target = gh if not acc else Act.new(h.N, h.H, h.W, C, h.dtype, dev, zero=False)
        ws2 = torch.empty_like(ws)
        TE._chk(lib.hiseg_se_train_bwd(hdtype(h.dtype), h.ptr(), N, HW, C, w1.data_ptr(), rd, w2.data_ptr(), ACT_SILU,
                                       gap.data_ptr(), hpre.data_ptr(), gate.data_ptr(), gout.ptr(), target.ptr(),
                                       ws2.data_ptr(), S.grad(w1).data_ptr(), S.grad(b1).data_ptr(),
                                       S.grad(w2).data_ptr(), S.grad(b2).data_ptr(), TE._stream()), "se_train_bwd")
        if acc:
            TE._chk(lib.hiseg_add_inplace(hdtype(h.dtype), h.N * HW, C, TE.ew(gh), TE.ew(target), TE._stream()), "add")
        T.mark(h)
    T.push(back)
    return out


def mbconv_train(T: TE.Tape, blk: nn.Module, x: Act, need_dx: bool) -> Act:
    """An unfrozen MBConv block with the tape backward (timm block order; SE gate materialised)."""
    res = x if blk.has_skip else None
    if isinstance(blk, DepthwiseSeparableConv):
        h = dw_bn_silu(T, blk.conv_dw, blk.bn1, x, need_dx)
        hs = se_train(T, blk.se, h)
        return TE.conv_bn_act(T, blk.conv_pw, blk.bn2, ACT_NONE, hs, residual=res)
    if isinstance(blk, InvertedResidual):
        h = TE.conv_bn_act(T, blk.conv_pw, blk.bn1, ACT_SILU, x, need_dx=need_dx)
        h = dw_bn_silu(T, blk.conv_dw, blk.bn2, h, True)
        hs = se_train(T, blk.se, h)
        return TE.conv_bn_act(T, blk.conv_pwl, blk.bn3, ACT_NONE, hs, residual=res)
    raise TypeError(type(blk))


FEATURE_STAGES = (-1, 1, 2, 4, 6)   # encoder stage producing feats[j] (-1: stem, never unfrozen)


def first_trainable_stage(enc: nn.Module) -> int:
    """Index of the shallowest encoder stage with trainable parameters (len(blocks) if none).  Progressive
    unfreezing (unet_decoder_distillation.py:233-274) unfreezes a suffix of enc.blocks; the stem never."""
    if any(p.requires_grad for p in list(enc.conv_stem.parameters()) + list(enc.bn1.parameters())):
        raise NotImplementedError("hiseg distillation: a trainable encoder stem is not on the training path")
    n = len(enc.blocks)
    u0 = n
    for i, stage in enumerate(enc.blocks):
        if any(p.requires_grad for p in stage.parameters()):
            u0 = min(u0, i)
    for i in range(u0, n):
        if not all(p.requires_grad for p in enc.blocks[i].parameters()):
            raise NotImplementedError("hiseg distillation: trainable encoder stages must be a suffix of enc.blocks")
    return u0


def encoder_features(E: EG.Ctx, T: TE.Tape, enc: nn.Module, x: Act) -> List[Act]:
    """smp encoder taps (stride 2, 4, 8, 16, 32) in train mode: frozen stages forward-only on the inference
    kernels, the unfrozen suffix (progressive unfreezing) on the tape."""
    u0 = first_trainable_stage(enc)
    x = _bn(T, enc.bn1, ops.conv2d(E.conv(enc.conv_stem), x), ACT_SILU)
    feats = [x]
    for si, stage in enumerate(enc.blocks):
        for bi, blk in enumerate(stage):
            if si < u0:
                x = _mbconv(E, T, blk, x)
            else:
                x = mbconv_train(T, blk, x, need_dx=not (si == u0 and bi == 0))
        if si + 1 in (2, 3, 5, 7):
            feats.append(x)
    return feats


# ======================================================================================= trainable decoder
def up_conv_bn_relu(T: TE.Tape, conv: nn.Conv2d, bn: nn.BatchNorm2d, x_low: Act, skip: Optional[Act],
                    need_dx: bool, skip_dx: bool = False) -> Act:
    """DecoderBlock.conv1: Conv2dReLU over cat(upsample2x(x_low), skip) with the upsample fused into the
    conv loader (a_up = 2); backward: BN bwd, wgrad, and (need_dx) dgrad + 2x2 sum into x_low's gradient."""
    S, lib = T.S, L.lib()
    split = (x_low.C, skip.C) if skip is not None else None
    p = S.conv(conv, split=split)
    H, W = 2 * x_low.H, 2 * x_low.W
    dev = x_low.t.device
    z = Act.new(x_low.N, H, W, p.cout, x_low.dtype, dev)
    d = TE._desc(S, p, x_low, skip, z)
    d.H, d.W, d.Ho, d.Wo, d.a_up = H, W, H, W, 2
    stats = [] if isinstance(bn, nn.BatchNorm2d) else None
    TE.conv_fwd(S, p, x_low, skip, d=d, stats=stats)
    y, st = TE.bn_forward(T, bn, z, act=ACT_RELU, stats=stats)   # d holds x_low and skip for the weight gradient

    def back():
        dz = Act.new(z.N, z.H, z.W, z.C, z.dtype, dev, cpad=z.cstride, zero=z.cstride != z.C)
        TE.bn_backward(T, bn, z, y, st, dz, act=ACT_RELU)
        if TE._needs_wgrad(p):
            TE.conv_wgrad(T, p, d, dz, bias_from_gemm=False)
        if not need_dx and not skip_dx:
            return
        nout = p.ca + (p.cb if skip_dx else 0)
        dg = L.Conv2dDesc()
        dg.dtype = dg.out_dtype = hdtype(dz.dtype)
        dg.N, dg.H, dg.W, dg.Ho, dg.Wo = dz.N, H, W, H, W
        dg.KH, dg.KW, dg.stride, dg.pad = p.kh, p.kw, 1, p.kh - 1 - p.pad
        dg.srcA, dg.a_cstride, dg.a_coff, dg.Ca, dg.a_up = dz, dz.cstride, dz.coff, p.cop, 1
        # rows 0..ca-1 of the packed dgrad weights are the upsampled source's input channels, ca.. the skip's
        dg.weight, dg.Cout, dg.Cout_pad, dg.K_pad = p.w_dgrad, nout, round_up(nout, 16), p.dg_k_pad
        ones = torch.ones(round_up(nout, 16), dtype=torch.float32, device=dev)
        zeros = torch.zeros_like(ones)
        dg.scale, dg.shift, dg.act = ones, zeros, ACT_NONE
        full = Act.new(z.N, H, W, nout, dz.dtype, dev, cpad=nout, zero=False)
        dg.out, dg.o_cstride, dg.o_coff = full, full.cstride, 0
        TE._chk(TE._dgrad_launch(dg), "conv2d(decoder dgrad)")
        if need_dx:
            gx, acc = T.grad(x_low)
            TE._chk(lib.hiseg_upsample2x_bwd(hdtype(dz.dtype), x_low.N, x_low.H, x_low.W, x_low.C,
                                             TE.ew(full.slice(0, x_low.C)), TE.ew(gx), int(acc), TE._stream()),
                    "upsample2x_bwd")
            T.mark(x_low)
        if skip_dx:
            gs, acc_s = T.grad(skip)
            if acc_s:
                TE._chk(lib.hiseg_add_inplace(hdtype(dz.dtype), skip.N * H * W, skip.C, TE.ew(gs),
                                              TE.ew(full.slice(p.ca, skip.C)), TE._stream()), "add")
            else:       # first contribution: copy
                part = TE.ew(full.slice(p.ca, skip.C))
                TE._chk(lib.hiseg_act_bwd_pre(hdtype(dz.dtype), skip.N * H * W, skip.C, part, part, ACT_NONE, 1.0,
                                              TE.ew(gs), 0, TE._stream()), "copy")
            T.mark(skip)
    T.push(back)
    return y


def decoder_head(T: TE.Tape, net: nn.Module, feats: List[Act], u0: int = 7) -> Act:
    """UnetDecoder (5 DecoderBlocks) + SegmentationHead conv; returns the f32 logit Act [B,H,W,1].  ``u0`` =
    first trainable encoder stage: feature taps from stages >= u0 receive gradients through the decoder."""
    skips = feats[-2::-1]
    sk_stage = FEATURE_STAGES[-2::-1]
    x = feats[-1]
    for i, blk in enumerate(net.decoder.blocks):
        skip = skips[i] if i < len(skips) else None
        skip_dx = skip is not None and sk_stage[i] >= u0
        x = up_conv_bn_relu(T, blk.conv1[0], blk.conv1[1], x, skip, need_dx=i > 0 or FEATURE_STAGES[-1] >= u0,
                            skip_dx=skip_dx)
        x = TE.conv_bn_act(T, blk.conv2[0], blk.conv2[1], ACT_RELU, x)
    u = Act.new(x.N, x.H, x.W, 1, torch.float32, x.t.device, cpad=1, zero=False)
    TE.conv_plain(T, net.segmentation_head[0], ACT_NONE, x, out=u)
    return u


# ======================================================================================= autograd boundary
class _StudentFunction(torch.autograd.Function):
    """The student forward (frozen encoder + decoder + head) as one autograd node; parameter gradients are
    written into the FlatParams buffer by the backward kernels (the node returns None for them)."""

    @staticmethod
    def forward(ctx, handle, x, *params):
        net, S, E = handle["net"], handle["state"], handle["enc_ctx"]
        T = TE.Tape(S)
        S.pack()
        xa = Act.from_nchw(x, S.dtype)
        feats = encoder_features(E, T, net.encoder, xa)
        u = decoder_head(T, net, feats, first_trainable_stage(net.encoder))
        S.flush_counters()
        ctx.tape, ctx.state, ctx.u = T, S, u
        return u.t.view(u.N, 1, u.H, u.W)

    @staticmethod
    def backward(ctx, g):
        T, S, u = ctx.tape, ctx.state, ctx.u
        S.flat.prepare_backward()
        gt = g.contiguous().float()
        T.grads[id(u)] = Act(gt.view(-1), u.N, u.H, u.W, 1, 1, 0)
        T.mark(u)
        T.run_backward()
        return (None, None) + tuple(None for _ in range(len(ctx.needs_input_grad) - 2))


def _trainable_key(module: nn.Module):
    return tuple(id(p) for p in module.parameters() if p.requires_grad)


def student_train_forward(owner: nn.Module, net: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Train-mode forward of an EfficientNetUnet ``net`` owned by ``owner`` (UNetDecoderOnly): logits
    [B,1,H,W] f32, differentiable w.r.t. the trainable parameters through the HIP backward."""
    if not x.is_cuda:
        raise RuntimeError("hiseg student training runs on the GPU (libhiseg); got a CPU tensor")
    B, C, H, W = x.shape
    if C != 3 or H % 32 or W % 32:
        raise ValueError(f"student input must be [B,3,H,W] with H, W multiples of 32, got {tuple(x.shape)}")
    dtype = EG._root_dtype(owner)
    key = _trainable_key(owner)
    S = owner.__dict__.get("_hiseg_train")
    if S is None or S.dtype != dtype or S.device != x.device or owner.__dict__.get("_hiseg_train_key") != key:
        S = TE.TrainState(owner, dtype, x.device)
        owner.__dict__["_hiseg_train"] = S
        owner.__dict__["_hiseg_train_key"] = key
    S.sync = owner.__dict__.get("_hiseg_grad_sync")
    E = EG.Ctx(net.encoder, dtype, x.device)
    handle = {"net": net, "state": S, "enc_ctx": E}
    params = [p for _, p in S.flat.named]
    return _StudentFunction.apply(handle, x.contiguous().float(), *params)

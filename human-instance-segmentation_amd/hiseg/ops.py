"""Tensor-level wrappers over the libhiseg C ABI.

Activations live in HBM as NHWC tensors whose channel dimension is padded to whole 16-byte
chunks (8 bf16 / 4 f32).  An :class:`Act` is a view (tensor, grid, real channels, channel
stride, channel offset) so that concatenations are produced in place: a producer writes its
channels at an offset of the consumer's buffer and no concat copy is ever made.

Every function launches on ``torch.cuda.current_stream()`` and requires CUDA (HIP) tensors:
there is no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib as L

_TORCH_TO_HISEG = {torch.float32: L.HISEG_F32, torch.bfloat16: L.HISEG_BF16}


def chunk_elems(dtype: torch.dtype) -> int:
    return 8 if dtype == torch.bfloat16 else 4


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def hdtype(dtype: torch.dtype) -> int:
    try:
        return _TORCH_TO_HISEG[dtype]
    except KeyError:
        raise TypeError(f"hiseg supports float32 and bfloat16 activations, got {dtype}") from None


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("hiseg kernels run on the GPU only (got a CPU tensor); there is no CPU fallback")


@dataclass
class Act:
    """NHWC activation view: element (n, y, x, c) at t[((n*H + y)*W + x)*cstride + coff + c]."""
    t: torch.Tensor
    N: int
    H: int
    W: int
    C: int
    cstride: int
    coff: int = 0

    @staticmethod
    def new(N, H, W, C, dtype, device, cpad=None, zero=None) -> "Act":
        ce = chunk_elems(dtype)
        cs = round_up(C, ce) if cpad is None else cpad
        if zero is None:
            zero = cs != C
        alloc = torch.zeros if zero else torch.empty
        t = alloc(N * H * W * cs, dtype=dtype, device=device)
        return Act(t, N, H, W, C, cs, 0)

    def slice(self, coff: int, C: int) -> "Act":
        return Act(self.t, self.N, self.H, self.W, C, self.cstride, self.coff + coff)

    @property
    def dtype(self):
        return self.t.dtype

    @property
    def cpad(self) -> int:
        return round_up(self.C, chunk_elems(self.t.dtype))

    def ptr(self) -> int:
        return self.t.data_ptr()

    def to_nchw(self) -> torch.Tensor:
        out = torch.empty(self.N, self.C, self.H, self.W, dtype=torch.float32, device=self.t.device)
        L.check(L.lib().hiseg_nhwc_to_nchw_fwd(hdtype(self.dtype), self.ptr(), self.N, self.H, self.W, self.C,
                                               self.cstride, self.coff, out.data_ptr(), L.stream_ptr()),
                "nhwc_to_nchw")
        return out

    @staticmethod
    def from_nchw(x: torch.Tensor, dtype: torch.dtype) -> "Act":
        _require_gpu(x)
        x = x.contiguous().float()
        N, C, H, W = x.shape
        a = Act.new(N, H, W, C, dtype, x.device, zero=False)
        L.check(L.lib().hiseg_nchw_to_nhwc_fwd(hdtype(dtype), x.data_ptr(), N, C, H, W, a.ptr(), a.cstride,
                                               L.stream_ptr()), "nchw_to_nhwc")
        return a


# ---------------------------------------------------------------------------------------- RoIAlign
def roi_align(feat: torch.Tensor, rois: torch.Tensor, oh: int, ow: int, scale_h: float, scale_w: float,
              aligned: bool, out: Optional[Act] = None, aff_w: Optional[torch.Tensor] = None,
              aff_b: Optional[torch.Tensor] = None, nchw_out: Optional[torch.Tensor] = None,
              zero_to: int = 0) -> None:
    """DynamicRoIAlign.forward (dynamic_roi_align.py:56-171) into an NHWC Act or an NCHW f32 tensor."""
    _require_gpu(feat, rois)
    assert feat.dtype == torch.float32 and feat.is_contiguous() and feat.dim() == 4
    rois = rois.contiguous().float()
    assert rois.dim() == 2 and rois.shape[1] == 5
    B, C, H, W = feat.shape
    d = L.RoiAlignDesc()
    d.feat, d.B, d.C, d.H, d.W = feat, B, C, H, W
    d.rois, d.N = rois, rois.shape[0]
    d.oh, d.ow = int(oh), int(ow)
    d.scale_h, d.scale_w = float(scale_h), float(scale_w)
    d.aligned = int(bool(aligned))
    if aff_w is not None:
        d.aff_w, d.aff_b, d.n_aff = aff_w, (aff_b), aff_w.numel()
    if nchw_out is not None:
        assert nchw_out.dtype == torch.float32 and nchw_out.is_contiguous()
        d.out, d.out_dtype, d.o_nchw = nchw_out, L.HISEG_F32, 1
        d.o_cstride = 1
    else:
        d.out, d.out_dtype, d.o_cstride, d.o_coff = out, hdtype(out.dtype), out.cstride, out.coff
        d.zero_to = zero_to
    L.check(L.lib().hiseg_roi_align_fwd(ctypes.byref(d), L.stream_ptr()), "roi_align")


# ---------------------------------------------------------------------------------------- conv
class LaunchProbe:
    """Optional per-launch HIP-event timing of selected conv launches (used by bench.py's roofline).

    ``select(desc) -> key or None`` picks launches; events are recorded on the launch stream.
    """

    def __init__(self, select):
        self.select = select
        self.events = []  # (key, start, end, flops)

    def around(self, key, flops, launch):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        st = launch()
        e.record()
        self.events.append((key, s, e, flops))
        return st

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for key, s, e, fl in self.events:
            d = out.setdefault(key, {"launches": 0, "ms": 0.0, "flops": fl})
            d["launches"] += 1
            d["ms"] += s.elapsed_time(e)
        for d in out.values():
            d["avg_ms"] = d["ms"] / d["launches"]
        return out


PROBE: Optional[LaunchProbe] = None
# Serving-schedule hook (hiseg.model.StreamPipelinedExport(gate=True)): ``GATE.before()`` / ``GATE.after()`` run on the
# host around every conv launch of at least ``GATE.min_flops``, on the launching stream.
GATE = None
# Developer hook (tools/layer_profile.py): when a list, every conv launch appends
# (descriptor copy, tensors kept alive, flops).
RECORD: Optional[list] = None


@dataclass
class ConvPlan:
    """A conv (or ConvTranspose 2x2/s2) layer packed for hiseg_conv2d_fwd."""
    weight: torch.Tensor  # [Cout_pad, K_pad]
    scale: torch.Tensor   # f32 [Cout_pad]
    shift: torch.Tensor   # f32 [Cout_pad]
    kh: int
    kw: int
    stride: int
    pad: int
    ca: int               # padded channels read from source A
    cb: int               # padded channels read from source B
    cout: int             # real output channels (per output pixel)
    gemm_cols: int        # = cout, or 4*cout for convT
    cout_pad: int
    k_pad: int
    act: int
    convT: bool = False
    weight_frag: Optional[torch.Tensor] = None  # MFMA-fragment order (3x3 halo kernel), bf16 only


def pack_conv(weight: torch.Tensor, bias: Optional[torch.Tensor], bn: Optional[torch.nn.BatchNorm2d], act: int,
              dtype: torch.dtype, device, stride: int = 1, pad: int = 0, split=None) -> ConvPlan:
    """Pack an nn.Conv2d weight [Cout, Cin, kh, kw] (+ eval BN + bias) for the implicit GEMM.

    ``split`` = (ca_real, cb_real) partitions the input channels into the two loader sources
    (each padded to whole chunks); default: all channels from source A.  A third entry pads source B's
    channels further (zero weights) to that count -- a skip feature stored with a 64-multiple channel
    stride so the decoder conv takes the halo-tiled kernels (engine.effunet_forward).
    """
    ce = chunk_elems(dtype)
    w = weight.detach().float()
    cout, cin, kh, kw = w.shape
    ca_r, cb_r = split[:2] if split is not None else (cin, 0)
    assert ca_r + cb_r == cin
    ca, cb = round_up(ca_r, ce), round_up(cb_r, ce)
    if split is not None and len(split) > 2:
        cb = max(cb, int(split[2]))
    wk = torch.zeros(cout, kh, kw, ca + cb, dtype=torch.float32, device=w.device)
    wt = w.permute(0, 2, 3, 1)
    wk[..., :ca_r] = wt[..., :ca_r]
    if cb_r:
        wk[..., ca:ca + cb_r] = wt[..., ca_r:]
    k = kh * kw * (ca + cb)
    k_pad = round_up(k, 64)
    cout_pad = round_up(cout, 16)
    wp = torch.zeros(cout_pad, k_pad, dtype=torch.float32, device=w.device)
    wp[:cout, :k] = wk.reshape(cout, k)
    scale, shift = fold_affine(cout, bias, bn, w.device)
    sc = torch.zeros(cout_pad, dtype=torch.float32, device=w.device)
    sh = torch.zeros(cout_pad, dtype=torch.float32, device=w.device)
    sc[:cout], sh[:cout] = scale, shift
    frag = None
    if dtype == torch.bfloat16 and kh == 3 and kw == 3 and stride == 1 and ca % 64 == 0 and cb % 64 == 0 and k == k_pad:
        frag = frag_pack(wp, kh * kw, ca + cb).to(device=device, dtype=dtype).contiguous()
    return ConvPlan(wp.to(device=device, dtype=dtype).contiguous(), sc.to(device), sh.to(device), kh, kw, stride, pad,
                    ca, cb, cout, cout, cout_pad, k_pad, act, weight_frag=frag)


def frag_pack(wp: torch.Tensor, taps: int, cin: int) -> torch.Tensor:
    """[Cout_pad][taps*cin] -> MFMA A-fragment order [Cout_pad/16][cb][tap][s][lane(64)][8].

    K blocks run channel-block-major, tap-minor (the halo kernel's loop order); inside a K block,
    k-step s covers channels 32s..32s+31 and lane l holds row l&15, channels 8(l>>4)..+7
    (v_mfma_f32_16x16x32_bf16 A-operand map, cdna_hip_programming.md §3).
    """
    cp = wp.shape[0]
    v = wp.reshape(cp // 16, 16, taps, cin // 64, 2, 4, 8)      # ct, row, tap, cb, s, lg, e
    v = v.permute(0, 3, 2, 4, 5, 1, 6)                           # ct, cb, tap, s, lg, row, e
    return v.reshape(-1)


def pack_convT2x2(weight: torch.Tensor, bias: Optional[torch.Tensor], bn, act: int, dtype, device) -> ConvPlan:
    """Pack nn.ConvTranspose2d(k=2, s=2) weight [Cin, Cout, 2, 2] as a 1x1 GEMM with 4*Cout columns."""
    ce = chunk_elems(dtype)
    w = weight.detach().float()
    cin, cout, kh, kw = w.shape
    assert kh == 2 and kw == 2 and cout % 4 == 0
    ca = round_up(cin, ce)
    cols = 4 * cout
    k_pad = round_up(ca, 64)
    cout_pad = round_up(cols, 16)
    wp = torch.zeros(cout_pad, k_pad, dtype=torch.float32, device=w.device)
    # column q*cout + co  <->  (dy, dx) = (q // 2, q % 2)
    wp[:cols, :cin] = w.permute(2, 3, 1, 0).reshape(cols, cin)
    scale, shift = fold_affine(cout, bias, bn, w.device)
    sc = torch.zeros(cout_pad, dtype=torch.float32, device=w.device)
    sh = torch.zeros(cout_pad, dtype=torch.float32, device=w.device)
    sc[:cols], sh[:cols] = scale.repeat(4), shift.repeat(4)
    return ConvPlan(wp.to(device=device, dtype=dtype).contiguous(), sc.to(device), sh.to(device), 1, 1, 1, 0,
                    ca, 0, cout, cols, cout_pad, k_pad, act, convT=True)


def fold_affine(cout: int, bias: Optional[torch.Tensor], bn, device):
    """scale/shift such that bn(conv(x) + bias) == conv(x)*scale + shift (eval-mode BN)."""
    scale = torch.ones(cout, dtype=torch.float32, device=device)
    shift = torch.zeros(cout, dtype=torch.float32, device=device)
    if bias is not None:
        shift = bias.detach().float().to(device).clone()
    if bn is not None:
        g = bn.weight.detach().float() if bn.weight is not None else torch.ones(cout, device=device)
        b = bn.bias.detach().float() if bn.bias is not None else torch.zeros(cout, device=device)
        inv = g / torch.sqrt(bn.running_var.detach().float() + bn.eps)
        shift = (shift - bn.running_mean.detach().float()) * inv + b
        scale = inv
    return scale, shift


def conv2d(p: ConvPlan, xa: Act, xb: Optional[Act] = None, out: Optional[Act] = None, *, a_up: int = 1,
           residual: Optional[Act] = None, mul: Optional[Act] = None, out2: Optional[Act] = None,
           in_scale: Optional[torch.Tensor] = None, out_dtype: Optional[torch.dtype] = None,
           variant: int = 0, out_cpad: Optional[int] = None, split_k_3x3: bool = False) -> Act:
    """hiseg_conv2d_fwd.  Returns the output Act (allocated when ``out`` is None; ``out_cpad``: its channel
    stride, the pad channels zero).

    ``variant`` != 0 forces a kernel variant (hiseg_conv2d_fwd_variant; -1 = generic kernel).  ``split_k_3x3``
    passes the split-K workspace to a 3x3 layer too (images of <= 256 pixels, K >= 1536: the library then splits
    its K loop; the train engine's small-batch choice, off on the inference path).
    """
    dt = xa.dtype
    H, W = xa.H * a_up, xa.W * a_up
    if xb is not None:
        assert xb.dtype == dt and (xb.H, xb.W, xb.N) == (H, W, xa.N)
    if p.convT:
        Ho, Wo = H, W
        oH, oW = 2 * H, 2 * W
    else:
        Ho = (H + 2 * p.pad - p.kh) // p.stride + 1
        Wo = (W + 2 * p.pad - p.kw) // p.stride + 1
        oH, oW = Ho, Wo
    if out is None:
        out = Act.new(xa.N, oH, oW, p.cout, out_dtype or dt, xa.t.device, cpad=out_cpad,
                      zero=None if out_cpad is None else out_cpad != p.cout)
    assert (out.N, out.H, out.W) == (xa.N, oH, oW), ((out.N, out.H, out.W), (xa.N, oH, oW))
    assert xa.C <= p.ca and (xb is None or xb.C <= p.cb)
    d = L.Conv2dDesc()
    d.dtype, d.out_dtype = hdtype(dt), hdtype(out.dtype)
    d.N, d.H, d.W, d.Ho, d.Wo = xa.N, H, W, Ho, Wo
    d.KH, d.KW, d.stride, d.pad = p.kh, p.kw, p.stride, p.pad
    d.srcA, d.a_cstride, d.a_coff, d.Ca, d.a_up = xa, xa.cstride, xa.coff, p.ca, a_up
    if xb is not None:
        d.srcB, d.b_cstride, d.b_coff, d.Cb = xb, xb.cstride, xb.coff, p.cb
    if in_scale is not None:
        d.in_scale = in_scale
    d.weight, d.Cout, d.Cout_pad, d.K_pad = p.weight, p.gemm_cols, p.cout_pad, p.k_pad
    d.scale, d.shift, d.act, d.act_beta = p.scale, p.shift, int(p.act), L.act_beta(p.act)
    if residual is not None:
        d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
    if mul is not None:
        d.mul, d.m_cstride, d.m_coff = mul, mul.cstride, mul.coff
    d.out, d.o_cstride, d.o_coff = out, out.cstride, out.coff
    if out2 is not None:
        assert out2.dtype == dt
        d.out2, d.o2_cstride, d.o2_coff = out2, out2.cstride, out2.coff
    d.convT = int(p.convT)
    if p.weight_frag is not None:
        d.weight_frag = p.weight_frag
    ws = None
    if dt == torch.bfloat16 and not p.convT and ((p.kh * p.kw == 1 and p.k_pad >= 384) or
                                                 (split_k_3x3 and p.kh * p.kw == 9)):
        # small-grid, long-K 1x1 layers (the EfficientNet's deep SE-gated projections) split their K loop over
        # workgroups into this stream-ordered workspace (hiseg_conv2d_workspace_bytes: 0 when the layer does not).
        # (The 3x3 small-image split is the train engine's alone: it pays only for a small batch, and the inference
        # path's kernel choice must not depend on the batch.)
        nbytes = L.lib().hiseg_conv2d_workspace_bytes(ctypes.byref(d))
        if nbytes > 0:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=xa.t.device)
            d.workspace, d.workspace_bytes = ws, nbytes
    if RECORD is not None:
        dc = d.copy()
        keep = [t for t in (xa, xb, out, residual, mul, out2, ws) if t is not None]
        flops = 2.0 * d.N * d.Ho * d.Wo * p.gemm_cols * p.kh * p.kw * (xa.C + (xb.C if xb is not None else 0))
        RECORD.append((dc, keep, p, flops))
    gate = GATE
    if gate is not None:
        flops = 2.0 * d.N * d.Ho * d.Wo * p.gemm_cols * p.kh * p.kw * (xa.C + (xb.C if xb is not None else 0))
        if flops >= gate.min_flops and not variant:
            gate.before()
            _launch_conv(d, p, xa, xb)
            gate.after()
            return out
        gate.light()
    _launch_conv(d, p, xa, xb, variant)
    return out


def _launch_conv(d, p, xa, xb, variant=0):
    if PROBE is not None:
        key = PROBE.select(d)
        if key is not None:
            flops = 2.0 * d.N * d.Ho * d.Wo * p.gemm_cols * p.kh * p.kw * (xa.C + (xb.C if xb is not None else 0))
            L.check(PROBE.around(key, flops, lambda: L.lib().hiseg_conv2d_fwd(ctypes.byref(d), L.stream_ptr())),
                    "conv2d")
            return
    if variant:
        L.check(L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), variant, L.stream_ptr()), "conv2d")
    else:
        L.check(L.lib().hiseg_conv2d_fwd(ctypes.byref(d), L.stream_ptr()), "conv2d")


# ---------------------------------------------------------------------------------------- misc
def maxpool2x2(x: Act) -> Act:
    assert x.coff == 0 and x.cstride == x.cpad
    out = Act.new(x.N, x.H // 2, x.W // 2, x.C, x.dtype, x.t.device, cpad=x.cstride, zero=False)
    L.check(L.lib().hiseg_maxpool2x2_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.cstride, out.ptr(),
                                         L.stream_ptr()), "maxpool2x2")
    return out


def attn_spatial(x: Act, w7: torch.Tensor) -> Act:
    """SpatialAttentionModule (attention_modules.py:92-113)."""
    assert x.coff == 0 and x.cstride == x.C
    P = x.N * x.H * x.W
    stats = torch.empty(P * 2, dtype=torch.float32, device=x.t.device)
    att = torch.empty(P, dtype=torch.float32, device=x.t.device)
    out = Act.new(x.N, x.H, x.W, x.C, x.dtype, x.t.device, zero=False)
    k = w7.shape[-1]
    L.check(L.lib().hiseg_attn_spatial_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.C, w7.data_ptr(), k,
                                           stats.data_ptr(), att.data_ptr(), out.ptr(), L.stream_ptr()),
            "attn_spatial")
    return out


def se_gate(x: Act, w1, b1, w2, b2, act: int) -> torch.Tensor:
    """GAP -> 1x1 -> act -> 1x1 -> sigmoid; returns gate [N, C] f32."""
    assert x.coff == 0 and x.cstride == x.C
    HW = x.H * x.W
    lib = L.lib()
    splits = lib.hiseg_gap_splits(HW)
    partial = torch.empty(x.N * splits * x.C, dtype=torch.float32, device=x.t.device)
    gate = torch.empty(x.N, x.C, dtype=torch.float32, device=x.t.device)
    cr = w1.shape[0]
    L.check(lib.hiseg_se_gate_fwd(hdtype(x.dtype), x.ptr(), x.N, HW, x.C, w1.data_ptr(), _ptr(b1), cr,
                                  w2.data_ptr(), _ptr(b2), int(act), L.act_beta(act), partial.data_ptr(), gate.data_ptr(),
                                  L.stream_ptr()), "se_gate")
    return gate


def channel_scale(x: Act, gate: torch.Tensor) -> Act:
    assert x.coff == 0 and x.cstride == x.C
    out = Act.new(x.N, x.H, x.W, x.C, x.dtype, x.t.device, zero=False)
    L.check(L.lib().hiseg_channel_scale_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H * x.W, x.C, gate.data_ptr(),
                                            out.ptr(), L.stream_ptr()), "channel_scale")
    return out


def dwconv(x: Act, w: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, k: int, stride: int, act: int) -> Act:
    assert x.coff == 0 and x.cstride == x.C
    pad = k // 2
    Ho = (x.H + 2 * pad - k) // stride + 1
    Wo = (x.W + 2 * pad - k) // stride + 1
    out = Act.new(x.N, Ho, Wo, x.C, x.dtype, x.t.device, zero=False)
    L.check(L.lib().hiseg_dwconv_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.C, k, stride, w.data_ptr(),
                                     scale.data_ptr(), shift.data_ptr(), act, out.ptr(), Ho, Wo, L.stream_ptr()),
            "dwconv")
    return out


def dwconv_se_gate(x: Act, w: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, k: int, stride: int, act: int,
                   w1, b1, w2, b2, se_act: int):
    """Depthwise conv + folded BN + act with the SqueezeExcite pool fused into it; returns (h, gate [N, C])."""
    assert x.coff == 0 and x.cstride == x.C
    pad = k // 2
    Ho = (x.H + 2 * pad - k) // stride + 1
    Wo = (x.W + 2 * pad - k) // stride + 1
    lib = L.lib()
    out = Act.new(x.N, Ho, Wo, x.C, x.dtype, x.t.device, zero=False)
    tiles = lib.hiseg_dw_gap_parts(hdtype(x.dtype), x.N, Ho, Wo, x.C, k, stride)
    partial = torch.empty(x.N * tiles * x.C, dtype=torch.float32, device=x.t.device)
    L.check(lib.hiseg_dwconv_gap_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.C, k, stride, w.data_ptr(),
                                     scale.data_ptr(), shift.data_ptr(), act, out.ptr(), Ho, Wo, partial.data_ptr(),
                                     L.stream_ptr()), "dwconv_gap")
    gate = torch.empty(x.N, x.C, dtype=torch.float32, device=x.t.device)
    L.check(lib.hiseg_se_gate_partials_fwd(partial.data_ptr(), tiles, x.N, Ho * Wo, x.C, w1.data_ptr(), _ptr(b1),
                                           w1.shape[0], w2.data_ptr(), _ptr(b2), se_act, gate.data_ptr(),
                                           L.stream_ptr()), "se_gate_partials")
    return out, gate


def input_norm(images: torch.Tensor, mean: torch.Tensor, std: torch.Tensor, dtype: torch.dtype) -> Act:
    """normalize_input (hierarchical_segmentation_unet.py:1885-1890) with a device-side max flag."""
    _require_gpu(images)
    x = images.contiguous().float()
    B, C, H, W = x.shape
    lib = L.lib()
    maxbuf = torch.empty(1, dtype=torch.float32, device=x.device)
    L.check(lib.hiseg_image_max_fwd(x.data_ptr(), x.numel(), maxbuf.data_ptr(), L.stream_ptr()), "image_max")
    out = Act.new(B, H, W, C, dtype, x.device, zero=False)
    L.check(lib.hiseg_input_norm_fwd(hdtype(dtype), x.data_ptr(), B, C, H, W, maxbuf.data_ptr(), mean.data_ptr(),
                                     std.data_ptr(), out.ptr(), out.cstride, L.stream_ptr()), "input_norm")
    return out


def hier_combine(low: torch.Tensor, N: int, h: int, w: int, tfeat: Act, ut_w, ut_scale, ut_shift, ut_act, u1_w, u1_b,
                 t_w, t_b, want_aux: bool, per_sample: bool = False):
    """Fused upsample_bg_fg + target 1x1 + hierarchical combine; ``per_sample``: ut_scale/ut_shift are the
    [N][32] LayerNorm2d tables of hiseg_ubf_ln_tables."""
    assert tfeat.coff == 0 and tfeat.cstride == tfeat.C and (tfeat.H, tfeat.W) == (2 * h, 2 * w)
    dev = low.device
    logits = torch.empty(N, 3, 2 * h, 2 * w, dtype=torch.float32, device=dev)
    bgfg = torch.empty(N, 2, 2 * h, 2 * w, dtype=torch.float32, device=dev) if want_aux else None
    tn = torch.empty(N, 2, 2 * h, 2 * w, dtype=torch.float32, device=dev) if want_aux else None
    L.check(L.lib().hiseg_hier_combine_fwd(hdtype(tfeat.dtype), low.data_ptr(), N, h, w, tfeat.ptr(), tfeat.C,
                                           ut_w.data_ptr(), ut_scale.data_ptr(), ut_shift.data_ptr(), int(ut_act),
                                           L.act_beta(ut_act), int(per_sample), u1_w.data_ptr(), u1_b.data_ptr(), t_w.data_ptr(), t_b.data_ptr(),
                                           logits.data_ptr(), _ptr(bgfg), _ptr(tn), L.stream_ptr()), "hier_combine")
    return logits, bgfg, tn


def layernorm2d(z: Act, weight: torch.Tensor, bias: torch.Tensor, eps: float, act: int,
                residual: Optional[Act] = None, out: Optional[Act] = None) -> Act:
    """LayerNorm2d (model.py:18-38) of a conv output z, then (+ residual) and the activation:
    per-sample statistics over (C, H, W) (hiseg_ln_fwd_stats) and one apply pass with the folded
    per-sample tables (hiseg_bn_apply, per_sample = 1).  weight / bias: f32 [C]."""
    lib = L.lib()
    dev = z.t.device
    N, HW, C = z.N, z.H * z.W, z.C
    ws = torch.empty(int(lib.hiseg_ln_ws(N, HW, C)), dtype=torch.float32, device=dev)
    mean = torch.empty(N, dtype=torch.float32, device=dev)
    invstd = torch.empty_like(mean)
    scale = torch.empty(N * C, dtype=torch.float32, device=dev)
    shift = torch.empty_like(scale)
    L.check(lib.hiseg_ln_fwd_stats(hdtype(z.dtype), z.ptr(), N, HW, C, z.cstride, z.coff, weight.data_ptr(),
                                   bias.data_ptr(), float(eps), ws.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                   scale.data_ptr(), shift.data_ptr(), L.stream_ptr()), "ln_fwd_stats")
    y = out if out is not None else Act.new(N, z.H, z.W, C, z.dtype, dev, cpad=z.cstride)
    d = L.BnApplyDesc()
    d.dtype, d.P, d.HW, d.C = hdtype(z.dtype), N * HW, HW, C
    d.z, d.z_cstride, d.z_coff = z, z.cstride, z.coff
    d.scale, d.shift, d.per_sample = scale, shift, 1
    if residual is not None:
        d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
    d.act, d.act_beta = int(act), L.act_beta(act)
    d.y, d.y_cstride, d.y_coff = y, y.cstride, y.coff
    L.check(lib.hiseg_bn_apply(ctypes.byref(d), L.stream_ptr()), "ln_apply")
    return y


def instance_masks(logits: torch.Tensor, dilation: int = 0) -> torch.Tensor:
    N, _, mh, mw = logits.shape
    out = torch.empty(N, 1, mh, mw, dtype=torch.float32, device=logits.device)
    L.check(L.lib().hiseg_instance_masks_fwd(logits.contiguous().data_ptr(), N, mh, mw, int(dilation), out.data_ptr(),
                                             L.stream_ptr()), "instance_masks")
    return out


def binary_masks(u: torch.Tensor, oc_w: torch.Tensor, oc_b: torch.Tensor) -> torch.Tensor:
    B, _, H, W = u.shape
    out = torch.empty(B, 1, H, W, dtype=torch.float32, device=u.device)
    L.check(L.lib().hiseg_binary_masks_fwd(L.HISEG_F32, u.data_ptr(), 1, B, H, W, oc_w.data_ptr(), oc_b.data_ptr(),
                                           out.data_ptr(), L.stream_ptr()), "binary_masks")
    return out

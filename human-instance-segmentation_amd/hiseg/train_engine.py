"""Training execution of the RGB hierarchical ROI path on libhiseg kernels.

The reference trains with PyTorch autograd over its nn.Modules (train_advanced.py:680-762).  Here the
whole ROI path of one forward is ONE autograd node: the forward records a tape of fused kernel launches
(conv + train-mode BatchNorm + activation + residual + Dropout2d, attention gates, RoIAlign, the
upsample/combine head) and the backward replays it in reverse with the hand-written backward kernels
of include/hiseg_train.h / hiseg_head_train.h.  Parameter gradients are written straight into one flat
f32 gradient buffer whose slices are the parameters' ``.grad`` tensors (FlatParams), so
``loss.backward(); clip_grad_norm_; optimizer.step()`` keep working, and the fused AdamW of
hiseg.optim and the bucketed gradient all-reduce of hiseg.distributed work on contiguous memory.

Layouts as in hiseg.engine: activations NHWC with 16-B channel padding (pad channels zero), compute
dtype float32 (parity) or bfloat16 (throughput; BatchNorm statistics, losses and parameter gradients
stay f32).  The frozen full-image UNet runs in inference mode (hierarchical_segmentation_unet.py:
1870-1875,1892-1899); only its trainable 1->2 output_conv receives a gradient, straight from the
RoIAlign backward.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import engine as EG
from . import ops
from .layers import LayerNorm2d
from .ops import Act, chunk_elems, hdtype, round_up

ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_SILU = L.ACT_NONE, L.ACT_RELU, L.ACT_SIGMOID, L.ACT_SILU
ACT_GELU, ACT_SWISH = L.ACT_GELU, L.ACT_SWISH
SMOOTH_ACTS = (ACT_SILU, ACT_GELU, ACT_SWISH)   # derivative needs the pre-activation
_P = ctypes.c_void_p
# developer knob: force a conv kernel variant for the data-gradient convs (0 = automatic, -1 = generic)
_DGRAD_VARIANT = int(os.environ.get("HISEG_DGRAD_VARIANT", "0"))


def _dgrad_launch(dg, device=None) -> int:
    lib = L.lib()
    if device is not None:
        _splitk_workspace(dg, dg.KH, dg.KW, device)
    if _DGRAD_VARIANT:
        return lib.hiseg_conv2d_fwd_variant(ctypes.byref(dg), _DGRAD_VARIANT, _stream())
    return lib.hiseg_conv2d_fwd(ctypes.byref(dg), _stream())


def _stream():
    return L.stream_ptr()


def _chk(st, what):
    L.check(st, what)


def _ptr(t):
    return None if t is None else t.data_ptr()


def ew(a: Optional[Act]) -> L.EwView:
    v = L.EwView()
    if a is not None:
        v.p, v.cstride, v.coff = a.t, a.cstride, a.coff
    return v


# ======================================================================================= flat parameters
class FlatParams:
    """All trainable parameters of a module as views into one flat f32 buffer (and their gradients into
    another), in ``named_parameters`` order, so that the optimiser and the gradient all-reduce stream over
    contiguous memory and gradient buckets complete in reverse order during the backward."""

    # parameters that require grad but never receive one on this path (the reference leaves their .grad None,
    # so AdamW skips them): DistanceTransformDecoder.threshold only feeds distance_mask (refinement.py:298-344)
    NO_GRAD_SUFFIXES = ("distance_decoder.threshold",)

    def __init__(self, module: nn.Module):
        self.named = [(n, p) for n, p in module.named_parameters()
                      if p.requires_grad and not n.endswith(self.NO_GRAD_SUFFIXES)]
        if not self.named:
            raise ValueError("no trainable parameters")
        dev = self.named[0][1].device
        self.numel = sum(p.numel() for _, p in self.named)
        self.data = torch.empty(self.numel, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.offsets: Dict[int, Tuple[int, int]] = {}
        off = 0
        with torch.no_grad():
            for _, p in self.named:
                k = p.numel()
                self.data[off:off + k].copy_(p.detach().reshape(-1).float())
                p.data = self.data[off:off + k].view(p.shape)
                self.offsets[id(p)] = (off, k)
                off += k
        self.attach_grads()

    def owns(self, p: nn.Parameter) -> bool:
        return id(p) in self.offsets and p.data_ptr() == self.data.data_ptr() + 4 * self.offsets[id(p)][0]

    def grad_view(self, p: nn.Parameter) -> torch.Tensor:
        off, k = self.offsets[id(p)]
        return self.grad[off:off + k].view(p.shape)

    def attach_grads(self):
        for _, p in self.named:
            p.grad = self.grad_view(p)

    def prepare_backward(self):
        """Gradient-accumulation semantics of autograd: parameters whose .grad is None (zero_grad
        set_to_none) start from zero; an existing .grad elsewhere is copied into the flat buffer."""
        if all(p.grad is None for _, p in self.named):   # (zero_grad(set_to_none)): one fill, not one per tensor
            self.grad.zero_()
            self.attach_grads()
            return
        for _, p in self.named:
            g = p.grad
            view = self.grad_view(p)
            if g is None:
                view.zero_()
            elif g.data_ptr() != view.data_ptr():
                view.copy_(g)
            p.grad = view


# ======================================================================================= layer plans
@dataclass
class TConv:
    """A conv / convT layer prepared for training: packed forward and data-gradient weights (refreshed
    by one hiseg_pack_weights launch per step), geometry and its parameters."""
    conv: nn.Module
    convT: bool
    kh: int
    kw: int
    stride: int
    pad: int
    ca: int
    ca_real: int
    cb: int
    cb_real: int
    cout: int          # real output channels
    gemm_cols: int     # cout, or 4*cout for convT
    cout_pad: int
    k_pad: int
    w_fwd: torch.Tensor
    w_dgrad: torch.Tensor
    cop: int           # padded output channels (dgrad K layout)
    dg_cols: int       # dgrad GEMM columns (= ca + cb)
    dg_cout_pad: int
    dg_k_pad: int
    ones: torch.Tensor
    shift: torch.Tensor  # bias or zeros (f32, padded to cout_pad)
    has_bias: bool
    w_fwd_frag: Optional[torch.Tensor] = None    # MFMA fragment order (3x3 bf16, 64-multiple K channels): conv_hwr
    w_dgrad_frag: Optional[torch.Tensor] = None


class TrainState:
    """Per-model training state: flat parameters, conv plans, one packing table."""

    def __init__(self, model: nn.Module, dtype: torch.dtype, device):
        self.dtype, self.device = dtype, device
        self.flat = FlatParams(model)
        self.convs: Dict[int, TConv] = {}
        self.entries: List[L.PackEntry] = []
        self.table: Optional[torch.Tensor] = None
        self.max_total = 0
        # Dropout2d seeds: a device-resident base advanced once per step (begin_step) + the draw's index within
        # the step, so a step captured into a HIP graph draws fresh masks on every replay
        self.seed_base = torch.full((1,), int(torch.initial_seed()) & 0xFFFFFFFF, dtype=torch.int64, device=device)
        self.seed_offset = 0
        self.cached: Dict = {}
        self.sync = None          # hiseg.distributed.GradBucketSync (data-parallel gradient exchange)
        self.op_index: Optional[int] = None
        self.nbt: List[torch.Tensor] = []   # BatchNorm num_batches_tracked counters to advance after this forward

    def flush_counters(self):
        """Advance every train-mode BatchNorm's num_batches_tracked of this forward by one -- one multi-tensor
        launch instead of one torch add per layer (~50 per step)."""
        if self.nbt:
            torch._foreach_add_(self.nbt, 1)
            self.nbt = []

    # -- plans
    def conv(self, conv: nn.Module, split=None, convT: bool = False) -> TConv:
        p = self.convs.get(id(conv))
        if p is not None:
            return p
        ce = chunk_elems(self.dtype)
        w = conv.weight
        dev = self.device
        if convT:
            cin, cout, kh, kw = w.shape
            assert (kh, kw) == (2, 2) and conv.stride == (2, 2)
            ca, cb, ca_r, cb_r = round_up(cin, ce), 0, cin, 0
            cols = 4 * cout
            k_pad = round_up(ca, 64)
            cop = round_up(cout, ce)
            dg_cols, dg_k = ca, round_up(4 * cop, 64)
            stride, pad = 2, 0
        else:
            cout, cin, kh, kw = w.shape
            assert conv.groups == 1 and conv.stride[0] == 1, "training path: stride-1 convs"
            ca_r, cb_r = split if split is not None else (cin, 0)
            ca, cb = round_up(ca_r, ce), round_up(cb_r, ce)
            cols = cout
            k_pad = round_up(kh * kw * (ca + cb), 64)
            cop = round_up(cout, ce)
            dg_cols, dg_k = ca + cb, round_up(kh * kw * cop, 64)
            stride, pad = 1, conv.padding[0]
        cout_pad = round_up(cols, 16)
        # data-gradient GEMM columns padded to 64 past 64 (e.g. 256+8 -> 320) so the LDS-DMA kernels take them
        dg_cout_pad = round_up(dg_cols, 64) if dg_cols > 64 else round_up(dg_cols, 16)
        wf = torch.empty(cout_pad, k_pad, dtype=self.dtype, device=dev)
        wd = torch.empty(dg_cout_pad, dg_k, dtype=self.dtype, device=dev)
        ones = torch.ones(cout_pad, dtype=torch.float32, device=dev)
        shift = torch.zeros(cout_pad, dtype=torch.float32, device=dev)
        has_bias = conv.bias is not None
        p = TConv(conv, convT, kh, kw, stride, pad, ca, ca_r, cb, cb_r, cout, cols, cout_pad, k_pad, wf, wd, cop,
                  dg_cols, dg_cout_pad, dg_k, ones, shift, has_bias)
        # second copies in MFMA fragment order for the register-streamed-weight 3x3 kernel (conv_hwr.hip): the
        # forward when its K channels (ca + cb, each a 64 multiple) allow it, the data gradient when cop does
        frag_ok = self.dtype == torch.bfloat16 and not convT and (kh, kw) == (3, 3)
        jobs = [(2 if convT else 0, wf, cout_pad, k_pad), (3 if convT else 1, wd, dg_cout_pad, dg_k)]
        if frag_ok and ca % 64 == 0 and cb % 64 == 0 and k_pad == 9 * (ca + cb):
            p.w_fwd_frag = torch.empty_like(wf)
            jobs.append((0 | L.HISEG_PACK_FRAG, p.w_fwd_frag, cout_pad, k_pad))
        if frag_ok and cop % 64 == 0 and dg_k == 9 * cop:
            p.w_dgrad_frag = torch.empty_like(wd)
            jobs.append((1 | L.HISEG_PACK_FRAG, p.w_dgrad_frag, dg_cout_pad, dg_k))
        src = w.detach()
        assert src.dtype == torch.float32 and src.is_contiguous()
        if has_bias:   # the bias into the epilogue shift (ConvTranspose: once per sub-pixel column block)
            jobs.append((L.HISEG_PACK_BIAS, shift, 1, 4 * cout if convT else cout))
        for mode, dst, rows, kp in jobs:
            e = L.PackEntry()
            bias = mode == L.HISEG_PACK_BIAS
            e.src = conv.bias.detach() if bias else src
            e.dst, e.dtype, e.mode = dst, (L.HISEG_F32 if bias else hdtype(self.dtype)), mode
            e.Cout, e.Cin_real, e.KH, e.KW = cout, (cin if convT else ca_r + cb_r), kh, kw
            e.ca, e.ca_real, e.cb, e.cb_real = ca, ca_r, cb, cb_r
            e.rows, e.K_pad, e.cop, e.total = rows, kp, cop, rows * kp
            self.entries.append(e)
            self.max_total = max(self.max_total, rows * kp)
        self.table = None
        self.convs[id(conv)] = p
        # pack the new layer now (later steps re-pack every layer in one launch at forward start)
        raw = b"".join(bytes(e) for e in self.entries[-len(jobs):])
        tab = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        _chk(L.lib().hiseg_pack_weights(tab.data_ptr(), len(jobs), max(r * kp for _, _, r, kp in jobs),
                                        _stream()), "pack_weights")
        self.cached.setdefault("keep_tables", []).append(tab)
        return p

    def pack(self):
        """One launch re-packs every conv's forward and dgrad weights and epilogue biases from the current
        parameters."""
        if not self.entries:
            return
        if self.table is None:
            raw = b"".join(bytes(e) for e in self.entries)
            self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        _chk(L.lib().hiseg_pack_weights(self.table.data_ptr(), len(self.entries), self.max_total, _stream()),
             "pack_weights")

    def grad(self, p: nn.Parameter) -> torch.Tensor:
        """Gradient slice of p; during a backward also tells the gradient exchange which tape op writes it."""
        if self.sync is not None:
            self.sync.record(p, self.op_index)
        return self.flat.grad_view(p)

    def begin_step(self):
        """Start of a training step (the ROI path's forward): advance the device seed base (a kernel)."""
        _chk(L.lib().hiseg_seed_advance(self.seed_base.data_ptr(), _stream()), "seed_advance")
        self.seed_offset = 0

    def next_seed(self) -> int:
        """Offset of the next Dropout2d draw within the step."""
        self.seed_offset += 1
        return self.seed_offset


# ======================================================================================= tape
class Tape:
    """Backward closures in forward order + the gradient buffers of the recorded activations."""

    def __init__(self, S: TrainState):
        self.S = S
        # a forward that raised before flush_counters left its BatchNorm counters queued: drop them, so the
        # next forward advances each num_batches_tracked once, as torch does
        S.nbt = []
        self.ops: List[Callable[[], None]] = []
        self.grads: Dict[int, Act] = {}
        self.written: Dict[int, bool] = {}
        self.keep: List = []
        self.ctx: Dict = {}   # per-forward values the backward needs (output gradients, resize keys)
        # BatchNorm layers whose backward reduction the one data-gradient conv that writes their output gradient
        # computes in its epilogue (id(y) -> {"z", "st", "act", "part", "S"}; residual_block, _fused_bn_bwd)
        self.bnb: Dict[int, dict] = {}

    def push(self, fn: Callable[[], None]):
        self.ops.append(fn)

    def grad(self, a: Act) -> Tuple[Act, bool]:
        """(gradient buffer of a, whether it already holds a contribution) -- for a backward that WRITES a's
        gradient: with the flag False it must overwrite every channel < a.C (pad channels are zero-filled
        here; the rest is not: the zero-fills were ~2 % of the train step)."""
        g = self.grads.get(id(a))
        if g is None:
            g = Act.new(a.N, a.H, a.W, a.C, a.dtype, a.t.device, cpad=a.cstride)
            self.grads[id(a)] = g
            self.keep.append(a)
        return g, self.written.get(id(a), False)

    def grad_in(self, a: Act) -> Act:
        """The gradient of a for a backward that READS it (a is that op's output): zeros if nothing wrote it."""
        g = self.grads.get(id(a))
        if g is not None and self.written.get(id(a), False):
            return g
        if g is None:
            g = Act.new(a.N, a.H, a.W, a.C, a.dtype, a.t.device, cpad=a.cstride, zero=True)
            self.grads[id(a)] = g
            self.keep.append(a)
        else:
            g.t.zero_()
        self.written[id(a)] = True
        return g

    def mark(self, a: Act):
        self.written[id(a)] = True

    def has(self, a: Act) -> bool:
        return self.written.get(id(a), False)

    def run_backward(self):
        S, ops = self.S, self.ops[::-1]
        sync = S.sync
        if sync is not None:
            sync.attach(S)
            sync.begin(len(ops))
        for i, fn in enumerate(ops):
            S.op_index = i
            fn()
            if sync is not None:
                sync.after_op(i)
        S.op_index = None
        if sync is not None:
            sync.end(len(ops))
        self.ops.clear()


# ======================================================================================= conv primitives
def _desc(S: TrainState, p: TConv, xa: Act, xb: Optional[Act], out: Act, *, act=ACT_NONE, shift=None,
          residual: Optional[Act] = None, mul: Optional[Act] = None, out2: Optional[Act] = None) -> L.Conv2dDesc:
    d = L.Conv2dDesc()
    d.dtype, d.out_dtype = hdtype(xa.dtype), hdtype(out.dtype)
    H, W = xa.H, xa.W
    d.N, d.H, d.W = xa.N, H, W
    d.Ho, d.Wo = (H, W) if p.convT else ((H + 2 * p.pad - p.kh) // p.stride + 1, (W + 2 * p.pad - p.kw) // p.stride + 1)
    d.KH, d.KW, d.stride, d.pad = (1, 1, 1, 0) if p.convT else (p.kh, p.kw, p.stride, p.pad)
    d.srcA, d.a_cstride, d.a_coff, d.Ca, d.a_up = xa, xa.cstride, xa.coff, p.ca, 1
    if xb is not None:
        d.srcB, d.b_cstride, d.b_coff, d.Cb = xb, xb.cstride, xb.coff, p.cb
    d.weight, d.Cout, d.Cout_pad, d.K_pad = p.w_fwd, p.gemm_cols, p.cout_pad, p.k_pad
    if p.w_fwd_frag is not None:
        d.weight_frag = p.w_fwd_frag
    d.scale, d.shift = p.ones, (shift if shift is not None else p.shift)
    d.act, d.act_beta = int(act), L.act_beta(act)
    if residual is not None:
        d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
    if mul is not None:
        d.mul, d.m_cstride, d.m_coff = mul, mul.cstride, mul.coff
    d.out, d.o_cstride, d.o_coff = out, out.cstride, out.coff
    if out2 is not None:
        d.out2, d.o2_cstride, d.o2_coff = out2, out2.cstride, out2.coff
    d.convT = int(p.convT)
    return d


def conv_fwd(S: TrainState, p: TConv, xa: Act, xb: Optional[Act] = None, *, act=ACT_NONE, out_dtype=None,
             out: Optional[Act] = None, out2: Optional[Act] = None, stats: Optional[list] = None,
             d: Optional[L.Conv2dDesc] = None) -> Tuple[Act, L.Conv2dDesc]:
    """Forward conv of the train path.  ``stats`` (a list): when the library fuses the BatchNorm batch statistics of
    the output into the conv's epilogue (hiseg_conv2d_stats_tiles > 0: the bf16 3x3 halo-kernel layers), the
    partials buffer and its split count are appended to it and bn_forward skips its statistics pass.  ``d``: a
    prepared descriptor (up_conv_bn_relu's upsampled form)."""
    if d is None:
        if p.convT:
            oH, oW = 2 * xa.H, 2 * xa.W
        else:
            oH = (xa.H + 2 * p.pad - p.kh) // p.stride + 1
            oW = (xa.W + 2 * p.pad - p.kw) // p.stride + 1
        if out is None:
            out = Act.new(xa.N, oH, oW, p.cout, out_dtype or xa.dtype, xa.t.device)
        d = _desc(S, p, xa, xb, out, act=act, out2=out2)
        _splitk_workspace(d, p.kh, p.kw, xa.t.device)
    else:
        out = d.out
    if stats is not None and _fuse_bn_stats():
        tiles = L.lib().hiseg_conv2d_stats_tiles(ctypes.byref(d))
        if tiles > 0:
            part = torch.empty(tiles * 3 * d.Cout, dtype=torch.float32, device=xa.t.device)
            d.stats_partial = part
            stats += [part, tiles]
    _chk(L.lib().hiseg_conv2d_fwd(ctypes.byref(d), _stream()), "conv2d(train)")
    d.stats_partial = None   # the descriptor is reused by the backward (weight gradient)
    return out, d


def _fuse_bn_stats() -> bool:
    """HISEG_FUSED_BN_STATS=0: the separate statistics pass everywhere (A/B timing, the equivalence test); read per
    call."""
    return os.environ.get("HISEG_FUSED_BN_STATS", "1") != "0"


def _splitk_workspace(d: L.Conv2dDesc, kh: int, kw: int, device) -> None:
    """The split-K workspace of a small-image, long-K 3x3 layer over a small batch (<= 8192 pixels in all: the B7
    EnhancedUNet's 768-channel pair over 8 x 16 x 12; the ROI heads' 16 x 12 levels over 256 ROIs fill the GPU on
    the halo kernel and would move 400 MB of partials) -- hiseg_conv2d_workspace_bytes; stream-ordered, held by
    the descriptor until the launch is enqueued.  Without a workspace the library does not split."""
    if (kh == 3 and kw == 3 and d.Ho * d.Wo <= 256 and d.N * d.Ho * d.Wo <= 8192 and d.K_pad >= 1536 and
            d.dtype == L.HISEG_BF16 and not d.convT):
        nbytes = L.lib().hiseg_conv2d_workspace_bytes(ctypes.byref(d))
        if nbytes > 0:
            d.workspace, d.workspace_bytes = torch.empty(nbytes, dtype=torch.uint8, device=device), nbytes


def _needs_wgrad(p: TConv) -> bool:
    return p.conv.weight.requires_grad


def conv_wgrad(T: Tape, p: TConv, d: L.Conv2dDesc, dz: Act, bias_from_gemm: bool = True):
    """Weight (and GEMM-column bias) gradient of the conv described by d: MFMA wgrad + split reduce
    accumulated into the flat gradient."""
    S, lib = T.S, L.lib()
    want_bias = int(p.has_bias and bias_from_gemm)
    wd = d.copy()
    ce = chunk_elems(S.dtype)
    if wd.Cout % ce:            # 1-/2-channel heads: the gradient buffer is padded with zeros
        wd.Cout = round_up(wd.Cout, ce)
    Cg, Kg, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _chk(lib.hiseg_conv2d_wgrad_dims(ctypes.byref(wd), want_bias, ctypes.byref(Cg), ctypes.byref(Kg),
                                     ctypes.byref(sp)), "wgrad_dims")
    ws = torch.empty(sp.value * Cg.value * Kg.value, dtype=torch.float32, device=dz.t.device)
    _chk(lib.hiseg_conv2d_wgrad(ctypes.byref(wd), dz.ptr(), dz.cstride, dz.coff, want_bias, ws.data_ptr(), sp.value,
                                _stream()), "wgrad")
    m = L.WgradMap()
    m.Cout, m.KH, m.KW = p.gemm_cols, (1 if p.convT else p.kh), (1 if p.convT else p.kw)
    m.ca, m.ca_real, m.cb, m.cb_real = p.ca, p.ca_real, p.cb, p.cb_real
    m.convT, m.Cg, m.Kg, m.want_bias = int(p.convT), Cg.value, Kg.value, want_bias
    gw = S.grad(p.conv.weight)
    gb = S.grad(p.conv.bias) if want_bias else None
    _chk(lib.hiseg_conv2d_wgrad_reduce(ws.data_ptr(), sp.value, ctypes.byref(m), gw.data_ptr(), _ptr(gb), 1,
                                       _stream()), "wgrad_reduce")


def conv_bwd(T: Tape, p: TConv, d: L.Conv2dDesc, xa: Act, xb: Optional[Act], dz: Act, *, need_dx: bool = True,
             bias_from_gemm: bool = True):
    """Weight/bias gradient (MFMA wgrad + split reduce into the flat gradient) and the data gradient
    (forward implicit-GEMM kernel with the packed dgrad weights), accumulated into the inputs' grads."""
    S, lib = T.S, L.lib()
    if _needs_wgrad(p):
        conv_wgrad(T, p, d, dz, bias_from_gemm)
    if not need_dx:
        return
    # data gradient: conv over dz with the dgrad weights
    dg = L.Conv2dDesc()
    dg.dtype = dg.out_dtype = hdtype(dz.dtype)
    if p.convT:
        dg.N, dg.H, dg.W, dg.Ho, dg.Wo = dz.N, dz.H, dz.W, xa.H, xa.W
        dg.KH, dg.KW, dg.stride, dg.pad = 2, 2, 2, 0
    else:
        dg.N, dg.H, dg.W, dg.Ho, dg.Wo = dz.N, dz.H, dz.W, xa.H, xa.W
        dg.KH, dg.KW, dg.stride, dg.pad = p.kh, p.kw, 1, p.kh - 1 - p.pad
    dg.srcA, dg.a_cstride, dg.a_coff, dg.Ca, dg.a_up = dz, dz.cstride, dz.coff, p.cop, 1
    dg.weight, dg.Cout, dg.Cout_pad, dg.K_pad = p.w_dgrad, p.dg_cols, p.dg_cout_pad, p.dg_k_pad
    if p.w_dgrad_frag is not None:
        dg.weight_frag = p.w_dgrad_frag
    zeros = S.cached.get(("zeros", p.dg_cout_pad))
    if zeros is None:
        zeros = torch.zeros(max(p.dg_cout_pad, 16), dtype=torch.float32, device=dz.t.device)
        ones = torch.ones(max(p.dg_cout_pad, 16), dtype=torch.float32, device=dz.t.device)
        S.cached[("zeros", p.dg_cout_pad)] = zeros
        S.cached[("ones", p.dg_cout_pad)] = ones
    dg.scale, dg.shift, dg.act = S.cached[("ones", p.dg_cout_pad)], zeros, ACT_NONE
    if xb is None:
        gx, acc = T.grad(xa)
        if acc:
            dg.residual, dg.r_cstride, dg.r_coff = gx, gx.cstride, gx.coff
        dg.out, dg.o_cstride, dg.o_coff = gx, gx.cstride, gx.coff
        fb = T.bnb.get(id(xa)) if not acc and not _DGRAD_VARIANT else None
        if fb is not None:   # the producing BatchNorm's backward reduction from this data gradient's epilogue
            z, st = fb["z"], fb["st"]
            dg.bnb_partial, dg.bnb_z, dg.bnb_z_cstride, dg.bnb_z_coff = gx, z, z.cstride, z.coff   # (query)
            dg.bnb_scale, dg.bnb_shift, dg.bnb_mean, dg.bnb_invstd = st.scale, st.shift, st.mean, st.invstd
            dg.bnb_act = int(fb["act"])
            S_ = int(lib.hiseg_conv2d_stats_tiles(ctypes.byref(dg)))
            if S_ > 0:
                part = torch.empty((S_ + (S_ + 63) // 64 + 1) * 3 * z.C, dtype=torch.float32, device=dz.t.device)
                dg.bnb_partial = part
                fb["part"], fb["S"] = part, S_
            else:
                for f in ("bnb_partial", "bnb_z", "bnb_scale", "bnb_shift", "bnb_mean", "bnb_invstd"):
                    setattr(dg, f, None)
        _chk(_dgrad_launch(dg, dz.t.device), "conv2d(dgrad)")
        T.mark(xa)
    else:
        tmp = Act.new(xa.N, xa.H, xa.W, p.ca + p.cb, dz.dtype, dz.t.device, cpad=p.ca + p.cb, zero=False)
        dg.out, dg.o_cstride, dg.o_coff = tmp, tmp.cstride, 0
        _chk(_dgrad_launch(dg, dz.t.device), "conv2d(dgrad)")
        for src_act, off, c in ((xa, 0, p.ca), (xb, p.ca, p.cb)):
            g, acc = T.grad(src_act)
            part = tmp.slice(off, c)
            P = src_act.N * src_act.H * src_act.W
            if acc:
                _chk(lib.hiseg_add_inplace(hdtype(dz.dtype), P, src_act.C, ew(g), ew(part), _stream()), "add")
            else:       # first contribution: copy
                _chk(lib.hiseg_act_bwd_pre(hdtype(dz.dtype), P, src_act.C, ew(part), ew(part), ACT_NONE, 1.0, ew(g), 0,
                                           _stream()), "copy")
            T.mark(src_act)


# ======================================================================================= BN(train) layers
class BNState:
    def __init__(self, C, device):
        self.mean = torch.empty(C, dtype=torch.float32, device=device)
        self.invstd = torch.empty_like(self.mean)
        self.scale = torch.empty_like(self.mean)
        self.shift = torch.empty_like(self.mean)


class LNState:
    """LayerNorm2d forward state: per-sample mean / invstd [N], folded tables scale / shift [N][C], workspace."""

    def __init__(self, N, HW, C, device):
        self.mean = torch.empty(N, dtype=torch.float32, device=device)
        self.invstd = torch.empty_like(self.mean)
        self.scale = torch.empty(N * C, dtype=torch.float32, device=device)
        self.shift = torch.empty_like(self.scale)
        self.ws = torch.empty(int(L.lib().hiseg_ln_ws(N, HW, C)), dtype=torch.float32, device=device)


def _bn_module(bn):
    assert isinstance(bn, (nn.BatchNorm2d, LayerNorm2d)), type(bn)
    return bn


def ln_forward(T: Tape, ln: LayerNorm2d, z: Act, *, act: int, residual: Optional[Act] = None,
               drop: Optional[torch.Tensor] = None, out: Optional[Act] = None) -> Tuple[Act, LNState]:
    """LayerNorm2d (model.py:18-38): per-sample statistics of z over (C, H, W), y = act(ln(z) + residual) * drop."""
    lib = L.lib()
    N, HW, C = z.N, z.H * z.W, z.C
    st = LNState(N, HW, C, z.t.device)
    _chk(lib.hiseg_ln_fwd_stats(hdtype(z.dtype), z.ptr(), N, HW, C, z.cstride, z.coff, ln.weight.data_ptr(),
                                ln.bias.data_ptr(), float(ln.eps), st.ws.data_ptr(), st.mean.data_ptr(),
                                st.invstd.data_ptr(), st.scale.data_ptr(), st.shift.data_ptr(), _stream()),
         "ln_fwd_stats")
    y = out if out is not None else Act.new(N, z.H, z.W, C, z.dtype, z.t.device, cpad=z.cstride)
    d = L.BnApplyDesc()
    d.dtype, d.P, d.HW, d.C = hdtype(z.dtype), N * HW, HW, C
    d.z, d.z_cstride, d.z_coff = z, z.cstride, z.coff
    d.scale, d.shift, d.per_sample = st.scale, st.shift, 1
    if residual is not None:
        d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
    d.act, d.act_beta = int(act), L.act_beta(act)
    d.chan_mul = (drop)
    d.y, d.y_cstride, d.y_coff = y, y.cstride, y.coff
    _chk(lib.hiseg_bn_apply(ctypes.byref(d), _stream()), "ln_apply")
    return y, st


def ln_backward(T: Tape, ln: LayerNorm2d, z: Act, y: Act, st: LNState, dz: Act, *, act: int,
                residual: Optional[Act] = None, drop=None, conv_bias: Optional[torch.Tensor] = None):
    lib, S = L.lib(), T.S
    gy = T.grad_in(y)
    d = L.LnBwdDesc()
    d.dtype, d.N, d.HW, d.C = hdtype(z.dtype), z.N, z.H * z.W, z.C
    d.dy, d.dy_cstride, d.dy_coff = gy, gy.cstride, gy.coff
    d.z, d.z_cstride, d.z_coff = z, z.cstride, z.coff
    d.chan_mul, d.act, d.act_beta = (drop), int(act), L.act_beta(act)
    d.mean, d.invstd, d.scale, d.shift = st.mean, st.invstd, st.scale, \
        st.shift
    d.gamma = ln.weight
    d.dgamma = (S.grad(ln.weight)) if ln.weight.requires_grad else None
    d.dbeta = (S.grad(ln.bias)) if ln.bias.requires_grad else None
    d.dconv_bias = (conv_bias)
    d.accumulate_params = 1
    d.dz, d.dz_cstride, d.dz_coff = dz, dz.cstride, dz.coff
    d.ws = st.ws
    if residual is not None:
        gr, acc = T.grad(residual)
        d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
        d.dres, d.dres_cstride, d.dres_coff, d.dres_accumulate = gr, gr.cstride, gr.coff, int(acc)
    _chk(lib.hiseg_ln_bwd(ctypes.byref(d), _stream()), "ln_bwd")
    if residual is not None:
        T.mark(residual)


def bn_forward(T: Tape, bn: nn.BatchNorm2d, z: Act, *, act: int, residual: Optional[Act] = None,
               drop: Optional[torch.Tensor] = None, out: Optional[Act] = None,
               stats: Optional[list] = None) -> Tuple[Act, BNState]:
    """Batch statistics of z (+ running update), y = act(bn(z) + residual) * drop.  ``stats`` = [partials, splits]
    the producing conv's epilogue wrote (conv_fwd), else a statistics pass over z."""
    if isinstance(bn, LayerNorm2d):
        return ln_forward(T, bn, z, act=act, residual=residual, drop=drop, out=out)
    lib = L.lib()
    C = z.C
    P = z.N * z.H * z.W
    st = BNState(C, z.t.device)
    if stats:
        part, splits = stats
    else:
        part, splits = torch.empty(lib.hiseg_bn_partials() * 3 * C, dtype=torch.float32, device=z.t.device), None
        _chk(lib.hiseg_bn_stats(hdtype(z.dtype), z.ptr(), P, C, z.cstride, z.coff, part.data_ptr(), _stream()),
             "bn_stats")
    track = bn.track_running_stats and bn.running_mean is not None
    mom = bn.momentum if bn.momentum is not None else 0.1
    if track and bn.num_batches_tracked is not None:
        T.S.nbt.append(bn.num_batches_tracked)
    fin_args = (C, P, _ptr(bn.weight), _ptr(bn.bias), float(bn.eps), float(mom),
                _ptr(bn.running_mean) if track else None, _ptr(bn.running_var) if track else None,
                st.mean.data_ptr(), st.invstd.data_ptr(), st.scale.data_ptr(), st.shift.data_ptr(), _stream())
    if splits is not None:
        _chk(lib.hiseg_bn_finalize_n(part.data_ptr(), splits, *fin_args), "bn_finalize_n")
    else:
        _chk(lib.hiseg_bn_finalize(part.data_ptr(), *fin_args), "bn_finalize")
    if track:   # the kernel updated the running statistics in place: invalidate eval plans folded from them
        torch.autograd.graph.increment_version([bn.running_mean, bn.running_var])
    y = out if out is not None else Act.new(z.N, z.H, z.W, C, z.dtype, z.t.device, cpad=z.cstride)
    d = L.BnApplyDesc()
    d.dtype, d.P, d.HW, d.C = hdtype(z.dtype), P, z.H * z.W, C
    d.z, d.z_cstride, d.z_coff = z, z.cstride, z.coff
    d.scale, d.shift = st.scale, st.shift
    if residual is not None:
        d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
    d.act, d.act_beta = int(act), L.act_beta(act)
    d.chan_mul = (drop)
    d.y, d.y_cstride, d.y_coff = y, y.cstride, y.coff
    _chk(lib.hiseg_bn_apply(ctypes.byref(d), _stream()), "bn_apply")
    return y, st


def bn_backward(T: Tape, bn: nn.BatchNorm2d, z: Act, y: Act, st: BNState, dz: Act, *, act: int,
                residual: Optional[Act] = None, drop=None, conv_bias: Optional[torch.Tensor] = None):
    if isinstance(bn, LayerNorm2d):
        return ln_backward(T, bn, z, y, st, dz, act=act, residual=residual, drop=drop, conv_bias=conv_bias)
    lib, S = L.lib(), T.S
    gy = T.grad_in(y)
    C = z.C
    P = z.N * z.H * z.W
    fb = T.bnb.pop(id(y), None)
    if fb is not None and fb["part"] is not None:   # the data gradient's epilogue did the reduction
        part, pre_splits = fb["part"], fb["S"]
        FUSED_BN_BWD_TAKEN[0] += 1
    else:
        part, pre_splits = torch.empty((lib.hiseg_bn_partials() + 1) * 3 * C, dtype=torch.float32,
                                       device=z.t.device), 0
    d = L.BnBwdDesc()
    d.partial_splits = pre_splits
    d.dtype, d.P, d.HW, d.C = hdtype(z.dtype), P, z.H * z.W, C
    d.dy, d.dy_cstride, d.dy_coff = gy, gy.cstride, gy.coff
    d.y, d.y_cstride, d.y_coff = y, y.cstride, y.coff
    d.z, d.z_cstride, d.z_coff = z, z.cstride, z.coff
    d.chan_mul, d.act, d.act_beta = (drop), int(act), L.act_beta(act)
    d.mean, d.invstd, d.gamma, d.beta = st.mean, st.invstd, (bn.weight), (bn.bias)
    d.partial = part
    d.dgamma = (S.grad(bn.weight)) if bn.weight is not None and bn.weight.requires_grad else None
    d.dbeta = (S.grad(bn.bias)) if bn.bias is not None and bn.bias.requires_grad else None
    d.dconv_bias = (conv_bias)
    d.accumulate_params = 1
    d.dz, d.dz_cstride, d.dz_coff = dz, dz.cstride, dz.coff
    if residual is not None:
        gr, acc = T.grad(residual)
        d.dres, d.dres_cstride, d.dres_coff, d.dres_accumulate = gr, gr.cstride, gr.coff, int(acc)
    elif act == ACT_RELU:   # ReLU mask recomputed from z with the forward's folded affine: y is not re-read
        d.fwd_scale, d.fwd_shift = st.scale, st.shift
    if int(act) in (ACT_GELU, ACT_SWISH) or (int(act) == ACT_SILU and residual is not None):
        # derivative at the forward's own pre-activation z*scale + shift (+ residual)
        d.fwd_scale, d.fwd_shift = st.scale, st.shift
        if residual is not None:
            d.residual, d.r_cstride, d.r_coff = residual, residual.cstride, residual.coff
    _chk(lib.hiseg_bn_bwd(ctypes.byref(d), _stream()), "bn_bwd")
    if residual is not None:
        T.mark(residual)


FUSED_BN_BWD_TAKEN = [0]   # BatchNorm backward passes that used a data gradient's epilogue reduction (tests)


def _fused_bn_bwd() -> bool:
    """HISEG_FUSED_BN_BWD=1 (read per forward; default off): the ResidualBlocks' first BatchNorm takes its backward
    reduction from conv2's data-gradient epilogue.  Measured (profiles/r5_fused_bn_bwd.txt): BatchNorm class 18.2 ->
    16.8 ms per B0 train step, data-gradient class 13.1 -> 14.4 ms, the step unchanged (71.5 vs 71.1-72.1 ms) -- the
    extra read of z lands in the epilogues every workgroup of the grid runs at the same time, as the residual's does."""
    return os.environ.get("HISEG_FUSED_BN_BWD", "0") == "1"


def conv_bn_act(T: Tape, conv: nn.Conv2d, bn, act: int, x: Act, xb: Optional[Act] = None, *,
                residual: Optional[Act] = None, drop=None, split=None, convT: bool = False,
                need_dx: bool = True, sole_consumer: bool = False) -> Act:
    """Conv (+bias) -> BatchNorm(train) -> (+residual) -> act -> (*Dropout2d mask).  ``sole_consumer``: the caller
    guarantees one conv alone consumes y (ResidualBlock's conv1 -> conv2), so that conv's data gradient -- the only
    write of y's gradient -- may compute this BatchNorm's backward reduction in its epilogue."""
    S = T.S
    bn = _bn_module(bn)
    p = S.conv(conv, split=split, convT=convT)
    stats = [] if isinstance(bn, nn.BatchNorm2d) else None
    z, d = conv_fwd(S, p, x, xb, stats=stats)
    y, st = bn_forward(T, bn, z, act=act, residual=residual, drop=drop, stats=stats)
    if (sole_consumer and isinstance(bn, nn.BatchNorm2d) and residual is None and drop is None and
            int(act) in (ACT_RELU, ACT_NONE) and z.dtype == torch.bfloat16 and _fused_bn_bwd()):
        T.bnb[id(y)] = {"z": z, "st": st, "act": int(act), "part": None, "S": 0}

    def back():
        dz = Act.new(z.N, z.H, z.W, z.C, z.dtype, z.t.device, cpad=z.cstride, zero=z.cstride != z.C)
        cb = S.grad(conv.bias) if conv.bias is not None and conv.bias.requires_grad else None
        bn_backward(T, bn, z, y, st, dz, act=act, residual=residual, drop=drop, conv_bias=cb)
        conv_bwd(T, p, d, x, xb, dz, bias_from_gemm=False, need_dx=need_dx)
    T.push(back)
    return y


def conv_plain(T: Tape, conv: nn.Conv2d, act: int, x: Act, xb: Optional[Act] = None, *, split=None,
               convT: bool = False, out_dtype=None, out: Optional[Act] = None, out2: Optional[Act] = None) -> Act:
    """Conv (+bias) (+act ReLU/Sigmoid fused in the epilogue), no normalisation.  SiLU / GELU / Swish: the
    conv writes the pre-activation, one element-wise pass the activation (its derivative needs the former)."""
    S = T.S
    p = S.conv(conv, split=split, convT=convT)
    if int(act) in SMOOTH_ACTS:
        assert out is None and out2 is None and out_dtype is None
        return _conv_smooth_act(T, p, act, x, xb)
    y, d = conv_fwd(S, p, x, xb, act=act, out_dtype=out_dtype, out=out, out2=out2)

    def back():
        lib = L.lib()
        gy = T.grad_in(y)
        P = y.N * y.H * y.W
        if y.dtype != S.dtype or act == ACT_SIGMOID or y.cstride % chunk_elems(S.dtype):
            # f32 / narrow heads: convert (and apply the activation derivative) into a padded compute-dtype buffer
            dz = Act.new(y.N, y.H, y.W, y.C, S.dtype, y.t.device, cpad=round_up(y.C, chunk_elems(S.dtype)), zero=True)
            _chk(lib.hiseg_act_bwd_cvt(hdtype(S.dtype), P, y.C, ew(gy), ew(y), act if act == ACT_SIGMOID else ACT_NONE,
                                       ew(dz), 0, _stream()), "act_bwd_cvt")
            if act == ACT_RELU:
                raise NotImplementedError("ReLU conv with a non-compute-dtype output")
        elif act == ACT_RELU:
            dz = Act.new(y.N, y.H, y.W, y.C, S.dtype, y.t.device, cpad=y.cstride, zero=y.cstride != y.C)
            _chk(lib.hiseg_relu_bwd(hdtype(S.dtype), P, y.H * y.W, y.C, ew(gy), ew(y), None, ew(dz), _stream()),
                 "relu_bwd")
        else:
            dz = gy
        conv_bwd(T, p, d, x, xb, dz)
    T.push(back)
    return y


def _conv_smooth_act(T: Tape, p: TConv, act: int, x: Act, xb: Optional[Act]) -> Act:
    S, lib = T.S, L.lib()
    z, d = conv_fwd(S, p, x, xb)
    y = Act.new(z.N, z.H, z.W, z.C, z.dtype, z.t.device, cpad=z.cstride)
    one = torch.ones(z.C, dtype=torch.float32, device=z.t.device)
    zero = torch.zeros(z.C, dtype=torch.float32, device=z.t.device)
    a = L.BnApplyDesc()
    a.dtype, a.P, a.HW, a.C = hdtype(z.dtype), z.N * z.H * z.W, z.H * z.W, z.C
    a.z, a.z_cstride, a.z_coff = z, z.cstride, z.coff
    a.scale, a.shift, a.act, a.act_beta = one, zero, int(act), L.act_beta(act)
    a.y, a.y_cstride, a.y_coff = y, y.cstride, y.coff
    _chk(lib.hiseg_bn_apply(ctypes.byref(a), _stream()), "act_apply")

    def back():
        gy = T.grad_in(y)
        dz = Act.new(z.N, z.H, z.W, z.C, z.dtype, z.t.device, cpad=z.cstride, zero=z.cstride != z.C)
        _chk(lib.hiseg_act_bwd_pre(hdtype(z.dtype), z.N * z.H * z.W, z.C, ew(gy), ew(z), int(act), L.act_beta(act),
                                   ew(dz), 0, _stream()), "act_bwd_pre")
        conv_bwd(T, p, d, x, xb, dz)
    T.push(back)
    return y


# ======================================================================================= blocks
def act_of(m) -> int:
    return EG.act_code(m)


def residual_block(T: Tape, blk: nn.Module, x: Act, drop=None) -> Act:
    """ResidualBlock (refinement.py:46-55 / unet.py:52-58) in train mode; `drop` = Dropout2d mask applied to
    the block output (the shared_features Sequential, refinement.py:484-486)."""
    a1 = act_of(blk.activation1 if hasattr(blk, "activation1") else blk.activation)
    a2 = act_of(blk.activation2 if hasattr(blk, "activation2") else blk.activation)
    h = conv_bn_act(T, blk.conv1, blk.norm1, a1, x, sole_consumer=True)
    return conv_bn_act(T, blk.conv2, blk.norm2, a2, h, residual=x, drop=drop)


def dropout_mask(T: Tape, m: nn.Module, N: int, C: int, device) -> Optional[torch.Tensor]:
    """Dropout2d mask [N, C] (0 or 1/(1-p)), or None when the module is a no-op.  A backward reaches the mask
    through a descriptor built in the forward (_dropout_after's BnApplyDesc) or a closure variable; both keep it
    alive (hiseg._lib.Desc holds every tensor assigned to a pointer field).  Round 3's flake was this mask held
    only as a raw address: freed after the forward, its block went to the next small tensor and the backward
    scaled by whatever that tensor held."""
    p = float(getattr(m, "p", 0.0))
    if p <= 0.0:
        return None
    out = torch.empty(N * C, dtype=torch.float32, device=device)
    _chk(L.lib().hiseg_dropout2d_mask_dev(N, C, p, T.S.seed_base.data_ptr(), T.S.next_seed(), out.data_ptr(),
                                          _stream()), "dropout2d_mask")
    return out


def rgb_feature_extractor(T: Tape, seq: nn.Sequential, x: Act) -> Act:
    h = conv_bn_act(T, seq[0], seq[1], act_of(seq[2]), x, need_dx=False)  # RoI RGB patches need no gradient
    h = residual_block(T, seq[3], h)
    h = conv_bn_act(T, seq[4], seq[5], act_of(seq[6]), h)
    h = residual_block(T, seq[7], h)
    h = conv_bn_act(T, seq[8], seq[9], act_of(seq[10]), h)
    h = residual_block(T, seq[11], h)
    return conv_bn_act(T, seq[12], seq[13], act_of(seq[14]), h)


def maxpool(T: Tape, x: Act) -> Act:
    y = ops.maxpool2x2(x)

    def back():
        gy = T.grad_in(y)
        gx, acc = T.grad(x)
        _chk(L.lib().hiseg_maxpool2x2_bwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.cstride, gy.ptr(), gx.ptr(),
                                          int(acc), _stream()), "maxpool_bwd")
        T.mark(x)
    T.push(back)
    return y


def gate(T: Tape, a: Act, g: Act) -> Act:
    """out = a * g (g = a sigmoid output); backward: da (+)= dy*g, dz_g = dy*a*g*(1-g) into g's grad."""
    lib = L.lib()
    out = Act.new(a.N, a.H, a.W, a.C, a.dtype, a.t.device, cpad=a.cstride)
    P = a.N * a.H * a.W
    _chk(lib.hiseg_gate_fwd(hdtype(a.dtype), P, a.C, ew(a), ew(g), ew(out), _stream()), "gate_fwd")

    def back():
        gy = T.grad_in(out)
        ga, acc = T.grad(a)
        gg, accg = T.grad(g)
        assert not accg, "sigmoid gate consumed twice"
        _chk(lib.hiseg_gate_bwd(hdtype(a.dtype), P, a.C, ew(gy), ew(a), ew(g), ew(ga), int(acc), ew(gg), _stream()),
             "gate_bwd")
        T.mark(a)
        T.mark(g)
        T.grads[id(g)] = gg
    T.push(back)
    return out


class _PreAct:
    """Marker: the gradient stored for a sigmoid-gate output already includes the sigmoid derivative."""


def conv_sigmoid_gate(T: Tape, conv: nn.Conv2d, x: Act) -> Act:
    """Conv (+bias) + Sigmoid whose only consumer is `gate` (which writes dL/dz, not dL/dy)."""
    S = T.S
    p = S.conv(conv)
    y, d = conv_fwd(S, p, x, act=ACT_SIGMOID)

    def back():
        dz = T.grad_in(y)  # gate_bwd wrote dy * a * g * (1-g) = dL/dz here
        conv_bwd(T, p, d, x, None, dz)
    T.push(back)
    return y


def enhanced_unet(T: Tape, u: nn.Module, x: Act) -> Tuple[Act, Act]:
    """EnhancedUNet.forward (hierarchical_segmentation_unet.py:375-417), train mode.  Returns the f32 logits
    [N,h,w,2] (combine input) and their compute-dtype copy (fg_gate input), written by one launch."""
    d = u.depth
    feats = []
    for i in range(d):
        enc = u.encoders[i]
        if i == 0:
            x = conv_bn_act(T, enc[0], enc[1], act_of(enc[2]), x)
            x = residual_block(T, enc[3], x)
            x = residual_block(T, enc[4], x)
        else:
            x = residual_block(T, enc[0], x)
            x = residual_block(T, enc[1], x)
            x = conv_bn_act(T, enc[2], enc[3], act_of(enc[4]), x)
        feats.append(x)
        if i < d - 1:
            x = maxpool(T, x)
    b = u.bottleneck
    a = residual_block(T, b[0], x)
    a = residual_block(T, b[1], a)
    a = conv_bn_act(T, b[2], b[3], act_of(b[4]), a)
    att = conv_sigmoid_gate(T, b[5], a)
    bc = conv_plain(T, u.bottleneck_conv, ACT_NONE, x)
    x = gate(T, bc, att)
    for i in range(d - 1):
        up = conv_plain(T, u.upconvs[i], ACT_NONE, x, convT=True)
        skip = feats[d - 2 - i]
        dec = u.decoders[i]
        x = conv_bn_act(T, dec[0], dec[1], act_of(dec[2]), up, skip, split=(up.C, skip.C))
        x = residual_block(T, dec[3], x)
        x = residual_block(T, dec[4], x)
    f = u.final
    h = conv_bn_act(T, f[0], f[1], act_of(f[2]), x)
    low = Act.new(h.N, h.H, h.W, 2, torch.float32, h.t.device, cpad=2, zero=False)
    low_t = Act.new(h.N, h.H, h.W, 2, T.S.dtype, h.t.device)
    S = T.S
    p = S.conv(f[3])
    _, dsc = conv_fwd(S, p, h, out=low, out2=low_t)

    def back():
        lib = L.lib()
        P = h.N * h.H * h.W
        dz = Act.new(h.N, h.H, h.W, 2, S.dtype, h.t.device, zero=True)
        g_low, acc1 = T.grad(low)
        g_lt, acc2 = T.grad(low_t)
        if acc2:
            _chk(lib.hiseg_add_inplace(hdtype(S.dtype), P, 2, ew(dz), ew(g_lt), _stream()), "add")
        if acc1:
            _chk(lib.hiseg_act_bwd_cvt(hdtype(S.dtype), P, 2, ew(g_low), L.EwView(), ACT_NONE, ew(dz), 1, _stream()),
                 "act_bwd_cvt")
        conv_bwd(T, p, dsc, h, None, dz)
    T.push(back)
    return low, low_t


# ======================================================================================= head
def spatial_attention(T: Tape, m: nn.Module, x: Act, drop) -> Act:
    lib, S = L.lib(), T.S
    assert x.coff == 0 and x.cstride == x.C
    P = x.N * x.H * x.W
    dev = x.t.device
    stats = torch.empty(P * 2, dtype=torch.float32, device=dev)
    amax = torch.empty(P, dtype=torch.int32, device=dev)
    att = torch.empty(P, dtype=torch.float32, device=dev)
    out = Act.new(x.N, x.H, x.W, x.C, x.dtype, dev, zero=False)
    w7 = m.conv.weight
    k = w7.shape[-1]
    _chk(lib.hiseg_attn_spatial_train_fwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.C, w7.data_ptr(), k, _ptr(drop),
                                          stats.data_ptr(), amax.data_ptr(), att.data_ptr(), out.ptr(), _stream()),
         "attn_spatial_train_fwd")

    def back():
        gy = T.grad_in(out)
        gx, acc = T.grad(x)
        ws = torch.empty(lib.hiseg_attn_spatial_ws(x.N, x.H, x.W, k), dtype=torch.float32, device=dev)
        target = gx if not acc else Act.new(x.N, x.H, x.W, x.C, x.dtype, dev, zero=False)
        _chk(lib.hiseg_attn_spatial_bwd(hdtype(x.dtype), x.ptr(), x.N, x.H, x.W, x.C, w7.data_ptr(), k, _ptr(drop),
                                        stats.data_ptr(), amax.data_ptr(), att.data_ptr(), gy.ptr(), target.ptr(),
                                        ws.data_ptr(), S.grad(w7).data_ptr(), _stream()), "attn_spatial_bwd")
        if acc:
            _chk(lib.hiseg_add_inplace(hdtype(x.dtype), P, x.C, ew(gx), ew(target), _stream()), "add")
        T.mark(x)
    T.push(back)
    return out


def channel_attention(T: Tape, m: nn.Module, x: Act, drop) -> Act:
    lib, S = L.lib(), T.S
    assert x.coff == 0 and x.cstride == x.C
    dev = x.t.device
    C, Cr, HW = x.C, m.fc1.out_channels, x.H * x.W
    w1, w2 = m.fc1.weight, m.fc2.weight
    act = act_of(m.activation)
    ws = torch.empty(lib.hiseg_attn_channel_ws(x.N, C, Cr), dtype=torch.float32, device=dev)
    gap = torch.empty(x.N * C, dtype=torch.float32, device=dev)
    hpre = torch.empty(x.N * Cr, dtype=torch.float32, device=dev)
    g = torch.empty(x.N * C, dtype=torch.float32, device=dev)
    out = Act.new(x.N, x.H, x.W, C, x.dtype, dev, zero=False)
    _chk(lib.hiseg_attn_channel_train_fwd(hdtype(x.dtype), x.ptr(), x.N, HW, C, w1.data_ptr(), Cr, w2.data_ptr(),
                                          int(act), L.act_beta(act), _ptr(drop), ws.data_ptr(), gap.data_ptr(), hpre.data_ptr(), g.data_ptr(),
                                          out.ptr(), _stream()), "attn_channel_train_fwd")

    def back():
        gy = T.grad_in(out)
        gx, acc = T.grad(x)
        target = gx if not acc else Act.new(x.N, x.H, x.W, C, x.dtype, dev, zero=False)
        _chk(lib.hiseg_attn_channel_bwd(hdtype(x.dtype), x.ptr(), x.N, HW, C, w1.data_ptr(), Cr, w2.data_ptr(),
                                        int(act), L.act_beta(act), _ptr(drop), gap.data_ptr(), hpre.data_ptr(), g.data_ptr(), gy.ptr(),
                                        target.ptr(), ws.data_ptr(), S.grad(w1).data_ptr(), S.grad(w2).data_ptr(),
                                        _stream()), "attn_channel_bwd")
        if acc:
            _chk(lib.hiseg_add_inplace(hdtype(x.dtype), x.N * HW, C, ew(gx), ew(target), _stream()), "add")
        T.mark(x)
    T.push(back)
    return out


def _dropout_after(T: Tape, m: nn.Module, y: Act) -> Act:
    """Stand-alone Dropout2d on a ReLU output (fg_gate, refinement.py:540): y * mask, as one pass."""
    drop = dropout_mask(T, m, y.N, y.C, y.t.device)
    if drop is None:
        return y
    lib, S = L.lib(), T.S
    out = Act.new(y.N, y.H, y.W, y.C, y.dtype, y.t.device, cpad=y.cstride)
    one = torch.ones(y.C, dtype=torch.float32, device=y.t.device)
    zero = torch.zeros(y.C, dtype=torch.float32, device=y.t.device)
    d = L.BnApplyDesc()
    d.dtype, d.P, d.HW, d.C = hdtype(y.dtype), y.N * y.H * y.W, y.H * y.W, y.C
    d.z, d.z_cstride, d.z_coff = y, y.cstride, y.coff
    d.scale, d.shift, d.act, d.chan_mul = one, zero, ACT_NONE, drop
    d.y, d.y_cstride, d.y_coff = out, out.cstride, out.coff
    _chk(lib.hiseg_bn_apply(ctypes.byref(d), _stream()), "dropout2d")

    def back():
        gy = T.grad_in(out)
        gx, acc = T.grad(y)
        assert not acc
        d2 = d.copy()
        d2.z, d2.z_cstride, d2.z_coff = gy, gy.cstride, gy.coff
        d2.y, d2.y_cstride, d2.y_coff = gx, gx.cstride, gx.coff
        _chk(lib.hiseg_bn_apply(ctypes.byref(d2), _stream()), "dropout2d_bwd")
        T.mark(y)
    T.push(back)
    return out


def hier_head_train(T: Tape, head: nn.Module, feat: Act):
    """RefinedHierarchicalSegmentationHead.forward (refinement.py:734-804) over
    ExtendedHierarchicalSegmentationHeadUNetV2.forward (:550-606), train mode."""
    S, lib = T.S, L.lib()
    dev = feat.t.device
    bh = head.base_head
    sf = bh.shared_features
    N = feat.N
    d1 = dropout_mask(T, sf[3], N, sf[0].out_channels, dev)
    s = conv_bn_act(T, sf[0], sf[1], act_of(sf[2]), feat, drop=d1)
    d2 = dropout_mask(T, sf[5], N, sf[0].out_channels, dev)
    s = residual_block(T, sf[4], s, drop=d2)
    s = residual_block(T, sf[6], s)
    low, low_t = enhanced_unet(T, bh.bg_vs_fg_unet, s)
    fg = bh.fg_gate
    g = conv_plain(T, fg[0], act_of(fg[1]), low_t)
    g = _dropout_after(T, fg[2], g)
    g = conv_plain(T, fg[3], act_of(fg[4]), g)
    att = conv_sigmoid_gate(T, fg[5], g)
    gated = gate(T, s, att)
    tb = bh.target_vs_nontarget_branch
    if not bh.use_attention_module:
        raise NotImplementedError("training path implements the attention-module target branch (all presets)")
    t = residual_block(T, tb[0], gated)
    t = spatial_attention(T, tb[1], t, dropout_mask(T, tb[2], N, t.C, dev))
    t = conv_bn_act(T, tb[3], tb[4], act_of(tb[5]), t, convT=True)
    t = channel_attention(T, tb[6], t, dropout_mask(T, tb[7], N, t.C, dev))
    t = residual_block(T, tb[8], t)
    last = tb[9]
    mh, mw = bh.mask_height, bh.mask_width
    if (t.H, t.W) != (mh, mw) or (2 * low.H, 2 * low.W) != (mh, mw):
        raise NotImplementedError(f"mask size {mh}x{mw} must be 2x the ROI size {low.H}x{low.W} on the hiseg path")
    up = bh.upsample_bg_fg
    ubn = _bn_module(up[1])
    uln = isinstance(ubn, LayerNorm2d)
    uact = act_of(up[2])
    h, w = low.H, low.W
    logits = torch.empty(N, 3, mh, mw, dtype=torch.float32, device=dev)
    bgfg = torch.empty(N, 2, mh, mw, dtype=torch.float32, device=dev)
    tn = torch.empty(N, 2, mh, mw, dtype=torch.float32, device=dev)
    bst = BNState(32, dev)
    if uln:   # per-sample statistics: mean / invstd [N], tables [N][32]
        bst.mean = torch.empty(N, dtype=torch.float32, device=dev)
        bst.invstd = torch.empty_like(bst.mean)
        bst.scale = torch.empty(N * 32, dtype=torch.float32, device=dev)
        bst.shift = torch.empty_like(bst.scale)
    ud = L.UbfDesc()
    ud.dtype = hdtype(S.dtype)
    ud.low, ud.N, ud.h, ud.w = low, N, h, w
    ud.ut_w, ud.ut_b = up[0].weight, up[0].bias
    ud.gamma, ud.beta = ubn.weight, ubn.bias
    ud.mean, ud.invstd, ud.scale, ud.shift = bst.mean, bst.invstd, bst.scale, \
        bst.shift
    ud.u1_w, ud.u1_b = up[3].weight, up[3].bias
    ud.tfeat, ud.Ct, ud.t_w, ud.t_b = t, t.C, last.weight, last.bias
    ud.logits, ud.bgfg, ud.tn = logits, bgfg, tn
    ud.act, ud.act_beta, ud.layernorm = int(uact), L.act_beta(uact), int(uln)
    ws = torch.empty(lib.hiseg_ubf_ws(N), dtype=torch.float32, device=dev)
    if uln:
        _chk(lib.hiseg_ubf_train_fwd(ctypes.byref(ud), float(ubn.eps), 0.0, None, None, ws.data_ptr(), _stream()),
             "ubf_train_fwd")
    else:
        if ubn.num_batches_tracked is not None:
            S.nbt.append(ubn.num_batches_tracked)
        _chk(lib.hiseg_ubf_train_fwd(ctypes.byref(ud), float(ubn.eps), float(ubn.momentum or 0.1),
                                     ubn.running_mean.data_ptr(), ubn.running_var.data_ptr(), ws.data_ptr(),
                                     _stream()), "ubf_train_fwd")
        torch.autograd.graph.increment_version([ubn.running_mean, ubn.running_var])
    aux = {"bg_fg_logits": bgfg, "target_nontarget_logits": tn}

    def back():
        dl = T.ctx["dlogits"]
        P = N * mh * mw
        db = torch.empty(P * 2, dtype=torch.float32, device=dev)
        dtn = torch.empty(P * 2, dtype=torch.float32, device=dev)
        glow, acc = T.grad(low)
        assert not acc
        gr = L.UbfGrads()
        gr.dut_w, gr.dut_b = S.grad(up[0].weight), S.grad(up[0].bias)
        gr.dgamma, gr.dbeta = S.grad(ubn.weight), S.grad(ubn.bias)
        gr.du1_w, gr.du1_b = S.grad(up[3].weight), S.grad(up[3].bias)
        _chk(lib.hiseg_ubf_train_bwd(ctypes.byref(ud), dl.data_ptr(), _ptr(T.ctx.get("dbgfg")),
                                     _ptr(T.ctx.get("dtn")), db.data_ptr(), dtn.data_ptr(), glow.ptr(),
                                     ws.data_ptr(), ctypes.byref(gr), _stream()), "ubf_train_bwd")
        T.mark(low)
        gt, acc2 = T.grad(t)
        assert not acc2
        pws = torch.empty(lib.hiseg_pw2_ws(t.C), dtype=torch.float32, device=dev)
        _chk(lib.hiseg_pw2_bwd(hdtype(S.dtype), t.ptr(), P, t.C, dtn.data_ptr(), last.weight.data_ptr(), gt.ptr(),
                               pws.data_ptr(), S.grad(last.weight).data_ptr(), S.grad(last.bias).data_ptr(), _stream()),
             "pw2_bwd")
        T.mark(t)
    T.push(back)

    # auxiliary heads on the shared features (refinement.py:760-800)
    if head.use_contour_detection:
        cb = head.contour_branch.contour_branch
        c = conv_bn_act(T, cb[0], cb[1], act_of(cb[2]), s)
        c = conv_bn_act(T, cb[3], cb[4], act_of(cb[5]), c)
        cm = Act.new(c.N, c.H, c.W, 1, torch.float32, dev, cpad=1, zero=False)
        conv_plain(T, cb[6], ACT_SIGMOID, c, out=cm)
        aux["contours"] = _resize_train(T, cm, mh, mw)
    if head.use_distance_transform:
        dd = head.distance_decoder
        dh = dd.distance_head
        x = conv_bn_act(T, dh[0], dh[1], act_of(dh[2]), s)
        x = residual_block(T, dh[3], x)
        dm = Act.new(x.N, x.H, x.W, 1, torch.float32, dev, cpad=1, zero=False)
        conv_plain(T, dh[4], ACT_NONE, x, out=dm)
        dmap = dm.t.view(x.N, 1, x.H, x.W)
        dmask = torch.empty_like(dmap)
        _chk(lib.hiseg_distance_mask_fwd(dmap.data_ptr(), dmap.numel(), dd.threshold.data_ptr(), dmask.data_ptr(),
                                         _stream()), "distance_mask")
        aux["distance_mask"] = EG._resize(dmask, mh, mw, lib)
        aux["distance_map"] = _resize_train(T, dm, mh, mw)
    aux.update({"bg_fg_logits_low": low.t.view(N, h, w, 2).permute(0, 3, 1, 2),
                "fg_attention": att.t.view(N, att.H, att.W, att.cstride)[..., :att.C].permute(0, 3, 1, 2),
                "shared_features": s.t.view(N, s.H, s.W, s.cstride)[..., :s.C].permute(0, 3, 1, 2)})
    return logits, aux


def _resize_train(T: Tape, a: Act, H: int, W: int) -> torch.Tensor:
    """F.interpolate(bilinear, align_corners=False) of a 1-channel f32 head output to the mask size; the
    output gradient arrives through T.S.cached[<tensor id>] (set by the autograd Function)."""
    lib = L.lib()
    src = a.t.view(a.N, 1, a.H, a.W)
    out = EG._resize(src, H, W, lib)
    key = ("dout", out.data_ptr())

    def back():
        g = T.ctx.get(key)
        if g is None:
            return
        gx, acc = T.grad(a)
        assert not acc
        if (a.H, a.W) == (H, W):
            gx.t.copy_(g.reshape(-1))
        else:
            _chk(lib.hiseg_resize_bilinear_bwd(g.data_ptr(), a.N, a.H, a.W, H, W, gx.ptr(), _stream()), "resize_bwd")
        T.mark(a)
    T.push(back)
    T.ctx.setdefault("resize_keys", []).append(key)
    return out


def roi_path_train(model: nn.Module, S: TrainState, T: Tape, images: torch.Tensor, rois: torch.Tensor,
                   u: torch.Tensor):
    """HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet.forward (rgb.py:729-774), train mode,
    from the (frozen) UNet logit map u."""
    lib = L.lib()
    dev = images.device
    N = rois.shape[0]
    rh, rw = model.roi_size
    oc = model.pretrained_unet.output_conv
    ma, mr = model.roi_align_mask, model.roi_align_rgb
    roi_logits = Act.new(N, rh, rw, 2, S.dtype, dev, zero=False)
    ops.roi_align(u, rois, rh, rw, ma.spatial_scale_h, ma.spatial_scale_w, ma.aligned, out=roi_logits,
                  aff_w=oc.weight.view(2), aff_b=oc.bias, zero_to=roi_logits.cstride)
    rgb = Act.new(N, rh, rw, 3, S.dtype, dev, zero=False)
    ops.roi_align(images, rois, rh, rw, mr.spatial_scale_h, mr.spatial_scale_w, mr.aligned, out=rgb,
                  zero_to=rgb.cstride)
    def back_roi():
        g, acc = T.grad(roi_logits)
        if not acc or not oc.weight.requires_grad:
            return
        d = L.RoiAlignDesc()
        d.feat, d.B, d.C, d.H, d.W = u, u.shape[0], 1, u.shape[2], u.shape[3]
        d.rois, d.N = rois, N
        d.oh, d.ow = rh, rw
        d.scale_h, d.scale_w = float(ma.spatial_scale_h), float(ma.spatial_scale_w)
        d.aligned = int(bool(ma.aligned))
        d.aff_w, d.aff_b, d.n_aff = oc.weight, oc.bias, 2
        ws = torch.empty(lib.hiseg_roi_align_ws(N), dtype=torch.float32, device=dev)
        _chk(lib.hiseg_roi_align_bwd_affine(ctypes.byref(d), g.ptr(), hdtype(g.dtype), g.cstride, g.coff,
                                            ws.data_ptr(), S.grad(oc.weight).data_ptr(), S.grad(oc.bias).data_ptr(),
                                            _stream()), "roi_align_bwd_affine")
    T.push(back_roi)
    feats = rgb_feature_extractor(T, model.rgb_feature_extractor, rgb)
    comb = conv_plain(T, model.feature_combiner, ACT_NONE, feats, roi_logits, split=(feats.C, 2))
    logits, aux = hier_head_train(T, model.segmentation_head, comb)
    aux["full_image_logits"] = EG._output_conv(EG.Ctx(model, S.dtype, dev), oc, u)
    aux["roi_features"] = roi_logits.t.view(N, rh, rw, roi_logits.cstride)[..., :2].permute(0, 3, 1, 2)
    aux["roi_patches"] = rgb.t.view(N, rh, rw, rgb.cstride)[..., :3].permute(0, 3, 1, 2)
    return logits, aux


# ======================================================================================= autograd boundary
DIFF_AUX = ("bg_fg_logits", "target_nontarget_logits", "contours", "distance_map")


class _RoiPathFunction(torch.autograd.Function):
    """The whole train-mode ROI path as one autograd node.  Inputs: a handle dict, images, rois and the
    trainable parameters (so autograd knows the outputs depend on them); the parameter gradients are
    written into the FlatParams buffer by the kernels (the node returns None for them)."""

    @staticmethod
    def forward(ctx, handle, images, rois, *params):
        model, S = handle["model"], handle["state"]
        T = Tape(S)
        S.begin_step()
        S.pack()
        u = handle["u"]
        logits, aux = roi_path_train(model, S, T, images, rois, u)
        S.flush_counters()
        ctx.tape, ctx.state = T, S
        diff = [aux.get(k) for k in DIFF_AUX]
        ctx.diff_present = [t is not None for t in diff]
        outs = [logits] + [t for t in diff if t is not None]
        ctx.out_keys = ["logits"] + [k for k, t in zip(DIFF_AUX, diff) if t is not None]
        nondiff = {k: v for k, v in aux.items() if k not in DIFF_AUX}
        handle["nondiff"] = nondiff
        handle["aux_order"] = list(aux.keys())
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        T, S = ctx.tape, ctx.state
        S.flat.prepare_backward()
        gmap = dict(zip(ctx.out_keys, grads))

        def f32(g, like_shape):
            if g is None:
                return None
            return g.contiguous().float()
        T.ctx["dlogits"] = f32(gmap["logits"], None)
        if T.ctx["dlogits"] is None:
            raise RuntimeError("hiseg train path: logits received no gradient")
        T.ctx["dbgfg"] = f32(gmap.get("bg_fg_logits"), None)
        T.ctx["dtn"] = f32(gmap.get("target_nontarget_logits"), None)
        keys = T.ctx.get("resize_keys", [])
        # resize keys are registered in forward order: contours first, then distance_map
        order = [k for k in ("contours", "distance_map") if k in gmap]
        for key, name in zip(keys, order):
            g = gmap.get(name)
            if g is not None:
                T.ctx[key] = f32(g, None)
        T.run_backward()
        hook = S.cached.get("after_backward")
        if hook is not None:
            hook()
        return (None, None, None) + tuple(None for _ in range(len(ctx.needs_input_grad) - 3))


def train_forward(model: nn.Module, images: torch.Tensor, rois: torch.Tensor, u_override=None):
    """Train-mode forward with the reference's return signature (logits, aux dict)."""
    EG._check_input(images, "HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet")
    dev = images.device
    dtype = EG._root_dtype(model)
    S = model.__dict__.get("_hiseg_train")
    if S is None or S.dtype != dtype or S.device != dev:
        S = TrainState(model, dtype, dev)
        model.__dict__["_hiseg_train"] = S
    S.sync = model.__dict__.get("_hiseg_grad_sync")
    images = images.contiguous().float()
    rois = rois.to(device=dev, dtype=torch.float32).contiguous()
    pre = model.pretrained_unet
    with torch.no_grad():
        if u_override is not None:
            u = u_override.to(device=dev, dtype=torch.float32).contiguous()
        else:
            E = EG.Ctx(pre.model, dtype, dev)
            u = EG.unet_logit(E, pre.model, images)
    handle = {"model": model, "state": S, "u": u}
    params = [p for _, p in S.flat.named]
    outs = _RoiPathFunction.apply(handle, images, rois, *params)
    logits = outs[0]
    aux = {}
    it = iter(outs[1:])
    nondiff = handle["nondiff"]
    for k in handle["aux_order"]:
        if k in DIFF_AUX:
            aux[k] = next(it)
        else:
            aux[k] = nondiff[k]
    return logits, aux

"""Training path on the GPU (libhiseg backward / train-mode kernels through the C ABI).

Each op is run through hiseg.train_engine (forward + tape backward) on seeded inputs and checked
against torch autograd of the same op in float64 on the GPU (the reference semantics; the oracle's
functional forms where the op is the reference's composite).  Tolerances: f32 compute 1e-4
relative to the tensor's max magnitude (2e-4 for reductions over > 1e5 terms); bf16 compute 3e-2.
The whole-model step is additionally compared with the CPU oracle (oracle/train.py) and the loss
kernel with the reference's golden vectors (tests/golden/train_loss.npz).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import filler
from helpers import b0_kwargs, hiseg_kwargs, load

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def rel2(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def err(dt):
    """f32: max-abs error relative to the tensor's max (1e-4 bar).  bf16: relative L2 error -- a ReLU whose
    pre-activation rounds across zero in bf16 flips single gradient elements by their full size, so the
    element-wise maximum is not a meaningful bf16 metric."""
    return rel if dt == torch.float32 else rel2


def tol(dt):
    return 1e-4 if dt == torch.float32 else 3e-2


class _Holder(nn.Module):
    def __init__(self, **mods):
        super().__init__()
        for k, v in mods.items():
            setattr(self, k, v)


def engine(module, dt):
    from hiseg import train_engine as TE
    module = module.to(DEV)
    S = TE.TrainState(module, dt, torch.device(DEV))
    return TE, S, TE.Tape(S)


def inject(T, y, g_nchw, dt):
    from hiseg.ops import Act
    ga = Act.from_nchw(g_nchw.to(DEV), dt)
    if ga.cstride != y.cstride:  # match the activation's padded layout
        full = Act.new(y.N, y.H, y.W, y.C, dt, DEV, cpad=y.cstride, zero=True)
        full.t.view(-1, y.cstride)[:, :y.C].copy_(ga.t.view(-1, ga.cstride)[:, :y.C])
        ga = full
    T.grads[id(y)] = ga
    T.mark(y)


def grad_nchw(T, a):
    g, _ = T.grad(a)
    return g.to_nchw()


# ------------------------------------------------------------------------------------------ conv wgrad / dgrad
CONV_CASES = [  # (cin, cout, k, H, W, N, bias, two-source split)
    (64, 64, 3, 12, 10, 3, True, None),
    (256, 256, 3, 16, 12, 2, False, None),
    (258, 256, 1, 8, 6, 2, True, (256, 2)),
    (3, 64, 3, 16, 12, 2, True, None),
    (128, 2, 1, 8, 6, 3, True, None),
    (128, 64, 3, 8, 6, 2, True, (64, 64)),
    # transposed-read wgrad forms: GEMM-bias column in a K tile of its own (Ktot = 1152), narrow Cout 32 / 8
    (128, 128, 3, 9, 7, 2, True, None),
    (64, 32, 3, 10, 9, 2, False, None),
    (128, 8, 1, 12, 10, 3, True, None),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_backward_matches_autograd(case, dt):
    from hiseg.ops import Act
    cin, cout, k, H, W, N, bias, split = case
    conv = nn.Conv2d(cin, cout, k, padding=k // 2, bias=bias)
    filler.fill_module(conv, seed=7)
    TE, S, T = engine(_Holder(c=conv), dt)
    x = torch.from_numpy(filler.normal(1, (N, cin, H, W))).to(DEV)
    if split is None:
        xa, xb = Act.from_nchw(x, dt), None
    else:
        xa, xb = Act.from_nchw(x[:, :split[0]], dt), Act.from_nchw(x[:, split[0]:], dt)
    y = TE.conv_plain(T, conv, TE.ACT_NONE, xa, xb, split=split)
    g = torch.from_numpy(filler.normal(2, (N, cout, H, W))).to(DEV)
    inject(T, y, g, dt)
    S.flat.prepare_backward()
    T.run_backward()
    xr = x.double().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    br = conv.bias.detach().double().requires_grad_(True) if bias else None
    yr = F.conv2d(xr, wr, br, padding=k // 2)
    (yr * g.double()).sum().backward()
    assert err(dt)(y.to_nchw(), yr.detach()) < tol(dt)
    assert err(dt)(conv.weight.grad, wr.grad) < tol(dt) * 2
    if bias:
        assert err(dt)(conv.bias.grad, br.grad) < tol(dt) * 2
    if split is None:
        assert err(dt)(grad_nchw(T, xa), xr.grad) < tol(dt)
    else:
        assert err(dt)(grad_nchw(T, xa), xr.grad[:, :split[0]]) < tol(dt)
        assert err(dt)(grad_nchw(T, xb), xr.grad[:, split[0]:]) < tol(dt)


WIDE_WGRAD_CASES = [  # (cin, cout, k, H, W, N, bias, two-source split): 128-multiple GEMM columns (wgrad_wide.hip)
    (256, 256, 3, 16, 12, 2, False, None),
    (256, 256, 3, 32, 24, 4, False, None),        # many pixel splits
    (256, 256, 3, 12, 10, 2, True, None),         # bias column in the last K tile of a shared-tap layer
    (128, 128, 3, 9, 7, 2, True, None),           # ragged K tile (1152 + bias column), C tile 128
    (256, 128, 3, 12, 10, 2, False, None),
    (128, 256, 3, 12, 10, 3, True, None),
    (258, 256, 1, 8, 6, 2, True, (256, 2)),       # two sources + bias in one K tile
    (256, 128, 3, 10, 8, 2, False, (128, 128)),   # decoder concat: two 128-channel sources
]


@pytest.mark.parametrize("reduce_taps", ["1", "0"])
@pytest.mark.parametrize("case", WIDE_WGRAD_CASES)
def test_wgrad_wide_matches_f64_of_bf16_operands(case, reduce_taps, monkeypatch):
    """bf16 weight gradients of the 128-multiple-column layers (the wide-tile kernel) against float64 autograd of
    the same bf16-rounded operands: the kernel's only error is its f32 accumulation, so 1e-4 of the max holds --
    with the split partials reduced by the tap-major kernel (3x3 single-source layers, coalesced reference-layout
    stores) and by the quad-of-K kernel (HISEG_WGRAD_REDUCE_TAPS=0)."""
    from hiseg.ops import Act
    monkeypatch.setenv("HISEG_WGRAD_REDUCE_TAPS", reduce_taps)
    monkeypatch.setenv("HISEG_WGRAD_HWC", "0")   # the transposed-read / wide tiles (the halo tile: below)
    cin, cout, k, H, W, N, bias, split = case
    dt = torch.bfloat16
    conv = nn.Conv2d(cin, cout, k, padding=k // 2, bias=bias)
    filler.fill_module(conv, seed=17)
    TE, S, T = engine(_Holder(c=conv), dt)
    x = torch.from_numpy(filler.normal(11, (N, cin, H, W))).to(DEV)
    if split is None:
        xa, xb = Act.from_nchw(x, dt), None
    else:
        xa, xb = Act.from_nchw(x[:, :split[0]], dt), Act.from_nchw(x[:, split[0]:], dt)
    y = TE.conv_plain(T, conv, TE.ACT_NONE, xa, xb, split=split)
    g = torch.from_numpy(filler.normal(12, (N, cout, H, W))).to(DEV)
    inject(T, y, g, dt)
    S.flat.prepare_backward()
    T.run_backward()
    xr = x.to(dt).double().requires_grad_(True)
    wr = conv.weight.detach().to(dt).double().requires_grad_(True)
    br = torch.zeros(cout, dtype=torch.float64, device=DEV, requires_grad=True) if bias else None
    yr = F.conv2d(xr, wr, br, padding=k // 2)
    (yr * g.to(dt).double()).sum().backward()
    assert rel(conv.weight.grad, wr.grad) < 1e-4
    if bias:
        assert rel(conv.bias.grad, br.grad) < 1e-4


HWC_WGRAD_CASES = [  # (cin, cout, H, W, N, bias[, split]): wgrad_hwc.hip's 64 x 64 x 9-tap tiles over 8 x 16 pixels
    (256, 256, 20, 30, 3, True),     # ragged pixel tiles both ways, bias column
    (64, 64, 16, 12, 2, False),
    (128, 256, 9, 7, 2, True),       # images smaller than one pixel tile
    (128, 128, 33, 40, 2, False),
    (192, 64, 64, 48, 4, True),      # the ROI head's grid, many splits
    (128, 64, 24, 20, 2, True, (64, 64)),     # decoder concat: up ++ skip, one resource per source
    (192, 128, 16, 18, 2, False, (128, 64)),
]


@pytest.mark.parametrize("case", HWC_WGRAD_CASES)
def test_wgrad_hwc_matches_f64_of_bf16_operands(case):
    """Round 5: the halo weight-gradient tile (3x3 single-source layers, Cin / Cout multiples of 64: 9 tap
    accumulators of 32 x 32 per wave over double-buffered dY / X-halo pixel tiles, 32x32x16 MFMAs fed by
    ds_read_b64_tr_b16) against float64 autograd of the same bf16-rounded operands (1e-4 of the max, its only error
    the f32 accumulation), the bias column included; and the halo path actually taken."""
    from hiseg import _lib as L
    from hiseg.ops import Act
    cin, cout, H, W, N, bias = case[:6]
    split = case[6] if len(case) > 6 else None
    dt = torch.bfloat16
    conv = nn.Conv2d(cin, cout, 3, padding=1, bias=bias)
    filler.fill_module(conv, seed=19)
    TE, S, T = engine(_Holder(c=conv), dt)
    x = torch.from_numpy(filler.normal(13, (N, cin, H, W))).to(DEV)
    if split is None:
        y = TE.conv_plain(T, conv, TE.ACT_NONE, Act.from_nchw(x, dt), None)
    else:
        y = TE.conv_plain(T, conv, TE.ACT_NONE, Act.from_nchw(x[:, :split[0]], dt), Act.from_nchw(x[:, split[0]:], dt),
                          split=split)
    g = torch.from_numpy(filler.normal(14, (N, cout, H, W))).to(DEV)
    inject(T, y, g, dt)
    S.flat.prepare_backward()
    L.wgrad_path_stats(reset=True)
    T.run_backward()
    torch.cuda.synchronize()
    assert L.wgrad_path_stats()["halo"] == 1
    xr = x.to(dt).double().requires_grad_(True)
    wr = conv.weight.detach().to(dt).double().requires_grad_(True)
    br = torch.zeros(cout, dtype=torch.float64, device=DEV, requires_grad=True) if bias else None
    yr = F.conv2d(xr, wr, br, padding=1)
    (yr * g.to(dt).double()).sum().backward()
    assert rel(conv.weight.grad, wr.grad) < 1e-4
    if bias:
        assert rel(conv.bias.grad, br.grad) < 1e-4


TR_WGRAD_CASES = [  # (cin, cout, k, H, W, N, bias, two-source split): conv_wgrad_tr_kernel's 128 / 64-column tiles
    (128, 128, 3, 12, 10, 3, True, None),
    (64, 64, 3, 16, 12, 2, False, None),
    (128, 64, 3, 9, 7, 2, True, None),           # ragged pixel block, bias column
    (128, 128, 3, 10, 8, 2, False, (64, 64)),    # decoder concat: two 64-channel sources
    (96, 128, 1, 8, 6, 2, True, None),
]


@pytest.mark.parametrize("knob,values,case",
                         [("HISEG_WGRAD_SHT", ("2", "1", "0"), c) for c in WIDE_WGRAD_CASES
                          if c[0] % 256 == 0 and c[7] is None] +
                         [("HISEG_WGRAD_TOG", ("1", "0"), c) for c in WIDE_WGRAD_CASES
                          if c[0] % 256 == 0 and c[7] is None] +
                         [("HISEG_WGRAD_TOG", ("1", "0"), c) for c in TR_WGRAD_CASES] +
                         [("HISEG_WGRAD_INC", ("1", "0"), c) for c in TR_WGRAD_CASES])
def test_wgrad_dma_addressing_bit_identical(knob, values, case, monkeypatch):
    """The weight-gradient kernels' cheaper DMA addressing lands the same operands as the per-stage (n, y, x)
    products: equal gradients.  Wide tile (wgrad_wide.hip, one source, 256-multiple Cin): the shared-tap addressing
    of its two X images with and without per-stage incremental byte offsets (HISEG_WGRAD_SHT=2 / 1) vs 0, and its
    image-major ring with per-stage flipped fragment-read registers (HISEG_WGRAD_TOG=1) vs the stage-major one;
    conv_wgrad_tr_kernel: incremental offsets (HISEG_WGRAD_INC=1) vs 0 and the flipped read registers (TOG), one and
    two sources."""
    from hiseg.ops import Act
    monkeypatch.setenv("HISEG_WGRAD_HWC", "0")   # these knobs belong to the transposed-read / wide tiles
    cin, cout, k, H, W, N, bias, split = case
    dt = torch.bfloat16
    x = torch.from_numpy(filler.normal(11, (N, cin, H, W))).to(DEV)
    g = torch.from_numpy(filler.normal(12, (N, cout, H, W))).to(DEV)
    grads = []
    for v in values:
        monkeypatch.setenv(knob, v)
        conv = nn.Conv2d(cin, cout, k, padding=k // 2, bias=bias)
        filler.fill_module(conv, seed=17)
        TE, S, T = engine(_Holder(c=conv), dt)
        if split is None:
            xa, xb = Act.from_nchw(x, dt), None
        else:
            xa, xb = Act.from_nchw(x[:, :split[0]], dt), Act.from_nchw(x[:, split[0]:], dt)
        y = TE.conv_plain(T, conv, TE.ACT_NONE, xa, xb, split=split)
        inject(T, y, g, dt)
        S.flat.prepare_backward()
        T.run_backward()
        grads.append((conv.weight.grad.clone(), conv.bias.grad.clone() if bias else None))
    for gw, gb in grads[1:]:
        assert torch.equal(grads[0][0], gw)
        if bias:
            assert torch.equal(grads[0][1], gb)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cio", [(256, 128), (128, 64), (64, 32)])
def test_convT_backward_matches_autograd(dt, cio):
    """ConvTranspose2d(k=2, s=2) backward; 128 -> 64 has two sub-pixels per 128-column wgrad tile."""
    from hiseg.ops import Act
    cin, cout = cio
    conv = nn.ConvTranspose2d(cin, cout, 2, stride=2)
    filler.fill_module(conv, seed=9)
    TE, S, T = engine(_Holder(c=conv), dt)
    x = torch.from_numpy(filler.normal(3, (2, cin, 8, 6))).to(DEV)
    xa = Act.from_nchw(x, dt)
    y = TE.conv_plain(T, conv, TE.ACT_NONE, xa, convT=True)
    g = torch.from_numpy(filler.normal(4, (2, cout, 16, 12))).to(DEV)
    inject(T, y, g, dt)
    S.flat.prepare_backward()
    T.run_backward()
    xr = x.double().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    br = conv.bias.detach().double().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, br, stride=2)
    (yr * g.double()).sum().backward()
    assert err(dt)(y.to_nchw(), yr.detach()) < tol(dt)
    assert err(dt)(conv.weight.grad, wr.grad) < tol(dt) * 2
    assert err(dt)(conv.bias.grad, br.grad) < tol(dt) * 2
    assert err(dt)(grad_nchw(T, xa), xr.grad) < tol(dt)


# ------------------------------------------------------------------------------------------ BN / residual / dropout
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_residual_block_train_matches_reference(dt):
    """ResidualBlock(64) train forward/backward against the reference's golden vectors (train_blocks.npz)."""
    from hiseg.layers import ResidualBlock
    from hiseg.ops import Act
    g = load("train_blocks")
    blk = filler.fill_module(ResidualBlock(64, "batchnorm", 8, "relu")).train()
    rm0 = blk.norm1.running_mean.clone()
    TE, S, T = engine(_Holder(b=blk), dt)
    x = torch.from_numpy(filler.normal(71, tuple(g["res_gx"].shape))).to(DEV)
    xa = Act.from_nchw(x, dt)
    y = TE.residual_block(T, blk, xa)
    gy = torch.from_numpy(filler.normal(81, tuple(g["res_y"].shape)))
    inject(T, y, gy, dt)
    S.flat.prepare_backward()
    T.run_backward()
    t = tol(dt)
    assert err(dt)(y.to_nchw(), g["res_y"]) < t
    assert err(dt)(grad_nchw(T, xa), g["res_gx"]) < t * 2
    names = list(g["res_names"])
    for j, n in enumerate(names):
        p = dict(blk.named_parameters())[n]
        sq = float((p.grad.double() ** 2).sum())
        ref = float(g["res_sumsq"][j])
        if n.endswith(".bias") and n.replace("bias", "weight") in names and \
                ref < 1e-6 * float(g["res_sumsq"][names.index(n.replace("bias", "weight"))]):
            continue
        assert sq == pytest.approx(ref, rel=4 * t), n
    # running statistics moved with momentum 0.1 (unbiased variance)
    assert not torch.equal(blk.norm1.running_mean.cpu(), rm0.cpu())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_dropout_residual_vs_autograd(dt):
    """conv -> BN(train) -> +residual -> ReLU -> Dropout2d mask, against float64 autograd with the same mask."""
    from hiseg.ops import Act
    conv = nn.Conv2d(64, 64, 3, padding=1)
    bn = nn.BatchNorm2d(64)
    filler.fill_module(_Holder(c=conv, b=bn), seed=11)
    TE, S, T = engine(_Holder(c=conv, b=bn), dt)
    x = torch.from_numpy(filler.normal(5, (3, 64, 10, 8))).to(DEV)
    r = torch.from_numpy(filler.normal(6, (3, 64, 10, 8))).to(DEV)
    xa, ra = Act.from_nchw(x, dt), Act.from_nchw(r, dt)
    drop = nn.Dropout2d(0.3)
    mask = TE.dropout_mask(T, drop, 3, 64, DEV)
    keep = (mask > 0).float().mean().item()
    assert 0.4 < keep < 0.95 and torch.all((mask == 0) | ((mask - 1 / 0.7).abs() < 1e-6))
    y = TE.conv_bn_act(T, conv, bn, TE.ACT_RELU, xa, residual=ra, drop=mask)
    g = torch.from_numpy(filler.normal(7, (3, 64, 10, 8))).to(DEV)
    inject(T, y, g, dt)
    S.flat.prepare_backward()
    T.run_backward()
    xr, rr = x.double().requires_grad_(True), r.double().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    br = conv.bias.detach().double().requires_grad_(True)
    gam = bn.weight.detach().double().requires_grad_(True)
    bet = bn.bias.detach().double().requires_grad_(True)
    z = F.conv2d(xr, wr, br, padding=1)
    zn = F.batch_norm(z, None, None, gam, bet, True, 0.1, 1e-5)
    dm = mask.double().view(3, 64, 1, 1)
    t = tol(dt)
    assert err(dt)(y.to_nchw(), (F.relu(zn + rr) * dm).detach()) < t
    # gradient at the kernel's own activation pattern (see relu_pattern_oracle)
    live = (y.to_nchw() > 0) | (dm == 0)
    yr = torch.where(live, zn + rr, torch.zeros_like(zn)) * dm
    (yr * g.double()).sum().backward()
    assert err(dt)(grad_nchw(T, xa), xr.grad) < 2 * t
    assert err(dt)(grad_nchw(T, ra), rr.grad) < t
    assert err(dt)(conv.weight.grad, wr.grad) < 2 * t
    assert err(dt)(bn.weight.grad, gam.grad) < 2 * t
    assert err(dt)(bn.bias.grad, bet.grad) < 2 * t
    assert conv.bias.grad.abs().max().item() < 1e-3 * bn.bias.grad.abs().max().item() + 1e-6


# ------------------------------------------------------------------------------------------ attention / gates / pool
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_attention_modules_train_match_reference(dt):
    from hiseg.layers import ChannelAttentionModule, SpatialAttentionModule
    from hiseg.ops import Act
    g = load("train_blocks")
    t = tol(dt)
    for i, key, mod in ((1, "sa", SpatialAttentionModule(7)), (2, "ca", ChannelAttentionModule(128, 8, act="relu"))):
        m = filler.fill_module(mod)
        TE, S, T = engine(_Holder(m=m), dt)
        x = torch.from_numpy(filler.normal(71 + i, tuple(g[f"{key}_gx"].shape))).to(DEV)
        xa = Act.from_nchw(x, dt)
        y = TE.spatial_attention(T, m, xa, None) if key == "sa" else TE.channel_attention(T, m, xa, None)
        inject(T, y, torch.from_numpy(filler.normal(81 + i, tuple(g[f"{key}_y"].shape))), dt)
        S.flat.prepare_backward()
        T.run_backward()
        assert err(dt)(y.to_nchw(), g[f"{key}_y"]) < t, key
        assert err(dt)(grad_nchw(T, xa), g[f"{key}_gx"]) < 2 * t, key
        for j, n in enumerate(g[f"{key}_names"]):
            p = dict(m.named_parameters())[n]
            assert float((p.grad.double() ** 2).sum()) == pytest.approx(float(g[f"{key}_sumsq"][j]), rel=6 * t), (key, n)


class relu_pattern_oracle:
    """Records the ReLU activation pattern of the hiseg train forward (every BN+ReLU output, in launch order)
    and replays it into the oracle's ``act(x, "relu")`` calls, so that a float64 oracle differentiates the
    same piecewise-linear branch the kernels took.  A ReLU whose pre-activation lies within f32 rounding of
    zero (1 in ~10^6 elements; e.g. 4.7e-8 in ResidualBlock(64) over 4x16x12 at these seeds) otherwise flips
    between implementations and moves that element's gradient by its full size -- after train-mode BN and
    a 3x3 conv that is a 3e-3 change of the input gradient, far above f32 rounding, and not a defect of
    either side.  The forward is still compared with the unmodified oracle."""

    def __init__(self, monkeypatch):
        from hiseg import train_engine as TE
        from oracle import rgb_model as O
        self.masks, self.i = [], 0
        orig_bn, orig_act = TE.bn_forward, O.act

        def bn_spy(T, bn, z, *, act, **kw):
            y, st = orig_bn(T, bn, z, act=act, **kw)
            if act == TE.ACT_RELU:
                self.masks.append(y.to_nchw() > 0)
            return y, st

        def act_replay(x, kind, beta=1.0):
            if kind != "relu" or not self.replay:
                return orig_act(x, kind, beta)
            m = self.masks[self.i]
            self.i += 1
            assert m.shape == x.shape, (m.shape, x.shape)
            return torch.where(m.to(x.device), x, torch.zeros_like(x))

        self.replay = False
        monkeypatch.setattr(TE, "bn_forward", bn_spy)
        monkeypatch.setattr(O, "act", act_replay)


def _unet_oracle(x, gy, dtype, device, masks=None):
    """Torch autograd of the oracle's EnhancedUNet (oracle/rgb_model.py:82) in `dtype` on `device`."""
    from hiseg.layers import EnhancedUNet
    from oracle import rgb_model as O
    from oracle import train as OT
    u = filler.fill_module(EnhancedUNet(256, 64, 3, "batchnorm", 8, "relu")).train()
    sd = {"m." + k: v.detach().to(device, dtype).requires_grad_(v.requires_grad) for k, v in OT.params_of(u).items()}
    xx = x.to(device, dtype).requires_grad_(True)
    with OT.train_mode():
        y = O.enhanced_unet(sd, "m", xx, 3, "relu")
    (y.double() * gy.to(device).double()).sum().backward()
    return y.detach().double().cpu(), xx.grad.double().cpu(), {k[2:]: v.grad for k, v in sd.items()
                                                               if v.grad is not None}


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_enhanced_unet_train_matches_reference(dt, monkeypatch):
    """EnhancedUNet(256, 64, depth 3) train forward/backward: maxpool, sigmoid bottleneck gate, ConvTranspose
    up-path with skip concatenation, f32 final logits, 20 train-mode BN layers over 4x16x12 pixels.

    Forward: the reference's golden vectors (1e-4 f32 / 0.1 bf16).  Backward, f32: the float64 oracle on the
    kernels' own ReLU pattern (relu_pattern_oracle) at 1e-4, and the golden input gradient by relative L2
    (< 1e-2: one pattern flip at these seeds costs 4e-3).  Backward, bf16: no better bound exists than
    PyTorch's own bf16 autograd of the same network (the BN stack amplifies bf16 activation rounding to
    ~50 % L2 of the input gradient), so hiseg must stay within 1.25x of torch-bf16's error against the golden
    vectors, input gradient and per-parameter gradients alike."""
    from hiseg.layers import EnhancedUNet
    from hiseg.ops import Act
    g = load("train_blocks")
    rp = relu_pattern_oracle(monkeypatch)
    u = filler.fill_module(EnhancedUNet(256, 64, 3, "batchnorm", 8, "relu")).train()
    TE, S, T = engine(_Holder(m=u), dt)
    x = torch.from_numpy(filler.normal(74, tuple(g["unet_gx"].shape)))
    xa = Act.from_nchw(x.to(DEV), dt)
    low, low_t = TE.enhanced_unet(T, u, xa)
    gy = torch.from_numpy(filler.normal(84, tuple(g["unet_y"].shape)))
    inject(T, low, gy.to(DEV), torch.float32)
    S.flat.prepare_backward()
    T.run_backward()
    gx = grad_nchw(T, xa).double().cpu()
    ry, rgx = torch.from_numpy(g["unet_y"]).double(), torch.from_numpy(g["unet_gx"]).double()
    grads = {n: p.grad.double().cpu() for n, p in u.named_parameters() if p.grad is not None}
    assert rel(low.to_nchw(), ry) < (1e-4 if dt == torch.float32 else 1e-1)
    if dt == torch.float32:
        rp.replay = True
        _, mgx, mp = _unet_oracle(x, gy, torch.float64, DEV)
        assert rp.i == len(rp.masks)
        assert rel(gx, mgx) < 1e-4
        for n, rg in mp.items():
            if n.endswith(".bias") and rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5:
                continue  # conv bias before train-mode BN: zero gradient in exact arithmetic
            assert rel2(grads[n], rg) < 1e-4, n
        assert rel2(gx, rgx) < 1e-2
    else:
        _, tgx, tp = _unet_oracle(x, gy, torch.bfloat16, DEV)
        assert rel2(gx, rgx) < 1.25 * rel2(tgx, rgx) + 1e-2
        names = list(g["unet_names"])
        mine = np.array([float((grads[n] ** 2).sum()) for n in names])
        theirs = np.array([float((tp[n].double() ** 2).sum()) for n in names])
        ref = g["unet_sumsq"]
        assert abs(mine.sum() / ref.sum() - 1) < 1.25 * abs(theirs.sum() / ref.sum() - 1) + 3e-2


# ------------------------------------------------------------------------------------------ loss
@pytest.mark.parametrize("case", ["a", "b", "c", "d", "e"])
def test_loss_kernel_matches_reference_golden(case):
    import hiseg
    from test_oracle_train import loss_inputs, loss_targets
    g = load("train_loss")
    keys = list(g["dict_keys"])
    names = sorted({k.split("_")[0] for k in g.files if k.endswith("_meta")})
    loss_fn = hiseg.RefinedHierarchicalLoss(bg_weight=1.5, fg_weight=1.5, target_weight=1.2, consistency_weight=0.3,
                                            use_dynamic_weights=True, dice_weight=1.0, ce_weight=1.0,
                                            boundary_aware_weight=0.1, contour_loss_weight=0.1,
                                            distance_loss_weight=0.1, use_boundary_aware_loss=True,
                                            use_contour_detection=True, use_distance_transform=True)
    for key in [n for n in names if n[0] == case]:
        seed, n, mh, mw = (int(v) for v in g[f"{key}_meta"])
        ins = [t.to(DEV).requires_grad_(True) for t in loss_inputs(seed, n, mh, mw)]
        tgt = loss_targets(str(g[f"{key}_kind"]), seed, n, mh, mw).to(DEV)
        aux = {"bg_fg_logits": ins[1], "target_nontarget_logits": ins[2], "contours": ins[3], "distance_map": ins[4]}
        loss, d = loss_fn(ins[0], tgt, aux)
        loss.backward()
        assert loss.item() == pytest.approx(float(g[f"{key}_loss"]), rel=1e-5, abs=1e-6), key
        for k, rv in zip(keys, g[f"{key}_dict"]):
            if np.isnan(rv):
                assert k not in d, (key, k)
            else:
                assert d[k] == pytest.approx(float(rv), rel=1e-4, abs=1e-6), (key, k)
        for i, nm in enumerate(["pred", "bgfg", "tn", "cont", "dist"]):
            ref = torch.from_numpy(g[f"{key}_grad_{nm}"])
            got = ins[i].grad.cpu()
            if ref.numel() == 0:
                assert not got.any(), (key, nm)
                continue
            assert (got - ref).abs().max().item() <= 1e-7 + 1e-4 * ref.abs().max().item(), (key, nm)


# ------------------------------------------------------------------------------------------ optimiser
def test_fused_adamw_matches_torch():
    import hiseg
    from hiseg import train_engine as TE
    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(8, 16, 3), nn.Conv2d(16, 4, 1)).to(DEV)
    ref = [p.detach().clone().requires_grad_(True) for p in m.parameters()]
    S = TE.TrainState(m, torch.float32, torch.device(DEV))
    m.__dict__["_hiseg_train"] = S
    opt = hiseg.FusedAdamW(m, lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    ropt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.01)
    for step in range(3):
        grads = [torch.randn_like(p) * (3.0 if step == 1 else 0.1) for p in ref]
        for p, g in zip(m.parameters(), grads):
            p.grad.copy_(g)
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        norm = opt.step()
        rn = torch.nn.utils.clip_grad_norm_(ref, 1.0)
        ropt.step()
        assert norm.item() == pytest.approx(rn.item(), rel=1e-5)
        for p, r in zip(m.parameters(), ref):
            assert (p.detach() - r.detach()).abs().max().item() < 1e-6


# ------------------------------------------------------------------------------------------ whole model
def _kwargs(name="b0"):
    from helpers import configs
    return hiseg_kwargs(dict(configs()[name]["model_kwargs"]))


def _model(dt, p_drop_zero=True, name="b0"):
    import hiseg
    m = hiseg.create_rgb_hierarchical_model(**_kwargs(name))
    filler.fill_module(m)
    if p_drop_zero:
        for mod in m.modules():
            if isinstance(mod, (nn.Dropout, nn.Dropout2d)):
                mod.p = 0.0
    hiseg.set_compute_dtype(m, dt)
    return m


@pytest.mark.parametrize("name", ["b0", "b1", "b7"])
def test_train_step_f32_matches_oracle(name):
    """B0-std (and the B1-enhanced 80x60 / B7-ultra 128x96, depth-4 presets) train forward + RefinedHierarchicalLoss + backward in f32 against the CPU oracle (torch autograd
    of the restated model, oracle/train.py) on the same inputs.  Loss and logits: 1e-4 relative.  Gradients:
    the ~50-layer train-mode BN stack at initialisation amplifies 1e-7 input changes into ~5 % gradient changes
    (tests/test_oracle_train.py), so parameter gradients are compared by cosine similarity (> 0.99 for every
    tensor with a non-negligible gradient) and the total gradient norm (2 %)."""
    import hiseg
    from oracle import rgb_model as O
    from oracle import train as OT
    m = _model(torch.float32, name=name)
    sd = OT.params_of(m)
    m = m.to(DEV).train()
    cfg = O.cfg_from_kwargs(_kwargs(name))
    images = torch.from_numpy(filler.uniform(61, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(62, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]])
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    tgt = torch.from_numpy(filler.ellipse_targets(63, 3, *cfg["mask_hw"]))
    from hiseg import train_engine as TE
    logits, aux = TE.train_forward(m, images.to(DEV), rois.to(DEV), u_override=u.to(DEV))
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    loss, d = loss_fn(logits, tgt.to(DEV), aux)
    loss.backward()
    rlog, raux = OT.forward_train(sd, images, rois, u, cfg, (96, 128))
    rloss, rd = OT.RefinedHierarchicalLoss()(rlog, tgt, raux)
    rloss.backward()
    # logits: the f32 oracle itself sits 6e-5 from float64 at this initialisation, and a 1e-7 relative
    # change of the input images moves the logits by 7.5e-5 (train-mode BN over 3 ROIs); 3e-3 ~ 4e-6
    # relative input-level rounding, the RoIAlign bilinear taps on uniform-noise images
    assert rel(logits.detach(), rlog.detach()) < 3e-3
    assert loss.item() == pytest.approx(rloss.item(), rel=1e-4)
    for k in ("bg_fg_loss", "final_loss", "dice_loss", "boundary_aware", "contour", "distance_transform"):
        assert d[k] == pytest.approx(rd[k], rel=1e-3), k
    tot_m, tot_r = 0.0, 0.0
    for n, p in m.named_parameters():
        if n not in sd or not sd[n].requires_grad:
            continue
        rg = sd[n].grad
        if rg is None:
            assert p.grad is None or not p.grad.any(), n
            continue
        mg = p.grad.detach().cpu().double().reshape(-1)
        rg = rg.double().reshape(-1)
        tot_m += float((mg ** 2).sum())
        tot_r += float((rg ** 2).sum())
        if rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5 or (n.endswith(".bias") and rg.norm() < 1e-4):
            continue
        cos = float((mg * rg).sum() / (mg.norm() * rg.norm()))
        # a 2-element tensor (output_conv: one weight per logit channel, a sum over every mask pixel of the
        # bilinear taps) has a cosine of its own angle only: both f32 implementations sit 2e-2 from float64 there
        # (tests/test_gpu_c1_u4_f64.py: hiseg 2.0e-2, oracle-f32 1.9e-2), so two independent 2e-2 errors may part
        # them by more than 0.99's 8 degrees
        assert cos > (0.95 if rg.numel() <= 4 else 0.99), (n, cos)
    assert abs(tot_m / tot_r - 1) < 4e-2


def test_train_loop_bf16_decreases_loss():
    """bf16 training with the fused AdamW: five steps on one batch (dropout on) lower the loss."""
    import hiseg
    m = _model(torch.bfloat16, p_drop_zero=False).to(DEV).train()
    images = torch.from_numpy(filler.uniform(91, (4, 3, 160, 192))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(92, 4, 1)).to(DEV)
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 160, 192
    tgt = torch.from_numpy(filler.ellipse_targets(93, 4, 128, 96)).to(DEV)
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    opt = None
    losses = []
    for step in range(6):
        logits, aux = m(images, rois)
        loss, d = loss_fn(logits, tgt, aux)
        if opt is None:
            opt = hiseg.FusedAdamW(m, lr=5e-4)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses
    assert set(d.keys()) >= {"bg_fg_loss", "final_loss", "dice_loss", "contour", "distance_transform"}


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cskip", [0, 24, 128])
def test_up_conv_backward_matches_autograd(dt, cskip):
    """smp DecoderBlock.conv1 (hiseg.effunet_train.up_conv_bn_relu): conv3x3 over cat(nearest-x2(x), skip)
    -> BN(train) -> ReLU; weight gradient through the upsampled + concatenated loader, data gradient through
    the 2x2 upsample sum, against float64 autograd on the kernels' ReLU pattern."""
    from hiseg import effunet_train as ET
    from hiseg.ops import Act
    cin = 64 if cskip != 128 else 128
    conv = nn.Conv2d(cin + cskip, 32, 3, padding=1, bias=False)
    bn = nn.BatchNorm2d(32)
    filler.fill_module(_Holder(c=conv, b=bn), seed=13)
    TE, S, T = engine(_Holder(c=conv, b=bn), dt)
    x = torch.from_numpy(filler.normal(14, (2, cin, 4, 6))).to(DEV)
    sk = torch.from_numpy(filler.normal(15, (2, max(cskip, 1), 8, 12))).to(DEV)[:, :cskip]
    xa = Act.from_nchw(x, dt)
    ska = Act.from_nchw(sk, dt) if cskip else None
    y = ET.up_conv_bn_relu(T, conv, bn, xa, ska, need_dx=True)
    g = torch.from_numpy(filler.normal(16, (2, 32, 8, 12))).to(DEV)
    inject(T, y, g, dt)
    S.flat.prepare_backward()
    T.run_backward()
    xr = x.double().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    inp = F.interpolate(xr, scale_factor=2, mode="nearest")
    if cskip:
        inp = torch.cat([inp, sk.double()], 1)
    zn = F.batch_norm(F.conv2d(inp, wr, None, padding=1), None, None, bn.weight.detach().double(),
                      bn.bias.detach().double(), True, 0.1, 1e-5)
    live = y.to_nchw() > 0
    yr = torch.where(live, zn, torch.zeros_like(zn))
    (yr * g.double()).sum().backward()
    t = tol(dt)
    assert err(dt)(conv.weight.grad, wr.grad) < 2 * t
    assert err(dt)(grad_nchw(T, xa), xr.grad) < 2 * t


def test_grad_sync_nccl_world1_matches_local():
    """hiseg.distributed over RCCL (world size 1 on the one-GPU box): the bucketed all-reduce on the
    communication stream, first-step schedule recording and the overlapped launches of the second step
    leave the gradients of two B0 train steps bit-identical to the unsynchronised run."""
    import os
    import torch.distributed as dist
    import hiseg
    from hiseg import distributed as HD
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    try:
        grads = []
        for sync in (False, True):
            m = _model(torch.bfloat16).to(DEV).train()
            for mm in (m.roi_align_mask, m.roi_align_rgb):
                mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
            if sync:
                s = HD.enable_grad_sync(m, bucket_mb=1.0)
            images = torch.from_numpy(filler.uniform(41, (2, 3, 96, 128))).to(DEV)
            rois = torch.from_numpy(filler.box_rois(42, 2, 2)).to(DEV)
            tgt = torch.from_numpy(filler.ellipse_targets(43, 4, 128, 96)).to(DEV)
            loss_fn = hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)
            out = []
            for step in range(2):
                logits, aux = m(images, rois)
                loss, _ = loss_fn(logits, tgt, aux)
                for p in m.parameters():
                    p.grad = None
                loss.backward()
                torch.cuda.synchronize()
                out.append(m.__dict__["_hiseg_train"].flat.grad.clone())
            if sync:
                assert len(s.buckets) > 3 and any(k >= 0 for k in s.launch_after)
                assert sorted(s.launched) == list(range(len(s.buckets)))
            grads.append(out)
        for a, b in zip(*grads):
            assert torch.equal(a, b)
    finally:
        dist.destroy_process_group()


def test_checkpoint_resume_continues_training_identically(tmp_path):
    """Two bf16 train steps, save_checkpoint (reference format, AdamW-layout optimizer state, torch cosine
    scheduler), resume into a fresh model + optimizer, one more step on both: identical parameters."""
    import hiseg
    images = torch.from_numpy(filler.uniform(191, (2, 3, 160, 192))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(192, 2, 1)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(193, 2, 128, 96)).to(DEV)

    def setup():
        m = _model(torch.bfloat16).to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 160, 192
        return m, hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)

    def step(m, loss_fn, state):
        if state.get("opt") is None:
            if state.get("resume"):
                m(images, rois)   # lays the parameters out flat (the optimiser's moments index into it)
            state["opt"] = hiseg.FusedAdamW(m, lr=5e-4)
            state["sched"] = torch.optim.lr_scheduler.CosineAnnealingLR(state["opt"], T_max=5, eta_min=1e-6)
            if state.get("resume"):
                hiseg.resume_from_checkpoint(state["resume"], m, state["opt"], state["sched"], map_location=DEV)
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        state["opt"].zero_grad()
        loss.backward()
        state["opt"].step()
        state["sched"].step()

    a, la = setup()
    sa = {}
    step(a, la, sa)
    step(a, la, sa)
    path = str(tmp_path / "ck.pth")
    hiseg.save_checkpoint(path, a, sa["opt"], epoch=1, best_miou=0.5, scheduler=sa["sched"])
    from hiseg.checkpoint import _reseed_output_conv
    _reseed_output_conv(a)   # what the resume does (train_advanced.py:1230-1241)
    b, lb = setup()
    sb = {"resume": path}
    # the loss EMA state is not part of the reference checkpoint: carry it over as the reference process would
    lb._state = la._state.clone()
    step(a, la, sa)
    step(b, lb, sb)
    torch.cuda.synchronize()
    assert sb["opt"].step_count == sa["opt"].step_count == 3
    assert sb["opt"].param_groups[0]["lr"] == sa["opt"].param_groups[0]["lr"]
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(pa, pb), n


def test_eval_after_training_sees_the_updated_weights():
    """Eval plans are cached per layer and keyed by the versions of the tensors they were packed from;
    FusedAdamW and the train-mode BN kernels write parameters / running statistics in place and must
    invalidate them: an eval forward after a train step equals a fresh model loaded with the new state."""
    import hiseg
    images = torch.from_numpy(filler.uniform(291, (2, 3, 160, 192))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(292, 2, 1)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(293, 2, 128, 96)).to(DEV)

    def prep(m):
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 160, 192
        return m

    m = prep(_model(torch.float32).to(DEV))
    with torch.no_grad():
        before, _ = m.eval()(images, rois)
    m.train()
    logits, aux = m(images, rois)
    loss, _ = hiseg.RefinedHierarchicalLoss()(logits, tgt, aux)
    opt = hiseg.FusedAdamW(m, lr=1e-3)
    opt.zero_grad()
    loss.backward()
    opt.step()
    with torch.no_grad():
        after, _ = m.eval()(images, rois)
    fresh = _model(torch.float32)
    fresh.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    fresh = prep(fresh.to(DEV))
    with torch.no_grad():
        ref, _ = fresh.eval()(images, rois)
    assert not torch.equal(before, after)
    assert torch.equal(after, ref)


def test_loss_class_weights_data_parallel_equal_single_process():
    """Two data-parallel ranks (each half of the ROI batch) with their class pixel counts summed -- what
    hiseg.distributed.sync_loss_class_weights does over RCCL -- carry, step after step, the dynamic class
    weights (and their EMA) of one process on the whole batch (hierarchical_segmentation.py:227-255, 286-309);
    without the sum they differ."""
    import ctypes
    import hiseg
    from hiseg import _lib as L
    N, H, W = 6, 64, 48
    g = torch.Generator().manual_seed(5)

    def batch(k):
        pred = torch.randn(N, 3, H, W, generator=g).to(DEV)
        aux = {"bg_fg_logits": torch.randn(N, 2, H, W, generator=g).to(DEV),
               "target_nontarget_logits": torch.randn(N, 2, H, W, generator=g).to(DEV)}
        tgt = torch.from_numpy(filler.ellipse_targets(40 + k, N, H, W)).to(DEV)
        return pred, aux, tgt

    def make():
        return hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=False)

    def counts_of(loss, tgt):   # hiseg_loss_fwd_begin on another rank's half
        cfg, _ = loss._cfg(H, W, False, False)
        n = tgt.shape[0]
        ws = torch.empty(int(L.lib().hiseg_loss_ws(n, H, W)), dtype=torch.float32, device=DEV)
        c = torch.empty(4, dtype=torch.float64, device=DEV)
        L.check(L.lib().hiseg_loss_fwd_begin(ctypes.byref(cfg), n, H, W, tgt.contiguous().data_ptr(), ws.data_ptr(),
                                             c.data_ptr(), L.stream_ptr()), "begin")
        return c

    full, r0, r1, solo = make(), make(), make(), make()
    keys = ("bg_weight", "fg_weight", "target_weight", "nontarget_weight")
    for k in range(3):
        pred, aux, tgt = batch(k)
        h0, h1 = slice(0, N // 2), slice(N // 2, N)
        _, d_full = full(pred, tgt, aux)
        r0.count_sync = lambda c, t=tgt[h1]: c.add_(counts_of(r0, t))
        r1.count_sync = lambda c, t=tgt[h0]: c.add_(counts_of(r1, t))
        _, d0 = r0(pred[h0].contiguous(), tgt[h0].contiguous(), {a: v[h0].contiguous() for a, v in aux.items()})
        _, d1 = r1(pred[h1].contiguous(), tgt[h1].contiguous(), {a: v[h1].contiguous() for a, v in aux.items()})
        _, ds = solo(pred[h0].contiguous(), tgt[h0].contiguous(), {a: v[h0].contiguous() for a, v in aux.items()})
        for key in keys:
            assert d0[key] == pytest.approx(d_full[key], rel=1e-6), (k, key)
            assert d1[key] == pytest.approx(d_full[key], rel=1e-6), (k, key)
    assert any(abs(ds[key] - d_full[key]) > 1e-4 for key in keys)


def test_graphed_train_step_equals_eager():
    """hiseg.GraphedStep (one HIP graph per training step) against eager steps from the same initial state:
    Dropout2d on (device seed base), FusedAdamW with clipping (device step count), the loss's EMA (device state)
    -- after 4 steps the parameters, the optimizer moments and the loss are identical."""
    import hiseg
    torch.manual_seed(0)
    images = torch.from_numpy(filler.uniform(31, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(32, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(33, 4, 128, 96)).to(DEV)
    runs, diag, gnorms = [], [], []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = _model(torch.bfloat16, p_drop_zero=False).to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
        loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                                use_distance_transform=True, boundary_aware_weight=0.1,
                                                contour_loss_weight=0.1, distance_loss_weight=0.1)
        st = {"opt": None}

        def step():
            logits, aux = m(images, rois)
            loss, _ = loss_fn(logits, tgt, aux)
            if st["opt"] is None:
                st["opt"] = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
            st["opt"].zero_grad()
            loss.backward()
            st["opt"].step()
            return loss

        run = hiseg.GraphedStep(step, lambda: st["opt"]) if graphed else step
        losses, norms = [], []
        for _ in range(4):
            losses.append(float(run().detach()))
            norms.append((float(st["opt"].last_norm), st["opt"].step_count, st["opt"].skipped_steps))
            if not np.isfinite(norms[-1][0]):   # name the parameters whose gradient is not finite
                bad = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
                norms.append(("non-finite grads", bad[:8], len(bad)))
            if len(losses) == 1:   # per-parameter gradient norms of the first step (after clipping)
                gnorms.append({n: float(p.grad.float().norm()) for n, p in m.named_parameters() if p.grad is not None})
        torch.cuda.synchronize()
        if graphed:
            assert run.captures == 1
        params = torch.cat([p.detach().float().reshape(-1) for p in m.parameters()]).cpu()
        runs.append((losses, params, st["opt"].exp_avg.cpu(), st["opt"].step_count))
        diag.append(norms)
    (l0, p0, m0, s0), (l1, p1, m1, s1) = runs
    # diag: per step (pre-clip gradient norm, applied steps, skipped steps) of the eager / graphed runs
    if l0 != l1:
        print("graphed-vs-eager diagnostics:", repr((l0, l1, diag)), flush=True)
        ge, gg = gnorms
        c0, c1 = diag[0][0][0], diag[1][0][0]   # pre-clip totals: compare unclipped per-parameter norms
        s0, s1 = min(1.0, 1.0 / (c0 + 1e-6)), min(1.0, 1.0 / (c1 + 1e-6))
        rows = sorted(((abs(ge[k] / s0 - gg[k] / s1) / (gg[k] / s1 + 1e-12), k, ge[k] / s0, gg[k] / s1) for k in gg),
                      reverse=True)
        print("first-step gradient norms, eager vs graphed (largest relative differences):", flush=True)
        for r in rows[:25]:
            print("   %.3e  %-70s %.6e %.6e" % r, flush=True)
    assert l0 == l1, f"eager {l0} vs graphed {l1}; per step (grad norm, steps, skipped): {diag}"
    assert s0 == s1 == 4
    assert torch.equal(p0, p1) and torch.equal(m0, m1)
    assert l0[-1] != l0[0]


def test_graphed_step_recaptures_after_optimizer_swap():
    """the captured graph holds the optimizer's buffer addresses.  Replacing the optimizer between
    replays (the reference's progressive-unfreezing pattern: a new AdamW with the old state transferred,
    train_distillation_staged.py:1531-1552) must make GraphedStep run eagerly again and re-capture, so its
    trajectory stays bit-identical to eager steps that do the same swap."""
    import hiseg
    images = torch.from_numpy(filler.uniform(131, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(132, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(133, 4, 128, 96)).to(DEV)
    runs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = _model(torch.bfloat16).to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
        loss_fn = hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)
        st = {"opt": None}

        def step():
            logits, aux = m(images, rois)
            loss, _ = loss_fn(logits, tgt, aux)
            if st["opt"] is None:
                st["opt"] = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
            st["opt"].zero_grad()
            loss.backward()
            st["opt"].step()
            return loss

        run = hiseg.GraphedStep(step, lambda: st["opt"]) if graphed else step
        losses = [float(run().detach()) for _ in range(4)]
        old = st["opt"]
        new = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
        for p in new.param_groups[0]["params"]:
            if p in old.state:
                new.state[p] = old.state[p]
        st["opt"] = new
        losses += [float(run().detach()) for _ in range(4)]
        torch.cuda.synchronize()
        if graphed:
            assert run.captures == 2
        params = torch.cat([p.detach().float().reshape(-1) for p in m.parameters()]).cpu()
        runs.append((losses, params, new.exp_avg.cpu(), new.step_count))
    (l0, p0, m0, s0), (l1, p1, m1, s1) = runs
    assert l0 == l1, (l0, l1)
    assert s0 == s1 == 8
    assert torch.equal(p0, p1) and torch.equal(m0, m1)


def test_side_stream_train_step_equals_default_stream():
    """a fresh model's bf16 train steps (Dropout2d on, FusedAdamW with clipping) issued on the default
    stream and under torch.cuda.stream(side) -- every buffer created in the first step (flat parameters, packing
    tables, optimizer state) then lives on the side stream -- are bit-identical over 3 steps."""
    import hiseg
    images = torch.from_numpy(filler.uniform(141, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(142, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(143, 4, 128, 96)).to(DEV)
    runs = []
    for side in (None, torch.cuda.Stream(), torch.cuda.Stream()):
        torch.manual_seed(0)
        m = _model(torch.bfloat16, p_drop_zero=False).to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
        loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                                use_distance_transform=True)
        opt = None
        losses = []
        for _ in range(3):
            if side is not None:
                side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side) if side is not None else torch.cuda.stream(torch.cuda.current_stream()):
                logits, aux = m(images, rois)
                loss, _ = loss_fn(logits, tgt, aux)
                if opt is None:
                    opt = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
                opt.zero_grad()
                loss.backward()
                opt.step()
            if side is not None:
                torch.cuda.current_stream().wait_stream(side)
            losses.append(float(loss.detach()))
        torch.cuda.synchronize()
        params = torch.cat([p.detach().float().reshape(-1) for p in m.parameters()]).cpu()
        runs.append((losses, params, opt.exp_avg_sq.cpu(), opt.step_count))
    for l, p, v, s in runs[1:]:
        assert l == runs[0][0]
        assert s == runs[0][3] == 3
        assert torch.equal(p, runs[0][1]) and torch.equal(v, runs[0][2])


@pytest.mark.parametrize("cin,cout,split", [(128, 256, None), (256, 128, None), (128, 128, (64, 64)), (64, 64, None)])
def test_train_pack_fragment_order_matches_frag_pack(cin, cout, split):
    """hiseg_pack_weights with HISEG_PACK_FRAG (the training path's weights for conv_hwr.hip): the forward and the
    data-gradient matrices in MFMA fragment order equal hiseg.ops.frag_pack of the row-major packs, bit for bit."""
    from hiseg import ops
    from hiseg import train_engine as TE
    torch.manual_seed(3)
    m = nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1)).to(DEV)
    S = TE.TrainState(m, torch.bfloat16, torch.device(DEV))
    p = S.conv(m[0], split=split)
    torch.cuda.synchronize()
    assert p.w_fwd_frag is not None
    ref = ops.frag_pack(p.w_fwd.float(), 9, p.ca + p.cb).to(torch.bfloat16)
    assert torch.equal(p.w_fwd_frag.reshape(-1), ref.reshape(-1))
    if p.cop % 64 == 0:
        assert p.w_dgrad_frag is not None
        refd = ops.frag_pack(p.w_dgrad.float(), 9, p.cop).to(torch.bfloat16)
        assert torch.equal(p.w_dgrad_frag.reshape(-1), refd.reshape(-1))


def _placed(big, off_elems, x_nchw, dt):
    """An NHWC Act over big[off_elems:] (bf16) holding x: its address is chosen by the caller."""
    from hiseg.ops import Act
    a = Act.from_nchw(x_nchw, dt)
    n = a.t.numel()
    t = big[off_elems:off_elems + n]
    t.copy_(a.t)
    return Act(t, a.N, a.H, a.W, a.C, a.cstride, a.coff)


@pytest.mark.parametrize("case", [(64, 32, 3, 12, 16, 2, 2, 32), (128, 128, 3, 8, 6, 2, 1, 128),
                                  (256, 8, 1, 8, 6, 2, 1, 256), (64, 64, 3, 10, 9, 2, 1, 64),
                                  (72, 72, 3, 10, 9, 2, 1, 72), (96, 96, 3, 8, 6, 2, 1, 96),
                                  (320, 112, 3, 8, 8, 2, 2, 256), (128, 24, 3, 12, 16, 2, 2, 64)])
def test_two_source_results_do_not_depend_on_operand_placement(case):
    """Kernels that address both sources of a concat through one buffer resource decline layers whose sources lie
    more than 2 GiB apart; the kernel then chosen must give bit-identical results (conv_rows -> conv_small; the
    weight gradient's pixel splits follow one geometry for every kernel).  Same layer, the sources 64 MiB apart
    vs 3 GiB apart inside one allocation: forward outputs and weight / bias gradients bit-identical.
    VERDICT r4 next #1: the weight gradient of a far-apart concat never falls back to the generic kernel (the
    transposed-read tile takes it with one buffer resource per source) -- the EnhancedUNet decoders' 64 / 72 / 96 /
    192 + same concats and the smp decoder's upsampled conv1 (320 + 112, 128 + 24) ran it 10-80x slower."""
    from hiseg.ops import Act
    from hiseg import effunet_train as EU
    ca, cb, k, H, W, N, up, cout = case
    dt = torch.bfloat16
    big = torch.zeros((3 << 30) + (64 << 20), dtype=torch.uint8, device=DEV).view(dt)
    x = torch.from_numpy(filler.normal(61, (N, ca, H // up, W // up))).to(DEV)
    s_ = torch.from_numpy(filler.normal(62, (N, cb, H, W))).to(DEV)
    g = torch.from_numpy(filler.normal(63, (N, cout, H, W))).to(DEV)
    from hiseg import _lib as L
    res = []
    for far in (False, True):
        L.placement_stats(reset=True)
        L.wgrad_path_stats(reset=True)
        conv = nn.Conv2d(ca + cb, cout, k, padding=k // 2, bias=up == 1)
        filler.fill_module(conv, seed=64)
        bn = nn.BatchNorm2d(cout)
        filler.fill_module(bn, seed=65)
        TE, S, T = engine(_Holder(c=conv, b=bn), dt)
        xa = _placed(big, 0, x, dt)
        xb = _placed(big, ((3 << 30) if far else (64 << 20)) // 2, s_, dt)
        assert abs(xb.ptr() - xa.ptr()) >= (3 << 30) if far else abs(xb.ptr() - xa.ptr()) < (1 << 30)
        if up == 1:
            y = TE.conv_plain(T, conv, TE.ACT_NONE, xa, xb, split=(ca, cb))
            inject(T, y, g, dt)
            S.flat.prepare_backward()
            T.run_backward()
            torch.cuda.synchronize()
            res.append((y.t.clone(), conv.weight.grad.clone(), conv.bias.grad.clone()))
        else:   # the smp decoder's conv1 form (upsampled src A ++ skip)
            from hiseg import ops
            p = ops.pack_conv(conv.weight, conv.bias, None, 1, dt, DEV, pad=1, split=(ca, cb))
            yy = ops.conv2d(p, xa, xb, a_up=2)
            torch.cuda.synchronize()
            # the row-streaming kernel takes the layer wherever its sources lie (one buffer
            # resource per source when far apart), never a placement fallback
            declined, far_taken = L.placement_stats(reset=True)
            assert declined == 0, "a kernel declined the decoder conv1 for its sources' placement"
            # its training form: forward, train-mode BN + ReLU, weight gradient of the upsampled concat
            y = EU.up_conv_bn_relu(T, conv, bn, xa, xb, need_dx=False)
            inject(T, y, g, dt)
            S.flat.prepare_backward()
            T.run_backward()
            torch.cuda.synchronize()
            res.append((yy.t.clone(), y.t.clone(), conv.weight.grad.clone()))
        paths = L.wgrad_path_stats()
        assert paths["generic_bf16"] == 0, f"generic weight-gradient kernel ran (far={far}): {paths}"
        assert paths["wide"] + paths["transposed_read"] + paths["halo"] == 1, paths
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("case", [(256, 256, 3, 20, 30, 0), (128, 128, 2, 37, 21, 0), (128, 256, 2, 16, 16, 0),
                                  (320, 256, 2, 16, 20, 64), (128, 128, 24, 40, 40, 0), (64, 64, 2, 37, 45, 0),
                                  (128, 64, 2, 18, 34, 64)])
def test_fused_bn_statistics_match_the_statistics_pass(case, monkeypatch):
    """Round 5: the conv feeding a train-mode BatchNorm writes the batch-statistics partials of
    its bf16 output from the epilogue (conv_hwc's ST form: per 16 x 16-pixel tile and channel count / mean / M2,
    merged by hiseg_bn_finalize_n) instead of a statistics pass over z.  Against HISEG_FUSED_BN_STATS=0 (the pass):
    the conv output z bit-identical, batch mean / invstd within f32 re-association (1e-5 relative), running stats
    likewise, the BN output within one bf16 ulp, and the fused path actually taken (hiseg_conv2d_stats_tiles > 0).
    Ragged tiles; the smp decoder's upsampled conv1 form (Cb > 0: x2-upsampled src A ++ skip)."""
    from hiseg import _lib as L
    from hiseg import effunet_train as EU
    from hiseg.ops import Act
    ca, cout, N, H, W, cb = case
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(5)
    up = cb > 0
    x = torch.randn(N, ca, H // 2 if up else H, W // 2 if up else W, device=DEV, generator=g)
    sk = torch.randn(N, cb, H, W, device=DEV, generator=g) if up else None
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("HISEG_FUSED_BN_STATS", fused)
        conv = nn.Conv2d(ca + cb, cout, 3, padding=1, bias=True)
        filler.fill_module(conv, seed=66)
        bn = nn.BatchNorm2d(cout)
        filler.fill_module(bn, seed=67)
        TE, S, T = engine(_Holder(c=conv, b=bn), dt)
        xa = Act.from_nchw(x, dt)
        seen = []
        real = TE.bn_forward

        def spy(*a, **k):
            seen.append(bool(k.get("stats")))
            return real(*a, **k)
        monkeypatch.setattr(TE, "bn_forward", spy)
        if up:
            y = EU.up_conv_bn_relu(T, conv, bn, xa, Act.from_nchw(sk, dt), need_dx=False)
        else:
            y = TE.conv_bn_act(T, conv, bn, TE.ACT_RELU, xa)
        monkeypatch.setattr(TE, "bn_forward", real)
        torch.cuda.synchronize()
        assert seen == [fused == "1"], seen
        res[fused] = (y.t.float().clone(), bn.running_mean.clone(), bn.running_var.clone())
    (y1, m1, v1), (y0, m0, v0) = res["1"], res["0"]
    assert torch.isfinite(y1).all()
    assert torch.allclose(m1, m0, rtol=1e-5, atol=1e-6) and torch.allclose(v1, v0, rtol=1e-5, atol=1e-6)
    # one bf16 ulp of the output (the normalised value may round either way when mean / invstd differ in the last bit)
    assert ((y1 - y0).abs() <= y0.abs() * 2 ** -7 + 1e-6).all()
    assert (y1 == y0).float().mean() > 0.98


@pytest.mark.parametrize("S,C", [(40, 64), (3001, 80), (12288, 256)])
def test_bn_finalize_n_matches_f64_merge(S, C):
    """hiseg_bn_finalize_n over S split partials [S][3][C] (count, mean, M2; some splits empty): more than 256 splits
    are pre-merged in groups of 64 in place (bn_premerge_kernel) before the per-channel merge.  Mean / invstd /
    scale / shift / running statistics against a float64 Chan merge of the same partials (1e-6 relative)."""
    from hiseg import _lib as L
    rng = np.random.default_rng(S + C)
    n = rng.integers(0, 65, size=(S, C)).astype(np.float32)
    n[rng.random((S, C)) < 0.05] = 0
    n[0] = 7   # every channel has data
    mu = (rng.standard_normal((S, C)) * 0.3 + 2.0).astype(np.float32)
    m2 = (rng.random((S, C)) * n).astype(np.float32)
    mu[n == 0] = 0
    m2[n == 0] = 0
    part = np.stack([n, mu, m2], axis=1)   # [S][3][C]
    P = int(n.sum(axis=0).max())
    tot = n.astype(np.float64).sum(axis=0)
    mean = (n * mu.astype(np.float64)).sum(axis=0) / tot
    var = (m2.astype(np.float64).sum(axis=0) + (n * (mu.astype(np.float64) - mean) ** 2).sum(axis=0)) / tot
    gamma = torch.from_numpy(rng.standard_normal(C).astype(np.float32)).to(DEV)
    beta = torch.from_numpy(rng.standard_normal(C).astype(np.float32)).to(DEV)
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    out = [torch.empty(C, device=DEV) for _ in range(4)]
    pt = torch.from_numpy(part).to(DEV).contiguous()
    eps, mom = 1e-5, 0.1
    L.check(L.lib().hiseg_bn_finalize_n(pt.data_ptr(), S, C, P, gamma.data_ptr(), beta.data_ptr(), eps, mom,
                                        rm.data_ptr(), rv.data_ptr(), *[o.data_ptr() for o in out], L.stream_ptr()),
            "bn_finalize_n")
    torch.cuda.synchronize()
    m_o, inv_o, sc_o, sh_o = [o.double().cpu().numpy() for o in out]
    inv = 1.0 / np.sqrt(var + eps)
    g, b = gamma.double().cpu().numpy(), beta.double().cpu().numpy()
    np.testing.assert_allclose(m_o, mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(inv_o, inv, rtol=1e-6)
    np.testing.assert_allclose(sc_o, g * inv, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(sh_o, b - mean * g * inv, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rm.double().cpu().numpy(), mom * mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(rv.double().cpu().numpy(), (1 - mom) + mom * var * P / (P - 1), rtol=1e-6)


@pytest.mark.parametrize("case", [(256, 3, 20, 30), (128, 2, 37, 21), (64, 2, 33, 50)])
def test_fused_bn_backward_reduction_matches_the_reduction_pass(case, monkeypatch):
    """Round 5 (second half): in a ResidualBlock the first BatchNorm's output feeds conv2 alone,
    so conv2's data gradient -- the one write of that gradient -- computes the BatchNorm backward reduction (sums of
    g, g * xhat, xhat per channel, g masked by the forward's ReLU) in its epilogue (conv_hwc BR form) and hiseg_bn_bwd
    skips its reduction pass (partial_splits).  Against HISEG_FUSED_BN_BWD=0: every parameter gradient and the input
    gradient within f32 re-association of the sums (one bf16 ulp of the tensor's largest value: a coefficient moved
    by an f32 ulp can round a bf16 dz, and the bf16 input gradient, either way), the fused path taken."""
    from hiseg import train_engine as TEm
    from hiseg.layers import ResidualBlock
    from hiseg.ops import Act
    C, N, H, W = case
    dt = torch.bfloat16
    x = torch.from_numpy(filler.normal(81, (N, C, H, W))).to(DEV)
    g = torch.from_numpy(filler.normal(82, (N, C, H, W))).to(DEV)
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("HISEG_FUSED_BN_BWD", fused)
        blk = ResidualBlock(C, "batchnorm", 8, "relu", 1.0)
        filler.fill_module(blk, seed=83)
        TE, S, T = engine(_Holder(b=blk), dt)
        xa = Act.from_nchw(x, dt)
        before = TEm.FUSED_BN_BWD_TAKEN[0]
        y = TE.residual_block(T, blk, xa)
        inject(T, y, g, dt)
        S.flat.prepare_backward()
        T.run_backward()
        torch.cuda.synchronize()
        taken = TEm.FUSED_BN_BWD_TAKEN[0] - before
        assert taken == (1 if fused == "1" else 0), taken
        res[fused] = [p.grad.detach().float().clone() for p in blk.parameters()] + [grad_nchw(T, xa).clone()]
    for a, b in zip(res["1"], res["0"]):
        assert torch.isfinite(a).all()
        assert (a - b).abs().max() <= 2 ** -7 * b.abs().max() + 1e-6, ((a - b).abs().max(), b.abs().max())


@pytest.mark.parametrize("case", [(32, 3, 1, 2, 40, 48), (144, 5, 1, 2, 20, 24), (96, 3, 2, 2, 33, 27),
                                  (240, 5, 2, 1, 16, 20), (1152, 3, 1, 2, 10, 10)])
def test_train_depthwise_on_inference_kernels_matches_train_kernels(case, monkeypatch):
    """Round 5: the unfrozen EfficientNet stages' depthwise conv (dw_bn_silu) in bf16 runs its forward -- and, at stride
    1, its data gradient as the conv with the 180-degree rotated kernel -- on the inference depthwise kernels
    (hiseg_dwconv_fwd, unit affine, no activation) instead of hiseg_dw_train_fwd / hiseg_dw_bwd_data
    (HISEG_TRAIN_DW_FAST=0).  Both are bf16 executions of the same math: outputs and gradients within bf16 rounding of
    each other (2e-2 relative to the tensor's scale; the depthwise weight gradient within 2e-2), stride 1 / 2, k 3 / 5,
    ragged images."""
    from hiseg import effunet_train as EU
    from hiseg.ops import Act
    C, k, st, N, H, W = case
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    Ho, Wo = (H + 2 * (k // 2) - k) // st + 1, (W + 2 * (k // 2) - k) // st + 1
    gy = torch.randn(N, C, Ho, Wo, device=DEV, generator=g)
    res = {}
    for fast in ("1", "0"):
        monkeypatch.setenv("HISEG_TRAIN_DW_FAST", fast)
        conv = nn.Conv2d(C, C, k, stride=st, padding=k // 2, groups=C, bias=False)
        filler.fill_module(conv, seed=71)
        bn = nn.BatchNorm2d(C)
        filler.fill_module(bn, seed=72)
        TE, S, T = engine(_Holder(c=conv, b=bn), dt)
        xa = Act.from_nchw(x, dt)
        y = EU.dw_bn_silu(T, conv, bn, xa, need_dx=True)
        inject(T, y, gy, dt)
        S.flat.prepare_backward()
        T.run_backward()
        torch.cuda.synchronize()
        res[fast] = (y.to_nchw().float(), grad_nchw(T, xa).float(), conv.weight.grad.clone())
    for a, b in zip(res["1"], res["0"]):
        assert torch.isfinite(a).all()
        assert ((a - b).abs().max() / b.abs().max()).item() < 2e-2


@pytest.mark.gpu
def test_train_step_independent_of_allocator_churn_between_forward_and_backward():
    """Every buffer a backward reads through a raw address stays alive until that backward ran: one bf16 train step
    with Dropout2d on, once plainly and once with the caching allocator's small blocks reused and overwritten
    between the forward and the backward -- bit-identical parameter gradients.  (Regression: fg_gate's Dropout2d
    mask was released after the forward while the backward's copied descriptor still pointed at it.)"""
    import hiseg
    images = torch.from_numpy(filler.uniform(31, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(32, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(33, 4, 128, 96)).to(DEV)
    grads = []
    for churn in (False, True):
        torch.manual_seed(0)
        m = _model(torch.bfloat16, p_drop_zero=False).to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
        loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                                use_distance_transform=True, boundary_aware_weight=0.1,
                                                contour_loss_weight=0.1, distance_loss_weight=0.1)
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if churn:   # small tensors of every size class the step frees, filled with a value no mask holds
            held = [torch.full((n,), 7.0, device=DEV) for n in (64, 128, 256, 512, 1024, 4096, 16384) for _ in range(64)]
            del held
        loss.backward()
        torch.cuda.synchronize()
        S = m.__dict__["_hiseg_train"]
        grads.append(S.flat.grad.clone())
    assert torch.isfinite(grads[0]).all()
    assert torch.equal(grads[0], grads[1])


def test_ubf_backward_two_pixel_loop_bit_identical(monkeypatch):
    """The upsample_bg_fg backward's first pass with two pixels per iteration and its ConvTranspose weights held in
    registers (HISEG_UBF_U2, default) against the one-pixel loop (HISEG_UBF_U2=0): same per-pixel arithmetic, sums in
    pixel order -- a bf16 B0 train step's loss and every parameter gradient equal bit for bit."""
    import hiseg
    from hiseg import train_engine as TE
    images = torch.from_numpy(filler.uniform(71, (2, 3, 96, 128))).to(DEV)
    u = torch.from_numpy(filler.normal(72, (2, 1, 96, 128)) * 2.0).to(DEV)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]]).to(DEV)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("HISEG_UBF_U2", mode)
        m = _model(torch.bfloat16).to(DEV).train()
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
        tgt = torch.from_numpy(filler.ellipse_targets(73, 3, *m.mask_size)).to(DEV)
        logits, aux = TE.train_forward(m, images, rois, u_override=u)
        loss, _ = hiseg.RefinedHierarchicalLoss()(logits, tgt, aux)
        loss.backward()
        torch.cuda.synchronize()
        res[mode] = (loss.detach().clone(), [p.grad.detach().clone() for p in m.parameters() if p.grad is not None])
    (l1, g1), (l0, g0) = res["1"], res["0"]
    assert torch.isfinite(l1) and torch.equal(l1, l0)
    assert len(g1) == len(g0) and all(torch.equal(a, b) for a, b in zip(g1, g0))


def test_train_step_bf16_within_torch_bf16_of_oracle(monkeypatch):
    """the bf16 training bar, tied to PyTorch's own bf16.  The f32 oracle (torch autograd of the
    restated B0-std model, oracle/train.py) is the reference; the same oracle run by torch in bf16 (bf16 weights,
    activations and autograd, the loss in f32 as under the reference's autocast, train_advanced.py:693-762) sets
    the error a bf16 execution incurs.  hiseg's bf16 step -- including the BatchNorm statistics fused into the
    conv_hwc epilogue and the bf16 weight / data gradient kernels -- must stay within a small multiple of it: loss
    and logits within 1.5x (+1e-3) of torch-bf16's relative error, the whole gradient's direction within 2x of
    torch-bf16's (1 - cosine, +1e-4) and its norm within 2x (+1e-2).
    Why not an absolute bar: at this random initialisation the train-mode head is chaotic -- rounding only the
    WEIGHTS to bf16 and running the f32 oracle moves its logits by ~30 % (max-relative) and its gradient's cosine to
    ~0.4 (measured on the CPU oracle, round 6), torch-bf16 lands at ~0.5 / ~0.2 (GPU run: hiseg 0.52 / 0.20, torch
    0.62 / 0.16; loss 6.0e-4 vs 1.2e-3).  So no bf16 execution is within a fixed tolerance of f32 here; the claim
    tested is that hiseg's bf16 step is no further from f32 than PyTorch's own bf16 step."""
    import hiseg
    from oracle import rgb_model as O
    from oracle import train as OT
    from hiseg import train_engine as TE
    m = _model(torch.bfloat16)
    sd = OT.params_of(m)
    m = m.to(DEV).train()
    cfg = O.cfg_from_kwargs(_kwargs())
    images = torch.from_numpy(filler.uniform(71, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(72, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70],
                         [1, .05, .30, .60, .85]])
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    tgt = torch.from_numpy(filler.ellipse_targets(73, 4, *cfg["mask_hw"]))
    # hiseg bf16 (the weights are the bf16 roundings of the f32 initialisation: the oracle starts from those too)
    logits, aux = TE.train_forward(m, images.to(DEV), rois.to(DEV), u_override=u.to(DEV))
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    loss, _ = loss_fn(logits, tgt.to(DEV), aux)
    loss.backward()

    def oracle_step(params, dt):
        if dt == torch.bfloat16:
            orig = OT.roi_align_torch
            monkeypatch.setattr(OT, "roi_align_torch", lambda feat, *a, **k: orig(feat.float(), *a, **k).to(feat.dtype))
        rlog, raux = OT.forward_train(params, images.to(dt), rois, u.to(dt), cfg, (96, 128))
        rloss, _ = OT.RefinedHierarchicalLoss()(rlog.float(), tgt, {k: v.float() for k, v in raux.items()})
        rloss.backward()
        monkeypatch.undo()
        return rloss.item(), rlog.detach().float()

    sd16 = {k: (v.detach().bfloat16().requires_grad_(True) if v.requires_grad else v.detach().bfloat16())
            for k, v in sd.items()}
    l32, g32 = oracle_step(sd, torch.float32)
    l16, g16 = oracle_step(sd16, torch.bfloat16)

    def flat_grads(get):
        out = []
        for n, p in m.named_parameters():
            if n in sd and sd[n].requires_grad and sd[n].grad is not None:
                out.append(get(n, p).double().reshape(-1))
        return torch.cat(out)
    gr = flat_grads(lambda n, p: sd[n].grad)
    gt = flat_grads(lambda n, p: sd16[n].grad.float())
    gh = flat_grads(lambda n, p: p.grad.detach().float().cpu())

    def cos(a, b):
        return float((a * b).sum() / (a.norm() * b.norm()))
    e_loss_h, e_loss_t = abs(loss.item() - l32) / abs(l32), abs(l16 - l32) / abs(l32)
    e_log_h, e_log_t = rel(logits.detach().float(), g32), rel(g16, g32)
    c_h, c_t = 1 - cos(gh, gr), 1 - cos(gt, gr)
    n_h, n_t = abs(float(gh.norm() / gr.norm()) - 1), abs(float(gt.norm() / gr.norm()) - 1)
    print(f"bf16 train vs f32 oracle: loss {e_loss_h:.2e} (torch {e_loss_t:.2e}), logits {e_log_h:.2e} "
          f"(torch {e_log_t:.2e}), 1-cos {c_h:.2e} (torch {c_t:.2e}), norm {n_h:.2e} (torch {n_t:.2e})")
    assert e_loss_h < 1.5 * e_loss_t + 1e-3
    assert e_log_h < 1.5 * e_log_t + 1e-3
    assert c_h < 2 * c_t + 1e-4
    assert n_h < 2 * n_t + 1e-2


@pytest.mark.parametrize("tiled", ["1", "0"])
@pytest.mark.parametrize("case", [(4, 32, 320, 320, 3, 1), (4, 96, 320, 320, 3, 2), (4, 144, 160, 160, 5, 1),
                                  (4, 240, 80, 80, 5, 2), (4, 1152, 20, 20, 5, 1), (2, 200, 37, 45, 5, 1),
                                  (3, 104, 33, 21, 3, 2), (1, 40, 9, 7, 5, 2)])
def test_depthwise_weight_gradient_matches_f64_at_encoder_scale(case, tiled, monkeypatch):
    """The depthwise weight gradient of the unfrozen encoder's largest-pixel layers (B0 at 640 x 640, 4 images: up to
    409 600 output pixels, 1 024 split partials per weight) against float64 autograd of the same bf16 operands.  The
    split partials are f32 sums of ~32 exact bf16 products; their reduce runs in double: the result sits
    within 1e-5 of the float64 gradient's scale.  Both forms (HISEG_DW_WGRAD_TILE: 1 the LDS-tiled kernel of round 6,
    per-tile-row f32 partials of 16 x K products, one- or two-pass double reduce; 0 the split kernel), ragged tiles,
    partial channel groups, and the gradient accumulated onto a non-zero buffer."""
    from hiseg import _lib as L
    from hiseg.ops import Act, hdtype
    monkeypatch.setenv("HISEG_DW_WGRAD_TILE", tiled)
    N, C, H, W, k, st = case
    g = torch.Generator(device=DEV).manual_seed(123)
    x = torch.randn(N, C, H, W, device=DEV, generator=g).bfloat16()
    Ho, Wo = (H + 2 * (k // 2) - k) // st + 1, (W + 2 * (k // 2) - k) // st + 1
    dy = torch.randn(N, C, Ho, Wo, device=DEV, generator=g).bfloat16()
    xa, dya = Act.from_nchw(x.float(), torch.bfloat16), Act.from_nchw(dy.float(), torch.bfloat16)
    lib = L.lib()
    ws = torch.empty(int(lib.hiseg_dw_bwd_weight_ws(hdtype(torch.bfloat16), N, Ho, Wo, C, k)), dtype=torch.float32,
                     device=DEV)
    dw0 = torch.randn(C * k * k, dtype=torch.float32, device=DEV, generator=g)
    dw = dw0.clone()
    L.check(lib.hiseg_dw_bwd_weight(hdtype(torch.bfloat16), xa.ptr(), dya.ptr(), N, H, W, C, k, st, Ho, Wo,
                                    ws.data_ptr(), dw.data_ptr(), L.stream_ptr()), "dw_bwd_weight")
    w64 = torch.zeros(C, 1, k, k, dtype=torch.float64, device=DEV, requires_grad=True)
    y = F.conv2d(x.double(), w64, stride=st, padding=k // 2, groups=C)
    y.backward(dy.double())
    ref = w64.grad.reshape(-1) + dw0.double()
    err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-5, err


@pytest.mark.parametrize("case", [(4, 96, 320, 320, 3), (4, 144, 160, 160, 5), (4, 240, 80, 80, 3), (4, 672, 40, 40, 5),
                                  (2, 200, 37, 45, 5), (3, 104, 33, 21, 3), (1, 40, 9, 7, 5)])
def test_depthwise_stride2_data_gradient_tiled_matches_per_pixel_and_f64(case, monkeypatch):
    """The stride-2 depthwise data gradient: the LDS-tiled kernel (dw_dgrad_s2_tile_kernel, round 6; dy window in
    LDS, wave-uniform row parity) against the per-pixel kernel (HISEG_DW_DGRAD_TILE=0) and float64 autograd of the
    same bf16 operands -- the B0 student's four stride-2 layers at 640 x 640 plus ragged tiles, odd sizes and partial
    channel groups; written over and accumulated onto a bf16 buffer."""
    from hiseg import _lib as L
    from hiseg.ops import Act, hdtype
    N, C, H, W, k = case
    g = torch.Generator(device=DEV).manual_seed(321)
    Ho, Wo = (H + 2 * (k // 2) - k) // 2 + 1, (W + 2 * (k // 2) - k) // 2 + 1
    dy = torch.randn(N, C, Ho, Wo, device=DEV, generator=g).bfloat16()
    w = torch.randn(C, k * k, device=DEV, generator=g) * 0.3
    prev = torch.randn(N, C, H, W, device=DEV, generator=g).bfloat16()
    dya = Act.from_nchw(dy.float(), torch.bfloat16)
    lib = L.lib()
    out = {}
    for tiled in ("1", "0"):
        monkeypatch.setenv("HISEG_DW_DGRAD_TILE", tiled)
        for acc in (0, 1):
            gx = Act.from_nchw(prev.float(), torch.bfloat16)
            L.check(lib.hiseg_dw_bwd_data(hdtype(torch.bfloat16), dya.ptr(), N, H, W, C, k, 2, w.data_ptr(), Ho, Wo,
                                          gx.ptr(), acc, L.stream_ptr()), "dw_bwd_data")
            out[tiled, acc] = gx.to_nchw().float()
    x64 = torch.zeros(N, C, H, W, dtype=torch.float64, device=DEV, requires_grad=True)
    y = F.conv2d(x64, w.double().reshape(C, 1, k, k), stride=2, padding=k // 2, groups=C)
    y.backward(dy.double())
    ref = x64.grad
    for acc in (0, 1):
        r = ref + (prev.double() if acc else 0)
        t, p = out["1", acc].double(), out["0", acc].double()
        scale = r.abs().max().item()
        # bf16 output rounding: within one bf16 ulp of the f64 value, and the two kernels within one ulp of each other
        assert ((t - r).abs() <= r.abs() * 2 ** -8 + 1e-6 * scale).all(), acc
        assert ((t - p).abs() <= p.abs() * 2 ** -7 + 1e-6 * scale).all(), acc

"""Every conv form the automatic kernel choice can route to the persistent pointwise kernel (conv_pw.hip) either
runs there or falls back -- it is never silently skipped.  Round 4 found the ConvTranspose 2x2/s2 GEMM of the
B1 / B7 EnhancedUNet decoders (144 -> 72, 192 -> 96: 5 / 6 k-steps of 32 channels) accepted by the pointwise plan,
whose launcher then declined the form without launching anything, so the output kept whatever the allocator left
there (hierarchical_segmentation_unet.py:277-417 upconvs).  The outputs here start as NaN: a form that writes
nothing fails loudly.  Bar: the automatic choice equals the generic kernel (variant -1) bit for bit."""
import ctypes

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("cin,cout", [(144, 72), (192, 96), (288, 144), (256, 128), (128, 64), (72, 36), (96, 48),
                                      (160, 80), (64, 32)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_conv_transpose_auto_choice_writes_every_output(cin, cout, dt):
    from hiseg import _lib as L
    from hiseg import train_engine as TE
    from hiseg.ops import Act
    torch.manual_seed(1)
    N, H, W = 2, 12, 10
    conv = nn.ConvTranspose2d(cin, cout, 2, stride=2).to(DEV)
    S = TE.TrainState(nn.Sequential(conv), dt, torch.device(DEV))
    p = S.conv(conv, convT=True)
    x = Act.new(N, H, W, cin, dt, torch.device(DEV))
    x.t.view(N * H * W, x.cstride)[:, :cin].copy_(torch.randn(N * H * W, cin, device=DEV).to(dt))
    outs = {}
    for v in (-1, 0):
        out = Act(torch.full((N * 2 * H * 2 * W * cout,), float("nan"), dtype=dt, device=DEV), N, 2 * H, 2 * W,
                  cout, cout, 0)
        d = TE._desc(S, p, x, None, out)
        assert L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), v, None) == 0, L.lib().hiseg_last_error_string()
        torch.cuda.synchronize()
        outs[v] = out.t.view(N, 2 * H, 2 * W, cout).permute(0, 3, 1, 2).clone()
    assert torch.isfinite(outs[0].float()).all(), "the automatic choice left outputs unwritten"
    assert torch.equal(outs[0], outs[-1])
    xin = x.t.view(N, H, W, x.cstride)[..., :cin].permute(0, 3, 1, 2).float()
    ref = F.conv_transpose2d(xin, conv.weight.to(dt).float(), conv.bias.float(), stride=2)
    tol = 1e-2 if dt == torch.bfloat16 else 1e-5
    assert ((outs[0].float() - ref).abs().max() / ref.abs().max()).item() < tol


@pytest.mark.parametrize("cin", [40, 72, 144, 160, 192, 224, 256])
@pytest.mark.parametrize("form", ["residual", "mul", "plain"])
def test_pointwise_forms_auto_choice_writes_every_output(cin, form):
    """1x1 layers with 256-multiple columns and a residual / mul / plain epilogue at every k-step count."""
    from hiseg import ops
    dt = torch.bfloat16
    N, H, W, cout = 2, 9, 14, 256
    g = torch.Generator(device=DEV).manual_seed(7)
    x = ops.Act.from_nchw(torch.randn(N, cin, H, W, device=DEV, generator=g), dt)
    w = torch.randn(cout, cin, 1, 1, device=DEV, generator=g) / cin ** 0.5
    act = 2 if form == "mul" else 1   # sigmoid x mul (fg_gate), ReLU otherwise
    p = ops.pack_conv(w, torch.randn(cout, device=DEV, generator=g) * 0.1, None, act, dt, DEV, pad=0)
    X = ops.Act.from_nchw(torch.randn(N, cout, H, W, device=DEV, generator=g), dt)
    kw = {"residual": X} if form == "residual" else {"mul": X} if form == "mul" else {}
    outs = {}
    for v in (-1, 0):
        out = ops.Act.new(N, H, W, cout, dt, torch.device(DEV))
        out.t.fill_(float("nan"))
        outs[v] = ops.conv2d(p, x, out=out, variant=v, **kw).t.clone()
        torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all(), "the automatic choice left outputs unwritten"
    assert torch.equal(outs[0], outs[-1])

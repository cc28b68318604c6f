"""HIP path (libhiseg through the C ABI) against the oracle and the reference's golden vectors.

Tolerances: f32 compute — the north-star bar of 1e-4 (relative to the output's magnitude);
bf16 compute — 8-bit mantissa storage of every activation over ~70 layers: checked with a
relative bound plus agreement of the exported instance masks (argmax == 1).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import filler
from helpers import b0_kwargs, hiseg_kwargs, load, max_abs

pytestmark = pytest.mark.gpu

DEV = "cuda"
F32_TOL = 1e-4


def _rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1.0)).item()


# ------------------------------------------------------------------------------------------ RoIAlign
def test_roi_align_kernel_matches_reference_golden():
    from hiseg import DynamicRoIAlign
    g = load("roi_align")
    feat, rois = torch.from_numpy(g["feat"]).to(DEV), torch.from_numpy(g["rois"]).to(DEV)
    for i in range(5):
        oh, ow, sh, sw, al = g[f"c{i}_meta"]
        m = DynamicRoIAlign((float(sh), float(sw)), aligned=bool(al))
        out = m(feat, rois, int(oh), int(ow))
        assert max_abs(out.cpu(), g[f"c{i}_out"]) < 1e-5, i
    m = DynamicRoIAlign(20, aligned=True)
    out = m(torch.from_numpy(g["feat2"]).to(DEV), torch.from_numpy(g["rois2"]).to(DEV), 6, 4)
    assert max_abs(out.cpu(), g["out2"]) < 1e-5


def test_roi_align_nhwc_affine_bf16_and_edge_cases():
    from hiseg import ops
    from oracle.roi_align import roi_align as roi_np
    u = torch.from_numpy(filler.normal(3, (2, 1, 40, 56))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(4, 2, 5)).to(DEV)
    rois = torch.cat([rois, torch.tensor([[1, 0.0, 0.0, 1.0, 1.0], [0, 0.3, 0.3, 0.3, 0.3]], device=DEV)])
    w, b = torch.tensor([0.7, -1.3], device=DEV), torch.tensor([0.1, 0.2], device=DEV)
    for dt in (torch.float32, torch.bfloat16):
        a = ops.Act.new(rois.shape[0], 16, 12, 2, dt, DEV, zero=False)
        a.t.fill_(float("nan"))
        ops.roi_align(u, rois, 16, 12, 40, 56, True, out=a, aff_w=w, aff_b=b, zero_to=a.cstride)
        got = a.to_nchw().cpu()
        two = (w.view(1, 2, 1, 1) * u + b.view(1, 2, 1, 1)).cpu().numpy()
        ref = roi_np(two, rois.cpu().numpy(), 16, 12, 40, 56, True)
        tol = 1e-5 if dt == torch.float32 else 2e-2
        assert max_abs(got, ref) < tol * max(1, np.abs(ref).max())
        pads = a.t.view(-1, a.cstride)[:, 2:].float()
        assert torch.all(pads == 0)
    # empty ROI list is a no-op
    a = ops.Act.new(0, 4, 4, 2, torch.float32, DEV)
    ops.roi_align(u, torch.zeros(0, 5, device=DEV), 4, 4, 40, 56, True, out=a, zero_to=a.cstride)


# ------------------------------------------------------------------------------------------ conv kernel
def _conv_ref(x, w, b, stride, pad, act, res=None, mul=None):
    y = F.conv2d(x.double(), w.double(), None if b is None else b.double(), stride=stride, padding=pad)
    if res is not None:
        y = y + res.double()
    if act == 1:
        y = F.relu(y)
    elif act == 2:
        y = torch.sigmoid(y)
    elif act == 3:
        y = F.silu(y)
    if mul is not None:
        y = y * mul.double()
    return y.float()


CONV_CASES = [
    # N, Cin, Cout, H, W, k, stride, act
    (2, 64, 64, 20, 18, 3, 1, 1), (2, 256, 256, 16, 12, 3, 1, 1), (3, 3, 64, 17, 13, 3, 1, 1),
    (2, 128, 32, 15, 9, 3, 1, 2), (2, 32, 2, 15, 9, 1, 1, 0), (2, 24, 40, 31, 33, 3, 2, 3),
    (1, 258, 256, 8, 6, 1, 1, 0), (2, 16, 96, 11, 7, 1, 1, 3), (1, 16, 1, 12, 20, 3, 1, 0),
    (2, 96, 112, 9, 11, 1, 1, 0), (2, 40, 240, 6, 7, 3, 1, 3), (2, 200, 672, 5, 4, 1, 1, 1),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_igemm_single_source(case, dt):
    from hiseg import ops
    N, Cin, Cout, H, W, k, s, act = case
    torch.manual_seed(hash(case) % 1000)
    x = torch.randn(N, Cin, H, W, device=DEV)
    w = torch.randn(Cout, Cin, k, k, device=DEV) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, device=DEV) * 0.1
    p = ops.pack_conv(w, b, None, act, dt, DEV, stride=s, pad=k // 2)
    y = ops.conv2d(p, ops.Act.from_nchw(x, dt)).to_nchw().cpu()
    ref = _conv_ref(x.to(dt).float().cpu(), w.to(dt).float().cpu(), b.cpu(), s, k // 2, act)
    tol = 2e-5 if dt == torch.float32 else 1e-2
    assert _rel(y, ref) < tol


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_igemm_fused_epilogue_two_sources_upsample(dt):
    """split K over two loader sources, src A upsampled x2 (smp decoder), residual, mul, out2, f32 out."""
    from hiseg import ops
    torch.manual_seed(1)
    N, Ca, Cb, H, W, Cout = 2, 32, 24, 12, 10, 48
    xa = torch.randn(N, Ca, H // 2, W // 2, device=DEV)
    xb = torch.randn(N, Cb, H, W, device=DEV)
    res = torch.randn(N, Cout, H, W, device=DEV)
    mul = torch.rand(N, Cout, H, W, device=DEV)
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV) / ((Ca + Cb) * 9) ** 0.5
    bn = torch.nn.BatchNorm2d(Cout).to(DEV).eval()
    filler.fill_module(bn)
    p = ops.pack_conv(w, None, bn, 1, dt, DEV, pad=1, split=(Ca, Cb))
    A, B = ops.Act.from_nchw(xa, dt), ops.Act.from_nchw(xb, dt)
    R, M = ops.Act.from_nchw(res, dt), ops.Act.from_nchw(mul, dt)
    out2 = ops.Act.new(N, H, W, Cout, dt, DEV)
    y = ops.conv2d(p, A, B, a_up=2, residual=R, mul=M, out2=out2, out_dtype=torch.float32)
    cat = torch.cat([F.interpolate(xa.to(dt).float(), scale_factor=2, mode="nearest"), xb.to(dt).float()], 1)
    z = F.conv2d(cat.double(), w.to(dt).double(), padding=1)
    z = F.batch_norm(z, bn.running_mean.double(), bn.running_var.double(), bn.weight.double(), bn.bias.double(),
                     False, 0.0, bn.eps)
    ref = (F.relu(z + res.to(dt).double()) * mul.to(dt).double()).float().cpu()
    tol = 2e-5 if dt == torch.float32 else 1e-2
    assert _rel(y.to_nchw().cpu(), ref) < tol
    assert _rel(out2.to_nchw().cpu(), ref) < tol


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_transpose_and_in_scale(dt):
    from hiseg import ops
    torch.manual_seed(2)
    x = torch.randn(3, 64, 7, 5, device=DEV)
    w = torch.randn(64, 32, 2, 2, device=DEV) / 8
    b = torch.randn(32, device=DEV) * 0.1
    y = ops.conv2d(ops.pack_convT2x2(w, b, None, 1, dt, DEV), ops.Act.from_nchw(x, dt)).to_nchw().cpu()
    ref = F.relu(F.conv_transpose2d(x.to(dt).double(), w.to(dt).double(), b.double(), stride=2)).float().cpu()
    assert _rel(y, ref) < (2e-5 if dt == torch.float32 else 1e-2)
    g = torch.rand(3, 64, device=DEV)
    w1 = torch.randn(40, 64, 1, 1, device=DEV) / 8
    y = ops.conv2d(ops.pack_conv(w1, None, None, 0, dt, DEV), ops.Act.from_nchw(x, dt), in_scale=g).to_nchw().cpu()
    xs = (x.to(dt).float() * g[:, :, None, None])
    if dt == torch.bfloat16:
        xs = xs.to(dt).float()
    ref = F.conv2d(xs.double(), w1.to(dt).double()).float().cpu()
    assert _rel(y, ref) < (2e-5 if dt == torch.float32 else 1e-2)


# Every tap-major bf16 kernel variant must reproduce the generic kernel bit for bit: same K order per
# accumulator, same fp32 epilogue.  name: (N, Ca, Cb, Cout, H, W, k, convT, residual, mul, out2)
VARIANT_CASES = {
    "3x3_256_res_mul_out2": (3, 256, 0, 256, 13, 11, 3, False, True, True, True),
    "3x3_128+128": (2, 128, 128, 128, 9, 7, 3, False, False, False, False),
    "3x3_64_ragged": (3, 64, 0, 64, 7, 5, 3, False, True, False, False),
    "1x1_256_cout120": (2, 256, 0, 120, 10, 9, 1, False, True, False, False),
    "3x3_128_cout250": (2, 128, 0, 250, 9, 8, 3, False, True, False, True),
    "convT_128_to_64": (2, 128, 0, 64, 6, 5, 1, True, False, False, False),
    "convT_256_to_128_res": (2, 256, 0, 128, 5, 7, 1, True, True, False, False),
    "1x1_96_to_112_overhang": (2, 96, 0, 112, 9, 11, 1, False, True, False, False),
    "3x3_40_to_240_overhang": (2, 40, 0, 240, 6, 7, 3, False, False, True, True),
    "1x1_256+8_combiner_tail": (2, 256, 8, 256, 9, 7, 1, False, True, False, True),
    "1x1_128+40_tail_cout64": (2, 128, 40, 64, 5, 13, 1, False, False, True, False),
    # the wide-tile kernel's classes (variants 70 / 72): ragged pixel tiles, two sources, Cout 128 / 256
    "3x3_256_res_ragged": (3, 256, 0, 256, 13, 11, 3, False, True, False, False),
    "3x3_128+128_to_256": (2, 128, 128, 256, 9, 7, 3, False, False, False, False),
    "1x1_256_to_128_res": (2, 256, 0, 128, 10, 9, 1, False, True, False, False),
    "3x3_256_smp_decoder0_30x40": (2, 256, 0, 256, 30, 40, 3, False, False, False, False),
    # the persistent pointwise kernel's classes (variant 90): 4 / 8 / 9 k-steps, ConvTranspose column tiles
    "1x1_256_to_256_res_ragged": (3, 256, 0, 256, 13, 11, 1, False, True, False, False),
    "1x1_128_to_256": (2, 128, 0, 256, 9, 7, 1, False, False, False, False),
    "1x1_256+8_combiner": (2, 256, 8, 256, 9, 7, 1, False, False, False, False),
    "convT_256_to_128": (2, 256, 0, 128, 5, 7, 1, True, False, False, False),
}


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_conv_kernel_variants_bit_identical(name):
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, k, convT, res, mul, o2 = VARIANT_CASES[name]
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(7)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    if convT:
        w = torch.randn(Ca, Cout, 2, 2, device=DEV, generator=g) / Ca ** 0.5
        p = ops.pack_convT2x2(w, torch.randn(Cout, device=DEV, generator=g), None, 1, dt, DEV)
        oH, oW = 2 * H, 2 * W
    else:
        w = torch.randn(Cout, Ca + Cb, k, k, device=DEV, generator=g) / ((Ca + Cb) * k * k) ** 0.5
        bn = torch.nn.BatchNorm2d(Cout).to(DEV).eval()
        filler.fill_module(bn)
        p = ops.pack_conv(w, None, bn, 1, dt, DEV, pad=k // 2, split=(Ca, Cb) if Cb else None)
        oH, oW = H, W
    R = ops.Act.from_nchw(torch.randn(N, Cout, oH, oW, device=DEV, generator=g), dt) if res else None
    M = ops.Act.from_nchw(torch.rand(N, Cout, oH, oW, device=DEV, generator=g), dt) if mul else None
    outs = {}
    # the automatic choice (variant 0) may take the channel-major halo kernel: checked within bf16 rounding by
    # test_conv_halo_wide_within_bf16 / test_conv_automatic_choice_within_bf16
    for v in (-1, 1, 2, 3, 4, 5, 6, 7, 8, 61, 62, 66, 67, 68, 69, 70, 71, 72, 90):
        o2a = ops.Act.new(N, oH, oW, Cout, dt, DEV) if o2 else None
        y = ops.conv2d(p, xa, xb, residual=R, mul=M, out2=o2a, variant=v)
        torch.cuda.synchronize()
        outs[v] = (y.t.clone(), None if o2a is None else o2a.t.clone())
    ref, ref2 = outs[-1]
    assert torch.isfinite(ref.float()).all()
    for v, (y, y2) in outs.items():
        assert torch.equal(y, ref), f"variant {v} differs from the generic kernel"
        if o2:
            assert torch.equal(y2, ref2), f"variant {v} out2 differs"


@pytest.mark.parametrize("act", [0, 2])
@pytest.mark.parametrize("shape", [(3, 128, 256, 13, 11), (2, 256, 256, 64, 48)])
def test_conv_pointwise_gate_mul_bit_identical(shape, act):
    """The fg_gate form (refinement.py:255-268: 1x1 conv, sigmoid, times the shared features) on the persistent
    pointwise kernel (variant 90) vs the generic kernel, bit for bit."""
    from hiseg import ops
    N, Cin, Cout, H, W = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(5)
    x = ops.Act.from_nchw(torch.randn(N, Cin, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Cin, 1, 1, device=DEV, generator=g) / Cin ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, act, dt, DEV, pad=0)
    m = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt)
    ref = ops.conv2d(p, x, mul=m, variant=-1).t.clone()
    y = ops.conv2d(p, x, mul=m, variant=90).t.clone()
    auto = ops.conv2d(p, x, mul=m, variant=0).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(ref.float()).all()
    assert torch.equal(y, ref) and torch.equal(auto, ref)


# Narrow / ragged layers (full-resolution decoder, EfficientNet projections) on the halo-tiled
# direct kernel (variants 50-58) vs the generic kernel, bit for bit.
# name: (N, Ca, Cb, Cout, H, W, k, a_up, in_scale, residual, mul+out2, f32 out)
NARROW_CASES = {
    "up2_32_to_16": (2, 32, 0, 16, 10, 70, 3, 2, False, False, False, False),
    "16_to_16_res": (2, 16, 0, 16, 9, 66, 3, 1, False, True, False, False),
    "16_to_1_f32": (2, 16, 0, 1, 11, 40, 3, 1, False, False, False, True),
    "up2_64+32_to_32": (2, 64, 32, 32, 12, 20, 3, 2, False, False, True, False),
    "1x1_24_to_144_ins_res": (3, 24, 0, 144, 7, 9, 1, 1, True, True, False, False),
    "1x1_16_to_96": (2, 16, 0, 96, 5, 130, 1, 1, False, False, False, False),
    "3x3_8_to_64": (2, 8, 0, 64, 9, 13, 3, 1, False, False, False, False),
    "3x3_64+8_to_64_ins": (2, 64, 8, 64, 6, 7, 3, 1, True, False, True, False),
}


@pytest.mark.parametrize("name", list(NARROW_CASES))
def test_conv_small_kernel_bit_identical(name):
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, k, up, ins, res, mul, f32o = NARROW_CASES[name]
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(11)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H // up, W // up, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, k, k, device=DEV, generator=g) / ((Ca + Cb) * k * k) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=k // 2,
                      split=(Ca, Cb) if Cb else None)
    gate = torch.rand(N, p.ca, device=DEV, generator=g) if ins else None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    M = ops.Act.from_nchw(torch.rand(N, Cout, H, W, device=DEV, generator=g), dt) if mul else None
    outs = {}
    for v in (-1, 0, 50, 51, 52, 54, 58):
        o2 = ops.Act.new(N, H, W, Cout, dt, DEV) if mul else None
        y = ops.conv2d(p, xa, xb, a_up=up, residual=R, mul=M, out2=o2, in_scale=gate,
                       out_dtype=torch.float32 if f32o else None, variant=v)
        torch.cuda.synchronize()
        outs[v] = (y.t.clone(), None if o2 is None else o2.t.clone())
    ref, ref2 = outs[-1]
    assert torch.isfinite(ref.float()).all()
    for v, (y, y2) in outs.items():
        assert torch.equal(y, ref), f"variant {v} differs from the generic kernel"
        if mul:
            assert torch.equal(y2, ref2), f"variant {v} out2 differs"


# The full-image UNet's narrow decoder layers on the row-streaming kernel (conv_rows.hip, variant 98 and the
# automatic choice) vs the generic kernel, bit for bit: smp DecoderBlock conv1 over up(x) ++ skip (B0/B1 stem
# skip 32, B7 64), conv2, the last block's 32 -> 16 / 16 -> 16 and the 16 -> 1 f32 segmentation head; heights
# spanning several workgroups' row runs (segments crossing strips and images), ragged strip widths.
# name: (N, Ca, Cb, Cout, H, W, a_up, f32 out)
ROWS_CASES = {
    "up2_64+32_to_32": (2, 64, 32, 32, 96, 200, 2, False),
    "up2_64+64_to_32_b7": (2, 64, 64, 32, 50, 70, 2, False),
    "32_to_32": (3, 32, 0, 32, 61, 130, 1, False),
    "up2_32_to_16": (2, 32, 0, 16, 90, 300, 2, False),
    "16_to_16": (2, 16, 0, 16, 77, 260, 1, False),
    "16_to_1_f32": (2, 16, 0, 1, 64, 150, 1, True),
    "16_to_16_tiny": (1, 16, 0, 16, 3, 5, 1, False),
}


@pytest.mark.parametrize("name", list(ROWS_CASES))
def test_conv_rows_bit_identical(name):
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, up, f32o = ROWS_CASES[name]
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(19)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H // up, W // up, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 0 if f32o else 1, dt, DEV, pad=1,
                      split=(Ca, Cb) if Cb else None)
    outs = {}
    for v in (-1, 50, 98, 0):
        y = ops.conv2d(p, xa, xb, a_up=up, out_dtype=torch.float32 if f32o else None, variant=v)
        torch.cuda.synchronize()
        outs[v] = y.t.clone()
    assert torch.isfinite(outs[-1].float()).all()
    for v in (50, 98, 0):
        assert torch.equal(outs[v], outs[-1]), f"variant {v} differs from the generic kernel"


@pytest.mark.parametrize("shape", [(2, 3, 32, 20, 150), (3, 16, 24, 9, 70), (1, 8, 64, 33, 17)])
def test_conv_small_stride2_bit_identical(shape):
    """The EfficientNet stem form (3x3 / stride 2 / pad 1, timm conv_stem + bn1 + SiLU) on the halo-tiled
    direct kernel's stride-2 configuration (automatic choice) vs the generic kernel, bit for bit; odd sizes."""
    from hiseg import ops
    N, Cin, Cout, H, W = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(17)
    x = ops.Act.from_nchw(torch.randn(N, Cin, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (Cin * 9) ** 0.5
    bn = torch.nn.BatchNorm2d(Cout).to(DEV).eval()
    filler.fill_module(bn)
    p = ops.pack_conv(w, None, bn, 3, dt, DEV, stride=2, pad=1)
    ref = ops.conv2d(p, x, variant=-1).t.clone()
    auto = ops.conv2d(p, x, variant=0).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(ref.float()).all()
    assert torch.equal(auto, ref)


# The EfficientNet encoder's 1x1 layers and the head's narrow 1x1 layers on the persistent pointwise kernel
# (variant 90 and the automatic choice) vs the generic kernel, bit for bit: SiLU expansions (channel tails of
# 24 / 40 input channels, ragged 256-column tiles at 672 / 1152, run-time k-step counts), SE-gated projections
# with and without the skip (narrow column tiles of 16..80), the head's 8->64 / 64->128 forms.
# name: (N, Ca, Cout, H, W, act, in_scale, residual)
PW_EFF_CASES = {
    "exp_16_96_silu": (2, 16, 96, 9, 70, 3, False, False),
    "exp_24_144_silu": (3, 24, 144, 7, 9, 3, False, False),
    "exp_40_240_silu": (2, 40, 240, 11, 13, 3, False, False),
    "exp_112_672_silu": (2, 112, 672, 5, 7, 3, False, False),
    "exp_192_1152_silu": (2, 192, 1152, 3, 5, 3, False, False),
    "proj_144_24_ins_res": (3, 144, 24, 7, 9, 0, True, True),
    "proj_96_24_ins": (2, 96, 24, 9, 11, 0, True, False),
    "proj_240_40_ins_res": (2, 240, 40, 6, 10, 0, True, True),
    "proj_240_80_ins": (2, 240, 80, 5, 6, 0, True, False),
    "ds_32_16_ins": (2, 32, 16, 9, 70, 0, True, False),
    "head_8_64_relu": (2, 8, 64, 6, 9, 1, False, False),
    "head_64_128_relu_res": (2, 64, 128, 9, 7, 1, False, True),
    # 9-10 k-steps at narrow tiles (round 3): the B7 encoder's 288-channel SE-gated projections
    "proj_288_48_ins_res": (2, 288, 48, 9, 13, 0, True, True),
    "proj_320_32_ins": (3, 320, 32, 7, 9, 0, True, False),
    "proj_264_16_ins_tail": (2, 264, 16, 5, 5, 0, True, False),
}


@pytest.mark.parametrize("name", list(PW_EFF_CASES))
def test_conv_pointwise_efficientnet_bit_identical(name):
    from hiseg import ops
    N, Ca, Cout, H, W, act, ins, res = PW_EFF_CASES[name]
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(13)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Ca, 1, 1, device=DEV, generator=g) / Ca ** 0.5
    bn = torch.nn.BatchNorm2d(Cout).to(DEV).eval()
    filler.fill_module(bn)
    p = ops.pack_conv(w, None, bn, act, dt, DEV, pad=0)
    gate = torch.rand(N, p.ca, device=DEV, generator=g) if ins else None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    outs = {}
    for v in (-1, 0, 90):
        y = ops.conv2d(p, xa, residual=R, in_scale=gate, variant=v)
        torch.cuda.synchronize()
        outs[v] = y.t.clone()
    assert torch.isfinite(outs[-1].float()).all()
    for v in (0, 90):
        assert torch.equal(outs[v], outs[-1]), f"variant {v} differs from the generic kernel"


@pytest.mark.parametrize("Ca,Cout,N", [(240, 40, 80), (288, 48, 60), (96, 24, 200)])
def test_conv_gated_pointwise_batch_invariant_above_gate_bound(Ca, Cout, N):
    """the pointwise kernel stages an SE-gated layer's gate [N][Ca] in 64 KiB of LDS, so its plan depended
    on the batch (N * Ca * 4 > 64 KiB declined it).  conv2d_impl now runs such a layer in image ranges the gate fits
    (conv_pw_gate_images): a batch above the bound gives every image the bits it gets alone or in a small batch."""
    from hiseg import ops
    dt = torch.bfloat16
    H, W = 10, 12
    assert N * Ca * 4 > 64 * 1024
    g = torch.Generator(device=DEV).manual_seed(23)
    x = torch.randn(N, Ca, H, W, device=DEV, generator=g)
    w = torch.randn(Cout, Ca, 1, 1, device=DEV, generator=g) / Ca ** 0.5
    bn = torch.nn.BatchNorm2d(Cout).to(DEV).eval()
    filler.fill_module(bn)
    p = ops.pack_conv(w, None, bn, 0, dt, DEV, pad=0)
    gate = torch.rand(N, p.ca, device=DEV, generator=g)
    r = torch.randn(N, Cout, H, W, device=DEV, generator=g)
    y = ops.conv2d(p, ops.Act.from_nchw(x, dt), residual=ops.Act.from_nchw(r, dt), in_scale=gate).to_nchw()
    for lo, hi in ((0, 1), (N - 3, N), (N // 2, N // 2 + 7)):
        ys = ops.conv2d(p, ops.Act.from_nchw(x[lo:hi].contiguous(), dt), residual=ops.Act.from_nchw(r[lo:hi].contiguous(), dt),
                        in_scale=gate[lo:hi].contiguous()).to_nchw()
        torch.cuda.synchronize()
        assert torch.equal(ys, y[lo:hi]), (lo, hi)
    yg = ops.conv2d(p, ops.Act.from_nchw(x, dt), residual=ops.Act.from_nchw(r, dt), in_scale=gate, variant=-1).to_nchw()
    assert torch.equal(yg, y)


# Split-K generic kernel (round 3): small-grid, long-K 1x1 layers -- the deep SE-gated EfficientNet projections of
# the B7 teacher / B0 student in distillation (N, Ca, Cout, H, W, act, in_scale, residual)
SPLITK_CASES = {
    "b7_2304_384_ins_res": (4, 2304, 384, 20, 20, 0, True, True),
    "b7_3840_640_ins": (4, 3840, 640, 20, 20, 0, True, False),
    "b7_1344_224_ins_res": (4, 1344, 224, 40, 40, 0, True, True),
    "b0_1152_192_ins_res": (2, 1152, 192, 20, 20, 0, True, True),
    "b7_960_160_ins": (4, 960, 160, 40, 40, 0, True, False),
    "plain_1536_96_relu_ragged": (3, 1536, 96, 7, 9, 1, False, False),
}


@pytest.mark.parametrize("name", list(SPLITK_CASES))
def test_conv_splitk_within_reassociation(name):
    """The split-K generic kernel (variant 99, and the automatic choice that picks it with the workspace ops.conv2d
    supplies) against the unsplit generic kernel and a float64 reference of the same bf16 operands (the SE gate
    applied and rounded to bf16 as the loader does): f32 re-association only, so the bf16 outputs agree with the
    generic kernel's up to one rounding step, and the error against float64 is no larger than the generic kernel's
    own (+ one bf16 ulp).  Deterministic run to run."""
    from hiseg import ops
    from hiseg import _lib as L
    import ctypes
    N, Ca, Cout, H, W, act, ins, res = SPLITK_CASES[name]
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(17)
    x = torch.randn(N, Ca, H, W, device=DEV, generator=g)
    xa = ops.Act.from_nchw(x, dt)
    w = torch.randn(Cout, Ca, 1, 1, device=DEV, generator=g) / Ca ** 0.5
    bn = torch.nn.BatchNorm2d(Cout).to(DEV).eval()
    filler.fill_module(bn)
    p = ops.pack_conv(w, None, bn, act, dt, DEV, pad=0)
    gate = torch.rand(N, p.ca, device=DEV, generator=g) if ins else None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    # the library plans a split for this layer
    d = L.Conv2dDesc()
    d.dtype = d.out_dtype = 1
    d.N, d.H, d.W, d.Ho, d.Wo, d.KH, d.KW, d.stride = N, H, W, H, W, 1, 1, 1
    d.Ca, d.Cout, d.Cout_pad, d.K_pad = p.ca, p.gemm_cols, p.cout_pad, p.k_pad
    with L.raw_pointers():   # planning only, never launched
        d.srcA = d.weight = d.scale = d.shift = d.out = 1
        d.in_scale = 16 if ins else None
    assert L.lib().hiseg_conv2d_workspace_bytes(ctypes.byref(d)) > 0
    outs = {}
    for v in (-1, 99, 0, "again"):
        y = ops.conv2d(p, xa, residual=R, in_scale=gate, variant=0 if v == "again" else v)
        torch.cuda.synchronize()
        outs[v] = y.to_nchw().float()
    assert torch.equal(outs[0], outs[99]) and torch.equal(outs[0], outs["again"])
    xq = xa.to_nchw().float().double()
    if ins:
        xq = (xq.float() * gate[:, :Ca, None, None]).to(dt).double()
    wq = p.weight[:Cout, :Ca].float().double()
    z = torch.einsum("nchw,oc->nohw", xq, wq) * p.scale[:Cout].double()[:, None, None] + p.shift[:Cout].double()[:, None, None]
    if res:
        z = z + R.to_nchw().double()
    if act == 1:
        z = torch.relu(z)
    e_gen = (outs[-1].double() - z).abs().max().item()
    e_spl = (outs[99].double() - z).abs().max().item()
    ulp = z.abs().max().item() * 2.0 ** -8
    assert e_spl <= e_gen + ulp, (e_spl, e_gen, ulp)
    diff = (outs[99] - outs[-1]).abs()
    assert (diff <= outs[-1].abs() * 2.0 ** -7 + 1e-6).all()
    assert (diff == 0).float().mean().item() > 0.9


# ------------------------------------------------------------------------------------------ misc kernels
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_pointwise_kernels(dt):
    from hiseg import ops
    torch.manual_seed(3)
    x = torch.randn(2, 64, 10, 8, device=DEV)
    xq = x.to(dt).float()
    A = ops.Act.from_nchw(x, dt)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert _rel(ops.maxpool2x2(A).to_nchw().cpu(), F.max_pool2d(xq, 2).cpu()) < tol
    w7 = torch.randn(1, 2, 7, 7, device=DEV) * 0.2
    s = torch.cat([xq.mean(1, keepdim=True), xq.max(1, keepdim=True)[0]], 1)
    ref = (xq * torch.sigmoid(F.conv2d(s, w7, padding=3))).cpu()
    assert _rel(ops.attn_spatial(A, w7.contiguous()).to_nchw().cpu(), ref) < tol * 2
    w1, w2 = torch.randn(8, 64, device=DEV) * 0.2, torch.randn(64, 8, device=DEV) * 0.2
    b1, b2 = torch.randn(8, device=DEV) * 0.1, torch.randn(64, device=DEV) * 0.1
    for act, bias in ((1, False), (3, True)):
        gate = ops.se_gate(A, w1, b1 if bias else None, w2, b2 if bias else None, act)
        m = xq.mean((2, 3))
        h = m @ w1.t() + (b1 if bias else 0)
        h = F.relu(h) if act == 1 else F.silu(h)
        ref_g = torch.sigmoid(h @ w2.t() + (b2 if bias else 0))
        assert _rel(gate.cpu(), ref_g.cpu()) < 1e-4
        out = ops.channel_scale(A, gate).to_nchw().cpu()
        assert _rel(out, (xq * gate[:, :, None, None]).cpu()) < tol
    for k, stride in ((3, 1), (5, 2), (3, 2)):
        wd = torch.randn(64, 1, k, k, device=DEV) * 0.3
        sc, sh = torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV) * 0.1
        out = ops.dwconv(A, wd.view(64, k * k).t().contiguous(), sc, sh, k, stride, 3).to_nchw().cpu()
        ref = F.silu(F.conv2d(xq, wd, stride=stride, padding=k // 2, groups=64) * sc[:, None, None] + sh[:, None, None])
        assert _rel(out, ref.cpu()) < tol * 2


def test_input_norm_device_flag():
    from hiseg import ops
    mean = torch.tensor([0.485, 0.456, 0.406], device=DEV)
    std = torch.tensor([0.229, 0.224, 0.225], device=DEV)
    for scale in (1.0, 255.0):
        img = torch.rand(2, 3, 8, 6, device=DEV) * scale
        a = ops.input_norm(img, mean, std, torch.float32)
        x = img / 255.0 if img.max() > 1 else img
        ref = (x - mean.view(1, 3, 1, 1)) / std.view(1, 3, 1, 1)
        assert max_abs(a.to_nchw().cpu(), ref.cpu()) < 1e-5
        assert torch.all(a.t.view(-1, a.cstride)[:, 3:] == 0)


def test_export_mask_kernels_match_oracle():
    from hiseg import ops
    from oracle import rgb_model as O
    torch.manual_seed(4)
    logits = torch.randn(5, 3, 16, 12, device=DEV) * 3
    for dil in (0, 1, 2):
        got = ops.instance_masks(logits, dil).cpu()
        ref = O.instance_masks(logits.cpu(), dil)
        assert torch.equal(got, ref), dil
    u = torch.randn(2, 1, 9, 7, device=DEV) * 4
    w, b = torch.tensor([1.0, -1.0], device=DEV), torch.tensor([0.0, 0.0], device=DEV)
    sd = {"pretrained_unet.output_conv.weight": w.view(2, 1, 1, 1).cpu(), "pretrained_unet.output_conv.bias": b.cpu()}
    assert max_abs(ops.binary_masks(u, w, b).cpu(), O.binary_masks(sd, u.cpu())) < 1e-6


# ------------------------------------------------------------------------------------------ blocks / head / model
def _filled(m):
    return filler.fill_module(m).eval()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_residual_block_and_enhanced_unet_match_golden(dt):
    import hiseg
    from hiseg.layers import EnhancedUNet, ResidualBlock
    g = load("blocks")
    blk = hiseg.set_compute_dtype(_filled(ResidualBlock(64, "batchnorm", 8, "relu")).to(DEV), dt)
    y = blk(torch.from_numpy(g["res_x"]).to(DEV)).cpu()
    tol = F32_TOL if dt == torch.float32 else 3e-2
    assert _rel(y, g["res_y"]) < tol
    un = hiseg.set_compute_dtype(_filled(EnhancedUNet(256, 64, 3, "batchnorm", 8, "relu")).to(DEV), dt)
    y = un(torch.from_numpy(g["unet_x"]).to(DEV)).cpu()
    assert _rel(y, g["unet_y"]) < (F32_TOL if dt == torch.float32 else 5e-2)


def _model(dt):
    import hiseg
    from hiseg import create_rgb_hierarchical_model
    m = _filled(create_rgb_hierarchical_model(**hiseg_kwargs(b0_kwargs()))).to(DEV)
    return hiseg.set_compute_dtype(m, dt)


def test_head_matches_golden_f32():
    import hiseg
    from hiseg.layers import RefinedHierarchicalSegmentationHead
    kw = b0_kwargs()
    g = load("head_b0")
    head = _filled(RefinedHierarchicalSegmentationHead(
        256, 256, 3, tuple(kw["mask_size"]), use_attention_module=True, use_contour_detection=True,
        use_distance_transform=True, normalization_type="batchnorm", activation_function="relu",
        hierarchical_base_channels=kw["hierarchical_base_channels"], hierarchical_depth=kw["hierarchical_depth"])).to(DEV)
    hiseg.set_compute_dtype(head, torch.float32)
    x = torch.from_numpy(filler.normal(31, (2, 256, 64, 48))).to(DEV)
    logits, aux = head(x)
    assert _rel(logits.cpu(), g["logits"]) < F32_TOL
    for k in ("bg_fg_logits", "bg_fg_logits_low", "target_nontarget_logits", "contours", "distance_mask",
              "distance_map"):
        assert _rel(aux[k].cpu(), g["aux_" + k]) < F32_TOL, k
    for k in ("fg_attention", "shared_features"):
        assert _rel(aux[k].mean(dim=(0, 2, 3)).cpu(), g[f"aux_{k}__chmean"]) < F32_TOL, k


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_model_matches_reference_golden(dt):
    from hiseg import engine
    g = load("model_b0")
    model = _model(dt)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 96, 128
    images, rois, u = (torch.from_numpy(g[k]).to(DEV) for k in ("images", "rois", "u"))
    logits, aux = engine.rgb_model_forward(model, images, rois, "full", unet_logit_override=u)
    ref = torch.from_numpy(g["logits"])
    if dt == torch.float32:
        assert _rel(logits.cpu(), ref) < F32_TOL
        for k in ("bg_fg_logits", "target_nontarget_logits", "full_image_logits", "roi_features", "roi_patches",
                  "contours", "distance_map", "distance_mask", "bg_fg_logits_low"):
            assert _rel(aux[k].cpu(), g["aux_" + k]) < F32_TOL, k
    else:
        assert _rel(logits.cpu(), ref) < 0.1
        agree = (logits.argmax(1) == ref.to(DEV).argmax(1)).float().mean().item()
        assert agree > 0.97, agree
    # training-semantics scale (640 scalar) on 640x640 inputs
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h = m.spatial_scale_w = 640.0
    images = torch.from_numpy(filler.uniform(43, (1, 3, 640, 640))).to(DEV)
    u = torch.from_numpy(filler.normal(44, (1, 1, 640, 640)) * 2.0).to(DEV)
    logits, _ = engine.rgb_model_forward(model, images, torch.from_numpy(g["rois640"]).to(DEV), "none",
                                         unet_logit_override=u)
    tol = F32_TOL if dt == torch.float32 else 0.1
    assert _rel(logits.cpu(), g["logits640"]) < tol


def test_full_pipeline_with_effunet_matches_oracle():
    """Whole path incl. the EfficientNet-B0 UNet (parity of that sub-network vs the restated oracle only)."""
    from oracle import rgb_model as O
    from hiseg import RGBHierarchicalExportWrapper
    model = _model(torch.float32)
    sd = O.np_state(model)
    cfg = O.cfg_from_kwargs(b0_kwargs())
    images = torch.from_numpy(filler.uniform(51, (2, 3, 96, 128)))
    rois = torch.from_numpy(filler.box_rois(52, 2, 2))
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 96, 128
    logits, aux = model(images.to(DEV), rois.to(DEV))
    with torch.no_grad():
        ref_logits, ref_aux, ref_u = O.rgb_model(sd, images, rois, cfg, (96, 128), "b0")
    assert _rel(aux["full_image_logits"].cpu(), ref_aux["full_image_logits"]) < F32_TOL
    assert _rel(logits.cpu(), ref_logits) < F32_TOL
    wrap = RGBHierarchicalExportWrapper(model)
    inst, binary = wrap(images.to(DEV), rois.to(DEV))
    assert inst.shape == (4, 1, 128, 96) and binary.shape == (2, 1, 96, 128)
    ref_inst = O.instance_masks(ref_logits)
    assert (inst.cpu() == ref_inst).float().mean().item() > 0.999
    assert max_abs(binary.cpu(), O.binary_masks(sd, ref_u)) < 1e-4


def test_bf16_pipeline_instance_mask_agreement():
    from oracle import rgb_model as O
    from hiseg import RGBHierarchicalExportWrapper
    model = _model(torch.bfloat16)
    sd = O.np_state(model)
    cfg = O.cfg_from_kwargs(b0_kwargs())
    images = torch.from_numpy(filler.uniform(61, (2, 3, 96, 128)))
    rois = torch.from_numpy(filler.box_rois(62, 2, 2))
    inst, binary = RGBHierarchicalExportWrapper(model)(images.to(DEV), rois.to(DEV))
    with torch.no_grad():
        ref_logits, _, ref_u = O.rgb_model(sd, images, rois, cfg, (96, 128), "b0")
    agree = (inst.cpu() == O.instance_masks(ref_logits)).float().mean().item()
    assert agree > 0.97, agree
    assert max_abs(binary.cpu(), O.binary_masks(sd, ref_u)) < 0.05


@pytest.mark.parametrize("gate", [None, 0.001, 0.05])
def test_stream_pipelined_export_matches_serial(gate):
    """hiseg.StreamPipelinedExport (UNet of batch k+1 on a second stream beside the head of batch k) returns
    exactly the per-batch outputs of the serial RGBHierarchicalExportWrapper -- also with gate=True (the UNet issued
    in chunks into the windows between the head's heavy convs; thresholds here small enough that most / some of this
    small model's convs count as heavy), over 4 batches (the first learns the windows, the rest use them)."""
    import filler
    import hiseg
    from helpers import b0_kwargs, hiseg_kwargs
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(b0_kwargs()))).eval().to("cuda")
    hiseg.set_compute_dtype(m, torch.bfloat16)
    w = hiseg.RGBHierarchicalExportWrapper(m)
    batches = []
    for k in range(4):
        images = torch.from_numpy(filler.uniform(200 + k, (2, 3, 96, 128))).cuda()
        rois = torch.from_numpy(filler.box_rois(300 + k, 2, 3)).cuda()
        batches.append((images, rois))
    with torch.no_grad():
        serial = [w(i, r) for i, r in batches]
        runner = (hiseg.StreamPipelinedExport(w) if gate is None
                  else hiseg.StreamPipelinedExport(w, gate=True, gate_min_gflop=gate))
        piped = runner.run(batches)
        if gate is not None:
            assert runner._windows is not None and len(runner._windows) > 2, runner._windows
            piped2 = runner.run(batches)   # learned windows from the first call on
            for (a, b), (c, d) in zip(piped, piped2):
                assert torch.equal(a, c) and torch.equal(b, d)
    torch.cuda.synchronize()
    for (a, b), (c, d) in zip(serial, piped):
        assert torch.equal(a, c) and torch.equal(b, d)


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_conv_wide_channel_major_variant_within_bf16(name):
    """Variant 74: the wide-tile kernel with the channel-major K order (the 9 taps of a 32-channel slice back
    to back) -- the same products, another f32 summation order: within bf16 output rounding of the generic
    kernel (layers the wide kernel does not take fall back to the automatic choice)."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, k, convT, res, mul, o2 = VARIANT_CASES[name]
    if convT:
        pytest.skip("ConvTranspose layers are not wide-kernel layers")
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(8)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, k, k, device=DEV, generator=g) / ((Ca + Cb) * k * k) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=k // 2,
                      split=(Ca, Cb) if Cb else None)
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    ref = ops.conv2d(p, xa, xb, residual=R, variant=-1).to_nchw().float()
    y = ops.conv2d(p, xa, xb, residual=R, variant=74).to_nchw().float()
    assert torch.isfinite(y).all()
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 8e-3


# ------------------------------------------------------------------------------------------ whole path, C3 / C4 presets
def _preset_model(name, dt):
    import hiseg
    from helpers import configs
    kw = hiseg_kwargs(dict(configs()[name]["model_kwargs"]))
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**kw)).eval().to(DEV)
    return hiseg.set_compute_dtype(m, dt), kw


@pytest.mark.parametrize("name", ["b1", "b7"])
def test_full_pipeline_preset_matches_oracle(name):
    """C3 (B1-enhanced: ROI 80x60, mask 160x120) and C4 (B7-ultra: 128x96 / 256x192, EnhancedUNet depth 4) whole
    export path in f32 -- the EfficientNet-B1 / B7 UNet included, no injected UNet output -- against the oracle
    at the 1e-4 bar: full-image UNet logits, ROI logits, instance and binary masks."""
    from oracle import rgb_model as O
    from hiseg import RGBHierarchicalExportWrapper
    model, kw = _preset_model(name, torch.float32)
    sd = O.np_state(model)
    cfg = O.cfg_from_kwargs(kw)
    images = torch.from_numpy(filler.uniform(71, (2, 3, 96, 128)))
    rois = torch.from_numpy(filler.box_rois(72, 2, 2))
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 96, 128
    logits, aux = model(images.to(DEV), rois.to(DEV))
    with torch.no_grad():
        ref_logits, ref_aux, ref_u = O.rgb_model(sd, images, rois, cfg, (96, 128), name)
    assert logits.shape == ref_logits.shape == (4, 3) + tuple(cfg["mask_hw"])
    assert _rel(aux["full_image_logits"].cpu(), ref_aux["full_image_logits"]) < F32_TOL
    assert _rel(logits.cpu(), ref_logits) < F32_TOL
    inst, binary = RGBHierarchicalExportWrapper(model)(images.to(DEV), rois.to(DEV))
    assert (inst.cpu() == O.instance_masks(ref_logits)).float().mean().item() > 0.999
    assert max_abs(binary.cpu(), O.binary_masks(sd, ref_u)) < 1e-4


def test_c2_shape_bf16_properties_and_oracle():
    """The bench's C2 workload (32 images 480x640 x 8 ROIs, bf16): output shapes and value sets, run-to-run
    determinism, batch invariance (image 0 alone gives bit-identical masks), and image 0's 8 ROIs against the
    f32 oracle (instance-mask agreement, binary-mask error)."""
    from oracle import rgb_model as O
    from hiseg import RGBHierarchicalExportWrapper
    model, kw = _preset_model("b0", torch.bfloat16)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 480, 640
    wrap = RGBHierarchicalExportWrapper(model)
    images = torch.from_numpy(filler.uniform(81, (32, 3, 480, 640))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(82, 32, 8)).to(DEV)
    with torch.no_grad():
        inst, binary = wrap(images, rois)
        inst2, binary2 = wrap(images, rois)
        inst0, binary0 = wrap(images[:1].contiguous(), rois[:8].contiguous())
    torch.cuda.synchronize()
    assert inst.shape == (256, 1, 128, 96) and binary.shape == (32, 1, 480, 640)
    assert torch.isfinite(binary).all() and ((inst == 0) | (inst == 1)).all()
    assert binary.min().item() >= 0.0 and binary.max().item() <= 1.0
    assert 0.0 < inst.float().mean().item() < 1.0
    assert torch.equal(inst, inst2) and torch.equal(binary, binary2)
    assert torch.equal(inst0, inst[:8]) and torch.equal(binary0, binary[:1])
    sd = O.np_state(model)
    with torch.no_grad():
        ref_logits, _, ref_u = O.rgb_model(sd, images[:1].cpu(), rois[:8].cpu(), O.cfg_from_kwargs(kw), (480, 640),
                                           "b0")
    agree = (inst[:8].cpu() == O.instance_masks(ref_logits)).float().mean().item()
    assert agree > 0.97, agree
    assert max_abs(binary[:1].cpu(), O.binary_masks(sd, ref_u)) < 0.05


def test_c2_size_bf16_within_torch_bf16(monkeypatch):
    """the bf16 bar at the benchmark's own size.  One 480x640 image with 8 ROIs from the C2 ROI
    generator (bench.py synthetic_batch), B0-std in bf16 through the exported contract, against the f32 oracle; the
    same network run by torch in bf16 on the GPU sets what bf16 execution costs.  hiseg's instance masks must agree
    with the f32 oracle's at least as well as torch-bf16's do, less 0.5 points, and its ROI logits and full-image
    UNet logits must stay within 1.5x (+1e-3) of torch-bf16's relative error."""
    from oracle import rgb_model as O
    from oracle.roi_align import roi_align as roi_np
    from hiseg import RGBHierarchicalExportWrapper
    model, kw = _preset_model("b0", torch.bfloat16)
    cfg = O.cfg_from_kwargs(kw)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 480, 640
    images = torch.from_numpy(filler.uniform(1, (1, 3, 480, 640)))
    rois = torch.from_numpy(filler.box_rois(1, 1, 8))
    sd = O.np_state(model)
    with torch.no_grad():
        inst, _ = RGBHierarchicalExportWrapper(model)(images.to(DEV), rois.to(DEV))
        logits, aux = model(images.to(DEV), rois.to(DEV))
        ref_logits, ref_aux, _ = O.rgb_model(sd, images, rois, cfg, (480, 640), "b0")

        def roi_bf16(feat, r, oh, ow, sh, sw, aligned=True):
            out = roi_np(feat.float().cpu().numpy(), r.float().cpu().numpy(), oh, ow, sh, sw, aligned)
            return torch.from_numpy(out).to(feat.device, feat.dtype)

        monkeypatch.setattr(O, "roi_align", roi_bf16)
        sd16 = {k: v.to(DEV, torch.bfloat16) for k, v in sd.items()}
        t_logits, t_aux, _ = O.rgb_model(sd16, images.to(DEV, torch.bfloat16), rois.to(DEV), cfg, (480, 640), "b0")
    ref_masks = O.instance_masks(ref_logits)
    agree_h = (inst.cpu() == ref_masks).float().mean().item()
    agree_t = (O.instance_masks(t_logits.float().cpu()) == ref_masks).float().mean().item()
    e_h, e_t = _rel(logits.float().cpu(), ref_logits), _rel(t_logits.float().cpu(), ref_logits)
    u_h = _rel(aux["full_image_logits"].float().cpu(), ref_aux["full_image_logits"])
    u_t = _rel(t_aux["full_image_logits"].float().cpu(), ref_aux["full_image_logits"])
    print(f"C2-size bf16: mask agreement {agree_h:.5f} (torch-bf16 {agree_t:.5f}); logits {e_h:.2e} "
          f"(torch {e_t:.2e}); UNet logits {u_h:.2e} (torch {u_t:.2e})")
    assert agree_h >= agree_t - 0.005, (agree_h, agree_t)
    assert e_h < 1.5 * e_t + 1e-3, (e_h, e_t)
    assert u_h < 1.5 * u_t + 1e-3, (u_h, u_t)


@pytest.mark.parametrize("preset", ["b0", "b1", "b7"])
def test_bf16_logits_error_within_torch_bf16(monkeypatch, preset):
    """The bf16 inference bar, tied to PyTorch's own bf16: the same network run by torch in bf16 on the GPU
    (the oracle's functional forms with bf16 weights and activations) sets the error a bf16 execution of this
    model incurs against the f32 oracle; hiseg's bf16 path must stay within 1.5x of it (logits, full-image
    UNet logits).  All three presets: the B1 / B7 EnhancedUNets' 144 -> 72 / 192 -> 96 up-convolutions once took
    a pointwise-kernel form that was never launched (round 4), invisible to the f32 tests."""
    from oracle import rgb_model as O
    from oracle.roi_align import roi_align as roi_np
    model, kw = _preset_model(preset, torch.bfloat16)
    cfg = O.cfg_from_kwargs(kw)
    sd = O.np_state(model)
    images = torch.from_numpy(filler.uniform(91, (2, 3, 96, 128)))
    rois = torch.from_numpy(filler.box_rois(92, 2, 3))
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 96, 128
    with torch.no_grad():
        logits, aux = model(images.to(DEV), rois.to(DEV))
        ref_logits, ref_aux, _ = O.rgb_model(sd, images, rois, cfg, (96, 128), preset)

        def roi_bf16(feat, r, oh, ow, sh, sw, aligned=True):   # RoIAlign in f32 (numpy), result back in bf16
            out = roi_np(feat.float().cpu().numpy(), r.float().cpu().numpy(), oh, ow, sh, sw, aligned)
            return torch.from_numpy(out).to(feat.device, feat.dtype)

        monkeypatch.setattr(O, "roi_align", roi_bf16)
        sd16 = {k: v.to(DEV, torch.bfloat16) for k, v in sd.items()}
        t_logits, t_aux, _ = O.rgb_model(sd16, images.to(DEV, torch.bfloat16), rois.to(DEV), cfg, (96, 128), preset)
    for mine, theirs, ref in ((logits, t_logits, ref_logits),
                              (aux["full_image_logits"], t_aux["full_image_logits"], ref_aux["full_image_logits"])):
        e_h, e_t = _rel(mine.float().cpu(), ref), _rel(theirs.float().cpu(), ref)
        assert e_h < 1.5 * e_t + 1e-3, (e_h, e_t)


@pytest.mark.parametrize("dilation", [0, 1, 2])
def test_export_dilation_matches_reference_golden(dilation):
    """The exported contract with MaskDilationModule (export_hierarchical_instance_peopleseg_onnx.py:85-181) at
    dilation 0 / 1 / 2: instance masks and binary masks from the injected UNet map against the reference's own
    outputs (tests/golden/export.npz), f32 compute."""
    from hiseg import engine, ops
    g = load("export")
    model = _model(torch.float32)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = 96, 128
    images = torch.from_numpy(filler.uniform(71, (2, 3, 96, 128))).to(DEV)
    u = torch.from_numpy(filler.normal(72, (2, 1, 96, 128)) * 2.0).to(DEV)
    inst = engine.export_head_phase(model, images, torch.from_numpy(g["rois"]).to(DEV), u, dilation)
    ref = torch.from_numpy(g[f"d{dilation}_instance"]).float()
    assert inst.shape == ref.shape
    assert (inst.cpu() == ref).float().mean().item() > 0.999
    # the dilation kernel alone on the reference's own logits: exact
    logits0 = torch.from_numpy(g["d0_logits"]).to(DEV)
    assert torch.equal(ops.instance_masks(logits0, dilation).cpu(), ref)
    oc = model.pretrained_unet.output_conv
    binary = ops.binary_masks(u, oc.weight.detach().float().reshape(2).contiguous(), oc.bias.detach().float())
    assert max_abs(binary.cpu(), g["binary"]) < 1e-5


def test_conv_operands_over_2gib_split_by_image_range():
    """A conv whose input and output each span 2.26 GB (360 images x 128x96 x 256 ch bf16): the LDS-DMA kernels
    address through 32-bit buffer offsets, so hiseg_conv2d_fwd splits the launch into image ranges.  Images are
    independent, so the first, a middle and the last images equal the same conv run on those images alone."""
    from hiseg import ops
    dt = torch.bfloat16
    N, C, H, W = 360, 256, 128, 96
    g = torch.Generator(device=DEV).manual_seed(3)
    x = ops.Act.new(N, H, W, C, dt, DEV, zero=False)
    x.t.copy_(torch.randn(x.t.numel(), device=DEV, generator=g, dtype=torch.float32).to(dt))
    assert x.t.numel() * 2 > (1 << 31)
    w = torch.randn(C, C, 3, 3, device=DEV, generator=g) / (C * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(C, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=1)
    r = ops.Act.new(N, H, W, C, dt, DEV, zero=False)
    r.t.copy_(torch.randn(r.t.numel(), device=DEV, generator=g, dtype=torch.float32).to(dt))
    y = ops.conv2d(p, x, residual=r)
    torch.cuda.synchronize()
    per = H * W * C
    for n in (0, 1, 179, 358, 359):
        xi = ops.Act.new(1, H, W, C, dt, DEV, zero=False)
        xi.t.copy_(x.t[n * per:(n + 1) * per])
        ri = ops.Act.new(1, H, W, C, dt, DEV, zero=False)
        ri.t.copy_(r.t[n * per:(n + 1) * per])
        yi = ops.conv2d(p, xi, residual=ri)
        torch.cuda.synchronize()
        assert torch.equal(yi.t, y.t[n * per:(n + 1) * per]), n
    del x, r, y
    torch.cuda.empty_cache()


# The halo-tiled wide kernel (conv_hw.hip, variants 80 = BCO 256, 82 = BCO 128): channel-major K order, so
# within bf16 output rounding of the generic kernel.  name: (N, Cin, Cout, H, W, residual, relu, a_coff)
HW_CASES = {
    "256_res_ragged_13x11": (3, 256, 256, 13, 11, True, True, 0),
    "256_roi_64x48": (4, 256, 256, 64, 48, True, True, 0),
    "256_plain_relu_30x40": (2, 256, 256, 30, 40, False, True, 0),
    "128_to_128_res_37x20": (2, 128, 128, 37, 20, True, True, 0),
    "64_to_128_16x12": (3, 64, 128, 16, 12, False, False, 0),
    "128_to_384_offset_view_9x23": (2, 128, 384, 9, 23, True, False, 64),
    "64_res_roi_64x48": (3, 64, 64, 64, 48, True, True, 0),
    "256_to_64_ragged_21x13": (2, 256, 64, 21, 13, False, False, 0),
    "128_to_192_offset_view_17x9": (2, 128, 192, 17, 9, True, True, 32),
    # BCO 64 over fewer than 64 output columns (EnhancedUNet final 64 -> 32): one partial Cout tile
    "64_to_32_roi_64x48": (3, 64, 32, 64, 48, False, True, 0),
    "128_to_16_res_13x9": (2, 128, 16, 13, 9, True, True, 0),
}

# BCO-128/256 configurations need a 128-multiple Cout, the BCO-64 ones (88 / 89) a 64-multiple or 16 / 32 / 48
HW_VARIANT_CMUL = {80: 256, 82: 128, 84: 256, 86: 128, 88: 64, 89: 64}


@pytest.mark.parametrize("variant", [80, 82, 84, 86, 88, 89])
@pytest.mark.parametrize("name", list(HW_CASES))
def test_conv_halo_wide_within_bf16(name, variant):
    from hiseg import ops
    N, Cin, Cout, H, W, res, relu, coff = HW_CASES[name]
    narrow = variant in (88, 89) and Cout < 64 and Cout % 16 == 0
    if Cout % HW_VARIANT_CMUL[variant] and not narrow:
        pytest.skip("configuration needs a larger Cout multiple (the kernel declines; covered by the fallback tests)")
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(11)
    full = ops.Act.new(N, H, W, Cin + coff, dt, DEV, zero=False)
    full.t.copy_(torch.randn(full.t.numel(), device=DEV, generator=g).to(dt))
    xa = full.slice(coff, Cin) if coff else full
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (Cin * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, int(relu), dt, DEV, pad=1)
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    ref = ops.conv2d(p, xa, residual=R, variant=-1).to_nchw().float()
    y = ops.conv2d(p, xa, residual=R, variant=variant).to_nchw().float()
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 8e-3


@pytest.mark.parametrize("name", list(HW_CASES))
def test_conv_hwr_bit_identical_to_halo_kernel(name):
    """The register-streamed-weight halo kernel (conv_hwr.hip, variant 92: weights in MFMA fragment order straight
    into registers, one barrier per 32-channel slice) accumulates in conv_hw's non-reuse order (variant 82: slice,
    then taps 0..8), so its output equals that kernel's bit for bit -- ragged tiles, offset views, residual / ReLU
    epilogues, Cout 128 / 256 / 384."""
    from hiseg import ops
    N, Cin, Cout, H, W, res, relu, coff = HW_CASES[name]
    if Cout % 128 or Cin % 64:
        pytest.skip("variant 92 needs a 128-multiple Cout and fragment-packed weights (64-multiple Cin)")
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(13)
    full = ops.Act.new(N, H, W, Cin + coff, dt, DEV, zero=False)
    full.t.copy_(torch.randn(full.t.numel(), device=DEV, generator=g).to(dt))
    xa = full.slice(coff, Cin) if coff else full
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (Cin * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, int(relu), dt, DEV, pad=1)
    assert p.weight_frag is not None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    y82 = ops.conv2d(p, xa, residual=R, variant=82).t.clone()
    y86 = ops.conv2d(p, xa, residual=R, variant=86).t.clone()
    ys = {v: ops.conv2d(p, xa, residual=R, variant=v).t.clone() for v in (92, 93, 94, 95, 96, 97)}
    auto = ops.conv2d(p, xa, residual=R, variant=0).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(ys[92].float()).all()
    for v in (92, 93, 94, 95):    # ky-major taps: variant 82's accumulation order
        assert torch.equal(ys[v], y82), v
    for v in (96, 97):            # kx-major taps with B reuse: variant 86's
        assert torch.equal(ys[v], y86), v
    assert torch.equal(auto, ys[97])   # the automatic choice takes variant 97


@pytest.mark.parametrize("shape", [(2, 64, 0, 64, 64, 48, True), (3, 64, 0, 64, 21, 37, False), (2, 128, 0, 64, 16, 33, True),
                                   (2, 64, 64, 64, 20, 31, False), (2, 256, 0, 128, 18, 40, True),
                                   (2, 128, 128, 256, 9, 23, False), (1, 256, 0, 256, 64, 48, True)])
def test_conv_hwr_wide_tile_bit_identical(shape):
    """Variants 100 (64-Cout x 16 x 32-pixel tiles, four waves) and 101 (128-Cout x 16 x 32, eight waves): the same
    per-element accumulation order as variant 97 / conv_hw's 86 and 89 (channel-major slices, kx-major taps) -- bit
    for bit, ragged pixel tiles, residual, two sources; the automatic choice on 64-channel layers takes 100."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, res = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(29)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=1,
                      split=(Ca, Cb) if Cb else None)
    assert p.weight_frag is not None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    y100 = ops.conv2d(p, xa, xb, residual=R, variant=100).t.clone()
    ref = ops.conv2d(p, xa, xb, residual=R, variant=89).t.clone()
    auto = ops.conv2d(p, xa, xb, residual=R, variant=0).t.clone()
    if Cout % 128 == 0:
        y97 = ops.conv2d(p, xa, xb, residual=R, variant=97).t.clone()
        y101 = ops.conv2d(p, xa, xb, residual=R, variant=101).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(y100.float()).all()
    assert torch.equal(y100, ref)
    if Cout % 128 == 0:
        assert torch.equal(y97, ref) and torch.equal(y101, ref)
        assert torch.equal(auto, y97)
    else:
        assert torch.equal(auto, y100)


@pytest.mark.parametrize("shape", [(2, 128, 128, 128, 32, 24, False), (3, 64, 64, 128, 21, 13, True),
                                   (2, 192, 64, 256, 9, 23, True)])
def test_conv_hwr_two_source_bit_identical(shape):
    """Variants 92 / 97 over a two-source concat (EnhancedUNet decoder up ++ skip): bit-identical to 82 / 86."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, res = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(23)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=1, split=(Ca, Cb))
    assert p.weight_frag is not None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    y82 = ops.conv2d(p, xa, xb, residual=R, variant=82).t.clone()
    y92 = ops.conv2d(p, xa, xb, residual=R, variant=92).t.clone()
    y86 = ops.conv2d(p, xa, xb, residual=R, variant=86).t.clone()
    y97 = ops.conv2d(p, xa, xb, residual=R, variant=97).t.clone()
    torch.cuda.synchronize()
    assert torch.equal(y92, y82)
    assert torch.equal(y97, y86)


@pytest.mark.parametrize("variant", [86, 89])
@pytest.mark.parametrize("shape", [(3, 64, 64, 64, 64, 48, True), (2, 128, 128, 128, 32, 24, False),
                                   (2, 64, 32, 64, 21, 13, True), (2, 96, 64, 128, 9, 23, False),
                                   # B7-ultra head widths (round 3): 96-channel input (K padded past 9 x Cin),
                                   # 96 / 160 outputs (partial last 64-column tile)
                                   (2, 96, 0, 96, 20, 17, True), (2, 96, 96, 96, 12, 9, False),
                                   (2, 192, 0, 160, 10, 21, True)])
def test_conv_halo_two_source_within_bf16(shape, variant):
    """The halo-tiled kernel over a two-source concat (EnhancedUNet decoder: up ++ skip, hierarchical_segmentation_unet.py
    decoders) -- each 32-channel slice read from its own source -- vs the generic kernel within bf16 rounding."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, res = shape
    if variant == 86 and Cout % 128:
        pytest.skip("BCO 128 needs a 128-multiple Cout")
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(19)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=1,
                      split=(Ca, Cb) if Cb else None)
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    ref = ops.conv2d(p, xa, xb, residual=R, variant=-1).to_nchw().float()
    y = ops.conv2d(p, xa, xb, residual=R, variant=variant).to_nchw().float()
    auto = ops.conv2d(p, xa, xb, residual=R, variant=0).to_nchw().float()
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 8e-3
    assert ((auto - ref).abs().max() / ref.abs().max()).item() < 8e-3


@pytest.mark.parametrize("shape", [(2, 320, 112, 128, 256, 12, 16, 97), (2, 256, 40, 64, 128, 10, 14, 97),
                                   (2, 128, 24, 64, 64, 16, 20, 89), (1, 640, 224, 256, 256, 8, 8, 97),
                                   (3, 128, 64, 64, 128, 6, 22, 86)])
def test_conv_halo_upsampled_decoder_within_bf16(shape):
    """smp decoder conv1 on the halo-tiled kernels (round 3): src A nearest-x2 upsampled from (H/2, W/2), src B the
    encoder skip stored with a 64-multiple channel stride and zero pad channels (engine.effunet_forward).  The
    forced halo variant and the automatic choice against the generic kernel on the same padded operands, and the
    generic kernel on the padded operands against the unpadded layout (zero channels add exact zeros)."""
    from hiseg import ops
    N, Ca, Cb, Cbp, Cout, H, W, variant = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(23)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H // 2, W // 2, device=DEV, generator=g), dt)
    skip = torch.randn(N, Cb, H, W, device=DEV, generator=g)
    xb = ops.Act.from_nchw(skip, dt)
    xbp = ops.Act.new(N, H, W, Cb, dt, DEV, cpad=Cbp, zero=True)
    xbp.t.view(-1, Cbp)[:, :Cb].copy_(xb.t.view(-1, xb.cstride)[:, :Cb])
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    bias = torch.randn(Cout, device=DEV, generator=g) * 0.1
    p = ops.pack_conv(w, bias, None, 1, dt, DEV, pad=1, split=(Ca, Cb, Cbp))
    p0 = ops.pack_conv(w, bias, None, 1, dt, DEV, pad=1, split=(Ca, Cb))
    assert p.cb == Cbp
    ref0 = ops.conv2d(p0, xa, xb, a_up=2, variant=-1).to_nchw().float()
    ref = ops.conv2d(p, xa, xbp, a_up=2, variant=-1).to_nchw().float()
    y = ops.conv2d(p, xa, xbp, a_up=2, variant=variant).to_nchw().float()
    auto = ops.conv2d(p, xa, xbp, a_up=2, variant=0).to_nchw().float()
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    scale = ref.abs().max()
    assert ((ref - ref0).abs().max() / scale).item() < 8e-3
    assert ((y - ref).abs().max() / scale).item() < 8e-3
    assert ((auto - ref).abs().max() / scale).item() < 8e-3
    # the ReLU output against float64 of the same bf16 operands
    up = torch.nn.functional.interpolate(xa.to_nchw().double(), scale_factor=2, mode="nearest")
    xin = torch.cat([up, xb.to_nchw().double()], 1)
    z = torch.relu(torch.nn.functional.conv2d(xin, p0.weight[:Cout, :9 * (p0.ca + p0.cb)].float().double()
                                              .view(Cout, 3, 3, p0.ca + p0.cb).permute(0, 3, 1, 2)[:, :Ca + Cb],
                                              bias.double(), padding=1))
    assert ((y.double() - z).abs().max() / z.abs().max()).item() < 1e-2


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_conv_automatic_choice_within_bf16(name):
    """hiseg_conv2d_fwd's automatic kernel choice on every VARIANT_CASES layer: bit-identical to the generic kernel
    where it takes a tap-major kernel, within bf16 rounding where it takes the channel-major halo kernel."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, k, convT, res, mul, o2 = VARIANT_CASES[name]
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(7)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    if convT:
        w = torch.randn(Ca, Cout, 2, 2, device=DEV, generator=g) / Ca ** 0.5
        p = ops.pack_convT2x2(w, torch.randn(Cout, device=DEV, generator=g), None, 1, dt, DEV)
        oH, oW = 2 * H, 2 * W
    else:
        w = torch.randn(Cout, Ca + Cb, k, k, device=DEV, generator=g) / ((Ca + Cb) * k * k) ** 0.5
        p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=k // 2,
                          split=(Ca, Cb) if Cb else None)
        oH, oW = H, W
    R = ops.Act.from_nchw(torch.randn(N, Cout, oH, oW, device=DEV, generator=g), dt) if res else None
    M = ops.Act.from_nchw(torch.rand(N, Cout, oH, oW, device=DEV, generator=g), dt) if mul else None
    ref = ops.conv2d(p, xa, xb, residual=R, mul=M, variant=-1).to_nchw().float()
    y = ops.conv2d(p, xa, xb, residual=R, mul=M, variant=0).to_nchw().float()
    torch.cuda.synchronize()
    # the halo kernel also takes two-source layers whose sources are whole 32-channel slices (round 2 v10)
    halo = (not convT and k == 3 and Cb % 32 == 0 and not mul and not o2 and Cout % 128 == 0 and Ca % 32 == 0
            and Ca >= 64)
    if halo:
        assert ((y - ref).abs().max() / ref.abs().max()).item() < 8e-3
    else:
        assert torch.equal(y, ref)


@pytest.mark.parametrize("shape", [(2, 256, 0, 256, 64, 48, True, True), (3, 128, 0, 128, 37, 21, True, False),
                                   (2, 128, 0, 256, 33, 17, False, True), (2, 128, 128, 128, 32, 24, False, True),
                                   (2, 64, 64, 384, 20, 30, True, True), (1, 256, 0, 128, 16, 16, False, False)])
def test_conv_hwt_bit_identical_to_hwr(shape):
    """Variant 103 (conv_hwt.hip: one wave per SIMD, 64 x 256 wave tiles, A fragments two K steps ahead, 32 x 16-pixel
    x 128-Cout workgroup tiles): conv_hwr's per-element accumulation order (channel-major slices, kx-major taps, the
    same MFMA) -- equal to variant 97 bit for bit: ragged pixel tiles, residual / ReLU / none, two sources, Cout
    128 / 256 / 384."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, res, relu = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(31)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, int(relu), dt, DEV, pad=1,
                      split=(Ca, Cb) if Cb else None)
    assert p.weight_frag is not None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    outs = {}
    for v in (97, 103, 0):
        o = ops.Act.new(N, H, W, Cout, dt, torch.device(DEV))
        o.t.fill_(float("nan"))
        outs[v] = ops.conv2d(p, xa, xb, out=o, residual=R, variant=v).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(outs[97].float()).all()
    assert torch.equal(outs[103], outs[97])
    assert torch.equal(outs[0], outs[97])


@pytest.mark.parametrize("shape", [(2, 256, 0, 256, 64, 48, True, True), (3, 128, 0, 128, 37, 21, True, False),
                                   (2, 128, 0, 256, 33, 17, False, True), (2, 128, 128, 128, 32, 24, False, True),
                                   (2, 64, 64, 384, 20, 30, True, True), (1, 256, 0, 128, 16, 16, False, False),
                                   (2, 192, 64, 256, 9, 23, True, False)])
def test_conv_hwc_bit_identical_to_hwr(shape):
    """Variants 104 / 106 (conv_hwc.hip, round 5: each wave 32 Cout x all 256 pixels of the tile, every halo row's B
    fragment reused across the 3 ky taps; 106 with the residual tile prefetched into LDS) and 105 (256-Cout workgroups):
    conv_hwr's per-element accumulation order (channel-major slices, kx-major / ky-inner taps, one 32-channel MFMA per
    (slice, tap)) -- equal to variant 97 bit for bit: ragged pixel tiles, residual / ReLU / none, two sources, Cout
    128 / 256 / 384; the automatic choice takes 108 (round 6: 104 with a ring of three halo buffers) for 128-multiple
    Cout; 109 (round 6): multi-tile workgroups, each walking HISEG_CONV_HWC_MT work items with the next tile's first halo
    slice DMA'd during the last slice and a two-half epilogue (ragged item counts: the last workgroups take fewer).
    Outputs NaN-prefilled."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, res, relu = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(37)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, int(relu), dt, DEV, pad=1,
                      split=(Ca, Cb) if Cb else None)
    assert p.weight_frag is not None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    outs = {}
    vs = (97, 104, 106, 108, 109, 0) + ((105,) if Cout % 256 == 0 else ())
    for v in vs:
        o = ops.Act.new(N, H, W, Cout, dt, torch.device(DEV))
        o.t.fill_(float("nan"))
        outs[v] = ops.conv2d(p, xa, xb, out=o, residual=R, variant=v).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(outs[97].float()).all()
    for v in vs:
        assert torch.equal(outs[v], outs[97]), f"variant {v}"


@pytest.mark.parametrize("shape", [(2, 64, 0, 64, 64, 48, True, True), (3, 64, 0, 64, 37, 21, False, False),
                                   (2, 256, 0, 64, 33, 50, False, True), (2, 64, 64, 64, 32, 24, False, True),
                                   (2, 128, 0, 192, 20, 30, True, True), (1, 64, 0, 64, 9, 7, True, True)])
def test_conv_hwc64_bit_identical_to_hwr(shape):
    """Variant 107 (round 5: conv_hwc on 64-Cout workgroups over 16 x 32-pixel tiles, two 16 x 16 pixel blocks side
    by side sharing one 18 x 34 halo) equals conv_hwr's 64-Cout form (variant 100) bit for bit -- ragged tiles (also
    images narrower than one block), residual / ReLU / none, two sources, Cout 64 / 192 -- and is the automatic choice
    for 64-multiple Cout that is no 128-multiple.  Outputs NaN-prefilled."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W, res, relu = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(39)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt) if Cb else None
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, int(relu), dt, DEV, pad=1,
                      split=(Ca, Cb) if Cb else None)
    assert p.weight_frag is not None
    R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
    outs = {}
    for v in (100, 107, 102, 0):
        o = ops.Act.new(N, H, W, Cout, dt, torch.device(DEV))
        o.t.fill_(float("nan"))
        outs[v] = ops.conv2d(p, xa, xb, out=o, residual=R, variant=v).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(outs[100].float()).all()
    assert torch.equal(outs[107], outs[100]) and torch.equal(outs[0], outs[100])
    assert torch.equal(outs[102], outs[100])   # (round 6: variant 102, the multi-tile form of 107)


@pytest.mark.parametrize("shape", [(2, 128, 64, 64, 36, 40), (1, 64, 64, 64, 18, 34)])
def test_conv_hwc64_upsampled_decoder_bit_identical(shape):
    """The smp decoder's conv1 form at 64 output channels on variant 107 equals conv_hwr's 64-Cout form (100)."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(47)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H // 2, W // 2, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=1, split=(Ca, Cb))
    outs = {}
    for v in (100, 107, 0):
        o = ops.Act.new(N, H, W, Cout, dt, torch.device(DEV))
        o.t.fill_(float("nan"))
        outs[v] = ops.conv2d(p, xa, xb, out=o, a_up=2, variant=v).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(outs[100].float()).all()
    assert torch.equal(outs[107], outs[100]) and torch.equal(outs[0], outs[100])


@pytest.mark.parametrize("shape", [(2, 320, 128, 256, 30, 40), (2, 256, 64, 128, 20, 24), (1, 128, 64, 128, 18, 34)])
def test_conv_hwc_upsampled_decoder_bit_identical(shape):
    """The smp decoder's conv1 form (src A nearest-x2 upsampled, src B the encoder skip; ReLU, no residual) on
    conv_hwc (variants 104, 108) equals conv_hwr (97) bit for bit."""
    from hiseg import ops
    N, Ca, Cb, Cout, H, W = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(43)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H // 2, W // 2, device=DEV, generator=g), dt)
    xb = ops.Act.from_nchw(torch.randn(N, Cb, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Ca + Cb, 3, 3, device=DEV, generator=g) / ((Ca + Cb) * 9) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=1, split=(Ca, Cb))
    outs = {}
    for v in (97, 104, 108, 0):
        o = ops.Act.new(N, H, W, Cout, dt, torch.device(DEV))
        o.t.fill_(float("nan"))
        outs[v] = ops.conv2d(p, xa, xb, out=o, a_up=2, variant=v).t.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(outs[97].float()).all()
    assert torch.equal(outs[104], outs[97]) and torch.equal(outs[108], outs[97]) and torch.equal(outs[0], outs[97])


@pytest.mark.parametrize("shape", [(2, 37, 45, 240, 5, 1), (3, 20, 20, 2304, 5, 1), (2, 33, 47, 144, 3, 2),
                                   (2, 40, 40, 480, 5, 2), (1, 9, 7, 192, 3, 1), (2, 64, 48, 200, 3, 1)])
def test_dwconv_lds_tile_bit_identical_to_gather_kernel(shape, monkeypatch):
    """The LDS-tiled depthwise conv (dwconv_t_kernel: 8 x 16 output tiles x 64 channels, the input window loaded
    once; bf16 stride-1 layers of >= 192 channels; 4 and 2 channels per thread, HISEG_DWCONV_CP) against the register-gather kernel (dwconv_q_kernel,
    HISEG_DWCONV_T=0): bit-identical outputs (same taps, order and epilogue) at ragged tiles and partial channel
    groups, k3 / k5; the fused SE pool and gate within f32 re-association (one partial per tile instead of per strip
    range), the gate batch-invariant (the automatic choice's tiled layers).  HISEG_DWCONV_T=2 forces the tiled kernel
on the stride-2 and narrow layers the automatic choice gives the gather kernel."""
    from hiseg import ops
    N, H, W, C, k, stride = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(41)
    A = ops.Act.from_nchw(torch.randn(N, C, H, W, device=DEV, generator=g), dt)
    wd = (torch.randn(k * k, C, device=DEV, generator=g) * 0.3).contiguous()
    sc, sh = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.1
    cr = max(1, C // 24)
    w1, b1 = torch.randn(cr, C, device=DEV, generator=g) * 0.1, torch.randn(cr, device=DEV, generator=g) * 0.1
    w2, b2 = torch.randn(C, cr, device=DEV, generator=g) * 0.1, torch.randn(C, device=DEV, generator=g) * 0.1
    res = {}
    # 2: the LDS-tiled kernel for every bf16 layer, stride 2 and narrow ones included, at 4 and 2 channels per thread
    for mode, cp in (("2", "4"), ("2", "2"), ("0", "4")):
        monkeypatch.setenv("HISEG_DWCONV_T", mode)
        monkeypatch.setenv("HISEG_DWCONV_CP", cp)
        plain = ops.dwconv(A, wd, sc, sh, k, stride, 3).t.clone()
        h, gate = ops.dwconv_se_gate(A, wd, sc, sh, k, stride, 3, w1, b1, w2, b2, 3)
        res[mode + cp] = (plain, h.t.clone(), gate.clone())
    monkeypatch.delenv("HISEG_DWCONV_CP")
    torch.cuda.synchronize()
    (p0, h0, g0) = res["04"]
    for key in ("24", "22"):
        p1, h1, g1 = res[key]
        assert torch.isfinite(p1.float()).all()
        assert torch.equal(p1, p0) and torch.equal(h1, h0) and torch.equal(p1, h1), key
        assert (g1 - g0).abs().max().item() < 1e-5, key
    g1 = res["22" if k == 5 or C < 512 else "24"][2]   # the default channels per thread (dw_cp): the pool sums' order
    if not (192 <= C < 2048 and (stride == 1 or k == 5)):   # the automatic choice's tiled layers (dw_use_tiles)
        return
    # batch invariance of the pooled gate (tile partials do not depend on the batch): image 0 alone
    monkeypatch.setenv("HISEG_DWCONV_T", "1")
    one = ops.Act(A.t[:H * W * A.cstride].clone(), 1, H, W, C, A.cstride, 0)
    _, g_one = ops.dwconv_se_gate(one, wd, sc, sh, k, stride, 3, w1, b1, w2, b2, 3)
    assert torch.equal(g_one[0], g1[0])


@pytest.mark.parametrize("case", [(4, 20, 20, 3840, 160, 5, 1), (2, 40, 40, 240, 10, 3, 2), (3, 15, 11, 104, 25, 3, 1),
                                  (2, 9, 7, 1152, 48, 5, 1), (1, 30, 30, 2304, 96, 3, 1)])
def test_se_two_launch_matches_three_launch_and_f64(case, monkeypatch):
    """The two-launch SqueezeExcite (se_pool_w1_kernel + se_gate_out_kernel: the pooled channels multiplied into
    W1 per 64-channel block, hidden partials parked in the partial columns that block alone read) against the
    three-launch path (HISEG_SE2=0: gap_reduce, se_hidden, se_out) and a float64 restatement, at the B7 / B0 deep
    shapes, a ragged channel block (C = 104), Cr not a multiple of 4 (scalar W2 rows) and the gather kernel's many
    partials; batch-invariant (image 0 alone gives the same gate bits); the module-level se_gate as well."""
    from hiseg import ops
    N, H, W, C, cr, k, stride = case
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(43)
    A = ops.Act.from_nchw(torch.randn(N, C, H, W, device=DEV, generator=g), dt)
    wd = (torch.randn(k * k, C, device=DEV, generator=g) * 0.3).contiguous()
    sc, sh = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.1
    w1, b1 = torch.randn(cr, C, device=DEV, generator=g) * 0.1, torch.randn(cr, device=DEV, generator=g) * 0.1
    w2, b2 = torch.randn(C, cr, device=DEV, generator=g) * 0.1, torch.randn(C, device=DEV, generator=g) * 0.1
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("HISEG_SE2", mode)
        h, gate = ops.dwconv_se_gate(A, wd, sc, sh, k, stride, 3, w1, b1, w2, b2, 3)
        sg = ops.se_gate(A, w1, b1, w2, b2, 3)
        res[mode] = (h.t.clone(), gate.clone(), sg.clone())
    torch.cuda.synchronize()
    (h1, g1, s1), (h0, g0, s0) = res["1"], res["0"]
    assert torch.equal(h1, h0)
    assert torch.isfinite(g1).all() and torch.isfinite(s1).all()
    assert (g1 - g0).abs().max().item() < 2e-6
    assert (s1 - s0).abs().max().item() < 2e-6
    # float64 restatement of the gate from the kernel's own depthwise output (the fused pool sums the f32 values
    # before their bf16 rounding: 1e-3)
    hm = h.to_nchw().double().mean((2, 3))
    hid = F.silu(hm @ w1.double().t() + b1.double())
    ref = torch.sigmoid(hid @ w2.double().t() + b2.double())
    assert (g1.double() - ref).abs().max().item() < 1e-3
    xm = A.to_nchw().double().mean((2, 3))
    ref_s = torch.sigmoid(F.silu(xm @ w1.double().t() + b1.double()) @ w2.double().t() + b2.double())
    assert (s1.double() - ref_s).abs().max().item() < 1e-5
    # the float4 weight paths are taken by alignment: misaligned copies of W1 / W2 give the same bits
    monkeypatch.setenv("HISEG_SE2", "1")
    w1u = torch.empty(w1.numel() + 1, device=DEV)[1:].view_as(w1).copy_(w1)
    w2u = torch.empty(w2.numel() + 1, device=DEV)[1:].view_as(w2).copy_(w2)
    _, g_u = ops.dwconv_se_gate(A, wd, sc, sh, k, stride, 3, w1u, b1, w2u, b2, 3)
    assert torch.equal(g_u, g1)
    if not (192 <= C < 2048 and (stride == 1 or k == 5)) or N == 1:   # tiled layers: batch-independent partials
        return
    one = ops.Act(A.t[:H * W * A.cstride].clone(), 1, H, W, C, A.cstride, 0)
    _, g_one = ops.dwconv_se_gate(one, wd, sc, sh, k, stride, 3, w1, b1, w2, b2, 3)
    assert torch.equal(g_one[0], g1[0])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_roi_align_whole_pixel_stores_bit_identical(dt, monkeypatch):
    """RoIAlign into NHWC with whole-pixel 16-B stores (channels then the zero padding, HISEG_ROI_VEC=1) against the
    per-channel stores (HISEG_ROI_VEC=0): bit-identical at C2's shapes -- the RGB crop (3 -> cstride 8 / 4) and the
    1 -> 2 output_conv affine over the UNet logit -- including ROIs outside the image, a bad batch index and a NaN
    coordinate (zero outputs), and the padding is written (NaN-prefilled outputs)."""
    from hiseg import ops
    g = torch.Generator(device=DEV).manual_seed(47)
    B, H, W, N, oh, ow = 4, 120, 160, 37, 64, 48
    images = torch.rand(B, 3, H, W, device=DEV, generator=g)
    u = torch.randn(B, 1, H, W, device=DEV, generator=g)
    x1 = torch.rand(N, device=DEV, generator=g) * 500 - 40
    y1 = torch.rand(N, device=DEV, generator=g) * 380 - 40
    rois = torch.stack([torch.randint(0, B, (N,), device=DEV, generator=g).float(), x1, y1,
                        x1 + torch.rand(N, device=DEV, generator=g) * 300 + 1,
                        y1 + torch.rand(N, device=DEV, generator=g) * 200 + 1], 1)
    rois[3, 0] = B + 2          # batch index out of range
    rois[5, 1] = float("nan")   # NaN coordinate
    aw, ab = torch.randn(2, device=DEV, generator=g), torch.randn(2, device=DEV, generator=g)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("HISEG_ROI_VEC", mode)
        outs = []
        for feat, kw, C in ((images, {}, 3), (u, {"aff_w": aw, "aff_b": ab}, 2)):
            o = ops.Act.new(N, oh, ow, C, dt, torch.device(DEV), zero=False)
            o.t.fill_(float("nan"))
            ops.roi_align(feat, rois, oh, ow, 480.0, 640.0, True, out=o, zero_to=o.cstride, **kw)
            outs.append(o.t.clone())
        res[mode] = outs
    torch.cuda.synchronize()
    for a, b in zip(res["1"], res["0"]):
        assert torch.isfinite(a.float()).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(3, 768, 768, 16, 12, True), (2, 256, 256, 12, 10, False), (5, 192, 384, 8, 8, True)])
def test_conv3x3_small_image_splitk(shape):
    """3x3 layers over images of <= 256 pixels with K >= 1536 (the B7 EnhancedUNet's 768-channel pair at 16 x 12)
    split their K loop over workgroups on the generic kernel when the caller passes the workspace (the train engine
    does for small batches; hiseg_conv2d_workspace_bytes > 0): against the halo kernel (variant 97) within bf16
    rounding and against float32 torch, and batch-invariant bit for bit (the split depends on the per-image grid)."""
    from hiseg import ops
    N, Ci, Co, H, W, res = shape
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(53)
    x = torch.randn(N, Ci, H, W, device=DEV, generator=g)
    xa = ops.Act.from_nchw(x, dt)
    w = torch.randn(Co, Ci, 3, 3, device=DEV, generator=g) / (Ci * 9) ** 0.5
    b = torch.randn(Co, device=DEV, generator=g) * 0.1
    p = ops.pack_conv(w, b, None, 1, dt, DEV, pad=1)
    R = ops.Act.from_nchw(torch.randn(N, Co, H, W, device=DEV, generator=g), dt) if res else None
    out = ops.conv2d(p, xa, residual=R, split_k_3x3=True).to_nchw().float()
    ref = F.conv2d(x.to(dt).float(), w.to(dt).float(), b, padding=1)
    if res:
        ref = ref + R.to_nchw().float()
    ref = F.relu(ref)
    assert _rel(out.cpu(), ref.cpu()) < 1e-2
    if Co % 128 == 0:
        h = ops.conv2d(p, xa, residual=R, variant=97).to_nchw().float()
        assert _rel(out.cpu(), h.cpu()) < 1e-2
    one = ops.Act.from_nchw(x[:1].contiguous(), dt)
    R1 = ops.Act.from_nchw(R.to_nchw()[:1].contiguous(), dt) if res else None
    o1 = ops.conv2d(p, one, residual=R1, split_k_3x3=True).to_nchw()
    assert torch.equal(o1[0], ops.conv2d(p, xa, residual=R, split_k_3x3=True).to_nchw()[0])


LIN_CASES = {  # (N, Ca, Cout, H, W, stride, SE gate, residual[, k]): layers of the generic kernel
    "b7_proj_2304to384_gated_split": (4, 2304, 384, 20, 20, 1, True, True),
    "gated_480to80": (2, 480, 80, 24, 20, 1, True, True),
    "ragged_k_200to72": (2, 200, 72, 13, 11, 1, False, False),
    "stride2_96to40": (2, 96, 40, 17, 15, 2, False, True),
    "narrow_64to16": (2, 64, 16, 30, 30, 1, False, False),
    "expand_160to960": (2, 160, 960, 12, 10, 1, False, False),
    "k3_72to72": (2, 72, 72, 16, 12, 1, False, True, 3),          # the B1 EnhancedUNet's 72-channel 3x3 class
    "k3_144to144": (2, 144, 144, 11, 9, 1, False, False, 3),
    "k3_s2_40to96": (2, 40, 96, 15, 13, 2, False, False, 3),      # chunks cross taps inside a K block
    "k5_24to32": (2, 24, 32, 10, 14, 1, False, False, 5),
    "k3_768to768_split": (2, 768, 768, 16, 12, 1, False, False, 3),
}


@pytest.mark.parametrize("name", sorted(LIN_CASES))
def test_igemm_linear_gather_bit_identical(name, monkeypatch):
    """The generic kernel's buffer-offset gathers (HISEG_IGEMM_LIN=2, the default: 1x1 layers through per-chunk
    offsets + a K-block SGPR offset; k x k layers through a per-thread tap delta + per-row tap masks) load the same
    activations, gates and weights as the (n, y, x) gather (=0): equal outputs, for the forced generic kernel (-1),
    the split-K form (99, where the layer splits) and the automatic choice (0) -- ragged last K block, chunks crossing
    taps, stride 2, SE gate, residual, every tile width."""
    from hiseg import ops
    N, Ca, Cout, H, W, stride, ins, res = LIN_CASES[name][:8]
    k = LIN_CASES[name][8] if len(LIN_CASES[name]) > 8 else 1
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(23)
    xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
    w = torch.randn(Cout, Ca, k, k, device=DEV, generator=g) / (Ca * k * k) ** 0.5
    p = ops.pack_conv(w, torch.randn(Cout, device=DEV, generator=g) * 0.1, None, 1, dt, DEV,
                      stride=stride, pad=k // 2)
    gate = torch.rand(N, p.ca, device=DEV, generator=g) if ins else None
    Ho, Wo = (H + 2 * (k // 2) - k) // stride + 1, (W + 2 * (k // 2) - k) // stride + 1
    R = ops.Act.from_nchw(torch.randn(N, Cout, Ho, Wo, device=DEV, generator=g), dt) if res else None
    variants = (-1, 99, 0) if name.endswith("_split") else (-1, 0)
    for v in variants:
        outs = []
        for lin in ("2", "0"):
            monkeypatch.setenv("HISEG_IGEMM_LIN", lin)
            y = ops.conv2d(p, xa, residual=R, in_scale=gate, variant=v, split_k_3x3=(k == 3))
            torch.cuda.synchronize()
            outs.append(y.to_nchw().float())
        assert torch.isfinite(outs[0]).all()
        assert torch.equal(outs[0], outs[1]), (name, v)

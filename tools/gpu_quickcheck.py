"""First GPU sanity check of libhiseg ops against torch references (developer tool)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
import torch, torch.nn.functional as F
from hiseg import ops
from hiseg import _lib as L

dev = "cuda"
torch.manual_seed(0)

def ref_conv(x, w, b, stride, pad, act):
    y = F.conv2d(x, w, b, stride=stride, padding=pad)
    if act == 1: y = F.relu(y)
    return y

def check_conv(N, Cin, Cout, H, W, k, stride, dtype, act=1):
    x = torch.randn(N, Cin, H, W, device=dev)
    w = torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, device=dev) * 0.1
    p = ops.pack_conv(w, b, None, act, dtype, dev, stride=stride, pad=k // 2)
    xa = ops.Act.from_nchw(x, dtype)
    y = ops.conv2d(p, xa)
    torch.cuda.synchronize()
    got = y.to_nchw()
    xr = x.to(dtype).float(); wr = w.to(dtype).float()
    ref = ref_conv(xr.double(), wr.double(), b.double(), stride, k // 2, act).float()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"conv N{N} {Cin}->{Cout} {H}x{W} k{k} s{stride} {dtype}: maxerr {err:.3e} (ref max {scale:.2f})")
    return err / max(scale, 1e-6)

def check_convT(N, Cin, Cout, H, W, dtype):
    x = torch.randn(N, Cin, H, W, device=dev)
    w = torch.randn(Cin, Cout, 2, 2, device=dev) / Cin ** 0.5
    b = torch.randn(Cout, device=dev) * 0.1
    p = ops.pack_convT2x2(w, b, None, 0, dtype, dev)
    y = ops.conv2d(p, ops.Act.from_nchw(x, dtype))
    got = y.to_nchw()
    ref = F.conv_transpose2d(x.to(dtype).double(), w.to(dtype).double(), b.double(), stride=2).float()
    err = (got - ref).abs().max().item()
    print(f"convT {Cin}->{Cout} {H}x{W} {dtype}: maxerr {err:.3e}")
    return err / ref.abs().max().item()

def roi_ref(feat, rois, oh, ow, sh, sw):
    bi = rois[:, 0].long()
    x1 = rois[:, 1] * sw; y1 = rois[:, 2] * sh; x2 = rois[:, 3] * sw; y2 = rois[:, 4] * sh
    gx = torch.linspace(0, 1, ow, device=feat.device); gy = torch.linspace(0, 1, oh, device=feat.device)
    GY, GX = torch.meshgrid(gy, gx, indexing="ij")
    fx = x1[:, None, None] + GX[None] * (x2 - x1)[:, None, None]
    fy = y1[:, None, None] + GY[None] * (y2 - y1)[:, None, None]
    H, W = feat.shape[2:]
    g = torch.stack([fx / (W - 1) * 2 - 1, fy / (H - 1) * 2 - 1], -1)
    return F.grid_sample(feat[bi], g, mode="bilinear", padding_mode="zeros", align_corners=True)

rel = []
for dt in (torch.float32, torch.bfloat16):
    rel.append(check_conv(2, 64, 64, 20, 18, 3, 1, dt))
    rel.append(check_conv(2, 256, 256, 16, 12, 3, 1, dt))
    rel.append(check_conv(3, 3, 64, 17, 13, 3, 1, dt))
    rel.append(check_conv(2, 128, 32, 15, 9, 3, 1, dt))
    rel.append(check_conv(2, 32, 2, 15, 9, 1, 1, dt, act=0))
    rel.append(check_conv(2, 24, 40, 31, 33, 3, 2, dt))
    rel.append(check_convT(2, 256, 128, 8, 6, dt))
    rel.append(check_convT(2, 8, 32, 8, 6, dt))
print("max rel err", max(rel))

feat = torch.rand(2, 3, 48, 64, device=dev)
rois = torch.tensor([[0, .1, .1, .4, .9], [1, .35, .15, .6, .95], [0, .0, .0, 1.0, 1.0], [1, .7, .3, .95, .99]], device=dev)
ref = roi_ref(feat, rois, 16, 12, 48, 64)
out = torch.empty(4, 3, 16, 12, device=dev)
ops.roi_align(feat, rois, 16, 12, 48, 64, True, nchw_out=out)
print("roi_align maxerr", (out - ref).abs().max().item())

# perf probe: the dominant conv (256->256 3x3 @ 64x48, 256 ROIs), bf16
for dt in (torch.bfloat16, torch.float32):
    N, C, H, W = 256, 256, 64, 48
    x = ops.Act.new(N, H, W, C, dt, dev, zero=False); x.t.normal_()
    w = torch.randn(C, C, 3, 3, device=dev) * 0.02
    p = ops.pack_conv(w, None, None, 1, dt, dev, pad=1)
    for _ in range(3): y = ops.conv2d(p, x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): y = ops.conv2d(p, x, out=y)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    fl = 2 * N * H * W * C * C * 9
    print(f"perf conv 256->256 3x3 N{N} {dt}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TFLOP/s")

"""GPU probe: one two-source 3x3 conv (the EnhancedUNet decoder's cat(up, skip) conv) with its sources carved
out of NaN-filled memory: any read outside the sources' valid elements shows up as NaN in the output
(developer tool, round 4)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "human-instance-segmentation_amd")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from hiseg import train_engine as TE  # noqa: E402
from hiseg.ops import Act  # noqa: E402

DEV = "cuda"


def carve(buf, off, N, H, W, C):
    n = N * H * W * C
    t = buf[off:off + n]
    t.copy_((torch.rand(n, device=DEV) * 2 - 1).to(buf.dtype))
    return Act(t, N, H, W, C, C, 0), off + n


def one(N, H, W, ca, cb, cout, dt, gap):
    torch.manual_seed(0)
    conv = nn.Conv2d(ca + cb, cout, 3, padding=1).to(DEV)
    S = TE.TrainState(nn.Sequential(conv), dt, torch.device(DEV))
    p = S.conv(conv, split=(ca, cb))
    total = N * H * W * (ca + cb) + 3 * gap
    buf = torch.full((total,), float("nan"), dtype=dt, device=DEV)
    xa, o = carve(buf, gap, N, H, W, ca)
    xb, _ = carve(buf, o + gap, N, H, W, cb)
    y, _ = TE.conv_fwd(S, p, xa, xb)
    torch.cuda.synchronize()
    yt = y.t.view(N, H, W, y.cstride)[..., :cout].permute(0, 3, 1, 2).float()
    xin = torch.cat([xa.t.view(N, H, W, ca), xb.t.view(N, H, W, cb)], -1).permute(0, 3, 1, 2).float()
    ref = F.conv2d(xin, conv.weight.to(dt).float(), conv.bias.float(), padding=1)
    nan = int((~torch.isfinite(yt)).sum())
    err = ((yt - ref).abs().max() / ref.abs().max()).item() if nan == 0 else float("nan")
    print(f"N {N} {H}x{W} {ca}+{cb}->{cout} {dt} gap {gap}: non-finite {nan}/{yt.numel()}  rel err {err:.3e}",
          flush=True)


if __name__ == "__main__":
    for dt in (torch.bfloat16, torch.float32):
        for (N, H, W, ca, cb, cout) in ((2, 40, 30, 144, 144, 144), (8, 40, 30, 144, 144, 144),
                                        (2, 64, 48, 192, 192, 192), (2, 32, 24, 384, 384, 384),
                                        (2, 128, 96, 96, 96, 96), (2, 80, 60, 72, 72, 72),
                                        (2, 32, 24, 128, 128, 128), (2, 64, 48, 64, 64, 64)):
            for gap in (0, 4096):
                one(N, H, W, ca, cb, cout, dt, gap)

"""GPU probe: the EnhancedUNet's ConvTranspose 2x2/s2 (train path packing) with its input carved from NaN-filled
memory and a NaN-prefilled output, per forced kernel variant (developer tool, round 4)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "human-instance-segmentation_amd")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from hiseg import _lib as L  # noqa: E402
from hiseg import train_engine as TE  # noqa: E402
from hiseg.ops import Act  # noqa: E402

DEV = "cuda"


def one(N, H, W, cin, cout, dt, variants):
    torch.manual_seed(0)
    conv = nn.ConvTranspose2d(cin, cout, 2, stride=2).to(DEV)
    S = TE.TrainState(nn.Sequential(conv), dt, torch.device(DEV))
    p = S.conv(conv, convT=True)
    gap = 4096
    n = N * H * W * cin
    buf = torch.full((n + 2 * gap,), float("nan"), dtype=dt, device=DEV)
    xa = Act(buf[gap:gap + n], N, H, W, cin, cin, 0)
    xa.t.copy_((torch.rand(n, device=DEV) * 2 - 1).to(dt))
    xin = xa.t.view(N, H, W, cin).permute(0, 3, 1, 2).float()
    ref = F.conv_transpose2d(xin, conv.weight.to(dt).float(), conv.bias.float(), stride=2)
    for v in variants:
        out = Act(torch.full((N * 2 * H * 2 * W * cout,), float("nan"), dtype=dt, device=DEV), N, 2 * H, 2 * W, cout,
                  cout, 0)
        d = TE._desc(S, p, xa, None, out)
        st = L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), v, None)
        torch.cuda.synchronize()
        if st != 0:
            print(f"  convT {cin}->{cout} N{N} {H}x{W} {dt} variant {v}: status {st} "
                  f"{L.lib().hiseg_last_error_string().decode()}", flush=True)
            continue
        y = out.t.view(N, 2 * H, 2 * W, cout).permute(0, 3, 1, 2).float()
        nan = int((~torch.isfinite(y)).sum())
        err = ((y - ref).abs().max() / ref.abs().max()).item() if nan == 0 else float("nan")
        print(f"  convT {cin}->{cout} N{N} {H}x{W} {dt} variant {v}: K_pad {d.K_pad} Cout_pad {d.Cout_pad} non-finite "
              f"{nan}/{y.numel()} rel err {err:.3e}", flush=True)


if __name__ == "__main__":
    for dt in (torch.bfloat16, torch.float32):
        for (N, H, W, cin, cout) in ((2, 40, 30, 144, 72), (2, 20, 15, 288, 144), (2, 32, 24, 192, 96),
                                     (2, 16, 12, 384, 192), (2, 8, 6, 768, 384), (2, 16, 12, 256, 128),
                                     (2, 32, 24, 128, 64)):
            one(N, H, W, cin, cout, dt, (0, 90, 61, 68, -1))

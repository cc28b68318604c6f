"""Generic implicit-GEMM kernel: Cout-tile choice on the layers it runs (developer tool, GPU).  Times the forced
generic kernel (variant -1) per HISEG_IGEMM_BCO tile width with HIP events and checks every tile gives the same
bits (the tile changes only which workgroup computes an output, never its accumulation order)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
from hiseg import ops  # noqa: E402

DEV = torch.device("cuda")
# (name, N, Cin, Cout, H, W, k)
SHAPES = [("b1_72to72_3x3_80x60", 32, 72, 72, 80, 60, 3), ("b1_144to144_3x3_40x30", 32, 144, 144, 40, 30, 3),
          ("b7_96to96_3x3_128x96", 8, 96, 96, 128, 96, 3), ("c3_16to96_1x1_320x320", 32, 16, 96, 320, 320, 1)]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dt = torch.bfloat16
    for name, N, Ci, Co, H, W, k in SHAPES:
        g = torch.Generator(device=DEV).manual_seed(5)
        x = ops.Act.from_nchw(torch.randn(N, Ci, H, W, device=DEV, generator=g), dt)
        w = torch.randn(Co, Ci, k, k, device=DEV, generator=g) / (Ci * k * k) ** 0.5
        p = ops.pack_conv(w, torch.randn(Co, device=DEV, generator=g) * 0.1, None, 1, dt, DEV, pad=k // 2)
        o = ops.Act.new(N, H, W, Co, dt, DEV, zero=False)
        flops = 2.0 * N * H * W * Co * Ci * k * k
        res, ref = [], None
        for bco in (None, "128", "64", "32", "16"):
            if bco is None:
                os.environ.pop("HISEG_IGEMM_BCO", None)
            else:
                os.environ["HISEG_IGEMM_BCO"] = bco
            fn = lambda: ops.conv2d(p, x, out=o, variant=-1)   # noqa: E731
            fn()
            torch.cuda.synchronize()
            same = True if ref is None else torch.equal(o.t, ref)
            if ref is None:
                ref = o.t.clone()
            us = timed(fn)
            res.append(f"{bco or 'auto'}: {us:7.1f} us {flops / us / 1e6:6.1f} TF{'' if same else ' (BITS DIFFER)'}")
        os.environ.pop("HISEG_IGEMM_BCO", None)
        auto = timed(lambda: ops.conv2d(p, x, out=o))
        print(f"{name:26s} automatic kernel {auto:7.1f} us | generic " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()

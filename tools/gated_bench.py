"""SE-gated 1x1 projections of the B7 teacher (distillation leg) -- timing of the alternatives (developer tool, GPU):
the gated conv as dispatched (variant 0: split-K igemm with the gate applied by the loader), the channel-scale pass
(bf16(h * gate), the loader's own rounding) followed by the ungated conv (variant 0 and the LDS-DMA ring kernel,
variant 61), and the ungated conv alone.  Reports us per launch (HIP events) and whether the premultiplied path
gives the gated conv's bits."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
from hiseg import ops  # noqa: E402

DEV = torch.device("cuda")
# (name, N, H, W, Cin, Cout, residual)
SHAPES = [("b7_s6_2304to384_20x20", 4, 20, 20, 2304, 384, True), ("b7_s7_3840to640_20x20", 4, 20, 20, 3840, 640, True),
          ("b7_s5_1344to224_40x40", 4, 40, 40, 1344, 224, True), ("b7_s4_960to160_40x40", 4, 40, 40, 960, 160, True),
          ("b7_s3_480to80_80x80", 4, 80, 80, 480, 80, True), ("b0_s6_1152to192_20x20", 4, 20, 20, 1152, 192, True)]


def timed(fn, reps=30):
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
    for name, N, H, W, Ci, Co, res in SHAPES:
        g = torch.Generator(device=DEV).manual_seed(3)
        x = ops.Act.from_nchw(torch.randn(N, Ci, H, W, device=DEV, generator=g), dt)
        gate = torch.rand(N, Ci, device=DEV, generator=g).contiguous()
        w = torch.randn(Co, Ci, 1, 1, device=DEV, generator=g) / Ci ** 0.5
        p = ops.pack_conv(w, torch.randn(Co, device=DEV, generator=g) * 0.1, None, 0, dt, DEV, pad=0)
        r = ops.Act.from_nchw(torch.randn(N, Co, H, W, device=DEV, generator=g), dt) if res else None
        o = ops.Act.new(N, H, W, Co, dt, DEV, zero=False)
        xs = ops.Act.new(N, H, W, Ci, dt, DEV, zero=False)
        gated = lambda: ops.conv2d(p, x, out=o, residual=r, in_scale=gate)   # noqa: E731
        scale = lambda: ops.channel_scale(x, gate)                         # noqa: E731
        un0 = lambda: ops.conv2d(p, xs, out=o, residual=r)                  # noqa: E731
        un61 = lambda: ops.conv2d(p, xs, out=o, residual=r, variant=61)     # noqa: E731
        gated()
        ref = o.t.clone()
        xs.t.copy_(scale().t)
        un0()
        same0 = torch.equal(o.t, ref)
        un61()
        same61 = torch.equal(o.t, ref)
        err61 = ((o.t.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        tg, ts, t0, t61 = timed(gated), timed(scale), timed(un0), timed(un61)
        os.environ["HISEG_IGEMM_LIN"] = "0"
        tg_nolin, tgen_nolin = timed(gated), timed(lambda: ops.conv2d(p, xs, out=o, residual=r, variant=-1))
        os.environ.pop("HISEG_IGEMM_LIN")
        tgen = timed(lambda: ops.conv2d(p, xs, out=o, residual=r, variant=-1))
        print(f"{name:24s} generic-kernel gather: gated {tg_nolin:7.1f} -> {tg:7.1f} us, ungated (variant -1) "
              f"{tgen_nolin:7.1f} -> {tgen:7.1f} us", flush=True)
        print(f"{name:24s} gated {tg:7.1f} us | scale {ts:6.1f} + ungated auto {t0:7.1f} (bits equal {same0}) "
              f"/ ring61 {t61:7.1f} (bits equal {same61}, rel err {err61:.1e})", flush=True)


if __name__ == "__main__":
    main()

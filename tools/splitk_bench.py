"""A/B timing of the deep SE-gated 1x1 projections (developer tool, GPU): the unsplit generic kernel (variant -1)
against the split-K generic kernel (variant 99) and the automatic choice, HIP events around each call; run under
`rocprofv3 --kernel-trace --stats` to split the split-K time into its GEMM and reduce kernels.
Usage: python tools/splitk_bench.py [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch  # noqa: E402

from hiseg import ops  # noqa: E402

DEV = "cuda"
# name: (N, Ca, Cout, H, W, in_scale, residual) -- the distillation step's B7 teacher / B0 student projections
CASES = {
    "b7_2304_384_20x20": (4, 2304, 384, 20, 20, True, True),
    "b7_3840_640_20x20": (4, 3840, 640, 20, 20, True, True),
    "b7_1344_224_40x40": (4, 1344, 224, 40, 40, True, True),
    "b7_960_160_40x40": (4, 960, 160, 40, 40, True, True),
    "b7_480_80_80x80": (4, 480, 80, 80, 80, True, True),
    "b7_288_48_160x160": (4, 288, 48, 160, 160, True, True),
    "b0_1152_192_20x20": (4, 1152, 192, 20, 20, True, True),
    "b0_672_112_40x40": (4, 672, 112, 40, 40, True, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="-1,99,0")
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--no-gate", action="store_true")
    args = ap.parse_args()
    dt = torch.bfloat16
    for name in args.cases.split(","):
        N, Ca, Cout, H, W, ins, res = CASES[name]
        ins = ins and not args.no_gate
        g = torch.Generator(device=DEV).manual_seed(0)
        xa = ops.Act.from_nchw(torch.randn(N, Ca, H, W, device=DEV, generator=g), dt)
        w = torch.randn(Cout, Ca, 1, 1, device=DEV, generator=g) / Ca ** 0.5
        p = ops.pack_conv(w, None, None, 0, dt, DEV, pad=0)
        gate = torch.rand(N, p.ca, device=DEV, generator=g) if ins else None
        R = ops.Act.from_nchw(torch.randn(N, Cout, H, W, device=DEV, generator=g), dt) if res else None
        out = ops.Act.new(N, H, W, Cout, dt, DEV, zero=False)
        row = []
        for v in [int(x) for x in args.variants.split(",")]:
            try:
                for _ in range(3):
                    ops.conv2d(p, xa, residual=R, in_scale=gate, out=out, variant=v)
            except Exception as e:  # variant 99 where the layer does not split
                row.append(f"v{v}: n/a")
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                ops.conv2d(p, xa, residual=R, in_scale=gate, out=out, variant=v)
            e1.record()
            torch.cuda.synchronize()
            row.append(f"v{v}: {e0.elapsed_time(e1) / args.reps * 1e3:7.1f} us")
        fl = 2.0 * N * H * W * Ca * Cout
        print(f"{name:22s} {fl / 1e9:6.2f} GFLOP  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()

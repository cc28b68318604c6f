"""Run one conv shape with one or more kernel variants R times each (developer tool, GPU), for
rocprofv3 --pmc / --kernel-trace passes over a single launch class.

Usage: python tools/conv_one.py --shape res256_3x3_64x48 --variants 61,40 [--reps 20]
Shapes are tools/conv_bench.SHAPES.

Diagnostic variants (timing-only, stamps, experimental kernels) need the DIAG=1 library:
`make -C human-instance-segmentation_amd DIAG=1` and HISEG_LIB=human-instance-segmentation_amd/hiseg/libhiseg_diag.so.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
import torch  # noqa: E402

import conv_bench as CB  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="res256_3x3_64x48")
    ap.add_argument("--variants", default="61")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    p, xa, xb, r, out = CB.make(CB.SHAPES[args.shape], torch.bfloat16)
    d = CB.desc(p, xa, xb, r, out)
    for v in [int(x) for x in args.variants.split(",")]:
        for _ in range(args.reps):
            CB.run(d, v)
        torch.cuda.synchronize()
    print("done", args.shape, args.variants, flush=True)


if __name__ == "__main__":
    main()

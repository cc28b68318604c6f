"""A/B timing of libhiseg conv kernel variants on the path's conv shapes (developer tool, GPU).

For every shape: checks each variant against the generic kernel (variant -1), then times all
variants in interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
Usage: python tools/conv_bench.py [--variants -1,0,1,2] [--reps 20] [--rounds 3]

Diagnostic variants (timing-only, stamps, experimental kernels) need the DIAG=1 library:
`make -C human-instance-segmentation_amd DIAG=1` and HISEG_LIB=human-instance-segmentation_amd/hiseg/libhiseg_diag.so.
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
import torch  # noqa: E402

from hiseg import _lib as L  # noqa: E402
from hiseg import ops  # noqa: E402

DEV = "cuda"
# name: (N, Ca, Cb, Cout, H, W, k, residual)
SHAPES = {
    "res256_3x3_64x48": (256, 256, 0, 256, 64, 48, 3, True),
    "c256to256_3x3_64x48": (256, 256, 0, 256, 64, 48, 3, False),
    "res128_3x3_128x96": (256, 128, 0, 128, 128, 96, 3, True),
    "c128to256_3x3_64x48": (256, 128, 0, 256, 64, 48, 3, False),
    "res64_3x3_64x48": (256, 64, 0, 64, 64, 48, 3, True),
    "dec_128+128to128_3x3_32x24": (256, 128, 128, 128, 32, 24, 3, False),
    "c256to256_1x1_64x48": (256, 256, 0, 256, 64, 48, 1, False),
    "comb_256+8to256_1x1_64x48": (256, 256, 8, 256, 64, 48, 1, False),
    "c128to256_1x1_64x48": (256, 128, 0, 256, 64, 48, 1, False),
    "res256_1x1_64x48": (256, 256, 0, 256, 64, 48, 1, True),
    "c256to64_3x3_64x48": (256, 256, 0, 64, 64, 48, 3, False),
    "res256_3x3_16x12": (256, 256, 0, 256, 16, 12, 3, True),
    "dec16_3x3_480x640": (32, 16, 0, 16, 480, 640, 3, False),
    "dec32_3x3_240x320": (32, 32, 0, 32, 240, 320, 3, False),
    "c16to96_1x1_240x320": (32, 16, 0, 96, 240, 320, 1, False),
    # the distillation teacher's (B7, 4 x 640 x 640) MBConv expansions
    "b7exp_48to288_1x1_160x160": (4, 48, 0, 288, 160, 160, 1, False),
    "b7exp_80to480_1x1_80x80": (4, 80, 0, 480, 80, 80, 1, False),
    "b7exp_160to960_1x1_40x40": (4, 160, 0, 960, 40, 40, 1, False),
    "b7exp_224to1344_1x1_40x40": (4, 224, 0, 1344, 40, 40, 1, False),
    "b7exp_384to2304_1x1_20x20": (4, 384, 0, 2304, 20, 20, 1, False),
    # smp decoder blocks 3/4 (nearest-x2 upsampled src A + skip), B0 at 480x640
    "dec3_up64+32to32_3x3_240x320": (32, 64, 32, 32, 240, 320, 3, False, 2),
    "dec4_up32to16_3x3_480x640": (32, 32, 0, 16, 480, 640, 3, False, 2),
    "dec3_b7_up64+64to32_3x3_240x320": (8, 64, 64, 32, 240, 320, 3, False, 2),
    # smp decoder blocks 0-2 with 64-multiple padded skips (round 3), B0 at 480x640 x 32 images
    "dec0_up320+128to256_3x3_30x40": (32, 320, 128, 256, 30, 40, 3, False, 2),
    "dec1_up256+64to128_3x3_60x80": (32, 256, 64, 128, 60, 80, 3, False, 2),
    "dec2_up128+64to64_3x3_120x160": (32, 128, 64, 64, 120, 160, 3, False, 2),
}


def make(shape, dt):
    N, Ca, Cb, Cout, H, W, k, res = shape[:8]
    up = shape[8] if len(shape) > 8 else 1
    g = torch.Generator(device=DEV).manual_seed(0)
    xa = ops.Act.new(N, H // up, W // up, Ca, dt, DEV, zero=False)
    xa.up = up
    xa.t.copy_(torch.randn(xa.t.numel(), device=DEV, generator=g))
    xb = None
    if Cb:
        xb = ops.Act.new(N, H, W, Cb, dt, DEV, zero=False)
        xb.t.copy_(torch.randn(xb.t.numel(), device=DEV, generator=g))
    w = torch.randn(Cout, Ca + Cb, k, k, device=DEV, generator=g) / ((Ca + Cb) * k * k) ** 0.5
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    p = ops.pack_conv(w, b, None, 1, dt, DEV, pad=k // 2, split=(Ca, Cb) if Cb else None)
    r = None
    if res:
        r = ops.Act.new(N, H, W, Cout, dt, DEV, zero=False)
        r.t.copy_(torch.randn(r.t.numel(), device=DEV, generator=g))
    out = ops.Act.new(N, H, W, Cout, dt, DEV, zero=False)
    return p, xa, xb, r, out


def desc(p, xa, xb, r, out):
    d = L.Conv2dDesc()
    d.dtype = d.out_dtype = ops.hdtype(xa.dtype)
    up = getattr(xa, "up", 1)
    d.N, d.H, d.W, d.Ho, d.Wo = xa.N, xa.H * up, xa.W * up, xa.H * up, xa.W * up
    d.KH, d.KW, d.stride, d.pad = p.kh, p.kw, 1, p.pad
    d.srcA, d.a_cstride, d.a_coff, d.Ca, d.a_up = xa.ptr(), xa.cstride, 0, p.ca, up
    if xb is not None:
        d.srcB, d.b_cstride, d.b_coff, d.Cb = xb.ptr(), xb.cstride, 0, p.cb
    d.weight, d.Cout, d.Cout_pad, d.K_pad = p.weight.data_ptr(), p.gemm_cols, p.cout_pad, p.k_pad
    d.scale, d.shift, d.act = p.scale.data_ptr(), p.shift.data_ptr(), p.act
    if r is not None:
        d.residual, d.r_cstride, d.r_coff = r.ptr(), r.cstride, 0
    d.out, d.o_cstride, d.o_coff = out.ptr(), out.cstride, 0
    if p.weight_frag is not None:
        d.weight_frag = p.weight_frag.data_ptr()
    return d


def run(d, v):
    L.check(L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), v, L.stream_ptr()), f"conv variant {v}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="-1,0,1,2,4")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--bitref", type=int, default=None, help="also report bit-equality against this variant")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    results = {}
    for name in args.shapes.split(","):
        shape = SHAPES[name]
        N, Ca, Cb, Cout, H, W, k, res = shape[:8]
        flops = 2.0 * N * H * W * Cout * k * k * (Ca + Cb)
        up = shape[8] if len(shape) > 8 else 1
        nbytes = 2.0 * N * (H * W // (up * up) * Ca + H * W * Cb + H * W * Cout * (2 if res else 1))
        p, xa, xb, r, out = make(shape, torch.bfloat16)
        d = desc(p, xa, xb, r, out)
        run(d, -1)
        torch.cuda.synchronize()
        ref = out.t.float().clone()
        ok, same = {}, {}
        bref = None
        if args.bitref is not None:
            out.t.fill_(float("nan"))
            run(d, args.bitref)
            torch.cuda.synchronize()
            bref = out.t.clone()
        for v in variants:
            out.t.fill_(float("nan"))
            run(d, v)
            torch.cuda.synchronize()
            err = ((out.t.float() - ref).abs().max() / ref.abs().max()).item()
            ok[v] = err
            if bref is not None:
                same[v] = bool(torch.equal(out.t, bref))
        times = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                for _ in range(3):
                    run(d, v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    run(d, v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps)
        row = {}
        for v in variants:
            ms = min(times[v])
            row[str(v)] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                           "alg_gbs": round(nbytes / ms / 1e6, 1), "rel_err_vs_generic": ok[v]}
            if v in same:
                row[str(v)]["bit_equal_ref"] = same[v]
        results[name] = row
        print(name, json.dumps(row), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/conv_bench.json", "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()

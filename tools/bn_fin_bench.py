"""Train-mode BatchNorm forward passes at the distillation student's encoder shapes (developer tool, GPU):
hiseg_bn_stats, hiseg_bn_finalize and hiseg_bn_apply (SiLU) timed separately, HIP events over --reps calls each,
under every --ab setting (the launcher reads HISEG_BN_FIN per call).

Usage: python tools/bn_fin_bench.py [--reps 50] [--ab HISEG_BN_FIN=0,HISEG_BN_FIN=2]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
import torch  # noqa: E402

from hiseg import _lib as L  # noqa: E402
from hiseg.ops import Act  # noqa: E402

# (pixels, channels): B0 at 4 x 640 x 640 -- stage resolutions 320, 160, 80, 40, 20
SHAPES = [(4 * 320 * 320, 32), (4 * 160 * 160, 144), (4 * 80 * 80, 240), (4 * 80 * 80, 40), (4 * 40 * 40, 480),
          (4 * 40 * 40, 672), (4 * 40 * 40, 112), (4 * 20 * 20, 1152), (4 * 20 * 20, 192), (4 * 20 * 20, 320)]


def timed(fn, reps):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--ab", default="HISEG_BN_FIN=0,HISEG_BN_FIN=2")
    a = ap.parse_args()
    lib = L.lib()
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    for P, C in SHAPES:
        H = W = int((P // 4) ** 0.5)
        z = Act.from_nchw(torch.randn(4, C, H, W, device=dev) * 2 + 0.5, torch.bfloat16)
        y = Act.new(4, H, W, C, torch.bfloat16, dev, zero=False)
        part = torch.empty(lib.hiseg_bn_partials() * 3 * C, device=dev)
        g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        outs = [torch.empty(C, device=dev) for _ in range(4)]
        d = L.BnApplyDesc()
        d.dtype, d.P, d.HW, d.C = 1, P, H * W, C
        d.z, d.z_cstride, d.z_coff = z, C, 0
        d.scale, d.shift = outs[2], outs[3]
        d.act, d.act_beta = L.ACT_SILU, 1.0
        d.y, d.y_cstride, d.y_coff = y, C, 0

        def stats():
            assert lib.hiseg_bn_stats(1, z.ptr(), P, C, C, 0, part.data_ptr(), s) == 0

        def fin():
            assert lib.hiseg_bn_finalize(part.data_ptr(), C, P, g.data_ptr(), b.data_ptr(), 1e-5, 0.1, rm.data_ptr(),
                                         rv.data_ptr(), *[o.data_ptr() for o in outs], s) == 0

        def apply():
            assert lib.hiseg_bn_apply(ctypes.byref(d), s) == 0

        stats()
        row = [f"stats {timed(stats, a.reps):6.1f} us", f"apply {timed(apply, a.reps):6.1f} us"]
        ref = None
        for st in a.ab.split(","):
            k, v = st.split("=", 1)
            os.environ[k] = v
            t = timed(fin, a.reps)
            fin()
            torch.cuda.synchronize()
            cur = torch.stack(outs[:2]).clone()
            dev_max = 0.0 if ref is None else ((cur - ref).abs() / ref.abs().clamp_min(1e-30)).max().item()
            ref = cur if ref is None else ref
            row.append(f"fin[{v}] {t:6.1f} us (rel {dev_max:.1e})")
        print(f"P={P:7d} C={C:5d}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()

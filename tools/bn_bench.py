"""HBM rate of the train-mode BatchNorm passes on the ROI head's shapes (developer tool, GPU).

Times hiseg_bn_stats (+finalize), hiseg_bn_apply and hiseg_bn_bwd (reduce + finalize + apply) with HIP
events on the launch stream and prints algorithmic GB/s per call (bytes each pass must move once).
Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split.
Usage: python tools/bn_bench.py [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
import torch  # noqa: E402

from hiseg import _lib as L  # noqa: E402

DEV = "cuda"
# name: (P, C, residual)
SHAPES = {
    "head256_64x48": (256 * 64 * 48, 256, False),
    "head256_64x48_res": (256 * 64 * 48, 256, True),
    "grid128_128x96": (256 * 128 * 96, 128, False),
    "grid128_128x96_res": (256 * 128 * 96, 128, True),
    "head64_64x48": (256 * 64 * 48, 64, False),
}


def timed(fn, reps):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    lib = L.lib()
    st = L.stream_ptr()
    out = {}
    for name in args.shapes.split(","):
        P, C, res = SHAPES[name]
        g = torch.Generator(device=DEV).manual_seed(0)
        mk = lambda: torch.randn(P * C, device=DEV, generator=g).to(torch.bfloat16)  # noqa: E731
        z, dy, y = mk(), mk(), mk()
        r = mk() if res else None
        dz = torch.empty_like(z)
        dres = torch.zeros_like(z) if res else None
        S = lib.hiseg_bn_partials()
        part = torch.empty((S + 1) * 3 * C, device=DEV)
        f = lambda: torch.empty(C, device=DEV)  # noqa: E731
        gamma, beta = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
        mean, invstd, scale, shift, dg, db = f(), f(), f(), f(), torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        bpe = P * C * 2

        def stats():
            L.check(lib.hiseg_bn_stats(L.HISEG_BF16, z.data_ptr(), P, C, C, 0, part.data_ptr(), st), "stats")
            L.check(lib.hiseg_bn_finalize(part.data_ptr(), C, P, gamma.data_ptr(), beta.data_ptr(), 1e-5, 0.1, None,
                                          None, mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(),
                                          shift.data_ptr(), st), "finalize")
        stats()

        ad = L.BnApplyDesc()
        ad.dtype, ad.P, ad.HW, ad.C = L.HISEG_BF16, P, 64 * 48, C
        ad.z, ad.z_cstride, ad.z_coff = z.data_ptr(), C, 0
        ad.scale, ad.shift = scale.data_ptr(), shift.data_ptr()
        if res:
            ad.residual, ad.r_cstride, ad.r_coff = r.data_ptr(), C, 0
        ad.act = L.ACT_RELU
        ad.y, ad.y_cstride, ad.y_coff = y.data_ptr(), C, 0

        def apply():
            L.check(lib.hiseg_bn_apply(ctypes.byref(ad), st), "apply")

        bd = L.BnBwdDesc()
        bd.dtype, bd.P, bd.HW, bd.C = L.HISEG_BF16, P, 64 * 48, C
        bd.dy, bd.dy_cstride, bd.dy_coff = dy.data_ptr(), C, 0
        bd.y, bd.y_cstride, bd.y_coff = y.data_ptr(), C, 0
        bd.z, bd.z_cstride, bd.z_coff = z.data_ptr(), C, 0
        bd.act = L.ACT_RELU
        bd.mean, bd.invstd, bd.gamma, bd.beta = mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr()
        bd.partial = part.data_ptr()
        bd.dgamma, bd.dbeta, bd.accumulate_params = dg.data_ptr(), db.data_ptr(), 1
        bd.dz, bd.dz_cstride, bd.dz_coff = dz.data_ptr(), C, 0
        if res:
            bd.dres, bd.dres_cstride, bd.dres_coff, bd.dres_accumulate = dres.data_ptr(), C, 0, 0
        else:
            bd.fwd_scale, bd.fwd_shift = scale.data_ptr(), shift.data_ptr()

        def bwd():
            L.check(lib.hiseg_bn_bwd(ctypes.byref(bd), st), "bwd")

        row = {}
        ms = timed(stats, args.reps)
        row["stats"] = {"ms": round(ms, 4), "GBps": round(bpe / ms / 1e6, 1)}
        ms = timed(apply, args.reps)
        nb = bpe * (3 if res else 2)
        row["apply"] = {"ms": round(ms, 4), "GBps": round(nb / ms / 1e6, 1)}
        ms = timed(bwd, args.reps)
        # reduce: dy, z (+ y when the mask comes from y); apply: dy, z (+y), dz (+dres)
        nb = bpe * ((3 + 5) if res else (2 + 3))
        row["bwd"] = {"ms": round(ms, 4), "GBps": round(nb / ms / 1e6, 1)}
        out[name] = row
        print(name, json.dumps(row), flush=True)
        del z, dy, y, r, dz, dres
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bn_bench.json", "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()

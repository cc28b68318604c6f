"""Train-mode BatchNorm element-wise passes at the ROI head's shapes (developer tool, GPU): hiseg_bn_apply (ReLU,
residual) and hiseg_bn_bwd (ReLU at the pre-activation, residual gradient) with one pixel per thread iteration
(HISEG_BN_U=1) and two (HISEG_BN_U=2); HIP events, GB/s of algorithmic bytes, bit-identity of the two forms."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
from hiseg import _lib as L  # noqa: E402

DEV = "cuda"
SHAPES = [("c256_64x48x256", 256 * 64 * 48, 256), ("c128_128x96x256", 256 * 128 * 96, 128),
          ("c64_64x48x256", 256 * 64 * 48, 64)]


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
    lib, st = L.lib(), L.stream_ptr()
    for name, P, C in SHAPES:
        g = torch.Generator(device=DEV).manual_seed(1)
        mk = lambda: torch.randn(P * C, device=DEV, generator=g).to(torch.bfloat16)   # noqa: E731
        z, res, dy = mk(), mk(), mk()
        y, dz, dres = (torch.empty(P * C, device=DEV, dtype=torch.bfloat16) for _ in range(3))
        scale, shift = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.1
        mean, invstd = torch.randn(C, device=DEV, generator=g) * 0.1, torch.rand(C, device=DEV, generator=g) + 0.5
        gamma, beta = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.1
        part = torch.empty((lib.hiseg_bn_partials() + 1) * 3 * C, device=DEV)
        dgamma, dbeta = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        a = L.BnApplyDesc()
        a.dtype, a.P, a.HW, a.C = L.HISEG_BF16, P, 64 * 48, C
        a.z, a.z_cstride, a.z_coff = z, C, 0
        a.scale, a.shift = scale, shift
        a.residual, a.r_cstride, a.r_coff = res, C, 0
        a.act, a.act_beta = 1, 1.0
        a.y, a.y_cstride, a.y_coff = y, C, 0
        b = L.BnBwdDesc()
        b.dtype, b.P, b.HW, b.C = L.HISEG_BF16, P, 64 * 48, C
        b.dy, b.dy_cstride, b.dy_coff = dy, C, 0
        b.y, b.y_cstride, b.y_coff = y, C, 0
        b.z, b.z_cstride, b.z_coff = z, C, 0
        b.act, b.act_beta = 1, 1.0
        b.mean, b.invstd, b.gamma, b.beta = mean, invstd, gamma, beta
        b.partial, b.dgamma, b.dbeta, b.accumulate_params = part, dgamma, dbeta, 0
        b.dz, b.dz_cstride, b.dz_coff = dz, C, 0
        b.dres, b.dres_cstride, b.dres_coff, b.dres_accumulate = dres, C, 0, 0
        b.fwd_scale, b.fwd_shift = scale, shift
        b.residual, b.r_cstride, b.r_coff = res, C, 0
        out, outs = [], {}
        for u in ("1", "2"):
            os.environ["HISEG_BN_U"] = u
            fa = lambda: L.check(lib.hiseg_bn_apply(ctypes.byref(a), st), "bn_apply")   # noqa: E731
            fb = lambda: L.check(lib.hiseg_bn_bwd(ctypes.byref(b), st), "bn_bwd")      # noqa: E731
            fa()
            fb()
            torch.cuda.synchronize()
            outs[u] = (y.clone(), dz.clone(), dres.clone())
            ta, tb = timed(fa), timed(fb)
            ab = P * C * 2 * 3 / ta / 1e3
            bb = P * C * 2 * 7 / tb / 1e3   # reduce: dy, z, residual; apply: dy, z, residual, write dz, dres
            out.append(f"U={u}: apply {ta:7.1f} us {ab:6.0f} GB/s  bwd {tb:7.1f} us {bb:6.0f} GB/s")
        same = all(torch.equal(p, q) for p, q in zip(outs["1"], outs["2"]))
        print(f"{name:18s} " + " | ".join(out) + f" | identical {same}", flush=True)


if __name__ == "__main__":
    main()

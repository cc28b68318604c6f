"""Weight-gradient kernel timing on the ROI head's train shapes (developer tool, GPU).

Times hiseg_conv2d_wgrad (the split-K MFMA pass) and hiseg_conv2d_wgrad_reduce with HIP events and prints
TFLOP/s of the pass, plus a checksum of the reduced gradient so runs under different HISEG_WGRAD_CFG values
(read once per process) can be compared.
Usage: HISEG_WGRAD_CFG=1 python tools/wgrad_bench.py [--reps 10]
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
# name: (N, Cin, Cout, H, W, k)
SHAPES = {
    "w256_3x3_64x48": (256, 256, 256, 64, 48, 3),
    "w128_3x3_128x96": (256, 128, 128, 128, 96, 3),
    "w64_3x3_64x48": (256, 64, 64, 64, 48, 3),
    "w128_3x3_64x48": (256, 128, 128, 64, 48, 3),
    "w128to256_3x3_64x48": (256, 128, 256, 64, 48, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    lib = L.lib()
    st = L.stream_ptr()
    out = {"cfg": os.environ.get("HISEG_WGRAD_CFG", "0")}
    for name in args.shapes.split(","):
        N, Cin, Cout, H, W, k = SHAPES[name]
        g = torch.Generator(device=DEV).manual_seed(3)
        x = torch.randn(N * H * W * Cin, device=DEV, generator=g).to(torch.bfloat16)
        dy = torch.randn(N * H * W * Cout, device=DEV, generator=g).to(torch.bfloat16)
        d = L.Conv2dDesc()
        d.dtype = d.out_dtype = L.HISEG_BF16
        d.N, d.H, d.W, d.Ho, d.Wo = N, H, W, H, W
        d.KH, d.KW, d.stride, d.pad = k, k, 1, k // 2
        d.srcA, d.a_cstride, d.a_coff, d.Ca, d.a_up = x.data_ptr(), Cin, 0, Cin, 1
        d.Cout, d.Cout_pad = Cout, Cout
        Cg, Kg, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        L.check(lib.hiseg_conv2d_wgrad_dims(ctypes.byref(d), 0, ctypes.byref(Cg), ctypes.byref(Kg), ctypes.byref(sp)),
                "dims")
        ws = torch.empty(sp.value * Cg.value * Kg.value, device=DEV)
        m = L.WgradMap()
        m.Cout, m.KH, m.KW = Cout, k, k
        m.ca, m.ca_real, m.cb, m.cb_real = Cin, Cin, 0, 0
        m.convT, m.Cg, m.Kg, m.want_bias = 0, Cg.value, Kg.value, 0
        gw = torch.zeros(Cout * Cin * k * k, device=DEV)

        def wg():
            L.check(lib.hiseg_conv2d_wgrad(ctypes.byref(d), dy.data_ptr(), Cout, 0, 0, ws.data_ptr(), sp.value, st), "wgrad")

        def red():
            L.check(lib.hiseg_conv2d_wgrad_reduce(ws.data_ptr(), sp.value, ctypes.byref(m), gw.data_ptr(), None, 0, st),
                    "reduce")

        res = {}
        for nm, fn in (("wgrad", wg), ("reduce", red)):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[nm] = round(e0.elapsed_time(e1) / args.reps, 4)
        flops = 2.0 * N * H * W * Cout * Cin * k * k
        res["tflops"] = round(flops / res["wgrad"] / 1e9, 1)
        res["splits"] = sp.value
        res["checksum"] = float(gw.double().abs().sum())
        out[name] = res
        print(name, json.dumps(res), flush=True)
        del x, dy, ws, gw
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/wgrad_bench_{out['cfg']}.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

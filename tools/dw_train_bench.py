"""Depthwise training kernels per layer of the unfrozen B0 student (developer tool, GPU): the weight gradient
(hiseg_dw_bwd_weight, split partials + reduce), the stride-2 data gradient (hiseg_dw_bwd_data) and the stride-1 data
gradient as the forward tile kernel with the rotated kernel (hiseg_dwconv_fwd), HIP events, median of --reps.

Usage: python tools/dw_train_bench.py [--reps 20] [--ab KEY=V1+KEY2=V1,KEY=V2+KEY2=V2]
(--ab: comma-separated settings, each a '+'-joined list of KEY=VALUE; every layer timed under each)"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
import torch  # noqa: E402

from hiseg import _lib as L  # noqa: E402
from hiseg.ops import Act  # noqa: E402

# the B0 student's 16 depthwise layers at 4 x 640 x 640 (C, K, stride, input H = W)
LAYERS = [(32, 3, 1, 320), (96, 3, 2, 320), (144, 3, 1, 160), (144, 5, 2, 160), (240, 5, 1, 80), (240, 3, 2, 80),
          (480, 3, 1, 40), (480, 5, 1, 40), (672, 5, 1, 40), (672, 5, 2, 40), (1152, 5, 1, 20), (1152, 3, 1, 20)]
BF16 = 1


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ab", default="")
    a = ap.parse_args()
    lib = L.lib()
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    settings = [[kv.split("=", 1) for kv in st.split("+")] for st in a.ab.split(",")] if a.ab else [None]
    N = 4
    for C, K, st, H in LAYERS:
        Ho = (H + 2 * (K // 2) - K) // st + 1
        x = Act.from_nchw(torch.randn(N, C, H, H, device=dev), torch.bfloat16)
        dz = Act.from_nchw(torch.randn(N, C, Ho, Ho, device=dev), torch.bfloat16)
        w = torch.randn(C, K * K, device=dev) * 0.2
        dw = torch.zeros(C, K * K, device=dev)
        one, zero = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        gx = Act.new(N, H, H, C, torch.bfloat16, dev, zero=False)
        row = []
        for kv in settings:
            for key, val in kv or []:
                os.environ[key] = val
            nws = int(lib.hiseg_dw_bwd_weight_ws(BF16, N, Ho, Ho, C, K))
            ws = torch.empty(max(nws, 1), device=dev)

            def wgrad():
                assert lib.hiseg_dw_bwd_weight(BF16, x.ptr(), dz.ptr(), N, H, H, C, K, st, Ho, Ho, ws.data_ptr(),
                                               dw.data_ptr(), s) == 0

            if st == 1:
                wf = w.reshape(C, K, K).flip(1, 2).reshape(C, K * K).t().contiguous()

                def dgrad():
                    assert lib.hiseg_dwconv_fwd(BF16, dz.ptr(), N, H, H, C, K, 1, wf.data_ptr(), one.data_ptr(),
                                                zero.data_ptr(), 0, gx.ptr(), H, H, s) == 0
            else:
                def dgrad():
                    assert lib.hiseg_dw_bwd_data(BF16, dz.ptr(), N, H, H, C, K, st, w.data_ptr(), Ho, Ho, gx.ptr(), 0,
                                                 s) == 0
            for _ in range(3):
                wgrad()
                dgrad()
            tag = "[" + "/".join(v for _, v in kv) + "]" if kv is not None else ""
            row.append(f"wgrad{tag} {timed(wgrad, a.reps):7.1f} us  dgrad{tag} {timed(dgrad, a.reps):7.1f} us "
                       f"(ws {nws * 4 / 1e6:.1f} MB)")
        print(f"c{C:<5d} k{K} s{st} {H:4d}^2   " + "   ".join(row), flush=True)


if __name__ == "__main__":
    main()

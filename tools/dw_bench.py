"""Depthwise conv timing per EfficientNet layer shape (developer tool, GPU): the automatic choice, the LDS-tiled kernel
forced for every layer (HISEG_DWCONV_T=2) and the register-gather kernel (HISEG_DWCONV_T=0), HIP events, algorithmic GB/s (input + output read / written once).

Usage: python tools/dw_bench.py [--reps 20] [--shapes a,b] [--modes 1,2,0] [--ab HISEG_DWCONV_FW=0,HISEG_DWCONV_FW=1]
(--ab: each mode timed once per listed environment setting, in order; the launcher reads them per call)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
import torch  # noqa: E402

from hiseg import ops  # noqa: E402

# (name, N, H, W, C, k, stride): the distillation step's B7 teacher / B0 student stages at 640 x 640, 4 images
SHAPES = [("b7_s2_k3s2_c192", 4, 320, 320, 192, 3, 2), ("b7_s2_k3s1_c288", 4, 160, 160, 288, 3, 1),
          ("b7_s3_k5s2_c288", 4, 160, 160, 288, 5, 2), ("b7_s3_k5s1_c480", 4, 80, 80, 480, 5, 1),
          ("b7_s4_k3s1_c960", 4, 40, 40, 960, 3, 1), ("b7_s5_k5s1_c1344", 4, 40, 40, 1344, 5, 1),
          ("b7_s6_k5s1_c2304", 4, 20, 20, 2304, 5, 1), ("b7_s7_k3s1_c3840", 4, 20, 20, 3840, 3, 1),
          ("b0_s1_k3s1_c32", 4, 320, 320, 32, 3, 1), ("b0_s3_k5s1_c240", 4, 80, 80, 240, 5, 1),
          ("c2_b0_s2_k3s1_c144", 32, 120, 160, 144, 3, 1), ("c2_b0_s3_k5s1_c240", 32, 60, 80, 240, 5, 1),
          ("c2_b0_s1_k3s1_c32", 32, 240, 320, 32, 3, 1), ("c2_b0_s2_k3s2_c96", 32, 240, 320, 96, 3, 2),
          ("c2_b0_s3_k5s2_c144", 32, 120, 160, 144, 5, 2), ("c2_b0_s4_k3s2_c240", 32, 60, 80, 240, 3, 2),
          ("c2_b0_s6_k5s1_c1152", 32, 15, 20, 1152, 5, 1), ("b7_s1_k3s1_c64", 4, 320, 320, 64, 3, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--modes", default="1,2,0", help="HISEG_DWCONV_T values: 1 auto, 2 LDS tile, 0 gather")
    ap.add_argument("--ab", default="", help="comma-separated KEY=VALUE settings, each mode timed under each")
    a = ap.parse_args()
    dt = torch.bfloat16
    for name, N, H, W, C, k, st in SHAPES:
        if a.shapes and name not in a.shapes.split(","):
            continue
        x = ops.Act.from_nchw(torch.randn(N, C, H, W, device="cuda"), dt)
        w = (torch.randn(k * k, C, device="cuda") * 0.3).contiguous()
        sc, sh = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        cr = max(1, C // 24)
        w1, b1 = torch.randn(cr, C, device="cuda") * 0.1, torch.zeros(cr, device="cuda")
        w2, b2 = torch.randn(C, cr, device="cuda") * 0.1, torch.zeros(C, device="cuda")
        Ho, Wo = (H + 2 * (k // 2) - k) // st + 1, (W + 2 * (k // 2) - k) // st + 1
        nbytes = (N * H * W * C + N * Ho * Wo * C) * 2
        row = []
        settings = [kv.split("=", 1) for kv in a.ab.split(",")] if a.ab else [None]
        for mode, kv in [(m, kv) for m in a.modes.split(",") for kv in settings]:
            os.environ["HISEG_DWCONV_T"] = mode
            if kv is not None:
                os.environ[kv[0]] = kv[1]
            for _ in range(3):
                ops.dwconv_se_gate(x, w, sc, sh, k, st, 3, w1, b1, w2, b2, 3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                ops.dwconv(x, w, sc, sh, k, st, 3)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            tag = {'1': 'auto', '2': 'lds', '0': 'gather'}[mode] + (f"[{kv[1]}]" if kv is not None else "")
            row.append(f"{tag} {ms * 1e3:8.1f} us {nbytes / ms / 1e6:7.0f} GB/s")
        print(f"{name:22s} " + "   ".join(row), flush=True)


if __name__ == "__main__":
    main()

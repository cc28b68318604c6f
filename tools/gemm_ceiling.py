"""Practical bf16 MFMA ceiling on this box (developer tool, GPU): torch.matmul (hipBLASLt / rocBLAS) on the dominant
conv class's GEMM shape -- M = 256 ROIs x 64 x 48 pixels, N = 256 output channels, K = 9 x 256 -- and on a square
8192^3 GEMM, random bf16 data, HIP events over 20 launches after 5 warm-ups.  The dominant conv's TFLOP/s read
against these (not only against the 2.5 PF dense peak, which assumes a 2.4 GHz clock the chip does not hold under
MFMA load: MI355X_MICROARCH.md "DVFS give-back").
Usage: python tools/gemm_ceiling.py
"""
import json

import torch


def bench(m, n, k, reps=20):
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16, generator=g)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del c
    return {"m": m, "n": n, "k": k, "ms": round(ms, 4), "tflops": round(2.0 * m * n * k / ms / 1e9, 1)}


def main():
    out = {"dominant_conv_gemm (786432 x 256 x 2304)": bench(256 * 64 * 48, 256, 9 * 256),
           "dominant_conv_gemm_T (256 x 786432 x 2304)": bench(256, 256 * 64 * 48, 9 * 256),
           "square_8192": bench(8192, 8192, 8192)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

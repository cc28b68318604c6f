"""Per-layer conv timing of one bench step (developer tool, GPU).

Records every hiseg_conv2d_fwd launch of one RGBHierarchicalExportWrapper step of the bench
workload (ops.RECORD), replays each descriptor alone (HIP events, median of --reps), and prints
the layers grouped by shape with time, TFLOP/s and algorithmic GB/s.
Usage: python tools/layer_profile.py [--reps 5] [--variant 0]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "human-instance-segmentation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

import bench  # noqa: E402
from hiseg import _lib as L  # noqa: E402
from hiseg import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variant", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    model = bench.build_model(dev, torch.bfloat16)
    images, rois = bench.synthetic_batch(dev, 0)
    import hiseg
    wrap = hiseg.RGBHierarchicalExportWrapper(model)
    with torch.no_grad():
        wrap(images, rois)
        torch.cuda.synchronize()
        ops.RECORD = []
        wrap(images, rois)
        torch.cuda.synchronize()
    rec, ops.RECORD = ops.RECORD, None
    groups = {}
    total = 0.0
    for d, keep, p, flops in rec:
        def run():
            L.check(L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), args.variant, L.stream_ptr()), "replay")
        run()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[len(ts) // 2]
        esz = 2 if d.dtype == 1 else 4
        osz = 2 if d.out_dtype == 1 else 4
        px_in = d.N * d.H * d.W
        px_out = d.N * d.Ho * d.Wo
        cout = p.cout
        byts = px_in * (d.Ca + d.Cb) * esz / (d.a_up * d.a_up) + p.weight.numel() * esz
        byts += px_out * (4 if d.convT else 1) * cout * osz * (2 if d.out2 else 1)
        if d.residual:
            byts += px_out * cout * esz
        if d.mul:
            byts += px_out * cout * esz
        key = (f"k{d.KH}x{d.KW} s{d.stride} up{d.a_up} {d.Ca}+{d.Cb}->{d.Cout}(pad{d.Cout_pad}) "
               f"{d.N}x{d.Ho}x{d.Wo}{' T' if d.convT else ''}{' res' if d.residual else ''}"
               f"{' f32out' if d.out_dtype == 0 else ''}{' ins' if d.in_scale else ''}")
        g = groups.setdefault(key, {"n": 0, "ms": 0.0, "flops": flops, "bytes": byts})
        g["n"] += 1
        g["ms"] += ms
        total += ms
    rows = sorted(groups.items(), key=lambda kv: -kv[1]["ms"])
    print(f"{len(rec)} conv launches, replayed total {total:.2f} ms")
    out = []
    for k, g in rows:
        avg = g["ms"] / g["n"]
        tf = g["flops"] / avg / 1e9
        gbs = g["bytes"] / avg / 1e6
        print(f"{g['ms']:8.3f} ms {g['n']:3d}x {avg*1e3:8.1f}us {tf:7.1f} TF {gbs:7.0f} GB/s  {k}")
        out.append({"layer": k, "launches": g["n"], "ms": g["ms"], "avg_us": avg * 1e3, "tflops": tf, "gbps": gbs})
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/layer_profile.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""Is the inference leg's slowdown after the train legs a software state or the GPU's thermal / clock state?
(developer tool, GPU).  Runs the C2 inference leg, then the given legs, then inference again
immediately, then again after an idle pause.  Usage: python tools/order_probe.py [--pause S] [--legs c4,train]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pause", type=float, default=20.0)
    ap.add_argument("--legs", default="train,c3,c4")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ia = argparse.Namespace(steps=20, warmup=5, serial=False, no_cpu_baseline=True, gpus=1, dtype="bf16")

    def infer(tag):
        r = bench.infer_bench(ia, dev, torch.bfloat16, 0, 1, None)
        bench._release_leg()
        print(f"{tag}: {r['value']} ROI-masks/s, dominant {r['roofline']['avg_launch_ms']} ms", flush=True)

    infer("first")
    for leg in a.legs.split(","):
        kw = {"train": {}, "c3": dict(preset="b1", batch=32, rois_per_img=1, hw=(640, 640)),
              "c4": dict(preset="b7", batch=8, rois_per_img=1, hw=(640, 640))}[leg]
        t = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 10, 2, graph_train=True, **kw)
        bench._release_leg()
        print(f"{leg}: {t['ms_per_step']} ms", flush=True)
    infer("right after")
    time.sleep(a.pause)
    infer(f"after {a.pause:.0f} s idle")
    infer("again")


if __name__ == "__main__":
    main()

"""Developer check (GPU): the C3 train leg before and after bench.py's inference leg, same process."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def c3(dev):
    torch.cuda.empty_cache()
    r = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 5, 2, preset="b1", batch=32, rois_per_img=1, hw=(640, 640))
    return r["ms_per_step"], r["call_profile"]["step_ms_probed"]


def main():
    dev = torch.device("cuda", 0)
    print("C3 first", c3(dev), flush=True)
    args = argparse.Namespace(serial=False, warmup=3, steps=10)
    out = bench.infer_bench(args, dev, torch.bfloat16, 0, 1, None)
    print("infer", out["value"], flush=True)
    print("C3 after infer", c3(dev), flush=True)
    print("C3 again", c3(dev), flush=True)
    torch.cuda.synchronize()
    print("mem", torch.cuda.memory_reserved() / 1e9, torch.cuda.memory_allocated() / 1e9, flush=True)


if __name__ == "__main__":
    main()

"""Developer check (GPU): the C3 train leg before and after bench.py's inference leg, same process."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def c3(dev, per_step=True):
    torch.cuda.empty_cache()
    m0 = torch.cuda.memory_stats()
    bench.STEP_TIMES = [] if per_step else None
    r = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 8, 2, preset="b1", batch=32, rois_per_img=1, hw=(640, 640))
    st = bench.STEP_TIMES or []
    bench.STEP_TIMES = None
    per = [round((b - a) * 1e3, 1) for a, b in zip([0.0] + st[:-1], st)]
    m1 = torch.cuda.memory_stats()
    seg = {k: m1.get(k, 0) - m0.get(k, 0) for k in ("segment.all.allocated", "segment.all.freed", "num_alloc_retries",
                                                     "num_device_alloc", "num_device_free")}
    return r["ms_per_step"], r["call_profile"]["step_ms_probed"], per, seg


def main():
    dev = torch.device("cuda", 0)
    print("C3 first", c3(dev, False), flush=True)
    args = argparse.Namespace(serial=False, warmup=3, steps=10)
    out = bench.infer_bench(args, dev, torch.bfloat16, 0, 1, None)
    print("infer", out["value"], flush=True)
    print("C3 after infer", c3(dev, False), flush=True)
    print("C3 again", c3(dev, False), flush=True)
    print("C3 per-step sync", c3(dev, True), flush=True)
    torch.cuda.synchronize()
    print("mem", torch.cuda.memory_reserved() / 1e9, torch.cuda.memory_allocated() / 1e9, flush=True)


if __name__ == "__main__":
    main()

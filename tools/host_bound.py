"""Is the C2 inference step host-bound?  Times the Python enqueue of K pipelined steps (until
StreamPipelinedExport.run returns, no synchronize) against the wall time until the GPU finishes
(developer tool, GPU).  Usage: python tools/host_bound.py [--steps 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import hiseg
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, torch.bfloat16)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = bench.synthetic_batch(dev, 0)
    pipe = hiseg.StreamPipelinedExport(wrapper)
    with torch.no_grad():
        for _ in range(3):
            pipe.run([(images, rois)] * 2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.run([(images, rois)] * args.steps)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"enqueue {1e3 * (t1 - t0) / args.steps:.2f} ms/step, wall {1e3 * (t2 - t0) / args.steps:.2f} ms/step",
                  flush=True)


if __name__ == "__main__":
    main()

"""A/B of the C2 serving schedules (developer tool, GPU): serial wrapper vs StreamPipelinedExport with default /
prioritised streams, interleaved rounds in one process.  Usage: python tools/pipeline_ab.py [--steps 10]"""
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
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import hiseg
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, torch.bfloat16)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = bench.synthetic_batch(dev, 0)
    runners = {"serial": None, "pipe": hiseg.StreamPipelinedExport(wrapper, head_priority=False)}
    pr = hiseg.StreamPipelinedExport(wrapper)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    pr.s_head = torch.cuda.Stream(priority=-1)
    pr.s_unet = torch.cuda.Stream(priority=0)
    runners["pipe_headprio"] = pr
    pu = hiseg.StreamPipelinedExport(wrapper)
    pu.s_head = torch.cuda.Stream(priority=0)
    pu.s_unet = torch.cuda.Stream(priority=-1)
    runners["pipe_unetprio"] = pu
    # UNet stream restricted to a CU subset (bit patterns striped over the 8 words = 256 CUs)
    for name, word in (("pipe_unet_3of4", 0x77777777), ("pipe_unet_half", 0x55555555), ("pipe_unet_quarter", 0x11111111)):
        runners[name] = hiseg.StreamPipelinedExport(wrapper, unet_cu_mask=[word] * 8, head_priority=False)
    res = {k: [] for k in runners}
    with torch.no_grad():
        for _ in range(args.rounds):
            for name, r in runners.items():
                def go(k):
                    if r is None:
                        for _ in range(k):
                            wrapper(images, rois)
                    else:
                        r.run([(images, rois)] * k)
                go(2)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                go(args.steps)
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) / args.steps * 1e3)
    for k, v in res.items():
        print(f"{k:14s} ms/step min {min(v):.2f} all {[round(x, 2) for x in v]}", flush=True)


if __name__ == "__main__":
    main()

"""Distillation step time after K other streams exist in the process (developer tool, GPU): the concurrent teacher
stream ran 9.8 ms in a process of its own and 16.6 ms at the end of the full bench (which creates streams per leg);
HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues.
Usage: python tools/stream_probe.py K [--prio]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    k = int(sys.argv[1])
    if "--prio" in sys.argv:   # the teacher branch on the high-priority stream (its own queue and priority level)
        from hiseg import streams
        streams.ROLE["teacher"] = "head"
    dev = torch.device("cuda", 0)
    keep = []
    if "--hiprio-first" in sys.argv:   # as the C2 inference leg's head stream
        hp = torch.cuda.Stream(priority=-1)
        with torch.cuda.stream(hp):
            torch.zeros(16, device=dev).add_(1)
        keep.append(hp)
    if "--mem" in sys.argv:   # the train legs leave tens of GB cached in the allocator
        big = [torch.empty(8 << 30, dtype=torch.uint8, device=dev) for _ in range(8)]
        del big
    if "--train-first" in sys.argv:
        t = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 2, 2, graph_train=True)
        print(f"train first: {t['ms_per_step']} ms", flush=True)
        torch.cuda.empty_cache()
    if "--infer-first" in sys.argv:
        import argparse
        a = argparse.Namespace(steps=4, warmup=2, serial=False, no_cpu_baseline=True, gpus=1, dtype="bf16")
        try:
            r0 = bench.infer_bench(a, dev, torch.bfloat16, 0, 1, None)
            print(f"infer first: {r0.get('value')}", flush=True)
        except Exception as e:   # (attribute names of the bench's own args)
            print(f"infer first failed: {e!r}", flush=True)
        torch.cuda.empty_cache()
    for _ in range(k):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.zeros(16, device=dev).add_(1)
        keep.append(s)
    torch.cuda.synchronize()
    r = bench.distill_bench(dev, torch.bfloat16, 0, 1, None, 10, 3)
    print(f"streams before {k} {' '.join(sys.argv[2:])}: {r['ms_per_step']} ms", flush=True)


if __name__ == "__main__":
    main()

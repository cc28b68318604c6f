"""Sequence probe for the bench legs' process-state sensitivity (developer tool, GPU).
Runs the given actions in one process and prints one line each: legs `infer`, `infer_serial`, `train`, `c3`, `c4`,
`distill`; `empty` (torch.cuda.empty_cache), `gc`, `copy` (median of three 512 MB device copies), `mem` (reserved
GB), `sleep:S`.  Between actions the cache is kept unless `empty` says otherwise.
Usage: python tools/leg_probe.py infer,copy,distill"""
import argparse
import gc
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("seq")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    for act in a.seq.split(","):
        ts = f"[{time.perf_counter() - t0:6.1f}s]"
        if act == "hp":   # bind a high-priority stream to a hardware queue (one tiny kernel on it), nothing else
            hs = torch.cuda.Stream(priority=-1)
            with torch.cuda.stream(hs):
                torch.ones(1, device=dev).add_(1)
            torch.cuda.synchronize()
            print(f"{ts} hp stream bound", flush=True)
        elif act == "hp_destroyed":   # the same through a raw HIP stream that is destroyed again
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            h = ctypes.c_void_p()
            assert hip.hipStreamCreateWithPriority(ctypes.byref(h), 0, -1) == 0
            with torch.cuda.stream(torch.cuda.ExternalStream(h.value)):
                torch.ones(1, device=dev).add_(1)
            torch.cuda.synchronize()
            assert hip.hipStreamDestroy(h) == 0
            print(f"{ts} hp stream bound and destroyed", flush=True)
        elif act == "infer_normal":   # the inference leg with its head on a normal-priority stream
            from hiseg import streams as HS
            HS._PRIORITY.pop("head", None)
            ia = argparse.Namespace(steps=20, warmup=5, serial=False, no_cpu_baseline=True, gpus=1, dtype="bf16")
            r = bench.infer_bench(ia, dev, torch.bfloat16, 0, 1, None)
            gc.collect()
            print(f"{ts} {act}: {r['value']} ROI-masks/s, dominant {r['roofline']['avg_launch_ms']} ms", flush=True)
        elif act in ("infer", "infer_serial"):
            ia = argparse.Namespace(steps=20, warmup=5, serial=act == "infer_serial", no_cpu_baseline=True, gpus=1,
                                    dtype="bf16")
            r = bench.infer_bench(ia, dev, torch.bfloat16, 0, 1, None)
            gc.collect()
            print(f"{ts} {act}: {r['value']} ROI-masks/s, dominant {r['roofline']['avg_launch_ms']} ms", flush=True)
        elif act in ("train", "c3", "c4"):
            kw = {"train": {}, "c3": dict(preset="b1", batch=32, rois_per_img=1, hw=(640, 640)),
                  "c4": dict(preset="b7", batch=8, rois_per_img=1, hw=(640, 640))}[act]
            r = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 10, 2, graph_train=True, **kw)
            gc.collect()
            print(f"{ts} {act}: {r['ms_per_step']} ms", flush=True)
        elif act == "distill":
            from hiseg import _lib as HL
            HL.placement_stats(reset=True)
            r = bench.distill_bench(dev, torch.bfloat16, 0, 1, None, 10, 3)
            gc.collect()
            dec, far = HL.placement_stats(reset=True)
            print(f"{ts} distill: {r['ms_per_step']} ms (placement-dependent choices: {dec} declined, {far} far; "
                  f"reserved {torch.cuda.memory_reserved() / 2**30:.1f} GB)", flush=True)
        elif act == "empty":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            print(f"{ts} empty", flush=True)
        elif act == "gc":
            gc.collect()
        elif act == "copy":
            print(f"{ts} copy: {bench._copy_probe_ms():.3f} ms", flush=True)
        elif act == "mem":
            print(f"{ts} mem: reserved {torch.cuda.memory_reserved() / 2**30:.1f} GB, allocated "
                  f"{torch.cuda.memory_allocated() / 2**30:.1f} GB", flush=True)
        elif act.startswith("sleep:"):
            time.sleep(float(act[6:]))
        else:
            raise SystemExit(f"unknown action {act}")


if __name__ == "__main__":
    main()

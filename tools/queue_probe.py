"""Stream -> hardware-queue mapping of the graphed distillation step (developer tool, GPU).

The replayed two-branch distillation step (teacher on a side stream) measured 9.5-10 ms in a process of its own but
13.5-17 ms after the train legs.  HIP maps every stream (torch's pool streams, and the streams a graph executor
creates for a graph's parallel branches) onto GPU_MAX_HW_QUEUES hardware queues, and two branches on one in-order
queue cannot overlap.  Run:
    rocprofv3 --kernel-trace --output-format csv -d OUT -o t -- python tools/queue_probe.py run [--train-first]
    python tools/queue_probe.py parse OUT/.../t_kernel_trace.csv [--last N]
`run` prints the distillation step time; `parse` reports, for the last N kernels of the trace (the distillation
leg's timed replays: it runs last), the queues they ran on, how long each queue was busy and how much of the
queues' busy time overlapped."""
import csv
import os
import sys


def run():
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench
    dev = torch.device("cuda", 0)
    if "--b0-first" in sys.argv:
        t = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 4, 2, graph_train=True)
        print(f"b0 train first: {t['ms_per_step']} ms", flush=True)
        bench._release_leg()
    if "--train-first" in sys.argv:
        t = bench.train_bench(dev, torch.bfloat16, 0, 1, None, 2, 2, graph_train=True, preset="b7", batch=8,
                              rois_per_img=1, hw=(640, 640))
        print(f"c4 first: {t['ms_per_step']} ms", flush=True)
        bench._release_leg()
    if "--infer-first" in sys.argv:
        import argparse
        a = argparse.Namespace(steps=4, warmup=2, serial=False, no_cpu_baseline=True, gpus=1, dtype="bf16")
        r0 = bench.infer_bench(a, dev, torch.bfloat16, 0, 1, None)
        print(f"infer first: {r0.get('value')}", flush=True)
        bench._release_leg()
    r = bench.distill_bench(dev, torch.bfloat16, 0, 1, None, 10, 3)
    print(f"distill: {r['ms_per_step']} ms", flush=True)
    if "--infer-after" in sys.argv:
        import argparse
        bench._release_leg()
        a = argparse.Namespace(steps=10, warmup=3, serial=False, no_cpu_baseline=True, gpus=1, dtype="bf16")
        r0 = bench.infer_bench(a, dev, torch.bfloat16, 0, 1, None)
        print(f"infer after: {r0.get('value')}", flush=True)


def _union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def parse(path, last):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-last:]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    span = max(e for _, e in iv) - min(s for s, _ in iv)
    byq = {}
    for r, v in zip(rows, iv):
        byq.setdefault((r.get("Queue_Id"), r.get("Stream_Id")), []).append(v)
    print(f"last {len(rows)} kernels: span {span / 1e6:.2f} ms, busy (union) {_union(iv) / 1e6:.2f} ms, "
          f"sum of kernel times {sum(e - s for s, e in iv) / 1e6:.2f} ms")
    qs = 0
    for q, v in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        u = _union(v)
        qs += u
        print(f"  queue {q[0]} stream {q[1]}: {len(v)} kernels, busy {u / 1e6:.2f} ms")
    print(f"  overlap between queues: {(qs - _union(iv)) / 1e6:.2f} ms")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        n = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 3500
        parse(sys.argv[2], n)

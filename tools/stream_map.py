"""Which of torch's pool streams run concurrently with which (developer tool, GPU).
Two streams on one hardware queue serialise: a 3-ms spin on each takes ~6 ms together instead of ~3.  Prints the
overlap table of the null stream and the first 8 low-priority pool streams, then (with --distill K,..) times the
graphed distillation step with the teacher's side stream forced to pool stream K."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def pair_ms(s1, s2, cycles):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    main = torch.cuda.current_stream()
    e0.record(main)
    for s in (s1, s2):
        s.wait_stream(main)
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    main.wait_stream(s1)
    main.wait_stream(s2)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--distill", default="")
    ap.add_argument("--n", type=int, default=8)
    a = ap.parse_args()
    null = torch.cuda.default_stream()
    pool = [torch.cuda.Stream() for _ in range(a.n)]
    hi = torch.cuda.Stream(priority=-1)
    cyc = 3_000_000
    one = pair_ms(null, null, cyc) / 2
    print(f"one spin: {one:.2f} ms", flush=True)
    names = ["null"] + [f"p{i}" for i in range(a.n)] + ["hi0"]
    ss = [null] + pool + [hi]
    for i, s1 in enumerate(ss):
        row = []
        for j, s2 in enumerate(ss):
            row.append("  -" if i == j else f"{pair_ms(s1, s2, cyc) / one:4.1f}")
        print(f"{names[i]:>5} " + " ".join(row), flush=True)
    if a.distill:
        import bench
        import hiseg.distill as D
        dev = torch.device("cuda", 0)
        for k in [int(x) for x in a.distill.split(",")]:
            D.DistillationUNetWrapper._side = lambda self, device, _s=pool[k]: _s
            r = bench.distill_bench(dev, torch.bfloat16, 0, 1, None, 10, 3)
            print(f"distill, teacher on p{k}: {r['ms_per_step']} ms", flush=True)


if __name__ == "__main__":
    main()

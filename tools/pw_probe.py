"""GPU time of conv kernel variants on small-M layer shapes without host launch overhead (developer tool, GPU).

tools/conv_bench.py times back-to-back C-ABI calls from Python, which for the EfficientNet encoder's small layers
(a few microseconds of GPU work) measures the host's call rate.  Here each variant's `reps` launches are captured
into one HIP graph and the graph is replayed: the event interval is GPU time.  Run it under
`rocprofv3 --kernel-trace --stats` for per-kernel durations.
Usage: python tools/pw_probe.py [--variants 0,90] [--shapes a,b] [--reps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
import conv_bench as CB  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,90")
    ap.add_argument("--shapes", default="b7exp_224to1344_1x1_40x40")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    out = {}
    # calibration: a one-element kernel per graph node (the graph's own per-node cost)
    x = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(args.reps):
            x.add_(1)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print("graph_node_us", round(e0.elapsed_time(e1) / args.reps * 1e3, 2), flush=True)
    for name in args.shapes.split(","):
        shape = CB.SHAPES[name]
        N, Ca, Cb, Cout, H, W, k, res = shape[:8]
        flops = 2.0 * N * H * W * Cout * k * k * (Ca + Cb)
        nbytes = 2.0 * N * H * W * (Ca + Cb + Cout * (2 if res else 1))
        p, xa, xb, r, o = CB.make(shape, torch.bfloat16)
        d = CB.desc(p, xa, xb, r, o)
        CB.run(d, -1)
        torch.cuda.synchronize()
        ref = o.t.clone()
        row = {}
        for v in variants:
            o.t.fill_(float("nan"))
            CB.run(d, v)
            torch.cuda.synchronize()
            same = bool(torch.equal(o.t, ref))
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(args.reps):
                    CB.run(d, v)
            best = None
            for _ in range(args.rounds):
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.reps
                best = ms if best is None else min(best, ms)
            row[str(v)] = {"us": round(best * 1e3, 2), "tflops": round(flops / best / 1e9, 1),
                           "alg_gbs": round(nbytes / best / 1e6, 1), "bit_equal_generic": same}
        out[name] = row
        print(name, json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

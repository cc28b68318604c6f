"""Where the distillation step's device-to-device copies come from (developer tool, GPU).  Counts, per hiseg source
line, the calls of torch.Tensor.copy_ / clone / contiguous (that copied) / torch.cat during one eager distillation
step.  Usage: python tools/copy_probe.py [--unfrozen N]"""
import argparse
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

COUNTS = collections.Counter()
ON = [False]


def where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "hiseg" in fr.filename or "bench.py" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno}"
    return "?"


def wrap(owner, name):
    orig = getattr(owner, name)

    def f(*a, **k):
        out = orig(*a, **k)
        if ON[0]:
            t = a[0] if a and isinstance(a[0], torch.Tensor) else None
            if t is not None and t.is_cuda:
                if name != "contiguous" or out.data_ptr() != t.data_ptr():
                    COUNTS[(name, where())] += 1
        return out
    setattr(owner, name, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--unfrozen", type=int, default=0)
    a = ap.parse_args()
    for n in ("copy_", "clone", "contiguous"):
        wrap(torch.Tensor, n)
    orig_cat = torch.cat

    def cat(*x, **k):
        if ON[0]:
            COUNTS[("cat", where())] += 1
        return orig_cat(*x, **k)
    torch.cat = cat
    dev = torch.device("cuda", 0)
    import hiseg.distill as D
    real_fwd = D.DistillationUNetWrapper.forward
    calls = [0]

    def fwd(self, x):
        calls[0] += 1
        ON[0] = True
        return real_fwd(self, x)
    D.DistillationUNetWrapper.forward = fwd
    bench.distill_bench(dev, torch.bfloat16, 0, 1, None, 2, 2, graph=False, unfrozen=a.unfrozen)
    print(f"forward calls: {calls[0]} (counts below include every step from the first forward on)")
    for (n, w), c in COUNTS.most_common(40):
        print(f"{c:5d} {n:10s} {w}")


if __name__ == "__main__":
    main()

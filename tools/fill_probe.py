"""Diagnostic (GPU): test_graphed_train_step_equals_eager's eager schedule under tools/fill_alloc.so, an allocator
that fills every new allocation with one byte pattern (HISEG_FILL_BYTE, default 0xFF = NaN in bf16 / f32) and
never reuses memory.  Prints the step losses and, for the first step whose gradient is not finite or differs from
the expected losses, the parameters with non-finite gradients (developer tool; build the allocator with
hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/fill_alloc.cpp -o tools/fill_alloc.so)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.environ.get("HISEG_FILL_ALLOC", "1") != "0":   # 0: PyTorch's caching allocator (the reference run)
    alloc = torch.cuda.memory.CUDAPluggableAllocator(os.path.join(ROOT, "tools", "fill_alloc.so"), "fill_malloc",
                                                     "fill_free")
    torch.cuda.memory.change_current_allocator(alloc)

sys.argv.append("--no-graph")
import graph_probe  # noqa: E402

EXPECT = [4.503585338592529, 4.332995414733887, 4.0903239250183105, 3.9231648445129395]   # with the mask fix


def main():
    losses, grads, params, names = graph_probe.run(False, None)
    print("fill byte", os.environ.get("HISEG_FILL_BYTE", "0xFF"), "losses", losses, "expected", EXPECT, flush=True)
    for k in range(4):
        g = grads[k]
        off, bad = 0, []
        for n, c in names:
            if not torch.isfinite(g[off:off + c]).all():
                bad.append(n)
            off += c
        print(f"step {k}: {len(bad)} non-finite grads; first {bad[:6]}; last {bad[-4:]}", flush=True)
    if "--save" in sys.argv:   # step-1 gradient and parameters after it, for tools/fill_compare.py
        torch.save({"grad0": grads[0].cpu(), "param0": params[0].cpu(), "names": names, "losses": losses},
                   sys.argv[sys.argv.index("--save") + 1])


if __name__ == "__main__":
    main()

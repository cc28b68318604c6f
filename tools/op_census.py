"""Census of the torch-side device ops (copies, fills, allocating zeros) one distillation step issues (developer
tool, GPU).  Every aten op of the kind below that runs on a CUDA tensor during one eager step is counted by the
innermost hiseg / bench source line that issued it -- the copyBuffer / FillFunctor launches of the graphed step's
kernel trace, attributed.
Usage: python tools/op_census.py [--unfrozen N]"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402,F401  (sets up sys.path for hiseg / filler)

KINDS = ("copy_", "fill_", "zero_", "zeros", "zeros_like", "full", "clone", "cat", "_to_copy", "index_put_", "ones",
         "new_zeros", "masked_fill_", "copy")


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.n = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        out = func(*args, **(kwargs or {}))
        if name in KINDS:
            dev = [a for a in list(args) + list((kwargs or {}).values()) + [out] if isinstance(a, torch.Tensor)]
            if any(t.is_cuda for t in dev):
                where = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if ("hiseg" in fr.filename or "bench.py" in fr.filename) and "op_census" not in fr.filename:
                        where = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                        break
                self.n[(name, where)] += 1
        return out


def main():
    unfrozen = int(sys.argv[sys.argv.index("--unfrozen") + 1]) if "--unfrozen" in sys.argv else 0
    import filler
    import hiseg
    dev = torch.device("cuda", 0)
    model, loss_fn = hiseg.create_unet_distillation_model("timm-efficientnet-b0", "timm-efficientnet-b7",
                                                          teacher_checkpoint="absent.pth", device="cpu",
                                                          progressive_unfreeze=True)
    filler.fill_module(model.student, seed=11)
    filler.fill_module(model.teacher, seed=12)
    hiseg.set_compute_dtype(model, torch.bfloat16)
    model = model.to(dev).train()
    loss_fn.temperature = 4.0
    x = torch.randn(4, 3, 640, 640, device=dev)
    m = (torch.rand(4, 1, 640, 640, device=dev) > 0.5).float()
    enc = model.unfreeze_encoder_blocks(unfrozen, learning_rate_scale=0.1) if unfrozen else None
    opts = [hiseg.FusedAdamW(model.student, lr=1e-4, weight_decay=1e-4, max_grad_norm=1.0,
                             params=model.student.get_decoder_parameters())]
    if enc:
        opts.append(hiseg.FusedAdamW(model.student, lr=1e-5, weight_decay=1e-4, max_grad_norm=None, params=enc))

    def step():
        s, t = model(x)
        loss, _ = loss_fn(s, t, m)
        for o in opts:
            o.zero_grad()
        loss.backward()
        for o in opts:
            o.step()

    step()
    step()
    torch.cuda.synchronize()
    c = Census()
    with c:
        step()
    torch.cuda.synchronize()
    tot = collections.Counter()
    for (name, where), k in c.n.most_common():
        tot[name] += k
        print(f"{k:5d} {name:12s} {where}")
    print("totals", dict(tot), flush=True)


if __name__ == "__main__":
    main()

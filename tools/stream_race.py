"""Developer diagnostic (GPU): the same fresh-model bf16 train step issued under different stream schedules.

Prints, per schedule, the losses of 4 steps and a checksum of the parameters / optimizer moments after each
step, so a schedule-dependent result shows the step at which it first appears.  Schedules:
  default      every step on the default stream
  default2     the same again (run-to-run determinism)
  side         every step under one side stream
  fresh        every step on a fresh side stream (GraphedStep's eager phase)
  fresh_sync   fresh side stream + device synchronize after every step
  graphed      hiseg.GraphedStep
  poison_nan   default stream; before every step the caching allocator's free blocks are filled with NaN
  poison_rand  the same with random values (an uninitialised read then changes the result)
  lds_nan      default stream; before every libhiseg call every CU's LDS is filled with NaN (f32 and bf16)
  lds_big      the same with 8.5e37 (f32 and bf16): a kernel reading LDS it did not write then changes
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import filler  # noqa: E402
import hiseg  # noqa: E402
from helpers import b0_kwargs  # noqa: E402

DEV = "cuda"


def build():
    torch.manual_seed(0)
    m = hiseg.create_rgb_hierarchical_model(**hiseg_kwargs())
    filler.fill_module(m)
    hiseg.set_compute_dtype(m, torch.bfloat16)
    m = m.to(DEV).train()
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    return m


def hiseg_kwargs():
    from helpers import hiseg_kwargs as hk
    return hk(b0_kwargs())


def checksum(m, opt):
    p = torch.cat([q.detach().float().reshape(-1) for q in m.parameters()])
    bufs = torch.cat([b.detach().float().reshape(-1) for n, b in m.named_buffers() if b.is_floating_point()])
    out = [float(p.double().sum()), float(p.double().abs().sum()), float(bufs.double().sum())]
    if opt is not None and opt.exp_avg is not None:
        out += [float(opt.exp_avg.double().abs().sum()), float(opt.exp_avg_sq.double().sum()), opt.step_count]
    return out


def poison(kind):
    """Fill (most of) the caching allocator's free memory with a pattern, then free it again."""
    held = []
    sizes = [256 << 10] * 2000 + [(2 << 20) * k for k in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128)] * 6
    for n in sizes:
        t = torch.empty(n // 4, dtype=torch.float32, device=DEV)
        if kind == "nan":
            t.fill_(float("nan"))
        else:
            t.uniform_(-1e3, 1e3)
        held.append(t)
    del held


class LdsPoison:
    """Wrap every libhiseg entry point: fill all LDS with `pattern` right before the call (same stream)."""

    def __init__(self, pattern):
        from hiseg import _lib as L
        self.lib, self.real, self.pattern = L.lib(), {}, pattern
        fill = self.lib.hiseg_debug_fill_lds
        for name in L.EXPORTED:
            if not name.startswith("hiseg_") or name == "hiseg_debug_fill_lds":
                continue
            fn = getattr(self.lib, name)
            self.real[name] = fn

            def wrap(*a, _f=fn):
                fill(self.pattern, 2, L.stream_ptr())
                return _f(*a)
            setattr(self.lib, name, wrap)

    def close(self):
        for name, fn in self.real.items():
            setattr(self.lib, name, fn)


def run(schedule, steps=4):
    images = torch.from_numpy(filler.uniform(31, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(32, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(33, 4, 128, 96)).to(DEV)
    m = build()
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    st = {"opt": None}

    def step():
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if st["opt"] is None:
            st["opt"] = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
        st["opt"].zero_grad()
        loss.backward()
        st["opt"].step()
        return loss

    side = torch.cuda.Stream()
    lp = None
    if schedule.startswith("lds"):
        lp = LdsPoison(0x7FC07FC0 if schedule == "lds_nan" else 0x7E807E80)
    gs = hiseg.GraphedStep(step, lambda: st["opt"]) if schedule == "graphed" else None
    rows = []
    for i in range(steps):
        if schedule.startswith("lds"):
            loss = step()
        elif schedule.startswith("poison"):
            poison(schedule.split("_")[1])
            loss = step()
        elif schedule.startswith("default"):
            loss = step()
        elif schedule == "side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                loss = step()
            torch.cuda.current_stream().wait_stream(side)
        elif schedule.startswith("fresh"):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                loss = step()
            torch.cuda.current_stream().wait_stream(s)
            if schedule == "fresh_sync":
                torch.cuda.synchronize()
        else:
            loss = gs()
        torch.cuda.synchronize()
        rows.append((float(loss.detach()), checksum(m, st["opt"])))
    if lp is not None:
        lp.close()
    return rows


def main():
    scheds = sys.argv[1:] or ["default", "default2", "side", "fresh", "fresh_sync", "graphed"]
    res = {}
    for s in scheds:
        res[s] = run(s)
        print(s, flush=True)
        for i, (l, c) in enumerate(res[s]):
            print(f"  step {i}: loss {l:.6f} sums {['%.6g' % x for x in c]}", flush=True)
    base = res[scheds[0]]
    for s in scheds[1:]:
        first = next((i for i, (a, b) in enumerate(zip(base, res[s])) if a != b), None)
        print(f"{s}: first differing step vs {scheds[0]}: {first}")


if __name__ == "__main__":
    main()

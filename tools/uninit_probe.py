"""Diagnostic (GPU): repeat parts of one B0 train step with the caching allocator's free memory poisoned with
different random patterns in between, and report which part's results change -- an uninitialised read
(developer tool).  Parts: the train-mode forward (logits + aux), the loss forward on fixed logits, the backward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import filler  # noqa: E402
import hiseg  # noqa: E402
from ddp_diff import poison  # noqa: E402
from test_gpu_train import _model  # noqa: E402

DEV = "cuda"


def main():
    m = _model(torch.bfloat16).to(DEV).train()
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    images = torch.from_numpy(filler.uniform(41, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(42, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(43, 4, 128, 96)).to(DEV)
    for mod in m.modules():   # dropout off: masks would differ per step by design
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    logits0, aux0 = m(images, rois)
    torch.cuda.synchronize()
    ref = {k: v.detach().clone() for k, v in aux0.items() if torch.is_tensor(v)}
    ref["logits"] = logits0.detach().clone()
    # 1) the forward, repeated
    for seed in range(1, 9):
        poison(seed)
        lg, ax = m(images, rois)
        torch.cuda.synchronize()
        cur = {k: v.detach() for k, v in ax.items() if torch.is_tensor(v)}
        cur["logits"] = lg.detach()
        bad = {k: (cur[k].float() - ref[k].float()).abs().max().item() for k in ref if not torch.equal(cur[k], ref[k])}
        print(f"forward poison {seed}: differing outputs {bad}", flush=True)
    # 2) the loss on fixed inputs, repeated (fresh loss object each time: first-call state)
    lref = None
    for seed in range(1, 9):
        poison(seed)
        loss_fn = hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)
        lg = logits0.detach().clone().requires_grad_(True)
        loss, parts = loss_fn(lg, tgt, {k: v.detach() for k, v in aux0.items() if torch.is_tensor(v)})
        loss.backward()
        torch.cuda.synchronize()
        vals = (float(loss.detach()), lg.grad.detach().clone())
        if lref is None:
            lref = vals
        print(f"loss poison {seed}: loss {vals[0]:.7f} (ref {lref[0]:.7f}), grad max diff "
              f"{(vals[1] - lref[1]).abs().max().item():.3e}", flush=True)
    backward_probe(m, images, rois, tgt)


def backward_probe(m, images, rois, tgt):
    """3) the whole step (forward, a fresh loss, backward), repeated: flat gradient vs the first run."""
    gref = None
    fref = None
    for seed in range(1, 13):
        poison(seed)
        loss_fn = hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)
        from hiseg import ops
        ops.RECORD = []
        lg, ax = m(images, rois)
        torch.cuda.synchronize()
        rec = []
        for dc, keep, p, fl in ops.RECORD:
            o = next(k for k in keep if hasattr(k, "ptr") and k.ptr() == dc.out)
            rec.append((dc, o.t.clone()))
        ops.RECORD = None
        # the output Act is keep[2] (xa, xb, out, ...) when present: compare every recorded launch's output
        rec = [(dc, k) for dc, k in rec]
        if seed == 1:
            rref = rec
        else:
            for idx, ((dc, o), (_, o0)) in enumerate(zip(rec, rref)):
                if not torch.equal(o, o0):
                    print(f"   first differing conv launch #{idx}: N{dc.N} {dc.H}x{dc.W} Ca{dc.Ca} Cb{dc.Cb} -> {dc.Cout} "
                          f"k{dc.KH} a_up{dc.a_up} in_scale {bool(dc.in_scale)} res {bool(dc.residual)} "
                          f"max diff {(o.float() - o0.float()).abs().max().item():.3e}", flush=True)
                    break
        outs = {k: v.detach().clone() for k, v in ax.items() if torch.is_tensor(v)}
        outs["logits"] = lg.detach().clone()
        if seed == 1:
            fref = outs
        fbad = {k: (outs[k].float() - fref[k].float()).abs().max().item() for k in fref
                if not torch.equal(outs[k], fref[k])}
        loss, _ = loss_fn(lg, tgt, ax)
        for p in m.parameters():
            p.grad = None
        loss.backward()
        torch.cuda.synchronize()
        print(f"   forward outputs differing: {fbad}", flush=True)
        S = m.__dict__["_hiseg_train"]
        g = S.flat.grad.clone()
        if gref is None:
            gref = g
            offs, off = [], 0
            for n, p in S.flat.named:
                offs.append((n, off, p.numel()))
                off += p.numel()
        d = (g - gref).abs()
        bad = [(n, round(d[o:o + k].max().item(), 6)) for n, o, k in offs if d[o:o + k].max().item() > 0]
        print(f"step poison {seed}: loss {float(loss.detach()):.7f} max diff {d.max().item():.3e}; "
              f"{len(bad)} params differ, last in forward order: {bad[-8:]}", flush=True)


if __name__ == "__main__":
    main()

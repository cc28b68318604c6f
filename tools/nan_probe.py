"""GPU probe: repeated train forward/backward of one preset on the same process (no optimizer step in between),
reporting per call the loss and which parameter gradients are non-finite (developer tool, round 4)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
                os.path.join(ROOT, "tests"), ROOT]
import torch  # noqa: E402

import filler  # noqa: E402


def install_fwd_check():
    """Check every train-path conv forward's output (valid channels) for non-finite values right after it."""
    from hiseg import train_engine as TE
    orig = TE.conv_fwd
    seen = set()

    def checked(S, p, xa, xb=None, **kw):
        out, d = orig(S, p, xa, xb, **kw)
        torch.cuda.synchronize()
        v = out.t.view(out.N, out.H, out.W, out.cstride)[..., out.coff:out.coff + out.C]
        ins = [bool(torch.isfinite(a.t.view(a.N, a.H, a.W, a.cstride)[..., a.coff:a.coff + a.C]).all())
               for a in (xa, xb) if a is not None]
        if not torch.isfinite(v).all():
            key = (tuple(p.conv.weight.shape), xa.N, xa.H, xa.W, xb is not None, p.convT)
            if key not in seen:
                seen.add(key)
                bad = (~torch.isfinite(v)).nonzero()
                print(f"   NON-FINITE conv output: weight {tuple(p.conv.weight.shape)} convT {p.convT} in "
                      f"{xa.N}x{xa.H}x{xa.W} Ca {xa.C}/{xa.cstride} Cb {xb.C if xb is not None else 0} -> "
                      f"{out.C}/{out.cstride}; inputs finite {ins}; {bad.shape[0]} bad, first {bad[:4].tolist()}",
                      flush=True)
        return out, d
    TE.conv_fwd = checked


def run(preset, dt, H, W, n, calls, step_opt):
    import hiseg
    from helpers import configs, hiseg_kwargs
    m = hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(dict(configs()[preset]["model_kwargs"])))
    filler.fill_module(m)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    hiseg.set_compute_dtype(m, dt)
    m = m.cuda().train()
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = H, W
    mh, mw = configs()[preset]["model_kwargs"]["mask_size"]
    images = torch.from_numpy(filler.uniform(401, (n, 3, H, W))).cuda()
    rois = torch.from_numpy(filler.box_rois(402, n, 1)).cuda()
    tgt = torch.from_numpy(filler.ellipse_targets(403, n, mh, mw)).cuda()
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    opt = None
    names = [k for k, p in m.named_parameters() if p.requires_grad]
    for c in range(calls):
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        opt = opt or hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
        opt.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
        bad = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        fin_aux = {k: bool(torch.isfinite(v).all()) for k, v in aux.items() if torch.is_tensor(v)}
        print(f"{preset} {dt} call {c}: loss {float(loss):.6f} logits finite {bool(torch.isfinite(logits).all())} "
              f"non-finite aux {[k for k, v in fin_aux.items() if not v]} non-finite grads {len(bad)}/{len(names)}",
              flush=True)
        if bad:
            print("   last (forward order) non-finite:", bad[-12:], flush=True)
            print("   first finite after them:", [k for k in names[names.index(bad[-1]) + 1:][:5]], flush=True)
        if step_opt:
            opt.step()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="b7")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--hw", default="96,128")
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--step", action="store_true")
    ap.add_argument("--fill", action="store_true", help="NaN-filled, never reused allocations (tools/fill_alloc.so)")
    ap.add_argument("--check-fwd", action="store_true")
    a = ap.parse_args()
    if a.fill:
        alloc = torch.cuda.memory.CUDAPluggableAllocator(os.path.join(ROOT, "tools", "fill_alloc.so"), "fill_malloc",
                                                         "fill_free")
        torch.cuda.memory.change_current_allocator(alloc)
    if a.check_fwd:
        install_fwd_check()
    H, W = (int(v) for v in a.hw.split(","))
    run(a.preset, torch.bfloat16 if a.dtype == "bf16" else torch.float32, H, W, a.n, a.calls, a.step)

"""Per-call GPU time of one B0-std train step, grouped by C-ABI entry point and layer shape (developer tool, GPU).

Wraps every hiseg_* entry point of the loaded library with HIP events on the launch stream, runs one train
step of bench.py's B0-std workload (after warm-up steps), and prints the calls grouped by (entry point, shape):
conv forward / data-gradient convs (told apart by the caller), weight gradients (with the kernel family the
library picks: transposed-read or the register-transpose fallback), BN passes, loss, optimiser.
Usage: python tools/train_layer_profile.py [--warmup 2]
"""
import argparse
import ctypes
import json
import os
import re
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "human-instance-segmentation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

import bench  # noqa: E402
from hiseg import _lib as L  # noqa: E402


def entry_points():
    names = set()
    inc = os.path.join(ROOT, "include")
    for f in os.listdir(inc):
        if f.endswith(".h"):
            names |= set(re.findall(r"\bint\s+(hiseg_\w+)\s*\(", open(os.path.join(inc, f)).read()))
    return sorted(names)


def conv_key(d):
    return (f"k{d.KH}x{d.KW} s{d.stride} {d.Ca}+{d.Cb}->{d.Cout} {d.N}x{d.Ho}x{d.Wo}"
            f"{' T' if d.convT else ''}{' res' if d.residual else ''}{' f32out' if d.out_dtype == 0 else ''}")


def wgrad_family(d, want_bias):
    """The kernel family csrc/train_conv.hip wgrad_tr_try picks (shape rules only)."""
    tr = (d.dtype == 1 and (d.Cb == 0 or (d.Ca % 128 == 0 and (d.KH * d.KW == 1 or d.Cb % 128 == 0)))
          and (not d.convT or d.Cout % 32 == 0))
    return "tr" if tr else "legacy"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--leg", default="train", choices=["train", "distill", "unet", "head"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.leg == "distill":
        step = distill_step(dev)
    elif args.leg in ("unet", "head"):
        step = infer_phase(dev, args.leg)
    else:
        step = train_step(dev)
    profile(step, args.warmup)


def infer_phase(dev, leg):
    """One phase of bench.py's C2 inference step (engine.export_unet_phase / export_head_phase), no grad."""
    import hiseg
    from hiseg import engine
    model = bench.build_model(dev, torch.bfloat16)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = bench.synthetic_batch(dev, 0)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = bench.H, bench.W
    with torch.no_grad():
        u, _ = engine.export_unet_phase(model, images)

    def step():
        with torch.no_grad():
            if leg == "unet":
                engine.export_unet_phase(model, images)
            else:
                engine.export_head_phase(model, images, rois, u, wrapper.dilation_pixels)
    return step


def distill_step(dev):
    """bench.py's C5 distillation step (B7 teacher eval + B0 student decoder-only phase, 4 x 640x640)."""
    import filler
    import hiseg
    model, loss_fn = hiseg.create_unet_distillation_model("timm-efficientnet-b0", "timm-efficientnet-b7",
                                                          teacher_checkpoint="absent.pth", device="cpu",
                                                          progressive_unfreeze=True)
    filler.fill_module(model.student, seed=11)
    filler.fill_module(model.teacher, seed=12)
    hiseg.set_compute_dtype(model, torch.bfloat16)
    model = model.to(dev).train()
    loss_fn.temperature = 4.0
    x = torch.randn(4, 3, 640, 640, generator=torch.Generator().manual_seed(100)).to(dev)
    m = (torch.rand(4, 1, 640, 640, generator=torch.Generator().manual_seed(101)) > 0.5).float().to(dev)
    opt = hiseg.FusedAdamW(model.student, lr=1e-4, weight_decay=1e-4, max_grad_norm=1.0,
                           params=model.student.get_decoder_parameters())

    def step():
        s, t = model(x)
        loss, _ = loss_fn(s, t, m)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return step


def train_step(dev):
    import filler
    import hiseg
    model = bench.build_model(dev, torch.bfloat16).train()
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = bench.H, bench.W
    images, rois = bench.synthetic_batch(dev, 0)
    tgt = torch.from_numpy(filler.ellipse_targets(7, int(rois.shape[0]), *bench.MASK_HW)).to(dev)
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    opt = hiseg.FusedAdamW(model, lr=1e-4, weight_decay=0.01, max_grad_norm=1.0)

    def step():
        logits, aux = model(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return step


def profile(step, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()

    lib = L.lib()
    rec = []
    real = {}
    for name in entry_points():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            continue
        real[name] = fn

        def wrap(*a, _n=name, _f=fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = _f(*a)
            e1.record()
            key = ""
            if _n in ("hiseg_conv2d_fwd", "hiseg_conv2d_fwd_variant"):
                d = a[0]._obj
                caller = sys._getframe(1).f_code.co_name
                key = ("dgrad " if caller == "_dgrad_launch" else "fwd ") + conv_key(d)
            elif _n == "hiseg_conv2d_wgrad":
                d = a[0]._obj
                key = f"{wgrad_family(d, a[4])} {conv_key(d)}{' bias' if a[4] else ''}"
            elif _n in ("hiseg_dwconv_gap_fwd", "hiseg_dwconv_fwd"):
                # (dtype, in, N, H, W, C, K, stride, ...): algorithmic bytes = input + output activations (bf16)
                N, H, W, C, K, st = a[2], a[3], a[4], a[5], a[6], a[7]
                Ho, Wo = (H + 2 * (K // 2) - K) // st + 1, (W + 2 * (K // 2) - K) // st + 1
                key = f"k{K} s{st} C{C} {N}x{H}x{W} MB {2 * N * C * (H * W + Ho * Wo) / 1e6:.1f}"
            elif _n in ("hiseg_bn_stats",):
                key = f"P{a[2]} C{a[3]} MB {2 * a[2] * a[3] / 1e6:.1f}"
            rec.append((_n, key, e0, e1))
            return r
        setattr(lib, name, wrap)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    step()
    t1.record()
    torch.cuda.synchronize()
    for name, fn in real.items():
        setattr(lib, name, fn)
    step_ms = t0.elapsed_time(t1)
    groups = {}
    for n, k, e0, e1 in rec:
        g = groups.setdefault((n, k), [0, 0.0])
        g[0] += 1
        g[1] += e0.elapsed_time(e1)
    tot = sum(g[1] for g in groups.values())
    print(f"step {step_ms:.2f} ms (event-bracketed); {len(rec)} C-ABI calls, {tot:.2f} ms inside them")
    byname = {}
    for (n, k), g in groups.items():
        byname[n] = byname.get(n, 0.0) + g[1]
    for n, ms in sorted(byname.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{ms:8.3f} ms  {n}")
    print("---- by shape")
    out = []
    for (n, k), g in sorted(groups.items(), key=lambda kv: -kv[1][1])[:70]:
        print(f"{g[1]:8.3f} ms {g[0]:3d}x {g[1] / g[0] * 1e3:8.1f}us  {n} {k}")
        out.append({"call": n, "key": k, "count": g[0], "ms": g[1]})
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.environ.get("HISEG_PROFILE_OUT", "gpurun_out/train_layer_profile.json"), "w") as f:
        json.dump({"step_ms": step_ms, "rows": out}, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Headline benchmark: ROI-masks/s of the exported RGB hierarchical contract on MI355X.

Workload (BASELINE.json configs[1], "C2"): B0 EfficientNet-UNet + refined hierarchical head,
640x480 images, batch 32 per GPU x 8 ROIs per image (256 ROI masks per step), ROI 64x48,
mask 128x96, bf16 compute, synthetic data, deterministic random-init weights of that
architecture.  One step = RGBHierarchicalExportWrapper forward: full-image UNet, 2x RoIAlign,
ROI head, instance_masks [256,1,128,96] + binary_masks [32,1,480,640].

Schedule: hiseg.StreamPipelinedExport -- the full-image UNet of step k+1 runs on a second HIP stream while
the ROI head of step k runs (HBM/latency-bound depthwise/SE/decoder kernels beside MFMA-bound 256-channel
convs); every step still runs the complete contract (--serial: one stream).

Multi-GPU: one process per GPU (torch.distributed.run), each rank processes its own 32 images
(weak scaling, no data-path collective); barrier + synchronize around the K timed steps and the
max over ranks of the elapsed time.

Second measurement, reported under "train" in the same JSON line (the metric's "train step/s"): one
training step of the same B0-std model on the same 32-image x 8-ROI batch per GPU -- frozen full-image
UNet forward, train-mode ROI path (batch-statistics BN, Dropout2d), RefinedHierarchicalLoss with the
boundary/contour/distance terms, the hand-written backward, FusedAdamW (clip 1.0) -- with the gradients
averaged over the ranks by hiseg.distributed (bucketed RCCL all-reduce overlapped with the backward) when
N > 1.

Third, under "distill": the C5 B7 -> B0 distillation step (decoder-only phase) of 4 640x640 images per GPU.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--no-train] [--no-distill]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "human-instance-segmentation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import torch  # noqa: E402

METRIC = "ROI-masks/sec (fwd) + train step/s, B0 640×480×8-ROI, 1/2/4/8 MI355X"
B, R, H, W = 32, 8, 480, 640
ROI_HW, MASK_HW = (64, 48), (128, 96)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E (MI355X_MICROARCH.md)
# Algorithmic work per ROI mask: head 53.1 GFLOP (inference graph) + B0 UNet 27.7/8
GFLOP_PER_ROI_MASK = 53.1 + 27.7 / 8
# Algorithmic work per training sample: B0-std head fwd+bwd 173.5 GFLOP + UNet fwd per ROI
GFLOP_PER_TRAIN_ROI = 173.5 + 27.7 / 8

B0_KWARGS = dict(
    roi_size=ROI_HW, mask_size=MASK_HW, multi_scale=False, use_attention_module=True,
    use_boundary_refinement=False, use_progressive_upsampling=False, use_subpixel_conv=False,
    use_contour_detection=True, use_distance_transform=True, normalization_type="batchnorm",
    normalization_groups=8, activation_function="relu", activation_beta=1.0, use_pretrained_unet=True,
    pretrained_weights_path="ext_extractor/best_model_b0_0.8741.pth", freeze_pretrained_weights=True,
    use_full_image_unet=True, encoder_name="timm-efficientnet-b0", hierarchical_base_channels=64,
    hierarchical_depth=3)


def build_model(device, dtype):
    import filler
    import hiseg
    model = hiseg.create_rgb_hierarchical_model(**B0_KWARGS)
    filler.fill_module(model).eval()
    model = model.to(device)
    hiseg.set_compute_dtype(model, dtype)
    return model


def synthetic_batch(device, rank):
    import filler
    g = torch.Generator().manual_seed(rank)
    images = torch.rand(B, 3, H, W, generator=g).to(device)
    rois = torch.from_numpy(filler.box_rois(1 + 1000 * rank, B, R)).to(device)
    return images, rois


def dominant_select(d):
    """The dominant launch class: 256->256 3x3 conv at the ROI grid (9 launches/step, ~60 % of FLOPs)."""
    if d.KH == 3 and d.Ca == 256 and d.Cb == 0 and d.Cout == 256 and (d.Ho, d.Wo) == ROI_HW and not d.convT:
        return "conv3x3_256x256_roi"
    return None


def train_bench(device, dtype, rank, world, dist, steps, warmup):
    """Train steps/s of the B0-std ROI model on the C2-shaped batch (module docstring)."""
    import filler
    import hiseg
    from hiseg import distributed as HD
    model = build_model(device, dtype).train()
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = H, W
    images, rois = synthetic_batch(device, rank)
    tgt = torch.from_numpy(filler.ellipse_targets(7 + rank, B * R, *MASK_HW)).to(device)
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    if world > 1:
        HD.enable_grad_sync(model)
    state = {"opt": None}

    def step():
        logits, aux = model(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if state["opt"] is None:
            state["opt"] = hiseg.FusedAdamW(model, lr=1e-4, weight_decay=0.01, max_grad_norm=1.0)
        state["opt"].zero_grad()
        loss.backward()
        state["opt"].step()
        return loss

    for _ in range(warmup):
        loss = step()
    torch.cuda.synchronize()
    first = float(loss.detach())
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    last = float(loss.detach())
    if not (first == first and last == last):
        raise RuntimeError("train bench: non-finite loss")
    sps = steps / elapsed
    return {"metric": "train step/s", "value": round(sps, 3), "unit": "steps/s", "ms_per_step": round(1e3 / sps, 2),
            "steps": steps, "warmup": warmup, "samples_per_s": round(sps * B * R * world, 1),
            "pipeline_tflops": round(sps * B * R * world * GFLOP_PER_TRAIN_ROI / 1e3, 1),
            "loss_first_last": [round(first, 4), round(last, 4)],
            "config": {"workload": "B0-std train step: 32 img 640x480 x 8 ROIs/GPU (256 ROI samples), ROI 64x48, "
                                   "mask 128x96, frozen UNet fwd + ROI path fwd/bwd + RefinedHierarchicalLoss + "
                                   "FusedAdamW", "global_batch": B * world, "roi_samples_per_step": B * R * world,
                       "parallelism": f"dp{world} (DDP, bucketed RCCL grad all-reduce)" if world > 1 else "dp1"}}


def distill_bench(device, dtype, rank, world, dist, steps, warmup, batch=4, hw=640):
    """C5 (BASELINE.json configs[4]): B7 -> B0 staged distillation step, decoder-only phase of the progressive
    unfreezing schedule -- B7 teacher forward (eval), B0 student forward (train-mode BN) + decoder/head
    backward, UNetDistillationLoss (T = 4, targets), decoder-subset FusedAdamW with clip 1.0 -- 4 images
    640x640 per GPU (train_distillation_staged config batch_size 4), gradients averaged over ranks."""
    import filler
    import hiseg
    from hiseg import distributed as HD
    model, loss_fn = hiseg.create_unet_distillation_model("timm-efficientnet-b0", "timm-efficientnet-b7",
                                                          teacher_checkpoint="absent.pth", device="cpu",
                                                          progressive_unfreeze=True)
    filler.fill_module(model.student, seed=11)
    filler.fill_module(model.teacher, seed=12)
    hiseg.set_compute_dtype(model, dtype)
    model = model.to(device).train()
    loss_fn.temperature = 4.0
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(batch, 3, hw, hw, generator=g).to(device)
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, hw), torch.linspace(-1, 1, hw), indexing="ij")
    m = ((yy / 0.7) ** 2 + (xx / 0.45) ** 2 < 1).float()[None, None].expand(batch, 1, hw, hw).contiguous().to(device)
    if world > 1:
        HD.enable_grad_sync(model.student)
    state = {"opt": None}

    def step():
        s, t = model(x)
        loss, _ = loss_fn(s, t, m)
        if state["opt"] is None:
            state["opt"] = hiseg.FusedAdamW(model.student, lr=1e-4, weight_decay=1e-4, max_grad_norm=1.0,
                                            params=model.student.get_decoder_parameters())
        state["opt"].zero_grad()
        loss.backward()
        state["opt"].step()
        return loss

    for _ in range(warmup):
        loss = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    sps = steps / elapsed
    return {"metric": "distillation step/s", "value": round(sps, 3), "unit": "steps/s",
            "ms_per_step": round(1e3 / sps, 2), "steps": steps, "warmup": warmup,
            "images_per_s": round(sps * batch * world, 1), "loss_last": round(float(loss.detach()), 4),
            "config": {"workload": f"C5: B7 teacher (eval) -> B0 student (train-mode BN, decoder-only phase), "
                                   f"{batch} img {hw}x{hw}/GPU, UNetDistillationLoss T=4 + BCE/Dice targets, "
                                   f"decoder FusedAdamW clip 1.0", "global_batch": batch * world,
                       "parallelism": f"dp{world} (bucketed RCCL grad all-reduce)" if world > 1 else "dp1"}}


def eval_bench(device, steps=20, n_roi=2048, mh=128, mw=96):
    """(f)-row 3, GPU validation metrics: hiseg_seg_confusion (argmax + per-sample histogram, the whole
    metric state of train_utils.evaluate_model) over 2048 ROI masks of C2's output size -- logits f32
    [N,3,128,96] + int64 targets, 20 B per pixel read once (algorithmic bytes).  HIP events on the launch
    stream."""
    from hiseg.metrics import seg_confusion
    g = torch.Generator(device=device).manual_seed(7)
    logits = torch.randn(n_roi, 3, mh, mw, device=device, generator=g)
    masks = torch.randint(0, 3, (n_roi, mh, mw), device=device, generator=g)
    out = torch.zeros(n_roi, 5, 4, dtype=torch.int64, device=device)
    for _ in range(3):
        seg_confusion(logits, masks, 3, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        seg_confusion(logits, masks, 3, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = n_roi * mh * mw * (3 * 4 + 8)
    gbs = nbytes / ms / 1e6
    return {"metric": "validation ROI-masks/s (metrics kernel)", "value": round(n_roi / ms * 1e3, 1),
            "unit": "ROI-masks/s", "avg_launch_ms": round(ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4)},
            "config": {"workload": f"{n_roi} ROI masks 3x{mh}x{mw} f32 logits + int64 targets per launch "
                                   f"(argmax + per-sample 5x4 histogram; every evaluate_model metric derives from it)"}}


def data_bench(device, steps=10, batch=32, src_hw=(480, 640), image_size=(640, 640), mask_hw=(128, 96)):
    """(f)-row 2, on-device data path: a C3-shaped batch (32 decoded 480x640 RGB images, 3 instance masks
    each) -> PIL-exact 640x640 f32 CHW images + 3-class 128x96 ROI targets (resize_bilinear_pil +
    roi_targets, the two passes hiseg.GpuRoiBatchBuilder launches).  Inputs resident in HBM.  Beside it
    the reference's own host path for one image: PIL Image.resize (the library dataset.py:98 calls)."""
    import numpy as np
    from PIL import Image
    from hiseg.data import resize_bilinear_pil, roi_targets
    g = torch.Generator(device=device).manual_seed(3)
    H0, W0 = src_hw
    imgs = torch.randint(0, 256, (batch, H0, W0, 3), dtype=torch.uint8, device=device, generator=g)
    masks = (torch.rand(batch * 3, H0, W0, device=device, generator=g) > 0.5).to(torch.uint8).reshape(-1)
    descs = [(i * 3 * H0 * W0, 3, i % 3, H0, W0, 100, 120, 420, 600) for i in range(batch)]

    def step():
        resize_bilinear_pil(imgs, image_size)
        roi_targets(masks, descs, mask_hw, image_size)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # algorithmic bytes: source image read once, the resized row strip written + read once (8-bit), the
    # f32 output written; targets: (1 + instances) bytes gathered + 8 written per mask pixel
    rows = H0   # vertical support of a 480 -> 640 upscale spans every source row
    nbytes = batch * (H0 * W0 * 3 + 2 * rows * image_size[0] * 3 + 3 * image_size[0] * image_size[1] * 4
                      + mask_hw[0] * mask_hw[1] * (3 + 8))
    host = np.asarray(imgs[0].cpu())
    pil = Image.fromarray(host)
    pil.resize(image_size, Image.BILINEAR)
    t1 = time.perf_counter()
    n = 0
    while time.perf_counter() - t1 < 2.0:
        np.asarray(pil.resize(image_size, Image.BILINEAR), dtype=np.float32) / 255.0
        n += 1
    cpu_ips = n / (time.perf_counter() - t1)
    return {"metric": "training batches built on the GPU (images/s)", "value": round(batch / dt, 1),
            "unit": "images/s", "ms_per_batch": round(dt * 1e3, 3),
            "roofline": {"bound": "hbm", "achieved": round(nbytes / dt / 1e9, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(nbytes / dt / 1e9 / PEAK_HBM_GBS, 4)},
            "cpu_reference": {"value": round(cpu_ips, 1), "unit": "images/s", "cores": 1, "kind": "reference",
                              "sample": "PIL Image.resize(640x640, BILINEAR) + /255 of one 480x640 image, 2 s loop"},
            "config": {"workload": f"{batch} x {H0}x{W0} RGB -> {image_size[0]}x{image_size[1]} f32 CHW + "
                                   f"{mask_hw[0]}x{mask_hw[1]} ROI targets from 3 instance masks per image"}}


def cpu_baseline(seconds_budget=30.0):
    """The oracle (float32 CPU restatement of the reference path) on a bounded sample of the same
    workload: 1 image 480x640 with 8 ROIs through UNet + ROI head (exported contract)."""
    import filler
    from oracle import rgb_model as O
    import hiseg
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    model = hiseg.create_rgb_hierarchical_model(**B0_KWARGS)
    filler.fill_module(model).eval()
    sd = O.np_state(model)
    cfg = O.cfg_from_kwargs(B0_KWARGS)
    images = torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(0))
    rois = torch.from_numpy(filler.box_rois(1, 1, R))
    times = []
    with torch.no_grad():
        for i in range(3):
            t0 = time.perf_counter()
            logits, _, u = O.rgb_model(sd, images, rois, cfg, (H, W), "b0")
            O.instance_masks(logits)
            O.binary_masks(sd, u)
            times.append(time.perf_counter() - t0)
            if sum(times) > seconds_budget:
                break
    t = min(times[1:]) if len(times) > 1 else times[0]
    return {"value": round(R / t, 3), "unit": "ROI-masks/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/rgb_model.py fp32 CPU, 1 image 480x640 x {R} ROIs (UNet B0 + head + export masks), "
                      f"best of {len(times) - 1 if len(times) > 1 else 1} after 1 warm-up, {t:.2f} s/iter"}


def load_traffic():
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f).get("dominant_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--train-only", action="store_true")
    ap.add_argument("--no-distill", action="store_true")
    ap.add_argument("--distill-only", action="store_true", help="only the C5 distillation line (profiling)")
    ap.add_argument("--serial", action="store_true", help="one stream (no UNet/head overlap across steps)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    import hiseg  # noqa: F401
    out = {}
    if args.distill_only:
        args.train_only, args.no_train = True, True
        out["distill"] = distill_bench(device, dtype, rank, world, dist, max(2, args.steps // 2), 2)
    if not args.train_only:
        out = infer_bench(args, device, dtype, rank, world, dist)
    if not args.no_train:
        torch.cuda.empty_cache()
        out["train"] = train_bench(device, dtype, rank, world, dist, max(2, args.steps // 2), max(2, args.warmup))
    if not args.no_distill and not args.train_only:
        torch.cuda.empty_cache()
        out["distill"] = distill_bench(device, dtype, rank, world, dist, max(2, args.steps // 2), 2)
    if not args.train_only and world == 1:
        torch.cuda.empty_cache()
        out["eval"] = eval_bench(device)
        out["datapath"] = data_bench(device)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and not args.train_only:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def infer_bench(args, device, dtype, rank, world, dist):
    import hiseg
    from hiseg import ops
    model = build_model(device, dtype)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = synthetic_batch(device, rank)

    runner = None if args.serial else hiseg.StreamPipelinedExport(wrapper)

    def steps(k):
        if runner is None:
            out = None
            for _ in range(k):
                out = wrapper(images, rois)
            return out
        return runner.run([(images, rois)] * k)[-1]

    with torch.no_grad():
        steps(args.warmup)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        probe = ops.LaunchProbe(dominant_select)
        ops.PROBE = probe
        t0 = time.perf_counter()
        inst, binary = steps(args.steps)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ops.PROBE = None
    assert inst.shape == (B * R, 1) + MASK_HW and binary.shape == (B, 1, H, W)

    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    n = world
    ms_per_step = elapsed / args.steps * 1e3
    value = n * B * R * args.steps / elapsed

    summ = probe.summary().get("conv3x3_256x256_roi")
    roofline = None
    if summ:
        achieved = summ["flops"] / (summ["avg_ms"] * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": load_traffic(),
                    "kernel": "conv_fast_kernel<128,128,4,2,2,lds-epilogue> (LDS-DMA ring, 8 waves as 4 Cout x 2 pixel, LDS full-row epilogue) 256->256 3x3 @64x48 x256 ROIs",
                    "launches_timed": summ["launches"], "avg_launch_ms": round(summ["avg_ms"], 4),
                    "flop_per_launch": summ["flops"]}
    pipeline_tflops = value * GFLOP_PER_ROI_MASK / 1e3
    del wrapper, model
    return {
        "metric": METRIC, "value": round(value, 2), "unit": "ROI-masks/s", "n_gpus": n, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
        "data": "synthetic (U[0,1) images, SURVEY §8d ROI boxes; deterministic random-init B0 weights)",
        "config": {"workload": "C2: B0 inference 640x480, batch 32/GPU x 8 ROIs/img, ROI 64x48, mask 128x96",
                   "global_batch": B * n, "rois_per_step": B * R * n, "seq_len": None,
                   "parallelism": f"dp{n} (images sharded, model replicated, no collective)",
                   "schedule": "serial" if args.serial else "2-stream pipeline (UNet of step k+1 overlaps head of step k)"},
        "pipeline_tflops": round(pipeline_tflops, 1),
        "roofline": roofline,
    }


if __name__ == "__main__":
    main()

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

Fourth/fifth, under "train_c3" / "train_c4": the BASELINE C3 (B1-enhanced, 80x60 ROI / 160x120 mask) and C4
(B7-ultra, 128x96 ROI / 256x192 mask, depth-4 head) training steps in the reference's training semantics
(640x640 images, one ROI per image; 32 / 8 images per GPU).

Multi-GPU launch: under torch.distributed.run (WORLD_SIZE set) every rank runs this file; `python bench.py
--gpus N` without a launcher spawns the N rank processes itself (this parent never touches the GPU) and
exits non-zero if any rank fails.  Every rank checks that the process group has exactly N ranks.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--no-train] [--no-distill]
                        [--no-presets] [--backend nccl|gloo] [--dry-run]
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
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
# Distillation unit = one 640x640 image: B7 teacher fwd 120.3 + B0 student fwd+bwd ~111 GFLOP
GFLOP_PER_DISTILL_IMAGE = 120.3 + 111.0
# the staged schedule's last phase (all 7 encoder stages trainable) adds the B0 encoder's backward: data + weight
# gradients ~2x its forward, 0.39 GMAC at 224x224 (timm efficientnet_b0) -> 6.4 GFLOP forward at 640x640
GFLOP_PER_DISTILL_IMAGE_UNFROZEN = GFLOP_PER_DISTILL_IMAGE + 2 * 6.4

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


def preset_kwargs(name):
    """create_rgb_hierarchical_model kwargs of a reference preset (the reference's ConfigManager dump,
    tests/golden/configs.json: b0 = B0-std, b1 = B1-enhanced, b7 = B7-ultra)."""
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        kw = dict(json.load(f)[name]["model_kwargs"])
    kw["roi_size"], kw["mask_size"] = tuple(kw["roi_size"]), tuple(kw["mask_size"])
    return kw


# Algorithmic GFLOP per training sample (one 640x640 image + its ROI): head fwd+bwd + UNet fwd
GFLOP_PER_TRAIN_SAMPLE = {"b1": 279.0 + 40.0, "b7": 835.3 + 120.3}


def train_bench(device, dtype, rank, world, dist, steps, warmup, preset=None, batch=B, rois_per_img=R,
                hw=(H, W), local_first=False, graph_train=False):
    """Train steps/s of an ROI model (module docstring).  preset None: the B0-std model on the C2-shaped batch
    (32 images 640x480 x 8 ROIs, RoIAlign scale (H, W)); preset "b1"/"b7": the C3/C4 preset on `batch` 640x640
    images with one ROI each (the reference's training semantics: dataset.py:74-80, RoIAlign scale 640).
    local_first (world > 1): also time the same step with the gradient exchange off (each rank alone) first, so
    the line carries the DDP step's cost over a rank's local step."""
    import filler
    import hiseg
    from hiseg import distributed as HD
    if preset is None:
        model = build_model(device, dtype).train()
        for m in (model.roi_align_mask, model.roi_align_rgb):
            m.spatial_scale_h, m.spatial_scale_w = H, W
        images, rois = synthetic_batch(device, rank)
        mask_hw = MASK_HW
    else:
        kw = preset_kwargs(preset)
        model = hiseg.create_rgb_hierarchical_model(**kw)
        filler.fill_module(model).eval()
        model = model.to(device)
        hiseg.set_compute_dtype(model, dtype)
        model.train()
        g = torch.Generator().manual_seed(rank)
        images = torch.rand(batch, 3, hw[0], hw[1], generator=g).to(device)
        rois = torch.from_numpy(filler.box_rois(1 + 1000 * rank, batch, rois_per_img)).to(device)
        mask_hw = kw["mask_size"]
    n_samples = int(rois.shape[0])
    tgt = torch.from_numpy(filler.ellipse_targets(7 + rank, n_samples, *mask_hw)).to(device)
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
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

    # One HIP graph per step (hiseg.GraphedStep; every per-step state lives on the device): the eager C3 / C4 steps
    # take 28 / 33 ms of Python enqueue for 38 / 41 ms of GPU work (tools/host_bound.py --train), so any host
    # contention made them host-bound (C3 53-70 ms in full bench runs vs 38 ms alone); replayed, the step costs one
    # launch.  Same GPU time as eager on a quiet host (profiles/r3_graph_vs_eager.txt).  Data-parallel legs over RCCL
    # are captured with their bucketed all-reduces (graphs.py); a gloo group cannot be captured and stays eager.
    # --eager-train: eager always.
    graphable = graph_train and (world == 1 or _backend(dist) == "nccl")
    runner = {"run": hiseg.GraphedStep(step, lambda: state["opt"]) if graphable else step}

    def timed():
        run = runner["run"]
        for _ in range(max(warmup, 3 if run is not step else 1)):
            loss = run()
        torch.cuda.synchronize()
        first = float(loss.detach())
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = run()
            if STEP_TIMES is not None:
                torch.cuda.synchronize()
                STEP_TIMES.append(time.perf_counter() - t0)
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
        return elapsed, first, last

    local = None
    if world > 1 and local_first:
        el, _, _ = timed()
        local = steps / el
    if world > 1:
        HD.enable_grad_sync(model)
        HD.sync_loss_class_weights(loss_fn)   # class weights from the counts of the whole (all-rank) batch
        # the local leg left per-rank optimizer moments / loss EMA: start the DDP leg from rank 0's
        HD.broadcast_training_state(state["opt"], loss_fn)
        if graphable:   # a new graph: the exchange (and the loss's count all-reduce) must be in it
            runner["run"] = hiseg.GraphedStep(step, lambda: state["opt"])
    prof = None
    if world == 1:   # per-call profile of one eager step (before any graph capture: its pool would skew it)
        step()
        prof = call_profile(step, {None: "train", "b1": "c3", "b7": "c4"}.get(preset))
    elapsed, first, last = timed()
    sps = steps / elapsed
    gflop = GFLOP_PER_TRAIN_ROI if preset is None else GFLOP_PER_TRAIN_SAMPLE[preset]
    if preset is None:
        workload = ("B0-std train step: 32 img 640x480 x 8 ROIs/GPU (256 ROI samples), ROI 64x48, mask 128x96, "
                    "frozen UNet fwd + ROI path fwd/bwd + RefinedHierarchicalLoss + FusedAdamW")
    else:
        kw = preset_kwargs(preset)
        workload = (f"{'C3 B1-enhanced' if preset == 'b1' else 'C4 B7-ultra'} train step: {batch} img "
                    f"{hw[0]}x{hw[1]} x {rois_per_img} ROI/GPU, ROI {kw['roi_size'][0]}x{kw['roi_size'][1]}, mask "
                    f"{kw['mask_size'][0]}x{kw['mask_size'][1]}, head depth {kw['hierarchical_depth']}, frozen "
                    f"{kw['encoder_name'][-2:].upper()} UNet fwd + ROI path fwd/bwd + RefinedHierarchicalLoss + FusedAdamW")
    out = {"metric": "train step/s", "value": round(sps, 3), "unit": "steps/s", "ms_per_step": round(1e3 / sps, 2),
           "steps": steps, "warmup": warmup, "samples_per_s": round(sps * n_samples * world, 1),
           "pipeline_tflops": round(sps * n_samples * world * gflop / 1e3, 1),
           "loss_first_last": [round(first, 4), round(last, 4)],
           "config": {"workload": workload, "global_batch": int(images.shape[0]) * world,
                      "roi_samples_per_step": n_samples * world,
                      "parallelism": f"dp{world} (DDP, bucketed RCCL grad all-reduce)" if world > 1 else "dp1",
                      "schedule": "eager" if runner["run"] is step else
                      ("one HIP graph per step (hiseg.GraphedStep)" + (", all-reduces captured" if world > 1 else ""))}}
    pipe = out["pipeline_tflops"] / world
    out["pipeline_frac"] = round(pipe / PEAK_BF16_TFLOPS, 4)
    if prof is not None:
        out["roofline"] = prof.pop("roofline", None)
        out["call_profile"] = prof
    if local is not None:
        out["local_step_per_s"] = round(local, 3)
        out["ddp_over_local"] = round(sps / local, 4)   # 1.0 = the gradient exchange is fully hidden
    del model
    return out


def _copy_probe_ms(nbytes=1 << 29):
    """Median time of three device-to-device copies of `nbytes` (an HBM bandwidth probe, tools/leg_probe.py)."""
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    del a, b
    return sorted(ts)[1]


def _release_leg():
    """Between legs of an --in-process run: collect the finished leg's graphs / closures (reference cycles keep a
    GraphedStep, its captured graph and that graph's private memory pool alive until the cyclic collector runs).  The
    cached blocks are kept for the next leg (HISEG_BENCH_EMPTY_CACHE=1 returns them to the driver, after which the
    inference leg measured up to 16 % slower right after the train legs, profiles/r5_leg_order.txt)."""
    import gc
    torch.cuda.synchronize()
    gc.collect()
    if os.environ.get("HISEG_BENCH_EMPTY_CACHE", "0") == "1":
        torch.cuda.empty_cache()


def _backend(dist):
    return dist.get_backend() if dist else None


def distill_bench(device, dtype, rank, world, dist, steps, warmup, batch=4, hw=640, graph=True, unfrozen=0):
    """C5 (BASELINE.json configs[4]): B7 -> B0 staged distillation step, decoder-only phase of the progressive
    unfreezing schedule -- B7 teacher forward (eval), B0 student forward (train-mode BN) + decoder/head
    backward, UNetDistillationLoss (T = 4, targets), decoder-subset FusedAdamW with clip 1.0 -- 4 images
    640x640 per GPU (train_distillation_staged config batch_size 4), gradients averaged over ranks.
    ``unfrozen`` = N: the schedule's later phase after unfreeze_encoder_blocks(N) -- the encoder's last N stages
    trainable (backward through the MBConv depthwise / SqueezeExcite / BN stacks) and the reference's two
    parameter groups (train_distillation_staged.py:1509-1544: decoder lr with clip 1.0 on the decoder only,
    :300-313; encoder lr x encoder_lr_scale 0.1, :1215)."""
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
    enc = model.unfreeze_encoder_blocks(unfrozen, learning_rate_scale=0.1) if unfrozen else None
    if world > 1:
        HD.enable_grad_sync(model.student)
    state = {"opt": None, "enc_opt": None}

    def step(s=None, t=None):
        if s is None:
            s, t = model(x)
        loss, _ = loss_fn(s, t, m)
        if state["opt"] is None:
            state["opt"] = hiseg.FusedAdamW(model.student, lr=1e-4, weight_decay=1e-4, max_grad_norm=1.0,
                                            params=model.student.get_decoder_parameters())
            if enc:
                state["enc_opt"] = hiseg.FusedAdamW(model.student, lr=1e-4 * 0.1, weight_decay=1e-4,
                                                    max_grad_norm=None, params=enc)
        opts = [o for o in (state["opt"], state["enc_opt"]) if o is not None]
        for o in opts:
            o.zero_grad()
        loss.backward()
        for o in opts:
            o.step()
        return loss

    prof = None
    if world == 1:   # per-call profile of one eager step, before the graph capture
        step()
        step()
        # serial teacher for the per-call profile (concurrent branches would overlap the HIP-event intervals)
        model.concurrent_teacher = False
        prof = call_profile(step, "distill_unfrozen" if unfrozen else "distill")
        del model.concurrent_teacher
    graphable = graph and (world == 1 or _backend(dist) == "nccl")
    run = hiseg.GraphedStep(step, lambda: state["opt"]) if graphable else step
    branch_graphs = graphable and world == 1 and os.environ.get("HISEG_DISTILL_BRANCH_GRAPHS", "1") != "0"
    pipelined = branch_graphs and os.environ.get("HISEG_DISTILL_PIPELINE", "1") != "0"
    if branch_graphs:
        # teacher / student forwards as graphs of their own, launched side by side (GraphedBranchStep)
        fwd = {}

        def teacher():
            fwd["t"] = model.teacher(x)

        def student():
            fwd["s"] = model.student(x)

        def tail():
            return step(fwd["s"], fwd["t"])

        handoff = None
        if pipelined:
            # the frozen eval-mode teacher runs one batch ahead (overlapping this batch's backward): the timed K
            # steps still run K teacher forwards; the batch is the same synthetic x every step
            def teacher():
                fwd["t_next"] = model.teacher(x)

            def handoff():
                if "t" not in fwd:
                    fwd["t"] = torch.empty_like(fwd["t_next"])
                fwd["t"].copy_(fwd["t_next"])

        run = hiseg.GraphedBranchStep(teacher, student, tail, lambda: state["opt"], handoff_fn=handoff)
    for _ in range(max(warmup, 3 if run is not step else 1)):
        loss = run()
    if os.environ.get("HISEG_BENCH_STEP_TIMES") == "1":   # developer knob: per-replay times on stderr
        ts, hs = [], []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h0 = time.perf_counter()
            run()
            hs.append(round((time.perf_counter() - h0) * 1e3, 2))
            e1.record()
            torch.cuda.synchronize()
            ts.append(round(e0.elapsed_time(e1), 2))
        print(f"distill per-replay ms: {ts} host enqueue ms: {hs}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = run()
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
    extra = {}
    if prof is not None:
        extra["roofline"] = prof.pop("roofline", None)
        extra["call_profile"] = prof
    gfl = GFLOP_PER_DISTILL_IMAGE_UNFROZEN if unfrozen else GFLOP_PER_DISTILL_IMAGE
    extra["pipeline_tflops"] = round(sps * batch * world * gfl / 1e3, 1)
    extra["pipeline_frac"] = round(extra["pipeline_tflops"] / world / PEAK_BF16_TFLOPS, 4)
    return {"metric": "distillation step/s", "value": round(sps, 3), "unit": "steps/s",
            "ms_per_step": round(1e3 / sps, 2), "steps": steps, "warmup": warmup,
            "images_per_s": round(sps * batch * world, 1), "loss_last": round(float(loss.detach()), 4), **extra,
            "config": {"workload": f"C5: B7 teacher (eval) -> B0 student (train-mode BN, "
                                   + (f"encoder stages unfrozen: {unfrozen} of 7 -- encoder backward, two "
                                      f"parameter groups" if unfrozen else "decoder-only phase")
                                   + f"), {batch} img {hw}x{hw}/GPU, UNetDistillationLoss T=4 + BCE/Dice targets, "
                                   f"decoder FusedAdamW clip 1.0" + (", encoder FusedAdamW lr x 0.1 unclipped"
                                                                     if unfrozen else ""),
                       "global_batch": batch * world,
                       "schedule": "eager" if run is step else (
                           ("teacher / student-forward / loss-backward-optimizer graphs (hiseg.GraphedBranchStep)"
                            + (", teacher one batch ahead" if pipelined else "")) if branch_graphs
                           else "one HIP graph per step (hiseg.GraphedStep)"),
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


def cpu_threads():
    """Host threads the CPU baselines use: the CPUs this process may run on, capped by OMP_NUM_THREADS when the
    environment sets it (the GPU box sets 16 = its CPU share; os.cpu_count() there reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else max(1, n)


def _median_runs(fn, warmup=2, runs=5, budget_s=30.0):
    for _ in range(warmup):
        fn()
    times = []
    t_all = time.perf_counter()
    while len(times) < runs or (time.perf_counter() - t_all < 2.0 and len(times) < 2 * runs):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_all > budget_s and len(times) >= 3:
            break
    return statistics.median(times), len(times)


def cpu_baseline(seconds_budget=30.0):
    """The oracle (float32 CPU restatement of the reference path) on a bounded sample of the same
    workload: 1 image 480x640 with 8 ROIs through UNet + ROI head (exported contract).  BASELINE.md §3 /
    SURVEY §8d: 2 warm-up runs, then the median of >= 5."""
    import filler
    from oracle import rgb_model as O
    import hiseg
    torch.set_num_threads(cpu_threads())
    model = hiseg.create_rgb_hierarchical_model(**B0_KWARGS)
    filler.fill_module(model).eval()
    sd = O.np_state(model)
    cfg = O.cfg_from_kwargs(B0_KWARGS)
    images = torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(0))
    rois = torch.from_numpy(filler.box_rois(1, 1, R))

    def run():
        with torch.no_grad():
            logits, _, u = O.rgb_model(sd, images, rois, cfg, (H, W), "b0")
            O.instance_masks(logits)
            O.binary_masks(sd, u)

    t, n = _median_runs(run, budget_s=seconds_budget)
    return {"value": round(R / t, 3), "unit": "ROI-masks/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/rgb_model.py fp32 CPU, 1 image 480x640 x {R} ROIs (UNet B0 + head + export masks), "
                      f"median of {n} after 2 warm-ups, {t:.2f} s/iter"}


def cpu_train_baseline(seconds_budget=30.0):
    """The oracle's B0-std training step on the host cores (baseline beside `train`): 1 image 480x640 x 8 ROIs,
    fp32 -- frozen UNet forward, train-mode ROI path (oracle/train.py, torch autograd), RefinedHierarchicalLoss,
    backward, clip + AdamW.  2 warm-ups, median of >= 5."""
    import filler
    from oracle import rgb_model as O
    from oracle import train as OT
    import hiseg
    torch.set_num_threads(cpu_threads())
    model = hiseg.create_rgb_hierarchical_model(**B0_KWARGS)
    filler.fill_module(model)
    for m in model.modules():
        if isinstance(m, (torch.nn.Dropout, torch.nn.Dropout2d)):
            m.p = 0.0
    sd = OT.params_of(model)
    cfg = O.cfg_from_kwargs(B0_KWARGS)
    images = torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(0))
    rois = torch.from_numpy(filler.box_rois(1, 1, R))
    tgt = torch.from_numpy(filler.ellipse_targets(7, R, *MASK_HW))
    params = [v for v in sd.values() if v.requires_grad]
    state = {}
    loss_fn = OT.RefinedHierarchicalLoss()

    def run():
        with torch.no_grad():
            u = O.pretrained_unet_logits(sd, images, "b0")
        logits, aux = OT.forward_train(sd, images, rois, u, cfg, (H, W))
        loss, _ = loss_fn(logits, tgt, aux)
        for p in params:
            p.grad = None
        loss.backward()
        OT.adamw_step(params, [p.grad if p.grad is not None else torch.zeros_like(p) for p in params], state)

    t, n = _median_runs(run, budget_s=seconds_budget)
    return {"value": round(1.0 / t, 4), "unit": "steps/s", "samples_per_s": round(R / t, 3), "cores": torch.get_num_threads(),
            "kind": "port", "sample": f"oracle/train.py fp32 CPU B0-std train step, 1 image 480x640 x {R} ROI samples, "
                                      f"median of {n} after 2 warm-ups, {t:.2f} s/step"}


# developer hook (tools/c3_after_infer.py): a list collects the cumulative time after every timed train step
STEP_TIMES = None
DOMINANT_KERNEL_ID = "conv_hwc_128_256x256_roi"


def cpu_train_c3_baseline(bench_batch=32, seconds_budget=30.0, full_budget_s=90.0):
    """the oracle's C3 (B1-enhanced, 80x60 ROI / 160x120 mask) train step on the host cores at the
    reference batch (2 images 640x640 x 1 ROI: 2 warm-ups, median of >= 5) and at the bench batch (32) as a
    bounded sample: one step after the batch-2 warm-ups, skipped when the batch-2 time predicts more than
    `full_budget_s` for it."""
    import filler
    from oracle import rgb_model as O
    from oracle import train as OT
    import hiseg
    torch.set_num_threads(cpu_threads())
    kw = preset_kwargs("b1")
    model = hiseg.create_rgb_hierarchical_model(**kw)
    filler.fill_module(model)
    for m in model.modules():
        if isinstance(m, (torch.nn.Dropout, torch.nn.Dropout2d)):
            m.p = 0.0
    sd = OT.params_of(model)
    cfg = O.cfg_from_kwargs(kw)
    params = [v for v in sd.values() if v.requires_grad]

    def make(b):
        images = torch.rand(b, 3, 640, 640, generator=torch.Generator().manual_seed(0))
        rois = torch.from_numpy(filler.box_rois(1, b, 1))
        tgt = torch.from_numpy(filler.ellipse_targets(7, b, *kw["mask_size"]))
        state, loss_fn = {}, OT.RefinedHierarchicalLoss()

        def run():
            with torch.no_grad():
                u = O.pretrained_unet_logits(sd, images, "b1")
            logits, aux = OT.forward_train(sd, images, rois, u, cfg, (640, 640))
            loss, _ = loss_fn(logits, tgt, aux)
            for p in params:
                p.grad = None
            loss.backward()
            OT.adamw_step(params, [p.grad if p.grad is not None else torch.zeros_like(p) for p in params], state)
        return run

    t2, n2 = _median_runs(make(2), budget_s=seconds_budget)
    out = {"value": round(1.0 / t2, 4), "unit": "steps/s", "batch": 2, "cores": torch.get_num_threads(),
           "kind": "port", "sample": f"oracle/train.py fp32 CPU C3 B1-enhanced train step, 2 images 640x640 x 1 ROI, "
                                     f"median of {n2} after 2 warm-ups, {t2:.2f} s/step"}
    est = t2 * bench_batch / 2
    if est <= full_budget_s:
        run = make(bench_batch)
        t0 = time.perf_counter()
        run()
        tb = time.perf_counter() - t0
        out["bench_batch"] = {"value": round(1.0 / tb, 4), "unit": "steps/s", "batch": bench_batch,
                              "sample": f"one step of {bench_batch} images 640x640 x 1 ROI after the batch-2 "
                                        f"warm-ups (bounded sample), {tb:.2f} s/step"}
    else:
        out["bench_batch"] = {"value": None, "batch": bench_batch,
                              "sample": f"skipped: the batch-2 step predicts ~{est:.0f} s per step (> {full_budget_s:.0f} s budget)"}
    return out


def load_traffic():
    """Per-launch HBM bytes of the dominant kernel (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected)
    from roofline_traffic.json at the repository root -- a tracked file that travels with the tree (profiles/
    does not); None when it describes another kernel than the one timed here."""
    path = os.path.join(ROOT, "roofline_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("kernel_id") != DOMINANT_KERNEL_ID:
        return None
    return d.get("dominant_bytes_per_launch")


def _conv_flops(d):
    """Algorithmic FLOPs of one conv GEMM launch (forward, data gradient or weight gradient: the same
    2 * pixels * K * columns) from its hiseg_conv2d_desc."""
    if d.convT:
        return 2.0 * d.N * d.H * d.W * d.Ca * d.Cout
    return 2.0 * d.N * d.Ho * d.Wo * d.Cout * d.KH * d.KW * (d.Ca + d.Cb)


def _es(dtype_code):
    return 2 if int(dtype_code) == 1 else 4   # include/hiseg.h: HISEG_BF16 = 1, HISEG_F32 = 0


def _hbm_bytes(name, args):
    """Algorithmic HBM bytes of one call of an element-wise / statistics entry point (every operand read or
    written once), or None for entry points without a formula here.  SURVEY.md §8d: BN stat / apply, depthwise
    convs and the SE pools are HBM-bound."""
    try:
        if name == "hiseg_bn_stats":            # (dtype, z, P, C, cstride, coff, partial, stream): read z
            return float(args[2]) * args[3] * _es(args[0])
        if name == "hiseg_bn_apply":            # read z (+ residual), write y
            d = args[0]._obj
            return float(d.P) * d.C * _es(d.dtype) * (2 + (1 if d.residual else 0))
        if name == "hiseg_bn_bwd":              # read dy, z (+ residual), write dz (+ dres, read when accumulating)
            d = args[0]._obj
            n = 3 + (1 if d.residual else 0) + ((1 + (1 if d.dres_accumulate else 0)) if d.dres else 0)
            return float(d.P) * d.C * _es(d.dtype) * n
        if name in ("hiseg_dwconv_fwd", "hiseg_dwconv_gap_fwd"):   # (dtype, in, N, H, W, C, K, stride, ..., Ho, Wo)
            dt, N, H, W, C, Ho, Wo = args[0], args[2], args[3], args[4], args[5], args[13], args[14]
            return float(N) * (H * W + Ho * Wo) * C * _es(dt)
    except (AttributeError, IndexError, TypeError):
        return None
    return None


# kernel classes of the train / distill legs: every C-ABI entry point falls in one; a leg's `roofline` is the
# class that takes the most GPU time, bounded by MFMA (the conv classes, algorithmic FLOPs) or by HBM (the others,
# algorithmic bytes)
_HBM_CLASSES = {"hiseg_bn_stats": "BatchNorm (train)", "hiseg_bn_finalize": "BatchNorm (train)",
                "hiseg_bn_apply": "BatchNorm (train)", "hiseg_bn_bwd": "BatchNorm (train)",
                "hiseg_dwconv_fwd": "depthwise conv (+ SE pool)", "hiseg_dwconv_gap_fwd": "depthwise conv (+ SE pool)"}


def load_class_traffic(leg):
    """Measured HBM bytes per step of each kernel class of one leg (tools/pmc_classes.py over two rocprofv3 PMC passes
    of `bench.py --leg <leg> --eager-train`, FETCH_SIZE / WRITE_SIZE, gfx950-corrected) from roofline_traffic.json's
    "train_legs"; {} when absent."""
    try:
        with open(os.path.join(ROOT, "roofline_traffic.json")) as f:
            return json.load(f).get("train_legs", {}).get(leg, {})
    except (OSError, ValueError):
        return {}


_SLEEP_CYCLES_PER_MS = None


def _gpu_lead(ms):
    """Queue a GPU spin of about `ms` milliseconds on the current stream (torch.cuda._sleep, calibrated once)."""
    global _SLEEP_CYCLES_PER_MS
    if _SLEEP_CYCLES_PER_MS is None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda._sleep(10_000_000)
        e1.record()
        torch.cuda.synchronize()
        _SLEEP_CYCLES_PER_MS = 10_000_000 / max(e0.elapsed_time(e1), 1e-3)
    torch.cuda._sleep(int(ms * _SLEEP_CYCLES_PER_MS))


def call_profile(step, leg=None):
    """One extra (untimed) step with HIP events around every libhiseg C-ABI call on its launch stream:
    per-entry-point GPU time; per kernel class (conv forward / data gradient / weight gradient over all layers,
    train-mode BatchNorm, depthwise + SE pool) the time, the algorithmic FLOPs or bytes and the bound -- the
    class with the largest share of the step is the leg's `roofline`; the heaviest single conv layer class is
    reported beside it (`dominant_layer`)."""
    from hiseg import _lib as L
    lib = L.lib()
    real, rec = {}, []
    last_path = lib.hiseg_wgrad_last_path
    # one unprofiled eager step first: the timed legs replay graphs from their own memory pools, so the first eager
    # step after them meets a cold caching allocator (device allocations -- and frees of cached blocks, which
    # synchronise the device -- inside the step, each one draining the GPU's lead over the host)
    step()
    torch.cuda.synchronize()
    names = [n for n in (L.EXPORTED or []) if n.startswith("hiseg_")]
    for name in names:
        fn = getattr(lib, name, None)
        if fn is None or not callable(fn):
            continue
        real[name] = fn

        def wrap(*a, _n=name, _f=fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = _f(*a)
            e1.record()
            key, cls, flops, nbytes = None, _HBM_CLASSES.get(_n), 0.0, None
            if _n in ("hiseg_conv2d_fwd", "hiseg_conv2d_fwd_variant", "hiseg_conv2d_wgrad"):
                d = a[0]._obj
                kind = "wgrad" if _n == "hiseg_conv2d_wgrad" else (
                    "dgrad" if sys._getframe(1).f_code.co_name == "_dgrad_launch" else "fwd")
                key = (f"{kind} {d.KH}x{d.KW}{' T' if d.convT else ''} {d.Ca}+{d.Cb}->{d.Cout} "
                       f"{d.N}x{d.Ho}x{d.Wo}")
                if kind == "wgrad":   # which kernel took it (wide / transposed-read / generic fallback / f32)
                    key += f" [{L.WGRAD_PATHS[last_path()]}]"
                cls = {"fwd": "conv forward", "dgrad": "conv data gradient", "wgrad": "conv weight gradient"}[kind]
                flops = _conv_flops(d)
            elif cls is not None:
                nbytes = _hbm_bytes(_n, a)
            rec.append((_n, key, cls, flops, nbytes, e0, e1))
            return r
        setattr(lib, name, wrap)
    try:
        L.wgrad_path_stats(reset=True)
        torch.cuda.synchronize()
        # An eager step's Python enqueue can be as long as its GPU work (C3 / C4: ~30 ms per ~40), and an event
        # pair brackets GPU time only while the host stays ahead of the GPU: with an idle queue the interval holds
        # the host's own gap (an allocator call, the next descriptor's build).  A GPU spin queued first gives the
        # host that lead, so every interval -- and the step -- is kernel time.
        _gpu_lead(float(os.environ.get("HISEG_PROFILE_LEAD_MS", "250")))
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        step()
        t1.record()
        host_done = time.perf_counter()
        torch.cuda.synchronize()
        lead_left_ms = (time.perf_counter() - host_done) * 1e3
    finally:
        for name, fn in real.items():
            setattr(lib, name, fn)
    step_ms = t0.elapsed_time(t1)
    paths = L.wgrad_path_stats()
    by_entry, groups, classes = {}, {}, {}
    for n, k, cls, fl, nb, e0, e1 in rec:
        ms = e0.elapsed_time(e1)
        by_entry[n] = by_entry.get(n, 0.0) + ms
        if k is not None:
            g = groups.setdefault(k, [0, 0.0, fl])
            g[0] += 1
            g[1] += ms
        if cls is not None:
            c = classes.setdefault(cls, {"calls": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "bytes_ms": 0.0})
            c["calls"] += 1
            c["ms"] += ms
            c["flops"] += fl
            if nb is not None:   # bytes only over the calls with a formula (bn_finalize: a few KB, not counted)
                c["bytes"] += nb
                c["bytes_ms"] += ms
    conv_ms = sum(g[1] for g in groups.values())
    calls_ms = sum(e0.elapsed_time(e1) for _, _, _, _, _, e0, e1 in rec)
    out = {"step_ms_probed": round(step_ms, 3),
           # GPU time inside the C-ABI calls: the eager step minus its launch gaps between calls (a replayed graph
           # has almost none), the figure to hold against the graphed ms_per_step
           "calls_ms_sum": round(calls_ms, 3),
           # > step_ms: the GPU was still working when the host finished enqueueing, so no interval held host time
           "host_lead_left_ms": round(lead_left_ms, 3),
           "wgrad_paths": paths,
           "c_abi_calls": len(rec),
           "conv_share": round(conv_ms / step_ms, 4) if step_ms > 0 else None,
           "top_entry_points_ms": {n: round(ms, 3) for n, ms in sorted(by_entry.items(), key=lambda kv: -kv[1])[:6]}}
    table = {}
    for cls, c in classes.items():
        row = {"calls": c["calls"], "ms": round(c["ms"], 3), "share_of_step": round(c["ms"] / step_ms, 4)}
        if c["flops"] > 0:
            ach = c["flops"] / (c["ms"] * 1e-3) / 1e12
            row.update(bound="mfma", achieved=round(ach, 1), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                       frac=round(ach / PEAK_BF16_TFLOPS, 4))
        elif c["bytes_ms"] > 0:
            gbs = c["bytes"] / (c["bytes_ms"] * 1e-3) / 1e9
            row.update(bound="hbm", achieved=round(gbs, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                       frac=round(gbs / PEAK_HBM_GBS, 4), bytes=c["bytes"])
        legt = load_class_traffic(leg) if leg else {}
        meas = legt.get(cls)
        if meas is None and cls in ("conv forward", "conv data gradient"):
            # one PMC class for both (the same kernels run the forward and the data gradient)
            both = legt.get("conv forward + data gradient")
            if both:
                row["traffic_per_step_fwd_plus_dgrad"] = round(both["hbm_bytes_per_step"])
        if meas:   # PMC-measured HBM bytes of this class per step, and per C-ABI call like `bytes`
            row["traffic_per_step"] = round(meas["hbm_bytes_per_step"])
            row["traffic"] = round(meas["hbm_bytes_per_step"] / c["calls"])
            if c["bytes"] > 0:
                row["traffic_over_algorithmic"] = round(meas["hbm_bytes_per_step"] / c["bytes"], 3)
        table[cls] = row
    both = (load_class_traffic(leg) if leg else {}).get("conv forward + data gradient")
    if both:   # per call over the forward and data-gradient calls together (the PMC pass cannot tell them apart)
        convs = [table[k] for k in ("conv forward", "conv data gradient") if k in table]
        ncalls = sum(r["calls"] for r in convs)
        for r in convs:
            r["traffic"] = round(both["hbm_bytes_per_step"] / ncalls) if ncalls else None
            r["traffic_scope"] = "conv forward + data gradient calls together (one PMC class)"
    out["classes"] = table
    if table:
        cls, row = max(table.items(), key=lambda kv: kv[1]["ms"])
        out["roofline"] = {"bound": row.get("bound"), "achieved": row.get("achieved"), "peak": row.get("peak"),
                           "unit": row.get("unit"), "frac": row.get("frac"), "traffic": row.get("traffic"),
                           "kernel": f"{cls} (all layers of the step, {row['calls']} C-ABI calls)",
                           "share_of_step": row["share_of_step"], "avg_launch_ms": round(row["ms"] / row["calls"], 4),
                           "traffic_unit": "HBM bytes per C-ABI call of the class (rocprofv3 FETCH_SIZE / WRITE_SIZE "
                                           "passes, roofline_traffic.json train_legs)"}
    if groups:
        key, (cnt, ms, fl) = max(groups.items(), key=lambda kv: kv[1][1])
        avg = ms / cnt
        ach = fl / (avg * 1e-3) / 1e12
        out["dominant_layer"] = {"bound": "mfma", "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS,
                                 "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4), "kernel": key,
                                 "launches_timed": cnt, "avg_launch_ms": round(avg, 4), "flop_per_launch": fl,
                                 "share_of_step": round(ms / step_ms, 4) if step_ms > 0 else None}
        out["top_layers"] = [{"layer": k, "launches": cnt, "ms": round(ms, 3),
                              "tflops": round(fl * cnt / (ms * 1e-3) / 1e12, 1) if ms > 0 else None}
                             for k, (cnt, ms, fl) in sorted(groups.items(), key=lambda kv: -kv[1][1])[:10]]
        all_fl = sum(g[2] * g[0] for g in groups.values())
        out["conv_tflops"] = round(all_fl / (conv_ms * 1e-3) / 1e12, 1) if conv_ms > 0 else None
    return out


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` without a torch.distributed launcher: start N rank processes of this script (this process never
    touches the GPU), RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1.  Rank output passes through;
    the first rank that fails ends the others and sets the exit status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    if rc:
        print(f"bench.py: a rank failed (exit {rc})", file=sys.stderr)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE of a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--train-only", action="store_true")
    ap.add_argument("--no-distill", action="store_true")
    ap.add_argument("--no-presets", action="store_true", help="skip the C3 (B1) / C4 (B7) train lines")
    ap.add_argument("--distill-only", action="store_true", help="only the C5 distillation line (profiling)")
    ap.add_argument("--order", default="infer,train,c3,c4,distill,distill_unfrozen",
                    help="the legs of a full run, in this order (comma list of infer, train, c3, c4, distill, "
                         "distill_unfrozen)")
    ap.add_argument("--leg", choices=["train", "c3", "c4", "distill", "distill_unfrozen", "infer"], default=None,
                    help="profiling: run only this train / distillation leg (one JSON object)")
    ap.add_argument("--serial", action="store_true", help="one stream (no UNet/head overlap across steps)")
    ap.add_argument("--eager-train", action="store_true", help="train / distill legs as eager launches (default on one "
                                                                "GPU: one replayed HIP graph per step)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--in-process", action="store_true",
                    help="one GPU: run every leg in this process (default: each leg in a child process of its own)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + rendezvous check only (no GPU work): CPU tests of the multi-rank path")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if args.dry_run and os.environ.get("HISEG_BENCH_FAIL_RANK") == str(rank):
        sys.exit(5)   # test hook (tests/test_bench_launcher.py): a rank that dies before the rendezvous
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            probe = torch.ones(1, device=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
            probe = torch.ones(1)
        dist.all_reduce(probe)   # the communicator formed over every rank
        if dist.get_world_size() != world or int(probe.item()) != world:
            print(f"bench.py: rank {rank}: process group has {dist.get_world_size()} ranks, expected {world}",
                  file=sys.stderr)
            sys.exit(3)
    if args.dry_run:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "backend": args.backend}))
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    device = torch.device("cuda", local)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    import hiseg  # noqa: F401
    out = {}
    if args.leg is not None:   # one leg alone (rocprofv3 PMC passes per leg: tools/pmc_classes.py)
        steps, g = max(2, args.steps // 2), not args.eager_train
        if args.leg == "train":
            out["train"] = train_bench(device, dtype, rank, world, dist, steps, max(2, args.warmup), graph_train=g)
        elif args.leg == "c3":
            out["train_c3"] = train_bench(device, dtype, rank, world, dist, steps, 2, preset="b1", batch=32,
                                          rois_per_img=1, hw=(640, 640), graph_train=g)
        elif args.leg == "c4":
            out["train_c4"] = train_bench(device, dtype, rank, world, dist, steps, 2, preset="b7", batch=8,
                                          rois_per_img=1, hw=(640, 640), graph_train=g)
        elif args.leg == "distill_unfrozen":
            out["distill_unfrozen"] = distill_bench(device, dtype, rank, world, dist, steps, 2, graph=g, unfrozen=7)
        elif args.leg == "infer":
            out = infer_bench(args, device, dtype, rank, world, dist)
        else:
            out["distill"] = distill_bench(device, dtype, rank, world, dist, steps, 2, graph=g)
        if rank == 0:
            print(json.dumps(out))
        if dist:
            dist.destroy_process_group()
        return
    if args.distill_only:
        args.train_only, args.no_train = True, True
    # The legs run in the order --order names (default: inference, B0 train, C3, C4, distillation, unfrozen
    # distillation).  On one GPU each leg runs in a child process of its own (`bench.py --leg L`, whose JSON object this
    # process merges), so no leg inherits another's device state.  Round 6 measured every leg within 1.4 % of its
    # child-process time in one process, in either order -- and in a later run on the same tree the unfrozen
    # distillation leg at 18.6 ms after the others against 14.7 (profiles/r6_leg_order_inprocess.txt): the
    # stream-to-hardware-queue binding a process keeps still decides it now and then, so the isolation
    # stays the default.  --in-process runs all legs in this process; the multi-rank run always uses one process per rank.
    half, eager = max(2, args.steps // 2), args.eager_train
    legs = {
        "infer": (not args.train_only, lambda: out.update(infer_bench(args, device, dtype, rank, world, dist))),
        "train": (not args.no_train, lambda: out.__setitem__("train", train_bench(
            device, dtype, rank, world, dist, half, max(2, args.warmup), local_first=True, graph_train=not eager))),
        "c3": (not args.no_train and not args.no_presets, lambda: out.__setitem__("train_c3", train_bench(
            device, dtype, rank, world, dist, half, 2, preset="b1", batch=32, rois_per_img=1, hw=(640, 640),
            graph_train=not eager))),
        "c4": (not args.no_train and not args.no_presets, lambda: out.__setitem__("train_c4", train_bench(
            device, dtype, rank, world, dist, half, 2, preset="b7", batch=8, rois_per_img=1, hw=(640, 640),
            graph_train=not eager))),
        "distill": ((not args.no_distill and not args.train_only) or args.distill_only,
                    lambda: out.__setitem__("distill", distill_bench(device, dtype, rank, world, dist, half, 2,
                                                                     graph=not eager))),
        "distill_unfrozen": ((not args.no_distill and not args.train_only) or args.distill_only,
                             lambda: out.__setitem__("distill_unfrozen", distill_bench(
                                 device, dtype, rank, world, dist, half, 2, graph=not eager, unfrozen=7))),
    }
    order = [k.strip() for k in args.order.split(",") if k.strip()]
    bad = [k for k in order if k not in legs]
    if bad:
        print(f"bench.py: unknown legs in --order: {bad} (choose from {sorted(legs)})", file=sys.stderr)
        sys.exit(2)
    first = True
    for k in order:
        on, fn = legs[k]
        if not on:
            continue
        if world == 1 and not args.in_process:
            out.update(_leg_in_child(k, args))
        else:
            if not first:
                _release_leg()
            fn()
        first = False
        if k == "infer":   # the JSON line's head keys come first
            out = {**{kk: out[kk] for kk in out if kk not in ("train", "train_c3", "train_c4", "distill",
                                                                "distill_unfrozen")}, **out}
    if not args.train_only and world == 1:
        _release_leg()
        out["eval"] = eval_bench(device)
        out["datapath"] = data_bench(device)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and not args.train_only:
            out["cpu_baseline"] = cpu_baseline()
            if not args.no_train:
                out["cpu_baseline_train"] = cpu_train_baseline()
                if not args.no_presets:
                    out["cpu_baseline_train_c3"] = cpu_train_c3_baseline()
        emit(out)
    if dist:
        dist.destroy_process_group()


LINE_MAX_BYTES = 4096
_CONTRACT_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "vs_baseline", "dtype", "data", "config", "pipeline_tflops", "roofline")
_ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_id", "avg_launch_ms",
                  "launches_timed", "flop_per_launch", "share_of_step")
_LEGS = ("train", "train_c3", "train_c4", "distill", "distill_unfrozen", "eval", "datapath")
_LEG_KEYS = ("value", "unit", "ms_per_step", "ms_per_batch", "avg_launch_ms", "pipeline_frac", "roofline")
_CPU_KEYS = ("value", "unit", "cores", "kind", "sample")


def _compact_roofline(r):
    if not isinstance(r, dict):
        return r
    return {k: r[k] for k in _ROOFLINE_KEYS if k in r}


def detail_path():
    """Where the full result object goes (call profiles, per-class tables, top layers, kernel descriptions):
    $HISEG_BENCH_DETAIL, else gpurun_out/bench_detail.json under the repo root."""
    return os.environ.get("HISEG_BENCH_DETAIL") or os.path.join(ROOT, "gpurun_out", "bench_detail.json")


def compact_line(out, detail=None):
    """The one stdout JSON line of a full run: the contract keys of the headline (C2) measurement, its roofline
    and CPU baseline, and per leg only value / unit / time / pipeline_frac / roofline.  Everything else stays in
    the detail file.  Bounded by LINE_MAX_BYTES (round 5's 22.5 KB line was cut off by the driver's stdout tail);
    if a pathological result would exceed it, leg rooflines and then legs are dropped, never the headline."""
    line = {k: out[k] for k in _CONTRACT_KEYS if k in out}
    if "roofline" in line:
        line["roofline"] = _compact_roofline(line["roofline"])
    for k in ("cpu_baseline", "cpu_baseline_train", "cpu_baseline_train_c3"):
        if isinstance(out.get(k), dict):
            line[k] = {kk: out[k][kk] for kk in _CPU_KEYS if kk in out[k]}
    legs = {}
    for leg in _LEGS:
        v = out.get(leg)
        if not isinstance(v, dict):
            continue
        c = {k: v[k] for k in _LEG_KEYS if k in v}
        if "roofline" in c:
            c["roofline"] = _compact_roofline(c["roofline"])
        legs[leg] = c
    if legs:
        line["legs"] = legs
    if detail:
        line["detail"] = os.path.relpath(detail, ROOT) if os.path.isabs(detail) else detail
    s = json.dumps(line, separators=(",", ":"))
    for leg in reversed(list(legs)):
        if len(s.encode()) <= LINE_MAX_BYTES:
            break
        legs[leg].pop("roofline", None)
        s = json.dumps(line, separators=(",", ":"))
    for key in ("cpu_baseline_train_c3", "cpu_baseline_train", "data", "legs"):
        if len(s.encode()) <= LINE_MAX_BYTES:
            break
        line.pop(key, None)
        s = json.dumps(line, separators=(",", ":"))
    return s


def emit(out):
    """Write the full object to the detail file, then print the compact line (rank 0)."""
    path = detail_path()
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    except OSError as e:
        print(f"bench.py: could not write {path}: {e}", file=sys.stderr)
        path = None
    print(compact_line(out, path), flush=True)


def _leg_in_child(leg, args):
    """Run one leg as `bench.py --leg <leg>` in a child process (one GPU) and return its JSON object; the child's
    stderr passes through."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--leg", leg, "--steps", str(args.steps), "--warmup",
           str(args.warmup), "--dtype", args.dtype, "--no-cpu-baseline"]
    if args.serial:
        cmd.append("--serial")
    if args.eager_train:
        cmd.append("--eager-train")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        print(f"bench.py: leg {leg} failed (exit {r.returncode})", file=sys.stderr)
        sys.exit(r.returncode or 1)
    return json.loads(lines[-1])


def infer_bench(args, device, dtype, rank, world, dist):
    import hiseg
    from hiseg import ops
    model = build_model(device, dtype)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = synthetic_batch(device, rank)

    gate = os.environ.get("HISEG_PIPE_GATE", "0") == "1"
    head_prio = os.environ.get("HISEG_PIPE_HEAD_PRIO", "1") == "1"
    runner = None if args.serial else hiseg.StreamPipelinedExport(wrapper, head_priority=head_prio, gate=gate)

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
                    "kernel_id": DOMINANT_KERNEL_ID,
                    "kernel": "conv_hwc_kernel (halo-tiled: 16x16-pixel x 128-Cout workgroup tiles, one 18x18 halo per 32-channel slice in LDS by LDS-DMA, each wave 32 Cout x all 256 pixels with its weights in MFMA fragment order streamed into registers one kx block ahead and every halo row's B fragment reused across the 3 ky taps, one barrier per slice, 2 workgroups per CU, LDS-staged epilogue) 256->256 3x3 @64x48 x256 ROIs",
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

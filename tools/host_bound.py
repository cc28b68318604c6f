"""Is the C2 inference step host-bound?  Times the Python enqueue of K pipelined steps (until
StreamPipelinedExport.run returns, no synchronize) against the wall time until the GPU finishes
(developer tool, GPU).  Usage: python tools/host_bound.py [--steps 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def train(preset, steps, graphed=False, ddp=False):
    """The same for a train leg's step (bench.train_bench's model, loss and FusedAdamW): eager, or replayed as one
    HIP graph (--graphed), optionally with the data-parallel exchange enabled over a world-1 RCCL group (--ddp:
    the bucketed all-reduces and the loss's count all-reduce captured into the graph).  preset b0: the B0-std
    32 x 8-ROI leg."""
    import filler
    import hiseg
    dev = torch.device("cuda", 0)
    if preset == "b0":
        model = bench.build_model(dev, torch.bfloat16).train()
        for m in (model.roi_align_mask, model.roi_align_rgb):
            m.spatial_scale_h, m.spatial_scale_w = bench.H, bench.W
        images, rois = bench.synthetic_batch(dev, 0)
        tgt = torch.from_numpy(filler.ellipse_targets(7, rois.shape[0], *bench.MASK_HW)).to(dev)
    else:
        kw = bench.preset_kwargs(preset)
        model = hiseg.create_rgb_hierarchical_model(**kw)
        filler.fill_module(model).eval()
        model = model.to(dev)
        hiseg.set_compute_dtype(model, torch.bfloat16)
        model.train()
        batch = 32 if preset == "b1" else 8
        g = torch.Generator().manual_seed(0)
        images = torch.rand(batch, 3, 640, 640, generator=g).to(dev)
        rois = torch.from_numpy(filler.box_rois(1, batch, 1)).to(dev)
        tgt = torch.from_numpy(filler.ellipse_targets(7, batch, *kw["mask_size"])).to(dev)
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True)
    st = {"opt": None}
    if ddp:
        import torch.distributed as dist
        from hiseg import distributed as HD
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        HD.enable_grad_sync(model, bucket_mb=float(os.environ.get("HB_BUCKET_MB", "25")))
        if os.environ.get("HB_NO_COUNT_SYNC") != "1":
            HD.sync_loss_class_weights(loss_fn)

    def step():
        logits, aux = model(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if st["opt"] is None:
            st["opt"] = hiseg.FusedAdamW(model, lr=1e-4, weight_decay=0.01, max_grad_norm=1.0)
        st["opt"].zero_grad()
        loss.backward()
        st["opt"].step()
    run = hiseg.GraphedStep(step, lambda: st["opt"]) if graphed else step
    for _ in range(3):
        run()
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        caps = f", captures {run.captures} after {run.calls} calls" if graphed else ""
        print(f"train {preset}{' graphed' if graphed else ''}{' ddp(rccl world 1)' if ddp else ''}: enqueue {1e3 * (t1 - t0) / steps:.2f} ms/step, wall {1e3 * (t2 - t0) / steps:.2f} ms/step{caps}",
              flush=True)
    if graphed and run.graph is not None:   # the replay call alone
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run.graph.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"   graph.replay() alone: {1e3 * (t1 - t0) / steps:.2f} ms/call enqueue", flush=True)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run.graph.replay()
            ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        print(f"   graph.replay() on an idle GPU: {1e3 * sorted(ts)[2]:.2f} ms", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--train", default=None, help="b0 / b1 / b7: time a train leg instead")
    ap.add_argument("--graphed", action="store_true", help="train leg replayed as one HIP graph per step")
    ap.add_argument("--ddp", action="store_true", help="train leg with the gradient exchange (RCCL, world size 1)")
    args = ap.parse_args()
    if args.train:
        return train(args.train, args.steps, args.graphed, args.ddp)
    import hiseg
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, torch.bfloat16)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = bench.synthetic_batch(dev, 0)
    pipe = hiseg.StreamPipelinedExport(wrapper)
    with torch.no_grad():
        for _ in range(3):
            pipe.run([(images, rois)] * 2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.run([(images, rois)] * args.steps)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"enqueue {1e3 * (t1 - t0) / args.steps:.2f} ms/step, wall {1e3 * (t2 - t0) / args.steps:.2f} ms/step",
                  flush=True)


if __name__ == "__main__":
    main()

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


def train(preset, steps):
    """The same for a train leg's eager step (bench.train_bench's model, loss and FusedAdamW)."""
    import filler
    import hiseg
    dev = torch.device("cuda", 0)
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
    opt = hiseg.FusedAdamW(model, lr=1e-4) if False else None
    st = {"opt": opt}

    def step():
        logits, aux = model(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if st["opt"] is None:
            st["opt"] = hiseg.FusedAdamW(model, lr=1e-4, weight_decay=0.01, max_grad_norm=1.0)
        st["opt"].zero_grad()
        loss.backward()
        st["opt"].step()
    for _ in range(3):
        step()
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"train {preset}: enqueue {1e3 * (t1 - t0) / steps:.2f} ms/step, wall {1e3 * (t2 - t0) / steps:.2f} ms/step",
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--train", default=None, help="b1 / b7: time a train leg instead")
    args = ap.parse_args()
    if args.train:
        return train(args.train, args.steps)
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

"""C2 inference phases timed alone (developer tool, GPU): the full-image UNet phase and the ROI head phase of
RGBHierarchicalExportWrapper, each over the bench batch on one stream, then the serial wrapper and the
two-stream schedule, so the critical path of the pipelined step can be read off.
Usage: python tools/phase_alone.py [--steps 10] [--only unet|head]"""
import argparse
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--only", default=None, choices=[None, "unet", "head"])
    args = ap.parse_args()
    import hiseg
    from hiseg import engine
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, torch.bfloat16)
    wrapper = hiseg.RGBHierarchicalExportWrapper(model)
    images, rois = bench.synthetic_batch(dev, 0)
    H, W = images.shape[-2:]
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale = (H, W)
        m.spatial_scale_h, m.spatial_scale_w = H, W
    with torch.no_grad():
        u, _ = engine.export_unet_phase(model, images)
        res = {}
        if args.only in (None, "unet"):
            res["unet_ms"] = timed(lambda: engine.export_unet_phase(model, images), args.steps)
        if args.only in (None, "head"):
            res["head_ms"] = timed(lambda: engine.export_head_phase(model, images, rois, u, wrapper.dilation_pixels),
                                   args.steps)
        if args.only is None:
            res["serial_ms"] = timed(lambda: wrapper(images, rois), args.steps)
            pipe = hiseg.StreamPipelinedExport(wrapper)
            res["pipelined_ms"] = timed(lambda: pipe.run([(images, rois)] * 4), args.steps) / 4
    print({k: round(v, 3) for k, v in res.items()})


if __name__ == "__main__":
    main()

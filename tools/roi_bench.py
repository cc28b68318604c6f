"""RoIAlign throughput at C2's shapes (developer tool, GPU): the RGB crop (3 channels of the 32 x 480 x 640 f32
images -> NHWC bf16, cstride 8) and the UNet-logit crop with the 1 -> 2 output_conv affine, 256 ROIs of 8 per image,
per-channel stores (HISEG_ROI_VEC=0) vs whole-pixel 16-B stores.  Reports us per launch (HIP events, 50 launches)
and GB/s of algorithmic bytes = output bytes written (cstride x 2 B per pixel) + the 4 bilinear taps' f32 reads per
output channel of the source (4 x Cin x 4 B per pixel; taps shared between neighbouring outputs are counted once per
output, so this is an upper bound of the unique bytes)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
from hiseg import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    B, H, W, per, oh, ow = 32, 480, 640, 8, 64, 48
    images = torch.rand(B, 3, H, W, device=dev, generator=g)
    u = torch.randn(B, 1, H, W, device=dev, generator=g)
    N = B * per
    x1 = torch.rand(N, device=dev, generator=g) * 400
    y1 = torch.rand(N, device=dev, generator=g) * 300
    rois = torch.stack([torch.arange(N, device=dev).float() // per, x1, y1,
                        x1 + 40 + torch.rand(N, device=dev, generator=g) * 200,
                        y1 + 40 + torch.rand(N, device=dev, generator=g) * 160], 1)
    aw, ab = torch.randn(2, device=dev), torch.randn(2, device=dev)
    out = {}
    for mode in ("0", "1"):
        os.environ["HISEG_ROI_VEC"] = mode
        for name, feat, kw, C, cin in (("rgb", images, {}, 3, 3), ("logit_affine", u, {"aff_w": aw, "aff_b": ab}, 2, 1)):
            o = ops.Act.new(N, oh, ow, C, torch.bfloat16, dev, zero=False)

            def run():
                ops.roi_align(feat, rois, oh, ow, 480.0, 640.0, True, out=o, zero_to=o.cstride, **kw)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 50 * 1e3
            px = N * oh * ow
            byts = px * o.cstride * 2 + px * 4 * cin * 4
            out[f"{name}_vec{mode}"] = {"us": round(us, 2), "GBps": round(byts / us / 1e3, 1), "bytes": byts}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

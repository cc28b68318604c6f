"""GPU probe: hiseg's f32 RoIAlign (NCHW inference form and the NHWC train form) against the oracle's f32
restatement on the f64 train-step test's inputs; prints the largest differences and their sample coordinates
(developer tool, round 4)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import filler  # noqa: E402
from oracle import roi_align as R  # noqa: E402


def main():
    import hiseg
    from hiseg import ops
    images = torch.from_numpy(filler.uniform(61, (2, 3, 96, 128)))
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]])
    ref = torch.from_numpy(R.roi_align(images.numpy(), rois.numpy(), 64, 48, 96, 128, True))
    m = hiseg.DynamicRoIAlign((96, 128), aligned=True)
    mine = m(images.cuda(), rois.cuda(), 64, 48).cpu()
    a = ops.Act.new(3, 64, 48, 3, torch.float32, torch.device("cuda"), zero=False)
    ops.roi_align(images.cuda(), rois.cuda(), 64, 48, 96, 128, True, out=a, zero_to=a.cstride)
    nhwc = a.t.view(3, 64, 48, a.cstride)[..., :3].permute(0, 3, 1, 2).cpu()
    for name, x in (("nchw", mine), ("nhwc", nhwc)):
        d = (x - ref).abs()
        print(f"{name}: max abs diff {d.max().item():.3e}, elements differing {(d > 0).sum().item()}/{d.numel()}",
              flush=True)
        idx = torch.nonzero(d == d.max())[:3]
        for n, c, i, j in idx.tolist():
            print(f"   roi {n} ch {c} (i {i}, j {j}): hiseg {x[n, c, i, j].item():.9f} oracle {ref[n, c, i, j].item():.9f}")


if __name__ == "__main__":
    main()

"""Golden vectors of Pillow's bilinear Image.resize (the reference's image resize, dataset.py:98-99).

Run in the build container (Pillow 12.2.0 is installed here; the reference's own dependency):
    python tests/golden/gen_data_golden.py
Writes tests/golden/data_resize.npz: per case a seeded random 8-bit RGB image and PIL's resized output
(up- and down-scaling, non-integer ratios, one-axis-only resizes, identity).
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
# (src w, src h) -> (dst w, dst h)
CASES = [((160, 120), (64, 48)), ((45, 33), (100, 70)), ((101, 77), (101, 40)), ((64, 64), (48, 64)),
         ((256, 200), (80, 60)), ((33, 47), (33, 47)), ((7, 5), (96, 80)), ((300, 17), (29, 130))]


def main():
    rng = np.random.default_rng(11)
    out = {}
    for i, (src, dst) in enumerate(CASES):
        img = rng.integers(0, 256, size=(src[1], src[0], 3), dtype=np.uint8)
        if i == 0:   # smooth content too (rounding of mid-range sums)
            img[:, :, 1] = (np.arange(src[0])[None, :] * 255 // (src[0] - 1)).astype(np.uint8)
        res = np.array(Image.fromarray(img).resize(dst, Image.BILINEAR))
        out[f"c{i}_src"] = img
        out[f"c{i}_dst"] = res
        out[f"c{i}_size"] = np.array(dst, np.int64)
    out["n"] = np.int64(len(CASES))
    np.savez_compressed(os.path.join(HERE, "data_resize.npz"), **out)


if __name__ == "__main__":
    main()

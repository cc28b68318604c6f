"""Training data path CPU restatement -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).

* ``pil_table`` / ``pil_resize``: Pillow's bilinear ``Image.resize`` for 8-bit images (libImaging/Resample.c:
  precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal/Vertical_8bpc, ImagingResampleInner's
  two passes), in numpy integer arithmetic.  Pinned to Pillow itself (tests/golden/data_resize.npz,
  tests/golden/gen_data_golden.py; Pillow is the reference's own dependency, dataset.py:8, 98).
* ``cv2_nearest``: cv2.resize(..., INTER_NEAREST) (OpenCV imgproc resize.cpp resizeNN: source index
  min(floor(x * (1 / (dst / src))), src - 1)).  cv2 is absent from this image: parity of this formula is
  unpinned (restated from OpenCV's published source).
* ``get_item``: COCOInstanceSegmentationDataset.__getitem__ without transform (dataset.py:91-291) on decoded
  inputs, written the reference's way (every instance mask resized to the image size, cropped, composed,
  resized to the mask size) so that it checks the GPU's fused gather independently.
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def pil_table(in_size: int, out_size: int):
    """(ksize, bounds [out, 2], kk int [out, ksize]) for box [0, in_size] (Resample.c precompute_coeffs)."""
    scale = filterscale = float(np.float32(in_size)) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = int(center + support + 0.5)
        xmax = min(xmax, in_size) - xmin
        k = [0.0] * ksize
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            k[x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                k[x] /= ww
        bounds[xx] = (xmin, xmax)
        for x in range(ksize):           # normalize_coeffs_8bpc
            kk[xx, x] = int(-0.5 + k[x] * (1 << PRECISION_BITS)) if k[x] < 0 else int(0.5 + k[x] * (1 << PRECISION_BITS))
    return ksize, bounds, kk


def _dense(bounds, kk, in_size):
    m = np.zeros((bounds.shape[0], in_size), np.int64)
    for o, (lo, n) in enumerate(bounds):
        m[o, lo:lo + n] = kk[o, :n]
    return m


def _clip8(ss):
    return np.clip(ss >> PRECISION_BITS, 0, 255).astype(np.uint8)


def pil_resize(img: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """Image.resize(size=(w, h), BILINEAR) of an 8-bit [H, W, C] array."""
    H, W, C = img.shape
    w_out, h_out = size
    _, vb, vk = pil_table(H, h_out)
    cur = img.astype(np.int64)
    if w_out != W:                                     # horizontal pass over the rows the vertical pass uses
        _, hb, hk = pil_table(W, w_out)
        y0, y1 = int(vb[0, 0]), int(vb[-1, 0] + vb[-1, 1])
        mh = _dense(hb, hk, W)
        cur = _clip8(np.einsum("ow,hwc->hoc", mh, cur[y0:y1]) + (1 << (PRECISION_BITS - 1))).astype(np.int64)
        vb = vb.copy()
        vb[:, 0] -= y0
    if h_out != H:
        mv = _dense(vb, vk, cur.shape[0])
        cur = _clip8(np.einsum("oh,hwc->owc", mv, cur) + (1 << (PRECISION_BITS - 1)))
    return cur.astype(np.uint8)


def cv2_nearest(src: np.ndarray, dsize: Tuple[int, int]) -> np.ndarray:
    """cv2.resize(src, dsize=(w, h), interpolation=INTER_NEAREST) for a 2-D array."""
    sh, sw = src.shape[:2]
    dw, dh = dsize
    ifx, ify = 1.0 / (dw / sw), 1.0 / (dh / sh)
    xs = np.minimum(np.floor(np.arange(dw) * ifx).astype(np.int64), sw - 1)
    ys = np.minimum(np.floor(np.arange(dh) * ify).astype(np.int64), sh - 1)
    return src[ys[:, None], xs[None, :]]


def get_item(image: np.ndarray, instance_masks: np.ndarray, bboxes: Sequence[Sequence[float]], target: int,
             mask_size=(56, 56), image_size=(640, 640), roi_padding=0.0, min_roi_size=16):
    """dataset.py:91-291 (transform None): (image f32 [3, H, W], roi_mask int64 [mh, mw], roi_norm f32 [4])."""
    orig_h, orig_w = image.shape[:2]
    img = pil_resize(image, image_size)                                              # :98-99
    masks = [cv2_nearest(m, image_size) for m in instance_masks]                     # :117
    boxes = []
    for (x, y, w, h) in bboxes:                                                      # :121-127
        boxes.append([x * image_size[0] / orig_w, y * image_size[1] / orig_h,
                      w * image_size[0] / orig_w, h * image_size[1] / orig_h])
    x, y, w, h = boxes[target]
    pad_x, pad_y = w * roi_padding, h * roi_padding                                  # :134-141
    x1, y1 = max(0, int(x - pad_x)), max(0, int(y - pad_y))
    x2, y2 = min(image_size[0], int(x + w + pad_x)), min(image_size[1], int(y + h + pad_y))
    if x2 - x1 < min_roi_size:                                                       # :143-152
        cx = (x1 + x2) // 2
        x1 = max(0, cx - min_roi_size // 2)
        x2 = min(image_size[0], x1 + min_roi_size)
    if y2 - y1 < min_roi_size:
        cy = (y1 + y2) // 2
        y1 = max(0, cy - min_roi_size // 2)
        y2 = min(image_size[1], y1 + min_roi_size)
    roi_mask = np.zeros((y2 - y1, x2 - x1), np.uint8)                                # :155-170
    roi_mask[masks[target][y1:y2, x1:x2] > 0] = 1
    for i, m in enumerate(masks):
        if i != target:
            o = m[y1:y2, x1:x2]
            roi_mask[(o > 0) & (roi_mask == 0)] = 2
    roi_norm = np.array([x1 / image_size[0], y1 / image_size[1], x2 / image_size[0], y2 / image_size[1]],
                        dtype=np.float32)                                            # :172-178
    ms = (int(mask_size[1]), int(mask_size[0])) if isinstance(mask_size, (tuple, list)) else (mask_size, mask_size)
    roi_mask = cv2_nearest(roi_mask, ms)                                             # :262-275
    image_f = (img.astype(np.float32) / 255.0).transpose(2, 0, 1)                    # :281-284
    return image_f, roi_mask.astype(np.int64), roi_norm

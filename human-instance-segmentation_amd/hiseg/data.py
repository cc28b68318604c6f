"""Training data path on the GPU: COCOInstanceSegmentationDataset.__getitem__
(src/human_edge_detection/dataset.py:85-291, no augmentation) + convert_batch_format
(dataset_adapter.py:7-52) for a batch of decoded samples.

The reference decodes, resizes and rasterises every sample on a CPU DataLoader worker (PIL resize, one
cv2.resize per instance mask to the full image size, numpy masking, another cv2.resize to the mask size).
Here the host keeps only what is inherently host work -- decoding (PIL / pycocotools, outside) and the
per-sample ROI box arithmetic (a few float operations, done exactly as the reference) -- and two HIP passes
produce the batch on the device (include/hiseg_data.h):

* images: Pillow's bilinear resample (same 22-bit fixed-point tables, same two passes and 8-bit rounding,
  so the pixels equal PIL's), written straight as float32 CHW / 255;
* ROI targets: one gather per output pixel through the composed nearest-neighbour maps
  (ROI -> mask size, image size -> original mask size) -- the full-size instance masks the reference
  materialises per instance are never built.

Every function fails loudly without the HIP library; nothing falls back to the CPU.
"""
from __future__ import annotations

import ctypes
from functools import lru_cache
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L


@lru_cache(maxsize=256)
def pil_bilinear_table(in_size: int, out_size: int) -> Tuple[int, np.ndarray, np.ndarray]:
    """(ksize, bounds int32 [out, 2], weights int32 [out, ksize]) of Pillow's bilinear resample along one
    axis (Resample.c precompute_coeffs + normalize_coeffs_8bpc), computed by libhiseg on the host."""
    lib = L.lib()
    k = ctypes.c_int(0)
    L.check(lib.hiseg_pil_bilinear_table(in_size, out_size, ctypes.byref(k), None, None), "pil_bilinear_table")
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, k.value), np.int32)
    L.check(lib.hiseg_pil_bilinear_table(in_size, out_size, ctypes.byref(k), bounds.ctypes.data, kk.ctypes.data),
            "pil_bilinear_table")
    return k.value, bounds, kk


_DEV_TABLES: Dict[Tuple[int, int, str], Tuple[int, torch.Tensor, torch.Tensor, int, int]] = {}


def _identity_table(n: int):
    return 1, np.stack([np.arange(n, dtype=np.int32), np.ones(n, np.int32)], 1), np.full((n, 1), 1 << 22, np.int32)


def _device_table(in_size: int, out_size: int, device, identity: bool = False):
    key = (in_size, out_size, str(device), identity)
    t = _DEV_TABLES.get(key)
    if t is None:
        ks, bounds, kk = _identity_table(in_size) if identity else pil_bilinear_table(in_size, out_size)
        t = (ks, torch.from_numpy(np.ascontiguousarray(bounds)).to(device),
             torch.from_numpy(np.ascontiguousarray(kk)).to(device), int(bounds[0, 0]),
             int(bounds[-1, 0] + bounds[-1, 1]))
        _DEV_TABLES[key] = t
    return t


def resize_bilinear_pil(images: torch.Tensor, size: Tuple[int, int], out_f32: bool = True) -> torch.Tensor:
    """``PIL.Image.resize(size, Image.BILINEAR)`` of a batch of 8-bit images ``[B, H, W, C]`` (C 1..4) on the
    GPU; ``size`` = (width, height) as PIL's.  Returns float32 ``[B, C, h, w]`` with value / 255
    (dataset.py:281-284) or, with ``out_f32=False``, uint8 ``[B, h, w, C]``."""
    if not images.is_cuda:
        raise RuntimeError("hiseg data path runs on the GPU only (got a CPU tensor)")
    if images.dtype != torch.uint8 or images.dim() != 4 or not 1 <= images.shape[3] <= 4:
        raise ValueError(f"resize_bilinear_pil: expected uint8 [B, H, W, C<=4], got {images.dtype} {tuple(images.shape)}")
    B, H, W, C = images.shape
    w_out, h_out = int(size[0]), int(size[1])
    src = images.contiguous()
    lib = L.lib()
    s = L.stream_ptr()
    need_h, need_v = w_out != W, h_out != H              # Resample.c ImagingResampleInner (box = whole image)
    vks, vb, vk, y_first, y_last = _device_table(H, h_out, src.device, identity=not need_v)
    if need_h:
        hks, hb, hk, _, _ = _device_table(W, w_out, src.device)
        rows = y_last - y_first
        tmp = torch.empty(B, rows, w_out, C, dtype=torch.uint8, device=src.device)
        L.check(lib.hiseg_pil_resample_h(src.data_ptr(), B, H, W, C, y_first, rows, w_out, hks, hb.data_ptr(),
                                         hk.data_ptr(), tmp.data_ptr(), s), "pil_resample_h")
        vb = vb.clone()
        vb[:, 0] -= y_first                                # bounds of the vertical pass relative to tmp's rows
    else:
        tmp, rows = src, H
    if out_f32:
        out = torch.empty(B, C, h_out, w_out, dtype=torch.float32, device=src.device)
    else:
        out = torch.empty(B, h_out, w_out, C, dtype=torch.uint8, device=src.device)
    L.check(lib.hiseg_pil_resample_v(tmp.data_ptr(), B, rows, w_out, C, h_out, vks, vb.data_ptr(), vk.data_ptr(),
                                     int(out_f32), out.data_ptr(), s), "pil_resample_v")
    return out


def roi_box(bbox: Sequence[float], orig_wh: Tuple[int, int], image_size: Tuple[int, int], roi_padding: float = 0.0,
            min_roi_size: int = 16) -> Tuple[int, int, int, int]:
    """dataset.py:122-147: the COCO box scaled to the image size, padded, truncated to int, clamped, and
    widened to the minimum size (Python float arithmetic as the reference)."""
    ow, oh = orig_wh
    x, y, w, h = bbox
    x = x * image_size[0] / ow
    y = y * image_size[1] / oh
    w = w * image_size[0] / ow
    h = h * image_size[1] / oh
    pad_x, pad_y = w * roi_padding, h * roi_padding
    x1 = max(0, int(x - pad_x))
    y1 = max(0, int(y - pad_y))
    x2 = min(image_size[0], int(x + w + pad_x))
    y2 = min(image_size[1], int(y + h + pad_y))
    if x2 - x1 < min_roi_size:
        cx = (x1 + x2) // 2
        x1 = max(0, cx - min_roi_size // 2)
        x2 = min(image_size[0], x1 + min_roi_size)
    if y2 - y1 < min_roi_size:
        cy = (y1 + y2) // 2
        y1 = max(0, cy - min_roi_size // 2)
        y2 = min(image_size[1], y1 + min_roi_size)
    return x1, y1, x2, y2


def roi_targets(masks: torch.Tensor, descs: List[Tuple[int, int, int, int, int, int, int, int, int]],
                mask_size: Tuple[int, int], image_size: Tuple[int, int]) -> torch.Tensor:
    """3-class ROI targets int64 ``[B, mh, mw]`` (dataset.py:117, 149-160, 268-275) for B samples.
    ``masks``: uint8 device buffer holding every sample's instance masks back to back; ``descs``: per sample
    (mask element offset, n_inst, target, h0, w0, x1, y1, x2, y2) with the ROI in image-size pixels."""
    if not masks.is_cuda:
        raise RuntimeError("hiseg data path runs on the GPU only (got a CPU tensor)")
    mh, mw = int(mask_size[0]), int(mask_size[1])
    B = len(descs)
    arr = (L.RoiTargetDesc * B)()
    total = masks.numel()
    for i, (off, n, t, h0, w0, x1, y1, x2, y2) in enumerate(descs):
        if not (0 <= t < n and h0 > 0 and w0 > 0 and 0 <= off and off + n * h0 * w0 <= total):
            raise ValueError(f"roi_targets: sample {i}: bad instance-mask description")
        if not (0 <= x1 < x2 <= image_size[0] and 0 <= y1 < y2 <= image_size[1]):
            raise ValueError(f"roi_targets: sample {i}: empty or out-of-image ROI ({x1},{y1},{x2},{y2})")
        arr[i] = L.RoiTargetDesc(off, n, t, h0, w0, x1, y1, x2, y2, int(image_size[0]), int(image_size[1]))
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    dev = host.to(masks.device)
    out = torch.empty(B, mh, mw, dtype=torch.int64, device=masks.device)
    L.check(L.lib().hiseg_roi_targets(masks.data_ptr(), dev.data_ptr(), B, mh, mw, out.data_ptr(), L.stream_ptr()),
            "roi_targets")
    dev.record_stream(torch.cuda.current_stream(masks.device))
    return out


class GpuRoiBatchBuilder:
    """Builds the training batch of COCOInstanceSegmentationDataset + convert_batch_format on the GPU.

    ``build(samples)`` with samples = dicts {'image': uint8 [H0, W0, 3] (decoded RGB, numpy or tensor),
    'instance_masks': uint8 [K, H0, W0] (annToMask / RLE-decoded), 'bboxes': K COCO boxes [x, y, w, h] in
    original pixels, 'target': index of the target instance, 'image_id' (optional)} returns
    {'image' f32 [B, 3, H, W], 'roi_boxes' f32 [B, 5], 'roi_masks' int64 [B, mh, mw], 'instance_info'} on the
    device, with the reference's values.  Constructor arguments as the reference dataset's (mask_size is
    (height, width); image_size is (width, height), as PIL / cv2 take it)."""

    def __init__(self, device="cuda", mask_size: Tuple[int, int] = (56, 56), image_size: Tuple[int, int] = (640, 640),
                 roi_padding: float = 0.0, min_roi_size: int = 16, feature_size: Tuple[int, int] = (80, 80)):
        self.device = torch.device(device)
        self.mask_size = tuple(mask_size) if isinstance(mask_size, (tuple, list)) else (mask_size, mask_size)
        self.image_size, self.roi_padding, self.min_roi_size = tuple(image_size), roi_padding, min_roi_size
        self.feature_size = feature_size

    def build(self, samples: List[dict]) -> dict:
        dev = self.device
        B = len(samples)
        imgs = [torch.as_tensor(s["image"]) for s in samples]
        # images: one batched resample per distinct source size
        out = torch.empty(B, 3, self.image_size[1], self.image_size[0], dtype=torch.float32, device=dev)
        by_size: Dict[Tuple[int, int], List[int]] = {}
        for i, im in enumerate(imgs):
            by_size.setdefault(tuple(im.shape), []).append(i)
        for shape, idx in by_size.items():
            batch = torch.stack([imgs[i] for i in idx]).to(dev, non_blocking=True)
            res = resize_bilinear_pil(batch, self.image_size)
            out[torch.tensor(idx, device=dev)] = res
        # ROI boxes (host arithmetic, dataset.py:122-147, 163-168) and the instance masks in one buffer
        descs, chunks, norms = [], [], []
        off = 0
        for s, im in zip(samples, imgs):
            m = torch.as_tensor(s["instance_masks"])
            k, h0, w0 = m.shape
            oh, ow = im.shape[0], im.shape[1]
            if (h0, w0) != (oh, ow):
                raise ValueError("instance masks must have the decoded image's size (annToMask)")
            x1, y1, x2, y2 = roi_box(s["bboxes"][s["target"]], (ow, oh), self.image_size, self.roi_padding,
                                     self.min_roi_size)
            descs.append((off, k, int(s["target"]), h0, w0, x1, y1, x2, y2))
            chunks.append(m.reshape(-1).to(torch.uint8))
            off += m.numel()
            norms.append(np.array([x1 / self.image_size[0], y1 / self.image_size[1], x2 / self.image_size[0],
                                   y2 / self.image_size[1]], dtype=np.float32))
        masks = torch.cat(chunks).to(dev, non_blocking=True)
        roi_masks = roi_targets(masks, descs, self.mask_size, self.image_size)
        roi_boxes = torch.tensor([[i, *n.tolist()] for i, n in enumerate(norms)], dtype=torch.float32).to(dev)
        info = [{"image_id": s.get("image_id", 0), "instance_masks": [],
                 "instance_distances": torch.zeros(self.mask_size, dtype=torch.float32, device=dev)} for s in samples]
        return {"image": out, "roi_boxes": roi_boxes, "roi_masks": roi_masks, "instance_info": info}

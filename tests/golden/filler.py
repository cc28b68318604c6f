"""Deterministic, name-keyed parameter filler shared by the golden-vector generator and the tests.

Every parameter/buffer gets values from numpy PCG64 seeded by (seed, crc32(state_dict key)), so two
modules with the same state_dict keys (the reference's and hiseg's) receive identical weights without
committing any weight file.  Test infrastructure only.
"""
import zlib

import numpy as np
import torch
import torch.nn as nn


def _rng(seed: int, name: str):
    return np.random.default_rng([seed, zlib.crc32(name.encode())])


def fill_module(module: nn.Module, seed: int = 0) -> nn.Module:
    with torch.no_grad():
        for mname, m in module.named_modules():
            prefix = mname + "." if mname else ""
            for pname, t in list(m.named_parameters(recurse=False)) + list(m.named_buffers(recurse=False)):
                name = prefix + pname
                if pname == "num_batches_tracked" or pname in ("norm_mean", "norm_std"):
                    continue
                u = _rng(seed, name).uniform(-1.0, 1.0, size=tuple(t.shape)).astype(np.float32)
                if isinstance(m, nn.BatchNorm2d):
                    v = {"weight": 1.0 + 0.1 * u, "bias": 0.1 * u, "running_mean": 0.1 * u,
                         "running_var": 1.0 + 0.5 * np.abs(u)}[pname]
                elif isinstance(m, nn.ConvTranspose2d):
                    v = u * np.sqrt(3.0 / t.shape[0]) if pname == "weight" else 0.1 * u
                elif isinstance(m, nn.Conv2d):
                    fan_in = t[0].numel() if pname == "weight" else 1
                    v = u * np.sqrt(3.0 / fan_in) if pname == "weight" else 0.1 * u
                elif pname == "threshold":
                    v = 0.3 + 0.05 * u
                else:
                    v = 1.0 + 0.1 * u if pname == "weight" else 0.1 * u
                t.copy_(torch.from_numpy(np.asarray(v, dtype=np.float32)).reshape(t.shape))
    return module


def uniform(seed: int, shape, lo=0.0, hi=1.0) -> np.ndarray:
    return np.random.default_rng(seed).uniform(lo, hi, size=shape).astype(np.float32)


def normal(seed: int, shape) -> np.ndarray:
    return np.random.default_rng(seed).standard_normal(size=shape).astype(np.float32)


def box_rois(seed: int, n_images: int, per_image: int) -> np.ndarray:
    """SURVEY.md §8d box generator: w~U(.10,.45), h~U(.30,.95), x1~U(0,1-w), y1~U(0,1-h)."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_images):
        for _ in range(per_image):
            w = rng.uniform(0.10, 0.45)
            h = rng.uniform(0.30, 0.95)
            x1 = rng.uniform(0.0, 1.0 - w)
            y1 = rng.uniform(0.0, 1.0 - h)
            out.append([b, x1, y1, x1 + w, y1 + h])
    return np.asarray(out, dtype=np.float32)


def ellipse_targets(seed: int, n: int, mh: int, mw: int) -> np.ndarray:
    """SURVEY.md §8d synthetic 3-class ROI targets (int64 [n, mh, mw]): class 1 = an ellipse filling
    ~35 % of the ROI, class 2 = an offset ellipse ~15 % (drawn over class 1), 0 elsewhere."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:mh, 0:mw].astype(np.float32)
    out = np.zeros((n, mh, mw), dtype=np.int64)
    for i in range(n):
        cy, cx = rng.uniform(0.35, 0.65) * mh, rng.uniform(0.35, 0.65) * mw
        ry, rx = rng.uniform(0.30, 0.40) * mh, rng.uniform(0.28, 0.36) * mw
        e1 = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
        oy, ox = cy + rng.uniform(-0.3, 0.3) * mh, cx + rng.uniform(-0.35, 0.35) * mw
        sy, sx = rng.uniform(0.18, 0.26) * mh, rng.uniform(0.16, 0.24) * mw
        e2 = ((yy - oy) / sy) ** 2 + ((xx - ox) / sx) ** 2 <= 1.0
        out[i][e1] = 1
        out[i][e2] = 2
    return out

"""DynamicRoIAlign restated in numpy float32 (src/human_edge_detection/dynamic_roi_align.py:56-171).

Test infrastructure only.  Arithmetic order follows the reference on the CPU:
  linspace (:110-111, torch's two-sided formula), fx = x1 + g*(x2-x1) (:133-134),
  normalisation (:139-146), grid_sample unnormalise + bilinear with zero padding (:163-169,
  ATen's vectorised CPU grid sampler: (n+1)*((W-1)/2) for align_corners, (n+1)*(W/2)-0.5 otherwise).
"""
import numpy as np

f32 = np.float32


def linspace01(steps: int) -> np.ndarray:
    if steps == 1:
        return np.zeros(1, f32)
    step = f32(1.0) / f32(steps - 1)
    i = np.arange(steps)
    half = steps // 2
    lo = step * i.astype(f32)
    hi = f32(1.0) - step * (steps - 1 - i).astype(f32)
    return np.where(i < half, lo, hi).astype(f32)


def _unnorm(f: np.ndarray, size: int, aligned: bool) -> np.ndarray:
    if aligned:
        n = (f / f32(size - 1)) * f32(2) - f32(1)
        return (n + f32(1)) * (f32(size - 1) / f32(2))
    n = (f / f32(size)) * f32(2) - f32(1)
    return (n + f32(1)) * (f32(size) / f32(2)) - f32(0.5)


def roi_align(feat: np.ndarray, rois: np.ndarray, oh: int, ow: int, scale_h: float, scale_w: float,
              aligned: bool) -> np.ndarray:
    feat = np.asarray(feat, f32)
    rois = np.asarray(rois, f32)
    B, C, H, W = feat.shape
    N = rois.shape[0]
    b = np.trunc(rois[:, 0]).astype(np.int64)
    x1 = rois[:, 1] * f32(scale_w)
    y1 = rois[:, 2] * f32(scale_h)
    x2 = rois[:, 3] * f32(scale_w)
    y2 = rois[:, 4] * f32(scale_h)
    gx, gy = linspace01(ow), linspace01(oh)
    fx = x1[:, None] + gx[None, :] * (x2 - x1)[:, None]          # [N, ow]
    fy = y1[:, None] + gy[None, :] * (y2 - y1)[:, None]          # [N, oh]
    ix, iy = _unnorm(fx, W, aligned), _unnorm(fy, H, aligned)
    x0, y0 = np.floor(ix), np.floor(iy)
    wgt_w = ix - x0
    wgt_e = f32(1) - wgt_w
    wgt_n = iy - y0
    wgt_s = f32(1) - wgt_n
    x0i, y0i = x0.astype(np.int64), y0.astype(np.int64)
    out = np.zeros((N, C, oh, ow), f32)
    for n in range(N):
        if not (0 <= b[n] < B):
            continue
        fm = feat[b[n]]                                           # [C, H, W]

        def tap(yy, xx):
            ok = ((yy >= 0) & (yy < H))[:, None] & ((xx >= 0) & (xx < W))[None, :]
            v = fm[:, np.clip(yy, 0, H - 1)][:, :, np.clip(xx, 0, W - 1)]  # [C, oh, ow]
            return np.where(ok[None], v, f32(0))

        nw = wgt_s[n][:, None] * wgt_e[n][None, :]
        ne = wgt_s[n][:, None] * wgt_w[n][None, :]
        sw = wgt_n[n][:, None] * wgt_e[n][None, :]
        se = wgt_n[n][:, None] * wgt_w[n][None, :]
        v = tap(y0i[n], x0i[n]) * nw[None]
        v = v + tap(y0i[n], x0i[n] + 1) * ne[None]
        v = v + tap(y0i[n] + 1, x0i[n]) * sw[None]
        v = v + tap(y0i[n] + 1, x0i[n] + 1) * se[None]
        out[n] = v
    return out

"""Training data path on the GPU (hiseg.data over include/hiseg_data.h) against Pillow's resize
(tests/golden/data_resize.npz) and the CPU restatement of dataset.py (oracle/data.py)."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cases():
    z = np.load(os.path.join(ROOT, "tests", "golden", "data_resize.npz"))
    return [(z[f"c{i}_src"], z[f"c{i}_dst"], tuple(int(v) for v in z[f"c{i}_size"])) for i in range(int(z["n"]))]


def test_resize_matches_pillow_bit_exactly():
    from hiseg.data import resize_bilinear_pil
    for src, dst, size in _cases():
        x = torch.from_numpy(src)[None].to(DEV)
        u8 = resize_bilinear_pil(x, size, out_f32=False)[0].cpu().numpy()
        np.testing.assert_array_equal(u8, dst, err_msg=str((src.shape, size)))
        f = resize_bilinear_pil(x, size)[0].cpu().numpy()
        np.testing.assert_array_equal(f, (dst.astype(np.float32) / 255.0).transpose(2, 0, 1))


def test_resize_batched_and_single_channel():
    from hiseg.data import resize_bilinear_pil
    import oracle.data as OD
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, size=(3, 61, 83, 1), dtype=np.uint8)
    out = resize_bilinear_pil(torch.from_numpy(imgs).to(DEV), (40, 97), out_f32=False).cpu().numpy()
    for i in range(3):
        np.testing.assert_array_equal(out[i], OD.pil_resize(imgs[i], (40, 97)))


def _ellipses(rng, k, h, w):
    yy, xx = np.mgrid[0:h, 0:w]
    m = np.zeros((k, h, w), np.uint8)
    boxes = []
    for i in range(k):
        cy, cx = rng.uniform(0.2 * h, 0.8 * h), rng.uniform(0.2 * w, 0.8 * w)
        ry, rx = rng.uniform(0.1 * h, 0.4 * h), rng.uniform(0.1 * w, 0.4 * w)
        m[i] = (((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 < 1).astype(np.uint8)
        ys, xs = np.nonzero(m[i])
        boxes.append([float(xs.min()), float(ys.min()), float(xs.max() - xs.min() + 1), float(ys.max() - ys.min() + 1)])
    return m, boxes


@pytest.mark.parametrize("mask_size,image_size,pad", [((56, 56), (640, 640), 0.0), ((128, 96), (320, 240), 0.1)])
def test_batch_builder_matches_dataset_restatement(mask_size, image_size, pad):
    """dataset.py __getitem__ + convert_batch_format for 6 samples of 3 source sizes (some sharing a size,
    so one resize launch covers several images), overlapping instances, boxes near the border."""
    import oracle.data as OD
    from hiseg.data import GpuRoiBatchBuilder
    rng = np.random.default_rng(17)
    samples = []
    for i, (h, w) in enumerate([(180, 240), (180, 240), (97, 131), (300, 200), (97, 131), (180, 240)]):
        img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        k = int(rng.integers(1, 5))
        m, boxes = _ellipses(rng, k, h, w)
        samples.append({"image": img, "instance_masks": m, "bboxes": boxes, "target": int(rng.integers(0, k)),
                        "image_id": i})
    b = GpuRoiBatchBuilder(DEV, mask_size=mask_size, image_size=image_size, roi_padding=pad).build(samples)
    assert b["image"].shape == (6, 3, image_size[1], image_size[0])
    for i, s in enumerate(samples):
        img, roi_mask, norm = OD.get_item(s["image"], s["instance_masks"], s["bboxes"], s["target"], mask_size,
                                          image_size, pad)
        np.testing.assert_array_equal(b["image"][i].cpu().numpy(), img, err_msg=f"image {i}")
        np.testing.assert_array_equal(b["roi_masks"][i].cpu().numpy(), roi_mask, err_msg=f"roi mask {i}")
        np.testing.assert_array_equal(b["roi_boxes"][i].cpu().numpy(), np.array([i, *norm], np.float32))
    assert set(np.unique(b["roi_masks"].cpu().numpy())) <= {0, 1, 2}
    assert [d["image_id"] for d in b["instance_info"]] == list(range(6))


def test_full_size_batch_properties():
    """C3-sized batch: 32 decoded 480x640 images -> 640x640; two sampled images against the restatement,
    every image's mean within 1/255 of the source mean (resampling preserves the mean)."""
    import oracle.data as OD
    from hiseg.data import resize_bilinear_pil
    g = torch.Generator(device=DEV).manual_seed(0)
    imgs = torch.randint(0, 256, (32, 480, 640, 3), dtype=torch.uint8, device=DEV, generator=g)
    out = resize_bilinear_pil(imgs, (640, 640))
    assert out.shape == (32, 3, 640, 640)
    for i in (0, 31):
        want = OD.pil_resize(imgs[i].cpu().numpy(), (640, 640))
        np.testing.assert_array_equal(out[i].cpu().numpy(), (want.astype(np.float32) / 255.0).transpose(2, 0, 1))
    src_mean = imgs.float().mean(dim=(1, 2)) / 255.0
    assert (out.mean(dim=(2, 3)) - src_mean).abs().max().item() < 1.0 / 255

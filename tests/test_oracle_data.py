"""Training data path: the CPU restatement (oracle/data.py) against Pillow's own resize
(tests/golden/data_resize.npz), libhiseg's host-side resample tables against the restatement, and the
host ROI-box arithmetic of hiseg.data against the oracle's (dataset.py:122-147)."""
import os

import numpy as np
import pytest

from conftest import ROOT


def _cases():
    z = np.load(os.path.join(ROOT, "tests", "golden", "data_resize.npz"))
    return [(z[f"c{i}_src"], z[f"c{i}_dst"], tuple(int(v) for v in z[f"c{i}_size"])) for i in range(int(z["n"]))]


def test_oracle_resize_matches_pillow():
    import oracle.data as OD
    for src, dst, size in _cases():
        np.testing.assert_array_equal(OD.pil_resize(src, size), dst, err_msg=str((src.shape, size)))


def test_library_resample_tables_match_the_restatement():
    import oracle.data as OD
    from hiseg import data as HD
    pairs = {(s.shape[1], size[0]) for s, _, size in _cases()} | {(s.shape[0], size[1]) for s, _, size in _cases()}
    pairs |= {(1920, 640), (1080, 640), (480, 640), (640, 640), (1, 7), (1000, 3)}
    for n_in, n_out in sorted(pairs):
        k1, b1, kk1 = OD.pil_table(n_in, n_out)
        k2, b2, kk2 = HD.pil_bilinear_table(n_in, n_out)
        assert k1 == k2, (n_in, n_out)
        np.testing.assert_array_equal(b1, b2)
        np.testing.assert_array_equal(kk1, kk2)


@pytest.mark.parametrize("pad,minsz", [(0.0, 16), (0.1, 16), (0.0, 64)])
def test_roi_box_arithmetic_matches_oracle(pad, minsz):
    import oracle.data as OD
    from hiseg.data import roi_box
    rng = np.random.default_rng(3)
    for _ in range(60):
        ow, oh = int(rng.integers(20, 160)), int(rng.integers(20, 160))
        w, h = float(rng.uniform(1, ow)), float(rng.uniform(1, oh))
        x, y = float(rng.uniform(0, ow - w)), float(rng.uniform(0, oh - h))
        size = (int(rng.integers(32, 200)), int(rng.integers(32, 200)))
        box = roi_box((x, y, w, h), (ow, oh), size, pad, minsz)
        _, _, norm = OD.get_item(np.zeros((oh, ow, 3), np.uint8), np.zeros((1, oh, ow), np.uint8), [(x, y, w, h)],
                                 0, (4, 4), size, pad, minsz)
        want = np.array([box[0] / size[0], box[1] / size[1], box[2] / size[0], box[3] / size[1]], np.float32)
        np.testing.assert_array_equal(norm, want)
        assert 0 <= box[0] < box[2] <= size[0] and 0 <= box[1] < box[3] <= size[1]


def test_data_entry_points_refuse_cpu_tensors():
    import torch
    from hiseg.data import resize_bilinear_pil
    with pytest.raises(RuntimeError, match="GPU only"):
        resize_bilinear_pil(torch.zeros(1, 4, 4, 3, dtype=torch.uint8), (2, 2))

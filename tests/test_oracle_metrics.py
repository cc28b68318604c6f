"""Validation metrics: the CPU restatement (oracle/metrics.py) and the host arithmetic of hiseg.metrics
against the reference's own evaluate_model (tests/golden/metrics.npz, gen_metrics_golden.py)."""
import os

import numpy as np
import pytest

from conftest import ROOT


def _golden():
    z = np.load(os.path.join(ROOT, "tests", "golden", "metrics.npz"))
    nb = int(z["num_batches"])
    batches = [(z[f"b{i}_logits"], z[f"b{i}_masks"]) for i in range(nb)]
    want = {str(k): z[f"m_{k}"] for k in z["metric_keys"]}
    return z, batches, want


def _check(got, want, keys):
    for k in keys:
        if k.startswith("conf_"):
            np.testing.assert_array_equal(np.asarray(got[k]), want[k], err_msg=k)
        else:
            assert float(got[k]) == float(want[k]), (k, float(got[k]), float(want[k]))


def test_oracle_matches_reference_evaluate_model():
    import oracle.metrics as OM
    _, batches, want = _golden()
    got = OM.evaluate_metrics(batches)
    keys = [k for k in want if k in got]
    assert len(keys) == len(got) == 15
    _check(got, want, keys)


def _histograms(batches, C=3):
    """per-sample (target row, predicted column) counts, numpy (the GPU kernel's contract)."""
    out = []
    for logits, masks in batches:
        pred = np.argmax(logits, axis=1)
        for p, t in zip(pred, masks):
            h = np.zeros((C + 2, C + 1), np.int64)
            rows = np.where(t < 0, C + 1, np.where(t >= C, C, t))
            np.add.at(h, (rows.ravel(), p.ravel()), 1)
            out.append(h)
    return np.stack(out)


def test_host_metric_arithmetic_matches_reference():
    from hiseg.metrics import metrics_from_histograms
    _, batches, want = _golden()
    got = metrics_from_histograms(_histograms(batches))
    keys = [k for k in want if k in got]
    assert len(keys) == 15
    _check(got, want, keys)


def test_host_metric_arithmetic_edge_cases():
    from hiseg.metrics import metrics_from_histograms
    import oracle.metrics as OM
    rng = np.random.default_rng(0)
    # all background, perfect prediction; a sample with only ignore values; a single pixel
    cases = [
        [(np.stack([np.full((2, 4, 4), 1.0), np.zeros((2, 4, 4)), np.zeros((2, 4, 4))], 1), np.zeros((2, 4, 4), np.int64))],
        [(rng.normal(size=(1, 3, 3, 3)), np.full((1, 3, 3), 255, np.int64))],
        [(rng.normal(size=(1, 3, 1, 1)), np.ones((1, 1, 1), np.int64))],
    ]
    for batches in cases:
        want = OM.evaluate_metrics(batches)
        got = metrics_from_histograms(_histograms(batches))
        assert set(got) == set(want)
        for k in want:
            np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=k)


def test_metric_entry_points_refuse_cpu_tensors():
    import torch
    from hiseg.metrics import seg_confusion
    with pytest.raises(RuntimeError, match="GPU only"):
        seg_confusion(torch.zeros(1, 3, 2, 2), torch.zeros(1, 2, 2, dtype=torch.int64))

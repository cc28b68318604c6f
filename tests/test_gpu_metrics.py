"""Validation metrics on the GPU (hiseg.metrics over hiseg_seg_confusion, include/hiseg_metrics.h) against
the reference's own evaluate_model (tests/golden/metrics.npz) and against exact host counts."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _np_hist(pred, masks, C=3):
    """numpy per-sample (target row, predicted column) counts (the kernel's contract)."""
    out = []
    for p, t in zip(pred, masks):
        h = np.zeros((C + 2, C + 1), np.int64)
        rows = np.where(t < 0, C + 1, np.where(t >= C, C, t))
        cols = np.where((p >= 0) & (p < C), p, C)
        np.add.at(h, (rows.ravel(), cols.ravel()), 1)
        out.append(h)
    return np.stack(out)


def _golden():
    from test_oracle_metrics import _golden as g
    return g()


def test_confusion_kernel_matches_host_counts_on_reference_batches():
    from hiseg.metrics import seg_confusion
    _, batches, _ = _golden()
    for logits, masks in batches:
        got = seg_confusion(torch.from_numpy(logits).to(DEV), torch.from_numpy(masks).to(DEV)).cpu().numpy()
        np.testing.assert_array_equal(got, _np_hist(np.argmax(logits, 1), masks))
        # bf16 logits: argmax of the bf16-rounded values
        lb = torch.from_numpy(logits).bfloat16()
        got = seg_confusion(lb.to(DEV), torch.from_numpy(masks).to(DEV)).cpu().numpy()
        np.testing.assert_array_equal(got, _np_hist(np.argmax(lb.float().numpy(), 1), masks))


def test_evaluate_model_matches_reference_golden():
    """The reference's evaluate_model run on recorded logits / loss values; here the same batches through
    hiseg.evaluate_model (device loss tensors, device histograms)."""
    import hiseg
    z, batches, want = _golden()
    keys = [str(k) for k in z["loss_keys"]]

    class Replay(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.k = 0

        def forward(self, images, rois):
            x = torch.from_numpy(batches[self.k][0]).to(DEV)
            self.k += 1
            return x, {}

    class ReplayLoss:
        k = 0

        def __call__(self, logits, masks, aux):
            i = ReplayLoss.k
            ReplayLoss.k += 1
            d = {k: float(v) for k, v in zip(keys, z[f"b{i}_loss_terms"])}
            return torch.tensor(float(z[f"b{i}_loss_total"]), device=DEV), d

    loader = [{"image": torch.zeros(m.shape[0], 3, 8, 8), "roi_boxes": torch.zeros(m.shape[0], 5),
               "roi_masks": torch.from_numpy(m)} for _, m in batches]
    got = hiseg.evaluate_model(Replay(), loader, ReplayLoss(), DEV)
    assert set(got) == set(want)
    for k in want:
        if k.startswith("conf_"):
            np.testing.assert_array_equal(got[k], want[k], err_msg=k)
        else:
            assert float(got[k]) == float(want[k]), (k, got[k], float(want[k]))


@pytest.mark.parametrize("C", [2, 3, 4])
def test_confusion_kernel_shapes_paths_and_large_batch(C):
    """vector and scalar paths (HW % 4, misaligned views), class-label input, out-of-range targets and
    labels, NaN logits, and a C2-sized batch (2048 ROI masks of 128 x 96) against torch's own argmax."""
    from hiseg.metrics import seg_confusion
    g = torch.Generator(device=DEV).manual_seed(C)
    for n, h, w in ((3, 7, 5), (2, 1, 1), (4, 16, 12), (2048, 128, 96)):
        lg = torch.round(torch.randn(n, C, h, w, device=DEV, generator=g) * 3) / 3
        tg = torch.randint(-1, C + 2, (n, h, w), device=DEV, generator=g)
        if n < 100:
            lg.view(-1)[::7] = float("nan")
        got = seg_confusion(lg, tg, C)
        pred = lg.argmax(1)
        rows = torch.where(tg < 0, C + 1, torch.where(tg >= C, C, tg))
        want = torch.zeros(n, C + 2, C + 1, dtype=torch.int64, device=DEV)
        want.view(n, -1).scatter_add_(1, (rows * (C + 1) + pred).view(n, -1), torch.ones_like(pred).view(n, -1))
        assert torch.equal(got, want), (n, h, w)
        # class-label input with out-of-range labels
        lab = torch.randint(-2, C + 2, (n, h, w), device=DEV, generator=g)
        got = seg_confusion(lab, tg, C)
        cols = torch.where((lab >= 0) & (lab < C), lab, C)
        want.zero_().view(n, -1).scatter_add_(1, (rows * (C + 1) + cols).view(n, -1), torch.ones_like(lab).view(n, -1))
        assert torch.equal(got, want), (n, h, w, "labels")
    # misaligned planes (scalar path) give the same counts as the aligned copy
    base = torch.randn(2 * 3 * 64 + 1, device=DEV, generator=g)
    lg = base[1:].view(2, 3, 8, 8)
    tg = torch.randint(0, 3, (2, 8, 8), device=DEV, generator=g)
    assert torch.equal(seg_confusion(lg, tg), seg_confusion(lg.clone(), tg))


def test_calculate_helpers_match_reference_definitions():
    import hiseg
    g = torch.Generator(device=DEV).manual_seed(5)
    pred = torch.randint(0, 3, (4, 20, 16), device=DEV, generator=g)
    tgt = torch.randint(0, 3, (4, 20, 16), device=DEV, generator=g)
    cm = hiseg.calculate_confusion_matrix(pred, tgt)
    want = torch.zeros(3, 3, dtype=torch.int64)
    for t in range(3):
        for p in range(3):
            want[t, p] = ((tgt == t) & (pred == p)).sum().cpu()
    assert torch.equal(cm.cpu(), want)
    a, b = pred == 1, tgt == 1
    ref = ((a & b).float().sum() / (a | b).float().sum()).item()
    assert hiseg.calculate_iou(a, b) == ref
    z = torch.zeros(5, 5, dtype=torch.bool, device=DEV)
    assert hiseg.calculate_iou(z, z) == 1.0


def test_evaluate_model_with_the_hip_model_and_loss():
    """hiseg model + RefinedHierarchicalLoss: the metrics equal the oracle's on the same logits, and the
    loss averages equal per-batch materialised values of an identically-driven second loss."""
    import filler
    import hiseg
    import oracle.metrics as OM
    from helpers import b0_kwargs, hiseg_kwargs
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(b0_kwargs()))).eval().to(DEV)
    loader, recorded = [], []
    for k in range(3):
        images = torch.from_numpy(filler.uniform(400 + k, (2, 3, 96, 128)))
        rois = torch.from_numpy(filler.box_rois(500 + k, 2, 2))
        masks = torch.from_numpy(filler.ellipse_targets(600 + k, 4, 128, 96))
        loader.append({"image": images, "roi_boxes": rois, "roi_masks": masks})
    kw = dict(use_boundary_aware_loss=True, use_contour_detection=True, use_distance_transform=True)
    got = hiseg.evaluate_model(m, loader, hiseg.RefinedHierarchicalLoss(**kw), DEV)
    loss2 = hiseg.RefinedHierarchicalLoss(**kw)
    tot = ce = bnd = 0.0
    with torch.no_grad():
        for b in loader:
            logits, aux = m(b["image"].to(DEV), b["roi_boxes"].to(DEV))
            recorded.append((logits.float().cpu().numpy(), b["roi_masks"].numpy()))
            loss, d = loss2(logits, b["roi_masks"].to(DEV), aux)
            tot += loss.item()
            ce += d["ce_loss"]
            bnd += d["boundary_aware"]
    assert got["total_loss"] == tot / 3 and got["ce_loss"] == ce / 3 and got["boundary_aware"] == bnd / 3
    want = OM.evaluate_metrics(recorded)
    for k in want:
        np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=k)

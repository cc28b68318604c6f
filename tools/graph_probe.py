"""Diagnostic (GPU): test_graphed_train_step_equals_eager's schedule repeated with the allocator poisoned before each
run: eager 4 steps vs GraphedStep 4 steps; per run the step losses and, at the first differing step, the parameters
whose gradients differ (developer tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import filler  # noqa: E402
import hiseg  # noqa: E402
from ddp_diff import poison  # noqa: E402
from test_gpu_train import _model  # noqa: E402

DEV = "cuda"


BIG = "--big" in sys.argv


def run(graphed, seed, per_step=False):
    if seed is not None:
        poison(seed, big=BIG)
    torch.manual_seed(0)
    images = torch.from_numpy(filler.uniform(31, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(32, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(33, 4, 128, 96)).to(DEV)
    m = _model(torch.bfloat16, p_drop_zero=False).to(DEV).train()
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    st = {"opt": None}

    def step():
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if st["opt"] is None:
            st["opt"] = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01, max_grad_norm=1.0)
        st["opt"].zero_grad()
        loss.backward()
        st["opt"].step()
        return loss

    r = hiseg.GraphedStep(step, lambda: st["opt"]) if graphed else step
    losses, grads, params = [], [], []
    for k in range(4):
        if per_step and seed is not None:
            poison(seed * 100 + k, big=BIG)
        losses.append(float(r().detach()))
        S = m.__dict__["_hiseg_train"]
        grads.append(S.flat.grad.clone())
        params.append(S.flat.data.clone())
    names = [(n, p.numel()) for n, p in S.flat.named]
    return losses, grads, params, names


def main():
    ref = run(False, None)
    print("eager ref", ref[0], flush=True)
    if "--ref-only" in sys.argv:   # e.g. under HISEG_PLACEMENT_FAR=1: the far-apart fallbacks on every two-source layer
        return
    for i, (graphed, seed) in enumerate(((False, 3), (False, 5), (False, 9), (False, 11), (True, 3), (True, 5),
                                         (False, 13), (False, 17))):
        l, g, p, names = run(graphed, seed, per_step=True)
        first = next((k for k in range(4) if l[k] != ref[0][k]), None)
        msg = f"run {i} graphed={graphed} poison-per-step={seed}: losses {l} first differing step {first}"
        if first is not None:
            off, bad = 0, []
            for n, k in names:
                if not torch.equal(g[first][off:off + k], ref[1][first][off:off + k]):
                    bad.append(n)
                off += k
            pd = (p[max(first - 1, 0)] - ref[2][max(first - 1, 0)]).abs().max().item()
            msg += f"; params before that step max diff {pd:.3e}; {len(bad)} grads differ, last: {bad[-5:]}"
        print(msg, flush=True)


if __name__ == "__main__":
    main()

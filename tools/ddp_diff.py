"""Diagnostic (GPU): repeat test_grad_sync_nccl_world1_matches_local's two B0 train steps with the gradient
exchange off / on / off / on in one process (RCCL world 1) and print, per run and step, which parameters'
gradients differ from the first run (developer tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "human-instance-segmentation_amd"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import filler  # noqa: E402
import hiseg  # noqa: E402
from hiseg import distributed as HD  # noqa: E402
from test_gpu_train import _model  # noqa: E402

DEV = "cuda"
LOSSES = []


def poison(seed, big=False):
    """Fill most of the caching allocator's free memory with random values, then free it again: an uninitialised
    read then changes the result from run to run.  big: also 0.5-3 GiB segments (the full GPU suite leaves such
    segments cached, and a run's tensors are then carved out of them)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    held = []
    sizes = [256 << 10] * 1000 + [(2 << 20) * k for k in (1, 2, 4, 8, 16, 32, 64)] * 4
    if big:
        sizes += [512 << 20, 1 << 30, 2 << 30, 3 << 30]
    for n in sizes:
        t = torch.empty(n // 4, dtype=torch.float32, device=DEV)
        t.uniform_(-1e3, 1e3, generator=g)
        held.append(t)
    del held


def run(sync, seed=None, mode="bcast"):
    if seed is not None:
        poison(seed)
    m = _model(torch.bfloat16).to(DEV).train()
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    if sync:
        gs = HD.enable_grad_sync(m, bucket_mb=1.0, broadcast_from=None if mode in ("nobcast", "nolaunch") else 0)
        if mode == "bcast_sync":
            torch.cuda.synchronize()
        if mode == "nolaunch":   # the exchange's bookkeeping without any collective
            gs._launch = lambda b: gs.launched.append(b)
    images = torch.from_numpy(filler.uniform(41, (2, 3, 96, 128))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(42, 2, 2)).to(DEV)
    tgt = torch.from_numpy(filler.ellipse_targets(43, 4, 128, 96)).to(DEV)
    loss_fn = hiseg.RefinedHierarchicalLoss(use_contour_detection=True, use_distance_transform=True)
    out = []
    for _ in range(2):
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        for p in m.parameters():
            p.grad = None
        loss.backward()
        torch.cuda.synchronize()
        out.append(m.__dict__["_hiseg_train"].flat.grad.clone())
        LOSSES.append(float(loss.detach()))
    return out, m


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    ref, m0 = run(False)
    flat = m0.__dict__["_hiseg_train"].flat
    offs = []
    off = 0
    for n, p in flat.named:
        offs.append((n, off, p.numel()))
        off += p.numel()
    cases = [(True, 3, "nolaunch"), (True, 5, "nolaunch"), (True, 7, "nolaunch"), (True, 3, "nobcast"),
             (True, 5, "bcast"), (True, 7, "bcast"), (True, 8, "bcast"), (True, 9, "nolaunch")]
    for i, (sync, seed, mode) in enumerate(cases):
        LOSSES.clear()
        out, _ = run(sync, seed, mode)
        for st in range(2):
            d = (out[st] - ref[st]).abs()
            big = int(d.argmax())
            print(f"   losses {LOSSES}  at argmax: got {out[st][big].item():.5e} ref {ref[st][big].item():.5e}")
            bad = [n for n, o, k in offs if d[o:o + k].max().item() > 0]
            print(f"run {i} sync={sync} {mode} poison={seed} step {st}: max diff {d.max().item():.3e}, {len(bad)} params differ: {bad[:6]}",
                  flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

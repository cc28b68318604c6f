"""Two-launch SE gate: determinism and weight-alignment independence probe (developer tool, GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "human-instance-segmentation_amd"))
from hiseg import ops  # noqa: E402

DEV = "cuda"
g = torch.Generator(device=DEV).manual_seed(43)
N, H, W, C, cr, k, stride = 4, 20, 20, 3840, 160, 5, 1
A = ops.Act.from_nchw(torch.randn(N, C, H, W, device=DEV, generator=g), torch.bfloat16)
wd = (torch.randn(k * k, C, device=DEV, generator=g) * 0.3).contiguous()
sc, sh = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.1
w1, b1 = torch.randn(cr, C, device=DEV, generator=g) * 0.1, torch.randn(cr, device=DEV, generator=g) * 0.1
w2, b2 = torch.randn(C, cr, device=DEV, generator=g) * 0.1, torch.randn(C, device=DEV, generator=g) * 0.1


def mis(w):
    return torch.empty(w.numel() + 1, device=DEV)[1:].view_as(w).copy_(w)


def gate(a, b):
    return ops.dwconv_se_gate(A, wd, sc, sh, k, stride, 3, a, b1, b, b2, 3)[1].clone()


g0 = gate(w1, w2)
for name, (a, b) in {"again": (w1, w2), "w1_misaligned": (mis(w1), w2), "w2_misaligned": (w1, mis(w2)),
                     "both": (mis(w1), mis(w2))}.items():
    gg = gate(a, b)
    print(name, torch.equal(gg, g0), (gg - g0).abs().max().item())

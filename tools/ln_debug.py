"""Developer check (GPU): the small variant heads (tests/golden/variants.npz) against the reference's
outputs, per output / aux key (f32)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "human-instance-segmentation_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests", "golden"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import filler  # noqa: E402
import hiseg  # noqa: E402
from helpers import VARIANTS, variant_modules  # noqa: E402

DEV = "cuda"
g = np.load(os.path.join(HERE, "..", "tests", "golden", "variants.npz"))
xh = torch.from_numpy(filler.normal(63, (2, 64, 16, 12)))
for key, (norm, act, beta) in VARIANTS.items():
    head = hiseg.set_compute_dtype(variant_modules(norm, act, beta)[2].to(DEV), torch.float32)
    with torch.no_grad():
        logits, aux = head(xh.to(DEV))
    res = {"logits": logits}
    res.update(aux)
    for k, v in res.items():
        name = f"{key}_head_logits" if k == "logits" else f"{key}_head_aux_{k}"
        if name not in g.files:
            print(key, k, "missing")
            continue
        r = torch.from_numpy(g[name]).double()
        e = (v.cpu().double() - r).abs().max().item() / max(1.0, r.abs().max().item())
        print(key, k, f"{e:.3g}", flush=True)

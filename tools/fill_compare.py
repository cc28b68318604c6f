"""Compare two tools/fill_probe.py --save dumps: per parameter (backward order: last forward layer first), the
first-step gradients that differ and by how much (developer tool)."""
import sys

import torch

a, b = (torch.load(p, weights_only=True) for p in sys.argv[1:3])
print("losses", a["losses"], b["losses"])
off, rows = 0, []
for n, k in a["names"]:
    ga, gb = a["grad0"][off:off + k], b["grad0"][off:off + k]
    if not torch.equal(ga, gb):
        rows.append((n, k, float((ga - gb).abs().max()), float(ga.abs().max())))
    off += k
print(len(rows), "of", len(a["names"]), "first-step gradients differ; in backward order:")
for r in reversed(rows[-40:]):
    print("  %-72s n=%-8d maxdiff %.3e (max |g| %.3e)" % r)
print("params after step 1 equal:", torch.equal(a["param0"], b["param0"]))

"""(DIAG=1 library: make -C human-instance-segmentation_amd DIAG=1; HISEG_LIB=.../libhiseg_diag.so)
Per-workgroup s_memtime breakdown (prologue / K loop / epilogue) of a conv variant (diagnostic)."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "human-instance-segmentation_amd"))
import torch
from tools.conv_bench import SHAPES, make, desc, run

name = sys.argv[1] if len(sys.argv) > 1 else "res256_3x3_64x48"
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 18
p, xa, xb, r, out = make(SHAPES[name], torch.bfloat16)
d = desc(p, xa, xb, r, out)
buf = torch.zeros(4 * 200000, dtype=torch.int64, device="cuda")
d.out2 = buf.data_ptr()
for _ in range(3):
    run(d, variant)
torch.cuda.synchronize()
t = buf.view(-1, 4).cpu()
t = t[t[:, 3] != 0].double()
pro, loop, epi = (t[:, 1] - t[:, 0]), (t[:, 2] - t[:, 1]), (t[:, 3] - t[:, 2])
span = t[:, 3].max() - t[:, 0].min()
print(f"{name} variant {variant}: {t.shape[0]} WGs, span {span:.0f} ticks")
for nm, v in (("prologue", pro), ("k-loop", loop), ("epilogue", epi)):
    print(f"  {nm:9s} mean {v.mean():9.0f}  median {v.median():9.0f}  max {v.max():9.0f}")
tot = (pro + loop + epi).mean()
print(f"  WG lifetime mean {tot:.0f}; shares: pro {pro.mean()/tot:.2%} loop {loop.mean()/tot:.2%} epi {epi.mean()/tot:.2%}")

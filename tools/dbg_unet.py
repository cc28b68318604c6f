"""Conditioning check: hiseg (GPU f32 / bf16) and the CPU f32 oracle, each against a float64 oracle."""
import sys, torch
sys.path[:0] = ['tests', 'tests/golden', '.', 'human-instance-segmentation_amd']
import test_gpu_train as G
import filler
from helpers import load
from hiseg.layers import EnhancedUNet
from hiseg.ops import Act
from oracle import rgb_model as O, train as OT

g = load("train_blocks")
x = torch.from_numpy(filler.normal(74, tuple(g["unet_gx"].shape)))
gy = torch.from_numpy(filler.normal(84, tuple(g["unet_y"].shape)))


def oracle(dtype):
    u = filler.fill_module(EnhancedUNet(256, 64, 3, "batchnorm", 8, "relu")).train()
    sd = {"m." + k: v.detach().to(dtype).requires_grad_(v.requires_grad) for k, v in OT.params_of(u).items()}
    xx = x.to(dtype).requires_grad_(True)
    with OT.train_mode():
        y = O.enhanced_unet(sd, "m", xx, 3, "relu")
    (y * gy.to(dtype)).sum().backward()
    return y.detach(), xx.grad, {k[2:]: v.grad for k, v in sd.items() if v.grad is not None}


y64, gx64, p64 = oracle(torch.float64)
y32, gx32, p32 = oracle(torch.float32)
print("oracle f32 vs f64: y", G.rel(y32, y64), "gx", G.rel(gx32, gx64), G.rel2(gx32, gx64))
for dt in (torch.float32, torch.bfloat16):
    u = filler.fill_module(EnhancedUNet(256, 64, 3, "batchnorm", 8, "relu")).train()
    TE, S, T = G.engine(G._Holder(m=u), dt)
    xa = Act.from_nchw(x.cuda(), dt)
    low, low_t = TE.enhanced_unet(T, u, xa)
    G.inject(T, low, gy.cuda(), torch.float32)
    S.flat.prepare_backward()
    T.run_backward()
    gx = G.grad_nchw(T, xa).cpu()
    print(dt, "y", G.rel(low.to_nchw(), y64), "gx", G.rel(gx, gx64), G.rel2(gx, gx64))
    for n, p in u.named_parameters():
        if n in p64 and p.grad is not None and not n.endswith("bias"):
            print("   %.2e (oracle f32 %.2e) %s" % (G.rel2(p.grad, p64[n]), G.rel2(p32[n], p64[n]), n))
    if dt == torch.bfloat16:
        break

import sys, torch
sys.path[:0] = ['tests', 'tests/golden', '.', 'human-instance-segmentation_amd']
import test_gpu_train as G
import filler
from hiseg.layers import ResidualBlock
from hiseg.ops import Act
from hiseg import train_engine as TE

created = []
orig_fwd = TE.conv_fwd


def spy_fwd(S, p, xa, xb=None, **kw):
    out, d = orig_fwd(S, p, xa, xb, **kw)
    created.append(out)
    return out, d


TE.conv_fwd = spy_fwd
blk = ResidualBlock(64, "batchnorm", 8, "relu", two_acts=False)
mods = G._Holder(blk=blk)
filler.fill_module(mods, seed=3)
_, S, T = G.engine(mods, torch.float32)
x = torch.from_numpy(filler.normal(5, (4, 64, 16, 12))).cuda()
xa = Act.from_nchw(x, torch.float32)
h = TE.conv_bn_act(T, blk.conv1, blk.norm1, TE.ACT_RELU, xa)
y = TE.conv_bn_act(T, blk.conv2, blk.norm2, TE.ACT_RELU, h, residual=xa)
gy = torch.from_numpy(filler.normal(6, (4, 64, 16, 12))).cuda()
G.inject(T, y, gy, torch.float32)
names = {"x": xa, "h": h, "y": y, "z1": created[0], "z2": created[1]}
snap = {k: v.t.clone() for k, v in names.items()}
torch.cuda.synchronize()
S.flat.prepare_backward()
ops = list(T.ops)
T.ops.clear()
for i, fn in enumerate(reversed(ops)):
    fn()
    torch.cuda.synchronize()
    bad = {k: (v.t != snap[k]).sum().item() for k, v in names.items()}
    print("after back op", i, bad)
for k, v in names.items():
    print(k, v.t.data_ptr(), v.t.numel() * 4)

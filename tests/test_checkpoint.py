"""Checkpoint compatibility: hiseg.FusedAdamW state in torch.optim.AdamW's layout,
torch LR schedulers driving it, and save/resume in the reference's checkpoint format
(train_advanced.py:1204-1246, 1592-1599).  CPU: the flat parameter layout is built directly."""
import math
import types

import pytest
import torch
import torch.nn as nn


def _model():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.Conv2d(8, 4, 1), nn.Conv2d(4, 2, 1))
    m[0].weight.requires_grad_(False)   # a frozen parameter keeps its index, gets no state
    m[0].bias.requires_grad_(False)
    return m


def _flat(m):
    from hiseg import train_engine as TE
    m.__dict__["_hiseg_train"] = types.SimpleNamespace(flat=TE.FlatParams(m))
    return m.__dict__["_hiseg_train"].flat


def _torch_step(m, steps=2):
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.01)
    for s in range(steps):
        opt.zero_grad()
        m(torch.randn(2, 3, 8, 8, generator=torch.Generator().manual_seed(s))).square().mean().backward()
        opt.step()
    return opt


def test_fused_adamw_loads_and_writes_torch_adamw_state():
    import hiseg
    ref = _model()
    topt = _torch_step(ref)
    tsd = topt.state_dict()
    m = _model()
    m.load_state_dict(ref.state_dict())
    f = _flat(m)
    opt = hiseg.FusedAdamW(m, lr=5e-4, weight_decay=0.01)
    opt.load_state_dict(tsd)
    assert opt.step_count == 2 and opt.param_groups[0]["lr"] == 1e-3
    for i, p in enumerate(m.parameters()):
        if i in tsd["state"]:
            off, k = f.offsets[id(p)]
            assert torch.equal(opt.exp_avg[off:off + k], tsd["state"][i]["exp_avg"].reshape(-1))
            assert torch.equal(opt.exp_avg_sq[off:off + k], tsd["state"][i]["exp_avg_sq"].reshape(-1))
    sd = opt.state_dict()
    assert sorted(sd["state"]) == sorted(tsd["state"])          # frozen params 0, 1: no state
    assert sd["param_groups"] == tsd["param_groups"]
    for i in tsd["state"]:
        for k in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(sd["state"][i][k], tsd["state"][i][k]), (i, k)
    # and back into torch's optimiser
    back = torch.optim.AdamW(ref.parameters(), lr=1.0)
    back.load_state_dict(sd)
    assert back.state_dict()["param_groups"] == tsd["param_groups"]


def test_torch_cosine_scheduler_drives_fused_adamw():
    import hiseg
    m = _model()
    _flat(m)
    opt = hiseg.FusedAdamW(m, lr=1e-4)
    tm = _model()
    topt = torch.optim.AdamW(tm.parameters(), lr=1e-4)
    s1 = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=7, eta_min=1e-6)
    s2 = torch.optim.lr_scheduler.CosineAnnealingLR(topt, T_max=7, eta_min=1e-6)
    for _ in range(9):
        s1.step()
        s2.step()
        assert opt.param_groups[0]["lr"] == topt.param_groups[0]["lr"]
    assert math.isclose(hiseg.cosine_lr(1e-4, 3, 7, 1e-6),
                        1e-6 + (1e-4 - 1e-6) * 0.5 * (1 + math.cos(math.pi * 3 / 7)))
    sd = s1.state_dict()
    s3 = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=7, eta_min=1e-6)
    s3.load_state_dict(sd)
    assert s3.last_epoch == 9


def test_save_and_resume_in_the_reference_format(tmp_path):
    import hiseg
    ref = _model()
    topt = _torch_step(ref)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(topt, T_max=10, eta_min=1e-6)
    sched.step()
    path = str(tmp_path / "ref.pth")
    # a checkpoint as the reference writes it
    torch.save({"epoch": 4, "model_state_dict": ref.state_dict(), "optimizer_state_dict": topt.state_dict(),
                "scheduler_state_dict": sched.state_dict(), "best_miou": 0.61, "config": {"name": "x"}}, path)
    m = _model()
    _flat(m)
    opt = hiseg.FusedAdamW(m)
    s = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10, eta_min=1e-6)
    start, best = hiseg.resume_from_checkpoint(path, m, opt, s)
    assert (start, best) == (5, 0.61)
    for a, b in zip(m.state_dict().values(), ref.state_dict().values()):
        assert torch.equal(a, b)
    assert s.last_epoch == 1 and opt.step_count == 2
    # hiseg's own checkpoint loads into the reference's objects
    path2 = str(tmp_path / "hiseg.pth")
    hiseg.save_checkpoint(path2, m, opt, epoch=5, best_miou=0.7, scheduler=s, config={"name": "x"})
    ck = torch.load(path2, weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "best_miou",
                       "config"}
    r2 = _model()
    r2.load_state_dict(ck["model_state_dict"])
    o2 = torch.optim.AdamW(r2.parameters(), lr=1.0)
    o2.load_state_dict(ck["optimizer_state_dict"])
    for i, st in topt.state_dict()["state"].items():
        assert torch.equal(o2.state_dict()["state"][i]["exp_avg"], st["exp_avg"])


def test_resume_reseeds_output_conv_and_tolerates_missing_keys(tmp_path):
    import hiseg
    from helpers import b0_kwargs, hiseg_kwargs
    m = hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(b0_kwargs()))
    sd = {k: v for k, v in m.state_dict().items() if "distance_decoder" not in k}
    sd["pretrained_unet.output_conv.weight"] = torch.full_like(sd["pretrained_unet.output_conv.weight"], 3.0)
    path = str(tmp_path / "partial.pth")
    torch.save({"epoch": 0, "model_state_dict": sd, "best_miou": 0.1}, path)
    with pytest.warns(UserWarning, match="strict=False"):
        start, best = hiseg.resume_from_checkpoint(path, m)
    assert start == 1 and best == 0.1
    w = m.pretrained_unet.output_conv.weight.detach().reshape(-1)
    assert w.tolist() == [1.0, -1.0] and not m.pretrained_unet.output_conv.bias.detach().any()

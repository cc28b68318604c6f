"""FusedAdamW on the MI355X: non-finite steps are skipped on the device, the
optimizer follows a re-laid flat parameter layout and carries the moments over, and the reference's optimizer
state transfer at progressive unfreezing (train_distillation_staged.py:1537-1550) works between two FusedAdamW."""
import types

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.Conv2d(8, 4, 1), nn.Conv2d(4, 2, 1)).to(DEV)


def _flat(m):
    from hiseg import train_engine as TE
    m.__dict__["_hiseg_train"] = types.SimpleNamespace(flat=TE.FlatParams(m))
    return m.__dict__["_hiseg_train"].flat


def _grads(m, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return [torch.randn(p.shape, device=DEV, generator=g) for p in m.parameters()]


def test_non_finite_gradient_skips_the_step():
    import hiseg
    m, ref = _model(), _model()
    ref.load_state_dict(m.state_dict())
    _flat(m)
    opt = hiseg.FusedAdamW(m, lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    topt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.01)

    def fused_step(gs):
        opt.zero_grad()
        for p, g in zip(m.parameters(), gs):
            p.grad.copy_(g)
        return opt.step()

    def torch_step(gs):
        topt.zero_grad()
        for p, g in zip(ref.parameters(), gs):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        topt.step()

    g1 = _grads(m, 1)
    fused_step(g1)
    torch_step(g1)
    snap = [t.clone() for t in (opt._flat.data, opt.exp_avg, opt.exp_avg_sq)]
    for bad in (float("nan"), float("inf")):
        gb = _grads(m, 2)
        gb[2].view(-1)[5] = bad
        norm = fused_step(gb)
        torch.cuda.synchronize()
        assert not torch.isfinite(norm).all()
        for a, b in zip(snap, (opt._flat.data, opt.exp_avg, opt.exp_avg_sq)):
            assert torch.equal(a, b), "a non-finite step changed the parameters or the moments"
        assert opt.step_count == 1
    assert opt.skipped_steps == 2
    # the next finite step is the reference's second step (bias corrections of t = 2)
    g3 = _grads(m, 3)
    fused_step(g3)
    torch_step(g3)
    assert opt.step_count == 2
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-6, atol=2e-7)
    sd = opt.state_dict()
    tsd = topt.state_dict()
    for i, st in tsd["state"].items():
        assert float(sd["state"][i]["step"]) == float(st["step"]) == 2.0
        torch.testing.assert_close(sd["state"][i]["exp_avg"], st["exp_avg"], rtol=1e-6, atol=1e-9)


def test_rebind_after_the_flat_layout_changes_keeps_the_moments():
    """unfreeze_encoder_blocks / a dtype change build a new FlatParams: the optimizer re-binds on its next
    zero_grad and every kept parameter's moments and step count carry over; new parameters start at step 0."""
    import hiseg
    m = _model()
    m[0].weight.requires_grad_(False)
    m[0].bias.requires_grad_(False)
    _flat(m)
    opt = hiseg.FusedAdamW(m, lr=1e-3)
    for s in range(2):
        opt.zero_grad()
        torch.manual_seed(10 + s)
        for p in m.parameters():
            if p.requires_grad:
                p.grad.normal_()
        opt.step()
    before = {id(p): (opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone())
              for p in m.parameters() if p.requires_grad}
    old_flat = opt._flat
    m[0].weight.requires_grad_(True)        # a larger trainable set: a new layout
    m[0].bias.requires_grad_(True)
    f2 = _flat(m)
    opt.zero_grad()
    assert opt._flat is f2 and opt._flat is not old_flat
    assert opt.step_count == 2
    steps = opt.param_steps()
    for p in m.parameters():
        if id(p) in before:
            assert steps[p] == 2 and float(opt.state[p]["step"]) == 2.0
            assert torch.equal(opt.state[p]["exp_avg"], before[id(p)][0])
            assert torch.equal(opt.state[p]["exp_avg_sq"], before[id(p)][1])
        else:   # torch.optim.AdamW: no state (step 0) before a new parameter's first step
            assert steps[p] == 0 and p not in opt.state
            off = opt._flat.offsets[id(p)][0]
            assert not opt.exp_avg[off:off + p.numel()].any()


def test_unfreeze_midway_matches_torch_adamw():
    """a parameter that joins the optimizer partway through training gets its own step count, as in
    torch.optim.AdamW (the reference's progressive unfreezing builds a new optimizer and transfers the kept
    parameters' state, train_distillation_staged.py:1531-1552): its first update is lr * g / |g|-like, not the
    bias-corrected update of the global step.  3 steps with m[0] frozen, then 3 with everything trainable."""
    import hiseg
    m, ref = _model(), _model()
    ref.load_state_dict(m.state_dict())
    for mm in (m, ref):
        mm[0].weight.requires_grad_(False)
        mm[0].bias.requires_grad_(False)
    _flat(m)
    opt = hiseg.FusedAdamW(m, lr=1e-2, weight_decay=0.01, max_grad_norm=None)
    topt = torch.optim.AdamW([p for p in ref.parameters() if p.requires_grad], lr=1e-2, weight_decay=0.01)

    def both(seed):
        gs = _grads(m, seed)
        opt.zero_grad()
        for p, g in zip(m.parameters(), gs):
            if p.requires_grad:
                p.grad.copy_(g)
        opt.step()
        topt.zero_grad()
        for p, g in zip(ref.parameters(), gs):
            if p.requires_grad:
                p.grad = g.clone()
        topt.step()

    for s in range(3):
        both(20 + s)
    for mm in (m, ref):
        mm[0].weight.requires_grad_(True)
        mm[0].bias.requires_grad_(True)
    _flat(m)
    old = topt   # the reference pattern: a new optimizer over all trainable params, old state transferred
    topt = torch.optim.AdamW([p for p in ref.parameters() if p.requires_grad], lr=1e-2, weight_decay=0.01)
    for p in topt.param_groups[0]["params"]:
        if p in old.state:
            topt.state[p] = old.state[p]
    for s in range(3):
        both(30 + s)
    torch.cuda.synchronize()
    # same arithmetic op for op; contraction / rounding differences stay ~1e-6 over 6 steps, whereas a global
    # step count would move the new parameters' first updates by a factor 2.5-3 (~lr = 1e-2)
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)
    steps = opt.param_steps()
    assert [steps[p] for p in m.parameters()] == [int(topt.state[q]["step"]) for q in ref.parameters()] \
        == [3, 3, 6, 6, 6, 6, 6, 6]
    sd = opt.state_dict()
    tsd = topt.state_dict()
    for i, st in tsd["state"].items():
        assert float(sd["state"][i]["step"]) == float(st["step"])
        torch.testing.assert_close(sd["state"][i]["exp_avg_sq"], st["exp_avg_sq"], rtol=1e-5, atol=1e-12)


def test_reference_state_transfer_between_fused_optimizers():
    """The reference's unfreeze code copies optimizer.state[p] for the decoder params into the new optimizer."""
    import hiseg
    m = _model()
    _flat(m)
    dec = list(m[2].parameters()) + list(m[3].parameters())
    old = hiseg.FusedAdamW(m, lr=1e-3, params=dec)
    for s in range(3):
        old.zero_grad()
        for p in dec:
            p.grad.normal_()
        old.step()
    new = hiseg.FusedAdamW(m, lr=1e-3, params=dec)
    assert not new.state
    n = 0
    if hasattr(old, "state") and old.state:
        for new_p in new.param_groups[0]["params"]:
            for old_p in old.param_groups[0]["params"]:
                if new_p is old_p and old_p in old.state:
                    new.state[new_p] = old.state[old_p]
                    n += 1
                    break
    assert n == len(dec)
    assert new.step_count == 3
    assert torch.equal(new.exp_avg, old.exp_avg) and torch.equal(new.exp_avg_sq, old.exp_avg_sq)

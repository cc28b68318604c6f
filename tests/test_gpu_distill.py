"""Distillation path on the GPU: the UNetDistillationLoss kernels (include/hiseg_distill.h) against the
reference's golden vectors, and the student training step against the CPU oracle."""
import numpy as np
import pytest
import torch

from helpers import load
from test_oracle_distill import G, KEYS, NAMES, assert_grad_close, case_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _loss_fn(name):
    import hiseg
    ct = G[f"{name}_ctor"]
    fn = hiseg.UNetDistillationLoss(temperature=float(ct[0]), alpha=float(ct[1]), task_weight=float(ct[2]),
                                    use_dice_loss=bool(ct[3]), adaptive_distillation=bool(ct[4]))
    st = G[f"{name}_state"]
    fn.temperature, fn.alpha, fn.task_weight = float(st[0]), float(st[1]), float(st[2])
    fn.distillation_eliminated, fn.performance_ratio = bool(st[4]), float(st[5])
    return fn


@pytest.mark.parametrize("name", NAMES)
def test_distill_loss_kernel_matches_reference_golden(name):
    s, t, m, _ = case_inputs(name)
    fn = _loss_fn(name)
    sd = s.to(DEV).requires_grad_(True)
    total, d = fn(sd, t.to(DEV), m.to(DEV) if m is not None else None)
    total.backward()
    assert total.item() == pytest.approx(float(G[f"{name}_loss"]), rel=1e-5, abs=1e-6)
    for k, v in zip(KEYS, G[f"{name}_dict"]):
        assert d[k] == pytest.approx(float(v), rel=1e-4, abs=1e-6), k
    assert_grad_close(sd.grad.cpu(), torch.from_numpy(G[f"{name}_grad"]), 1e-5)


def test_distill_schedule_methods_match_reference_state():
    import hiseg
    fn = hiseg.UNetDistillationLoss(temperature=4.0, alpha=0.3, task_weight=0.7)
    fn.update_temperature(12, 50, final_temperature=1.0, schedule_type="cosine")
    assert fn.temperature == pytest.approx(float(G["dist_cos_sched_state"][0]))
    fn = hiseg.UNetDistillationLoss(temperature=2.0, alpha=0.3, task_weight=0.7)
    fn.update_distillation_weight(0.81, 0.80, min_alpha=0.0, amplification_factor=30.0,
                                  zero_distillation_threshold=0.03)
    st = G["dist_student_better_state"]
    assert (fn.alpha, fn.task_weight, fn.performance_ratio) == pytest.approx((st[1], st[2], st[5]))
    fn.update_distillation_weight(0.90, 0.80, amplification_factor=30.0)
    assert fn.distillation_eliminated and fn.alpha == 0.0 and fn.task_weight == 1.0


# ------------------------------------------------------------------------------------------ student training step
def _distill_model(dt):
    import filler
    import hiseg
    model, loss_fn = hiseg.create_unet_distillation_model("timm-efficientnet-b0", "timm-efficientnet-b7",
                                                          teacher_checkpoint="absent.pth", device="cpu",
                                                          progressive_unfreeze=True)
    filler.fill_module(model.student, seed=11)
    filler.fill_module(model.teacher, seed=12)
    hiseg.set_compute_dtype(model, dt)
    return model, loss_fn


def test_distill_student_step_f32_matches_oracle():
    """Decoder-only phase of train_distillation_staged.py (progressive unfreezing, epochs < start): student
    B0 smp-UNet in train mode (batch-statistics BN everywhere, frozen encoder), teacher B7 in eval, the
    distillation loss with targets, backward into the decoder + head.  Against oracle/ (torch autograd on
    the CPU, f32): teacher logits 1e-4; student logits, loss 1e-3 (train-mode BN over a 2-image batch with
    2x3-pixel deepest maps amplifies rounding, as in test_gpu_train); parameter gradients by cosine > 0.99
    per tensor and total norm within 3 %."""
    import filler
    from oracle import distill as OD
    from oracle import rgb_model as O
    from oracle import train as OT
    model, loss_fn = _distill_model(torch.float32)
    sd_s, sd_t = OT.params_of(model.student), OT.params_of(model.teacher)
    x = torch.from_numpy(filler.normal(21, (2, 3, 64, 96)))
    _, _, m = OD.np_inputs(22, 2, 64, 96)
    model = model.to(DEV).train()
    loss_fn.temperature = 4.0
    s, t = model(x.to(DEV))
    loss, d = loss_fn(s, t, m.to(DEV))
    loss.backward()
    with OT.train_mode():
        rs = O.effunet_logits(sd_s, "unet", x, "b0")
    with torch.no_grad():
        rt = O.effunet_logits(sd_t, "unet", x, "b7")
    rl, rd = OD.distill_loss(rs, rt, m, temperature=4.0, alpha=0.05, task_weight=0.7)
    rl.backward()

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return ((a - b).abs().max() / b.abs().max()).item()
    assert rel(t, rt) < 1e-4
    assert rel(s, rs) < 1e-3
    assert loss.item() == pytest.approx(rl.item(), rel=1e-3)
    for k in ("kl_loss", "mse_loss", "bce_loss", "dice_loss"):
        assert d[k] == pytest.approx(rd[k], rel=2e-3, abs=1e-6), k
    tot_m = tot_r = 0.0
    bad = []
    for n, p in model.student.named_parameters():
        if not p.requires_grad:
            assert n.startswith("unet.encoder."), n
            continue
        mg, rg = p.grad.detach().double().cpu().reshape(-1), sd_s[n].grad.double().reshape(-1)
        tot_m += float((mg ** 2).sum())
        tot_r += float((rg ** 2).sum())
        if rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5:
            continue
        cos = float((mg * rg).sum() / (mg.norm() * rg.norm()))
        if cos <= 0.99:
            bad.append((n, round(cos, 4), float(mg.norm()), float(rg.norm())))
    assert not bad, bad
    assert abs(tot_m / tot_r - 1) < 3e-2


def test_distill_bf16_training_lowers_loss():
    """bf16 decoder-only distillation: decoder AdamW (clip 1.0 on the decoder, train_distillation_staged.py
    :298-314) over a fixed batch lowers the loss; the segmentation head is not in the optimiser (the
    reference optimises unet.decoder.parameters() only) and keeps its weights."""
    import filler
    import hiseg
    model, loss_fn = _distill_model(torch.bfloat16)
    model = model.to(DEV).train()
    x = torch.from_numpy(filler.normal(31, (2, 3, 128, 128))).to(DEV)
    _, _, m = __import__("oracle.distill", fromlist=["np_inputs"]).np_inputs(32, 2, 128, 128)
    m = m.to(DEV)
    head_w = model.student.unet.segmentation_head[0].weight.detach().clone()
    opt, losses = None, []
    for step in range(6):
        s, t = model(x)
        loss, d = loss_fn(s, t, m)
        if opt is None:
            opt = hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                   params=model.student.get_decoder_parameters())
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
    assert torch.equal(model.student.unet.segmentation_head[0].weight.detach(), head_w)


@pytest.mark.parametrize("blocks", [1, 3, 7])
def test_distill_progressive_unfreeze_f32_matches_oracle(blocks):
    """After unfreeze_encoder_blocks(k) (unet_decoder_distillation.py:233-274): the deepest k encoder stages
    train too -- MBConv backward (1x1 convs, depthwise k3/k5 stride 1/2, SqueezeExcite, BN-SiLU) and the
    decoder's gradients into their skip features.  Against the oracle as the decoder-only test."""
    import filler
    from oracle import distill as OD
    from oracle import rgb_model as O
    from oracle import train as OT
    model, loss_fn = _distill_model(torch.float32)
    unfrozen = model.unfreeze_encoder_blocks(blocks)
    assert len(unfrozen) > 0
    sd_s, sd_t = OT.params_of(model.student), OT.params_of(model.teacher)
    x = torch.from_numpy(filler.normal(23, (2, 3, 64, 96)))
    _, _, m = OD.np_inputs(24, 2, 64, 96)
    model = model.to(DEV).train()
    s, t = model(x.to(DEV))
    loss, d = loss_fn(s, t, m.to(DEV))
    loss.backward()
    with OT.train_mode():
        rs = O.effunet_logits(sd_s, "unet", x, "b0")
    with torch.no_grad():
        rt = O.effunet_logits(sd_t, "unet", x, "b7")
    rl, rd = OD.distill_loss(rs, rt, m, temperature=1.0, alpha=0.05, task_weight=0.7)
    rl.backward()
    assert loss.item() == pytest.approx(rl.item(), rel=1e-3)
    bad, tot_m, tot_r, n_enc = [], 0.0, 0.0, 0
    for n, p in model.student.named_parameters():
        if not p.requires_grad:
            continue
        n_enc += n.startswith("unet.encoder.")
        mg, rg = p.grad.detach().double().cpu().reshape(-1), sd_s[n].grad.double().reshape(-1)
        tot_m += float((mg ** 2).sum())
        tot_r += float((rg ** 2).sum())
        if rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5:
            continue
        cos = float((mg * rg).sum() / (mg.norm() * rg.norm()))
        if cos <= 0.99:
            bad.append((n, round(cos, 4)))
    assert n_enc == len(unfrozen)
    assert not bad, bad
    assert abs(tot_m / tot_r - 1) < 3e-2


def test_distill_bf16_progressive_schedule_runs():
    """bf16, the reference's schedule in miniature: decoder-only steps, then unfreeze_encoder_blocks(2) with
    the reference's two parameter groups (decoder: lr, clip 1.0; encoder: lr * encoder_lr_scale, unclipped,
    train_distillation_staged.py:1516-1545) and its optimizer-state transfer for the decoder parameters
    (:1537-1550, new_optimizer.state[p] = optimizer.state[p]) -- the new trainable set re-lays the flat
    parameters, the decoder keeps its AdamW moments, the loss keeps decreasing and stays finite."""
    import filler
    import hiseg
    from oracle import distill as OD
    model, loss_fn = _distill_model(torch.bfloat16)
    model = model.to(DEV).train()
    x = torch.from_numpy(filler.normal(33, (2, 3, 96, 128))).to(DEV)
    _, _, m = OD.np_inputs(34, 2, 96, 128)
    m = m.to(DEV)
    losses = []
    opts, enc = None, None
    for step in range(8):
        if step == 4:
            enc = model.unfreeze_encoder_blocks(2, learning_rate_scale=0.3)
            assert enc
        s, t = model(x)
        loss, _ = loss_fn(s, t, m)
        if opts is None:
            opts = [hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                     params=model.student.get_decoder_parameters())]
        elif step == 4:
            old = opts[0]
            new = hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                   params=model.student.get_decoder_parameters())
            moved = 0
            if hasattr(old, "state") and old.state:
                for new_p in new.param_groups[0]["params"]:
                    for old_p in old.param_groups[0]["params"]:
                        if new_p is old_p and old_p in old.state:
                            new.state[new_p] = old.state[old_p]
                            moved += 1
                            break
            assert moved == len(new.param_groups[0]["params"]) and new.step_count == 4
            opts = [new, hiseg.FusedAdamW(model.student, lr=3e-4, weight_decay=1e-4, max_grad_norm=None,
                                          params=enc)]
        for o in opts:
            o.zero_grad()
        loss.backward()
        for o in opts:
            o.step()
        losses.append(loss.item())
    assert all(np.isfinite(losses)), losses
    assert losses[3] < losses[0] and losses[-1] < losses[4], losses


@pytest.mark.parametrize("graphed", [False, True])
def test_concurrent_teacher_stream_equals_serial(graphed, monkeypatch):
    """The frozen teacher's forward on a side stream beside the student's (DistillationUNetWrapper, forked from and
    joined into the caller's stream; a captured graph holds both branches) gives the serial order's loss, student
    gradients and updated parameters bit for bit over three bf16 decoder-only steps, eager and graphed."""
    import filler
    import hiseg
    from hiseg.distill import DistillationUNetWrapper
    x = torch.from_numpy(filler.normal(41, (2, 3, 128, 128))).to(DEV)
    _, _, m = __import__("oracle.distill", fromlist=["np_inputs"]).np_inputs(42, 2, 128, 128)
    m = m.to(DEV)
    res = {}
    for conc in (False, True):
        monkeypatch.setattr(DistillationUNetWrapper, "concurrent_teacher", conc)
        model, loss_fn = _distill_model(torch.bfloat16)
        model = model.to(DEV).train()
        state = {"opt": None}

        def step():
            s, t = model(x)
            loss, _ = loss_fn(s, t, m)
            if state["opt"] is None:
                state["opt"] = hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                                params=model.student.get_decoder_parameters())
            state["opt"].zero_grad()
            loss.backward()
            state["opt"].step()
            return loss

        run = hiseg.GraphedStep(step, lambda: state["opt"]) if graphed else step
        losses = [run().detach().clone() for _ in range(5 if graphed else 3)]
        torch.cuda.synchronize()
        res[conc] = (torch.stack(losses), [p.detach().clone() for p in model.student.parameters()])
    (l0, p0), (l1, p1) = res[False], res[True]
    assert torch.isfinite(l0).all()
    assert torch.equal(l0, l1), (l0, l1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))


@pytest.mark.parametrize("unfrozen", [0, 2])
def test_branch_graphs_equal_single_graph(unfrozen, monkeypatch):
    """hiseg.GraphedBranchStep (teacher forward, student forward and loss/backward/optimizer as three graphs, the two
    forwards launched side by side) against the serial step in one GraphedStep graph: loss, student parameters bit
    for bit over six steps (two eager, capture, three replays), decoder-only and with the encoder's last two stages
    unfrozen (second FusedAdamW group, backward through the MBConv stack)."""
    import filler
    import hiseg
    from hiseg.distill import DistillationUNetWrapper
    x = torch.from_numpy(filler.normal(43, (2, 3, 128, 128))).to(DEV)
    _, _, m = __import__("oracle.distill", fromlist=["np_inputs"]).np_inputs(44, 2, 128, 128)
    m = m.to(DEV)
    res = {}
    for split in (False, True):
        monkeypatch.setattr(DistillationUNetWrapper, "concurrent_teacher", False)
        model, loss_fn = _distill_model(torch.bfloat16)
        model = model.to(DEV).train()
        enc = model.unfreeze_encoder_blocks(unfrozen, learning_rate_scale=0.1) if unfrozen else None
        state = {"opt": None, "enc": None}
        fwd = {}

        def step(s=None, t=None):
            if s is None:
                s, t = model(x)
            loss, _ = loss_fn(s, t, m)
            if state["opt"] is None:
                state["opt"] = hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                                params=model.student.get_decoder_parameters())
                if enc:
                    state["enc"] = hiseg.FusedAdamW(model.student, lr=1e-4, weight_decay=1e-4, max_grad_norm=None,
                                                    params=enc)
            opts = [o for o in (state["opt"], state["enc"]) if o is not None]
            for o in opts:
                o.zero_grad()
            loss.backward()
            for o in opts:
                o.step()
            return loss

        def teacher():
            fwd["t"] = model.teacher(x)

        def student():
            fwd["s"] = model.student(x)

        if split:
            run = hiseg.GraphedBranchStep(teacher, student, lambda: step(fwd["s"], fwd["t"]), lambda: state["opt"])
        else:
            run = hiseg.GraphedStep(step, lambda: state["opt"])
        losses = [run().detach().clone() for _ in range(6)]
        torch.cuda.synchronize()
        if split:
            assert run.captures == 1
        res[split] = (torch.stack(losses), [p.detach().clone() for p in model.student.parameters()])
    (l0, p0), (l1, p1) = res[False], res[True]
    assert torch.isfinite(l0).all()
    assert torch.equal(l0, l1), (l0, l1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))


def test_pipelined_teacher_equals_serial_step():
    """GraphedBranchStep with handoff_fn (the frozen teacher's forward for batch k+1 launched during step k, beside
    step k's student forward and backward) against the serial step, over six steps on six DIFFERENT batches: same
    losses and student parameters bit for bit -- the handoff stages each batch and its teacher output in order."""
    import filler
    import hiseg
    from hiseg.distill import DistillationUNetWrapper
    nstep = 6
    xs = [torch.from_numpy(filler.normal(60 + k, (2, 3, 128, 128))).to(DEV) for k in range(nstep + 1)]
    _, _, m = __import__("oracle.distill", fromlist=["np_inputs"]).np_inputs(45, 2, 128, 128)
    m = m.to(DEV)
    res = {}
    for piped in (False, True):
        model, loss_fn = _distill_model(torch.bfloat16)
        model = model.to(DEV).train()
        model.concurrent_teacher = False
        state = {"opt": None}
        x_cur, x_next = xs[0].clone(), xs[0].clone()
        fwd, k = {}, [0]

        def step(s=None, t=None):
            if s is None:
                s, t = model(x_cur)
            loss, _ = loss_fn(s, t, m)
            if state["opt"] is None:
                state["opt"] = hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                                params=model.student.get_decoder_parameters())
            state["opt"].zero_grad()
            loss.backward()
            state["opt"].step()
            return loss

        def teacher():
            fwd["t_next"] = model.teacher(x_next)

        def student():
            fwd["s"] = model.student(x_cur)

        def handoff():   # step k: its teacher output and batch in place, batch k+1 staged for the next branch
            if "t" not in fwd:
                fwd["t"] = torch.empty_like(fwd["t_next"])
            fwd["t"].copy_(fwd["t_next"])
            x_cur.copy_(xs[k[0]])
            x_next.copy_(xs[k[0] + 1])

        losses = []
        for i in range(nstep):
            k[0] = i
            if piped:
                if i == 0:
                    run = hiseg.GraphedBranchStep(teacher, student, lambda: step(fwd["s"], fwd["t"]),
                                                  lambda: state["opt"], handoff_fn=handoff)
                losses.append(run().detach().clone())
            else:
                x_cur.copy_(xs[i])
                losses.append(step().detach().clone())
        if piped:
            run.drain()
            assert run.captures == 1
        torch.cuda.synchronize()
        res[piped] = (torch.stack(losses), [p.detach().clone() for p in model.student.parameters()])
    (l0, p0), (l1, p1) = res[False], res[True]
    assert torch.isfinite(l0).all()
    assert len(set(l0.tolist())) == nstep   # different batches, different losses
    assert torch.equal(l0, l1), (l0, l1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))


@pytest.mark.parametrize("branch", [False, True])
def test_temperature_and_lr_schedule_replay_one_graph(branch, monkeypatch):
    """the staged distillation's per-epoch schedules -- temperature 4 -> 1
    (UNetDistillationLoss.update_temperature, train_distillation_staged.py:1597-1610) and a cosine learning rate
    (:1126-1131 style) -- are device scalars a captured step reads, so 4 epochs x 2 steps replay ONE graph
    (GraphedStep and GraphedBranchStep), with losses and student parameters bit-identical to eager steps."""
    import math
    import filler
    import hiseg
    from hiseg.distill import DistillationUNetWrapper
    x = torch.from_numpy(filler.normal(45, (2, 3, 128, 128))).to(DEV)
    _, _, m = __import__("oracle.distill", fromlist=["np_inputs"]).np_inputs(46, 2, 128, 128)
    m = m.to(DEV)
    epochs, per_epoch = 4, 2
    res = {}
    for graphed in (False, True):
        monkeypatch.setattr(DistillationUNetWrapper, "concurrent_teacher", False)
        model, loss_fn = _distill_model(torch.bfloat16)
        loss_fn.initial_temperature = loss_fn.temperature = 4.0
        loss_fn.alpha = loss_fn.initial_alpha = 0.5
        loss_fn.task_weight = loss_fn.initial_task_weight = 0.5
        model = model.to(DEV).train()
        state = {"opt": None}
        fwd = {}

        def opt():
            if state["opt"] is None:
                state["opt"] = hiseg.FusedAdamW(model.student, lr=1e-3, weight_decay=1e-4, max_grad_norm=1.0,
                                                params=model.student.get_decoder_parameters())
            return state["opt"]

        def tail():
            loss, _ = loss_fn(fwd["s"], fwd["t"], m)
            o = opt()
            o.zero_grad()
            loss.backward()
            o.step()
            return loss

        def teacher():
            fwd["t"] = model.teacher(x)

        def student():
            fwd["s"] = model.student(x)

        def serial():
            fwd["s"], fwd["t"] = model(x)
            return tail()

        if not graphed:
            run = serial
        elif branch:
            run = hiseg.GraphedBranchStep(teacher, student, tail, lambda: state["opt"])
        else:
            run = hiseg.GraphedStep(serial, lambda: state["opt"])
        losses, temps = [], []
        for e in range(epochs):
            temps.append(loss_fn.update_temperature(e, epochs, final_temperature=1.0))
            if state["opt"] is not None:
                for g in state["opt"].param_groups:
                    g["lr"] = 1e-3 * 0.5 * (1 + math.cos(math.pi * e / epochs))
            for _ in range(per_epoch):
                losses.append(run().detach().clone())
        torch.cuda.synchronize()
        if graphed:
            assert run.captures == 1, run.captures
        res[graphed] = (torch.stack(losses), [p.detach().clone() for p in model.student.parameters()])
    assert temps == [4.0, 3.0, 2.0, 1.0]
    (l0, p0), (l1, p1) = res[False], res[True]
    assert torch.isfinite(l0).all()
    assert torch.equal(l0, l1), (l0, l1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))

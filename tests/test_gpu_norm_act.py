"""N2 LayerNorm2d and N3 GELU / Swish(beta) on the HIP path.

The presets all run batchnorm + ReLU; the reference's factories also offer normalization_type
'layernorm2d' (model.py:18-38 via normalization_comparison.py:159-206) and the activations of
activation_utils.py:71-101 (GELU, Swish(beta)) -- with unet.py's / rgb.py's own factory mapping
'swish' to nn.SiLU.  Inference is checked against the reference's outputs (tests/golden/variants.npz,
gen_golden.py variants) at the f32 bar of 1e-4; training against float64 autograd of the oracle's
functional forms (which variants.npz pins), also at 1e-4 -- these activations are smooth, so no
activation-pattern replay is needed.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

import filler
from helpers import VARIANTS, act_tag, b0_kwargs, hiseg_kwargs, load, variant_modules

pytestmark = pytest.mark.gpu
DEV = "cuda"
F32_TOL = 1e-4
KEYS = list(VARIANTS)


def _rel(a, b):
    a, b = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a).double().cpu(), \
        torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1.0)).item()


def _relm(a, b):
    """max-abs error relative to the reference tensor's own max (gradients of any scale)."""
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _inputs():
    return (torch.from_numpy(filler.normal(61, (2, 64, 12, 10))), torch.from_numpy(filler.normal(62, (2, 64, 16, 12))),
            torch.from_numpy(filler.normal(63, (2, 64, 16, 12))))


# ------------------------------------------------------------------------------------------ inference
@pytest.mark.parametrize("key", KEYS)
def test_variant_inference_matches_reference_golden(key):
    import hiseg
    norm, act, beta = VARIANTS[key]
    g = load("variants")
    x, xu, xh = _inputs()
    blk, unet, head = (hiseg.set_compute_dtype(m.to(DEV), torch.float32) for m in variant_modules(norm, act, beta))
    with torch.no_grad():
        assert _rel(blk(x.to(DEV)), g[f"{key}_res_y"]) < F32_TOL
        assert _rel(unet(xu.to(DEV)), g[f"{key}_unet_y"]) < F32_TOL
        logits, aux = head(xh.to(DEV))
    assert _rel(logits, g[f"{key}_head_logits"]) < F32_TOL
    n = 0
    for k, v in aux.items():
        if f"{key}_head_aux_{k}" in g.files:
            assert _rel(v, g[f"{key}_head_aux_{k}"]) < F32_TOL, k
            n += 1
    assert n >= 8, sorted(aux)


def test_variant_inference_bf16_agrees():
    """bf16 compute with LayerNorm2d + GELU: relative bound and argmax agreement of the head logits."""
    import hiseg
    norm, act, beta = VARIANTS["ln_gelu"]
    g = load("variants")
    _, _, xh = _inputs()
    head = hiseg.set_compute_dtype(variant_modules(norm, act, beta)[2].to(DEV), torch.bfloat16)
    with torch.no_grad():
        logits, _ = head(xh.to(DEV))
    ref = torch.from_numpy(g["ln_gelu_head_logits"])
    assert _rel(logits, ref) < 0.1
    agree = (logits.argmax(1).cpu() == ref.argmax(1)).float().mean().item()
    assert agree > 0.95, agree


def _model(kw, dt):
    import hiseg
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(kw))).eval().to(DEV)
    return hiseg.set_compute_dtype(m, dt)


def test_layernorm_gelu_model_matches_reference_golden():
    """The whole ROI path (rgb_feature_extractor, feature_combiner, 256-channel head) with layernorm2d + GELU."""
    from hiseg import engine
    g = load("variants")
    m = _model(dict(b0_kwargs(), normalization_type="layernorm2d", activation_function="gelu"), torch.float32)
    for r in (m.roi_align_mask, m.roi_align_rgb):
        r.spatial_scale_h, r.spatial_scale_w = 96, 128
    images, rois, u = (torch.from_numpy(g[k]).to(DEV) for k in ("model_images", "model_rois", "model_u"))
    logits, _ = engine.rgb_model_forward(m, images, rois, "none", unet_logit_override=u)
    assert _rel(logits, g["model_logits"]) < F32_TOL


# ------------------------------------------------------------------------------------------ training
class _Holder(nn.Module):
    def __init__(self, **mods):
        super().__init__()
        for k, v in mods.items():
            setattr(self, k, v)


def _engine(module, dt=torch.float32):
    from hiseg import train_engine as TE
    module = module.to(DEV)
    S = TE.TrainState(module, dt, torch.device(DEV))
    return TE, S, TE.Tape(S)


def _inject(T, y, g_nchw, dt):
    from hiseg.ops import Act
    ga = Act.from_nchw(g_nchw.to(DEV), dt)
    if ga.cstride != y.cstride:
        full = Act.new(y.N, y.H, y.W, y.C, dt, DEV, cpad=y.cstride, zero=True)
        full.t.view(-1, y.cstride)[:, :y.C].copy_(ga.t.view(-1, ga.cstride)[:, :y.C])
        ga = full
    T.grads[id(y)] = ga
    T.mark(y)


def _oracle_grads(module, fn, x, gy):
    """float64 autograd of an oracle functional form on the GPU: (y, dx, {param: grad})."""
    from oracle import train as OT
    sd = {"m." + k: v.detach().to(DEV, torch.float64).requires_grad_(v.requires_grad)
          for k, v in OT.params_of(module).items()}
    xx = x.to(DEV, torch.float64).requires_grad_(True)
    with OT.train_mode():
        y = fn(sd, xx)
    (y * gy.to(DEV, torch.float64)).sum().backward()
    return y.detach(), xx.grad, {k[2:]: v.grad for k, v in sd.items() if v.grad is not None}


def _check_params(module, ref, tol):
    for n, p in module.named_parameters():
        if n not in ref:
            continue
        rg = ref[n]
        if n.endswith(".bias") and isinstance(getattr(module, "norm1", None), nn.BatchNorm2d) \
                and rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5:
            continue   # conv bias before train-mode BatchNorm: zero gradient in exact arithmetic
        assert p.grad is not None, n
        assert _relm(p.grad, rg) < tol, (n, _relm(p.grad, rg))


@pytest.mark.parametrize("key", KEYS)
def test_variant_residual_block_train_vs_autograd(key):
    """ResidualBlock (refinement.py:31-55) in train mode: LayerNorm2d / BatchNorm(train) with GELU / Swish(beta),
    incl. the activation after the residual add (derivative at the forward's own pre-activation)."""
    from oracle import rgb_model as O
    from hiseg.ops import Act
    norm, act, beta = VARIANTS[key]
    blk = variant_modules(norm, act, beta)[0].train()
    x, _, _ = _inputs()
    gy = torch.from_numpy(filler.normal(64, tuple(x.shape)))
    TE, S, T = _engine(_Holder(b=blk))
    xa = Act.from_nchw(x.to(DEV), torch.float32)
    y = TE.residual_block(T, blk, xa)
    _inject(T, y, gy, torch.float32)
    S.flat.prepare_backward()
    T.run_backward()
    a = act_tag(act, beta)
    ry, rgx, rp = _oracle_grads(blk, lambda sd, xx: O.residual(sd, "m", xx, a), x, gy)
    assert _relm(y.to_nchw(), ry) < F32_TOL
    gx, _ = T.grad(xa)
    assert _relm(gx.to_nchw(), rgx) < F32_TOL
    _check_params(blk, rp, 2 * F32_TOL)


@pytest.mark.parametrize("key", KEYS)
def test_variant_enhanced_unet_train_vs_autograd(key):
    """EnhancedUNet(64, 32, depth 3) train forward/backward with the variant norm / activation."""
    from oracle import rgb_model as O
    from hiseg.ops import Act
    norm, act, beta = VARIANTS[key]
    u = variant_modules(norm, act, beta)[1].train()
    _, xu, _ = _inputs()
    gy = torch.from_numpy(filler.normal(65, (2, 2, 16, 12)))
    TE, S, T = _engine(_Holder(m=u))
    xa = Act.from_nchw(xu.to(DEV), torch.float32)
    low, _ = TE.enhanced_unet(T, u, xa)
    _inject(T, low, gy, torch.float32)
    S.flat.prepare_backward()
    T.run_backward()
    a = act_tag(act, beta)
    ry, rgx, rp = _oracle_grads(u, lambda sd, xx: O.enhanced_unet(sd, "m", xx, 3, a), xu, gy)
    assert _relm(low.to_nchw(), ry) < F32_TOL
    gx, _ = T.grad(xa)
    assert _relm(gx.to_nchw(), rgx) < 2 * F32_TOL
    for n, p in u.named_parameters():
        rg = rp.get(n)
        if rg is None or (norm == "batchnorm" and n.endswith(".bias") and rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5):
            continue
        assert p.grad is not None, n
        assert _relm(p.grad, rg) < 4 * F32_TOL, (n, _relm(p.grad, rg))


@pytest.mark.parametrize("key", ["ln_gelu", "bn_swish"])
def test_variant_train_step_f32_matches_oracle(key):
    """The whole train step (B0 ROI path + RefinedHierarchicalLoss) with the variant norm / activation against
    the CPU oracle: channel attention with Swish(beta), the fused upsample_bg_fg with LayerNorm2d and GELU,
    GELU fg_gate convs, LayerNorm2d in every block.  Bars as test_gpu_train.test_train_step_f32_matches_oracle."""
    import hiseg
    from hiseg import train_engine as TE
    from oracle import rgb_model as O
    from oracle import train as OT
    norm, act, beta = VARIANTS[key]
    kw = hiseg_kwargs(dict(b0_kwargs(), normalization_type=norm, activation_function=act, activation_beta=beta))
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**kw))
    for mod in m.modules():
        if isinstance(mod, (nn.Dropout, nn.Dropout2d)):
            mod.p = 0.0
    hiseg.set_compute_dtype(m, torch.float32)
    sd = OT.params_of(m)
    m = m.to(DEV).train()
    cfg = O.cfg_from_kwargs(kw)
    images = torch.from_numpy(filler.uniform(61, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(62, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]])
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    tgt = torch.from_numpy(filler.ellipse_targets(63, 3, *cfg["mask_hw"]))
    logits, aux = TE.train_forward(m, images.to(DEV), rois.to(DEV), u_override=u.to(DEV))
    loss_fn = hiseg.RefinedHierarchicalLoss(use_boundary_aware_loss=True, use_contour_detection=True,
                                            use_distance_transform=True, boundary_aware_weight=0.1,
                                            contour_loss_weight=0.1, distance_loss_weight=0.1)
    loss, d = loss_fn(logits, tgt.to(DEV), aux)
    loss.backward()
    rlog, raux = OT.forward_train(sd, images, rois, u, cfg, (96, 128))
    rloss, rd = OT.RefinedHierarchicalLoss()(rlog, tgt, raux)
    rloss.backward()
    assert _relm(logits.detach(), rlog.detach()) < 3e-3
    assert loss.item() == pytest.approx(rloss.item(), rel=1e-4)
    tot_m = tot_r = 0.0
    for n, p in m.named_parameters():
        if n not in sd or not sd[n].requires_grad:
            continue
        rg = sd[n].grad
        if rg is None:
            assert p.grad is None or not p.grad.any(), n
            continue
        mg = p.grad.detach().cpu().double().reshape(-1)
        rg = rg.double().reshape(-1)
        tot_m += float((mg ** 2).sum())
        tot_r += float((rg ** 2).sum())
        if rg.norm() < 1e-6 * (1 + rg.numel()) ** 0.5 or (n.endswith(".bias") and rg.norm() < 1e-4):
            continue
        cos = float((mg * rg).sum() / (mg.norm() * rg.norm()))
        assert cos > 0.99, (n, cos)
    assert abs(tot_m / tot_r - 1) < 4e-2


def test_layernorm_gelu_bf16_training_decreases_loss():
    import hiseg
    kw = hiseg_kwargs(dict(b0_kwargs(), normalization_type="layernorm2d", activation_function="gelu"))
    m = filler.fill_module(hiseg.create_rgb_hierarchical_model(**kw))
    hiseg.set_compute_dtype(m, torch.bfloat16)
    m = m.to(DEV).train()
    images = torch.from_numpy(filler.uniform(91, (2, 3, 160, 192))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(92, 2, 2)).to(DEV)
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 160, 192
    tgt = torch.from_numpy(filler.ellipse_targets(93, 4, 128, 96)).to(DEV)
    loss_fn = hiseg.RefinedHierarchicalLoss()
    opt, losses = None, []
    for _ in range(5):
        logits, aux = m(images, rois)
        loss, _ = loss_fn(logits, tgt, aux)
        if opt is None:
            opt = hiseg.FusedAdamW(m, lr=5e-4)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses

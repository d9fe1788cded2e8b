"""16-frame two-view step (train_hardway.py:126-144) on libavt: kernels against fp64 autograd, and the
whole step (fused TwoViewTrainStep and the drop-in AVENet + autograd path) against golden vectors the
reference's own AVENet produced (oracle/gen_golden_twoview.py).

End-to-end tolerances follow tests/test_model_gpu.py: max(floor, 3 x the deviation of the reference's
own trunks run under bf16 autocast with the fp32 head/losses, measured against the same fp64 run).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import avenet_oracle as orc
from avt_amd._lib import call, query
from avt_amd.losses import PropagationLoss
from avt_amd.model import AVENet
from avt_amd.train import TwoViewTrainStep
from avt_amd.trunk import P
from gradcheck import check_grads

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def S():
    import ctypes

    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def rel_err(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _golden(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False))


def _model(seed=0):
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(seed))
    return m.to(DEV).train()


def _inputs(g):
    b, t, s, f, ft = g["shape"].tolist()
    return orc.make_frames(b, t, s, seed=3), orc.make_frames(b, t, s, seed=4), orc.make_spectrogram(b, f, ft)


# ------------------------------------------------------------------------------------ kernels
def test_ncthw_fold_matches_einops():
    g = torch.Generator().manual_seed(30)
    x = torch.randn(2, 3, 5, 9, 11, generator=g)
    y = torch.empty(10, 9, 11, 4, device=DEV, dtype=torch.bfloat16)
    xd = x.to(DEV)
    call("avt_ncthw_to_nhwc_bf16", P(xd), P(y), 2, 3, 5, 9, 11, 4, S())
    ref = torch.zeros(10, 9, 11, 4, dtype=torch.bfloat16)
    ref[..., :3] = orc.fold_frames(x).permute(0, 2, 3, 1).to(torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), ref)


@pytest.mark.parametrize("B,h,w", [(6, 14, 14), (4, 4, 4), (32, 14, 14)])
def test_hardway_bwd_through_weighted_A(B, h, w):
    """d(CE(logits) + <dwA, weighted_A>) w.r.t. the vision map and the unit audio vectors."""
    C, Pn = 512, h * w
    g = torch.Generator().manual_seed(31)
    v = (torch.randn(B, h, w, C, generator=g).abs() + 0.3 * torch.rand(B, 1, 1, C, generator=g)).to(torch.bfloat16)
    an = F.normalize(torch.randn(B, C, generator=g).abs() + 0.5, dim=1)
    dwA = torch.randn(B, Pn, generator=g)
    f32 = dict(device=DEV, dtype=torch.float32)
    L = B + 2
    inv, vsum = torch.empty(B, Pn, **f32), torch.empty(B, Pn, **f32)
    A0 = torch.empty(B, Pn, B, **f32)
    save = torch.empty(int(query("avt_hardway_save_floats", B)), **f32)
    logits, A, Pos, Neg, wA = (torch.empty(B, L, **f32),) + tuple(torch.empty(B, Pn, **f32) for _ in range(4))
    vd, and_ = v.to(DEV), an.to(DEV)
    call("avt_hardway_fwd", P(vd), P(and_), B, Pn, C, 0.65, 0.4, 0.03, 1, 1, P(inv), P(vsum), P(A0), P(save),
         P(logits), P(A), P(Pos), P(Neg), P(wA), S())
    loss = torch.empty((), **f32)
    dl = torch.empty(B, L, **f32)
    call("avt_hardway_ce", P(logits), B, L, 1.0, P(loss), P(dl), S())
    dA0, dvh, dm = torch.empty(B, Pn, B, **f32), torch.empty(B, Pn, C, **f32), torch.empty(B, Pn, **f32)
    gv, gan = torch.empty_like(vd), torch.empty(B, C, **f32)
    dwd = dwA.to(DEV)
    call("avt_hardway_bwd", P(vd), P(and_), P(inv), P(A0), P(save), P(dl), B, Pn, C, 0.65, 0.4, 0.03, 1, 1, P(dwd),
         P(vsum), P(dm), P(dA0), P(dvh), P(gv), P(gan), 0, S())
    gan1 = gan.clone()
    # second call accumulating into gan (two views sharing one audio batch)
    gv2 = torch.empty_like(vd)
    call("avt_hardway_bwd", P(vd), P(and_), P(inv), P(A0), P(save), P(dl), B, Pn, C, 0.65, 0.4, 0.03, 1, 1, P(dwd),
         P(vsum), P(dm), P(dA0), P(dvh), P(gv2), P(gan), 1, S())
    torch.cuda.synchronize()
    vt = v.double().permute(0, 3, 1, 2).requires_grad_(True)
    at = an.double().requires_grad_(True)
    rA, rlog, rwA, _, _ = orc.hardway_head(F.normalize(vt, dim=1), at)
    (orc.hardway_ce(rlog) + (rwA.reshape(B, Pn) * dwA.double()).sum()).backward()
    assert (wA.cpu().double() - rwA.detach().reshape(B, Pn)).abs().max() < 1e-5
    assert rel_err(gan1, at.grad) < 2e-3
    assert rel_err(gv, vt.grad.permute(0, 2, 3, 1)) < 1e-2
    assert torch.equal(gv, gv2)
    assert rel_err(gan, 2 * gan1) < 1e-6
    # the weighted_A term is not negligible in these inputs (the test exercises that path)
    at2 = an.double().requires_grad_(True)
    _, rlog2, _, _, _ = orc.hardway_head(F.normalize(v.double().permute(0, 3, 1, 2), dim=1), at2)
    orc.hardway_ce(rlog2).backward()
    assert rel_err(at2.grad, at.grad) > 1e-2


@pytest.mark.parametrize("b,t,Pn,ties", [(2, 3, 16, False), (8, 16, 196, False), (3, 4, 196, True)])
def test_twoview_loss_kernel(b, t, Pn, ties):
    g = torch.Generator().manual_seed(32)
    w1 = torch.randn(b * t, Pn, generator=g).abs() * 0.05
    w2 = w1 + 0.01 * torch.randn(b * t, Pn, generator=g)
    if ties:  # equal neighbouring frames: |diff| = 0, torch's abs'(0) = 0
        w1.view(b, t, Pn)[:, 1] = w1.view(b, t, Pn)[:, 0]
    ce = torch.tensor([1.7, 2.3])
    lw = 0.1
    out = torch.empty(5, device=DEV)
    d1, d2 = torch.empty(b * t, Pn, device=DEV), torch.empty(b * t, Pn, device=DEV)
    ced, w1d, w2d = ce.to(DEV), w1.to(DEV), w2.to(DEV)  # kept referenced until the kernel has run
    call("avt_twoview_loss", P(ced[0:1]), P(ced[1:2]), P(w1d), P(w2d), b, t, Pn, lw, P(out), P(d1), P(d2), S())
    torch.cuda.synchronize()
    x1, x2 = w1.double().requires_grad_(True), w2.double().requires_grad_(True)
    hw = (1, Pn)
    l2 = F.mse_loss(x1, x2) * (100 - lw)
    cons = orc.propagation_loss(x1.reshape(b, t, *hw)) + orc.propagation_loss(x2.reshape(b, t, *hw))
    hard, aug = lw * ce[0].double(), lw * ce[1].double()
    comb = (hard + aug) / 2 + l2 + cons
    comb.backward()
    ref = torch.stack([comb, hard, aug, l2, cons]).detach()
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), rtol=2e-5, atol=1e-8)
    assert rel_err(d1, x1.grad) < 1e-5
    assert rel_err(d2, x2.grad) < 1e-5


def test_propagation_loss_module():
    g = torch.Generator().manual_seed(33)
    x = torch.randn(3, 5, 14, 14, generator=g)
    x[:, 2] = x[:, 1]  # ties
    xd = x.to(DEV).requires_grad_(True)
    loss = PropagationLoss()(xd)
    loss.backward(torch.tensor(2.5, device=DEV))
    xr = x.double().requires_grad_(True)
    ref = orc.propagation_loss(xr)
    (2.5 * ref).backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    assert rel_err(xd.grad, xr.grad) < 1e-6


@pytest.mark.parametrize("b,t", [(3, 5), (8, 16), (1, 2), (300, 16)])
def test_npratio_loss_module(b, t):
    """losses.NPRatio (losses.py:7-14; train_3D.py:113, 135) vs its torch restatement in fp64."""
    from avt_amd.losses import NPRatio

    g = torch.Generator().manual_seed(34)
    x = torch.rand(b, t, 14, 14, generator=g)
    if t > 2:
        x[:, 2] = x[:, 1]  # a tie: sgn(0) = 0
    xd = x.to(DEV).requires_grad_(True)
    loss = NPRatio()(xd)
    loss.backward(torch.tensor(1.5, device=DEV))
    xr = x.double().requires_grad_(True)
    ref = orc.npratio_loss(xr)
    (1.5 * ref).backward()
    assert abs(loss.item() - ref.item()) < 2e-5 * max(1e-3, abs(ref.item()))
    assert rel_err(xd.grad, xr.grad) < 1e-6


@pytest.mark.parametrize("shape", [(4, 1, 14, 14), (2, 3, 7, 9), (5, 224), (64, 1, 224, 224)])
def test_flip_loss_module(shape):
    """losses.FlipLoss (losses.py:25-36): L1(flipped, hflip(heatmap)) and both gradients, fp64 ref."""
    from avt_amd.losses import FlipLoss

    g = torch.Generator().manual_seed(35)
    x, y = torch.randn(*shape, generator=g), torch.randn(*shape, generator=g)
    y.view(-1, shape[-1])[0] = x.view(-1, shape[-1])[0].flip(-1)  # exact zeros: sgn(0) = 0
    xd, yd = x.to(DEV).requires_grad_(True), y.to(DEV).requires_grad_(True)
    loss = FlipLoss()(xd, yd)
    loss.backward(torch.tensor(0.7, device=DEV))
    xr, yr = x.double().requires_grad_(True), y.double().requires_grad_(True)
    ref = orc.flip_loss(xr, yr)
    (0.7 * ref).backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    assert rel_err(xd.grad, xr.grad) < 1e-6 and rel_err(yd.grad, yr.grad) < 1e-6
    # a multi-block grid (a full-resolution batch is 3.2 M elements) with a fixed-order reduction
    assert FlipLoss()(xd, yd).item() == loss.item()


# ------------------------------------------------------------------------------ whole step
FLOORS = {"logits_off_abs": 2e-2, "logits_diag_rel": 2e-3, "wA_rel": 5e-2}


def _check_step(name, g, losses, logits1, wA1, wA2, grads):
    """logits, weighted_A and the five loss terms against the fp64 reference run, and every parameter gradient
    against its own bf16-autocast yardstick (tests/gradcheck.check_grads, as the 1-frame tests).  grads: name ->
    gradient shaped like the Parameter (OIHW)."""
    b, t = g["shape"].tolist()[:2]
    B = b * t
    logits1 = logits1.detach().cpu().double().numpy()
    diag = np.eye(B, B + 2, k=1, dtype=bool)
    lg = g["logits1_f64"]
    wmax = max(np.abs(g["wA1_f64"]).max(), np.abs(g["wA2_f64"]).max())
    dev = {
        "logits_off_abs": np.abs(logits1[~diag] - lg[~diag]).max(),
        "logits_diag_rel": (np.abs(logits1[diag] - lg[diag]) / np.abs(lg[diag])).max(),
        "wA_rel": max(np.abs(wA1.detach().cpu().double().numpy().reshape(g["wA1_f64"].shape) - g["wA1_f64"]).max(),
                      np.abs(wA2.detach().cpu().double().numpy().reshape(g["wA2_f64"].shape) - g["wA2_f64"]).max())
        / wmax,
    }
    for k, v in dev.items():
        tol = max(FLOORS[k], 3 * float(g["bf16ref_dev/" + k]))
        print(f"{name}: {k} = {v:.3e} (bf16 reference {float(g['bf16ref_dev/' + k]):.3e}, tol {tol:.3e})")
        assert v <= tol, (k, v, tol)
    # loss terms: |term - fp64| in units of the combined fp64 loss (the 99.9 x MSE term is a small difference of the
    # two views' maps, so its own relative error is no measure), each within max(1e-3, 3 x the yardstick's)
    l = losses.detach().cpu().double().numpy()
    labs = np.abs(l - g["losses_f64"]) / abs(float(g["losses_f64"][0]))
    ltol = np.maximum(1e-3, 3 * g["bf16ref_dev/loss_abs"])
    print(f"{name}: losses {l} ref {g['losses_f64']} |d|/combined {labs} tol {ltol}")
    assert np.all(labs <= ltol), (labs, ltol)
    check_grads(g, grads, tag=name)


def _oihw(views):
    """flat-buffer gradient views (conv weights OHWI) -> the Parameters' OIHW shapes"""
    return {n: (v.permute(0, 3, 1, 2) if v.dim() == 4 else v) for n, v in views.items()}


@pytest.mark.parametrize("name", ["twoview_tiny_b2t3", "twoview_full_b2t2", "twoview_full_b2t16"])
@pytest.mark.parametrize("dedup", [True, False])
def test_fused_twoview_step_vs_reference(golden_dir, name, dedup):
    g = _golden(golden_dir, name)
    fr, au, sp = (x.to(DEV) for x in _inputs(g))
    lw, lr, wd = g["hyper"].tolist()
    model = _model()
    step = TwoViewTrainStep(model, lr=lr, weight_decay=wd, loss_weight=lw, dedup_audio=dedup)
    outs = {}  # the outputs of the forward the step runs
    orig = step.engine.forward

    def spy(*a, **k):
        out, tape = orig(*a, **k)
        outs.update(out)
        return out, tape

    step.engine.forward = spy
    losses = step.step(fr, au, sp)
    torch.cuda.synchronize()
    o1, o2 = outs["views"]
    _check_step(f"{name}/dedup={dedup}", g, losses, o1["logits"], o1["weighted_A"], o2["weighted_A"],
                _oihw(step.flat.grad_views(step.grad)))
    sd = model.state_dict()
    from gen_golden import BUF_SLICES

    for k in BUF_SLICES:  # both forwards' running-stat updates
        ref = g["buf_f64/" + k]
        got = sd[k][:16].cpu().double().numpy()
        assert np.abs(got - ref).max() <= 2e-2 * max(1.0, np.abs(ref).max()), k
    assert int(sd["imgnet.bn1.num_batches_tracked"]) == int(sd["audnet.bn1.num_batches_tracked"]) == 2
    before = orc.make_state(0)
    for n in ["imgnet.conv1.weight", "audnet.layer4.1.conv2.weight", "imgnet.bn1.weight"]:
        got = (sd[n].cpu().double() - before[n].double()).flatten()[:64].numpy()
        ref = g["delta_slice_f64/" + n]
        agree = np.mean(np.sign(got) == np.sign(ref))
        # the first Adam update is ~ -lr sign(g + wd w): a bf16 gradient flips the sign of its near-zero entries.
        # Bound: 0.75, or the bf16-autocast reference's own agreement on these 64 values less 2 binomial sigmas
        w0 = before[n].double().flatten()[:64].numpy()
        a_ref = np.mean(np.sign(-(g["bf16ref_slice/" + n] + wd * w0)) == np.sign(ref))
        bound = min(0.75, a_ref - 2 * np.sqrt(a_ref * (1 - a_ref) / 64))
        print(f"{n}: sign agreement of first Adam update {agree:.3f} (bf16 reference {a_ref:.3f}, bound {bound:.3f})")
        assert agree >= bound, n
        assert np.abs(got).max() <= lr + 1.2e-7, n


def test_dropin_autograd_twoview_vs_reference(golden_dir):
    """train_hardway.py's own loop (126-144) on the drop-in AVENet: two forwards, nn.CrossEntropyLoss /
    nn.MSELoss / PropagationLoss, autograd backward.  Against the reference's golden run, with the same
    bounds as the fused step; and against the fused step (audio not de-duplicated: the same kernel
    sequence).  Two numerically different but equivalent paths differ at the bf16 noise floor: a
    1e-7 perturbation (torch's vs libavt's softmax) flips bf16 roundings of activation gradients,
    which BN-backward cancellation over these tiny maps amplifies to ~1 % of a weight gradient
    (measured 0.6 % for the 1-frame drop-in vs fused step, 1.5 % here; run-to-run spread of one
    path: 5e-7)."""
    g = _golden(golden_dir, "twoview_tiny_b2t3")
    fr, au, sp = (x.to(DEV) for x in _inputs(g))
    lw, lr, wd = g["hyper"].tolist()
    b, t = fr.shape[0], fr.shape[2]
    m1 = _model()
    spec = orc.fold_spec(sp, t)
    heat, out, weighted, _, _ = m1(orc.fold_frames(fr), spec)
    heat2, out2, weighted2, _, _ = m1(orc.fold_frames(au), spec)
    target = torch.zeros(out.shape[0], dtype=torch.long, device=DEV)
    ce = torch.nn.CrossEntropyLoss()
    hardway_loss = ce(out, target) * lw
    aug_loss = ce(out2, target) * lw
    l2_loss = torch.nn.MSELoss()(weighted, weighted2) * (100 - lw)
    h, w = weighted.shape[-2:]
    prop = PropagationLoss()
    consistency = prop(weighted.reshape(b, t, h, w)) + prop(weighted2.reshape(b, t, h, w))
    combined = (hardway_loss + aug_loss) / 2 + l2_loss + consistency
    combined.backward()
    ref = torch.stack([combined, hardway_loss, aug_loss, l2_loss, consistency]).detach()
    p1 = dict(m1.named_parameters())
    _check_step("twoview_tiny_b2t3/drop-in", g, ref, out, weighted, weighted2,
                {n: p.grad for n, p in p1.items() if p.grad is not None})
    assert int(m1.state_dict()["imgnet.bn1.num_batches_tracked"]) == 2
    m2 = _model()
    step = TwoViewTrainStep(m2, lr=lr, weight_decay=wd, loss_weight=lw, dedup_audio=False)
    step.opt.lr = 0.0  # compare gradients only
    losses = step.step(fr, au, sp)
    torch.cuda.synchronize()
    assert rel_err(losses, ref) < 1e-5
    views = step.flat.grad_views(step.grad)
    tot_d, tot_n = 0.0, 0.0
    for n, gv in views.items():
        g1 = p1[n].grad
        assert g1 is not None, n
        g1 = g1.permute(0, 2, 3, 1) if g1.dim() == 4 else g1
        tot_d += (g1 - gv).double().pow(2).sum().item()
        tot_n += gv.double().pow(2).sum().item()
    print("drop-in vs fused: global rel grad diff", (tot_d / tot_n) ** 0.5)
    assert (tot_d / tot_n) ** 0.5 < 5e-2
    for n, p in p1.items():  # exactly the reference's trainable set gets gradients
        assert (p.grad is not None) == (n in views), n


def test_twoview_graph_replay_matches_eager():
    b, t = 2, 3
    data = [(orc.make_frames(b, t, 64, seed=s), orc.make_frames(b, t, 64, seed=s + 10),
             orc.make_spectrogram(b, 65, 76, seed=s)) for s in (1, 2, 3)]
    m_e, m_g = _model(), _model()
    s_e, s_g = TwoViewTrainStep(m_e), TwoViewTrainStep(m_g)
    le, lg = [], []
    for x in data:
        le.append(s_e.step(*(y.to(DEV) for y in x)).cpu().numpy())
    for i, x in enumerate(data):
        x = [y.to(DEV) for y in x]
        lg.append(s_g.step(*x).cpu().numpy())
        if i == 0:
            s_g.capture(*(y.clone() for y in x))
    print("eager", le, "graph", lg)
    np.testing.assert_allclose(np.array(lg), np.array(le), rtol=1e-4, atol=1e-7)
    assert s_e.opt.t == s_g.opt.t == 3
    sd_e, sd_g = m_e.state_dict(), m_g.state_dict()
    for k in sd_e:
        a, c = sd_e[k].double(), sd_g[k].double()
        if k.endswith("num_batches_tracked"):
            assert int(a) == int(c) == 6, k
        elif "running" in k:
            assert (a - c).abs().max().item() <= 1e-3 * max(1.0, a.abs().max().item()), k
        else:  # <= lr per step; atomics can flip a ~0 gradient's update
            assert (a - c).abs().max().item() <= 3 * 2 * 4e-6 + 5e-7, k


def test_twoview_loss_decreases():
    b, t = 2, 4
    fr, au = orc.make_frames(b, t, 64, seed=5).to(DEV), orc.make_frames(b, t, 64, seed=6).to(DEV)
    sp = orc.make_spectrogram(b, 65, 76, seed=7).to(DEV)
    step = TwoViewTrainStep(_model(), lr=1e-4)
    hist = [step.step(fr, au, sp)[0].item() for _ in range(8)]
    assert np.all(np.isfinite(hist))
    assert hist[-1] < hist[0], hist

"""Golden vectors for the 16-frame two-view step (train_hardway.py:126-144) from the REFERENCE's
own AVENet (survey container only; imports /root/reference/model.py exactly as gen_golden.py does).

Run here:   python oracle/gen_golden_twoview.py   -> tests/golden/twoview_*.npz

The step: spec [b,1,F,T] repeated t times and folded '(b t)'; frames / augmented [b,3,t,H,W]
folded '(b t)'; two AVENet forwards (BN running stats updated by both, num_batches_tracked += 2);
combined = (0.1*CE1 + 0.1*CE2)/2 + 99.9*MSE(weighted, weighted2) + Prop(weighted) + Prop(weighted2);
backward; torch.optim.Adam(lr 4e-6, weight_decay 1e-4) (train_hardway.py:58-59, 115).
losses.py is not importable, so PropagationLoss is the restatement in
avenet_oracle.propagation_loss (a one-line formula, losses.py:22-23); everything else — the model,
its autograd through weighted_A, MSE, CE, Adam — is the reference / torch itself.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import avenet_oracle as orc  # noqa: E402
from gen_golden import BUF_SLICES, OUT, SLICE_PARAMS, checksum, grad_sample, import_reference  # noqa: E402

LW = 0.1
LR = 4e-6


def run_reference(ref_model, sd, frames, augmented, spec, dtype):
    b, t = frames.shape[0], frames.shape[2]
    net = ref_model.AVENet(orc.Args(), False)
    net.load_state_dict(sd, strict=True)
    net = net.to(dtype).train()
    aud = orc.fold_spec(spec, t).to(dtype)
    out1 = net(orc.fold_frames(frames).to(dtype), aud)
    out2 = net(orc.fold_frames(augmented).to(dtype), aud)
    losses = orc.twoview_losses(out1, out2, b, t, LW)
    opt = torch.optim.Adam(net.parameters(), lr=LR, weight_decay=1e-4)
    opt.zero_grad()
    losses[0].backward()
    names = [n for n, p in net.named_parameters() if p.grad is not None]
    grads = {n: p.grad.detach().clone() for n in names for p in [dict(net.named_parameters())[n]]}
    before = {n: p.detach().clone() for n, p in net.named_parameters()}
    opt.step()
    after = {n: p.detach().clone() for n, p in net.named_parameters()}
    bufs = {n: x.detach().clone() for n, x in net.named_buffers()}
    return dict(losses=torch.stack([x.detach() for x in losses]), logits1=out1[1].detach(), logits2=out2[1].detach(),
                wA1=out1[2].detach(), wA2=out2[2].detach(), A1=out1[0].detach(), names=names, grads=grads,
                before=before, after=after, bufs=bufs)


def run_reference_bf16_trunks(ref_model, sd, frames, augmented, spec):
    """The reference's own trunks under CPU bf16 autocast + the fp32 head and losses: the yardstick
    for a bf16-trunk build's deviation from fp64 on this step."""
    b, t = frames.shape[0], frames.shape[2]
    net = ref_model.AVENet(orc.Args(), False)
    net.load_state_dict(sd, strict=True)
    net.train()
    aud = orc.fold_spec(spec, t)
    outs = []
    for x in (orc.fold_frames(frames), orc.fold_frames(augmented)):
        with torch.autocast("cpu", dtype=torch.bfloat16):
            img = net.imgnet(x)
            a = net.audnet(aud)
        img = torch.nn.functional.normalize(img.float(), dim=1)
        a = torch.nn.functional.normalize(torch.nn.functional.adaptive_max_pool2d(a.float(), 1).flatten(1), dim=1)
        outs.append(orc.hardway_head(img, a))
    losses = orc.twoview_losses(outs[0], outs[1], b, t, LW)
    losses[0].backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    return dict(losses=torch.stack([x.detach() for x in losses]), logits1=outs[0][1].detach(),
                wA1=outs[0][2].detach(), wA2=outs[1][2].detach(), grads=grads)


def loss_abs_dev(res, r64):
    """|loss term - fp64| of each of the five terms, in units of the combined fp64 loss (the MSE term is a small
    difference of two views' maps: its own relative deviation says little)"""
    return np.abs(res["losses"].double().numpy() - r64["losses"].numpy()) / abs(float(r64["losses"][0]))


def deviation(res, r64, names):
    gn = np.array([res["grads"][n].double().norm().item() for n in names])
    g64 = np.array([r64["grads"][n].norm().item() for n in names])
    l, l64 = res["losses"].double().numpy(), r64["losses"].numpy()
    wmax = max(np.abs(r64["wA1"].numpy()).max(), np.abs(r64["wA2"].numpy()).max())
    lg, lg64 = res["logits1"].double().numpy(), r64["logits1"].numpy()
    B = lg.shape[0]
    diag = np.eye(B, B + 2, k=1, dtype=bool)
    return {
        "loss_rel": np.abs(l - l64) / np.abs(l64),
        "logits_off_abs": np.abs(lg[~diag] - lg64[~diag]).max(),
        "logits_diag_rel": (np.abs(lg[diag] - lg64[diag]) / np.abs(lg64[diag])).max(),
        "wA_rel": max(np.abs(res["wA1"].double().numpy() - r64["wA1"].numpy()).max(),
                      np.abs(res["wA2"].double().numpy() - r64["wA2"].numpy()).max()) / wmax,
        "gradnorm_rel": np.abs(gn - g64) / g64,
    }


def make_fixture(ref_model, name, b, t, img_size, freq, frames_t, seed_w=0):
    sd = orc.make_state(seed_w, torch.float32)
    frames = orc.make_frames(b, t, img_size, seed=3)
    augmented = orc.make_frames(b, t, img_size, seed=4)
    spec = orc.make_spectrogram(b, freq, frames_t)
    res = {tag: run_reference(ref_model, sd, frames, augmented, spec, dt)
           for tag, dt in (("f64", torch.float64), ("f32", torch.float32))}
    r64, r32 = res["f64"], res["f32"]
    names = r64["names"]
    out = {"param_names": np.array(names)}
    for k in ("losses", "logits1", "logits2", "wA1", "wA2", "A1"):
        out[k + "_f64"] = r64[k].numpy()
        out[k + "_f32"] = r32[k].float().numpy()
    out["grad_norm_f64"] = np.array([r64["grads"][n].norm().item() for n in names])
    out["grad_norm_f32"] = np.array([r32["grads"][n].float().norm().item() for n in names])
    for n in SLICE_PARAMS:
        out["grad_slice_f64/" + n] = r64["grads"][n].flatten()[:64].numpy()
        out["delta_slice_f64/" + n] = (r64["after"][n] - r64["before"][n]).flatten()[:64].numpy()
    for n in BUF_SLICES:
        out["buf_f64/" + n] = r64["bufs"][n][:16].numpy()
    out["nbt_f64"] = np.array([r64["bufs"]["imgnet.bn1.num_batches_tracked"].item(),
                               r64["bufs"]["audnet.bn1.num_batches_tracked"].item()])
    for n in names:  # strided samples of every gradient, fp64 and the bf16-autocast yardstick (tests/gradcheck.py)
        out["grad_sample_f64/" + n] = grad_sample(r64["grads"][n])
    rb = run_reference_bf16_trunks(ref_model, sd, frames, augmented, spec)
    for n in names:
        out["bf16ref_sample/" + n] = grad_sample(rb["grads"][n])
    for n in SLICE_PARAMS:
        out["bf16ref_slice/" + n] = rb["grads"][n].flatten()[:64].double().numpy()
    dev = deviation(rb, r64, names)
    dev["loss_abs"] = loss_abs_dev(rb, r64)
    for k, v in dev.items():
        out["bf16ref_dev/" + k] = np.asarray(v)
    print(f"[{name}] bf16-trunk reference deviation: " + ", ".join(f"{k}={np.max(v):.3e}" for k, v in dev.items()))
    out["frames_checksum"] = checksum(frames)
    out["augmented_checksum"] = checksum(augmented)
    out["spec_checksum"] = checksum(spec)
    out["shape"] = np.array([b, t, img_size, freq, frames_t])
    out["hyper"] = np.array([LW, LR, 1e-4])
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)

    # pin the restatement against the reference on the same inputs (fp64, bit-level)
    sd64 = orc.OrderedDict((k, v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items())
    losses, o1, o2, grads = orc.twoview_step(sd64, frames.double(), augmented.double(), spec.double(),
                                             orc.AdamRef(lr=LR), None, LW)
    dl = (torch.stack(losses) - r64["losses"]).abs().max().item()
    dw = (o1[2] - r64["wA1"]).abs().max().item()
    dg = max(abs(grads[n].norm().item() - r64["grads"][n].norm().item()) / max(r64["grads"][n].norm().item(), 1e-30)
             for n in names)
    dd = max((sd64[n] - r64["after"][n]).abs().max().item() for n in names)
    print(f"[{name}] losses ref64={r64['losses'].tolist()}  oracle |dloss|={dl:.2e} |dwA|={dw:.2e} "
          f"max rel dgradnorm={dg:.2e} |dparam after Adam|={dd:.2e} -> {path}")
    assert set(grads) == set(names), sorted(set(grads) ^ set(names))
    assert dl < 1e-9 and dw < 1e-12 and dg < 1e-9 and dd < 1e-12


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    ref_model = import_reference()
    make_fixture(ref_model, "twoview_tiny_b2t3", b=2, t=3, img_size=64, freq=65, frames_t=76)
    make_fixture(ref_model, "twoview_full_b2t2", b=2, t=2, img_size=224, freq=257, frames_t=300)
    # train_hardway.py's own 16 frames per clip at full size: 32 head rows per view
    make_fixture(ref_model, "twoview_full_b2t16", b=2, t=16, img_size=224, freq=257, frames_t=300)


if __name__ == "__main__":
    main()

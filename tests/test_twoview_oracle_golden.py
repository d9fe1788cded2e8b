"""The oracle's 16-frame two-view step (avenet_oracle.twoview_step, restating train_hardway.py:126-144)
against golden vectors the REFERENCE's own AVENet produced (oracle/gen_golden_twoview.py).  CPU-only."""
import os

import numpy as np
import pytest
import torch

import avenet_oracle as orc
from gen_golden import checksum

NAMES = ["twoview_tiny_b2t3", "twoview_full_b2t2"]
# the 16-frame fixture: its inputs regenerate here; its fp64 oracle run (64 images at 224^2) is left to the generator,
# which asserts the oracle == the reference on it bit for bit (oracle/gen_golden_twoview.py)
ALL = NAMES + ["twoview_full_b2t16"]


def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False))


def _inputs(g):
    b, t, s, f, ft = g["shape"].tolist()
    return orc.make_frames(b, t, s, seed=3), orc.make_frames(b, t, s, seed=4), orc.make_spectrogram(b, f, ft)


@pytest.mark.parametrize("name", ALL)
def test_twoview_inputs_regenerate(golden_dir, name):
    g = _load(golden_dir, name)
    fr, au, sp = _inputs(g)
    np.testing.assert_allclose(checksum(fr), g["frames_checksum"], rtol=1e-12)
    np.testing.assert_allclose(checksum(au), g["augmented_checksum"], rtol=1e-12)
    np.testing.assert_allclose(checksum(sp), g["spec_checksum"], rtol=1e-12)


@pytest.mark.parametrize("name", NAMES)
def test_twoview_oracle_fp64_matches_reference(golden_dir, name):
    """fp64 restatement == the reference's fp64 run (same arithmetic order: bit-level agreement)."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = _load(golden_dir, name)
    fr, au, sp = _inputs(g)
    lw, lr, wd = g["hyper"].tolist()
    sd = orc.OrderedDict((k, v.double() if v.is_floating_point() else v.clone()) for k, v in orc.make_state(0).items())
    before = {k: v.clone() for k, v in sd.items()}
    losses, o1, o2, grads = orc.twoview_step(sd, fr.double(), au.double(), sp.double(),
                                             orc.AdamRef(lr=lr, weight_decay=wd), None, lw)
    np.testing.assert_allclose(torch.stack(losses).numpy(), g["losses_f64"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(o1[1].numpy(), g["logits1_f64"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(o2[2].numpy(), g["wA2_f64"], rtol=1e-12, atol=1e-15)
    names = [str(n) for n in g["param_names"]]
    assert sorted(names) == sorted(grads)
    gn = np.array([grads[n].norm().item() for n in names])
    np.testing.assert_allclose(gn, g["grad_norm_f64"], rtol=1e-10)
    from gen_golden import BUF_SLICES, SLICE_PARAMS

    for n in SLICE_PARAMS:
        np.testing.assert_allclose(grads[n].flatten()[:64].numpy(), g["grad_slice_f64/" + n], rtol=1e-9, atol=1e-14)
        np.testing.assert_allclose((sd[n] - before[n]).flatten()[:64].numpy(), g["delta_slice_f64/" + n],
                                   rtol=1e-6, atol=1e-15)
    for n in BUF_SLICES:  # both forwards updated the running statistics
        np.testing.assert_allclose(sd[n][:16].numpy(), g["buf_f64/" + n], rtol=1e-12, atol=1e-15)
    assert int(sd["imgnet.bn1.num_batches_tracked"]) == int(g["nbt_f64"][0]) == 2


@pytest.mark.parametrize("name", ALL)
def test_twoview_loss_terms_are_the_reference_formulas(golden_dir, name):
    """Loss bookkeeping of train_hardway.py:134-142 on the stored fp64 outputs."""
    g = _load(golden_dir, name)
    b, t = g["shape"].tolist()[:2]
    lw = float(g["hyper"][0])
    w1, w2 = torch.from_numpy(g["wA1_f64"]), torch.from_numpy(g["wA2_f64"])
    l = g["losses_f64"]
    assert abs(l[0] - ((l[1] + l[2]) / 2 + l[3] + l[4])) < 1e-15
    np.testing.assert_allclose(l[3], torch.mean((w1 - w2) ** 2).item() * (100 - lw), rtol=1e-12)
    h, w = w1.shape[-2:]
    prop = orc.propagation_loss(w1.reshape(b, t, h, w)) + orc.propagation_loss(w2.reshape(b, t, h, w))
    np.testing.assert_allclose(l[4], prop.item(), rtol=1e-12)
    # Prop = mean_{clip, s, p} |x[:, s+1] - x[:, s]|
    x = w1.reshape(b, t, -1)
    np.testing.assert_allclose(orc.propagation_loss(w1.reshape(b, t, h, w)).item(),
                               (x[:, 1:] - x[:, :-1]).abs().mean().item(), rtol=1e-12)

"""The oracle (CPU restatement, oracle/avenet_oracle.py) against golden vectors that the
reference itself produced (oracle/gen_golden.py). CPU-only."""
import os

import numpy as np
import pytest
import torch

import avenet_oracle as orc
from gen_golden import checksum


def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False))


@pytest.mark.parametrize("name", ["avenet_tiny_b4", "avenet_full_b2"])
def test_inputs_and_weights_regenerate(golden_dir, name):
    g = _load(golden_dir, name)
    b, s, f, t = g["shape"].tolist()
    img = orc.make_image(b, s)
    aud = orc.make_spectrogram(b, f, t)
    np.testing.assert_allclose(checksum(img), g["image_checksum"], rtol=1e-12)
    np.testing.assert_allclose(checksum(aud), g["audio_checksum"], rtol=1e-12)
    sd = orc.make_state(0)
    from gen_golden import SLICE_PARAMS
    np.testing.assert_allclose([checksum(sd[n])[0] for n in SLICE_PARAMS], g["weight_checksum"], rtol=1e-12)


@pytest.mark.parametrize("name", ["avenet_tiny_b4", "avenet_full_b2"])
def test_oracle_fp32_forward_loss_grads(golden_dir, name):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = _load(golden_dir, name)
    b, s, f, t = g["shape"].tolist()
    img = orc.make_image(b, s)
    aud = orc.make_spectrogram(b, f, t)
    sd = orc.make_state(0)
    A, logits, wA, Pos, Neg = orc.avenet_forward(dict(sd), img, aud)
    # SURVEY §8(c) tolerances for an fp32 path vs the fp64 reference
    np.testing.assert_allclose(A.numpy(), g["A_f64"], atol=1e-5)
    off = ~np.eye(b, b + 2, k=1, dtype=bool)
    np.testing.assert_allclose(logits.numpy()[off], g["logits_f64"][off], atol=1e-3, rtol=1e-4)
    np.testing.assert_allclose(wA.numpy(), g["weighted_A_f64"], atol=1e-5)
    np.testing.assert_allclose(Pos.numpy(), g["Pos_f64"], atol=1e-3)
    np.testing.assert_allclose(Neg.numpy(), g["Neg_f64"], atol=1e-3)
    sd = orc.make_state(0)
    loss, _, grads = orc.train_step(sd, img, aud, orc.AdamRef())
    assert abs(loss.item() - g["loss_f64"].item()) <= 1e-5 * abs(g["loss_f64"].item())
    names = [str(n) for n in g["param_names"]]
    gn = np.array([grads[n].norm().item() for n in names])
    # fp32 grad norms drift up to ~2e-3 rel from fp64 in the reference itself (BN bias grads
    # are cancelling sums over B*H*W); the restatement reproduces the reference fp32 run.
    np.testing.assert_allclose(gn, g["grad_norm_f64"], rtol=5e-3)
    np.testing.assert_allclose(gn, g["grad_norm_f32"], rtol=1e-4)


def test_oracle_adam_delta(golden_dir):
    g = _load(golden_dir, "avenet_tiny_b4")
    b, s, f, t = g["shape"].tolist()
    sd = orc.make_state(0, torch.float64)
    sd32 = orc.make_state(0)
    for k in sd:
        if sd[k].is_floating_point():
            sd[k] = sd32[k].double()
    before = {k: v.clone() for k, v in sd.items()}
    orc.train_step(sd, orc.make_image(b, s).double(), orc.make_spectrogram(b, f, t).double(), orc.AdamRef())
    from gen_golden import SLICE_PARAMS, BUF_SLICES
    for n in SLICE_PARAMS:
        d = (sd[n] - before[n]).flatten()[:64].numpy()
        np.testing.assert_allclose(d, g["delta_slice_f64/" + n], rtol=1e-6, atol=1e-13)
    for n in BUF_SLICES:
        np.testing.assert_allclose(sd[n][:16].numpy(), g["buf_f64/" + n], rtol=1e-9, atol=1e-12)


def test_oracle_hardway_attention(golden_dir):
    g = _load(golden_dir, "hardway_attention_tiny")
    b, t, hw, c, seed = g["shape"].tolist()
    vid, aud = orc.make_tube_features(b, t, hw, c, seed)
    np.testing.assert_allclose(checksum(vid), g["vid_checksum"], rtol=1e-12)
    A, logits = orc.hardway_attention(aud, vid)
    np.testing.assert_allclose(logits.numpy(), g["logits_f64"], rtol=1e-12)
    np.testing.assert_allclose(A.numpy(), g["A_f64"], rtol=1e-12)

"""The tube oracle (oracle/tube_oracle.py: R3D-18 + FullModel + train_3D step) against golden
vectors the reference FullModel itself produced (oracle/gen_golden_tube.py). CPU-only."""
import os

import numpy as np
import pytest
import torch

import avenet_oracle as orc
import tube_oracle as tor
from gen_golden import checksum

NAMES = ["fullmodel_tiny_b2t4", "fullmodel_mid_b2t4"]


def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False))


def _inputs(g):
    b, t, size, f, fr = g["shape"].tolist()
    return tor.make_video(b, t, size), orc.make_spectrogram(b, f, fr)


@pytest.mark.parametrize("name", NAMES)
def test_tube_inputs_regenerate(golden_dir, name):
    g = _load(golden_dir, name)
    video, spec = _inputs(g)
    np.testing.assert_allclose(checksum(video), g["video_checksum"], rtol=1e-12)
    np.testing.assert_allclose(checksum(spec), g["spec_checksum"], rtol=1e-12)


def test_repeat_spectrogram_folds_b_major():
    spec = torch.arange(2 * 3 * 4, dtype=torch.float32).view(2, 1, 3, 4)
    r = tor.repeat_spectrogram(spec, 5)
    assert r.shape == (10, 1, 3, 4)
    for i in range(10):  # '(b t)': row i is sample i // t
        assert torch.equal(r[i], spec[i // 5])


@pytest.mark.parametrize("name", NAMES)
def test_tube_oracle_fp64_matches_reference(golden_dir, name):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = _load(golden_dir, name)
    video, spec = _inputs(g)
    sd = tor.make_tube_state(0, torch.float64)
    sd32 = tor.make_tube_state(0)
    for k in sd:  # the reference ran the fp32 weights cast to fp64
        if sd[k].is_floating_point():
            sd[k] = sd32[k].double()
    before = {k: v.clone() for k, v in sd.items()}
    loss, A, logits, grads = tor.tube_train_step(sd, spec.double(), video.double(), orc.AdamRef())
    np.testing.assert_allclose(logits.numpy(), g["logits_f64"], rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(A.numpy(), g["A_f64"], rtol=1e-10, atol=1e-12)
    assert abs(loss.item() - g["loss_f64"].item()) < 1e-10
    names = [str(n) for n in g["param_names"]]
    assert sorted(names) == sorted(tor.trainable_names_tube())
    np.testing.assert_allclose([grads[n].norm().item() for n in names], g["grad_norm_f64"], rtol=1e-9)
    for k in g:
        if k.startswith("delta_slice_f64/"):
            n = k.split("/", 1)[1]
            np.testing.assert_allclose((sd[n] - before[n]).flatten()[:64].numpy(), g[k], rtol=1e-6, atol=1e-13)
        if k.startswith("buf_f64/"):
            n = k.split("/", 1)[1]
            np.testing.assert_allclose(sd[n][:16].numpy(), g[k], rtol=1e-9, atol=1e-12)


def test_tube_oracle_fp32_tolerance(golden_dir):
    g = _load(golden_dir, "fullmodel_tiny_b2t4")
    video, spec = _inputs(g)
    sd = tor.make_tube_state(0)
    audio = tor.repeat_spectrogram(spec, video.shape[2])
    A, logits = tor.fullmodel_forward(sd, audio, video)
    np.testing.assert_allclose(A.numpy(), g["A_f64"], atol=1e-5)
    off = ~np.eye(logits.shape[0], logits.shape[1], k=1, dtype=bool)
    np.testing.assert_allclose(logits.numpy()[off], g["logits_f64"][off], atol=1e-3)


def test_per_clip_audio_is_exact_in_fp64(golden_dir):
    """Running the audio trunk once per clip and repeating its unit vector over the clip's t frames
    gives the folded repeated batch's loss and gradients exactly (fp64): the identity the GPU path's
    per-clip mode (tube.py, avt_repeat_rows_f32 / avt_sum_rep_rows_f32 / avt_bn_finalize_rep) uses."""
    g = _load(golden_dir, "fullmodel_tiny_b2t4")
    video, spec = _inputs(g)
    sd = tor.make_tube_state(0, torch.float64)
    sd_a = {k: v.clone() for k, v in sd.items()}
    loss, _, logits, grads = tor.tube_train_step(sd_a, spec.double(), video.double(), None)
    loss2, logits2, grads2 = tor.tube_train_step_per_clip(sd, spec.double(), video.double())
    assert abs(loss.item() - loss2.item()) < 1e-12
    torch.testing.assert_close(logits2, logits, rtol=1e-12, atol=1e-12)
    for n in grads:
        torch.testing.assert_close(grads2[n], grads[n], rtol=1e-9, atol=1e-14)

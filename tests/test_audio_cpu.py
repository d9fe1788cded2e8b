"""The audio front-end restatement (oracle/audio_oracle.py) against scipy, the reference's own call
(datasets/dataloader.py:94), on CPU."""
import numpy as np
import pytest

import audio_oracle as ao


@pytest.mark.parametrize("n,sr", [(153301, 15330), (160000, 16000), (4000, 8000)])
def test_restated_spectrogram_matches_scipy(n, sr):
    rng = np.random.default_rng(70)
    x = np.clip(0.3 * rng.standard_normal(n), -1, 1)
    x[: n // 5] = 0.25  # constant stretch: detrended segments of exact zeros hit the 1e-7 floor
    ref = ao.reference_spectrogram(x, sr)
    got = ao.restated_spectrogram(x, sr)
    assert ref.shape == got.shape == (1, 257, (n - 512) // 511 + 1)
    np.testing.assert_allclose(got, ref, atol=1e-9, rtol=0)


def test_clip_wave_tiles_and_clips():
    x = np.array([0.5, -2.0, 3.0])
    y = ao.clip_wave(x, 2)
    assert y.shape == (20,) and y.max() == 1.0 and y.min() == -1.0
    np.testing.assert_array_equal(y[:3], [0.5, -1.0, 1.0])

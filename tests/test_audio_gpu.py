"""avt_spectrogram (avt_amd.audio.spectrogram) against scipy.signal.spectrogram + log + Normalize,
the reference dataset's own arithmetic (oracle/audio_oracle.py)."""
import numpy as np
import pytest
import torch

import audio_oracle as ao
from avt_amd.audio import num_segments, spectrogram

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("n,sr", [(153301, 15330), (160000, 16000), (2000, 8000)])
def test_spectrogram_matches_scipy(n, sr):
    rng = np.random.default_rng(71)
    B = 3
    waves = 0.3 * rng.standard_normal((B, n))
    waves[0, : n // 4] = 0.25                        # constant stretch: detrended zeros -> the 1e-7 floor
    waves[1] *= 5.0                                  # clipping at +-1 (dataloader.py:92-93)
    waves[2] = 0.5 * np.sin(2 * np.pi * 440.0 * np.arange(n) / sr) + 1e-3 * rng.standard_normal(n)
    waves = waves.astype(np.float32)                 # 16-bit PCM is exact in fp32
    got = spectrogram(torch.from_numpy(waves).to(DEV), sr).cpu().numpy()
    assert got.shape == (B, 1, 257, num_segments(n))
    for b in range(B):
        ref = ao.reference_spectrogram(np.clip(waves[b].astype(np.float64), -1, 1), sr)
        err = np.abs(got[b] - ref).max()
        print(f"n={n} clip {b}: max |d| = {err:.2e} (normalised log units)")
        assert err < 5e-5, (b, err)


def test_spectrogram_shape_of_the_reference_input():
    """153,301 samples -> 257 x 300: the configuration BASELINE.json quotes."""
    assert num_segments(153301) == 300
    x = torch.zeros(2, 153301, device=DEV)
    out = spectrogram(x, 16000)
    assert out.shape == (2, 1, 257, 300)
    assert torch.allclose(out, torch.full_like(out, float(np.log(np.float32(1e-7)) / 12)), atol=1e-6)

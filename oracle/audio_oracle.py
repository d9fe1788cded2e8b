"""CPU restatement of the reference's audio front end — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module (the checker of ``avt_spectrogram`` / ``avt_amd.audio``).

datasets/dataloader.py:86-96 (and the Flickr subsets at 252-274) compute, per clip,
    resamples = samples[:samplerate*10];  resamples[resamples > 1.] = 1.;  resamples[resamples < -1.] = -1.
    frequencies, times, spectrogram = signal.spectrogram(resamples, samplerate, nperseg=512, noverlap=1)
    spectrogram = np.log(spectrogram + 1e-7)
    spectrogram = transforms.Normalize(mean=[0.0], std=[12.0])(transforms.ToTensor()(spectrogram))
The arithmetic lives in scipy (not vendored; this image pins scipy 1.15.3): ``reference_spectrogram``
calls it exactly as the reference does; ``restated_spectrogram`` restates its published algorithm
(periodic Tukey(0.25) window, per-segment constant detrend, rfft, one-sided density scaling) and is
pinned against scipy in tests/test_audio_cpu.py.  ToTensor of a 2-D float64 array adds the channel
axis; Normalize(0, 12) divides by 12.
"""
from __future__ import annotations

import numpy as np

NPERSEG, NOVERLAP = 512, 1


def clip_wave(samples: np.ndarray, samplerate: int) -> np.ndarray:
    """dataloader.py:86-93: tile to >= 10 s, keep 10 s, clip to [-1, 1]."""
    samples = np.asarray(samples, dtype=np.float64)
    if samples.shape[0] < samplerate * 10:
        n = int(samplerate * 10 / samples.shape[0]) + 1
        samples = np.tile(samples, n)
    resamples = samples[:samplerate * 10].copy()
    resamples[resamples > 1.] = 1.
    resamples[resamples < -1.] = -1.
    return resamples


def reference_spectrogram(resamples: np.ndarray, samplerate: float) -> np.ndarray:
    """The reference's own calls (scipy) on an already clipped waveform -> [1, 257, nseg] float64."""
    from scipy import signal

    _, _, spec = signal.spectrogram(resamples, samplerate, nperseg=NPERSEG, noverlap=NOVERLAP)
    return (np.log(spec + 1e-7) / 12.0)[None]


def tukey_periodic(m: int = NPERSEG, alpha: float = 0.25) -> np.ndarray:
    """scipy.signal.windows.tukey(m, alpha, sym=False)."""
    M = m + 1
    n = np.arange(0, M)
    width = int(np.floor(alpha * (M - 1) / 2.0))
    n1, n2, n3 = n[0:width + 1], n[width + 1:M - width - 1], n[M - width - 1:]
    w1 = 0.5 * (1 + np.cos(np.pi * (-1 + 2.0 * n1 / alpha / (M - 1))))
    w2 = np.ones(n2.shape)
    w3 = 0.5 * (1 + np.cos(np.pi * (-2.0 / alpha + 1 + 2.0 * n3 / alpha / (M - 1))))
    return np.concatenate((w1, w2, w3))[:m]


def restated_spectrogram(resamples: np.ndarray, samplerate: float) -> np.ndarray:
    x = np.asarray(resamples, dtype=np.float64)
    hop = NPERSEG - NOVERLAP
    nseg = (x.shape[0] - NPERSEG) // hop + 1
    idx = np.arange(nseg)[:, None] * hop + np.arange(NPERSEG)[None, :]
    seg = x[idx]
    seg = seg - seg.mean(axis=1, keepdims=True)
    w = tukey_periodic()
    X = np.fft.rfft(seg * w, n=NPERSEG, axis=1)
    p = (X.real ** 2 + X.imag ** 2) / (samplerate * (w * w).sum())
    p[:, 1:-1] *= 2
    return (np.log(p.T + 1e-7) / 12.0)[None]

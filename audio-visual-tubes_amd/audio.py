"""Audio front end of the reference's datasets on libavt.

``GetAudioVideoDataset.__getitem__`` (datasets/dataloader.py:86-96; the Flickr subsets at 252-274)
turns each clip's waveform into the network input on the host with scipy:
    resamples = clip(samples[:sr*10], -1, 1)
    spectrogram = log(scipy.signal.spectrogram(resamples, sr, nperseg=512, noverlap=1)[2] + 1e-7)
    spectrogram = Normalize(mean=[0.0], std=[12.0])(ToTensor()(spectrogram))      # [1, 257, nseg]
``spectrogram(wave, sr)`` does the clip + spectrogram + log + normalisation for a whole batch of
waveforms already on the GPU in one launch (``avt_spectrogram``: per-segment FFT in LDS), so the
audio pipeline no longer bounds the step at 10^4+ clips/s.  Repeating short clips to 10 s
(dataloader.py:88-90) and decoding the files stay with the loader.
"""
from __future__ import annotations

import torch

from ._lib import call, query
from .trunk import P, stream_ptr

NPERSEG = 512
NOVERLAP = 1


def num_segments(n_samples: int, nperseg: int = NPERSEG, noverlap: int = NOVERLAP) -> int:
    return int(query("avt_spectrogram_segments", n_samples, nperseg - noverlap))


def spectrogram(wave: torch.Tensor, sample_rate: float, nperseg: int = NPERSEG,
                noverlap: int = NOVERLAP) -> torch.Tensor:
    """wave [B, N] (or [N]) on the GPU -> [B, 1, 257, nseg] fp32, the dataset's normalised
    log-spectrogram."""
    if not wave.is_cuda:
        raise RuntimeError("avt: spectrogram runs on the GPU (no CPU path)")
    if nperseg != NPERSEG:
        raise ValueError(f"avt: nperseg must be {NPERSEG} (the reference's value)")
    if wave.dim() == 1:
        wave = wave[None]
    if wave.dim() != 2:
        raise ValueError(f"avt: wave must be [B, N], got {tuple(wave.shape)}")
    x = wave.detach().contiguous().float()
    B, N = x.shape
    nseg = num_segments(N, nperseg, noverlap)
    if nseg < 1:
        raise ValueError(f"avt: need at least {nperseg} samples, got {N}")
    out = torch.empty(B, 1, NPERSEG // 2 + 1, nseg, device=x.device, dtype=torch.float32)
    call("avt_spectrogram", P(x), B, N, nperseg - noverlap, float(sample_rate), P(out), stream_ptr())
    return out

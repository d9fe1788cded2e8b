"""Frame front end of the reference's datasets on libavt.

``GetAudioVideoDataset`` (datasets/dataloader.py:47-62, applied at :81) turns each decoded RGB frame
into the network input on the host with PIL + torchvision:
    train: Resize(int(224 * 1.1), BICUBIC) -> RandomCrop(224) -> RandomHorizontalFlip()
           -> CenterCrop(224) -> ToTensor() -> Normalize(mean, std)
    test:  Resize(224, BICUBIC) -> CenterCrop(224) -> ToTensor() -> Normalize(mean, std)
``FrameTransform`` does the same for a whole batch of decoded frames (any sizes) in two launches
(``avt_frames_transform``); its resize is bit-identical to Pillow's, and with the same torch RNG state
it draws the same crops and flips as torchvision (RandomCrop's two ``torch.randint`` then the flip's
``torch.rand``, per frame, in that order; no crop draw when the image already has the crop's size).
JPEG decoding stays with the loader.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import call
from .trunk import P, stream_ptr

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
MAX_DOWNSCALE = 7.5  # <= 32 bicubic taps per output pixel (csrc/frames.hip)


def resized_size(w: int, h: int, size: int) -> tuple[int, int]:
    """torchvision Resize(int) on a PIL image of size (w, h): the short side becomes `size`."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_short, new_long) if w <= h else (new_long, new_short)


class FrameTransform:
    """``img_transform`` of datasets/dataloader.py:47-62 on the GPU: frames (uint8 [H, W, 3] arrays,
    tensors or RGB PIL images) -> float32 [n, 3, S, S] on the device."""

    def __init__(self, image_size: int = 224, mode: str = "train", mean=MEAN, std=STD):
        if mode not in ("train", "test"):
            raise ValueError(f"avt: mode must be 'train' or 'test', got {mode!r}")
        if not 1 <= image_size <= 256:
            raise ValueError("avt: image_size must be in [1, 256]")
        self.size = image_size
        self.mode = mode
        self.resize_to = int(image_size * 1.1) if mode == "train" else image_size
        self._mean = (ctypes.c_float * 3)(*mean)
        self._std = (ctypes.c_float * 3)(*std)

    def params(self, w: int, h: int, generator: torch.Generator | None = None):
        """(resized_w, resized_h, crop_top, crop_left, flip) for a w x h frame; in train mode drawn
        from the torch RNG exactly as RandomCrop + RandomHorizontalFlip draw them."""
        s = self.size
        rw, rh = resized_size(w, h, self.resize_to)
        if rw < s or rh < s:
            raise ValueError(f"avt: resized frame {rw}x{rh} is smaller than the crop {s}")
        if self.mode == "train":
            if rw == s and rh == s:
                ci = cj = 0
            else:
                ci = int(torch.randint(0, rh - s + 1, size=(1,), generator=generator).item())
                cj = int(torch.randint(0, rw - s + 1, size=(1,), generator=generator).item())
            flip = bool(torch.rand(1, generator=generator).item() < 0.5)
        else:  # CenterCrop
            ci, cj, flip = int(round((rh - s) / 2.0)), int(round((rw - s) / 2.0)), False
        return rw, rh, ci, cj, flip

    def __call__(self, frames, params=None, device=None, generator: torch.Generator | None = None) -> torch.Tensor:
        frames = [_as_uint8(f) for f in frames]
        if not frames:
            raise ValueError("avt: no frames")
        device = torch.device(device) if device is not None else (
            frames[0].device if frames[0].is_cuda else torch.device("cuda"))
        if device.type != "cuda":
            raise RuntimeError("avt: the frame transform runs on the GPU (no CPU path)")
        if params is None:
            params = [self.params(f.shape[1], f.shape[0], generator) for f in frames]
        if len(params) != len(frames):
            raise ValueError("avt: one parameter tuple per frame")
        s, n = self.size, len(frames)
        desc = np.zeros((n, 8), dtype=np.int64)
        off = 0
        for i, (f, (rw, rh, ci, cj, flip)) in enumerate(zip(frames, params)):
            H, W = f.shape[0], f.shape[1]
            if not (0 <= ci <= rh - s and 0 <= cj <= rw - s):
                raise ValueError(f"avt: crop ({ci}, {cj}) of {s} outside the {rw}x{rh} resized frame")
            if H / rh > MAX_DOWNSCALE or W / rw > MAX_DOWNSCALE:
                raise ValueError(f"avt: downscale {W}x{H} -> {rw}x{rh} exceeds {MAX_DOWNSCALE}x")
            desc[i] = (off, H, W, rh, rw, ci, cj, int(bool(flip)))
            off += H * W * 3
        hmax = int(desc[:, 1].max())
        src = torch.cat([f.reshape(-1).to(device, non_blocking=True) for f in frames])
        d_desc = torch.from_numpy(desc).to(device)
        tmp = torch.empty(n * 3 * hmax * s, device=device, dtype=torch.uint8)
        out = torch.empty(n, 3, s, s, device=device, dtype=torch.float32)
        with torch.cuda.device(device):
            call("avt_frames_transform", P(src), P(d_desc), n, s, hmax, P(tmp),
                 ctypes.cast(self._mean, ctypes.c_void_p), ctypes.cast(self._std, ctypes.c_void_p), P(out),
                 stream_ptr())
        return out


def _as_uint8(f) -> torch.Tensor:
    if not isinstance(f, (torch.Tensor, np.ndarray)):
        if getattr(f, "mode", "RGB") != "RGB":
            f = f.convert("RGB")
        f = np.asarray(f)
    t = torch.as_tensor(f)
    if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
        raise ValueError(f"avt: frames must be uint8 [H, W, 3], got {t.dtype} {tuple(t.shape)}")
    return t.contiguous()

"""CPU restatement of the reference's frame transform — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module (the checker of ``avt_frames_transform`` /
``avt_amd.frames``).

datasets/dataloader.py:47-62 builds, per frame (a decoded RGB PIL image),
    train: Resize(int(224*1.1), BICUBIC) -> RandomCrop(224) -> RandomHorizontalFlip() -> CenterCrop(224)
           -> ToTensor() -> Normalize(mean, std)
    test:  Resize(224, BICUBIC) -> CenterCrop(224) -> ToTensor() -> Normalize(mean, std)
The arithmetic lives in two dependencies that are not vendored: Pillow (this image pins 12.2.0;
``Image.resize(size, BICUBIC)`` with reducing_gap=None) and torchvision (absent here; its
transforms are restated from their published semantics):

- torchvision Resize(int) on a PIL image: the short side becomes `size`, the long side
  int(size * long / short); an image already of that size is returned unchanged.
- RandomCrop(s): i = torch.randint(0, h - s + 1), then j = torch.randint(0, w - s + 1);
  RandomHorizontalFlip: flip when torch.rand(1) < 0.5 (drawn after the crop's two draws).
- CenterCrop(s): top = int(round((h - s) / 2.0)), left = int(round((w - s) / 2.0)).
- ToTensor: uint8 HWC -> float32 CHW / 255;  Normalize: (x - mean) / std in float32.

``pil_resize_restated`` restates Pillow's separable fixed-point resampler (Resample.c:
precompute_coeffs / normalize_coeffs_8bpc / ImagingResampleHorizontal_8bpc / ..Vertical_8bpc,
PRECISION_BITS = 22, bicubic a = -0.5, horizontal pass first, each pass rounded and clipped to
uint8) and is pinned against Pillow itself in tests/test_frames_cpu.py (bit-exact).
"""
from __future__ import annotations

import numpy as np

PRECISION_BITS = 32 - 8 - 2
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def bicubic_filter(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs(in_size: int, out_size: int):
    """Pillow's precompute_coeffs for box = (0, in_size) + normalize_coeffs_8bpc:
    per output index (xmin, count, int32 fixed-point weights)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    out = []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [bicubic_filter((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        k = [int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS)) for v in w]
        out.append((xmin, xmax, np.array(k, dtype=np.int64)))
    return out


def _clip8(ss: np.ndarray) -> np.ndarray:
    return np.clip(ss >> PRECISION_BITS, 0, 255).astype(np.uint8)


def pil_resize_restated(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """uint8 [H, W, 3] -> uint8 [out_h, out_w, 3], as Image.resize((out_w, out_h), BICUBIC)."""
    img = np.asarray(img, dtype=np.uint8)
    H, W, _ = img.shape
    if (W, H) == (out_w, out_h):
        return img.copy()
    src = img.astype(np.int64)
    tmp = np.empty((H, out_w, 3), dtype=np.uint8)
    for xx, (xmin, cnt, k) in enumerate(precompute_coeffs(W, out_w)):
        ss = (1 << (PRECISION_BITS - 1)) + np.einsum("hxc,x->hc", src[:, xmin:xmin + cnt], k)
        tmp[:, xx] = _clip8(ss)
    t = tmp.astype(np.int64)
    out = np.empty((out_h, out_w, 3), dtype=np.uint8)
    for yy, (ymin, cnt, k) in enumerate(precompute_coeffs(H, out_h)):
        ss = (1 << (PRECISION_BITS - 1)) + np.einsum("yxc,y->xc", t[ymin:ymin + cnt], k)
        out[yy] = _clip8(ss)
    return out


def resized_size(w: int, h: int, size: int) -> tuple[int, int]:
    """torchvision Resize(int) output (w, h) for a PIL image of size (w, h)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_short, new_long) if w <= h else (new_long, new_short)


def center_crop_offsets(w: int, h: int, s: int) -> tuple[int, int]:
    return int(round((h - s) / 2.0)), int(round((w - s) / 2.0))


def to_tensor_normalize(img: np.ndarray) -> np.ndarray:
    """uint8 [s, s, 3] -> float32 [3, s, s]: ToTensor() then Normalize(MEAN, STD)."""
    x = img.astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    mean = np.asarray(MEAN, dtype=np.float32)[:, None, None]
    std = np.asarray(STD, dtype=np.float32)[:, None, None]
    return (x - mean) / std


def frame_transform(img: np.ndarray, rw: int, rh: int, ci: int, cj: int, flip: bool, s: int = 224,
                    resize=pil_resize_restated) -> np.ndarray:
    """Resize to (rw, rh) -> crop s x s at (ci, cj) -> optional horizontal flip -> tensor."""
    r = resize(img, rw, rh)
    c = r[ci:ci + s, cj:cj + s]
    if flip:
        c = c[:, ::-1]
    return to_tensor_normalize(np.ascontiguousarray(c))


def pil_resize(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """Pillow itself (the reference's dependency)."""
    from PIL import Image

    return np.asarray(Image.fromarray(np.asarray(img, dtype=np.uint8), "RGB").resize((out_w, out_h), Image.BICUBIC))

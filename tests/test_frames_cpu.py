"""The frame-transform restatement (oracle/frames_oracle.py) against Pillow, the reference's own
resampler (datasets/dataloader.py:50/58 via torchvision Resize -> PIL Image.resize(BICUBIC)), and the
host-side parameter draws of avt_amd.frames against torchvision's published semantics, on CPU."""
import numpy as np
import pytest
import torch

import frames_oracle as fo
from avt_amd import frames as fr


@pytest.mark.parametrize("H,W,oh,ow", [
    (50, 70, 20, 30), (37, 41, 55, 60),              # down / up
    (480, 640, 246, 328), (300, 500, 246, 410),      # the train Resize(246) of common frame sizes
    (720, 1280, 224, 398), (246, 300, 246, 300),     # test Resize(224); identity
    (224, 300, 246, 328), (64, 64, 64, 97),          # one axis unchanged
    (10, 400, 33, 5),                                # extreme aspect ratios
])
def test_restated_resize_is_pillow(H, W, oh, ow):
    rng = np.random.default_rng(H * 1000 + W)
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    img[: H // 3] = 255                              # saturated band: clipping after both passes
    img[-2:, :, 1] = 0
    np.testing.assert_array_equal(fo.pil_resize_restated(img, ow, oh), fo.pil_resize(img, ow, oh))


def test_resized_size_and_center_crop():
    assert fr.resized_size(640, 480, 246) == fo.resized_size(640, 480, 246) == (328, 246)
    assert fr.resized_size(480, 640, 246) == (246, 328)
    assert fr.resized_size(333, 500, 224) == (224, int(224 * 500 / 333))
    t = fr.FrameTransform(224, "test")
    rw, rh, ci, cj, flip = t.params(500, 333)
    assert (ci, cj) == fo.center_crop_offsets(rw, rh, 224) and not flip


def test_train_params_follow_torchvision_draw_order():
    """RandomCrop: torch.randint(0, h-s+1) then torch.randint(0, w-s+1); RandomHorizontalFlip:
    torch.rand(1) < 0.5 — per frame, on the default generator."""
    t = fr.FrameTransform(224, "train")
    torch.manual_seed(5)
    got = [t.params(w, h) for w, h in [(640, 480), (300, 300), (246, 246)]]
    torch.manual_seed(5)
    exp = []
    for w, h in [(640, 480), (300, 300), (246, 246)]:
        rw, rh = fo.resized_size(w, h, 246)
        i = int(torch.randint(0, rh - 224 + 1, size=(1,)).item())
        j = int(torch.randint(0, rw - 224 + 1, size=(1,)).item())
        exp.append((rw, rh, i, j, bool(torch.rand(1).item() < 0.5)))
    assert got == exp


def test_frame_transform_rejects_cpu_and_bad_frames():
    t = fr.FrameTransform(224, "test")
    with pytest.raises(ValueError):
        t([np.zeros((10, 10), dtype=np.uint8)])
    with pytest.raises((RuntimeError, ValueError)):
        t([np.zeros((300, 300, 3), dtype=np.uint8)], device="cpu")


def test_frame_transform_rejects_excess_downscale_and_bad_crops():
    """Checked on the host before any launch: > 7.5x downscale (the kernel's 32-tap bound) and a crop
    outside the resized frame."""
    t = fr.FrameTransform(32, "train")
    f = np.zeros((300, 400, 3), dtype=np.uint8)
    rw, rh = fr.resized_size(400, 300, 35)
    with pytest.raises(ValueError, match="downscale"):
        t([f], params=[(rw, rh, 0, 0, False)])
    with pytest.raises(ValueError, match="crop"):
        t([f], params=[(rw, rh, rh - 31, 0, False)])

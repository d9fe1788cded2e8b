"""Throughput of the on-device frame front end (avt_frames_transform, datasets/dataloader.py:47-62) on a
batch of decoded 480x640 RGB frames already in HBM: train transform (Resize(246) BICUBIC -> RandomCrop(224)
-> flip -> Normalize).  Times the two-launch kernel pair alone (HIP events) and the whole
FrameTransform call (host descriptor build + packing the frames into one buffer + the launches)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import avtubes  # noqa: E402,F401
from avt_amd._lib import call  # noqa: E402
from avt_amd.frames import FrameTransform  # noqa: E402
from avt_amd.trunk import P, stream_ptr  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
H, W, S = 480, 640, 224
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(7)
frames = [torch.randint(0, 256, (H, W, 3), device=dev, dtype=torch.uint8, generator=g) for _ in range(B)]
t = FrameTransform(S, "train")
torch.manual_seed(8)
params = [t.params(W, H) for _ in range(B)]
desc = np.array([(i * H * W * 3, H, W, rh, rw, ci, cj, int(fl)) for i, (rw, rh, ci, cj, fl) in enumerate(params)],
                dtype=np.int64)
src = torch.stack(frames).reshape(-1)
d_desc = torch.from_numpy(desc).to(dev)
tmp = torch.empty(B * 3 * H * S, device=dev, dtype=torch.uint8)
out = torch.empty(B, 3, S, S, device=dev)
mean, std = (ctypes.c_float * 3)(0.485, 0.456, 0.406), (ctypes.c_float * 3)(0.229, 0.224, 0.225)


def kernels():
    call("avt_frames_transform", P(src), P(d_desc), B, S, H, P(tmp), ctypes.cast(mean, ctypes.c_void_p),
         ctypes.cast(std, ctypes.c_void_p), P(out), stream_ptr())


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ms_k = timed(kernels)
ref = out.clone()
ms_call = timed(lambda: t(frames, params=params))
assert torch.equal(t(frames, params=params), ref)
# algorithmic bytes: the source rows/columns the crop's taps read (~ crop/resized of each axis) once,
# the planar uint8 intermediate written and read, the fp32 output written
rw, rh = params[0][0], params[0][1]
src_b = B * 3 * (H * S / rh) * (W * S / rw)
nbytes = src_b + 2 * B * 3 * H * S + out.numel() * 4
print(json.dumps({"kernel": "avt_frames_transform", "frames": B, "src": f"{H}x{W}", "crop": S, "ms": round(ms_k, 4),
                  "frames_per_s": round(B / ms_k * 1e3, 1), "hbm_GBps": round(nbytes / ms_k / 1e6, 1),
                  "hbm_frac": round(nbytes / ms_k / 1e6 / 8000, 4), "call_ms": round(ms_call, 4),
                  "call_frames_per_s": round(B / ms_call * 1e3, 1)}))

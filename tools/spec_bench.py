"""Throughput of the on-device audio front end (avt_spectrogram) at the BASELINE shape (HIP events)."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import avtubes  # noqa: E402,F401
from avt_amd.audio import spectrogram  # noqa: E402

B, N, SR = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 153301, 16000
x = torch.randn(B, N, device="cuda") * 0.1
for _ in range(3):
    spectrogram(x, SR)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
e0.record()
for _ in range(reps):
    y = spectrogram(x, SR)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
nbytes = x.numel() * 4 + y.numel() * 4
print(json.dumps({"kernel": "avt_spectrogram", "batch": B, "samples": N, "ms": round(ms, 4),
                  "clips_per_s": round(B / ms * 1e3, 1), "hbm_GBps": round(nbytes / ms / 1e6, 1),
                  "hbm_frac": round(nbytes / ms / 1e6 / 8000, 4)}))

"""Which gradients differ between identical runs of the fused train step (determinism diagnostic): three runs of
three steps from the same weights on the same inputs; prints the parameters whose step-3 gradients differ.
usage: python tools/diag_det2.py   (AVT_CONCURRENT=0: one stream)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import avtubes  # noqa: E402,F401
import avenet_oracle as orc  # noqa: E402
from avt_amd.model import AVENet, HardWayArgs  # noqa: E402
from avt_amd.train import HardWayTrainStep  # noqa: E402

DEV = torch.device("cuda")
# DET_KEEP=1: keep every tensor a step allocates alive until the step has synchronised (no allocator reuse
# inside a step: isolates cross-stream reuse of freed blocks)
if os.environ.get("DET_KEEP"):
    _keep = []
    for _name in ("empty", "empty_like", "zeros", "zeros_like", "full"):
        _orig = getattr(torch, _name)

        def _wrap(*a, _o=_orig, **k):
            t = _o(*a, **k)
            _keep.append(t)
            return t
        setattr(torch, _name, _wrap)
_B = int(os.environ.get("DET_B", "6"))
if os.environ.get("DET_FULL"):  # the bench's input sizes (224 x 224 frames, 257 x 300 spectrograms)
    img, aud = orc.make_image(_B, 224).to(DEV), orc.make_spectrogram(_B, 257, 300).to(DEV)
else:
    img, aud = orc.make_image(_B, 96).to(DEV), orc.make_spectrogram(_B, 97, 110).to(DEV)
runs = []
NR = int(os.environ.get("DET_RUNS", "3"))
for r in range(NR):
    m = AVENet(HardWayArgs(), False)
    m.load_state_dict(orc.make_state(3))
    m = m.to(DEV).train()
    step = HardWayTrainStep(m, lr=1e-4, weight_decay=1e-4)
    per_step = []
    for _ in range(3):
        loss = step.step(img, aud).item()
        torch.cuda.synchronize()
        if os.environ.get("DET_KEEP"):
            _keep.clear()
        per_step.append((loss, step.grad.clone()))
    runs.append((m, per_step))
m0 = runs[0][0]
for s in range(3):
    g0 = runs[0][1][s][1]
    for r in range(1, NR):
        g = runs[r][1][s][1]
        if torch.equal(g, g0):
            print(f"step {s} run {r}: equal (loss {runs[r][1][s][0]} vs {runs[0][1][s][0]})", flush=True)
            continue
        v0, v = m0._flat.grad_views(g0), m0._flat.grad_views(g)
        bad = [(n, (v[n] - v0[n]).abs().max().item()) for n in v0 if not torch.equal(v[n], v0[n])]
        print(f"step {s} run {r}: {len(bad)} of {len(v0)} tensors differ; loss {runs[r][1][s][0]} vs "
              f"{runs[0][1][s][0]}", flush=True)
        for n, d in bad[-3:] if os.environ.get("DET_SHORT") else bad[:40]:
            print(f"   {n:50s} max|d| {d:.3e}", flush=True)

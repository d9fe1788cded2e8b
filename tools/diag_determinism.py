"""Run-to-run gradient spread of the fused and drop-in paths (diagnostic)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import avtubes  # noqa: E402,F401
import avenet_oracle as orc  # noqa: E402
from avt_amd.model import AVENet  # noqa: E402
from avt_amd.train import HardWayTrainStep, TwoViewTrainStep  # noqa: E402

DEV = torch.device("cuda")


def model():
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    return m.to(DEV).train()


def fused1(img, aud):
    m = model()
    s = HardWayTrainStep(m)
    s.opt.lr = 0.0
    s.step(img, aud)
    return s.grad.clone()


def dropin1(img, aud):
    m = model()
    _, lg, _, _, _ = m(img, aud)
    torch.nn.CrossEntropyLoss()(lg, torch.zeros(lg.shape[0], dtype=torch.long, device=DEV)).backward()
    g = torch.zeros(m._flat.n_train, device=DEV)
    views = m._flat.grad_views(g)
    for n, p in m.named_parameters():
        if n in views and p.grad is not None:
            views[n].copy_(p.grad.permute(0, 2, 3, 1) if p.grad.dim() == 4 else p.grad)
    return g


def fused2(fr, au, sp, dedup):
    m = model()
    s = TwoViewTrainStep(m, dedup_audio=dedup)
    s.opt.lr = 0.0
    s.step(fr, au, sp)
    return s.grad.clone()


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


img, aud = orc.make_image(4, 64).to(DEV), orc.make_spectrogram(4, 65, 76).to(DEV)
a, b = fused1(img, aud), fused1(img, aud)
c, d = dropin1(img, aud), dropin1(img, aud)
print("1-frame fused vs fused", rel(a, b), "dropin vs dropin", rel(c, d), "fused vs dropin", rel(a, c))
fr, au, sp = orc.make_frames(2, 3, 64, 3).to(DEV), orc.make_frames(2, 3, 64, 4).to(DEV), orc.make_spectrogram(2, 65, 76).to(DEV)
e, f = fused2(fr, au, sp, False), fused2(fr, au, sp, False)
h = fused2(fr, au, sp, True)
print("two-view fused vs fused", rel(e, f), "dedup vs folded", rel(h, e))

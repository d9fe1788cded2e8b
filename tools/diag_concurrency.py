"""Concurrent (audio trunk on a side stream) vs sequential train steps: losses over several steps."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import avtubes  # noqa: E402,F401
import avenet_oracle as orc  # noqa: E402
from avt_amd.model import AVENet  # noqa: E402
from avt_amd.train import HardWayTrainStep  # noqa: E402

DEV = torch.device("cuda")


def run(conc, graph, steps=6, B=2):
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    m = m.to(DEV).train()
    s = HardWayTrainStep(m, lr=1e-6)
    s.engine.concurrent = conc
    img, aud = orc.make_image(B, 64).to(DEV), orc.make_spectrogram(B, 65, 76).to(DEV)
    out = []
    for i in range(steps):
        out.append(round(s.step(img, aud).item(), 6))
        if graph and i == 0:
            s.capture(img.clone(), aud.clone())
    return out


for conc, graph in [(False, False), (True, False), (True, False), (False, True), (True, True)]:
    print("concurrent", conc, "graph", graph, run(conc, graph))


def run_two_shards(conc, steps=4):
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    m = m.to(DEV).train()
    ref = HardWayTrainStep(m, lr=1e-6)
    ref.engine.concurrent = conc
    img, aud = orc.make_image(4, 64), orc.make_spectrogram(4, 65, 76)
    shards = [(img[r * 2:(r + 1) * 2].to(DEV), aud[r * 2:(r + 1) * 2].to(DEV)) for r in range(2)]
    out = [[], []]
    for _ in range(steps):
        gsum = torch.zeros_like(ref.grad)
        for r, (i, a) in enumerate(shards):
            out[r].append(round(ref._fwd_bwd(i, a).item(), 6))
            gsum += ref.grad
        ref.opt.step(gsum, grad_scale=0.5)
    return out


for conc in (False, True, True):
    print("two shards concurrent", conc, run_two_shards(conc))

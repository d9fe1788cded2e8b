"""Segment-graph replay (HardWayTrainStep's world > 1 path: one HIP graph per backward segment) vs
eager, on one process with the collectives stubbed out: relative gradient difference per bucket.
This is how the hipMemsetAsync-node race in the head backward was found (garbage audio gradients
in about half of the replays); keep it as a regression check of the segmented capture."""
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


def seg_vs_eager(B=2, seed=0):
    dev = torch.device("cuda", 0)
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(seed))
    m = m.to(dev).train()
    step = HardWayTrainStep(m, lr=1e-6, weight_decay=1e-4)
    step.world, step.overlap = 2, True  # take the segmented-capture path (two streams); collectives are no-ops
    step._allreduce_bucket = lambda tag, works: None
    img, aud = orc.make_image(B, 64).to(dev), orc.make_spectrogram(B, 65, 76).to(dev)
    for _ in range(2):
        step.step(img, aud)
    torch.cuda.synchronize()
    snap = (m._flat.flat.clone(), m._flat.bflat.clone(), step.opt.exp_avg.clone(), step.opt.exp_avg_sq.clone(),
            step.opt.t_dev.clone())
    step.capture(img.clone(), aud.clone())
    step.step(img, aud)
    torch.cuda.synchronize()
    g_rep = step.grad.clone()
    m._flat.flat.copy_(snap[0])
    m._flat.bflat.copy_(snap[1])
    step.opt.exp_avg.copy_(snap[2])
    step.opt.exp_avg_sq.copy_(snap[3])
    step.opt.t_dev.copy_(snap[4])
    step._seg_graphs, step._graph_opt, step._graph = None, None, None
    step.step(img, aud)
    torch.cuda.synchronize()
    g_eag = step.grad
    return {tag: ((g_rep[lo:hi].double() - g_eag[lo:hi].double()).norm() / g_eag[lo:hi].double().norm()).item()
            for tag, (lo, hi) in step.buckets.items()}


if __name__ == "__main__":
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        print(seg_vs_eager(), flush=True)

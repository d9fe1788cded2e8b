"""Step schedules that must not change the result (world 1): each trunk's weight packing at the head of its
own branch with the dgrad packs behind the vision forward (AVEngine.split_pack), and Adam in two parts --
each trunk's region at the end of its backward branch, the rest after the join (HardWayTrainStep.
adam_branch) -- against one batched pack before the fork and one Adam launch after the backward; eager
and as one captured HIP graph.  Parameters agree to what the gradient's run-to-run spread (fp64 BN
statistic atomics) can move in one step (<= ~lr)."""
import pytest
import torch

import avenet_oracle as orc

pytestmark = pytest.mark.gpu
B, S, F, T = 4, 64, 65, 76


def _step(split: bool, graph: bool):
    from avt_amd.model import AVENet
    from avt_amd.train import HardWayTrainStep

    dev = torch.device("cuda", 0)
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    m = m.to(dev).train()
    step = HardWayTrainStep(m, lr=1e-6, weight_decay=1e-4)
    step.engine.split_pack = split
    step.adam_branch = split
    img, aud = orc.make_image(B, S).to(dev), orc.make_spectrogram(B, F, T).to(dev)
    state = (m._flat.flat, m._flat.bflat, step.opt.exp_avg, step.opt.exp_avg_sq, step.opt.t_dev)
    p0 = m._flat.flat.clone()
    if graph:
        snap = [t.clone() for t in state]
        step.step(img, aud)  # eager first (the engine allocates lazily), then capture
        torch.cuda.synchronize()
        step.capture(img.clone(), aud.clone())
        for dst, src in zip(state, snap):
            dst.copy_(src)
    step.step(img, aud)
    step.step(img, aud)
    torch.cuda.synchronize()
    return p0, m._flat.flat.clone(), step.opt.t_dev.item(), step.buckets


@pytest.mark.parametrize("graph", [False, True])
def test_split_pack_and_branch_adam_match(graph):
    p0, ref, t_ref, buckets = _step(False, graph)
    _, got, t_got, _ = _step(True, graph)
    assert t_got == t_ref
    d = (got - ref).abs().max().item()
    print(f"max |dparam| split schedule vs batched = {d:.3e}")
    assert d <= 2 * 2.1e-6, d
    for tag, (lo, hi) in buckets.items():  # every region was updated
        assert (got[lo:hi] - p0[lo:hi]).abs().max().item() > 0, tag

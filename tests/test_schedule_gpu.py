"""Step schedules that must not change the result: the weight-gradient launches forked onto their own
streams (AVEngine.wgrad_streams: 1 shared, 2 one per trunk) against the inline schedule, eager and as
captured HIP graphs (one graph at world 1; the per-segment graphs of the world > 1 path with the
collectives stubbed out).  The fused step's gradient per bucket (train.py) must match the inline
eager gradient to the run-to-run spread of the fp64 statistic atomics (~1e-7)."""
import pytest
import torch

import avenet_oracle as orc

pytestmark = pytest.mark.gpu
B, S, F, T = 4, 64, 65, 76


def _grads(nws: int, graph: bool, segmented: bool, adam_overlap: bool = True):
    from avt_amd.model import AVENet
    from avt_amd.train import HardWayTrainStep

    dev = torch.device("cuda", 0)
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    m = m.to(dev).train()
    step = HardWayTrainStep(m, lr=1e-6, weight_decay=1e-4)
    step.engine.wgrad_streams = nws
    step.adam_overlap = adam_overlap  # (world 1 only: the segmented world-2 path below never takes it)
    if segmented:
        step.world, step.overlap = 2, True  # the segmented path; the collectives are no-ops
        step._allreduce_bucket = lambda tags, works: None
    img, aud = orc.make_image(B, S).to(dev), orc.make_spectrogram(B, F, T).to(dev)
    if graph:
        state = (m._flat.flat, m._flat.bflat, step.opt.exp_avg, step.opt.exp_avg_sq, step.opt.t_dev)
        snap = [t.clone() for t in state]
        step.step(img, aud)  # eager first (the engine allocates lazily), then capture
        torch.cuda.synchronize()
        step.capture(img.clone(), aud.clone())
        for dst, src in zip(state, snap):
            dst.copy_(src)
    step.step(img, aud)  # eager, or the first replay from the same state
    torch.cuda.synchronize()
    return step.grad.clone(), step.buckets, m._flat.flat.clone()


@pytest.mark.parametrize("nws,graph,segmented", [(2, False, False), (1, True, False), (2, True, False),
                                                 (2, True, True)])
def test_wgrad_streams_match_inline(nws, graph, segmented):
    g0, buckets, _ = _grads(0, False, False)
    g1, _, _ = _grads(nws, graph, segmented)
    assert torch.isfinite(g1).all()
    rel = {tag: ((g1[lo:hi].double() - g0[lo:hi].double()).norm() / g0[lo:hi].double().norm()).item()
           for tag, (lo, hi) in buckets.items()}
    print(rel)
    assert all(v < 1e-5 for v in rel.values()), rel


@pytest.mark.parametrize("graph", [False, True])
def test_overlapped_adam_matches_one_launch(graph):
    """World 1: Adam on each trunk's layer3+4 region forked during the backward (+ the rest after it)
    vs one Adam launch after the backward: the same update, so the parameters agree to what the
    gradient's run-to-run spread can move in one step (<= ~lr)."""
    from avt_amd.model import AVENet

    g0, buckets, p0 = _grads(0, graph, False, adam_overlap=False)
    g1, _, p1 = _grads(2, graph, False, adam_overlap=True)
    d = (p1 - p0).abs().max().item()
    print(f"max |dparam| overlap vs one launch = {d:.3e}")
    assert d <= 2.1e-6, d
    m = AVENet(orc.Args(), False)
    m.load_state_dict(orc.make_state(0))
    p_init = m.to(p1.device)._flat.flat
    for tag, (lo, hi) in buckets.items():  # every region was updated
        assert (p1[lo:hi] - p_init[lo:hi]).abs().max().item() > 0, tag

"""Time the world > 1 step schedule on ONE GPU without communication: HardWayTrainStep with world = 2 forced and the
collectives stubbed (an all-reduce that is already complete, no buffer broadcast), so what is measured is the
schedule itself -- the backward in two captured segment graphs, the bucket boundaries, the "hi" buckets' Adam on the
side stream between the replays, the join -- against the world-1 step (one graph) on the same box.  Gradients are
not averaged (the stub leaves them), so the losses follow the world-1 ones; timing only.
usage: python tools/dp_sched_time.py --batch 32 --steps 30 --warmup 5"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


class _Done:
    def wait(self):
        return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import bench
    import avtubes  # noqa: F401
    import avt_amd.train as train
    from avt_amd.model import AVENet, HardWayArgs
    from avt_amd.train import HardWayTrainStep

    train.dist.all_reduce = lambda t, op=None, group=None, async_op=False: _Done() if async_op else None
    train.sync_buffers = lambda bflat, pg=None: None
    dev = torch.device("cuda", 0)
    inputs = bench.synthetic_inputs(args.batch, dev, seed=1000)
    for mode in ("world1", "world2-schedule", "world1", "world2-schedule"):
        torch.manual_seed(0)
        model = AVENet(HardWayArgs(), False).to(dev).train()
        step = HardWayTrainStep(model, lr=1e-6, weight_decay=1e-4)
        if mode != "world1":
            step.world, step.overlap, step.adam_branch = 2, True, False
        for i in range(max(args.warmup, 1)):
            step.step(*inputs)
            if i == 0:
                step.capture(*inputs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step.step(*inputs)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        segs = len(step._seg_graphs) if step._seg_graphs is not None else 0
        print(f"B={args.batch} {mode:16s} {ms:.3f} ms/step {args.batch * 1e3 / ms:.1f} clips/s segments {segs} "
              f"loss {float(loss.flatten()[0]):.4f}", flush=True)


if __name__ == "__main__":
    main()

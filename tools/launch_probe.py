"""Host-side cost of a step's HIP-graph replay: how long graph.replay() takes to return (the host
enqueue of every node) against the GPU time of the step.  If the two are close, the step is bound
by the graph launch, not by its kernels.  usage: python tools/launch_probe.py [--batch 32] [--reps 10]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import bench
    import avtubes  # noqa: F401
    from avt_amd.model import AVENet, HardWayArgs
    from avt_amd.train import HardWayTrainStep

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = AVENet(HardWayArgs(), False).to(dev).train()
    inputs = bench.synthetic_inputs(args.batch, dev, seed=1000)
    step = HardWayTrainStep(model, lr=1e-6, weight_decay=1e-4)
    step.step(*inputs)
    step.capture(*inputs)
    for _ in range(3):
        step.step(*inputs)
    torch.cuda.synchronize()
    g = step._graph
    enq, tot = [], []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    # back-to-back: host runs ahead, so the per-step time is max(host enqueue, GPU)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(f"B={args.batch}: single replay: host enqueue {med(enq):.3f} ms, enqueue+run {med(tot):.3f} ms; "
          f"{args.reps} back-to-back: host {(t1 - t0) * 1e3 / args.reps:.3f} ms/step, "
          f"total {(t2 - t0) * 1e3 / args.reps:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()

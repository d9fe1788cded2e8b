"""Host cost of a captured train-step replay (diagnostic): the host time of one step() call on an idle GPU,
then per-call host times of back-to-back calls, and the GPU time per step.
usage: python tools/replay_probe.py [--batch B]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
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
    for i in range(4):
        step.step(*inputs)
        if i == 0:
            step.capture(*inputs)
    torch.cuda.synchronize()
    idle = []
    for _ in range(5):  # one call on an idle GPU
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        step.step(*inputs)
        idle.append((time.perf_counter() - h0) * 1e3)
        torch.cuda.synchronize()
    per = []
    t0 = time.perf_counter()
    for _ in range(20):
        h0 = time.perf_counter()
        step.step(*inputs)
        per.append((time.perf_counter() - h0) * 1e3)
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) * 1e3 / 20
    g = step._graph
    print(f"B={args.batch}: idle-GPU call {min(idle):.3f}-{max(idle):.3f} ms; back-to-back calls "
          f"{' '.join(f'{x:.2f}' for x in per)} ms; {gpu:.3f} ms/step", flush=True)
    if g is not None:
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        g.replay()
        h1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"bare graph.replay(): host {1e3 * (h1 - h0):.3f} ms, to completion {1e3 * (time.perf_counter() - h0):.3f} ms")


if __name__ == "__main__":
    main()

"""Step timer for timing DIAGNOSTICS that bench.py refuses (wrong-results knobs such as AVT_DIAG_H1_SKIP):
the 1-frame train step on synthetic inputs, captured as bench.py does, K timed replays.  Prints one line.
usage: AVT_DIAG_H1_SKIP=1 AVT_DIAG_WRONG_RESULTS_OK=1 python tools/step_time.py --batch 128 --steps 20 --warmup 5"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
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
    for i in range(max(args.warmup, 1)):
        step.step(*inputs)
        if i == 0:
            step.capture(*inputs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        h0 = time.perf_counter()
        loss = step.step(*inputs)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    print(f"host time per step() call (graph replay issue): {host * 1e3 / args.steps:.3f} ms", flush=True)
    knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("AVT_"))
    print(f"B={args.batch} {ms:.3f} ms/step {args.batch * 1e3 / ms:.1f} clips/s loss {float(loss.flatten()[0]):.4f} "
          f"[{knobs}]", flush=True)


if __name__ == "__main__":
    main()

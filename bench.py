"""Train-step clips/s of the 1-frame audio-visual hard-way step (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]
    (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

Workload (BASELINE.json configs[1]): per GPU B=128 clips of one 224x224 RGB frame + one 257x300
log-spectrogram; ResNet-18 vision + ResNet-18 audio trunks (bf16 MFMA, fp32 statistics), fp32
hard-way head + CE, backward, Adam (lr 1e-6, wd 1e-4); N GPUs = weak scaling with local
negatives and one RCCL all-reduce of the 89.4 MB fp32 gradient per step.  Inputs are synthetic
and already resident in HBM when the timed region starts; weights are random-init (no checkpoints).

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel family (the implicit-GEMM
convolutions: fwd + dgrad + wgrad), measured live with HIP events around every conv launch inside
the timed steps: achieved = algorithmic conv FLOPs / summed kernel time.  `cpu_baseline` times the
oracle's fp32 PyTorch-CPU restatement of the same step (B=2) on the host cores (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

GFLOP_PER_CLIP = 46.87  # fwd 15.74 + bwd 31.12 (torch.utils.flop_counter on the reference)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def synthetic_inputs(B, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    img = torch.randn(B, 3, 224, 224, device=device, generator=g)
    spec = (torch.randn(B, 1, 257, 300, device=device, generator=g) * 0.08 - 1.16).clamp_(-1.35, -0.6)
    return img, spec


TRAFFIC_FILE = os.path.join(REPO, "profiles", "conv_traffic_b128.json")


def conv_traffic(launches_per_step, B, world):
    """HBM bytes per conv launch from the committed PMC summary (tools/pmc_traffic.sh ->
    tools/traffic_summary.py --json) of this same workload; None if absent or for another batch."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if t.get("per_gpu_batch") != B or launches_per_step <= 0:
        return None, None
    per_step = t["conv_read_bytes_per_step"] + t["conv_write_bytes_per_step"]
    return round(per_step / launches_per_step), os.path.relpath(TRAFFIC_FILE, REPO)


def cpu_baseline(budget_s: float = 20.0):
    """Oracle (fp32 PyTorch CPU restatement) full train step at B=2 on the host cores."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import avenet_oracle as orc

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    torch.set_num_threads(cores)
    B = 2
    sd = orc.make_state(0)
    img, aud = orc.make_image(B), orc.make_spectrogram(B)
    opt = orc.AdamRef()
    orc.train_step(sd, img, aud, opt)  # warm-up
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        orc.train_step(sd, img, aud, opt)
        times.append(time.perf_counter() - t0)
        if len(times) >= 50:
            break
    times.sort()
    med = times[len(times) // 2]
    return {"value": B / med, "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"oracle fp32 full train step (fwd+CE+bwd+Adam), B=2, 224^2 + 257x300, median of {len(times)}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="clips per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-graph", action="store_true", help="launch every kernel eagerly instead of replaying a "
                    "captured HIP graph of the step")
    ap.add_argument("--prof-steps", type=int, default=2, help="eager steps with HIP events around every conv "
                    "launch after the timed region (roofline)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import avtubes  # noqa: F401
    from avt_amd.model import AVENet
    from avt_amd.train import HardWayTrainStep
    from avt_amd.trunk import ConvProfiler

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import avenet_oracle as orc

    torch.manual_seed(0)
    model = AVENet(orc.Args(), False).to(dev).train()
    step = HardWayTrainStep(model, lr=1e-6, weight_decay=1e-4)
    B = args.batch
    img, aud = synthetic_inputs(B, dev, seed=1000 + rank)

    use_graph = not args.no_graph
    for i in range(max(args.warmup, 1 if use_graph else 0)):
        loss = step.step(img, aud)
        if use_graph and i == 0:
            step.capture(img, aud)  # later warm-up and all timed steps are graph replays
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step.step(img, aud)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    loss_v = float(loss)
    # roofline of the conv family: HIP events on the launch stream around every conv launch of a
    # few eager steps of the same workload (kept out of the timed region above)
    eager = HardWayTrainStep.__new__(HardWayTrainStep)
    eager.__dict__.update(step.__dict__)
    eager._graph = None
    with ConvProfiler() as prof:
        for _ in range(args.prof_steps):
            eager.step(img, aud)
        torch.cuda.synchronize()
    conv = prof.summary()
    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = el.item()
    if rank == 0:
        clips = B * world * args.steps
        value = clips / elapsed
        fl = sum(v[1] for v in conv.values())
        ms = sum(v[2] for v in conv.values())
        n_launch = sum(v[0] for v in conv.values())
        alg_bytes = sum(v[3] for v in conv.values())
        achieved = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        traffic, traffic_src = conv_traffic(n_launch / max(args.prof_steps, 1), B, world)
        rec = {
            "metric": "train-step clips/sec (whole node), ResNet18 vision + ResNet18 audio hard-way loss",
            "value": round(value, 2),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded N(0,1) frames, clipped N(-1.16,0.08^2) log-spectrograms; random-init weights)",
            "config": {"workload": "train_hardway_1frame step: 224x224 RGB + 257x300 spectrogram, fwd+CE+bwd+Adam",
                       "global_batch": B * world, "per_gpu_batch": B, "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "kernel": "conv implicit-GEMM (fwd+dgrad+wgrad)",
                         "achieved": round(achieved, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                         "traffic_unit": "HBM bytes per conv launch (PMC FETCH_SIZE/WRITE_SIZE, gfx950-corrected)",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": round(alg_bytes / max(n_launch, 1)),
                         "algorithmic_flops_per_launch": round(fl / max(n_launch, 1)),
                         "launches": n_launch,
                         "per_kind": {k: {"launches": v[0], "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2),
                                          "ms_per_step": round(v[2] / max(args.prof_steps, 1), 3)} for k, v in conv.items()},
                         "conv_ms_per_step": round(ms / max(args.prof_steps, 1), 3),
                         "measured": f"HIP events around each conv launch, {args.prof_steps} eager steps after the "
                                     "timed region"},
            "launch": "eager" if args.no_graph else "hip-graph replay",
            "step_tflops_per_gpu": round(value / world * GFLOP_PER_CLIP / 1e3, 2),
            "step_mfma_frac": round(value / world * GFLOP_PER_CLIP / 1e3 / MFMA_BF16_PEAK_TFLOPS, 4),
            "loss": round(loss_v, 6),
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_budget)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

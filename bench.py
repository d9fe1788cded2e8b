"""Train-step clips/s of the audio-visual hard-way step (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload 1frame|tube|twoview]
                    [--no-cpu-baseline]
    (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

Default workload: N=1 runs BASELINE.json configs[1], the headline: B=128 clips of one 224x224 RGB
frame + one 257x300 log-spectrogram; ResNet-18 vision + ResNet-18 audio trunks (bf16 MFMA, fp32
statistics), fp32 hard-way head + CE, backward, Adam (lr 1e-6, wd 1e-4).  N>1 runs configs[2]: a
global batch of 256 clips sharded over the N GPUs (256/N per GPU, 32 at N=8; strong scaling), local
negatives per rank as nn.DataParallel gives them, and the 89.4 MB fp32 gradient all-reduced over
RCCL in buckets overlapped with the backward.  --batch B fixes the per-GPU batch instead (weak
scaling at B per GPU).

--workload tube (configs[3], train_3D.py): per GPU b=8 clips of 16x224x224 frames + one 257x300
spectrogram each; R3D-18 forward (detached, as the reference's hook) + audio ResNet-18 fwd/bwd over
the 16-fold repeated spectrogram (run once per clip unless --tube-folded: exact, tube.py) + the
hard-way head over the (b t) = 128 rows + CE + Adam.

--workload twoview (train_hardway.py, the 16-frame two-view step): per GPU b=8 clips of 16x224x224
frames in two views (frames, augmented) + one 257x300 spectrogram each; two AVENet forwards over the
(b t) = 128 frames of each view, 0.1*CE x2 + 99.9*MSE(weighted_A) + PropagationLoss x2, backward,
Adam (lr 4e-6).  The audio trunk runs once per clip for both views unless --twoview-folded (exact:
twoview.py); a clip counts once however many frames/views it has.

Inputs are synthetic and already resident in HBM when the timed region starts; weights are
random-init (no checkpoints).  Prints ONE JSON line on rank 0.  `roofline` is for the dominant
kernel family (the implicit-GEMM convolutions), measured live with HIP events around every conv
launch of eager steps run right after the timed region: achieved = algorithmic conv FLOPs / summed
kernel time; `traffic` = PMC-measured HBM bytes per conv launch from the committed profile of the
same workload (tools/pmc_traffic.sh).  `cpu_baseline` times the oracle's fp32 PyTorch-CPU
restatement of the same step on the host cores (rank 0, N=1 only).
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

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0

METRIC = "train-step clips/sec (whole node), ResNet18+VGG-M hard-way loss at 1/2/4/8 GPU"
DATA = "synthetic (seeded N(0,1) frames, clipped N(-1.16,0.08^2) log-spectrograms; random-init weights)"


def synthetic_inputs(B, device, seed, frames=0):
    g = torch.Generator(device=device).manual_seed(seed)
    if frames:
        img = torch.randn(B, 3, frames, 224, 224, device=device, generator=g)
    else:
        img = torch.randn(B, 3, 224, 224, device=device, generator=g)
    spec = (torch.randn(B, 1, 257, 300, device=device, generator=g) * 0.08 - 1.16).clamp_(-1.35, -0.6)
    return img, spec


def traffic_file(workload, B):
    tag = {"1frame": "b", "tube": "tube_b", "twoview": "twoview_b"}[workload]
    return os.path.join(REPO, "profiles", f"conv_traffic_{tag}{B}.json")


def conv_traffic(path, launches_per_step, B):
    """HBM bytes per conv launch from the committed PMC summary (tools/pmc_traffic.sh ->
    tools/traffic_summary.py --json) of this same workload; None if absent or for another batch."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if t.get("per_gpu_batch") != B or launches_per_step <= 0:
        return None, None
    per_step = t["conv_read_bytes_per_step"] + t["conv_write_bytes_per_step"]
    return round(per_step / launches_per_step), os.path.relpath(path, REPO)


def _cores():
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def _time_loop(fn, budget_s, max_n=50, warmup=3):
    """Median wall time of fn() after `warmup` untimed runs (>= 3 warm-ups, median)."""
    for _ in range(warmup):
        fn()
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        if len(times) >= max_n:
            break
    times.sort()
    return times[len(times) // 2], len(times)


def cpu_baseline(workload: str, budget_s: float = 20.0):
    """The oracle (fp32 PyTorch-CPU restatement) of the same step on the host cores."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import avenet_oracle as orc

    cores = _cores()
    torch.set_num_threads(cores)
    cpu = _cpu_model()
    if workload == "twoview":
        t = 16
        sd = orc.make_state(0)
        fr, au, sp = orc.make_frames(1, t, 224, seed=3), orc.make_frames(1, t, 224, seed=4), orc.make_spectrogram(1)
        opt = orc.AdamRef(lr=4e-6)
        med, n = _time_loop(lambda: orc.twoview_step(sd, fr, au, sp, opt), budget_s, max_n=10, warmup=1)
        return {"value": 1 / med, "unit": "clips/s", "cores": cores, "kind": "port", "cpu": cpu,
                "sample": f"oracle fp32 train_hardway step (two views x 16 frames of 224^2, 16x-repeated 257x300 "
                          f"spectrogram, both AVENet forwards + 3 losses + backward + Adam), b=1 clip, 1 warm-up, "
                          f"median of {n}"}
    if workload == "tube":
        import tube_oracle as tor

        sd = tor.make_tube_state(0)
        video, spec = tor.make_video(1, 16, 224), orc.make_spectrogram(1)
        opt = orc.AdamRef()
        med, n = _time_loop(lambda: tor.tube_train_step(sd, spec, video, opt), budget_s, max_n=10, warmup=1)
        return {"value": 1 / med, "unit": "clips/s", "cores": cores, "kind": "port", "cpu": cpu,
                "sample": f"oracle fp32 train_3D step (R3D-18 fwd + 16x-repeated audio ResNet-18 fwd/bwd + head + "
                          f"Adam), b=1 clip of 16x224^2 + 257x300, 1 warm-up, median of {n}"}
    B = 2
    sd = orc.make_state(0)
    img, aud = orc.make_image(B), orc.make_spectrogram(B)
    opt = orc.AdamRef()
    med, n = _time_loop(lambda: orc.train_step(sd, img, aud, opt), budget_s * 0.6)

    def fwd_loss():  # configs[0]: the reference's forward + loss on the CPU
        with torch.no_grad():
            orc.hardway_ce(orc.avenet_forward(sd, img, aud, None, training=True)[1])

    med_f, n_f = _time_loop(fwd_loss, budget_s * 0.4)
    return {"value": B / med, "unit": "clips/s", "cores": cores, "kind": "port", "cpu": cpu,
            "fwd_loss_clips_per_s": B / med_f,
            "sample": f"oracle fp32 full train step (fwd+CE+bwd+Adam), B=2, 224^2 + 257x300, 3 warm-ups, median of "
                      f"{n}; fwd_loss_clips_per_s: forward + CE only (configs[0]), median of {n_f}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["1frame", "tube", "twoview"], default="1frame")
    ap.add_argument("--batch", type=int, default=0, help="clips per GPU (weak scaling; default: 128 at N=1, "
                    "256/N at N>1 -- configs[2]'s global batch; tube, twoview: 8 per GPU)")
    ap.add_argument("--global-batch", type=int, default=0, help="clips over all GPUs (strong scaling; 1frame "
                    "default for N>1: 256, BASELINE configs[2])")
    ap.add_argument("--frames", type=int, default=16, help="tube, twoview: frames per clip")
    ap.add_argument("--twoview-folded", action="store_true", help="twoview: run the audio trunk over the folded "
                    "16x-repeated spectrogram batch once per view (the reference's arithmetic)")
    ap.add_argument("--tube-folded", action="store_true", help="tube: run the audio trunk over the folded "
                    "16x-repeated spectrogram batch (the reference's arithmetic) instead of once per clip")
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
    if args.gpus != world:  # before any GPU call: a mismatch would report the wrong n_gpus
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 as "
                 f"python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}")
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import avtubes  # noqa: F401
    from avt_amd.model import AVENet, FullModel, HardWayArgs
    from avt_amd.train import HardWayTrainStep, TwoViewTrainStep
    from avt_amd.trunk import ConvProfiler

    tube = args.workload == "tube"
    twoview = args.workload == "twoview"
    strong = False
    if args.batch:
        B = args.batch
    elif args.global_batch or (world > 1 and not (tube or twoview)):
        G = args.global_batch or 256
        if G % world:
            sys.exit(f"bench.py: global batch {G} does not split over {world} GPUs")
        B, strong = G // world, True
    else:
        B = 8 if (tube or twoview) else 128
    torch.manual_seed(0)
    if twoview:
        model = AVENet(HardWayArgs(), False).to(dev).train()
        frames, spec = synthetic_inputs(B, dev, seed=1000 + rank, frames=args.frames)
        augmented, _ = synthetic_inputs(B, dev, seed=2000 + rank, frames=args.frames)
        inputs = (frames, augmented, spec)
        workload = (f"train_hardway step: b={B} clips x {args.frames} frames of 224x224 in two views + 257x300 "
                    f"spectrogram ({'folded (b t) batch per view' if args.twoview_folded else 'audio once per clip'}),"
                    f" two AVENet forwards over (b t)={B * args.frames} rows, CE x2 + MSE + PropagationLoss, bwd, Adam")
    elif tube:
        model = FullModel(HardWayArgs()).to(dev).train()
        video, spec = synthetic_inputs(B, dev, seed=1000 + rank, frames=args.frames)
        if args.tube_folded:  # train_3D.py:128-130
            spec = spec.unsqueeze(2).repeat(1, 1, args.frames, 1, 1).transpose(1, 2).reshape(
                B * args.frames, 1, 257, 300).contiguous()
        inputs = (spec, video)
        workload = (f"train_3D step: b={B} clips of {args.frames}x224x224 frames + 257x300 spectrogram, R3D-18 fwd "
                    f"+ audio ResNet-18 fwd/bwd ({'folded (b t) batch' if args.tube_folded else 'once per clip'}) "
                    f"+ hard-way head over (b t)={B * args.frames} rows + CE + Adam")
    else:
        model = AVENet(HardWayArgs(), False).to(dev).train()
        inputs = synthetic_inputs(B, dev, seed=1000 + rank)
        workload = "train_hardway_1frame step: 224x224 RGB + 257x300 spectrogram, fwd+CE+bwd+Adam" + (
            f"; configs[2]: global batch {B * world} sharded {B}/GPU" if strong else
            ("; configs[1]" if B == 128 and world == 1 else ""))
    if twoview:
        step = TwoViewTrainStep(model, lr=4e-6, weight_decay=1e-4, dedup_audio=not args.twoview_folded)
    else:
        step = HardWayTrainStep(model, lr=1e-6, weight_decay=1e-4)

    use_graph = not args.no_graph
    for i in range(max(args.warmup, 1 if use_graph else 0)):
        loss = step.step(*inputs)
        if use_graph and i == 0:
            step.capture(*inputs)  # later warm-up and all timed steps are graph replays
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step.step(*inputs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    loss_v = float(loss.flatten()[0])  # twoview: losses[0] = the combined loss
    # roofline of the conv family: HIP events on the launch stream around every conv launch of a
    # few eager steps of the same workload (kept out of the timed region above)
    eager = type(step).__new__(type(step))
    eager.__dict__.update(step.__dict__)
    eager._graph = None
    conc = step.engine.concurrent
    step.engine.concurrent = False  # per-kernel durations of the conv launches, not of overlapped pairs
    with ConvProfiler() as prof:
        for _ in range(args.prof_steps):
            eager.step(*inputs)
        torch.cuda.synchronize()
    step.engine.concurrent = conc
    conv = prof.summary()
    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = el.item()
    if rank == 0:
        ps = max(args.prof_steps, 1)
        clips = B * world * args.steps
        value = clips / elapsed
        ms_step = elapsed / args.steps * 1e3
        fl = sum(v[1] for v in conv.values())
        ms = sum(v[2] for v in conv.values())
        n_launch = sum(v[0] for v in conv.values())
        alg_bytes = sum(v[3] for v in conv.values())
        achieved = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        traffic, traffic_src = conv_traffic(traffic_file(args.workload, B), n_launch / ps, B)
        conv_tflop_step = fl / ps / 1e12
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": DATA,
            "config": {"workload": workload, "global_batch": B * world, "per_gpu_batch": B,
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "kernel": "conv implicit-GEMM (fwd+dgrad+wgrad)",
                         "achieved": round(achieved, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                         "traffic_unit": "HBM bytes per conv launch (PMC FETCH_SIZE/WRITE_SIZE, gfx950-corrected)",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": round(alg_bytes / max(n_launch, 1)),
                         "algorithmic_flops_per_launch": round(fl / max(n_launch, 1)),
                         "launches": n_launch,
                         "per_kind": {k: {"launches": v[0], "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2),
                                          "ms_per_step": round(v[2] / ps, 3)} for k, v in conv.items()},
                         "conv_ms_per_step": round(ms / ps, 3),
                         "measured": f"HIP events around each conv launch, {args.prof_steps} eager steps after the "
                                     "timed region"},
            "launch": ("eager" if args.no_graph else "hip-graph replay") + (
                ", audio trunk on a second stream" if step.engine.concurrent else ""),
            # whole step: algorithmic conv FLOPs of one step / step time (head, BN, Adam: < 1 %)
            "step_conv_tflop": round(conv_tflop_step, 4),
            "step_tflops_per_gpu": round(conv_tflop_step / (ms_step * 1e-3), 2),
            "step_mfma_frac": round(conv_tflop_step / (ms_step * 1e-3) / MFMA_BF16_PEAK_TFLOPS, 4),
            "loss": round(loss_v, 6),
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_budget)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

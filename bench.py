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
kernel time; `traffic` = PMC-measured HBM bytes per conv launch, measured live by two rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE) over child runs of the same workload on this build (N=1), else
taken from profiles/conv_traffic_*.json only if that record names this build's source hash, else null.
`peak` is the vendor dense bf16 peak; `peak_measured` re-measures it on this box in the same run (an
MFMA loop on random operands), next to a 16-byte HBM copy (`peaks_measured`), so a slow box can be
told from a slow build.  Every AVT_* variable is recorded (`avt_env`); the wrong-results diagnostics
(AVT_DIAG_SKIP, AVT_C64_DBG) and a -DAVT_DIAG build of the library are refused.  `cpu_baseline`
times the oracle's fp32 PyTorch-CPU restatement of the same step on the host cores (rank 0, N=1 only).
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


ALG_BYTES_PER_CLIP = 80.8e6  # each conv's input and output once in fwd, dgrad and wgrad (bf16)

# environment knobs that make the library compute WRONG results (timing diagnostics); a bench run refuses them.
# Every other AVT_* variable (A/B performance knobs) is recorded in the JSON line.
WRONG_RESULT_KNOBS = ("AVT_DIAG_SKIP", "AVT_C64_DBG", "AVT_TN_DBG", "AVT_HALO_DBG", "AVT_DIAG_H1_SKIP")


def check_env():
    """Refuse wrong-results knobs (before any GPU call); return every AVT_* variable for the record."""
    bad = [k for k in WRONG_RESULT_KNOBS if os.environ.get(k, "0") not in ("", "0")]
    if bad:
        sys.exit(f"bench.py: refusing to run with wrong-results diagnostics set: {', '.join(bad)}")
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("AVT_")}


def traffic_file(workload, B):
    tag = {"1frame": "b", "tube": "tube_b", "twoview": "twoview_b"}[workload]
    return os.path.join(REPO, "profiles", f"conv_traffic_{tag}{B}.json")


def _load_traffic(path, B, lib_hash):
    """A traffic record (tools/traffic_summary.py) if it is for this batch AND this library's sources."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "absent"
    if t.get("per_gpu_batch") != B:
        return None, f"{os.path.relpath(path, REPO)} is for batch {t.get('per_gpu_batch')}"
    if t.get("lib_source_hash") != lib_hash:
        return None, f"{os.path.relpath(path, REPO)} is stale (measured on another build of libavt)"
    return t, os.path.relpath(path, REPO)


def live_traffic(args, B, lib_hash, timeout_s=240):
    """HBM bytes of this build's step from PMC counters, measured now: two rocprofv3 passes (FETCH_SIZE,
    WRITE_SIZE; they do not fit one pass on gfx950), kernel-trace only, each over a child bench.py running
    1 warm-up + 1 eager step of the same workload (tools/pmc_traffic.sh's recipe).  The child is started
    as a subprocess (never exec'd) after this process's own measurements are done."""
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if exe is None:
        return None, "rocprofv3 not found"
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import traffic_summary as ts

    child = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1", "--warmup", "1", "--no-graph",
             "--prof-steps", "0", "--no-cpu-baseline", "--traffic", "off", "--no-peaks", "--batch", str(B),
             "--workload", args.workload, "--frames", str(args.frames)]
    child += ["--twoview-folded"] if args.twoview_folded else []
    child += ["--tube-folded"] if args.tube_folded else []
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    with tempfile.TemporaryDirectory(prefix="avt_pmc_") as d:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = [exe, "--pmc", ctr, "--kernel-trace", "--output-format", "csv", "-d", os.path.join(d, ctr),
                   "-o", "run", "--"] + child
            try:
                r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout_s)
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 --pmc {ctr} timed out"
            if r.returncode != 0:
                tail = r.stdout.decode(errors="replace").strip().splitlines()[-1:]
                return None, f"rocprofv3 --pmc {ctr} failed ({r.returncode}): {tail}"
        t = ts.summarize(d, 2.0, B, "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over 2 eager steps of this "
                         "workload (read = 2 x FETCH_SIZE KiB, gfx950 correction; write = WRITE_SIZE KiB)", lib_hash)
    if t["conv_dispatches_per_step"] <= 0:
        return None, "PMC passes saw no conv kernels"
    return t, "live"


def measure_peaks(dev, seconds=1.0):
    """Peaks of THIS box, now (the chip's clock varies 5-12 % across MI355X devices and with the data):
    bf16 MFMA loops on random register operands (32x32x16 and 16x16x32, one wave per SIMD), and a
    16-byte HBM copy over 2 x 1 GiB.  HIP events on the launch stream."""
    from avt_amd._lib import call, query

    st = torch.cuda.current_stream(dev)
    blocks = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.empty(blocks * 256, device=dev, dtype=torch.float32)
    out = {}

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    for shape, key in ((0, "mfma_32x32x16_bf16"), (1, "mfma_16x16x32_bf16")):
        iters = 4000
        launch = lambda: call("avt_peak_mfma", sink.data_ptr(), shape, blocks, iters, 12345, st.cuda_stream)
        t1 = timed(launch, 2) / 2  # warm-up + calibration
        iters = max(1000, int(iters * 0.02 / max(t1, 1e-6)))  # ~20 ms launches
        n = max(3, int(seconds / 0.02))
        t = timed(launch, n)
        out[key] = query("avt_peak_mfma_flops", shape, blocks, iters) * n / t / 1e12
    nbytes = 1 << 30
    src = torch.ones(nbytes // 4, device=dev, dtype=torch.float32)
    dst = torch.empty_like(src)
    cp = lambda: call("avt_copy16", dst.data_ptr(), src.data_ptr(), nbytes, blocks * 8, st.cuda_stream)
    timed(cp, 2)
    n = 20
    out["hbm_copy_tbs"] = 2 * nbytes * n / timed(cp, n) / 1e12  # read + write
    del src, dst
    return out


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


def eager_copy(step):
    """A view of the train step (same buffers, optimizer, engine) whose step() launches every kernel eagerly.
    Every captured form must be dropped -- world 1: _graph; world > 1: _seg_graphs (overlap schedule) or
    _graph + _graph_opt -- or step() replays it and the conv profiler sees no launch."""
    eager = type(step).__new__(type(step))
    eager.__dict__.update(step.__dict__)
    eager._graph = eager._graph_opt = eager._seg_graphs = None
    return eager


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
    ap.add_argument("--traffic", choices=["live", "file", "off"], default="live", help="roofline.traffic: live = "
                    "two rocprofv3 PMC passes over this workload after the measurement (N=1; falls back to file), "
                    "file = the committed profiles/conv_traffic_*.json if it was measured on this build, off = null")
    ap.add_argument("--traffic-out", default="", help="write the traffic record (tools/traffic_summary.py format) here")
    ap.add_argument("--no-peaks", action="store_true", help="skip the in-run MFMA / HBM peak measurement")
    args = ap.parse_args()
    avt_env = check_env()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:  # before any GPU call: a mismatch would report the wrong n_gpus
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 as "
                 f"python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}")
    # Test-only overrides (tests/test_bench_dist_gpu.py), recorded in avt_env and "backend": the one-GPU box runs the
    # world > 1 branch with every rank on cuda:0 over gloo, since RCCL needs one device per rank.
    backend = os.environ.get("AVT_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        sys.exit(f"bench.py: AVT_BENCH_BACKEND={backend!r}: expected nccl or gloo")
    if os.environ.get("AVT_BENCH_ONE_DEVICE", "0") not in ("", "0"):
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)

    import avtubes  # noqa: F401
    from avt_amd import _lib
    from avt_amd.model import AVENet, FullModel, HardWayArgs
    from avt_amd.train import HardWayTrainStep, TwoViewTrainStep
    from avt_amd.trunk import ConvProfiler

    if _lib.query("avt_build_flags") & 1:  # AVT_BUILD_DIAG
        sys.exit("bench.py: refusing to run on the -DAVT_DIAG timing-diagnostics build of libavt (wrong results)")
    lib_hash = _lib.source_hash() if _lib.LOAD_PATH == _lib.LIB_PATH else None
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
    eager = eager_copy(step)
    conc = step.engine.concurrent
    step.engine.concurrent = False  # per-kernel durations of the conv launches, not of overlapped pairs
    with ConvProfiler() as prof:
        for _ in range(args.prof_steps):
            eager.step(*inputs)
        torch.cuda.synchronize()
    step.engine.concurrent = conc
    conv = prof.summary()
    if args.prof_steps > 0 and not conv:
        sys.exit("bench.py: the profiled eager steps launched no conv kernel (a captured graph was replayed?)")
    peaks = None if args.no_peaks else measure_peaks(dev)
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
        conv_tflop_step = fl / ps / 1e12
        trec, traffic_src = None, "off"
        if args.traffic == "live" and world == 1 and lib_hash is not None:
            trec, traffic_src = live_traffic(args, B, lib_hash)
        if trec is None and args.traffic != "off":
            why = traffic_src
            trec, traffic_src = _load_traffic(traffic_file(args.workload, B), B, lib_hash)
            if trec is None and args.traffic == "live":
                traffic_src = f"live: {why}; file: {traffic_src}"
        if trec is not None and args.traffic_out:
            with open(args.traffic_out, "w") as f:
                json.dump(trec, f, indent=1)
        lps = n_launch / ps
        traffic = None
        if trec is not None and lps > 0:
            traffic = round((trec["conv_read_bytes_per_step"] + trec["conv_write_bytes_per_step"]) / lps)
        step_tflops = conv_tflop_step / (ms_step * 1e-3)
        peak_meas = peaks["mfma_32x32x16_bf16"] if peaks else None
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
            "backend": (backend if world > 1 else None),
            "roofline": {"bound": "mfma", "kernel": "conv implicit-GEMM (fwd+dgrad+wgrad)",
                         "achieved": round(achieved, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                         "traffic_unit": "HBM bytes per conv launch (PMC FETCH_SIZE/WRITE_SIZE, gfx950-corrected)",
                         "traffic_source": traffic_src,
                         "peak_measured": round(peak_meas, 1) if peak_meas else None,
                         "frac_vs_measured": round(achieved / peak_meas, 4) if peak_meas else None,
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
            "step_tflops_per_gpu": round(step_tflops, 2),
            "step_mfma_frac": round(step_tflops / MFMA_BF16_PEAK_TFLOPS, 4),
            "step_mfma_frac_vs_measured": round(step_tflops / peak_meas, 4) if peak_meas else None,
            # SURVEY 8(d)'s secondary HBM view: clips/s x 80.8 MB algorithmic bytes per clip / (G x 8 TB/s)
            "hbm_view_frac": round(value * ALG_BYTES_PER_CLIP / (world * HBM_PEAK_GBS * 1e9), 4)
            if args.workload == "1frame" else None,
            "step_hbm_bytes": round(trec["step_bytes"]) if trec else None,
            "step_hbm_tbs": round(trec["step_bytes"] / (ms_step * 1e-3) / 1e12, 3) if trec else None,
            "peaks_measured": {k: round(v, 2) for k, v in peaks.items()} if peaks else None,
            "peak_units": {"mfma_*": "TFLOP/s", "hbm_copy_tbs": "TB/s (read + write)"},
            "avt_env": avt_env,
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

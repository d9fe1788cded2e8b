"""Golden vectors at BASELINE.json's full per-GPU sizes, from the REFERENCE itself (survey container only).

    python oracle/gen_golden_full.py cfg3   # AVENet, B=32 (configs[2]'s per-GPU shard: 256 over 8 GPUs)
    python oracle/gen_golden_full.py cfg2   # AVENet, B=128 (configs[1], the bench workload)
    python oracle/gen_golden_full.py cfg4   # FullModel, b=8 clips x 16 frames (configs[3]'s per-GPU shard)

Imports /root/reference/model.py exactly as oracle/gen_golden.py does (stub cv2, Tensor.cuda ->
identity; no arithmetic touched) and runs one train step of the reference in fp64 (the truth) on the
seeded weights/inputs of avenet_oracle / tube_oracle: forward (model.py:112-154 / 17-60), CE(target
0), backward (train_hardway_1frame.py:129-134 / train_3D.py:126-138).  The same reference trunks are
also run under CPU bf16 autocast with the fp32 head: their deviation from fp64 at THIS size is the
yardstick for the GPU build's bf16-trunk tolerances.  Only small outputs are written
(tests/golden/<name>.npz): A, logits, loss, per-parameter gradient norms, gradient slices, and the
full running_mean / running_var of the BNs that reduce over the most rows per channel (the stems:
1.6 M vision / 2.5 M audio rows at B=128).  Inputs are regenerated from seeds on the GPU box.
"""
from __future__ import annotations

import os
import resource
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import avenet_oracle as orc  # noqa: E402
import tube_oracle as tor  # noqa: E402
from gen_golden import OUT, SAMPLE, SLICE_PARAMS, checksum, grad_sample, import_reference  # noqa: E402,F401

# BNs whose running statistics are stored in full: both stems' bn1 (the largest reductions), a
# layer1 BN, a stride-2 downsample BN and the last BN of each trunk
FULL_BUFS = [p + s for p in ("imgnet.", "audnet.") for s in
             ("bn1", "layer1.0.bn1", "layer2.0.downsample.1", "layer4.1.bn2")]
TUBE_BUFS = ["audnet.bn1", "audnet.layer1.0.bn1", "audnet.layer4.1.bn2", "vidnet.bn1", "vidnet.layer4.1.bn2"]


def _peak_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2 ** 20


def avenet_bf16_trunks(ref_model, sd, image, audio):
    """gen_golden.run_reference_bf16_trunks, also returning the BN buffers the bf16 forward updated."""
    import torch.nn.functional as F

    net = ref_model.AVENet(orc.Args(), False)
    net.load_state_dict(sd, strict=True)
    net.train()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        img = net.imgnet(image)
        aud = net.audnet(audio)
    img = F.normalize(img.float(), dim=1)
    aud = F.normalize(F.adaptive_max_pool2d(aud.float(), 1).flatten(1), dim=1)
    A, logits, wA, Pos, Neg = orc.hardway_head(img, aud)
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    bufs = {n: b.detach().clone() for n, b in net.named_buffers()}
    return dict(A=A.detach(), logits=logits.detach(), weighted_A=wA.detach(), loss=loss.detach(), grads=grads,
                bufs=bufs)


def bn_stat_dev(bufs, bufs64, bns):
    """Per BN: max |batch mean - fp64| / max fp64 batch std, and max relative error of the unbiased
    batch variance, both recovered from one momentum-0.1 update of (0, 1) running stats."""
    out = {}
    for bn in bns:
        m64 = bufs64[bn + ".running_mean"].double().numpy() / 0.1
        v64 = (bufs64[bn + ".running_var"].double().numpy() - 0.9) / 0.1
        m = bufs[bn + ".running_mean"].double().numpy() / 0.1
        v = (bufs[bn + ".running_var"].double().numpy() - 0.9) / 0.1
        out[bn] = (np.abs(m - m64).max() / np.sqrt(v64.max()), (np.abs(v - v64) / v64).max())
    return out


def avenet_fixture(ref_model, name, batch, seed_w=0):
    sd = orc.make_state(seed_w, torch.float32)
    image = orc.make_image(batch, 224)
    audio = orc.make_spectrogram(batch, 257, 300)
    t0 = time.time()
    net = ref_model.AVENet(orc.Args(), False)
    net.load_state_dict(sd, strict=True)
    net = net.double().train()
    A, logits, wA, Pos, Neg = net(image.double(), audio.double())
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(batch, dtype=torch.long))
    loss.backward()
    names = [n for n, p in net.named_parameters() if p.grad is not None]
    grads = {n: p.grad.detach() for n, p in net.named_parameters() if p.grad is not None}
    bufs = {n: b.detach() for n, b in net.named_buffers()}
    print(f"[{name}] fp64 reference step {time.time() - t0:.0f} s, peak RSS {_peak_gb():.1f} GB", flush=True)
    out = {"param_names": np.array(names), "shape": np.array([batch, 224, 257, 300])}
    out.update(A_f64=A.detach().numpy(), logits_f64=logits.detach().numpy(), loss_f64=loss.detach().numpy(),
               weighted_A_f64=wA.detach().numpy())
    g64 = np.array([grads[n].norm().item() for n in names])
    out["grad_norm_f64"] = g64
    for n in SLICE_PARAMS:
        out["grad_slice_f64/" + n] = grads[n].flatten()[:64].numpy()
    for n in names:
        out["grad_sample_f64/" + n] = grad_sample(grads[n])
    for b in FULL_BUFS:
        out["buf_f64/" + b + ".running_mean"] = bufs[b + ".running_mean"].numpy()
        out["buf_f64/" + b + ".running_var"] = bufs[b + ".running_var"].numpy()
    A64, log64, wA64 = A.detach(), logits.detach(), wA.detach()
    del net, A, logits, wA, Pos, Neg, loss, grads
    # yardstick: the reference's trunks under bf16 autocast, fp32 head (gen_golden.run_reference_bf16_trunks)
    t0 = time.time()
    rb = avenet_bf16_trunks(ref_model, sd, image, audio)
    print(f"[{name}] bf16-trunk reference {time.time() - t0:.0f} s", flush=True)
    off = ~np.eye(batch, batch + 2, k=1, dtype=bool)
    diag = np.eye(batch, batch + 2, k=1, dtype=bool)
    lg, l64 = rb["logits"].double().numpy(), log64.numpy()
    gb = np.array([rb["grads"][n].double().norm().item() for n in names])
    dev = {
        "A_abs": np.abs(rb["A"].double().numpy() - A64.numpy()).max(),
        "logits_off_abs": np.abs(lg[off] - l64[off]).max(),
        "logits_diag_rel": (np.abs(lg[diag] - l64[diag]) / np.abs(l64[diag])).max(),
        "loss_rel": abs(rb["loss"].item() - out["loss_f64"].item()) / abs(out["loss_f64"].item()),
        "wA_rel": np.abs(rb["weighted_A"].double().numpy() - wA64.numpy()).max() / np.abs(wA64.numpy()).max(),
        "gradnorm_rel": np.abs(gb - g64) / g64,
    }
    for k, v in dev.items():
        out["bf16ref_dev/" + k] = np.asarray(v)
    for n in SLICE_PARAMS:  # the yardstick's own gradient values (direction bounds of the GPU test)
        out["bf16ref_slice/" + n] = rb["grads"][n].flatten()[:64].double().numpy()
    for n in names:
        out["bf16ref_sample/" + n] = grad_sample(rb["grads"][n])
    for bn, (em, ev) in bn_stat_dev(rb["bufs"], bufs, FULL_BUFS).items():
        out["bf16ref_dev/bnstat/" + bn] = np.array([em, ev])
        print(f"[{name}] bf16-trunk reference {bn}: batch-mean err {em:.2e} of std, batch-var rel err {ev:.2e}")
    print(f"[{name}] bf16-trunk reference deviation: " + ", ".join(
        f"{k}={np.max(v):.3e}" + (f" (median {np.median(v):.3e})" if np.ndim(v) else "") for k, v in dev.items()))
    out["image_checksum"] = checksum(image)
    out["audio_checksum"] = checksum(audio)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"[{name}] loss f64 {out['loss_f64'].item():.9f} -> {path}", flush=True)


def tube_bf16(ref_model, sd, spec, video):
    """gen_golden_tube.run_reference_bf16_trunks, also returning the BN buffers."""
    import torch.nn.functional as F

    net = ref_model.FullModel(orc.Args())
    net.load_state_dict(sd, strict=True)
    net.train()
    audio = tor.repeat_spectrogram(spec, video.shape[2])
    with torch.autocast("cpu", dtype=torch.bfloat16):
        aud = net.audnet(audio)
        with torch.no_grad():  # the hook detaches layer4 (model.py:15): no vidnet gradient either way
            net.vidnet(video)
    vid = F.normalize(ref_model.activation["layer4"].float(), dim=1)
    aud = F.normalize(F.adaptive_max_pool2d(aud.float(), 1).flatten(1), dim=1)
    A, logits = orc.hardway_attention(aud, vid)
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    bufs = {n: x.detach().clone() for n, x in net.named_buffers()}
    return dict(A=A.detach(), logits=logits.detach(), loss=loss.detach(), grads=grads, bufs=bufs)


def tube_fixture(ref_model, name, b, t, seed_w=0):

    sd = tor.make_tube_state(seed_w, torch.float32)
    video = tor.make_video(b, t, 224)
    spec = orc.make_spectrogram(b, 257, 300)
    t0 = time.time()
    net = ref_model.FullModel(orc.Args())
    net.load_state_dict(sd, strict=True)
    net = net.double().train()
    for p in net.vidnet.parameters():  # the layer4 hook detaches (model.py:15): vidnet never gets a
        p.requires_grad_(False)          # gradient; skipping its autograd tape changes no arithmetic
    audio = tor.repeat_spectrogram(spec.double(), t)  # train_3D.py:128-130
    A, logits = net(audio, video.double())
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    loss.backward()
    names = sorted(n for n, p in net.named_parameters() if p.grad is not None)
    grads = {n: p.grad.detach() for n, p in net.named_parameters() if p.grad is not None}
    bufs = {n: x.detach() for n, x in net.named_buffers()}
    print(f"[{name}] fp64 reference step {time.time() - t0:.0f} s, peak RSS {_peak_gb():.1f} GB", flush=True)
    out = {"param_names": np.array(names), "shape": np.array([b, t, 224, 257, 300])}
    out.update(A_f64=A.detach().numpy(), logits_f64=logits.detach().numpy(), loss_f64=loss.detach().numpy())
    g64 = np.array([grads[n].norm().item() for n in names])
    out["grad_norm_f64"] = g64
    for n in names:
        out["grad_sample_f64/" + n] = grad_sample(grads[n])
    for bn in TUBE_BUFS:
        out["buf_f64/" + bn + ".running_mean"] = bufs[bn + ".running_mean"].numpy()
        out["buf_f64/" + bn + ".running_var"] = bufs[bn + ".running_var"].numpy()
    A64, log64 = A.detach(), logits.detach()
    del net, A, logits, loss, grads
    t0 = time.time()
    rb = tube_bf16(ref_model, sd, spec, video)
    print(f"[{name}] bf16-trunk reference {time.time() - t0:.0f} s", flush=True)
    nb = log64.shape[0]
    off = ~np.eye(nb, nb + 2, k=1, dtype=bool)
    diag = np.eye(nb, nb + 2, k=1, dtype=bool)
    lg, l64 = rb["logits"].double().numpy(), log64.numpy()
    gb = np.array([rb["grads"][n].double().norm().item() for n in names])
    dev = {
        "A_abs": np.abs(rb["A"].double().numpy() - A64.numpy()).max(),
        "logits_off_abs": np.abs(lg[off] - l64[off]).max(),
        "logits_diag_rel": (np.abs(lg[diag] - l64[diag]) / np.abs(l64[diag])).max(),
        "loss_rel": abs(rb["loss"].item() - out["loss_f64"].item()) / abs(out["loss_f64"].item()),
        "gradnorm_rel": np.abs(gb - g64) / g64,
    }
    for k, v in dev.items():
        out["bf16ref_dev/" + k] = np.asarray(v)
    for n in names:
        out["bf16ref_sample/" + n] = grad_sample(rb["grads"][n])
    for bn, (em, ev) in bn_stat_dev(rb["bufs"], bufs, TUBE_BUFS).items():
        out["bf16ref_dev/bnstat/" + bn] = np.array([em, ev])
        print(f"[{name}] bf16-trunk reference {bn}: batch-mean err {em:.2e} of std, batch-var rel err {ev:.2e}")
    print(f"[{name}] bf16-trunk reference deviation: " + ", ".join(
        f"{k}={np.max(v):.3e}" + (f" (median {np.median(v):.3e})" if np.ndim(v) else "") for k, v in dev.items()))
    out["video_checksum"] = checksum(video)
    out["spec_checksum"] = checksum(spec)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"[{name}] loss f64 {out['loss_f64'].item():.9f} -> {path}", flush=True)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(int(os.environ.get("AVT_GEN_THREADS", "8")))
    ref_model = import_reference()
    which = sys.argv[1:] or ["cfg3"]
    for w in which:
        if w == "cfg3":
            avenet_fixture(ref_model, "avenet_cfg3_b32", 32)
        elif w == "cfg2":
            avenet_fixture(ref_model, "avenet_cfg2_b128", 128)
        elif w == "cfg4":
            tube_fixture(ref_model, "fullmodel_cfg4_b8t16", 8, 16)
        else:
            raise SystemExit(f"unknown fixture {w}")


if __name__ == "__main__":
    main()

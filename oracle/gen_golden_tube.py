"""Golden vectors for the 3-D tube step (FullModel, cfg 4) from the REFERENCE itself.

Run here (CPU, /root/reference present):   python oracle/gen_golden_tube.py
Imports /root/reference/model.py exactly as oracle/gen_golden.py does (stub cv2, Tensor.cuda ->
identity; no arithmetic touched), builds ``FullModel(args)`` (model.py:17-36: R3D-18 vidnet +
audio ResNet-18 + HardWayAttention), loads the seeded weights of tube_oracle.make_tube_state,
and runs one train_3D.py step (126-138) in fp64 and fp32: spectrogram repeated t times and
folded (b t), CE(logits, 0), backward, torch.optim.Adam(model.parameters(), lr 1e-6, wd 1e-4).
Writes tests/golden/fullmodel_<name>.npz and checks the restatement (tube_oracle) against it.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import avenet_oracle as orc  # noqa: E402
import tube_oracle as tor  # noqa: E402
from gen_golden import OUT, checksum, import_reference  # noqa: E402

SLICE = ["audnet.conv1_a.weight", "audnet.layer1.0.conv1.weight", "audnet.layer4.1.conv2.weight",
         "audnet.layer2.0.downsample.0.weight", "audnet.bn1.weight", "audnet.layer4.1.bn2.bias"]
VBUF = ["vidnet.bn1.running_mean", "vidnet.bn1.running_var", "vidnet.layer4.1.bn2.running_mean",
        "vidnet.layer4.1.bn2.running_var", "vidnet.layer2.0.downsample.1.running_var"]


def run_reference(ref_model, sd, spec, video, dtype):
    net = ref_model.FullModel(orc.Args())
    net.load_state_dict(sd, strict=True)
    net = net.to(dtype).train()
    t = video.shape[2]
    audio = tor.repeat_spectrogram(spec.to(dtype), t)  # train_3D.py:128-130
    A, logits = net(audio, video.to(dtype))
    layer4 = ref_model.activation["layer4"].clone()
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    opt = torch.optim.Adam(net.parameters(), lr=1e-6, weight_decay=1e-4)
    opt.zero_grad()
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    before = {n: p.detach().clone() for n, p in net.named_parameters()}
    opt.step()
    after = {n: p.detach().clone() for n, p in net.named_parameters()}
    bufs = {n: b.detach().clone() for n, b in net.named_buffers()}
    return dict(A=A.detach(), logits=logits.detach(), loss=loss.detach(), layer4=layer4, grads=grads,
                before=before, after=after, bufs=bufs)


def run_reference_bf16_trunks(ref_model, sd, spec, video):
    """The reference's own trunks (net.audnet, net.vidnet) under CPU bf16 autocast with the fp32
    head: the yardstick for a bf16-trunk implementation's tolerances (as gen_golden.py)."""
    import torch.nn.functional as F

    net = ref_model.FullModel(orc.Args())
    net.load_state_dict(sd, strict=True)
    net.train()
    audio = tor.repeat_spectrogram(spec, video.shape[2])
    with torch.autocast("cpu", dtype=torch.bfloat16):
        aud = net.audnet(audio)
        net.vidnet(video)
    vid = F.normalize(ref_model.activation["layer4"].float(), dim=1)
    aud = F.normalize(F.adaptive_max_pool2d(aud.float(), 1).flatten(1), dim=1)
    A, logits = orc.hardway_attention(aud, vid)
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    return dict(A=A.detach(), logits=logits.detach(), loss=loss.detach(), grads=grads)


def make_fixture(ref_model, name, b, t, size, freq, frames, seed_w=0):
    sd = tor.make_tube_state(seed_w, torch.float32)
    video = tor.make_video(b, t, size)
    spec = orc.make_spectrogram(b, freq, frames)
    r64 = run_reference(ref_model, sd, spec, video, torch.float64)
    r32 = run_reference(ref_model, sd, spec, video, torch.float32)
    names = sorted(r64["grads"])
    assert set(names) == set(tor.trainable_names_tube()), sorted(set(names) ^ set(tor.trainable_names_tube()))
    assert not any(n.startswith("vidnet.") for n in names)  # the hook detaches layer4 (model.py:15)
    out = {"param_names": np.array(names), "shape": np.array([b, t, size, freq, frames])}
    for k in ("A", "logits", "loss"):
        out[k + "_f64"] = r64[k].numpy()
        out[k + "_f32"] = r32[k].float().numpy()
    l4 = r64["layer4"]
    out["layer4_f64_slice"] = l4.flatten()[:256].numpy()
    out["layer4_f64_checksum"] = checksum(l4)
    out["grad_norm_f64"] = np.array([r64["grads"][n].norm().item() for n in names])
    out["grad_norm_f32"] = np.array([r32["grads"][n].float().norm().item() for n in names])
    for n in SLICE:
        out["grad_slice_f64/" + n] = r64["grads"][n].flatten()[:64].numpy()
        out["delta_slice_f64/" + n] = (r64["after"][n] - r64["before"][n]).flatten()[:64].numpy()
    for n in VBUF + ["audnet.bn1.running_var", "audnet.layer4.1.bn2.running_mean"]:
        out["buf_f64/" + n] = r64["bufs"][n][:16].numpy()
    rb = run_reference_bf16_trunks(ref_model, sd, spec, video)
    n_b = rb["logits"].shape[0]
    off = ~np.eye(n_b, n_b + 2, k=1, dtype=bool)
    g64 = np.array([r64["grads"][n].norm().item() for n in names])
    dev = {"A_abs": np.abs(rb["A"].double().numpy() - r64["A"].numpy()).max(),
           "logits_off_abs": np.abs(rb["logits"].double().numpy()[off] - r64["logits"].numpy()[off]).max(),
           "loss_rel": abs(rb["loss"].item() - r64["loss"].item()) / abs(r64["loss"].item()),
           "gradnorm_rel": np.abs(np.array([rb["grads"][n].double().norm().item() for n in names]) - g64) / g64,
           # full-tensor cosine of each bf16-trunk gradient with the fp64 one (median ~0.8 at the
           # tiny size: stem-side gradients of an 8-row batch are dominated by bf16 noise)
           "grad_cos": np.array([torch.nn.functional.cosine_similarity(
               rb["grads"][n].double().flatten(), r64["grads"][n].flatten(), dim=0).item() for n in names])}
    for k, v in dev.items():
        out["bf16ref_dev/" + k] = np.asarray(v)
    print(f"[{name}] bf16-trunk reference deviation: " + ", ".join(
        f"{k}={np.max(v) if k != 'grad_cos' else np.median(v):.3e}" for k, v in dev.items()))
    out["video_checksum"] = checksum(video)
    out["spec_checksum"] = checksum(spec)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)

    # pin the restatement against the reference on the same inputs
    sd64 = orc.OrderedDict((k, v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items())
    loss, A, logits, grads = tor.tube_train_step(sd64, spec.double(), video.double(), orc.AdamRef())
    dl = (logits - r64["logits"]).abs().max().item()
    dg = max(abs(grads[n].norm().item() - r64["grads"][n].norm().item()) / max(r64["grads"][n].norm().item(), 1e-30)
             for n in names)
    dbuf = max((sd64[n] - r64["bufs"][n]).abs().max().item() for n in VBUF)
    print(f"[{name}] logits {tuple(r64['logits'].shape)} loss ref64={r64['loss'].item():.9f} "
          f"f32={r32['loss'].item():.9f} oracle64={loss.item():.9f} |dlogits|={dl:.2e} "
          f"max rel dgradnorm={dg:.2e} |dbuf|={dbuf:.2e} -> {path}")
    assert dl < 1e-9 and dg < 1e-9 and dbuf < 1e-12


TORCH_INIT_PARAMS = ["vidnet.conv1.weight", "vidnet.layer1.0.conv1.weight", "vidnet.layer2.0.downsample.0.weight",
                     "vidnet.layer4.1.conv2.weight", "vidnet.fc.weight", "vidnet.fc.bias", "audnet.conv1_a.weight",
                     "audnet.layer4.1.conv2.weight", "audnet.fc.bias", "vidnet.bn1.weight"]


def make_torch_init_fixture(ref_model, name="fullmodel_torch_init_seed0"):
    """The reference FullModel's own init under torch.manual_seed(0) (model.py:18-24 ->
    resnet3D.py:103-158, base_models.py:113-163), as per-tensor checksums."""
    torch.manual_seed(0)
    net = ref_model.FullModel(orc.Args())
    sd = net.state_dict()
    np.savez_compressed(os.path.join(OUT, name + ".npz"), names=np.array(TORCH_INIT_PARAMS),
                        keys=np.array(list(sd.keys())),
                        checksums=np.stack([checksum(sd[n]) for n in TORCH_INIT_PARAMS]))
    print(f"[{name}] {len(sd)} entries")


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    ref_model = import_reference()
    make_torch_init_fixture(ref_model)
    make_fixture(ref_model, "fullmodel_tiny_b2t4", b=2, t=4, size=32, freq=65, frames=76)
    make_fixture(ref_model, "fullmodel_mid_b2t4", b=2, t=4, size=112, freq=129, frames=150)


if __name__ == "__main__":
    main()

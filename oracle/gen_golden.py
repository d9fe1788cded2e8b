"""Generate golden vectors from the REFERENCE itself (survey container only).

Run here (CPU, /root/reference present):   python oracle/gen_golden.py
Writes small .npz fixtures under tests/golden/.  The reference never travels to the GPU
box: only these outputs do.  Inputs and weights are regenerated from seeds by
oracle/avenet_oracle.py (checksums of both are stored in each fixture so a drift is caught).

How the reference is imported: two patches that touch no arithmetic —
  1. a stub ``cv2`` module (model.py:1 imports ``threshold`` and never uses it);
  2. ``torch.Tensor.cuda`` -> identity (model.py:48-51,115 call ``.cuda()``; no GPU here).
The reference AVENet / HardWayAttention are then run in fp64 (truth) and fp32 on the
seeded weights, through CE(target 0), backward and one torch.optim.Adam step with the
train_hardway_1frame.py:116 hyper-parameters (lr 1e-6, wd 1e-4).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("AVT_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, HERE)
import avenet_oracle as orc  # noqa: E402


def import_reference():
    sys.modules.setdefault("cv2", types.SimpleNamespace(threshold=None))
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF)
    import model as ref_model  # noqa: E402  (the reference's model.py)
    return ref_model


SAMPLE = 256  # strided gradient sample per parameter (direction checks of every parameter)


def grad_sample(g: torch.Tensor) -> np.ndarray:
    """SAMPLE values of a gradient at a fixed stride over the whole tensor (all of it when smaller)."""
    f = g.detach().flatten()
    stride = max(1, f.numel() // SAMPLE)
    return f[::stride][:SAMPLE].double().numpy()


def checksum(t: torch.Tensor) -> np.ndarray:
    t = t.detach().double().flatten()
    return np.array([t.sum().item(), (t * t).sum().item(), t[: min(16, t.numel())].sum().item()])


def run_reference(ref_model, sd, image, audio, dtype):
    args = orc.Args()
    net = ref_model.AVENet(args, False)
    net.load_state_dict(sd, strict=True)
    net = net.to(dtype).train()
    image, audio = image.to(dtype), audio.to(dtype)
    A, logits, weighted_A, Pos, Neg = net(image, audio)
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    opt = torch.optim.Adam(net.parameters(), lr=1e-6, weight_decay=1e-4)
    opt.zero_grad()
    loss.backward()
    names = [n for n, p in net.named_parameters() if p.grad is not None]
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    before = {n: p.detach().clone() for n, p in net.named_parameters()}
    opt.step()
    after = {n: p.detach().clone() for n, p in net.named_parameters()}
    bufs = {n: b.detach().clone() for n, b in net.named_buffers()}
    return dict(A=A.detach(), logits=logits.detach(), weighted_A=weighted_A.detach(), Pos=Pos.detach(),
                Neg=Neg.detach(), loss=loss.detach(), names=names, grads=grads, before=before,
                after=after, bufs=bufs)


def run_reference_bf16_trunks(ref_model, sd, image, audio):
    """The reference's own trunks (net.imgnet / net.audnet, base_models.py:195-210) under CPU bf16
    autocast, with the fp32 head (model.py:116-154, restated bit-exactly by avenet_oracle) —
    the SURVEY §0.7 "bf16 backbone, fp32 similarity math" configuration.  Its deviation from the
    fp64 run is the yardstick for any bf16-trunk implementation's tolerances."""
    net = ref_model.AVENet(orc.Args(), False)
    net.load_state_dict(sd, strict=True)
    net.train()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        img = net.imgnet(image)
        aud = net.audnet(audio)
    img = torch.nn.functional.normalize(img.float(), dim=1)
    aud = torch.nn.functional.normalize(torch.nn.functional.adaptive_max_pool2d(aud.float(), 1).flatten(1), dim=1)
    A, logits, wA, Pos, Neg = orc.hardway_head(img, aud)
    loss = torch.nn.CrossEntropyLoss()(logits, torch.zeros(logits.shape[0], dtype=torch.long))
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    return dict(A=A.detach(), logits=logits.detach(), weighted_A=wA.detach(), loss=loss.detach(), grads=grads)


def deviation(res, r64, names, b):
    """Deviation metrics of a run from the fp64 reference (same metrics the GPU tests assert)."""
    off = ~np.eye(b, b + 2, k=1, dtype=bool)
    diag = np.eye(b, b + 2, k=1, dtype=bool)
    lg, l64 = res["logits"].double().numpy(), r64["logits"].numpy()
    gn = np.array([res["grads"][n].double().norm().item() for n in names])
    g64 = np.array([r64["grads"][n].norm().item() for n in names])
    cos = []
    for n in SLICE_PARAMS:
        a = res["grads"][n].double().flatten()[:64].numpy()
        r = r64["grads"][n].flatten()[:64].numpy()
        cos.append(float(a @ r / (np.linalg.norm(a) * np.linalg.norm(r))))
    return {
        "A_abs": np.abs(res["A"].double().numpy() - r64["A"].numpy()).max(),
        "logits_off_abs": np.abs(lg[off] - l64[off]).max(),
        "logits_diag_rel": (np.abs(lg[diag] - l64[diag]) / np.abs(l64[diag])).max(),
        "loss_rel": abs(res["loss"].item() - r64["loss"].item()) / abs(r64["loss"].item()),
        "wA_rel": np.abs(res["weighted_A"].double().numpy() - r64["weighted_A"].numpy()).max()
        / np.abs(r64["weighted_A"].numpy()).max(),
        "gradnorm_rel": np.abs(gn - g64) / g64,
        "slice_cos": np.array(cos),
    }


SLICE_PARAMS = [
    "imgnet.conv1.weight", "audnet.conv1_a.weight", "imgnet.layer1.0.conv1.weight",
    "imgnet.layer2.0.downsample.0.weight", "imgnet.layer4.1.conv2.weight",
    "audnet.layer4.1.conv2.weight", "audnet.layer3.0.conv1.weight", "imgnet.bn1.weight",
    "audnet.layer4.1.bn2.weight", "audnet.layer4.1.bn2.bias",
]
BUF_SLICES = ["imgnet.bn1.running_mean", "imgnet.bn1.running_var",
              "audnet.layer4.1.bn2.running_mean", "audnet.layer4.1.bn2.running_var"]


def make_fixture(ref_model, name, batch, img_size, freq, frames, seed_w=0):
    sd = orc.make_state(seed_w, torch.float32)
    image = orc.make_image(batch, img_size)
    audio = orc.make_spectrogram(batch, freq, frames)
    out = {}
    res = {}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        res[tag] = run_reference(ref_model, sd, image, audio, dt)
    r64, r32 = res["f64"], res["f32"]
    names = r64["names"]
    out["param_names"] = np.array(names)
    for k in ("A", "logits", "weighted_A", "Pos", "Neg", "loss"):
        out[k + "_f64"] = r64[k].numpy()
        out[k + "_f32"] = r32[k].float().numpy()
    out["grad_norm_f64"] = np.array([r64["grads"][n].norm().item() for n in names])
    out["grad_norm_f32"] = np.array([r32["grads"][n].float().norm().item() for n in names])
    for n in SLICE_PARAMS:
        out["grad_slice_f64/" + n] = r64["grads"][n].flatten()[:64].numpy()
        out["delta_slice_f64/" + n] = (r64["after"][n] - r64["before"][n]).flatten()[:64].numpy()
    for n in BUF_SLICES:
        out["buf_f64/" + n] = r64["bufs"][n][:16].numpy()
    rb = run_reference_bf16_trunks(ref_model, sd, image, audio)
    dev = deviation(rb, r64, names, batch)
    for k, v in dev.items():
        out["bf16ref_dev/" + k] = np.asarray(v)
    # per-parameter gradient samples of the fp64 truth and of the bf16-autocast yardstick (tests bound EVERY
    # parameter by its own yardstick: tests/gradcheck.py)
    for n in names:
        out["grad_sample_f64/" + n] = grad_sample(r64["grads"][n])
        out["bf16ref_sample/" + n] = grad_sample(rb["grads"][n])
    for n in SLICE_PARAMS:
        out["bf16ref_slice/" + n] = rb["grads"][n].flatten()[:64].double().numpy()
    print(f"[{name}] bf16-trunk reference deviation: " + ", ".join(
        f"{k}={np.max(v) if k != 'slice_cos' else np.min(v):.3e}" for k, v in dev.items()))
    out["image_checksum"] = checksum(image)
    out["audio_checksum"] = checksum(audio)
    out["weight_checksum"] = np.array([checksum(sd[n])[0] for n in SLICE_PARAMS])
    out["shape"] = np.array([batch, img_size, freq, frames])
    if batch * img_size * img_size <= 4 * 64 * 64:
        out["image"] = image.numpy()
        out["audio"] = audio.numpy()
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)

    # pin the restatement against the reference on the same inputs
    sd64 = orc.OrderedDict((k, v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items())
    loss, logits, grads = orc.train_step(sd64, image.double(), audio.double(), orc.AdamRef(), None)
    dl = (logits - r64["logits"]).abs().max().item()
    dg = max(abs(grads[n].norm().item() - r64["grads"][n].norm().item()) / max(r64["grads"][n].norm().item(), 1e-30)
             for n in names)
    print(f"[{name}] loss ref64={r64['loss'].item():.9f} f32={r32['loss'].item():.9f} "
          f"oracle64={loss.item():.9f}  |dlogits|={dl:.2e} max rel dgradnorm={dg:.2e}  -> {path}")
    assert set(grads) == set(names), (sorted(set(grads) ^ set(names)))
    assert dl < 1e-9 and dg < 1e-9


def make_attention_fixture(ref_model, name="hardway_attention_tiny", b=2, t=4, hw=14, c=512, seed=5):
    vid, aud = orc.make_tube_features(b, t, hw, c, seed)
    att = ref_model.HardWayAttention()
    A, logits = att(aud, vid)
    A2, logits2 = orc.hardway_attention(aud, vid)
    assert (logits - logits2).abs().max().item() < 1e-9
    np.savez_compressed(os.path.join(OUT, name + ".npz"), vid_checksum=checksum(vid), aud_checksum=checksum(aud),
                        shape=np.array([b, t, hw, c, seed]), A_f64=A.numpy(), logits_f64=logits.numpy())
    print(f"[{name}] logits[0,:4]={logits[0,:4].tolist()}")


TORCH_INIT_PARAMS = ["imgnet.conv1.weight", "imgnet.conv1_a.weight", "imgnet.layer1.0.conv1.weight",
                     "imgnet.layer4.1.bn2.weight", "audnet.conv1_a.weight", "audnet.layer4.1.conv2.weight",
                     "audnet.fc.weight", "audnet.fc.bias", "audnet.layer2.0.downsample.0.weight"]


def make_torch_init_fixture(ref_model, name="torch_init_seed0"):
    """The reference's own init under torch.manual_seed(0) (model.py:104-110 after the
    base_models.py:158-163 init and module construction), as per-tensor checksums."""
    torch.manual_seed(0)
    net = ref_model.AVENet(orc.Args(), False)
    sd = net.state_dict()
    np.savez_compressed(os.path.join(OUT, name + ".npz"), names=np.array(TORCH_INIT_PARAMS),
                        checksums=np.stack([checksum(sd[n]) for n in TORCH_INIT_PARAMS]))
    print(f"[{name}] {len(sd)} entries")


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    ref_model = import_reference()
    make_fixture(ref_model, "avenet_tiny_b4", batch=4, img_size=64, freq=65, frames=76)
    make_fixture(ref_model, "avenet_full_b2", batch=2, img_size=224, freq=257, frames=300)
    make_attention_fixture(ref_model)
    make_torch_init_fixture(ref_model)


if __name__ == "__main__":
    main()

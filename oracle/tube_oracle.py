"""CPU restatement of the reference 3-D "tube" step (FullModel) — TEST INFRASTRUCTURE ONLY.

Like ``avenet_oracle.py`` this is the oracle: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, as the checker / timed host baseline.  The
product path never imports it.

Parity pin: ``oracle/gen_golden_tube.py`` runs the reference ``FullModel`` itself (imported from
``/root/reference/model.py`` in the survey container) on the seeded weights/inputs below and
writes ``tests/golden/fullmodel_*.npz``; ``tests/test_oracle_golden.py`` checks this restatement
against them.

What it restates (reference file:line):
  * R3D-18 = resnet3D.generate_model(18, no_max_pool=True, n_classes=1039) — model.py:20;
    resnet3D.py:103-213: stem Conv3d 3->64 (7,7,7) stride (1,2,2) pad (3,3,3) (122-127), BN3d,
    ReLU, no max-pool (200-201), layer1 (64, stride 1, no downsample), layer2-4 stride (1,2,2)
    with conv1x1x1+BN3d downsample (shortcut 'B', 169-184), BasicBlock 31-61.
    ``avgpool``/``fc`` (208-212) produce a result the FullModel discards (model.py:33): skipped.
  * FullModel.forward — model.py:26-36: audio ResNet-18 (base_models, modal 'audio') ->
    AdaptiveMaxPool2d(1) -> normalize; video layer4 captured by the forward hook **detached**
    (model.py:12-15, 23, 34) -> normalize(dim=1) -> HardWayAttention (model.py:46-60).
  * The train_3D.py step (126-138): spectrogram repeated t times and folded (b t) (128-130),
    CE(logits, 0), backward (only audnet receives gradients), Adam(lr 1e-6, wd 1e-4) over
    model.parameters() (116; params without a gradient are skipped, as in torch).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

import avenet_oracle as orc

R3D_STAGES = [(64, 1), (128, 2), (256, 2), (512, 2)]  # (planes, spatial stride); temporal stride 1


def r3d18_entries(prefix: str) -> List[Tuple[str, tuple, str]]:
    """state_dict entries of resnet3D.generate_model(18, no_max_pool=True, n_classes=1039)."""
    e = [(prefix + "conv1.weight", (64, 3, 7, 7, 7), "conv")]
    e += orc._bn_entries(prefix + "bn1", 64)
    inplanes = 64
    for li, (planes, stride) in enumerate(R3D_STAGES, start=1):
        for bi in range(2):
            s = stride if bi == 0 else 1
            p = f"{prefix}layer{li}.{bi}."
            cin = inplanes if bi == 0 else planes
            e.append((p + "conv1.weight", (planes, cin, 3, 3, 3), "conv"))
            e += orc._bn_entries(p + "bn1", planes)
            e.append((p + "conv2.weight", (planes, planes, 3, 3, 3), "conv"))
            e += orc._bn_entries(p + "bn2", planes)
            if bi == 0 and (s != 1 or inplanes != planes):
                e.append((p + "downsample.0.weight", (planes, inplanes, 1, 1, 1), "conv"))
                e += orc._bn_entries(p + "downsample.1", planes)
        inplanes = planes
    e.append((prefix + "fc.weight", (1039, 512), "fc_w"))
    e.append((prefix + "fc.bias", (1039,), "fc_b"))
    return e


def fullmodel_entries() -> List[Tuple[str, tuple, str]]:
    """FullModel registers vidnet, audnet, avgpool, attention (model.py:19-24)."""
    return r3d18_entries("vidnet.") + orc.resnet18_entries("audnet.")


def make_tube_state(seed: int = 0, dtype=torch.float32) -> "OrderedDict[str, torch.Tensor]":
    """Seeded synthetic FullModel weights (the pretrained r3d18_KM_200ep.pth is absent).

    conv: N(0, 2/fan_out) (kaiming fan_out, resnet3D.py:154-157 / base_models.py:158-161);
    BN weight ~ N(1, 0.02) and bias ~ N(0, 0.02) (non-trivial affine, so the BN apply is
    exercised), running stats 0/1; fc: U(+-1/sqrt(512)).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for name, shape, kind in fullmodel_entries():
        if kind == "conv":
            fan_out = shape[0] * int(np.prod(shape[2:]))
            a = rng.standard_normal(shape, dtype=np.float64) * math.sqrt(2.0 / fan_out)
        elif kind == "bn_w":
            a = 1.0 + 0.02 * rng.standard_normal(shape, dtype=np.float64)
        elif kind == "bn_b":
            a = 0.02 * rng.standard_normal(shape, dtype=np.float64)
        elif kind == "rm":
            a = np.zeros(shape)
        elif kind == "rv":
            a = np.ones(shape)
        elif kind == "nbt":
            sd[name] = torch.zeros((), dtype=torch.long)
            continue
        elif kind in ("fc_w", "fc_b"):
            b = 1.0 / math.sqrt(512.0)
            a = rng.uniform(-b, b, size=shape)
        else:  # pragma: no cover
            raise ValueError(kind)
        sd[name] = torch.from_numpy(np.ascontiguousarray(a)).to(dtype)
    return sd


def make_video(b: int, t: int = 16, size: int = 224, seed: int = 3) -> torch.Tensor:
    """Normalised-frame-like clip [b, 3, t, size, size] (dataloader.py:252-274 layout)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.standard_normal((b, 3, t, size, size), dtype=np.float32))


def repeat_spectrogram(spec: torch.Tensor, t: int) -> torch.Tensor:
    """train_3D.py:128-130: [b,1,F,T] -> repeat t -> '(b t) 1 F T'."""
    b = spec.shape[0]
    return spec.unsqueeze(2).repeat(1, 1, t, 1, 1).permute(0, 2, 1, 3, 4).reshape(b * t, *spec.shape[1:])


def _bn3(x, sd, prefix, training):
    return orc._bn(x, sd, prefix, training)


def r3d18_forward(sd, prefix: str, x: torch.Tensor, training: bool = True, max_pool: bool = False) -> torch.Tensor:
    """resnet3D.ResNet.forward up to layer4 (resnet3D.py:196-206). x [b,3,t,H,W] -> [b,512,t,h,w].  max_pool: the
    stem's nn.MaxPool3d(kernel_size=3, stride=2, padding=1) of no_max_pool=False (resnet3D.py:129, 200-201)."""
    x = F.conv3d(x, sd[prefix + "conv1.weight"], stride=(1, 2, 2), padding=(3, 3, 3))
    x = F.relu(_bn3(x, sd, prefix + "bn1", training))
    if max_pool:
        x = F.max_pool3d(x, kernel_size=3, stride=2, padding=1)
    for li, (planes, stride) in enumerate(R3D_STAGES, start=1):
        for bi in range(2):
            s = stride if bi == 0 else 1
            p = f"{prefix}layer{li}.{bi}."
            res = x
            out = F.conv3d(x, sd[p + "conv1.weight"], stride=(1, s, s), padding=1)
            out = F.relu(_bn3(out, sd, p + "bn1", training))
            out = F.conv3d(out, sd[p + "conv2.weight"], stride=1, padding=1)
            out = _bn3(out, sd, p + "bn2", training)
            if (p + "downsample.0.weight") in sd:
                res = F.conv3d(x, sd[p + "downsample.0.weight"], stride=(1, s, s))
                res = _bn3(res, sd, p + "downsample.1", training)
            x = F.relu(out + res)
    return x


def fullmodel_forward(sd, audio: torch.Tensor, video: torch.Tensor, training: bool = True):
    """FullModel.forward (model.py:26-36): audio [(b t),1,F,T], video [b,3,t,H,W] -> (A, logits)."""
    B = audio.shape[0]
    aud = orc.resnet18_forward(sd, "audnet.", audio, "audio", training)
    aud = F.adaptive_max_pool2d(aud, 1).view(B, -1)
    aud = F.normalize(aud, dim=1)
    vid = r3d18_forward(sd, "vidnet.", video, training).detach()  # hook stores output.detach()
    vid = F.normalize(vid, dim=1)
    return orc.hardway_attention(aud, vid)


def trainable_names_tube() -> List[str]:
    """Parameters that receive a gradient on the tube step: the audio trunk only (vidnet is
    detached; audnet.conv1 / conv1_flow / fc are unused on the audio path)."""
    out = []
    for name, _, kind in orc.resnet18_entries("audnet."):
        if kind not in ("conv", "bn_w", "bn_b"):
            continue
        if name.endswith("conv1_flow.weight") or name == "audnet.conv1.weight":
            continue
        out.append(name)
    return out


def tube_train_step(sd, spec: torch.Tensor, video: torch.Tensor, opt: "orc.AdamRef" = None):
    """One train_3D.py step (126-138) on [b,1,F,T] spectrograms + [b,3,t,H,W] clips. Mutates sd."""
    t = video.shape[2]
    audio = repeat_spectrogram(spec, t)
    names = trainable_names_tube()
    leaves = {n: sd[n].detach().clone().requires_grad_(True) for n in names}
    work = OrderedDict(sd)
    work.update(leaves)
    A, logits = fullmodel_forward(work, audio, video, training=True)
    loss = orc.hardway_ce(logits)
    gl = torch.autograd.grad(loss, [leaves[n] for n in names])
    grads: Dict[str, torch.Tensor] = {n: g for n, g in zip(names, gl)}
    if opt is not None:
        with torch.no_grad():
            opt.step({n: sd[n] for n in names}, grads)
    return loss.detach(), A.detach(), logits.detach(), grads


def tube_train_step_per_clip(sd, spec: torch.Tensor, video: torch.Tensor):
    """The de-duplicated form of tube_train_step's forward/backward (what the GPU path runs for a
    per-clip spectrogram batch): the audio trunk over the b distinct spectrograms, its unit vectors
    repeated t times into the head.  BN statistics of the repeated batch equal the distinct batch's
    (the running variance's unbiased factor aside, not exercised here: no Adam, buffers unused).
    Returns (loss, logits, grads) for the identity test against tube_train_step."""
    t = video.shape[2]
    names = trainable_names_tube()
    leaves = {n: sd[n].detach().clone().requires_grad_(True) for n in names}
    work = OrderedDict((k, v.clone()) for k, v in sd.items())
    work.update(leaves)
    b = spec.shape[0]
    aud = orc.resnet18_forward(work, "audnet.", spec, "audio", True)
    aud = F.normalize(F.adaptive_max_pool2d(aud, 1).view(b, -1), dim=1)
    aud = aud.repeat_interleave(t, dim=0)  # '(b t)' rows, b-major (repeat_spectrogram)
    vid = F.normalize(r3d18_forward(work, "vidnet.", video, True).detach(), dim=1)
    A, logits = orc.hardway_attention(aud, vid)
    loss = orc.hardway_ce(logits)
    gl = torch.autograd.grad(loss, [leaves[n] for n in names])
    return loss.detach(), logits.detach(), {n: g for n, g in zip(names, gl)}

"""CPU restatement of the reference hard-way train step — TEST INFRASTRUCTURE ONLY.

This module is the *oracle*: a plain PyTorch-CPU (fp32/fp64) restatement of
the reference's 1-frame audio-visual hard-way step.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / the timed host baseline.  The product path
(``audio-visual-tubes_amd/``) never imports it.

Parity pin: the restatement is checked against golden vectors produced by the
reference itself (``oracle/gen_golden.py`` imports ``/root/reference/model.py``
in the survey container and writes ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.

What it restates (reference file:line):
  * ResNet-18 with modal-selected stem, layer4 stride 1 — models/base_models.py:113-169,
    _forward_impl 195-210, BasicBlock.forward 53-69, conv3x3/conv1x1 23-30.
  * AVENet.__init__ re-init (kaiming fan_out, BN ~ N(1, 0.02)) — model.py:104-110.
  * AVENet.forward: normalise, A / A0 einsums, sigmoid trimap, sim1/sim/sim2,
    logits/0.07, weighted_A — model.py:112-154.
  * HardWayAttention.forward (the 3-D tube head) — model.py:46-60.
  * CrossEntropy(target 0) at the call site — train_hardway_1frame.py:113,130-131.
  * Adam(lr, betas (0.9,0.999), eps 1e-8, coupled L2 weight_decay) —
    train_hardway_1frame.py:116,134 (torch.optim.Adam semantics).
  * nn.DataParallel semantics: per-replica local negatives — model.py:114-115.
  * The 16-frame two-view step: frame/spectrogram folding, two forwards, lw*CE x2,
    (100-lw)*MSE(weighted_A, weighted_A_aug), PropagationLoss x2 — train_hardway.py:126-144,
    losses.py:16-23 (restated from text: losses.py is not importable).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# parameter / buffer inventory (state_dict order of the reference AVENet)
# --------------------------------------------------------------------------------------

STAGES = [(64, 1), (128, 2), (256, 2), (512, 1)]  # (planes, stride); layer4 stride 1 — base_models.py:149


def _bn_entries(prefix: str, c: int) -> List[Tuple[str, tuple, str]]:
    return [
        (prefix + ".weight", (c,), "bn_w"),
        (prefix + ".bias", (c,), "bn_b"),
        (prefix + ".running_mean", (c,), "rm"),
        (prefix + ".running_var", (c,), "rv"),
        (prefix + ".num_batches_tracked", (), "nbt"),
    ]


def resnet18_entries(prefix: str) -> List[Tuple[str, tuple, str]]:
    """state_dict entries of base_models.resnet18 (base_models.py:113-169), in order."""
    e = [
        (prefix + "conv1_a.weight", (64, 1, 7, 7), "conv"),
        (prefix + "conv1.weight", (64, 3, 7, 7), "conv"),
        (prefix + "conv1_flow.weight", (64, 6, 7, 7), "conv"),
    ]
    e += _bn_entries(prefix + "bn1", 64)
    inplanes = 64
    for li, (planes, stride) in enumerate(STAGES, start=1):
        for bi in range(2):
            s = stride if bi == 0 else 1
            p = f"{prefix}layer{li}.{bi}."
            cin = inplanes if bi == 0 else planes
            e.append((p + "conv1.weight", (planes, cin, 3, 3), "conv"))
            e += _bn_entries(p + "bn1", planes)
            e.append((p + "conv2.weight", (planes, planes, 3, 3), "conv"))
            e += _bn_entries(p + "bn2", planes)
            if bi == 0 and (s != 1 or inplanes != planes):
                e.append((p + "downsample.0.weight", (planes, inplanes, 1, 1), "conv"))
                e += _bn_entries(p + "downsample.1", planes)
        inplanes = planes
    e.append((prefix + "fc.weight", (1000, 512), "fc_w"))
    e.append((prefix + "fc.bias", (1000,), "fc_b"))
    return e


def avenet_entries() -> List[Tuple[str, tuple, str]]:
    return resnet18_entries("imgnet.") + resnet18_entries("audnet.")


def make_state(seed: int = 0, dtype=torch.float32) -> "OrderedDict[str, torch.Tensor]":
    """Deterministic weights from a numpy PCG64 seed, following the reference init rule.

    conv: kaiming_normal_(mode='fan_out', nonlinearity='relu') -> N(0, 2/fan_out) (model.py:104-107);
    BN: weight ~ N(1, 0.02), bias 0 (model.py:108-110); running stats 0/1; fc: U(+-1/sqrt(512)).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for name, shape, kind in avenet_entries():
        if kind == "conv":
            fan_out = shape[0] * shape[2] * shape[3]
            a = rng.standard_normal(shape, dtype=np.float64) * math.sqrt(2.0 / fan_out)
        elif kind == "bn_w":
            a = 1.0 + 0.02 * rng.standard_normal(shape, dtype=np.float64)
        elif kind in ("bn_b", "rm"):
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


# --------------------------------------------------------------------------------------
# synthetic inputs
# --------------------------------------------------------------------------------------

def make_image(batch: int, size: int = 224, seed: int = 1) -> torch.Tensor:
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.standard_normal((batch, 3, size, size), dtype=np.float32))


def make_spectrogram(batch: int, freq: int = 257, frames: int = 300, seed: int = 2) -> torch.Tensor:
    """log-spectrogram recipe of datasets/dataloader.py:86-96 on clipped Gaussian noise.

    scipy.signal.spectrogram(nperseg=512, noverlap=1) gives 257 bins; the sample count is
    chosen so the frame count is exactly ``frames`` (511*frames + 1 samples).  Reduced
    frequency sizes (tiny fixtures) keep the first ``freq`` bins.
    """
    from scipy import signal

    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((batch, 1, freq, frames), dtype=np.float32)
    for b in range(batch):
        s = np.clip(0.1 * rng.standard_normal(511 * frames + 1), -1.0, 1.0)
        _, _, spec = signal.spectrogram(s, 16000, nperseg=512, noverlap=1)
        spec = np.log(spec + 1e-7) / 12.0
        out[b, 0] = spec[:freq, :frames].astype(np.float32)
    return torch.from_numpy(out)


def make_tube_features(b: int, t: int, hw: int, c: int, seed: int = 5):
    """Post-ReLU-like normalised features for the HardWayAttention head (fp64)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    vid = torch.from_numpy(np.abs(rng.standard_normal((b, c, t, hw, hw))))
    vid = F.normalize(vid, dim=1)
    aud = torch.from_numpy(np.abs(rng.standard_normal((b * t, c))) + 0.5)
    aud = F.normalize(aud, dim=1)
    return vid, aud


# --------------------------------------------------------------------------------------
# forward
# --------------------------------------------------------------------------------------

class Args:
    """The args namespace AVENet reads (model.py:98-102; defaults train_hardway_1frame.py:54-60)."""

    def __init__(self, epsilon=0.65, epsilon2=0.4, tri_map=True, Neg=True):
        self.epsilon, self.epsilon2, self.tri_map, self.Neg = epsilon, epsilon2, tri_map, Neg


def _bn(x, sd, prefix, training, momentum=0.1, eps=1e-5):
    # BatchNorm2d train mode: biased batch var for normalisation, unbiased var for running stats.
    if training and (prefix + ".num_batches_tracked") in sd:
        sd[prefix + ".num_batches_tracked"].add_(1)
    return F.batch_norm(x, sd[prefix + ".running_mean"], sd[prefix + ".running_var"],
                        sd[prefix + ".weight"], sd[prefix + ".bias"], training, momentum, eps)


def resnet18_forward(sd, prefix: str, x: torch.Tensor, modal: str, training: bool = True):
    """base_models.py:195-210 (stem chosen by modal, layer4 stride 1)."""
    stem = prefix + ("conv1_a.weight" if modal == "audio" else "conv1.weight")
    x = F.conv2d(x, sd[stem], stride=2, padding=3)
    x = F.relu(_bn(x, sd, prefix + "bn1", training))
    x = F.max_pool2d(x, 3, 2, 1)
    inplanes = 64
    for li, (planes, stride) in enumerate(STAGES, start=1):
        for bi in range(2):
            s = stride if bi == 0 else 1
            p = f"{prefix}layer{li}.{bi}."
            idt = x
            out = F.conv2d(x, sd[p + "conv1.weight"], stride=s, padding=1)
            out = F.relu(_bn(out, sd, p + "bn1", training))
            out = F.conv2d(out, sd[p + "conv2.weight"], stride=1, padding=1)
            out = _bn(out, sd, p + "bn2", training)
            if (p + "downsample.0.weight") in sd:
                idt = F.conv2d(x, sd[p + "downsample.0.weight"], stride=s)
                idt = _bn(idt, sd, p + "downsample.1", training)
            x = F.relu(out + idt)
        inplanes = planes
    return x


def hardway_head(img_n: torch.Tensor, aud_n: torch.Tensor, epsilon=0.65, epsilon2=0.4, tau=0.03,
                 tri_map=True, neg=True):
    """model.py:114-154 given the normalised maps: img_n [B,C,h,w], aud_n [B,C]."""
    B = img_n.shape[0]
    mask = 1 - 100 * torch.eye(B, B, dtype=img_n.dtype)
    A = torch.einsum("ncqa,nc->nqa", img_n, aud_n).unsqueeze(1)             # model.py:124
    A0 = torch.einsum("ncqa,kc->nkqa", img_n, aud_n)                         # model.py:125
    Pos = torch.sigmoid((A - epsilon) / tau)
    if tri_map:
        Neg = 1 - torch.sigmoid((A - epsilon2) / tau)
    else:
        Neg = 1 - Pos
    Pos_all = torch.sigmoid((A0 - epsilon) / tau)
    sim1 = (Pos * A).flatten(2).sum(-1) / Pos.flatten(2).sum(-1)
    sim = ((Pos_all * A0).flatten(2).sum(-1) / Pos_all.flatten(2).sum(-1)) * mask
    sim2 = (Neg * A).flatten(2).sum(-1) / Neg.flatten(2).sum(-1)
    logits = torch.cat((sim1, sim, sim2), 1) / 0.07 if neg else torch.cat((sim1, sim), 1) / 0.07
    norm_pos = F.normalize(Pos, dim=(2, 3))
    weighted_A = (img_n * norm_pos).mean(dim=1)
    return A, logits, weighted_A, Pos, Neg


def avenet_forward(sd, image, audio, args: Args = None, training: bool = True):
    """AVENet.forward (model.py:112-154). Returns (A, logits, weighted_A, Pos, Neg)."""
    args = args or Args()
    img = resnet18_forward(sd, "imgnet.", image, "vision", training)
    img = F.normalize(img, dim=1)
    aud = resnet18_forward(sd, "audnet.", audio, "audio", training)
    aud = F.adaptive_max_pool2d(aud, 1).flatten(1)
    aud = F.normalize(aud, dim=1)
    return hardway_head(img, aud, args.epsilon, args.epsilon2, 0.03, args.tri_map, args.Neg)


def hardway_attention(audio_features, video_features):
    """HardWayAttention.forward (model.py:46-60): aud [(b t), C], vid [b, C, t, h, w]."""
    b, c, t, h, w = video_features.shape
    vid = video_features.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    A, logits, _, _, _ = hardway_head(vid, audio_features, 0.65, 0.4, 0.03, True, True)
    return A, logits


def hardway_ce(logits: torch.Tensor) -> torch.Tensor:
    """nn.CrossEntropyLoss()(logits, zeros) — train_hardway_1frame.py:113,130-131."""
    target = torch.zeros(logits.shape[0], dtype=torch.long)
    return F.cross_entropy(logits, target)


# --------------------------------------------------------------------------------------
# train step (fwd + CE + bwd + Adam)
# --------------------------------------------------------------------------------------

def trainable_names(sd) -> List[str]:
    """Parameters that receive gradients on the 1-frame step (the stems of the other
    modality, conv1_flow and both fc never do — SURVEY §7 'Unused parameters')."""
    out = []
    for name, _, kind in avenet_entries():
        if kind not in ("conv", "bn_w", "bn_b"):
            continue
        if name.endswith("conv1_flow.weight"):
            continue
        if name.startswith("imgnet.") and name.endswith("conv1_a.weight"):
            continue
        if name.startswith("audnet.") and name.endswith("conv1.weight") and ".layer" not in name:
            continue
        out.append(name)
    return out


class AdamRef:
    """torch.optim.Adam (single-tensor, amsgrad=False, coupled weight decay) restated."""

    def __init__(self, lr=1e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4):
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.state: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
        self.t = 0

    def step(self, params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor]):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        step_size = self.lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        for name, p in params.items():
            g = grads[name]
            if self.wd != 0:
                g = g + self.wd * p
            m, v = self.state.get(name, (torch.zeros_like(p), torch.zeros_like(p)))
            m = m * self.b1 + (1 - self.b1) * g
            v = v * self.b2 + (1 - self.b2) * g * g
            self.state[name] = (m, v)
            denom = v.sqrt() / bc2_sqrt + self.eps
            p -= step_size * m / denom


def train_step(sd, image, audio, opt: AdamRef = None, args: Args = None):
    """One hard-way step: forward, CE(target 0), backward, Adam. Mutates ``sd`` in place.

    Returns (loss, logits, grads) with grads keyed by parameter name.
    """
    names = trainable_names(sd)
    leaves = {n: sd[n].detach().clone().requires_grad_(True) for n in names}
    work = OrderedDict(sd)
    work.update(leaves)
    _, logits, _, _, _ = avenet_forward(work, image, audio, args, training=True)
    loss = hardway_ce(logits)
    gl = torch.autograd.grad(loss, [leaves[n] for n in names])
    grads = {n: g for n, g in zip(names, gl)}
    # BN running stats / num_batches_tracked were updated in place (shared tensors with sd)
    if opt is not None:
        with torch.no_grad():
            opt.step({n: sd[n] for n in names}, grads)
    return loss.detach(), logits.detach(), grads


# --------------------------------------------------------------------------------------
# 16-frame two-view step (train_hardway.py:126-144)
# --------------------------------------------------------------------------------------

def propagation_loss(heatmap: torch.Tensor) -> torch.Tensor:
    """PropagationLoss.forward (losses.py:22-23) on heatmap [b, t, h, w].  losses.py is not
    importable here (`from turtle import pos`, pytorch_metric_learning, torchvision: SURVEY §8c),
    so this one-liner is restated from its text."""
    return torch.abs(torch.diff(heatmap, dim=1)).mean(dim=(2, 3)).mean(dim=1).mean(dim=0)


def npratio_loss(heatmap: torch.Tensor) -> torch.Tensor:
    """NPRatio.forward (losses.py:13-14) on heatmap [b, t, h, w], restated from its text (losses.py is
    not importable here: SURVEY §8c)."""
    return torch.abs(torch.diff(torch.sum(heatmap, dim=(2, 3)), dim=1)).mean(dim=1).mean(dim=0)


def flip_loss(heatmap: torch.Tensor, flipped_heatmap: torch.Tensor) -> torch.Tensor:
    """FlipLoss.forward (losses.py:34-36): nn.L1Loss()(flipped_heatmap, RandomHorizontalFlip(p=1)(heatmap));
    torchvision's tensor hflip is heatmap.flip(-1) (torchvision is absent here: restated)."""
    return F.l1_loss(flipped_heatmap, heatmap.flip(-1))


def twoview_losses(out1, out2, b: int, t: int, loss_weight: float = 0.1):
    """train_hardway.py:134-142 given the two AVENet outputs (A, logits, weighted_A, Pos, Neg).
    weighted.reshape(batch_size, frame_density, 14, 14) is written for the layer4 map's own (h, w).
    Returns (combined, hardway, aug, l2, consistency)."""
    _, logits1, w1, _, _ = out1
    _, logits2, w2, _, _ = out2
    hardway = hardway_ce(logits1) * loss_weight
    aug = hardway_ce(logits2) * loss_weight
    l2 = F.mse_loss(w1, w2) * (100 - loss_weight)
    h, w = w1.shape[-2:]
    consistency = propagation_loss(w1.reshape(b, t, h, w)) + propagation_loss(w2.reshape(b, t, h, w))
    combined = (hardway + aug) / 2 + l2 + consistency
    return combined, hardway, aug, l2, consistency


def fold_frames(frames: torch.Tensor) -> torch.Tensor:
    """einops 'b c t h w -> (b t) c h w' (train_hardway.py:130-131)."""
    b, c, t, h, w = frames.shape
    return frames.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)


def fold_spec(spec: torch.Tensor, t: int) -> torch.Tensor:
    """spec.unsqueeze(2).repeat(1, 1, t, 1, 1) then 'b c t h w -> (b t) c h w' (train_hardway.py:128-129)."""
    return fold_frames(spec.unsqueeze(2).repeat(1, 1, t, 1, 1))


def twoview_step(sd, frames, augmented, spec, opt: AdamRef = None, args: Args = None, loss_weight: float = 0.1):
    """One train_hardway.py step (126-144): two AVENet forwards (frames, augmented) on the 16x
    repeated spectrogram, the combined loss, backward, Adam.  Mutates ``sd`` (BN buffers are updated
    by both forwards; Adam if ``opt``).  frames/augmented [b,3,t,H,W], spec [b,1,F,T].
    Returns (losses (combined, hardway, aug, l2, consistency), out1, out2, grads)."""
    b, t = frames.shape[0], frames.shape[2]
    names = trainable_names(sd)
    leaves = {n: sd[n].detach().clone().requires_grad_(True) for n in names}
    work = OrderedDict(sd)
    work.update(leaves)
    aud = fold_spec(spec, t)
    out1 = avenet_forward(work, fold_frames(frames), aud, args, training=True)
    out2 = avenet_forward(work, fold_frames(augmented), aud, args, training=True)
    losses = twoview_losses(out1, out2, b, t, loss_weight)
    gl = torch.autograd.grad(losses[0], [leaves[n] for n in names])
    grads = {n: g for n, g in zip(names, gl)}
    if opt is not None:
        with torch.no_grad():
            opt.step({n: sd[n] for n in names}, grads)
    return (tuple(x.detach() for x in losses), tuple(o.detach() for o in out1), tuple(o.detach() for o in out2),
            grads)


def make_frames(b: int, t: int, size: int = 224, seed: int = 3) -> torch.Tensor:
    """Seeded synthetic clip frames [b,3,t,H,W] (ImageNet-normalised range, like make_image)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.standard_normal((b, 3, t, size, size), dtype=np.float32))

"""Drop-in ``AVENet`` (reference model.py:87-154) on the MI355X engine.

Same constructor (``AVENet(args, pretrained)``; args needs epsilon, epsilon2, tri_map, Neg), same
module tree and state_dict keys (``imgnet.*`` / ``audnet.*`` incl. the unused ``conv1_flow``,
other-modality stem and ``fc``), same init rule and RNG consumption order (so
``torch.manual_seed(s)`` gives the reference's weights), same forward signature and outputs
``(A, logits, weighted_A, Pos, Neg)``; gradients flow from ``logits`` and ``weighted_A`` through autograd into the
Parameters.  Compute runs in libavt (HIP, gfx950); there is no CPU path.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .engine import AVEngine, FlatStore, trainable

# ---------------------------------------------------------------------------------------------
# module shells: exactly the reference's module tree (models/base_models.py:32-69, 113-193)
# ---------------------------------------------------------------------------------------------


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride


class ResNet(nn.Module):
    """Parameter/buffer holder of base_models.ResNet(BasicBlock, [2,2,2,2], modal). Its compute
    runs inside AVENet's engine; calling it alone is not supported."""

    def __init__(self, modal: str):
        super().__init__()
        self.inplanes = 64
        self.modal = modal
        self.conv1_a = nn.Conv2d(1, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.conv1_flow = nn.Conv2d(6, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, 2, 1)
        self.layer2 = self._make_layer(128, 2, 2)
        self.layer3 = self._make_layer(256, 2, 2)
        self.layer4 = self._make_layer(512, 2, 1)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, 1000)
        for m in self.modules():  # base_models.py:158-163
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(BasicBlock(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):  # pragma: no cover - documented limitation
        raise RuntimeError("avt: the trunks run inside AVENet.forward (fused engine); call the parent model")


def resnet18(pretrained=False, progress=True, modal="vision", **kwargs):
    """base_models.resnet18 (the reference ignores `pretrained`, base_models.py:217-220)."""
    return ResNet(modal)


# ---------------------------------------------------------------------------------------------
# autograd bridge
# ---------------------------------------------------------------------------------------------


class _AVENetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine: AVEngine, training: bool, image, audio, *params):
        out, tape = engine.forward(image, audio, training)
        ctx.engine = engine
        ctx.tape = tape
        ctx.n_params = len(params)
        ctx.set_materialize_grads(False)
        return out["A"], out["logits"], out["weighted_A"], out["Pos"], out["Neg"]

    @staticmethod
    def backward(ctx, gA, glogits, gwA, gPos, gNeg):
        # the reference's train scripts back-propagate logits (CE, train_hardway_1frame.py:130-131) and
        # weighted_A (MSE + PropagationLoss, train_hardway.py:138-141); A/Pos/Neg only feed eval/logging
        for name, g in (("A", gA), ("Pos", gPos), ("Neg", gNeg)):
            if g is not None and bool(torch.any(g != 0)):
                raise NotImplementedError(
                    f"avt: gradients through `{name}` are not implemented (no reference train script "
                    "back-propagates it; see DESIGN.md)")
        engine: AVEngine = ctx.engine
        if ctx.tape is None:
            raise RuntimeError("avt: backward through an eval-mode forward (or a second backward)")
        nparams = ctx.n_params
        if glogits is None and gwA is None:
            return (None, None, None, None) + (None,) * nparams
        flat = engine.flat
        dev = (glogits if glogits is not None else gwA).device
        gflat = torch.zeros(flat.n_train, device=dev, dtype=torch.float32)
        engine.backward(ctx.tape, glogits, gflat, dwA=gwA)
        ctx.tape = None
        views = flat.param_grad_views(gflat)
        grads = tuple(views.get(n) for n in flat.pnames[:nparams])
        return (None, None, None, None) + grads


class AVENet(nn.Module):
    """model.py:87-154 on libavt."""

    def __init__(self, args, pretrained=False):
        super().__init__()
        self.imgnet = resnet18(modal="vision", pretrained=pretrained)
        self.audnet = resnet18(modal="audio", pretrained=pretrained)
        self.m = nn.Sigmoid()
        self.avgpool = nn.AdaptiveMaxPool2d((1, 1))
        self.epsilon = args.epsilon
        self.epsilon2 = args.epsilon2
        self.tau = 0.03
        self.trimap = args.tri_map
        self.Neg = args.Neg
        for m in self.modules():  # model.py:104-110
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.normal_(m.weight, mean=1, std=0.02)
                nn.init.constant_(m.bias, 0)
        self._flat = FlatStore(self)
        self._engine: Optional[AVEngine] = None

    # -- storage management: keep the flat buffers when moved (.cuda(), .to(dev)) --
    def _apply(self, fn, recurse=True):
        self._flat.apply(fn)
        self._engine = None
        return self

    def engine(self) -> AVEngine:
        if self._engine is None:
            self._engine = AVEngine(self._flat, self.epsilon, self.epsilon2, self.tau, self.trimap, self.Neg)
        e = self._engine
        e.epsilon, e.epsilon2, e.tau, e.tri_map, e.neg = self.epsilon, self.epsilon2, self.tau, self.trimap, self.Neg
        return e

    def ordered_parameters(self):
        mods = dict(self.named_parameters())
        return [mods[n] for n in self._flat.pnames]

    def forward(self, image, audio):
        eng = self.engine()
        params = self.ordered_parameters()
        n_train = sum(1 for n in self._flat.pnames if trainable(n))
        train_params = params[:n_train]
        need_grad = torch.is_grad_enabled() and self.training and any(p.requires_grad for p in train_params)
        if need_grad:
            A, logits, wA, Pos, Neg = _AVENetFunction.apply(eng, True, image, audio, *train_params)
        else:
            out, _ = eng.forward(image, audio, self.training)
            A, logits, wA, Pos, Neg = out["A"], out["logits"], out["weighted_A"], out["Pos"], out["Neg"]
        hooks = self.imgnet.layer4._forward_hooks
        if hooks:
            self._run_layer4_hooks()
        return A, logits, wA, Pos, Neg

    def _run_layer4_hooks(self):  # test.py:63 registers a forward hook on imgnet.layer4
        raise NotImplementedError("avt: forward hooks on imgnet.layer4 are not supported yet")


# ---------------------------------------------------------------------------------------------
# 3-D tube model (model.py:17-60; BASELINE config 4)
# ---------------------------------------------------------------------------------------------


class HardWayAttention(nn.Module):
    """model.py:38-60.  Standalone use takes fp32 features (the video map is rounded to bf16 on its
    way to the head kernel, the precision FullModel's trunk produces it in); inside FullModel the
    head runs fused on the trunk outputs."""

    def __init__(self):
        super().__init__()
        self.sigmoid = nn.Sigmoid()
        self.epsilon = 0.65
        self.epsilon2 = 0.4
        self.tau = 0.03

    def forward(self, audio_features, video_features):
        from ._lib import call, query
        from .trunk import P, stream_ptr

        if not video_features.is_cuda or not audio_features.is_cuda:
            raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        b, C, t, h, w = video_features.shape
        B, Pn = b * t, h * w
        if tuple(audio_features.shape) != (B, C):
            raise ValueError(f"avt: audio_features must be [{B},{C}], got {tuple(audio_features.shape)}")
        dev = video_features.device
        # '(b t) h w c' bf16 — the FullModel trunk's output layout
        v = video_features.detach().permute(0, 2, 3, 4, 1).contiguous().to(torch.bfloat16)
        an = audio_features.detach().float().contiguous()
        f32 = dict(device=dev, dtype=torch.float32)
        inv, vsum = torch.empty(B, Pn, **f32), torch.empty(B, Pn, **f32)
        A0 = torch.empty(B, Pn, B, **f32)
        save = torch.empty(int(query("avt_hardway_save_floats", B)), **f32)
        logits = torch.empty(B, B + 2, **f32)
        A, Pos, Neg = (torch.empty(B, 1, h, w, **f32) for _ in range(3))
        wA = torch.empty(B, h, w, **f32)
        call("avt_hardway_fwd", P(v), P(an), B, Pn, C, self.epsilon, self.epsilon2, self.tau, 1, 1, P(inv), P(vsum),
             P(A0), P(save), P(logits), P(A), P(Pos), P(Neg), P(wA), stream_ptr())
        return A, logits


class _FullModelFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, training: bool, audio, video, *params):
        out, tape = engine.forward(audio, video, training)
        ctx.engine, ctx.tape, ctx.n_params = engine, tape, len(params)
        ctx.set_materialize_grads(False)
        return out["A"], out["logits"]

    @staticmethod
    def backward(ctx, gA, glogits):
        if gA is not None and bool(torch.any(gA != 0)):
            raise NotImplementedError("avt: gradients through `A` are not implemented (train_3D.py back-propagates "
                                      "the logits CE only)")
        nparams = ctx.n_params
        if glogits is None:
            return (None, None, None, None) + (None,) * nparams
        engine = ctx.engine
        flat = engine.flat
        gflat = torch.zeros(flat.n_train, device=glogits.device, dtype=torch.float32)
        engine.backward(ctx.tape, glogits, gflat)
        ctx.tape = None
        views = flat.param_grad_views(gflat)
        return (None, None, None, None) + tuple(views.get(n) for n in flat.pnames[:nparams])


class FullModel(nn.Module):
    """model.py:17-36 on libavt: R3D-18 ``vidnet`` (forward only; its layer4 is detached as the
    reference's forward hook does), audio ResNet-18 ``audnet``, AdaptiveMaxPool2d + normalize,
    HardWayAttention.  ``forward(audio, video) -> (A, logits)`` with audio either the folded
    repeated spectrogram [b*t,1,F,T] (the reference call, train_3D.py:128-131) or one spectrogram
    per clip [b,1,F,T] (de-duplicated audio trunk, exact; tube.py)."""

    def __init__(self, args=None):
        super().__init__()
        from .resnet3D import generate_model

        self.vidnet = generate_model(model_depth=18, no_max_pool=True, n_classes=1039)
        self.audnet = resnet18(modal="audio")
        self.avgpool = nn.AdaptiveMaxPool2d((1, 1))
        self.attention = HardWayAttention()
        from .tube import tube_trainable

        self._flat = FlatStore(self, tube_trainable)
        self._engine = None

    def _apply(self, fn, recurse=True):
        self._flat.apply(fn)
        self._engine = None
        return self

    def engine(self):
        if self._engine is None:
            from .tube import TubeEngine

            self._engine = TubeEngine(self._flat)
        return self._engine

    def forward(self, audio, video):
        eng = self.engine()
        named = dict(self.named_parameters())
        n_train = sum(1 for n in self._flat.pnames if self._flat.trainable(n))
        train_params = [named[n] for n in self._flat.pnames[:n_train]]
        if torch.is_grad_enabled() and self.training and any(p.requires_grad for p in train_params):
            return _FullModelFunction.apply(eng, True, audio, video, *train_params)
        out, _ = eng.forward(audio, video, self.training)
        return out["A"], out["logits"]

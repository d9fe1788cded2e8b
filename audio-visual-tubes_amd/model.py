"""Drop-in ``AVENet`` (reference model.py:87-154) on the MI355X engine.

Same constructor (``AVENet(args, pretrained)``; args needs epsilon, epsilon2, tri_map, Neg), same
module tree and state_dict keys (``imgnet.*`` / ``audnet.*`` incl. the unused ``conv1_flow``,
other-modality stem and ``fc``), same init rule and RNG consumption order (so
``torch.manual_seed(s)`` gives the reference's weights), same forward signature and outputs
``(A, logits, weighted_A, Pos, Neg)``; gradients flow from ``logits`` through autograd into the
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
        for name, g in (("A", gA), ("weighted_A", gwA), ("Pos", gPos), ("Neg", gNeg)):
            if g is not None and bool(torch.any(g != 0)):
                raise NotImplementedError(
                    f"avt: gradients through `{name}` are not implemented yet (the 1-frame hard-way "
                    "step only back-propagates the logits; see DESIGN.md §next)")
        engine: AVEngine = ctx.engine
        if ctx.tape is None:
            raise RuntimeError("avt: backward through an eval-mode forward")
        nparams = ctx.n_params
        if glogits is None:
            return (None, None, None, None) + (None,) * nparams
        flat = engine.flat
        gflat = torch.zeros(flat.n_train, device=glogits.device, dtype=torch.float32)
        engine.backward(ctx.tape, glogits, gflat)
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

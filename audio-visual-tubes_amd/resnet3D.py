"""Module shells of the R3D-18 video trunk (reference models/resnet3D.py), for FullModel.vidnet.

Same module tree, construction order and init as ``resnet3D.generate_model(18, no_max_pool=True,
n_classes=1039)`` (model.py:20; resnet3D.py:103-234), so ``torch.manual_seed(s)`` gives the
reference's weights and ``state_dict`` keys/shapes match (``vidnet.conv1.weight`` [64,3,7,7,7],
``vidnet.layerL.B.downsample.{0,1}.*``, ``vidnet.fc.*``).  Inside FullModel the compute runs in its
engine (tube.py); called on its own (``FullModel.vidnet(video)`` or a standalone
``generate_model(18, ...)``, with the stem max-pool or without) the same kernels run through tube.R3DEngine and return
the ``fc`` logits as resnet3D.ResNet.forward does (resnet3D.py:197-213).  Forward only: the build
computes no gradients for the video trunk (FullModel detaches it), so a call that would need them raises.
"""
from __future__ import annotations

import weakref

import torch
from torch import nn


def get_inplanes():
    return [64, 128, 256, 512]


def conv3x3x3(in_planes, out_planes, stride=1):
    return nn.Conv3d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1x1(in_planes, out_planes, stride=1):
    return nn.Conv3d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3x3(in_planes, planes, stride)
        self.bn1 = nn.BatchNorm3d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3x3(planes, planes)
        self.bn2 = nn.BatchNorm3d(planes)
        self.downsample = downsample
        self.stride = stride


class ResNet(nn.Module):
    """resnet3D.ResNet(BasicBlock, layers, ...) parameter/buffer holder (shortcut 'B' only)."""

    def __init__(self, block, layers, block_inplanes, n_input_channels=3, conv1_t_size=7, conv1_t_stride=1,
                 no_max_pool=False, shortcut_type="B", widen_factor=1.0, n_classes=400):
        super().__init__()
        if shortcut_type != "B" or block is not BasicBlock or conv1_t_stride != 1:
            raise NotImplementedError("avt: R3D with BasicBlock, shortcut 'B' and temporal stride 1 only "
                                      "(the FullModel configuration, model.py:20)")
        block_inplanes = [int(x * widen_factor) for x in block_inplanes]
        self.in_planes = block_inplanes[0]
        self.no_max_pool = no_max_pool
        self.conv1 = nn.Conv3d(n_input_channels, self.in_planes, kernel_size=(conv1_t_size, 7, 7),
                               stride=(conv1_t_stride, 2, 2), padding=(conv1_t_size // 2, 3, 3), bias=False)
        self.bn1 = nn.BatchNorm3d(self.in_planes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool3d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, block_inplanes[0], layers[0])
        self.layer2 = self._make_layer(block, block_inplanes[1], layers[1], stride=(1, 2, 2))
        self.layer3 = self._make_layer(block, block_inplanes[2], layers[2], stride=(1, 2, 2))
        self.layer4 = self._make_layer(block, block_inplanes[3], layers[3], stride=(1, 2, 2))
        self.avgpool = nn.AdaptiveAvgPool3d((1, 1, 1))
        self.fc = nn.Linear(block_inplanes[3] * block.expansion, n_classes)
        for m in self.modules():  # resnet3D.py:152-158
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm3d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self._avt_parent = None  # (weakref to the owning FullModel, prefix) once adopted
        self._avt_engine = None
        self._own_flat = None  # a standalone module's flat storage, created at its first .to() / forward

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None  # built before the block, as resnet3D.py:169-184 (RNG order)
        if stride != 1 or self.in_planes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1x1(self.in_planes, planes * block.expansion, stride),
                                       nn.BatchNorm3d(planes * block.expansion))
        layers = [block(in_planes=self.in_planes, planes=planes, stride=stride, downsample=downsample)]
        self.in_planes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.in_planes, planes))
        return nn.Sequential(*layers)

    def _adopt(self, parent, prefix: str):
        self._avt_parent = (weakref.ref(parent), prefix)
        self._own_flat = None
        self._avt_engine = None

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_avt_engine"] = None
        return state

    def _flat_store(self):
        from .engine import FlatStore

        if self._own_flat is None:
            self._own_flat = FlatStore(self, lambda n: False)  # nothing of the video trunk is trained here
        return self._own_flat

    def _apply(self, fn, recurse=True):
        if self._avt_parent is not None and self._avt_parent[0]() is not None:
            self._avt_parent[0]()._apply(fn)
            return self
        self._flat_store().apply(fn)
        self._avt_engine = None
        return self

    def forward(self, x):
        """resnet3D.ResNet.forward (resnet3D.py:197-213): x fp32 [b,3,t,H,W] -> fc logits [b, n_classes]."""
        from .tube import R3DEngine

        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            raise NotImplementedError("avt: the R3D trunk is forward-only in this build (FullModel detaches it); "
                                      "call it under torch.no_grad() or with requires_grad_(False) parameters")
        if self._avt_parent is not None:
            parent, prefix = self._avt_parent[0](), self._avt_parent[1]
            if parent is None or getattr(parent, prefix.rstrip("."), None) is not self:
                raise RuntimeError("avt: this R3D trunk is no longer its parent's (a copied trunk; copy the whole model)")
            flat = parent._flat
        else:
            prefix, flat = "", self._flat_store()
        if self._avt_engine is None or self._avt_engine.flat is not flat:
            self._avt_engine = R3DEngine(flat, prefix, max_pool=not self.no_max_pool)
        return self._avt_engine.forward(x, self.training)


def generate_model(model_depth, **kwargs):
    if model_depth != 18:
        raise NotImplementedError("avt: only the R3D-18 used by FullModel (model.py:20) is built")
    return ResNet(BasicBlock, [2, 2, 2, 2], get_inplanes(), **kwargs)

"""Drop-in ``AVENet`` (reference model.py:87-154) on the MI355X engine.

Same constructor (``AVENet(args, pretrained)``; args needs epsilon, epsilon2, tri_map, Neg), same
module tree and state_dict keys (``imgnet.*`` / ``audnet.*`` incl. the unused ``conv1_flow``,
other-modality stem and ``fc``), same init rule and RNG consumption order (so
``torch.manual_seed(s)`` gives the reference's weights), same forward signature and outputs
``(A, logits, weighted_A, Pos, Neg)``; gradients flow from ``logits`` and ``weighted_A`` through autograd into the
Parameters.  Compute runs in libavt (HIP, gfx950); there is no CPU path.
"""
from __future__ import annotations

import weakref
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
    """base_models.ResNet(BasicBlock, [2,2,2,2], modal) on libavt.  Inside an AVENet its parameters are
    views of the parent's flat storage; constructed on its own it keeps a flat store of its own.
    ``forward(x)`` (base_models.py:195-213) returns the layer4 map [N,512,h,w] fp32 with gradients
    into the parameters, and into x when x requires grad (avt_conv_stem_dgrad)."""

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
        self._avt_parent = None  # (weakref to the owning AVENet, prefix) once adopted
        self._avt_engine = None
        # a standalone trunk's flat storage is created at its first .to()/.cuda() (or forward): creating
        # it here would turn the parameters into channels_last views before an enclosing AVENet re-inits
        # them (model.py:104-110), and normal_ fills a channels_last view in another element order
        self._own_flat = None

    def _make_layer(self, planes, blocks, stride):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(BasicBlock(self.inplanes, planes))
        return nn.Sequential(*layers)

    def _trainable(self, name: str) -> bool:
        """Parameters the standalone forward uses: the modal stem (base_models.py:197-200), bn1,
        layer1-4; never conv1_flow, the other stem, fc."""
        if name.startswith("fc.") or name == "conv1_flow.weight":
            return False
        return name != ("conv1.weight" if self.modal == "audio" else "conv1_a.weight")

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_avt_engine"] = None
        return state

    def _adopt(self, parent, prefix: str):
        """Called by the owning AVENet once its flat store holds this trunk's parameters."""
        self._avt_parent = (weakref.ref(parent), prefix)
        self._own_flat = None
        self._avt_engine = None

    def _flat_store(self) -> FlatStore:
        if self._own_flat is None:
            self._own_flat = FlatStore(self, lambda n, s=self: s._trainable(n))
        return self._own_flat

    def _apply(self, fn, recurse=True):
        if self._avt_parent is not None and self._avt_parent[0]() is not None:
            self._avt_parent[0]()._apply(fn)
            return self
        self._flat_store().apply(fn)
        self._avt_engine = None
        return self

    def _engine_and_params(self):
        from .engine import TrunkEngine

        if self._avt_parent is not None:
            parent, prefix = self._avt_parent[0](), self._avt_parent[1]
            if parent is None:
                raise RuntimeError("avt: the AVENet owning this trunk no longer exists")
            if getattr(parent, prefix.rstrip("."), None) is not self:
                raise RuntimeError("avt: this trunk is no longer its parent's (a copied trunk; copy the whole model)")
            flat = parent._flat
        else:
            parent, prefix, flat = self, "", self._flat_store()
        if self._avt_engine is None or self._avt_engine.flat is not flat:
            self._avt_engine = TrunkEngine(flat, prefix, self.modal)
        named = dict(parent.named_parameters())
        names = [n for n in flat.pnames if flat.trainable(n) and n.startswith(prefix)]
        return self._avt_engine, flat, names, [named[n] for n in names]

    def forward(self, x):
        eng, flat, names, params = self._engine_and_params()
        need_grad = torch.is_grad_enabled() and (x.requires_grad or (self.training and any(p.requires_grad for p in params)))
        if need_grad and not self.training:
            raise NotImplementedError("avt: gradients through an eval-mode trunk are not computed (train-mode "
                                      "BatchNorm only)")
        if need_grad:
            return _TrunkFunction.apply(eng, names, x, *params)
        out, _ = eng.forward(x, self.training)
        return out


class _TrunkFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, names, x, *params):
        out, tape = engine.forward(x, True)
        tape["want_dx"] = ctx.needs_input_grad[2]  # d(loss)/d(x) through the 7x7 stem (avt_conv_stem_dgrad)
        ctx.engine, ctx.tape, ctx.names = engine, tape, names
        ctx.set_materialize_grads(False)
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return (None, None, None) + (None,) * len(ctx.names)
        if ctx.tape is None:
            raise RuntimeError("avt: second backward through a trunk forward")
        flat = ctx.engine.flat
        gflat = torch.zeros(flat.n_train, device=g.device, dtype=torch.float32)
        gx = ctx.engine.backward(ctx.tape, g, gflat)
        ctx.tape = None
        views = flat.param_grad_views(gflat)
        return (None, None, gx) + tuple(views[n] for n in ctx.names)


class HardWayArgs:
    """The argparse fields AVENet reads (model.py:98-102), with train_hardway_1frame.py:54-60's
    defaults (--epsilon 0.65, --epsilon2 0.4, --tri_map / --Neg store_true default True)."""

    def __init__(self, epsilon=0.65, epsilon2=0.4, tri_map=True, Neg=True):
        self.epsilon, self.epsilon2, self.tri_map, self.Neg = epsilon, epsilon2, tri_map, Neg


def resnet18(pretrained=False, progress=True, modal="vision", **kwargs):
    """base_models.resnet18 (the reference ignores `pretrained`, base_models.py:217-220)."""
    return ResNet(modal)


# ---------------------------------------------------------------------------------------------
# autograd bridge
# ---------------------------------------------------------------------------------------------


def _nhwc_to_nchw_f32(x: torch.Tensor) -> torch.Tensor:
    """NHWC bf16 trunk map -> NCHW fp32 (the reference layout/dtype of a ResNet layer output)."""
    from ._lib import call
    from .trunk import P, stream_ptr

    N, H, W, C = x.shape
    y = torch.empty(N, C, H, W, device=x.device, dtype=torch.float32)
    call("avt_nhwc_bf16_to_nchw", P(x), P(y), N, C, H * W, stream_ptr())
    return y


# the only module hooks the fused engine can honour: forward hooks on each trunk's layer4 (test.py:63
# registers one on imgnet.layer4 and reads its output for the layer-4 activation map, test.py:103)
_HOOKABLE = ("imgnet.layer4", "audnet.layer4")


def _check_hooks(model: nn.Module):
    """Raise (before any state changes) on module hooks the fused engine cannot honour."""
    for name, m in model.named_modules():
        if not name.startswith(("imgnet", "audnet")):
            continue
        bad = bool(m._forward_pre_hooks) or bool(getattr(m, "_backward_hooks", None)) or bool(
            getattr(m, "_backward_pre_hooks", None))
        if m._forward_hooks and name not in _HOOKABLE:
            bad = True
        if bad:
            raise NotImplementedError(
                f"avt: hooks on `{name}` are not supported: the trunks run fused on the GPU; forward hooks "
                f"are honoured on {', '.join(_HOOKABLE)} only")


def _run_forward_hooks(module: nn.Module, inp: torch.Tensor, out: torch.Tensor):
    """Call module's forward hooks as nn.Module.__call__ would: hook(module, (input,), output).  A hook
    that returns a replacement output is not supported (the head already consumed the map)."""
    for hid, hook in list(module._forward_hooks.items()):
        if module._forward_hooks_with_kwargs.get(hid, False):
            res = hook(module, (inp,), {}, out)
        else:
            res = hook(module, (inp,), out)
        if res is not None:
            raise NotImplementedError("avt: a forward hook on layer4 returned a replacement output; only "
                                      "observing hooks (returning None) are supported")


class _AVENetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine: AVEngine, training: bool, sink: Optional[dict], image, audio, *params):
        out, tape = engine.forward(image, audio, training, layer_io=sink is not None)
        if sink is not None:
            sink.update(out)
        if tape is not None:  # d(loss)/d(frames, spectrogram) through the 7x7 stems when the inputs require it
            tape["img"]["want_dx"] = ctx.needs_input_grad[3]
            tape["aud"]["want_dx"] = ctx.needs_input_grad[4]
        ctx.engine = engine
        ctx.tape = tape
        ctx.n_params = len(params)
        ctx.set_materialize_grads(False)
        return out["A"], out["logits"], out["weighted_A"], out["Pos"], out["Neg"]

    @staticmethod
    def backward(ctx, gA, glogits, gwA, gPos, gNeg):
        engine: AVEngine = ctx.engine
        if ctx.tape is None:
            raise RuntimeError("avt: backward through an eval-mode forward (or a second backward)")
        nparams = ctx.n_params
        if glogits is None and gwA is None and gA is None and gPos is None and gNeg is None:
            return (None,) * 5 + (None,) * nparams
        flat = engine.flat
        dev = next(g for g in (glogits, gwA, gA, gPos, gNeg) if g is not None).device
        gflat = torch.zeros(flat.n_train, device=dev, dtype=torch.float32)
        engine.backward(ctx.tape, glogits, gflat, dwA=gwA, dA=gA, dPos=gPos, dNeg=gNeg)
        gimg, gaud = ctx.tape["img"].get("dx"), ctx.tape["aud"].get("dx")
        ctx.tape = None
        views = flat.param_grad_views(gflat)
        grads = tuple(views.get(n) for n in flat.pnames[:nparams])
        return (None, None, None, gimg, gaud) + grads


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
        # engines by device index: the model's own (over self._flat) and, for nn.DataParallel replicas on
        # other GPUs, one over a mirror of the flat store there.  A dict, so that replicas (which get a
        # shallow copy of this __dict__) create and find them in the model's cache.
        self._engines = {}
        for prefix, net in (("imgnet.", self.imgnet), ("audnet.", self.audnet)):
            net._adopt(self, prefix)

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_engines"] = {}  # device state (streams, packed weights) is rebuilt, never copied
        return state

    def __setstate__(self, state):
        """copy.deepcopy / unpickling: the trunks must point at this copy's flat store, not the original's
        (their parent link is a weakref, which deepcopy shares); engines are rebuilt lazily."""
        super().__setstate__(state)
        self._flat.module = self
        self._flat.rebind()  # deepcopy clones each Parameter on its own: make them views of the copied store again
        self._engines = {}
        for prefix, net in (("imgnet.", self.imgnet), ("audnet.", self.audnet)):
            net._adopt(self, prefix)

    # -- storage management: keep the flat buffers when moved (.cuda(), .to(dev)) --
    def _apply(self, fn, recurse=True):
        self._flat.apply(fn)
        self._engines.clear()
        for net in (self.imgnet, self.audnet):
            net._avt_engine = None
        return self

    def engine(self, device: Optional[torch.device] = None) -> AVEngine:
        """The engine on `device` (default: where the flat store lives)."""
        own = self._flat.flat.device
        dev = own if device is None else torch.device(device)
        key = dev.index if dev.type == "cuda" else -1
        e = self._engines.get(key)
        if e is None:
            flat = self._flat if dev == own else self._flat.mirror(dev)
            e = self._engines.setdefault(key, AVEngine(flat, self.epsilon, self.epsilon2, self.tau, self.trimap,
                                                       self.Neg))
        e.epsilon, e.epsilon2, e.tau, e.tri_map, e.neg = self.epsilon, self.epsilon2, self.tau, self.trimap, self.Neg
        return e

    def ordered_parameters(self):
        mods = dict(self.named_parameters())
        return [mods[n] for n in self._flat.pnames]

    def _replica_forward(self, image, audio):
        """Forward of an ``nn.DataParallel(model)`` replica (train_hardway_1frame.py:93 and every entry
        script).  torch's replicate() gives each replica a shallow copy of this module's __dict__, an
        empty _parameters and the broadcast copies of the parameters as plain attributes (on its GPU).
        The replica on the model's own GPU runs the model's engine, so its BN running statistics are the
        module's buffers (DataParallel keeps replica 0's); a replica on another GPU runs an engine over a
        mirror of the flat store there, refreshed from the model's store on every forward (its running-
        statistic updates are dropped, as DataParallel drops them).  Each replica contrasts only its own
        B/G clips, as in the reference.  The broadcast copies are the autograd inputs, so the gradients
        flow back through replicate()'s Broadcast, which sums them onto the module's parameters.
        The mirror is refreshed from the replica's OWN broadcast parameters and buffers (device-local
        copies): replicate() already moved them across GPUs once.  Forward hooks on a replica's layer4
        (copied from the module by replicate()) run per replica, as nn.Module.__call__ runs them."""
        _check_hooks(self)
        dev = image.device
        eng = self.engine(dev)
        n_train = sum(1 for n in self._flat.pnames if trainable(n))
        tensors = [self._replica_tensor(n) for n in self._flat.pnames[:n_train]]
        if any(t.device != dev for t in tensors):
            raise RuntimeError("avt: DataParallel replica parameters are not on the replica's device")
        if eng.flat is not self._flat:
            eng.flat.fill_from(self._replica_tensor)
        return self._forward_on(eng, tensors, image, audio)

    def _forward_on(self, eng: AVEngine, train_params, image, audio):
        """The forward on one engine with these parameter tensors as the autograd inputs, honouring
        forward hooks on this module's (or replica's) imgnet/audnet.layer4 (test.py:60-63)."""
        hooked = [(n, m) for n, m in (("imgnet", self.imgnet.layer4), ("audnet", self.audnet.layer4))
                  if m._forward_hooks]
        sink = {} if hooked else None
        if torch.is_grad_enabled() and not self.training and (image.requires_grad or audio.requires_grad):
            # as ResNet.forward: an input gradient through eval-mode BatchNorm is not computed -- refuse here rather
            # than return detached outputs whose backward() fails far from the cause
            raise NotImplementedError("avt: gradients through an eval-mode AVENet are not computed (train-mode "
                                      "BatchNorm only)")
        need_grad = torch.is_grad_enabled() and self.training and (
            image.requires_grad or audio.requires_grad or any(p.requires_grad for p in train_params))
        if need_grad:
            A, logits, wA, Pos, Neg = _AVENetFunction.apply(eng, True, sink, image, audio, *train_params)
        else:
            out, _ = eng.forward(image, audio, self.training, layer_io=sink is not None)
            A, logits, wA, Pos, Neg = out["A"], out["logits"], out["weighted_A"], out["Pos"], out["Neg"]
            if sink is not None:
                sink.update(out)
        for name, m in hooked:  # test.py:63: activation['layer4'] = output.detach()
            k_in, k_out = ("v_in", "v") if name == "imgnet" else ("a_in", "a")
            _run_forward_hooks(m, _nhwc_to_nchw_f32(sink[k_in]), _nhwc_to_nchw_f32(sink[k_out]))
        return A, logits, wA, Pos, Neg

    def _replica_tensor(self, name: str) -> torch.Tensor:
        obj = self
        parts = name.split(".")
        for part in parts[:-1]:
            obj = getattr(obj, part)
        return getattr(obj, parts[-1])

    def forward(self, image, audio):
        if getattr(self, "_is_replica", False):
            return self._replica_forward(image, audio)
        _check_hooks(self)
        n_train = sum(1 for n in self._flat.pnames if trainable(n))
        return self._forward_on(self.engine(), self.ordered_parameters()[:n_train], image, audio)


# ---------------------------------------------------------------------------------------------
# 3-D tube model (model.py:17-60; BASELINE config 4)
# ---------------------------------------------------------------------------------------------


class _HardWayAttentionFunction(torch.autograd.Function):
    """HardWayAttention.forward (model.py:46-60) on avt_hardway_attention_fwd/_bwd: fp32 features,
    gradients into both inputs."""

    @staticmethod
    def forward(ctx, audio_features, video_features, eps1: float, eps2: float, tau: float):
        from ._lib import call, query
        from .trunk import P, stream_ptr

        b, C, t, h, w = video_features.shape
        B, Pn = b * t, h * w
        dev = video_features.device
        # 'b c t h w -> (b t) (h w) c' (model.py:49 rearrange, channels innermost for the kernels)
        v = video_features.detach().float().permute(0, 2, 3, 4, 1).contiguous()
        an = audio_features.detach().float().contiguous()
        f32 = dict(device=dev, dtype=torch.float32)
        inv, vsum = torch.empty(B, Pn, **f32), torch.empty(B, Pn, **f32)
        A0 = torch.empty(B, Pn, B, **f32)
        save = torch.empty(int(query("avt_hardway_save_floats", B)), **f32)
        logits = torch.empty(B, B + 2, **f32)
        A, Pos, Neg = (torch.empty(B, 1, h, w, **f32) for _ in range(3))
        wA = torch.empty(B, h, w, **f32)
        call("avt_hardway_attention_fwd", P(v), P(an), B, Pn, C, eps1, eps2, tau, P(inv), P(vsum), P(A0), P(save),
             P(logits), P(A), P(Pos), P(Neg), P(wA), stream_ptr())
        ctx.save = (v, an, inv, A0, save)
        ctx.shape = (b, C, t, h, w)
        ctx.hp = (eps1, eps2, tau)
        ctx.dtypes = (audio_features.dtype, video_features.dtype)
        ctx.set_materialize_grads(False)
        return A, logits

    @staticmethod
    def backward(ctx, gA, glogits):
        from ._lib import call, query
        from .trunk import P, stream_ptr

        if gA is None and glogits is None:
            return None, None, None, None, None
        v, an, inv, A0, save = ctx.save
        b, C, t, h, w = ctx.shape
        B, Pn = b * t, h * w
        f32 = dict(device=v.device, dtype=torch.float32)
        dl = torch.zeros(B, B + 2, **f32) if glogits is None else glogits.float().contiguous()
        ga = None if gA is None else gA.float().contiguous()
        dA0, dvh, gv = torch.empty(B, Pn, B, **f32), torch.empty(B, Pn, C, **f32), torch.empty(B, Pn, C, **f32)
        gan = torch.empty(B, C, **f32)
        eps1, eps2, tau = ctx.hp
        ws = torch.empty(int(query("avt_hardway_bwd_ws_floats", B, C)), **f32)
        call("avt_hardway_attention_bwd", P(v), P(an), P(inv), P(A0), P(save), P(dl), P(ga), B, Pn, C, eps1, eps2,
             tau, P(dA0), P(dvh), P(gv), P(gan), P(ws), stream_ptr())
        g_vid = gv.view(b, t, h, w, C).permute(0, 4, 1, 2, 3).to(ctx.dtypes[1])
        return gan.to(ctx.dtypes[0]), g_vid, None, None, None


class HardWayAttention(nn.Module):
    """model.py:38-60: ``forward(audio_features [B,C], video_features [b,C,t,h,w]) -> (A, logits)`` with
    B = b*t, fp32 throughout, differentiable in both inputs.  Like the reference module it takes the
    features as given (FullModel normalises them before the call, model.py:31-35); inside FullModel
    the head runs fused on the trunk outputs instead."""

    def __init__(self):
        super().__init__()
        self.sigmoid = nn.Sigmoid()
        self.epsilon = 0.65
        self.epsilon2 = 0.4
        self.tau = 0.03

    def forward(self, audio_features, video_features):
        if not video_features.is_cuda or not audio_features.is_cuda:
            raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        if video_features.dim() != 5:
            raise ValueError(f"avt: video_features must be [b,C,t,h,w], got {tuple(video_features.shape)}")
        b, C, t, h, w = video_features.shape
        if tuple(audio_features.shape) != (b * t, C):
            raise ValueError(f"avt: audio_features must be [{b * t},{C}], got {tuple(audio_features.shape)}")
        if C % 8 != 0:
            raise ValueError(f"avt: the channel count must be a multiple of 8 (got {C})")
        return _HardWayAttentionFunction.apply(audio_features, video_features, self.epsilon, self.epsilon2, self.tau)


class _FullModelFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, training: bool, audio, video, *params):
        out, tape = engine.forward(audio, video, training)
        ctx.engine, ctx.tape, ctx.n_params = engine, tape, len(params)
        ctx.set_materialize_grads(False)
        return out["A"], out["logits"]

    @staticmethod
    def backward(ctx, gA, glogits):
        nparams = ctx.n_params
        if glogits is None and gA is None:
            return (None, None, None, None) + (None,) * nparams
        engine = ctx.engine
        if ctx.tape is None:
            raise RuntimeError("avt: backward through an eval-mode forward (or a second backward)")
        flat = engine.flat
        dev = (glogits if glogits is not None else gA).device
        gflat = torch.zeros(flat.n_train, device=dev, dtype=torch.float32)
        engine.backward(ctx.tape, glogits, gflat, dA=gA)
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
        self.audnet._adopt(self, "audnet.")
        self.vidnet._adopt(self, "vidnet.")

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_engine"] = None
        return state

    def __setstate__(self, state):
        """copy.deepcopy / unpickling: re-adopt the audio trunk (see AVENet.__setstate__)."""
        super().__setstate__(state)
        self._flat.module = self
        self._flat.rebind()
        self._engine = None
        self.audnet._adopt(self, "audnet.")
        self.vidnet._adopt(self, "vidnet.")

    def _apply(self, fn, recurse=True):
        self._flat.apply(fn)
        self._engine = None
        self.audnet._avt_engine = None
        self.vidnet._avt_engine = None
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

"""3-D tube step (BASELINE config 4) on libavt: FullModel = R3D-18 video trunk (forward only) +
audio ResNet-18 (forward + backward) + the hard-way attention head.

Restates model.py:17-60 and the train_3D.py step (126-138):
  spec [b,1,F,T] --repeat t, fold (b t)--> audio [bt,1,F,T] --audnet--> [bt,512,h',w']
      --AdaptiveMaxPool2d(1), normalize--> an [bt,512]
  video [b,3,t,H,W] --vidnet (R3D-18, no max-pool)--> layer4 [b,512,t,h,w] (forward hook,
      DETACHED: model.py:12-15, 34) --normalize, '(b t) c h w'--> HardWayAttention -> (A, logits)
  CE(logits, 0) -> backward into audnet only -> Adam.

Device data flow (NHWC / NDHWC bf16 activations, fp32 statistics):
  video fp32 NCDHW --avt_video_stem_im2col--> [b,t,H,W,32] (7 temporal taps folded into channels)
      --avt_conv2d_fwd 7x7/s2 (32 ch)--> stem --BN--> layer1..4: avt_conv3d_fwd 3x3x3 (spatial
      stride 2 on layer2-4's first conv), 1x1x1/s(1,2,2) downsample as avt_conv2d_fwd over the b*t
      frames, BN3d + ReLU (+ residual) by avt_bn_apply --> v [b*t, h, w, 512] = '(b t) h w c'.
  The vidnet's avgpool/fc (resnet3D.py:208-212) feed only the discarded `_` of model.py:33: not run.

Audio de-duplication: given the per-clip spectrogram [b,1,F,T] (what the dataloader yields, before
train_3D.py:128-130 repeats it), the audio trunk runs once per clip with BN statistics identical to
the repeated batch's (the running variance gets the repeated batch's unbiased factor,
avt_bn_finalize_rep); the unit vectors are repeated to the bt head rows and the head gradient is
summed back over each clip's t rows.  This is exact (the backward is linear in the upstream
gradient for the shared forward), and cuts the audio trunk's work by t.  Given the folded
[bt,1,F,T] batch (the reference's own API), the trunk runs over all bt rows.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ._lib import call, query
from .engine import AVEngine, FlatStore, _EngineStore
from .trunk import BNSpec, ConvProfiler, P, Trunk, _bn_finalize, conv_out, stream_ptr

R3D_STAGES = [(64, 1), (128, 2), (256, 2), (512, 2)]  # (planes, spatial stride) — resnet3D.py:136-150


def tube_trainable(name: str) -> bool:
    """FullModel parameters that receive gradients: the audio trunk on the audio path only (the
    vidnet output is detached; audnet.conv1 / conv1_flow / fc are unused)."""
    if not name.startswith("audnet."):
        return False
    if ".fc." in name or name.endswith("conv1_flow.weight") or name == "audnet.conv1.weight":
        return False
    return True


@dataclass
class Conv3dSpec:
    name: str
    cin: int
    cout: int
    kt: int
    k: int
    stride: int  # spatial (temporal stride is 1 throughout the R3D-18 of model.py:20)
    pad_t: int
    pad: int
    stem: bool = False

    @property
    def kg(self) -> int:
        return self.k * self.k * 32 if self.stem else self.kt * self.k * self.k * self.cin


class R3DTrunk:
    """resnet3D ResNet(BasicBlock, [2,2,2,2]) up to layer4, forward only; no_max_pool=True (FullModel, model.py:20)
    unless max_pool (the stem's MaxPool3d(3, 2, 1), resnet3D.py:129, 200-201)."""

    def __init__(self, prefix: str, max_pool: bool = False):
        self.prefix = prefix
        self.max_pool = max_pool
        self.stem = Conv3dSpec(prefix + "conv1.weight", 3, 64, 7, 7, 2, 3, 3, stem=True)
        self.bn1 = BNSpec(prefix + "bn1", 64)
        self.blocks = []
        inplanes = 64
        for li, (planes, stride) in enumerate(R3D_STAGES, start=1):
            for bi in range(2):
                s = stride if bi == 0 else 1
                p = f"{prefix}layer{li}.{bi}."
                cin = inplanes if bi == 0 else planes
                blk = {
                    "conv1": Conv3dSpec(p + "conv1.weight", cin, planes, 3, 3, s, 1, 1),
                    "bn1": BNSpec(p + "bn1", planes),
                    "conv2": Conv3dSpec(p + "conv2.weight", planes, planes, 3, 3, 1, 1, 1),
                    "bn2": BNSpec(p + "bn2", planes),
                    "down": None,
                    "bnd": None,
                }
                if bi == 0 and (s != 1 or inplanes != planes):
                    blk["down"] = Conv3dSpec(p + "downsample.0.weight", inplanes, planes, 1, 1, s, 0, 0)
                    blk["bnd"] = BNSpec(p + "downsample.1", planes)
                self.blocks.append(blk)
            inplanes = planes

    def convs(self) -> List[Conv3dSpec]:
        out = [self.stem]
        for b in self.blocks:
            out += [b["conv1"], b["conv2"]] + ([b["down"]] if b["down"] is not None else [])
        return out

    def bns(self) -> List[BNSpec]:
        out = [self.bn1]
        for b in self.blocks:
            out += [b["bn1"], b["bn2"]] + ([b["bnd"]] if b["bnd"] is not None else [])
        return out

    def _conv(self, x, b, T, H, W, spec: Conv3dSpec, bn: BNSpec, store, training):
        """Conv3d (+ BN statistics) -> (y [b*T, H', W', K] bf16, stats [4, K], H', W')."""
        Ho, Wo = conv_out(H, spec.k, spec.stride, spec.pad), conv_out(W, spec.k, spec.stride, spec.pad)
        y = torch.empty(b * T, Ho, Wo, spec.cout, device=x.device, dtype=torch.bfloat16)
        acc = store.stat_acc(bn, "fwd", b * T * Ho * Wo) if training else None
        wf = store.packed3d(spec)
        ev = ConvProfiler.begin()
        if spec.stem:  # 7 temporal taps folded into the 32 input channels (tube.hip)
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), b * T, H, W, 32, spec.cout, spec.k, spec.k, spec.stride,
                 spec.pad, spec.kg, stream_ptr())
            real_k = spec.kt * spec.k * spec.k * spec.cin
        elif spec.kt == 1:  # 1x1x1 downsample: a 2-D conv over the b*T frames
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), b * T, H, W, spec.cin, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, spec.kg, stream_ptr())
            real_k = spec.cin * spec.k * spec.k
        else:
            call("avt_conv3d_fwd", P(x), P(wf), P(y), P(acc), b, T, H, W, spec.cin, spec.cout, spec.kt, spec.k,
                 spec.k, spec.stride, spec.pad_t, spec.pad, stream_ptr())
            real_k = spec.kt * spec.k * spec.k * spec.cin
        ConvProfiler.end(ev, "fwd3d", 2.0 * y.numel() * real_k, 2.0 * (x.numel() + wf.numel() + y.numel()))
        stats = _bn_finalize(y, acc, y.numel() // spec.cout, bn, store, training)
        return y, stats, Ho, Wo

    def forward(self, video: torch.Tensor, store, training: bool) -> torch.Tensor:
        """video fp32 [b,3,T,H,W] -> layer4 map as '(b t) h w c' bf16 [b*T, h, w, 512]."""
        video = video.contiguous().float()
        b, C, T, H, W = video.shape
        if C != 3:
            raise ValueError(f"avt: expected video [b,3,t,H,W], got {tuple(video.shape)}")
        x = torch.empty(b, T, H, W, 32, device=video.device, dtype=torch.bfloat16)
        call("avt_video_stem_im2col", P(video), P(x), b, C, T, H, W, self.stem.kt, self.stem.pad_t, stream_ptr())
        c0, s0, H, W = self._conv(x, b, T, H, W, self.stem, self.bn1, store, training)
        del x
        rows = c0.numel() // 64
        h = torch.empty_like(c0)
        call("avt_bn_apply", P(c0), P(s0[0]), P(s0[1]), None, None, None, P(h), rows, 64, 1, stream_ptr())
        del c0
        if self.max_pool:  # resnet3D.py:200-201
            To, Ho, Wo = (T - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1
            hp = torch.empty(b * To, Ho, Wo, 64, device=h.device, dtype=torch.bfloat16)
            call("avt_maxpool3d_fwd", P(h), P(hp), b, T, H, W, 64, stream_ptr())
            h, T, H, W = hp, To, Ho, Wo
        for blk in self.blocks:
            c1, s1, Ho, Wo = self._conv(h, b, T, H, W, blk["conv1"], blk["bn1"], store, training)
            h1 = torch.empty_like(c1)
            K = c1.shape[-1]
            rows = c1.numel() // K
            call("avt_bn_apply", P(c1), P(s1[0]), P(s1[1]), None, None, None, P(h1), rows, K, 1, stream_ptr())
            del c1
            c2, s2, _, _ = self._conv(h1, b, T, Ho, Wo, blk["conv2"], blk["bn2"], store, training)
            del h1
            out = torch.empty_like(c2)
            if blk["down"] is not None:
                cd, sd, _, _ = self._conv(h, b, T, H, W, blk["down"], blk["bnd"], store, training)
                call("avt_bn_apply", P(c2), P(s2[0]), P(s2[1]), P(cd), P(sd[0]), P(sd[1]), P(out), rows, K, 1,
                     stream_ptr())
            else:
                call("avt_bn_apply", P(c2), P(s2[0]), P(s2[1]), P(h), None, None, P(out), rows, K, 1, stream_ptr())
            h, H, W = out, Ho, Wo
        return h


def _alloc_packs3d(engine, dev):
    """bf16 fwd operands of the R3D convs and the device table of the non-stem ones (one batched pack launch)."""
    import struct

    descs, max_k, max_row = [], 1, 1
    for spec in engine.vid.convs():
        wp = torch.empty(spec.cout, spec.kg, device=dev, dtype=torch.bfloat16)
        engine.packs3d[spec.name] = wp
        if not spec.stem:
            t = spec.kt * spec.k * spec.k
            descs.append(struct.pack("<QQiiii", engine.flat.raw(spec.name).data_ptr(), wp.data_ptr(), spec.cout,
                                     spec.cin, t, 0))
            max_k, max_row = max(max_k, spec.cout), max(max_row, spec.cin * t)
    assert descs and len(descs[0]) == int(query("avt_pack3d_desc_bytes"))
    engine._pack3d_table = torch.frombuffer(bytearray(b"".join(descs)), dtype=torch.uint8).to(dev)
    engine._pack3d_n, engine._pack3d_max = len(descs), (max_k, max_row)


def _pack3d(engine):
    """vidnet weights (fp32 OIDHW, never updated by the optimizer) -> bf16 fwd operands, repacked every step so a
    load_state_dict is always picked up: the folded stem (its own layout) and one launch for the other 19 convs."""
    stem = engine.vid.stem
    call("avt_pack_conv3d_weight", P(engine.flat.raw(stem.name)), P(engine.packs3d[stem.name]), stem.cout, stem.cin,
         stem.kt, stem.k, stem.k, 1, stream_ptr())
    call("avt_pack_conv3d_weights_batched", P(engine._pack3d_table), engine._pack3d_n, *engine._pack3d_max,
         stream_ptr())


class _TubeStore(_EngineStore):
    def packed3d(self, spec: Conv3dSpec):
        return self.e.packs3d[spec.name]


class TubeEngine(AVEngine):
    """R3D-18 + audio ResNet-18 + HardWayAttention head on one device."""

    def __init__(self, flat: FlatStore):
        super().__init__(flat, 0.65, 0.4, 0.03, True, True)  # HardWayAttention's fixed constants (model.py:41-44)
        self.store = _TubeStore(self)

    def _setup_trunks(self):
        self.aud = Trunk("audnet.", "audio")
        self.vid = R3DTrunk("vidnet.")
        self.packs3d: Dict[str, torch.Tensor] = {}
        self.trunks2d = [self.aud]
        self.bn_trunks = [self.aud, self.vid]

    def _alloc(self, dev):
        super()._alloc(dev)
        _alloc_packs3d(self, dev)

    def pack_weights(self):
        super().pack_weights()
        _pack3d(self)

    # ----------------------------------------------------------------------------- forward
    def forward(self, audio: torch.Tensor, video: torch.Tensor, training: bool, with_ce: bool = False,
                ce_scale: float = 1.0):
        """audio: [b*t,1,F,T] (folded repeated spectrogram, model.py API) or [b,1,F,T] (one per clip,
        de-duplicated); video: [b,3,t,H,W].  Returns ({'A', 'logits'[, 'loss', 'dlogits']}, tape)."""
        if not audio.is_cuda or not video.is_cuda:
            raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        if video.dim() != 5 or audio.dim() != 4 or audio.shape[1] != 1:
            raise ValueError(f"avt: expected audio [bt,1,F,T] and video [b,3,t,H,W], got {tuple(audio.shape)} "
                             f"and {tuple(video.shape)}")
        b, t = video.shape[0], video.shape[2]
        B = b * t
        if audio.shape[0] == B:
            rep = 1
        elif audio.shape[0] == b:
            rep = t
        else:
            raise ValueError(f"avt: audio batch {audio.shape[0]} must be b*t={B} (folded) or b={b} (per clip)")
        self.pack_weights()
        if training:
            self.flat.nbt.add_(1)
        dev = video.device
        xa = self._to_nhwc(audio, 1)
        self.aud.bn_rep = rep
        try:
            a, tape_a = self.aud.forward(xa, self.store, training)
        finally:
            self.aud.bn_rep = 1
        v = self.vid.forward(video, self.store, training)
        _, h, w, C = v.shape
        Pn = h * w
        Ba = a.shape[0]
        f32 = dict(device=dev, dtype=torch.float32)
        an_a = torch.empty(Ba, C, **f32)
        amax = torch.empty(Ba, C, device=dev, dtype=torch.int32)
        anorm = torch.empty(Ba, **f32)
        call("avt_audio_pool_norm_fwd", P(a), P(an_a), P(amax), P(anorm), Ba, a.shape[1] * a.shape[2], C, stream_ptr())
        if rep > 1:
            an = torch.empty(B, C, **f32)
            call("avt_repeat_rows_f32", P(an_a), P(an), Ba, rep, C, stream_ptr())
        else:
            an = an_a
        L = B + 2
        inv = torch.empty(B, Pn, **f32)
        vsum = torch.empty(B, Pn, **f32)
        A0 = torch.empty(B, Pn, B, **f32)
        save = torch.empty(int(query("avt_hardway_save_floats", B)), **f32)
        logits = torch.empty(B, L, **f32)
        A = torch.empty(B, 1, h, w, **f32)
        Pos = torch.empty(B, 1, h, w, **f32)
        Neg = torch.empty(B, 1, h, w, **f32)
        wA = torch.empty(B, h, w, **f32)
        call("avt_hardway_fwd", P(v), P(an), B, Pn, C, self.epsilon, self.epsilon2, self.tau, 1, 1, P(inv), P(vsum),
             P(A0), P(save), P(logits), P(A), P(Pos), P(Neg), P(wA), stream_ptr())
        out = {"A": A, "logits": logits, "v": v}
        tape = None
        if training:
            tape = {"aud": tape_a, "v": v, "a": a, "an": an, "an_a": an_a, "amax": amax, "anorm": anorm, "inv": inv,
                    "A0": A0, "save": save, "B": B, "P": Pn, "C": C, "rep": rep, "Ba": Ba}
        if with_ce:
            loss = torch.empty((), **f32)
            dlogits = torch.empty(B, L, **f32) if training else None
            call("avt_hardway_ce", P(logits), B, L, ce_scale, P(loss), P(dlogits), stream_ptr())
            out["loss"] = loss
            out["dlogits"] = dlogits
        return out, tape

    # ----------------------------------------------------------------------------- backward
    def backward_order(self):
        return [self.aud]

    def backward(self, tape, dlogits: Optional[torch.Tensor], gflat: torch.Tensor, on_boundary=None, dA=None):
        """Accumulate d(loss)/d(audnet params) into gflat[:n_train] (caller zeroes it).  dA (optional):
        upstream gradient of the returned A map (model.py:60)."""
        B, Pn, C, rep, Ba = tape["B"], tape["P"], tape["C"], tape["rep"], tape["Ba"]
        dev = tape["A0"].device
        f32 = dict(device=dev, dtype=torch.float32)
        dA0 = torch.empty(B, Pn, B, **f32)
        gan = torch.empty(B, C, **f32)
        dlogits = torch.zeros(B, B + 2, **f32) if dlogits is None else dlogits.contiguous().float()
        dA = None if dA is None else dA.contiguous().float()
        call("avt_hardway_bwd_ex", P(tape["v"]), P(tape["an"]), P(tape["inv"]), P(tape["A0"]), P(tape["save"]),
             P(dlogits), B, Pn, C, self.epsilon, self.epsilon2, self.tau, 1, 1, None, None, None, P(dA), None, None,
             P(dA0), None, None, P(gan), 0, P(self.head_ws(B, C)), stream_ptr())
        if rep > 1:
            gan_a = torch.empty(Ba, C, **f32)
            call("avt_sum_rep_rows_f32", P(gan), P(gan_a), Ba, rep, C, stream_ptr())
        else:
            gan_a = gan
        a = tape["a"]
        ga = torch.empty_like(a)
        call("avt_audio_pool_norm_bwd", P(gan_a), P(tape["an_a"]), P(tape["amax"]), P(tape["anorm"]), P(ga), Ba,
             a.shape[1] * a.shape[2], C, stream_ptr())
        self.store.grads = self.flat.grad_views(gflat)
        try:
            self.aud.backward(tape["aud"], ga, self.store, on_boundary)
            if on_boundary is not None:
                on_boundary(self.aud.prefix + "lo")
        finally:
            self.store.grads = None


class R3DEngine(AVEngine):
    """The R3D-18 trunk called on its own -- ``FullModel.vidnet(video)`` or a standalone
    ``resnet3D.generate_model(18, ...)(video)`` (resnet3D.py:197-213; with or without the stem max-pool): the conv stem ..
    layer4 on libavt as inside FullModel (R3DTrunk), then AdaptiveAvgPool3d((1,1,1)) + fc on the pooled
    fp32 features.  Forward only, as everywhere in this build (FullModel detaches the video trunk)."""

    def __init__(self, flat: FlatStore, prefix: str, max_pool: bool = False):
        self._prefix = prefix
        self._max_pool = max_pool
        super().__init__(flat)
        self.concurrent = False
        self.store = _TubeStore(self)
        self._nbt_idx = torch.tensor([i for i, n in enumerate(flat.nbt_names) if n.startswith(prefix)],
                                     device=flat.flat.device, dtype=torch.long)

    def _setup_trunks(self):
        self.vid = R3DTrunk(self._prefix, self._max_pool)
        self.packs3d: Dict[str, torch.Tensor] = {}
        self.trunks2d = []
        self.bn_trunks = [self.vid]

    def _alloc(self, dev):
        super()._alloc(dev)
        _alloc_packs3d(self, dev)

    def pack_weights(self):
        _pack3d(self)

    def forward(self, video: torch.Tensor, training: bool) -> torch.Tensor:
        """video fp32 [b,3,t,H,W] -> fc logits [b, n_classes] fp32."""
        if not video.is_cuda:
            raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        if video.dim() != 5:
            raise ValueError(f"avt: expected video [b,3,t,H,W], got {tuple(video.shape)}")
        self.pack_weights()
        if training and self._nbt_idx.numel():
            self.flat.nbt.index_add_(0, self._nbt_idx, torch.ones_like(self._nbt_idx))
        v = self.vid.forward(video, self.store, training)  # [(b t), h, w, 512] bf16
        b = video.shape[0]
        feat = v.view(b, -1, v.shape[-1]).float().mean(1)  # AdaptiveAvgPool3d((1,1,1)) + flatten
        w, bias = self.flat.raw(self._prefix + "fc.weight"), self.flat.raw(self._prefix + "fc.bias")
        return torch.addmm(bias, feat, w.t())  # nn.Linear (resnet3D.py:212)

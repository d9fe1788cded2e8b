"""16-frame two-view hard-way step (train_hardway.py:126-144) on libavt.

Reference step, per batch of b clips of t frames (``--frame_density`` 16):
  spec [b,1,F,T] --unsqueeze(2).repeat(1,1,t,1,1), '(b t)'--> [bt,1,F,T]            (128-129)
  frames, augmented [b,3,t,H,W] --'(b t)'--> [bt,3,H,W]                              (130-131)
  (A, logits, weighted, ..) = model(frames, spec); (.., logits2, weighted2, ..) = model(augmented, spec)
  combined = (lw*CE(logits) + lw*CE(logits2))/2 + (100-lw)*MSE(weighted, weighted2)
             + Prop(weighted.reshape(b,t,h,w)) + Prop(weighted2.reshape(b,t,h,w))    (134-142)
  backward, Adam(lr 4e-6, weight_decay 1e-4)                                         (115, 143-145)

Device plan (one process per GPU, b clips per rank):
  frames / augmented fp32 NCTHW --avt_ncthw_to_nhwc_bf16 (fold fused)--> [(bt),H,W,4] bf16
      --vision trunk, once per view (own BN batch statistics; running stats updated in view order)--> v1, v2
  audio, de-duplicated (default): the 2t identical copies of a clip's spectrogram (t frames x 2 views)
      run the audio trunk once per clip.  BN statistics equal the repeated batch's (running_var with
      the repeated batch's unbiased factor, avt_bn_finalize_rep); the reference's two momentum-0.1
      updates with identical statistics compose to one with momentum 1-(1-0.1)^2 = 0.19.  The unit
      vectors are repeated to the bt head rows of each view; the backward runs once, with the head
      gradient summed over both views (avt_hardway_bwd gan accumulation) and the t frames
      (avt_sum_rep_rows_f32).  Exact: for a fixed forward the trunk backward is linear in its
      upstream gradient.  ``dedup_audio=False`` runs the audio trunk over the folded bt rows once per
      view, as the reference does.
  head per view: avt_hardway_fwd -> logits, weighted_A; avt_hardway_ce (dlogits scale lw/2) x2;
  avt_twoview_loss -> combined loss and d weighted_A of both views; avt_hardway_bwd per view
  (weighted_A path included) -> gv1, gv2, gan; vision backward x2 (gradients accumulate); audio backward.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import call, query
from .engine import AVEngine
from .trunk import P, stream_ptr

MOMENTUM_TWO_UPDATES = 1.0 - (1.0 - 0.1) ** 2  # two BatchNorm momentum-0.1 updates with one statistic


class TwoViewEngine(AVEngine):
    """AVEngine running the train_hardway.py step: two views of b clips x t frames sharing one
    spectrogram per clip."""

    def __init__(self, flat, epsilon=0.65, epsilon2=0.4, tau=0.03, tri_map=True, neg=True, loss_weight=0.1,
                 dedup_audio=True):
        super().__init__(flat, epsilon, epsilon2, tau, tri_map, neg)
        self.loss_weight = loss_weight
        self.dedup_audio = dedup_audio

    def _fold_frames(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous().float()
        b, c, t, H, W = x.shape
        y = torch.empty(b * t, H, W, 4, device=x.device, dtype=torch.bfloat16)
        call("avt_ncthw_to_nhwc_bf16", P(x), P(y), b, c, t, H, W, 4, stream_ptr())
        return y

    def _head(self, v, an, B, f32):
        _, h, w, C = v.shape
        Pn = h * w
        L = B + (2 if self.neg else 1)
        inv, vsum = torch.empty(B, Pn, **f32), torch.empty(B, Pn, **f32)
        A0 = torch.empty(B, Pn, B, **f32)
        save = torch.empty(int(query("avt_hardway_save_floats", B)), **f32)
        logits = torch.empty(B, L, **f32)
        A, Pos, Neg = (torch.empty(B, 1, h, w, **f32) for _ in range(3))
        wA = torch.empty(B, h, w, **f32)
        call("avt_hardway_fwd", P(v), P(an), B, Pn, C, self.epsilon, self.epsilon2, self.tau, int(self.tri_map),
             int(self.neg), P(inv), P(vsum), P(A0), P(save), P(logits), P(A), P(Pos), P(Neg), P(wA), stream_ptr())
        out = {"A": A, "logits": logits, "weighted_A": wA, "Pos": Pos, "Neg": Neg}
        tape = {"v": v, "an": an, "inv": inv, "vsum": vsum, "A0": A0, "save": save, "B": B, "P": Pn, "C": C}
        return out, tape

    def _audio(self, xa, rep: int, momentum: float, training: bool, f32):
        """audio trunk + max-pool + normalize; rows of the result repeated `rep` times."""
        self.aud.bn_rep, self.aud.bn_momentum = rep, momentum
        try:
            a, tape_a = self.aud.forward(xa, self.store, training)
        finally:
            self.aud.bn_rep, self.aud.bn_momentum = 1, 0.1
        Ba, C = a.shape[0], a.shape[-1]
        an_a = torch.empty(Ba, C, **f32)
        amax = torch.empty(Ba, C, device=a.device, dtype=torch.int32)
        anorm = torch.empty(Ba, **f32)
        call("avt_audio_pool_norm_fwd", P(a), P(an_a), P(amax), P(anorm), Ba, a.shape[1] * a.shape[2], C, stream_ptr())
        an = an_a
        if rep > 1:
            an = torch.empty(Ba * rep, C, **f32)
            call("avt_repeat_rows_f32", P(an_a), P(an), Ba, rep, C, stream_ptr())
        return an, {"aud": tape_a, "a": a, "an_a": an_a, "amax": amax, "anorm": anorm, "Ba": Ba, "rep": rep}

    def forward(self, frames: torch.Tensor, augmented: torch.Tensor, spec: torch.Tensor, training: bool,
                with_ce: bool = True, ce_scale: Optional[float] = None):
        """frames, augmented [b,3,t,H,W]; spec [b,1,F,T] (one per clip, before the t-fold repeat of
        train_hardway.py:128).  Returns ({'views': [out1, out2], 'losses' [5] = (combined, hardway,
        aug, l2, consistency), 'dlogits': [..], 'dwA': [..]}, tape)."""
        for x in (frames, augmented, spec):
            if not x.is_cuda:
                raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        if frames.dim() != 5 or frames.shape[1] != 3 or augmented.shape != frames.shape:
            raise ValueError(f"avt: frames/augmented must both be [b,3,t,H,W], got {tuple(frames.shape)} and "
                             f"{tuple(augmented.shape)}")
        b, t = frames.shape[0], frames.shape[2]
        if spec.dim() != 4 or spec.shape[0] != b or spec.shape[1] != 1:
            raise ValueError(f"avt: spec must be [b={b},1,F,T], got {tuple(spec.shape)}")
        if t < 2:
            raise ValueError("avt: the two-view step needs t >= 2 frames per clip (PropagationLoss diff over t)")
        B = b * t
        dev = frames.device
        f32 = dict(device=dev, dtype=torch.float32)
        self.pack_weights()
        if training:
            self.flat.nbt.add_(2)  # two AVENet forwards per step
        x1, x2 = self._fold_frames(frames), self._fold_frames(augmented)
        v1, tape_i1 = self.img.forward(x1, self.store, training)
        v2, tape_i2 = self.img.forward(x2, self.store, training)
        auds = []
        if self.dedup_audio:
            xa = self._to_nhwc(spec, 1)
            an, ta = self._audio(xa, t, MOMENTUM_TWO_UPDATES if training else 0.1, training, f32)
            auds = [(an, ta), (an, ta)]
        else:
            rep_spec = torch.empty(B, 1, spec.shape[2], spec.shape[3], **f32)
            call("avt_repeat_rows_f32", P(spec.contiguous().float()), P(rep_spec), b, t, spec.shape[2] * spec.shape[3],
                 stream_ptr())
            xa = self._to_nhwc(rep_spec, 1)
            auds = [self._audio(xa, 1, 0.1, training, f32), self._audio(xa, 1, 0.1, training, f32)]
        o1, h1 = self._head(v1, auds[0][0], B, f32)
        o2, h2 = self._head(v2, auds[1][0], B, f32)
        out = {"views": [o1, o2]}
        L = o1["logits"].shape[1]
        Pn = h1["P"]
        if with_ce:
            lw = self.loss_weight
            ce = torch.empty(2, **f32)
            dl = [torch.empty(B, L, **f32), torch.empty(B, L, **f32)] if training else [None, None]
            scale = lw / 2 if ce_scale is None else ce_scale
            for k, o in enumerate((o1, o2)):
                call("avt_hardway_ce", P(o["logits"]), B, L, scale, P(ce[k:k + 1]), P(dl[k]), stream_ptr())
            losses = torch.empty(5, **f32)
            dw = [torch.empty(B, Pn, **f32), torch.empty(B, Pn, **f32)]
            call("avt_twoview_loss", P(ce[0:1]), P(ce[1:2]), P(o1["weighted_A"]), P(o2["weighted_A"]), b, t, Pn, lw,
                 P(losses), P(dw[0]), P(dw[1]), stream_ptr())
            out.update(losses=losses, loss=losses[0], ce=ce, dlogits=dl, dwA=dw)
        tape = None
        if training:
            tape = {"img": [tape_i1, tape_i2], "head": [h1, h2], "aud": [auds[0][1], auds[1][1]], "b": b, "t": t}
        return out, tape

    def backward(self, tape, grads_in, gflat: torch.Tensor, on_boundary=None):
        """grads_in = (dlogits [2], dwA [2]) as forward(with_ce=True) returns them.  Accumulates into
        gflat[:n_train] (caller zeroes it); on_boundary as AVEngine.backward."""
        dlogits, dwA = grads_in
        h1, h2 = tape["head"]
        ta1, ta2 = tape["aud"]
        shared = ta1 is ta2
        gv1, gan = self.head_backward(h1, dlogits[0], dwA[0])
        gv2, gan2 = self.head_backward(h2, dlogits[1], dwA[1], gan=gan if shared else None)
        self.store.grads = self.flat.grad_views(gflat)
        try:
            self.img.backward(tape["img"][0], gv1, self.store, None)
            self.img.backward(tape["img"][1], gv2, self.store, on_boundary)
            if on_boundary is not None:
                on_boundary(self.img.prefix + "lo")
            if shared:
                self._audio_backward(ta1, gan, on_boundary)
            else:
                self._audio_backward(ta1, gan, None)
                self._audio_backward(ta2, gan2, on_boundary)
            if on_boundary is not None:
                on_boundary(self.aud.prefix + "lo")
        finally:
            self.store.grads = None

    def _audio_backward(self, ta, gan, on_boundary):
        Ba, rep, a = ta["Ba"], ta["rep"], ta["a"]
        C = a.shape[-1]
        if rep > 1:
            gan_a = torch.empty(Ba, C, device=gan.device, dtype=torch.float32)
            call("avt_sum_rep_rows_f32", P(gan), P(gan_a), Ba, rep, C, stream_ptr())
        else:
            gan_a = gan
        ga = torch.empty_like(a)
        call("avt_audio_pool_norm_bwd", P(gan_a), P(ta["an_a"]), P(ta["amax"]), P(ta["anorm"]), P(ga), Ba,
             a.shape[1] * a.shape[2], C, stream_ptr())
        self.aud.backward(ta["aud"], ga, self.store, on_boundary)

"""AVENet train/eval step on libavt: flat parameter storage, forward with a tape, backward into a
flat fp32 gradient buffer.

Data flow of one 1-frame step (model.py:112-154, train_hardway_1frame.py:129-134):
  image [B,3,H,W] fp32 NCHW --avt_nchw_to_nhwc_bf16--> [B,H,W,4] bf16 --Trunk(vision)--> v [B,h,w,512]
  audio [B,1,F,T] fp32       --avt_nchw_to_nhwc_bf16--> [B,F,T,1] bf16 --Trunk(audio)--> a [B,h',w',512]
  a --avt_audio_pool_norm_fwd--> an [B,512];  (v, an) --avt_hardway_fwd--> A, logits, weighted_A, Pos, Neg
  CE (avt_hardway_ce) -> dlogits --avt_hardway_bwd--> gv, g_an --> trunk backward --> flat grads --> Adam.
"""
from __future__ import annotations

import contextlib
import os
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch

from ._lib import call, query
from .trunk import P, Store, Trunk, drive, stream_ptr


# ---------------------------------------------------------------------------------------------
# parameter inventory (state_dict of the reference AVENet, model.py:89-110 + base_models.py:113-169)
# ---------------------------------------------------------------------------------------------


def trainable(name: str) -> bool:
    """Parameters that receive gradients on the 1-frame step: everything except both fc layers,
    both conv1_flow stems and the other modality's stem (SURVEY §7 'Unused parameters')."""
    if ".fc." in name or name.endswith("conv1_flow.weight"):
        return False
    if name.startswith("imgnet.") and name.endswith("conv1_a.weight"):
        return False
    if name.startswith("audnet.conv1.weight"):
        return False
    return True


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


class FlatStore:
    """All parameters of a module in one flat fp32 buffer (trainable ones first), all float
    buffers in a second one, num_batches_tracked counters in a third.  Conv weights are kept in
    OHWI memory order, exposed as channels_last OIHW ``nn.Parameter`` views, so the kernels read
    them directly and ``state_dict``/``load_state_dict`` keep the reference's key names and shapes."""

    def __init__(self, module: torch.nn.Module, trainable_fn=None):
        self.module = module
        is_train = trainable_fn if trainable_fn is not None else trainable
        self.trainable = is_train
        params = [(n, p) for n, p in module.named_parameters()]
        order = [x for x in params if is_train(x[0])] + [x for x in params if not is_train(x[0])]
        self.pnames = [n for n, _ in order]
        self.n_train = 0
        self.poff: Dict[str, Tuple[int, tuple]] = OrderedDict()
        off = 0
        for n, p in order:
            if is_train(n):
                self.n_train = off + p.numel()
            self.poff[n] = (off, tuple(p.shape))
            off += (p.numel() + 3) // 4 * 4  # 16-byte aligned segments
        self.n_train = (self.n_train + 3) // 4 * 4
        device = params[0][1].device
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.boff: Dict[str, Tuple[int, tuple]] = OrderedDict()
        self.nbt_names: List[str] = []
        boff = 0
        for n, b in module.named_buffers():
            if n.endswith("num_batches_tracked"):
                self.nbt_names.append(n)
                continue
            self.boff[n] = (boff, tuple(b.shape))
            boff += b.numel()
        self.bflat = torch.zeros(max(boff, 1), dtype=torch.float32, device=device)
        self.nbt = torch.zeros(len(self.nbt_names), dtype=torch.long, device=device)
        with torch.no_grad():
            for n, p in params:
                src = p.detach().float()
                self.raw(n).copy_(src.permute(0, 2, 3, 1) if src.dim() == 4 else src)
            for n, b in module.named_buffers():
                if n in self.boff:
                    self.rawbuf(n).copy_(b.detach().float().reshape(-1))
                elif n in self.nbt_names:
                    self.nbt[self.nbt_names.index(n)] = b.detach().long()
        self.rebind()

    def mirror(self, device) -> "FlatStore":
        """A store with this one's layout on another device, bound to no module (the per-GPU weights of
        an nn.DataParallel replica; refresh with sync_from)."""
        m = FlatStore.__new__(FlatStore)
        m.module = None
        m.trainable, m.pnames, m.n_train = self.trainable, self.pnames, self.n_train
        m.poff, m.boff, m.nbt_names = self.poff, self.boff, self.nbt_names
        m.flat = torch.empty_like(self.flat, device=device)
        m.bflat = torch.empty_like(self.bflat, device=device)
        m.nbt = torch.empty_like(self.nbt, device=device)
        m.sync_from(self)
        return m

    def sync_from(self, src: "FlatStore"):
        """Copy src's parameters, float buffers and counters (same layout) into this store."""
        self.flat.copy_(src.flat)
        self.bflat.copy_(src.bflat)
        self.nbt.copy_(src.nbt)

    def fill_from(self, get):
        """Fill this (mirror) store from per-name tensors on its device -- an nn.DataParallel replica's
        broadcast parameters and buffers (get(name) -> tensor in the module's layout): local copies only."""
        dst, src = [], []
        for n in self.pnames:
            t = get(n).detach()
            r = self.raw(n)
            dst.append(r)
            src.append(t.permute(0, 2, 3, 1) if t.dim() == 4 else t)  # OIHW -> the store's OHWI
        for n in self.boff:
            dst.append(self.rawbuf(n))
            src.append(get(n))
        for i, n in enumerate(self.nbt_names):
            dst.append(self.nbt[i])
            src.append(get(n))
        with torch.no_grad():
            torch._foreach_copy_(dst, src)

    def raw(self, name: str) -> torch.Tensor:
        """fp32 storage of a parameter: conv weights as [K][R][S][C] (OHWI), others as-is."""
        off, shape = self.poff[name]
        n = 1
        for s in shape:
            n *= s
        t = self.flat[off:off + n]
        if len(shape) == 4:
            k, c, r, s = shape
            return t.view(k, r, s, c)
        return t.view(shape)

    def rawbuf(self, name: str) -> torch.Tensor:
        off, shape = self.boff[name]
        n = 1
        for s in shape:
            n *= s
        return self.bflat[off:off + n].view(shape)

    def _pview(self, name: str) -> torch.Tensor:
        r = self.raw(name)
        return r.permute(0, 3, 1, 2) if r.dim() == 4 else r

    def rebind(self):
        """(Re)point every registered Parameter/buffer of the module at the flat storage."""
        mods = dict(self.module.named_modules())
        for n in self.pnames:
            mname, _, pname = n.rpartition(".")
            m = mods[mname]
            old = m._parameters[pname]
            m._parameters[pname] = torch.nn.Parameter(self._pview(n), requires_grad=old.requires_grad)
        for n in self.boff:
            mname, _, bname = n.rpartition(".")
            mods[mname]._buffers[bname] = self.rawbuf(n)
        for i, n in enumerate(self.nbt_names):
            mname, _, bname = n.rpartition(".")
            mods[mname]._buffers[bname] = self.nbt[i]

    def apply(self, fn):
        if self.module is None:
            raise RuntimeError("avt: a mirrored FlatStore is not bound to a module")
        self.flat = fn(self.flat)
        self.bflat = fn(self.bflat)
        self.nbt = fn(self.nbt)
        if self.flat.dtype != torch.float32 or self.bflat.dtype != torch.float32:
            raise TypeError("avt AVENet keeps fp32 master weights; dtype casts are not supported "
                            "(the trunks compute in bf16 with fp32 statistics)")
        self.rebind()

    def grad_views(self, gflat: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for n in self.pnames:
            if not self.trainable(n):
                continue
            off, shape = self.poff[n]
            k = 1
            for s in shape:
                k *= s
            t = gflat[off:off + k]
            out[n] = t.view(shape[0], shape[2], shape[3], shape[1]) if len(shape) == 4 else t.view(shape)
        return out

    def param_grad_views(self, gflat: torch.Tensor) -> Dict[str, torch.Tensor]:
        """gradient views shaped/strided like the Parameters (channels_last OIHW)."""
        return {n: (g.permute(0, 3, 1, 2) if g.dim() == 4 else g) for n, g in self.grad_views(gflat).items()}


class _EngineStore(Store):
    def __init__(self, engine: "AVEngine"):
        self.e = engine
        self.grads: Optional[Dict[str, torch.Tensor]] = None

    def param(self, name):
        return self.e.flat.raw(name)

    def buffer(self, name):
        return self.e.flat.rawbuf(name)

    def grad(self, name):
        return self.grads[name]

    def packed(self, spec):
        return self.e.packs[spec.name]

    def stat_acc(self, bn, kind, rows):
        return self.e.stat_acc(bn, kind, rows)

    def splitk(self, spec, dgrad, N, H, W):
        return self.e.splitk_ws(spec, dgrad, N, H, W)

    def wgrad_tickets(self, spec, N, H, W):
        return self.e.wgrad_tickets(spec, N, H, W)

    pending: Optional[Dict[str, list]] = None  # trunk prefix -> deferred wgrad slabs (AVEngine.backward)

    def wgrad_pending(self, prefix):
        return None if self.pending is None else self.pending.get(prefix)


class AVEngine:
    """Two trunks + the hard-way head on one device."""

    def __init__(self, flat: FlatStore, epsilon=0.65, epsilon2=0.4, tau=0.03, tri_map=True, neg=True):
        self.flat = flat
        self._setup_trunks()
        self.epsilon, self.epsilon2, self.tau, self.tri_map, self.neg = epsilon, epsilon2, tau, tri_map, neg
        self.store = _EngineStore(self)
        self.packs: Dict[str, Tuple[torch.Tensor, Optional[torch.Tensor]]] = {}
        self._pack_table = None
        self._pack_max = 0
        self.stat_views: Dict = {}  # (BN prefix, 'fwd' | 'bwd') -> its statistics accumulator
        self._retired: List[torch.Tensor] = []
        self._alloc(flat.flat.device)
        # run the audio trunk on a second HIP stream, concurrently with the vision trunk (forward and
        # backward): the two trunks are independent until the head, and their kernels fill each
        # other's wave-quantisation tails.  With world > 1 the backward keeps both trunks concurrent
        # in two segments (layer4+3, then layer2..stem) joined at the boundary, where on_boundary(tags)
        # issues the bucketed all-reduce of the finished gradients (train.py).
        self.concurrent = os.environ.get("AVT_CONCURRENT", "1") != "0"
        self._side = None
        # split-K for the short layer3/4 grids (a few clips per GPU): per call site a persistent ticket
        # array (the kernel leaves it zero) and a partial-tile buffer per call; AVT_SPLITK=0: off
        self.splitk = os.environ.get("AVT_SPLITK", "0") != "0"
        self.split_pack = os.environ.get("AVT_SPLIT_PACK", "1") != "0"
        self._splitk_cnt: Dict = {}
        # the wgrads' in-kernel split-K reduce (avt_conv2d_wgrad_tk): per call site and stream a persistent ticket
        # array; AVT_WGRAD_FUSED=0 in the library turns the fused path off (the tickets are then 0 and unused)
        self._wgrad_tk: Dict = {}
        # the wgrads' split-K slab reduces deferred to one batched launch per trunk and backward segment
        # (avt_wgrad_reduce_batch; AVT_WGRAD_DEFER=1 -- until measured, off: a reduce launch per wgrad, the same bits)
        self.defer_wgrad = os.environ.get("AVT_WGRAD_DEFER", "0") != "0"

    def splitk_ws(self, spec, dgrad: bool, N: int, H: int, W: int):
        """(part, cnt) for a split-K conv call (avt_conv2d_splitk_plan), or None: no split for the shape,
        split-K off, or (first use) inside a graph capture -- the tickets are allocated zeroed outside
        capture (the engine runs an eager step before capturing)."""
        if not self.splitk or spec.k != 3 or spec.stride != 1 or spec.is_stem:
            return None
        # one ticket array per call site AND stream: two same-shape calls on different streams never share one
        key = (spec.name, dgrad, N, H, W, torch.cuda.current_stream().cuda_stream)
        ent = self._splitk_cnt.get(key)
        if ent is None:
            import ctypes
            nf, nc = ctypes.c_longlong(0), ctypes.c_int(0)
            call("avt_conv2d_splitk_plan", N, H, W, spec.cin, spec.cout, 3, 3, 1, 1, int(dgrad), ctypes.byref(nf),
                 ctypes.byref(nc))
            if nc.value == 0 or torch.cuda.is_current_stream_capturing():
                if nc.value == 0:
                    self._splitk_cnt[key] = (0, None)
                return None
            ent = self._splitk_cnt[key] = (nf.value, torch.zeros(nc.value, device=self.flat.flat.device,
                                                                  dtype=torch.int32))
        nf, cnt = ent
        if cnt is None:
            return None
        return torch.empty(nf, device=cnt.device, dtype=torch.float32), cnt

    def wgrad_tickets(self, spec, N: int, H: int, W: int):
        """Zeroed int32 tickets for this wgrad call (avt_conv2d_wgrad_tickets), allocated outside graph capture (the
        engine runs an eager step before capturing; the kernel leaves them zero, so replays reuse them), or None."""
        key = (spec.name, N, H, W, torch.cuda.current_stream().cuda_stream)
        t = self._wgrad_tk.get(key)
        if t is None:
            n = int(query("avt_conv2d_wgrad_tickets", N, H, W, spec.cp, spec.cin, spec.cout, spec.k, spec.k,
                          spec.stride, spec.pad))
            if n == 0 or torch.cuda.is_current_stream_capturing():
                return None
            t = self._wgrad_tk[key] = torch.zeros(n, device=self.flat.flat.device, dtype=torch.int32)
        return t

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.flat.flat.device)
        return self._side

    @contextlib.contextmanager
    def _branch(self, enabled: bool = True):
        """Run the body on the side stream, forked from the current one; join() must follow."""
        if not (self.concurrent and enabled):
            yield
            return
        side = self._side_stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            yield

    def _join(self, enabled: bool = True):
        if self.concurrent and enabled and self._side is not None:
            torch.cuda.current_stream().wait_stream(self._side)

    def _interleave(self, side_gen, main_gen, phase: str = "BWD"):
        """Issue two launch generators (Trunk.*_iter) alternately, side_gen's launches on the side
        stream, main_gen's on the current one, forked before and joined after; returns both values.
        (Measured at B=32: the two-stream step 4.03 ms vs 5.26 ms on one stream.  The issue order
        does not matter to a HIP graph replay -- same-box A/B of interleaved vs branch-after-branch
        issue: equal -- and cross-stream edges that keep the branches in lockstep cost 9-24 %.)
        Not concurrent: side_gen then main_gen on the current stream."""
        if not self.concurrent or os.environ.get("AVT_DEBUG_SERIAL_" + phase):  # (diagnostic: one phase serial)
            return drive(side_gen), drive(main_gen)
        side = self._side_stream()
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        res, live = [None, None], [True, True]
        while live[0] or live[1]:
            for i, (gen, st) in enumerate(((side_gen, side), (main_gen, main))):
                if not live[i]:
                    continue
                with torch.cuda.stream(st):
                    try:
                        next(gen)
                    except StopIteration as e:
                        live[i], res[i] = False, e.value
        main.wait_stream(side)
        return res[0], res[1]

    def _setup_trunks(self):
        self.img = Trunk("imgnet.", "vision")
        self.aud = Trunk("audnet.", "audio")
        self.trunks2d = [self.img, self.aud]  # packed by the batched 2-D weight pack
        self.bn_trunks = [self.img, self.aud]  # own fp64 BN accumulators in the arena

    def _alloc(self, dev):
        """Persistent device buffers: packed bf16 weights, the batched-pack descriptor table and the
        fp64 BN statistic accumulators (zero between uses)."""
        import struct

        descs = []
        maxel = 0
        self._pack_parts = {}  # trunk prefix -> (first descriptor, count, max elements)
        for tr in self.trunks2d:
            first, tmax = len(descs), 0
            for spec in tr.convs():
                wf = torch.empty(spec.cout, spec.kg, device=dev, dtype=torch.bfloat16)
                wt = None if spec.is_stem else torch.empty(spec.cin, spec.k * spec.k * spec.cout, device=dev,
                                                           dtype=torch.bfloat16)
                self.packs[spec.name] = (wf, wt)
                w = self.flat.raw(spec.name)
                rs = spec.k * spec.k
                descs.append(struct.pack("<QQQiiiiii", w.data_ptr(), wf.data_ptr(), 0 if wt is None else wt.data_ptr(),
                                         spec.cout, rs, spec.cin, spec.cp, spec.kg, 0))
                tmax = max(tmax, spec.cout * spec.kg + (0 if wt is None else wt.numel()))
            maxel = max(maxel, tmax)
            self._pack_parts[tr.prefix] = (first, len(descs) - first, tmax)
        if descs:  # (an engine of 3-D trunks only packs its own operands, tube.py)
            assert len(descs[0]) == int(query("avt_pack_desc_bytes"))
            blob = b"".join(descs)
            self._pack_table = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        self._pack_n, self._pack_max = len(descs), maxel

    def head_ws(self, B: int, C: int) -> torch.Tensor:
        """Split-K partials of the head backward's audio-vector GEMM (avt_hardway_bwd_ws_floats)."""
        n = int(query("avt_hardway_bwd_ws_floats", B, C))
        t = getattr(self, "_head_ws", None)
        if t is None or t.numel() < n:
            if t is not None:
                self._retired.append(t)
            t = self._head_ws = torch.empty(n, device=self.flat.flat.device, dtype=torch.float32)
        return t

    def stat_acc(self, bn, kind: str, rows: int) -> torch.Tensor:
        """A BN's fp64 statistics accumulator for `rows` rows (include/avt.h "BatchNorm statistics": the
        producing kernel overwrites its slots, no zeroing), kept per (BN, kind) and grown when a larger batch
        comes: a captured graph keeps the tensor it was captured with alive through this dict."""
        key = (bn.prefix, kind)
        need = int(query("avt_bn_acc_doubles", rows, bn.c)) if kind == "fwd" else \
            (int(query("avt_bn_bwd_workspace", rows, bn.c)) + 7) // 8
        t = self.stat_views.get(key)
        if t is None or t.numel() < need:
            if t is not None:
                self._retired.append(t)  # a graph captured on it may still replay
            t = torch.empty(need, device=self.flat.flat.device, dtype=torch.float64)
            self.stat_views[key] = t
        return t

    # ----------------------------------------------------------------------------- weights
    def pack_weights(self):
        """fp32 master weights -> bf16 fwd/dgrad operands of every conv (two batched launches)."""
        call("avt_pack_conv_weights_batched", P(self._pack_table), self._pack_n, self._pack_max, stream_ptr())

    def pack_trunk(self, tr: Trunk, which: int):
        """One trunk's bf16 operands: which = 1 the fwd images, 2 the dgrad images (one launch)."""
        first, n, mx = self._pack_parts[tr.prefix]
        off = first * int(query("avt_pack_desc_bytes"))
        call("avt_pack_conv_weights_part", P(self._pack_table[off:]), n, mx, which, stream_ptr())

    # ----------------------------------------------------------------------------- forward
    @staticmethod
    def _to_nhwc(x: torch.Tensor, cp: int) -> torch.Tensor:
        x = x.contiguous().float()
        N, C, H, W = x.shape
        y = torch.empty(N, H, W, cp, device=x.device, dtype=torch.bfloat16)
        call("avt_nchw_to_nhwc_bf16", P(x), P(y), N, C, H, W, cp, stream_ptr())
        return y

    def forward(self, image: torch.Tensor, audio: torch.Tensor, training: bool, with_ce: bool = False,
                ce_scale: float = 1.0, layer_io: bool = False, vision_pre=None):
        """layer_io: also return each trunk's layer4 input/output ("v_in"/"v", "a_in"/"a", NHWC bf16)
        for forward hooks registered on imgnet.layer4 / audnet.layer4 (test.py:63).  vision_pre():
        launches issued at the head of the vision trunk's branch (ordered before the head, concurrent
        with the audio trunk)."""
        if not image.is_cuda or not audio.is_cuda:
            raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        if image.shape[1] != 3 or audio.shape[1] != 1:
            raise ValueError(f"avt: expected image [B,3,H,W] and audio [B,1,F,T], got {tuple(image.shape)} "
                             f"and {tuple(audio.shape)}")
        B = image.shape[0]
        if audio.shape[0] != B:
            raise ValueError("avt: image and audio batch sizes differ")
        # split packing (concurrent trunks): each trunk's fwd operands at the head of its own branch, the
        # dgrad operands (backward only) behind the vision forward, which finishes before the audio one
        split_pack = self.concurrent and self.split_pack
        if not split_pack:
            self.pack_weights()
        # training: each trunk zeroes its BN accumulators on its own branch (Trunk.forward_iter), the batch
        # counters and vision_pre() (e.g. the gradient zeroing of the step) run on the vision branch -- the
        # shorter trunk's slack, not the serial section
        dev = image.device

        io_a = {} if layer_io else None
        io_v = {} if layer_io else None

        def audio_branch():
            if split_pack:
                self.pack_trunk(self.aud, 1)
            xa = self._to_nhwc(audio, 1)
            a, tape_a = yield from self.aud.forward_iter(xa, self.store, training, io_a)
            C = a.shape[-1]
            an = torch.empty(B, C, device=dev, dtype=torch.float32)
            amax = torch.empty(B, C, device=dev, dtype=torch.int32)
            anorm = torch.empty(B, device=dev, dtype=torch.float32)
            call("avt_audio_pool_norm_fwd", P(a), P(an), P(amax), P(anorm), B, a.shape[1] * a.shape[2], C,
                 stream_ptr())
            return a, tape_a, an, amax, anorm

        def vision_branch():
            if training:
                self.flat.nbt.add_(1)
            if vision_pre is not None:
                vision_pre()
            if split_pack:
                self.pack_trunk(self.img, 1)
            xi = self._to_nhwc(image, 4)
            out = yield from self.img.forward_iter(xi, self.store, training, io_v)
            if split_pack and training:
                self.pack_trunk(self.img, 2)
                self.pack_trunk(self.aud, 2)
            return out

        # audio trunk (side stream) || vision trunk (current stream), launches interleaved
        (a, tape_a, an, amax, anorm), (v, tape_i) = self._interleave(audio_branch(), vision_branch(), "FWD")
        _, h, w, C = v.shape
        Pn = h * w
        L = B + (2 if self.neg else 1)
        f32 = dict(device=dev, dtype=torch.float32)
        inv = torch.empty(B, Pn, **f32)
        vsum = torch.empty(B, Pn, **f32)
        A0 = torch.empty(B, Pn, B, **f32)
        save = torch.empty(int(query("avt_hardway_save_floats", B)), **f32)
        logits = torch.empty(B, L, **f32)
        A = torch.empty(B, 1, h, w, **f32)
        Pos = torch.empty(B, 1, h, w, **f32)
        Neg = torch.empty(B, 1, h, w, **f32)
        wA = torch.empty(B, h, w, **f32)
        call("avt_hardway_fwd", P(v), P(an), B, Pn, C, self.epsilon, self.epsilon2, self.tau, int(self.tri_map),
             int(self.neg), P(inv), P(vsum), P(A0), P(save), P(logits), P(A), P(Pos), P(Neg), P(wA), stream_ptr())
        out = {"A": A, "logits": logits, "weighted_A": wA, "Pos": Pos, "Neg": Neg, "v": v}
        if layer_io:
            out.update(v_in=io_v["layer4_in"], a=a, a_in=io_a["layer4_in"])
        tape = None
        if training:
            tape = {"img": tape_i, "aud": tape_a, "v": v, "a": a, "an": an, "amax": amax, "anorm": anorm,
                    "inv": inv, "vsum": vsum, "A0": A0, "save": save, "B": B, "P": Pn, "C": C}
        if with_ce:
            loss = torch.empty((), **f32)
            dlogits = torch.empty(B, L, **f32) if training else None
            call("avt_hardway_ce", P(logits), B, L, ce_scale, P(loss), P(dlogits), stream_ptr())
            out["loss"] = loss
            out["dlogits"] = dlogits
        return out, tape

    # ----------------------------------------------------------------------------- backward
    def grad_buckets(self):
        """Gradient all-reduce buckets in backward completion order, as (boundary tag, flat region):
        each trunk's layer3+layer4 ('<prefix>hi'), then the rest of it ('<prefix>lo').  backward()
        calls on_boundary(tag) when a bucket's gradients are final."""
        order = [tr for tr in self.backward_order()]
        out = []
        for tr in order:
            hi = lambda n, p=tr.prefix: n.startswith(p + "layer3.") or n.startswith(p + "layer4.")
            lo = lambda n, p=tr.prefix: n.startswith(p) and not (n.startswith(p + "layer3.") or
                                                                 n.startswith(p + "layer4."))
            for tag, sel in ((tr.prefix + "hi", hi), (tr.prefix + "lo", lo)):
                spans = [(self.flat.poff[n][0], self.flat.poff[n][0] + _numel(self.flat.poff[n][1]))
                         for n in self.flat.pnames if self.flat.trainable(n) and sel(n)]
                lo_off, hi_off = min(a for a, _ in spans), max(b for _, b in spans)
                # the region is exactly these parameters' grads (+ 16-byte alignment padding)
                assert sum(b - a for a, b in spans) <= hi_off - lo_off <= sum(b - a for a, b in spans) + 3 * len(spans)
                hi_off = min((hi_off + 3) // 4 * 4, self.flat.n_train)
                out.append((tag, (lo_off, hi_off)))
        return out

    def backward_order(self):
        return [self.img, self.aud]

    def head_backward(self, tape, dlogits: Optional[torch.Tensor], dwA: Optional[torch.Tensor] = None,
                      gan: Optional[torch.Tensor] = None, dA=None, dPos=None, dNeg=None):
        """Hard-way head backward: (d logits, d weighted_A[, d A, d Pos, d Neg]) -> (gv [B,h,w,C] bf16,
        gan [B,C] fp32).  A given ``gan`` is accumulated into (two views sharing one audio batch)."""
        B, Pn, C = tape["B"], tape["P"], tape["C"]
        dev = tape["v"].device
        f32 = dict(device=dev, dtype=torch.float32)
        L = B + (2 if self.neg else 1)
        dlogits = torch.zeros(B, L, **f32) if dlogits is None else dlogits.contiguous().float()
        dA0 = torch.empty(B, Pn, B, **f32)
        dvh = torch.empty(B, Pn, C, **f32)
        gv = torch.empty_like(tape["v"])
        accumulate = gan is not None
        if gan is None:
            gan = torch.empty(B, C, **f32)
        dm = None
        if dwA is not None:
            dwA = dwA.contiguous().float()
            dm = torch.empty(B, Pn, **f32)
        aux = [None if g is None else g.contiguous().float() for g in (dA, dPos, dNeg)]
        call("avt_hardway_bwd_ex", P(tape["v"]), P(tape["an"]), P(tape["inv"]), P(tape["A0"]), P(tape["save"]),
             P(dlogits), B, Pn, C, self.epsilon, self.epsilon2, self.tau, int(self.tri_map), int(self.neg), P(dwA),
             P(tape["vsum"] if dwA is not None else None), P(dm), P(aux[0]), P(aux[1]), P(aux[2]), P(dA0), P(dvh),
             P(gv), P(gan), int(accumulate), P(self.head_ws(B, C)), stream_ptr())
        return gv, gan

    def backward(self, tape, dlogits: Optional[torch.Tensor], gflat: torch.Tensor, on_boundary=None,
                 dwA: Optional[torch.Tensor] = None, dA=None, dPos=None, dNeg=None, on_trunk_end=None):
        """Accumulate d(loss)/d(params) into gflat[:n_train] (caller zeroes it).
        dwA: upstream gradient of weighted_A (the 16-frame losses, train_hardway.py:138-141); dA/dPos/dNeg:
        of the returned maps.  The two trunks' backward runs concurrently (audio on the side stream) in
        two segments: layer4+layer3 of both, then layer2..stem of both.  on_boundary(tags) is called
        with ("imgnet.hi", "audnet.hi") between the segments and ("imgnet.lo", "audnet.lo") at the end
        -- on the current stream, after the side stream has joined it, so a gradient all-reduce issued
        there sees those buckets final (train.py overlaps them with the second segment).
        on_trunk_end(trunk) (without on_boundary): called on each trunk's stream behind its last gradient
        launch -- that trunk's gradients are final there (train.py updates them while the other trunk's
        backward still runs)."""
        gv, gan = self.head_backward(tape, dlogits, dwA, dA=dA, dPos=dPos, dNeg=dNeg)
        a = tape["a"]
        B, C = tape["B"], tape["C"]
        self.store.grads = self.flat.grad_views(gflat)
        hi = self.img.HI_BLOCK
        seg = on_boundary is not None  # two segments (joined at the boundary) only when someone listens
        aud, img, ta, ti = self.aud, self.img, tape["aud"], tape["img"]

        def audio_hi():
            ga = torch.empty_like(a)
            call("avt_audio_pool_norm_bwd", P(gan), P(tape["an"]), P(tape["amax"]), P(tape["anorm"]), P(ga), B,
                 a.shape[1] * a.shape[2], C, stream_ptr())
            r = yield from aud.backward_blocks_iter(ta, ga, self.store, hi, len(aud.blocks))
            aud.flush_wgrad(self.store)  # the segment's deferred slab reduces, on the trunk's stream
            return r

        def img_hi_flushed():
            r = yield from img.backward_blocks_iter(ti, gv, self.store, hi, len(img.blocks))
            img.flush_wgrad(self.store)
            return r

        def lo(tr, tp, g, pm):
            g, _ = yield from tr.backward_blocks_iter(tp, g, self.store, 0, hi, pm)
            yield from tr.backward_stem_iter(tp, g, self.store)
            tr.flush_wgrad(self.store)

        def chain(tr, tp, first):
            g, pm = yield from first
            yield from lo(tr, tp, g, pm)
            if on_trunk_end is not None:  # on the trunk's stream, behind its last gradient launch
                on_trunk_end(tr)

        if self.defer_wgrad:
            self.store.pending = {img.prefix: [], aud.prefix: []}
        try:
            img_hi = img_hi_flushed()
            if seg:  # segment 1: layer4+layer3 of both trunks; boundary; segment 2: the rest
                (ga, pa), (gv, pv) = self._interleave(audio_hi(), img_hi)
                on_boundary((img.prefix + "hi", aud.prefix + "hi"))
                self._interleave(lo(aud, ta, ga, pa), lo(img, ti, gv, pv))
                on_boundary((img.prefix + "lo", aud.prefix + "lo"))
            else:
                self._interleave(chain(aud, ta, audio_hi()), chain(img, ti, img_hi))
            assert not self.store.pending or not any(self.store.pending.values()), "unflushed wgrad slabs"
        finally:
            self.store.grads = None
            self.store.pending = None

class TrunkEngine(AVEngine):
    """One ResNet-18 trunk called on its own (``model.imgnet(x)`` / a standalone ``resnet18(modal=...)``,
    base_models.py:195-213): NCHW fp32 input -> layer4 map NCHW fp32, backward into the trunk's
    parameter gradients (and the input gradient through the 7x7 stem when asked: avt_conv_stem_dgrad)."""

    def __init__(self, flat: FlatStore, prefix: str, modal: str):
        self._prefix, self._modal = prefix, modal
        super().__init__(flat)
        self.concurrent = False
        self._nbt_idx = torch.tensor([i for i, n in enumerate(flat.nbt_names) if n.startswith(prefix)],
                                     device=flat.flat.device, dtype=torch.long)

    def _setup_trunks(self):
        self.trunk = Trunk(self._prefix, self._modal)
        self.trunks2d = [self.trunk]
        self.bn_trunks = [self.trunk]

    def forward(self, x: torch.Tensor, training: bool):
        if not x.is_cuda:
            raise RuntimeError("avt: inputs must be on the GPU (no CPU path)")
        cin = 1 if self._modal == "audio" else 3
        if x.dim() != 4 or x.shape[1] != cin:
            raise ValueError(f"avt: {self._modal} trunk expects [N,{cin},H,W], got {tuple(x.shape)}")
        self.pack_weights()
        if training:
            self.flat.nbt.index_add_(0, self._nbt_idx, torch.ones_like(self._nbt_idx))
        xin = self._to_nhwc(x, self.trunk.stem.cp)
        y, tape = self.trunk.forward(xin, self.store, training)
        N, h, w, C = y.shape
        out = torch.empty(N, C, h, w, device=x.device, dtype=torch.float32)
        call("avt_nhwc_bf16_to_nchw", P(y), P(out), N, C, h * w, stream_ptr())
        return out, tape

    def backward(self, tape, g_out: torch.Tensor, gflat: torch.Tensor):
        """g_out [N,512,h,w] fp32 (any layout) -> parameter gradients accumulated into gflat; returns the input
        gradient [N,Cin,H,W] fp32 when tape["want_dx"] was set, else None."""
        g = g_out.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()  # layout plumbing
        self.store.grads = self.flat.grad_views(gflat)
        try:
            self.trunk.backward(tape, g, self.store, None)
        finally:
            self.store.grads = None
        return tape.get("dx")

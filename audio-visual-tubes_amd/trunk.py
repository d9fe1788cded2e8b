"""ResNet-18 trunk (one modality) as a sequence of libavt launches: forward with a saved tape,
backward into flat fp32 gradients.

Restates models/base_models.py: ResNet._forward_impl (195-210) with the modal-selected stem
(conv1 3->64 for vision, conv1_a 1->64 for audio, 7x7/s2/p3), bn1, ReLU, MaxPool(3,2,1),
layer1..4 of BasicBlocks (53-69) with layer4 stride 1 (149).  Activations are NHWC bf16 held in
torch.bfloat16 tensors (raw bits shared with the kernels); BN statistics fp32.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ._lib import BnBwdTarget, DgradBnEpi, SlabReduceDesc, call, query

STAGES = [(64, 1), (128, 2), (256, 2), (512, 1)]
# 1: BN-backward reductions fused into the dgrad epilogues (avt_conv2d_dgrad_bn); default 0: the separate
# reduce/apply passes of avt_bn_bwd (measured 1 % faster: DESIGN §6f)
FUSE_BN_BWD = os.environ.get("AVT_FUSE_BN_BWD", "0") == "1"
# timing diagnostic (WRONG results; bench.py refuses it, tools/step_time.py measures with it): conv2 reads the
# raw conv1 output instead of h1 = relu(bn1(conv1)) -- the upper bound of what fusing bn1 + ReLU into conv2's
# operand loads could save (the 16 h1 apply launches and their 2 x 1 GB/step of traffic at B = 128)
DIAG_H1_SKIP = os.environ.get("AVT_DIAG_H1_SKIP", "0") == "1"
if DIAG_H1_SKIP and os.environ.get("AVT_DIAG_WRONG_RESULTS_OK", "0") != "1":
    # a training run under this variable would silently train another network: it needs an explicit opt-in
    raise RuntimeError("avt: AVT_DIAG_H1_SKIP=1 computes WRONG results (timing diagnostic); set "
                       "AVT_DIAG_WRONG_RESULTS_OK=1 as well to run it (tools/step_time.py)")


def P(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def drive(gen):
    """Run a launch generator (Trunk.*_iter) to completion; return its value."""
    while True:
        try:
            next(gen)
        except StopIteration as e:
            return e.value


def conv_out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


class ConvProfiler:
    """Optional HIP-event bracketing of every conv launch (bench.py's live roofline).
    Records (kind, algorithmic FLOPs, algorithmic HBM bytes, start, end) on the launching stream.
    Algorithmic bytes = each operand read once + the output written once (fp32 wgrad output:
    read-modify-write)."""

    active: Optional["ConvProfiler"] = None

    def __init__(self):
        self.records = []

    def __enter__(self):
        ConvProfiler.active = self
        return self

    def __exit__(self, *exc):
        ConvProfiler.active = None

    @staticmethod
    def begin():
        p = ConvProfiler.active
        if p is None:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    @staticmethod
    def end(ev, kind: str, flops: float, nbytes: float = 0.0):
        p = ConvProfiler.active
        if p is None or ev is None:
            return
        e2 = torch.cuda.Event(enable_timing=True)
        e2.record()
        p.records.append((kind, flops, nbytes, ev, e2))

    def summary(self):
        """kind -> [launches, FLOPs, ms, algorithmic bytes]"""
        torch.cuda.synchronize()
        out = {}
        for kind, fl, nb, a, b in self.records:
            ms = a.elapsed_time(b)
            k = out.setdefault(kind, [0, 0.0, 0.0, 0.0])
            k[0] += 1
            k[1] += fl
            k[2] += ms
            k[3] += nb
        return out


@dataclass
class ConvSpec:
    name: str      # parameter name (state_dict key of the weight)
    cin: int       # real input channels
    cout: int
    k: int
    stride: int
    pad: int
    cp: int        # padded input channels in the activation layout (stems: 4 / 1)

    @property
    def kg(self) -> int:
        kg = self.k * self.k * self.cp
        return (kg + 31) // 32 * 32

    @property
    def is_stem(self) -> bool:
        return self.cp < 32


@dataclass
class BNSpec:
    prefix: str
    c: int


class Store:
    """Where a trunk finds its tensors: fp32 params (conv weights OHWI-contiguous), BN buffers,
    packed bf16 weights, and (during backward) fp32 gradient views."""

    def param(self, name: str) -> torch.Tensor: ...
    def buffer(self, name: str) -> torch.Tensor: ...
    def grad(self, name: str) -> Optional[torch.Tensor]: ...
    def packed(self, spec: ConvSpec): ...
    def stat_acc(self, bn: "BNSpec", kind: str, rows: int) -> torch.Tensor:
        """fp64 statistics accumulator of a BN over `rows` rows ('fwd': avt_bn_acc_doubles(rows, C) doubles;
        'bwd': the avt_bn_bwd_workspace(rows, C) workspace).  Any contents (the producers overwrite their
        slots); the same tensor for a BN's producer and its consumer within a step."""
        ...

    def splitk(self, spec: "ConvSpec", dgrad: bool, N: int, H: int, W: int):
        """(part, cnt) split-K workspace of this conv call (avt_conv2d_splitk_plan), or None."""
        return None

    def wgrad_pending(self, prefix: str) -> Optional[list]:
        """The list a trunk's deferred wgrad slab reduces go to (avt_conv2d_wgrad_defer; the engine sums them with one
        avt_wgrad_reduce_batch at the end of each backward segment), or None: each wgrad reduces its own slab."""
        return None

    def wgrad_tickets(self, spec: "ConvSpec", N: int, H: int, W: int) -> Optional[torch.Tensor]:
        """Persistent zeroed int32 tickets of this wgrad call site (avt_conv2d_wgrad_tickets; the kernel leaves
        them zero), or None: the split-K slab then goes through the separate reduce launch."""
        return None


def _bn_finalize(c_out, acc, rows, bn: BNSpec, store: Store, training: bool, momentum=0.1, eps=1e-5, rep: int = 1):
    """BN statistics -> (scale, shift, mean, invstd) [4, C]; train mode also updates the running
    stats.  rep > 1: every row stands for `rep` identical rows of the logical batch (tube step)."""
    C = bn.c
    stats = torch.empty(4, C, device=c_out.device, dtype=torch.float32)  # scale, shift, mean, invstd
    gamma = store.param(bn.prefix + ".weight")
    beta = store.param(bn.prefix + ".bias")
    if training and (rep > 1 or momentum != 0.1):
        call("avt_bn_finalize_rep", P(acc), rows, rep, C, P(gamma), P(beta),
             P(store.buffer(bn.prefix + ".running_mean")), P(store.buffer(bn.prefix + ".running_var")),
             ctypes.c_float(momentum), ctypes.c_float(eps), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]),
             stream_ptr())
    elif training:
        call("avt_bn_finalize", P(acc), rows, C, P(gamma), P(beta),
             P(store.buffer(bn.prefix + ".running_mean")), P(store.buffer(bn.prefix + ".running_var")),
             ctypes.c_float(momentum), ctypes.c_float(eps), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]),
             stream_ptr())
    else:
        rm = store.buffer(bn.prefix + ".running_mean")
        rv = store.buffer(bn.prefix + ".running_var")
        inv = torch.rsqrt(rv + eps)
        stats[0] = gamma * inv
        stats[1] = beta - rm * stats[0]
        stats[2] = rm
        stats[3] = inv
    return stats


class Trunk:
    """One ResNet-18 (base_models.resnet18(modal=...)) on libavt."""

    def __init__(self, prefix: str, modal: str):
        self.prefix, self.modal = prefix, modal
        self.bn_rep = 1  # >1: each input sample stands for bn_rep identical ones (tube audio de-dup)
        self.bn_momentum = 0.1  # 0.19: two reference forwards over the same batch in one (two-view audio)
        if modal == "audio":
            self.stem = ConvSpec(prefix + "conv1_a.weight", 1, 64, 7, 2, 3, 1)
        else:
            self.stem = ConvSpec(prefix + "conv1.weight", 3, 64, 7, 2, 3, 4)
        self.bn1 = BNSpec(prefix + "bn1", 64)
        self.blocks = []
        inplanes = 64
        for li, (planes, stride) in enumerate(STAGES, start=1):
            for bi in range(2):
                s = stride if bi == 0 else 1
                p = f"{prefix}layer{li}.{bi}."
                cin = inplanes if bi == 0 else planes
                blk = {
                    "conv1": ConvSpec(p + "conv1.weight", cin, planes, 3, s, 1, cin),
                    "bn1": BNSpec(p + "bn1", planes),
                    "conv2": ConvSpec(p + "conv2.weight", planes, planes, 3, 1, 1, planes),
                    "bn2": BNSpec(p + "bn2", planes),
                    "down": None,
                    "bnd": None,
                }
                if bi == 0 and (s != 1 or inplanes != planes):
                    blk["down"] = ConvSpec(p + "downsample.0.weight", inplanes, planes, 1, s, 0, inplanes)
                    blk["bnd"] = BNSpec(p + "downsample.1", planes)
                self.blocks.append(blk)
            inplanes = planes

    def convs(self) -> List[ConvSpec]:
        out = [self.stem]
        for b in self.blocks:
            out += [b["conv1"], b["conv2"]] + ([b["down"]] if b["down"] is not None else [])
        return out

    def bns(self) -> List[BNSpec]:
        out = [self.bn1]
        for b in self.blocks:
            out += [b["bn1"], b["bn2"]] + ([b["bnd"]] if b["bnd"] is not None else [])
        return out

    # ------------------------------------------------------------------ forward
    def _conv_bn(self, x, N, H, W, spec: ConvSpec, bn: BNSpec, store: Store, training: bool):
        """conv + its BN statistics (finalized: stats [4, C])."""
        Pq, Qq = conv_out(H, spec.k, spec.stride, spec.pad), conv_out(W, spec.k, spec.stride, spec.pad)
        y = torch.empty(N, Pq, Qq, spec.cout, device=x.device, dtype=torch.bfloat16)
        acc = store.stat_acc(bn, "fwd", N * Pq * Qq) if training else None
        wf, _ = store.packed(spec)
        ws = store.splitk(spec, False, N, H, W)
        ev = ConvProfiler.begin()
        if ws is not None:
            call("avt_conv2d_fwd_ws", P(x), P(wf), P(y), P(acc), N, H, W, spec.cp, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, spec.kg, P(ws[0]), ws[0].numel(), P(ws[1]), ws[1].numel(), stream_ptr())
        else:
            call("avt_conv2d_fwd", P(x), P(wf), P(y), P(acc), N, H, W, spec.cp, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, spec.kg, stream_ptr())
        ConvProfiler.end(ev, "fwd", 2.0 * N * Pq * Qq * spec.cout * spec.k * spec.k * spec.cin,
                         2.0 * (x.numel() + wf.numel() + y.numel()))
        stats = _bn_finalize(y, acc, N * Pq * Qq, bn, store, training, momentum=self.bn_momentum, rep=self.bn_rep)
        return y, stats, Pq, Qq

    def forward(self, x: torch.Tensor, store: Store, training: bool, io: Optional[Dict] = None):
        """x: [N,H,W,cp] bf16 NHWC. Returns (layer4 map [N,h,w,512] bf16, tape).  io (optional) receives
        "layer4_in": the layer3 output [N,h,w,256] (the input a forward hook on .layer4 sees)."""
        return drive(self.forward_iter(x, store, training, io))

    def forward_iter(self, x: torch.Tensor, store: Store, training: bool, io: Optional[Dict] = None):
        """forward() as a generator that yields after each launch group, so that two trunks' launches can
        be issued interleaved on two streams (engine._interleave); returns forward()'s result."""
        N, H, W, _ = x.shape
        tape: Dict = {"x": x, "N": N, "H": H, "W": W, "blocks": []}
        c0, st0, H1, W1 = self._conv_bn(x, N, H, W, self.stem, self.bn1, store, training)
        yield
        # bn1 -> relu -> maxpool fused: the full-resolution relu(bn1(c0)) is never stored
        H2, W2 = conv_out(H1, 3, 2, 1), conv_out(W1, 3, 2, 1)
        p0 = torch.empty(N, H2, W2, 64, device=x.device, dtype=torch.bfloat16)
        idx = torch.empty(N, H2, W2, 64, device=x.device, dtype=torch.uint8)
        carg = torch.empty_like(p0)
        call("avt_stem_bn_relu_maxpool_fwd", P(c0), P(st0[0]), P(st0[1]), P(p0), P(idx), P(carg), N, H1, W1, 64,
             stream_ptr())
        tape.update(c0=c0, st0=st0, idx=idx, carg=carg, H1=H1, W1=W1)
        yield
        cur, Hc, Wc = p0, H2, W2
        for bi, blk in enumerate(self.blocks):
            if io is not None and bi == 6:
                io["layer4_in"] = cur
            t = {"x": cur, "H": Hc, "W": Wc}
            c1, s1, Ho, Wo = self._conv_bn(cur, N, Hc, Wc, blk["conv1"], blk["bn1"], store, training)
            yield
            if DIAG_H1_SKIP:
                h1 = c1
            else:
                h1 = torch.empty_like(c1)
                call("avt_bn_apply", P(c1), P(s1[0]), P(s1[1]), None, None, None, P(h1), N * Ho * Wo, c1.shape[-1],
                     1, stream_ptr())
            yield
            c2, s2, _, _ = self._conv_bn(h1, N, Ho, Wo, blk["conv2"], blk["bn2"], store, training)
            yield
            out = torch.empty_like(c2)
            # training: the output's ReLU mask as bits ([rows][C/8] u8) for the backward, which then never
            # re-reads `out` (1/16 of its bytes)
            om = torch.empty(c2.numel() // 8, device=x.device, dtype=torch.uint8) if training else None
            if blk["down"] is not None:
                cd, sd, _, _ = self._conv_bn(cur, N, Hc, Wc, blk["down"], blk["bnd"], store, training)
                yield
                res = (P(cd), P(sd[0]), P(sd[1]))
                t.update(cd=cd, sd=sd)
            else:
                res = (P(cur), None, None)
            if training:
                call("avt_bn_apply_mask", P(c2), P(s2[0]), P(s2[1]), *res, P(out), P(om), N * Ho * Wo, c2.shape[-1],
                     stream_ptr())
            else:
                call("avt_bn_apply", P(c2), P(s2[0]), P(s2[1]), *res, P(out), N * Ho * Wo, c2.shape[-1], 1,
                     stream_ptr())
            t.update(c1=c1, s1=s1, h1=h1, c2=c2, s2=s2, out=out, om=om, Ho=Ho, Wo=Wo)
            tape["blocks"].append(t)
            yield
            cur, Hc, Wc = out, Ho, Wo
        if not training:
            tape = None
        return cur, tape

    # ------------------------------------------------------------------ backward
    def _bn_bwd(self, g, y, xc, stats, bn: BNSpec, store: Store, gmask_out=None):
        rows = xc.numel() // bn.c
        gc = torch.empty_like(xc)
        ws = store.stat_acc(bn, "bwd", rows)
        call("avt_bn_bwd", P(g), P(y), P(xc), P(stats[2]), P(stats[3]), P(store.param(bn.prefix + ".weight")),
             P(store.grad(bn.prefix + ".weight")), P(store.grad(bn.prefix + ".bias")), P(gc), P(gmask_out), P(ws),
             rows, bn.c, stream_ptr())
        return gc

    def _target(self, xc, stats, bn: BNSpec, store: Store) -> BnBwdTarget:
        t = BnBwdTarget()
        gc = torch.empty_like(xc)
        t.xc, t.mean, t.invstd = xc.data_ptr(), stats[2].data_ptr(), stats[3].data_ptr()
        t.gamma = store.param(bn.prefix + ".weight").data_ptr()
        dg, db = store.grad(bn.prefix + ".weight"), store.grad(bn.prefix + ".bias")
        t.dgamma = dg.data_ptr() if dg is not None else None
        t.dbeta = db.data_ptr() if db is not None else None
        t.gc = gc.data_ptr()
        t.workspace = store.stat_acc(bn, "bwd", xc.numel() // bn.c).data_ptr()
        t.keep = gc  # the output tensor (ctypes.Structure keeps no reference)
        return t

    def _bn_bwd_mask(self, g, mask, xc, stats, bn: BNSpec, store: Store, xc2=None, stats2=None, bn2=None):
        """Block-output BN backward(s) from the ReLU mask bits: bn2 alone, or bn2 + downsample.1 in one
        pass (avt_bn_bwd_mask).  Returns the gradient(s) of the pre-BN activation(s)."""
        t1 = self._target(xc, stats, bn, store)
        t2 = self._target(xc2, stats2, bn2, store) if bn2 is not None else None
        call("avt_bn_bwd_mask", P(g), P(mask), ctypes.byref(t1), ctypes.byref(t2) if t2 is not None else None,
             xc.numel() // bn.c, bn.c, stream_ptr())
        return t1.keep, (t2.keep if t2 is not None else None)

    def _bn_relu_bwd(self, g, xc, stats, bn: BNSpec, store: Store):
        """bn -> relu backward with the mask recomputed from (xc, scale, shift) (BasicBlock.bn1)."""
        rows = xc.numel() // bn.c
        gc = torch.empty_like(xc)
        ws = store.stat_acc(bn, "bwd", rows)
        call("avt_bn_relu_bwd", P(g), P(xc), P(stats[0]), P(stats[1]), P(stats[2]), P(stats[3]),
             P(store.param(bn.prefix + ".weight")), P(store.grad(bn.prefix + ".weight")),
             P(store.grad(bn.prefix + ".bias")), P(gc), P(ws), rows, bn.c, stream_ptr())
        return gc

    def _wgrad(self, x, gy, N, H, W, spec: ConvSpec, store: Store):
        dw = store.grad(spec.name)
        wsb = int(query("avt_conv2d_wgrad_workspace", N, H, W, spec.cp, spec.cin, spec.cout, spec.k, spec.k,
                        spec.stride, spec.pad))
        ws = torch.empty(wsb, device=x.device, dtype=torch.uint8) if wsb else None
        pending = store.wgrad_pending(self.prefix) if ws is not None else None
        tk = store.wgrad_tickets(spec, N, H, W) if ws is not None and pending is None else None
        ev = ConvProfiler.begin()
        if pending is not None:
            d = SlabReduceDesc()
            call("avt_conv2d_wgrad_defer", P(x), P(gy), P(dw), N, H, W, spec.cp, spec.cin, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, P(ws), wsb, ctypes.byref(d), stream_ptr())
            if d.splits > 0:
                pending.append((d, ws))  # the workspace stays alive until the batched reduce
        else:
            call("avt_conv2d_wgrad_tk", P(x), P(gy), P(dw), N, H, W, spec.cp, spec.cin, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, P(ws), wsb, P(tk), 0 if tk is None else tk.numel(), stream_ptr())
        ConvProfiler.end(ev, "wgrad", 2.0 * gy.numel() * spec.k * spec.k * spec.cin,
                         2.0 * (x.numel() + gy.numel()) + 8.0 * dw.numel())

    def flush_wgrad(self, store: Store):
        """Sum this trunk's deferred wgrad slabs (one launch per 24) on the current stream."""
        pending = store.wgrad_pending(self.prefix)
        if not pending:
            return
        arr = (SlabReduceDesc * len(pending))(*[d for d, _ in pending])
        call("avt_wgrad_reduce_batch", arr, len(pending), stream_ptr())
        pending.clear()  # (stream-ordered reuse of the workspaces: allocated and freed on this stream)

    def _dgrad(self, gy, N, H, W, spec: ConvSpec, store: Store, add=None, inplace=False, epi=None, add_mask=None):
        """inplace: accumulate into `add` (dx = add + dgrad); a strided 1x1 conv then only touches the
        pixels its taps reach (the other parity classes of avt_conv2d_dgrad are skipped).
        epi: DgradBnEpi -- the backward reductions of the BN+ReLU that produced dx's positions fused into
        the store (dx = the masked gradient g'; avt_conv2d_dgrad_bn)."""
        _, wt = store.packed(spec)
        gx = add if inplace else torch.empty(N, H, W, spec.cin, device=gy.device, dtype=torch.bfloat16)
        ws = store.splitk(spec, True, N, H, W) if epi is None else None
        ev = ConvProfiler.begin()
        if ws is not None:  # short grid: split-K (add / add_mask as below)
            call("avt_conv2d_dgrad_ws", P(gy), P(wt), P(gx), P(add), P(add_mask), N, H, W, spec.cin, spec.cout,
                 spec.k, spec.k, spec.stride, spec.pad, P(ws[0]), ws[0].numel(), P(ws[1]), ws[1].numel(), stream_ptr())
        elif add_mask is not None:  # dx = dgrad + add * mask bits
            assert epi is None
            call("avt_conv2d_dgrad_mask", P(gy), P(wt), P(gx), P(add), P(add_mask), N, H, W, spec.cin, spec.cout,
                 spec.k, spec.k, spec.stride, spec.pad, stream_ptr())
        elif epi is None:
            call("avt_conv2d_dgrad", P(gy), P(wt), P(gx), P(add), N, H, W, spec.cin, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, stream_ptr())
        else:
            call("avt_conv2d_dgrad_bn", P(gy), P(wt), P(gx), P(add), N, H, W, spec.cin, spec.cout, spec.k, spec.k,
                 spec.stride, spec.pad, ctypes.byref(epi), stream_ptr())
        ConvProfiler.end(ev, "dgrad", 2.0 * gy.numel() * spec.k * spec.k * spec.cin,
                         2.0 * (gy.numel() + wt.numel() + gx.numel() * (2 if add is not None else 1)))
        return gx

    # backward boundary: once layer3 and layer4 are done (~94 % of a ResNet-18's parameters) their
    # gradients can start their all-reduce while layer2..stem run (train.py bucketing)
    HI_BLOCK = 4  # index of layer3.0 in self.blocks

    def backward(self, tape: Dict, g_out: torch.Tensor, store: Store, on_boundary=None):
        g, pm = self.backward_blocks(tape, g_out, store, self.HI_BLOCK, len(self.blocks))
        if on_boundary is not None:
            on_boundary(self.prefix + "hi")
        g, _ = self.backward_blocks(tape, g, store, 0, self.HI_BLOCK, pm)
        self.backward_stem(tape, g, store)

    def _bn_bwd_premasked(self, gm, xc, stats, bn: BNSpec, store: Store):
        """BN backward of a pre-masked g' whose reductions a dgrad epilogue already accumulated."""
        gc = torch.empty_like(xc)
        call("avt_bn_bwd_premasked", P(gm), P(xc), P(stats[2]), P(stats[3]), P(store.param(bn.prefix + ".weight")),
             P(store.grad(bn.prefix + ".weight")), P(store.grad(bn.prefix + ".bias")), P(gc),
             P(store.stat_acc(bn, "bwd", xc.numel() // bn.c)), xc.numel() // bn.c, bn.c, stream_ptr())
        return gc

    def _epi(self, store: Store, bn: BNSpec, xc, stats, y=None, bn2: Optional[BNSpec] = None, xc2=None, stats2=None,
             skip00: bool = False, append: bool = False) -> DgradBnEpi:
        """append: this dgrad's partial sums follow those of the skip00 dgrad before it (a strided block's
        downsample dgrad finishing the same BN reductions, include/avt.h)."""
        e = DgradBnEpi()
        rows = xc.numel() // bn.c
        e.xc, e.y, e.stats = xc.data_ptr(), (y.data_ptr() if y is not None else None), stats.data_ptr()
        e.acc = store.stat_acc(bn, "bwd", rows).data_ptr()
        if bn2 is not None:
            e.xc2, e.stats2, e.acc2 = xc2.data_ptr(), stats2.data_ptr(), store.stat_acc(bn2, "bwd", rows).data_ptr()
        e.skip_class00 = int(skip00)
        e.append_slots = int(append)
        return e

    def backward_blocks(self, tape: Dict, g: torch.Tensor, store: Store, lo: int, hi: int, premasked: bool = False):
        return drive(self.backward_blocks_iter(tape, g, store, lo, hi, premasked))

    def backward_blocks_iter(self, tape: Dict, g: torch.Tensor, store: Store, lo: int, hi: int,
                             premasked: bool = False):
        """Backward of blocks hi-1 .. lo (BasicBlock.forward, base_models.py:53-69).  Returns (gradient of
        block lo's input, premasked): with premasked the gradient is already multiplied by block lo-1's
        output ReLU mask and that block's bn2 (+ downsample BN) reductions are accumulated -- each dgrad
        that produces a BN's input gradient carries the BN-backward epilogue (avt_conv2d_dgrad_bn), so
        the standalone reduction pass runs only where the gradient enters a trunk (from the head)."""
        N = tape["N"]
        for bi in reversed(range(lo, hi)):
            blk, t = self.blocks[bi], tape["blocks"][bi]
            Hc, Wc, Ho, Wo = t["H"], t["W"], t["Ho"], t["Wo"]
            identity = blk["down"] is None
            if premasked:  # g = g' (masked), reductions already in the bn2 / downsample-BN accumulators
                gres = g
                g_c2 = self._bn_bwd_premasked(g, t["c2"], t["s2"], blk["bn2"], store)
                g_cd = None if identity else self._bn_bwd_premasked(g, t["cd"], t["sd"], blk["bnd"], store)
            else:  # g' = g * [out > 0] from the forward's mask bits; an identity block's residual gradient
                # enters the conv1 dgrad below as (g, mask) instead of a stored g'
                gres = None
                if identity and FUSE_BN_BWD and bi > 0:  # conv1's dgrad below carries a BN epilogue: store g'
                    gres = torch.empty_like(t["c2"])
                    g_c2 = self._bn_bwd(g, t["out"], t["c2"], t["s2"], blk["bn2"], store, gmask_out=gres)
                    g_cd = None
                elif identity:
                    g_c2, g_cd = self._bn_bwd_mask(g, t["om"], t["c2"], t["s2"], blk["bn2"], store)
                else:
                    g_c2, g_cd = self._bn_bwd_mask(g, t["om"], t["c2"], t["s2"], blk["bn2"], store,
                                                   t["cd"], t["sd"], blk["bnd"])
            yield
            self._wgrad(t["h1"], g_c2, N, Ho, Wo, blk["conv2"], store)
            yield
            if FUSE_BN_BWD:  # conv2 dgrad with bn1's backward (ReLU mask from its pre-activation) in the epilogue
                g_h1 = self._dgrad(g_c2, N, Ho, Wo, blk["conv2"], store,
                                   epi=self._epi(store, blk["bn1"], t["c1"], t["s1"]))
                g_c1 = self._bn_bwd_premasked(g_h1, t["c1"], t["s1"], blk["bn1"], store)
            else:
                g_h1 = self._dgrad(g_c2, N, Ho, Wo, blk["conv2"], store)
                yield
                g_c1 = self._bn_relu_bwd(g_h1, t["c1"], t["s1"], blk["bn1"], store)
            yield
            self._wgrad(t["x"], g_c1, N, Hc, Wc, blk["conv1"], store)
            yield
            if not identity:
                self._wgrad(t["x"], g_cd, N, Hc, Wc, blk["down"], store)
                yield
            epi = None
            if bi > 0 and FUSE_BN_BWD:  # the next block down: its bn2 (+ downsample BN) backward rides on this dgrad
                pb, pt = self.blocks[bi - 1], tape["blocks"][bi - 1]
                has_d = pb["down"] is not None
                mk = lambda skip00, append=False: self._epi(
                    store, pb["bn2"], pt["c2"], pt["s2"], y=pt["out"], bn2=pb["bnd"] if has_d else None,
                    xc2=pt["cd"] if has_d else None, stats2=pt["sd"] if has_d else None, skip00=skip00, append=append)
                epi = mk(False)
            if identity and gres is None:
                g_x = self._dgrad(g_c1, N, Hc, Wc, blk["conv1"], store, add=g, epi=epi, add_mask=t["om"])
            elif identity:
                g_x = self._dgrad(g_c1, N, Hc, Wc, blk["conv1"], store, add=gres, epi=epi)
            else:
                # the downsample dgrad (in place) finishes every pixel it reaches: the epilogue goes there;
                # of a stride-2 conv1 dgrad only the (odd) pixels it alone writes carry it
                strided = blk["conv1"].stride == 2
                g_x = self._dgrad(g_c1, N, Hc, Wc, blk["conv1"], store,
                                  epi=mk(True) if (epi is not None and strided) else None)
                if epi is not None and strided:  # the BN sums go after those of the conv1 dgrad just issued
                    epi = mk(False, append=True)
                g_x = self._dgrad(g_cd, N, Hc, Wc, blk["down"], store, add=g_x, inplace=True, epi=epi)
            g = g_x
            premasked = epi is not None
            yield
        return g, premasked

    def backward_stem(self, tape: Dict, g: torch.Tensor, store: Store):
        """maxpool -> relu/bn1 -> stem wgrad (and, when the tape asks for it, the input gradient)."""
        drive(self.backward_stem_iter(tape, g, store))

    def backward_stem_iter(self, tape: Dict, g: torch.Tensor, store: Store):
        N = tape["N"]
        H1, W1 = tape["H1"], tape["W1"]
        c0, st0 = tape["c0"], tape["st0"]
        g_c0 = torch.empty_like(c0)
        ws = store.stat_acc(self.bn1, "bwd", c0.numel() // 64)
        call("avt_stem_maxpool_bn_relu_bwd", P(g), P(tape["idx"]), P(tape["carg"]), P(c0), P(st0[0]), P(st0[1]),
             P(st0[2]), P(st0[3]), P(store.param(self.bn1.prefix + ".weight")),
             P(store.grad(self.bn1.prefix + ".weight")), P(store.grad(self.bn1.prefix + ".bias")), P(g_c0), P(ws),
             N, H1, W1, 64, stream_ptr())
        yield
        self._wgrad(tape["x"], g_c0, N, tape["H"], tape["W"], self.stem, store)
        if tape.get("want_dx"):  # d(loss)/d(input), NCHW fp32 (a standalone trunk whose input requires grad)
            gx = torch.empty(N, self.stem.cin, tape["H"], tape["W"], device=g_c0.device, dtype=torch.float32)
            call("avt_conv_stem_dgrad", P(g_c0), P(store.param(self.stem.name)), P(gx), N, tape["H"], tape["W"],
                 self.stem.cin, stream_ptr())
            tape["dx"] = gx

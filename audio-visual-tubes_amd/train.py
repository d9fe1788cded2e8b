"""Fused hard-way train step: forward + CE + backward + (RCCL all-reduce) + Adam, no autograd.

Equivalent to one iteration of train_hardway_1frame.py:121-135 (or train_3D.py:126-138 for a
FullModel) with the model wrapped for data parallelism.  The reference uses ``nn.DataParallel`` (train_hardway_1frame.py:93): each replica
contrasts only its own B/G samples (model.py:114-115), its BN uses its local batch statistics, and
the loss is the mean over the gathered logits, so the gradient is the mean of the replicas' local
mean-CE gradients.  Here each process owns one GPU and its local batch (same local-negative
semantics); gradients are summed with ONE all-reduce of the flat fp32 gradient buffer over RCCL
(backend "nccl"), the 1/world factor is folded into the Adam kernel, and BN running statistics
follow rank 0 (DDP ``broadcast_buffers``, matching DP's replica-0 buffers).

The all-reduce is bucketed and overlapped with backward, with the two trunks still running
concurrently: the flat gradient splits into one bucket per trunk for layer3+layer4 (~42 MB each, 94 %
of a ResNet-18's parameters) and one for the rest (~2.7 MB).  The backward runs as two segments --
layer4+layer3 of both trunks (audio on a second HIP stream), then layer2..stem of both -- and the two
"hi" buckets' RCCL all-reduces are launched (async, on RCCL's stream) at the boundary, so they travel
over xGMI while the second segment computes; only the two small "lo" buckets are exposed.  With a
captured step each segment is one HIP graph (sharing one memory pool, replayed in capture order) and
the collectives are issued between the replays.  (TwoView/Tube engines call the boundary once per
trunk, sequentially.)
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .engine import AVEngine
from .optim import FlatAdam


def world_size(pg: Optional[dist.ProcessGroup] = None) -> int:
    return dist.get_world_size(pg) if dist.is_available() and dist.is_initialized() else 1


def sync_gradients(grad: torch.Tensor, pg: Optional[dist.ProcessGroup] = None) -> float:
    """Sum the flat gradient over ranks in place (one collective); return the scale (1/world) that
    turns the sum into the data-parallel mean."""
    w = world_size(pg)
    if w > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=pg)
    return 1.0 / w


def sync_buffers(bflat: torch.Tensor, pg: Optional[dist.ProcessGroup] = None):
    """BN running statistics follow rank 0 (torch DDP broadcast_buffers semantics)."""
    if world_size(pg) > 1:
        dist.broadcast(bflat, 0, group=pg)


class HardWayTrainStep:
    def __init__(self, model, lr: float = 1e-6, weight_decay: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 process_group: Optional[dist.ProcessGroup] = None, engine=None, overlap_allreduce: bool = True):
        self.model = model
        self.engine: AVEngine = engine if engine is not None else model.engine()
        self.flat = model._flat
        self.opt = FlatAdam(self.flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.grad = torch.zeros(self.flat.n_train, device=self.flat.flat.device, dtype=torch.float32)
        self.pg = process_group
        self.world = world_size(process_group)
        # world > 1: per-bucket all-reduces overlapped with the second backward segment (default), or
        # ONE all-reduce of the whole flat gradient after the backward (overlap_allreduce=False)
        self.overlap = overlap_allreduce and self.world > 1
        if self.world > 1:
            # start from identical weights everywhere (DDP constructor semantics)
            dist.broadcast(self.flat.flat, 0, group=self.pg)
            sync_buffers(self.flat.bflat, self.pg)
        self._graph = None
        self._graph_opt = None
        self._seg_graphs = None
        self.buckets = dict(self.engine.grad_buckets())  # boundary tag -> flat gradient region
        # world 1, concurrent trunks: Adam runs per trunk region at the end of that trunk's backward
        # branch (no extra stream: the shorter trunk's update overlaps the longer trunk's backward), the
        # rest of the flat buffer after the join (AVT_ADAM_BRANCH=0: one Adam launch after the backward)
        self.adam_branch = (self.world == 1 and os.environ.get("AVT_ADAM_BRANCH", "1") != "0"
                            and type(self)._fwd_bwd is HardWayTrainStep._fwd_bwd
                            and type(self.engine).backward is AVEngine.backward)
        # Adam's step counter and the gradient zeroing on the vision branch (AVT_VISION_PRE=0: serial)
        self.vision_pre = os.environ.get("AVT_VISION_PRE", "1") != "0"

    def _fwd_bwd(self, *inputs, on_boundary=None) -> torch.Tensor:
        image, audio = inputs
        out, tape = self.engine.forward(image, audio, training=True, with_ce=True, ce_scale=1.0)
        self.grad.zero_()
        self.engine.backward(tape, out["dlogits"], self.grad, on_boundary)
        return out["loss"]

    def _trunk_region(self, tr):
        spans = [self.buckets[tr.prefix + k] for k in ("hi", "lo")]
        return min(a for a, _ in spans), max(b for _, b in spans)

    def _fwd_bwd_adam(self, image, audio) -> torch.Tensor:
        """World 1: forward + CE + backward + Adam, each trunk's parameters updated on its own branch
        as soon as its gradients are final; the same update as opt.step(grad) after the backward."""
        def pre():  # on the vision trunk's branch, off the serial section
            self.opt.prep()
            self.grad.zero_()

        if self.vision_pre:
            out, tape = self.engine.forward(image, audio, training=True, with_ce=True, ce_scale=1.0, vision_pre=pre)
        else:
            self.opt.prep()
            out, tape = self.engine.forward(image, audio, training=True, with_ce=True, ce_scale=1.0)
            self.grad.zero_()
        done = []

        def trunk_end(tr):
            lo, hi = self._trunk_region(tr)
            self.opt.apply(self.grad, lo, hi)
            done.append((lo, hi))

        self.engine.backward(tape, out["dlogits"], self.grad, None, on_trunk_end=trunk_end)
        pos = 0
        for lo, hi in sorted(done) + [(self.flat.n_train, self.flat.n_train)]:
            if lo > pos:
                self.opt.apply(self.grad, pos, lo)
            pos = max(pos, hi)
        return out["loss"]

    def step(self, *inputs: torch.Tensor) -> torch.Tensor:
        """step(image, audio).  Returns the local mean CE loss (device scalar, no host sync)."""
        if self._graph is not None or self._seg_graphs is not None:
            return self._replay(*inputs)
        return self._eager_step(*inputs)

    def _eager_step(self, *inputs: torch.Tensor) -> torch.Tensor:
        if self.world == 1 and self.adam_branch:
            return self._fwd_bwd_adam(*inputs)
        if self.world == 1:
            loss = self._fwd_bwd(*inputs)
            self.opt.step(self.grad, grad_scale=1.0)
            return loss
        sync_buffers(self.flat.bflat, self.pg)
        if not self.overlap:
            loss = self._fwd_bwd(*inputs)
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM, group=self.pg)
            self.opt.step(self.grad, grad_scale=1.0 / self.world)
            return loss
        return self._fwd_bwd_dp(*inputs)

    def _adam_stream(self):
        if getattr(self, "_adam_side", None) is None:
            self._adam_side = torch.cuda.Stream(device=self.grad.device)
        return self._adam_side

    def _dp_boundary(self, tags, pending: list):
        """World > 1, at a backward boundary: the bucket(s) just made final go out as async all-reduces; an
        upper-layer ("hi") bucket is then updated on the Adam side stream as soon as its collective completes --
        while the next backward segment computes -- and a "lo" bucket is left for the end of the step."""
        side = self._adam_stream()
        for tag in ((tags,) if isinstance(tags, str) else tags):
            lo, hi = self.buckets[tag]
            work = dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            if tag.endswith("hi"):
                side.wait_stream(torch.cuda.current_stream())  # Adam's prep (step counter) and the gradients
                with torch.cuda.stream(side):
                    work.wait()  # the side stream waits for RCCL's (no host sync)
                    self.opt.apply(self.grad, lo, hi, grad_scale=1.0 / self.world)
            else:
                pending.append((lo, hi, work))

    def _dp_finish(self, pending: list):
        for lo, hi, work in pending:
            work.wait()
            self.opt.apply(self.grad, lo, hi, grad_scale=1.0 / self.world)
        torch.cuda.current_stream().wait_stream(self._adam_stream())

    def _fwd_bwd_dp(self, *inputs) -> torch.Tensor:
        """World > 1 (overlap): forward with Adam's prep and the gradient zeroing on the vision branch (as at world
        1), backward in two segments with each bucket's all-reduce issued at its boundary and its Adam update
        applied as soon as that collective completes (_dp_boundary); the update of every parameter equals
        opt.step(all-reduced gradient, 1/world)."""
        def pre():
            self.opt.prep()
            self.grad.zero_()

        image, audio = inputs
        if type(self)._fwd_bwd is HardWayTrainStep._fwd_bwd and self.vision_pre:
            out, tape = self.engine.forward(image, audio, training=True, with_ce=True, ce_scale=1.0, vision_pre=pre)
            pending: list = []
            self.engine.backward(tape, out["dlogits"], self.grad, lambda tags: self._dp_boundary(tags, pending))
            self._dp_finish(pending)
            return out["loss"]
        self.opt.prep()
        pending = []
        loss = self._fwd_bwd(*inputs, on_boundary=lambda tags: self._dp_boundary(tags, pending))
        self._dp_finish(pending)
        return loss

    def capture(self, *inputs: torch.Tensor) -> None:
        """Record one step into HIP graph(s) (torch.cuda.CUDAGraph is hipGraph on ROCm) so that
        later steps are replays: no per-kernel host launch cost and no launch gaps between the
        ~700 kernels of a step.  World 1: one graph (fwd + CE + bwd + Adam).  World > 1, overlap schedule
        (default): one graph per backward segment (fwd + layer4/3 backward of both trunks | layer2..stem), replayed
        in order; between and after the replays the bucket all-reduces and their Adam updates stay eager
        (_dp_boundary: a "hi" bucket's update on the Adam side stream behind its collective; _dp_finish: the "lo"
        buckets, then the join).  World > 1 without overlap: fwd+bwd graph, the eager all-reduce, an Adam graph.
        ``image``/``audio``
        become the static inputs; later steps copy theirs in unless they pass these tensors.
        Call after at least one eager step (the engine allocates its buffers lazily).  Capture
        records launches without running them, so it has no effect on the training state."""
        torch.cuda.synchronize()
        self._static_in = inputs
        if self.world == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if self.adam_branch:
                    loss = self._fwd_bwd_adam(*inputs)
                else:
                    loss = self._fwd_bwd(*inputs)
                    self.opt.step(self.grad, grad_scale=1.0)
            self._static_loss = loss
            self._graph = g
            return
        if not self.overlap:  # world > 1: fwd+bwd graph, the all-reduce (eager), the Adam graph
            stream = torch.cuda.Stream()
            stream.wait_stream(torch.cuda.current_stream())
            pool = torch.cuda.graph_pool_handle()
            with torch.cuda.stream(stream):
                g = torch.cuda.CUDAGraph()
                g.capture_begin(pool=pool)
                loss = self._fwd_bwd(*inputs)
                g.capture_end()
                g_opt = torch.cuda.CUDAGraph()
                g_opt.capture_begin(pool=pool)
                self.opt.step(self.grad, grad_scale=1.0 / self.world)
                g_opt.capture_end()
            torch.cuda.current_stream().wait_stream(stream)
            torch.cuda.synchronize()
            self._static_loss, self._graph, self._graph_opt = loss, g, g_opt
            return
        # overlap: one graph per backward segment between bucket boundaries, then the Adam graph
        last_tag = list(self.buckets)[-1]
        graphs, tags = [], []
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        pool = torch.cuda.graph_pool_handle()  # one memory pool for all segments (replayed in order)
        with torch.cuda.stream(stream):
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=pool)
            graphs.append(g)

            def boundary(tag):
                graphs[-1].capture_end()
                tags.append(tag)
                got = (tag,) if isinstance(tag, str) else tuple(tag)
                if last_tag not in got:  # nothing is launched after the last bucket's boundary
                    g2 = torch.cuda.CUDAGraph()
                    g2.capture_begin(pool=pool)
                    graphs.append(g2)

            # Adam's prep rides in the first segment (on the vision branch, as _fwd_bwd_dp); the per-bucket updates
            # stay eager between the replays (_dp_boundary / _dp_finish), each behind its collective
            if type(self)._fwd_bwd is HardWayTrainStep._fwd_bwd and self.vision_pre:
                def pre():
                    self.opt.prep()
                    self.grad.zero_()

                image, audio = inputs
                out, tape = self.engine.forward(image, audio, training=True, with_ce=True, ce_scale=1.0,
                                                vision_pre=pre)
                self.engine.backward(tape, out["dlogits"], self.grad, boundary)
                loss = out["loss"]
            else:
                self.opt.prep()
                loss = self._fwd_bwd(*inputs, on_boundary=boundary)
            if not tags or last_tag not in ((tags[-1],) if isinstance(tags[-1], str) else tuple(tags[-1])):
                raise RuntimeError("avt: backward did not reach its last gradient bucket")
        torch.cuda.current_stream().wait_stream(stream)
        torch.cuda.synchronize()
        self._static_loss = loss
        self._seg_graphs, self._seg_tags, self._graph_opt = graphs, tags, None

    def _replay(self, *inputs: torch.Tensor) -> torch.Tensor:
        if len(inputs) != len(self._static_in) or any(
                tuple(x.shape) != tuple(s.shape) for s, x in zip(self._static_in, inputs)):
            # e.g. the short last batch of a drop_last=False DataLoader: a copy_ would broadcast a
            # 1-clip batch over all B rows (wrong negatives) -- run that batch eagerly instead
            return self._eager_step(*inputs)
        for s, x in zip(self._static_in, inputs):
            if x is not s:
                s.copy_(x)
        if self._seg_graphs is not None:
            sync_buffers(self.flat.bflat, self.pg)
            pending: list = []
            for g, tag in zip(self._seg_graphs, self._seg_tags):
                g.replay()
                self._dp_boundary(tag, pending)  # collectives + "hi" updates overlap the next segment's replay
            self._dp_finish(pending)
        elif self._graph_opt is not None:
            sync_buffers(self.flat.bflat, self.pg)
            self._graph.replay()
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM, group=self.pg)
            self._graph_opt.replay()
        else:
            self._graph.replay()
        return self._static_loss


class TwoViewTrainStep(HardWayTrainStep):
    """One train_hardway.py iteration (126-145): ``step(frames, augmented, spec)`` with frames /
    augmented [b,3,t,H,W] and one spectrogram per clip [b,1,F,T]; returns the device tensor
    losses[5] = (combined, hardway, aug, l2, consistency) — the five terms the reference logs.
    Defaults are train_hardway.py's: Adam lr 4e-6, weight_decay 1e-4, loss_weight 0.1.  Data
    parallel as HardWayTrainStep (each rank: its own clips, local negatives)."""

    def __init__(self, model, lr: float = 4e-6, weight_decay: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 loss_weight: float = 0.1, dedup_audio: bool = True,
                 process_group: Optional[dist.ProcessGroup] = None):
        from .twoview import TwoViewEngine

        # its own engine (packed weights, BN arena) over the model's flat storage: model(image, audio)
        # keeps working alongside
        e = TwoViewEngine(model._flat, model.epsilon, model.epsilon2, model.tau, model.trimap, model.Neg,
                          loss_weight=loss_weight, dedup_audio=dedup_audio)
        super().__init__(model, lr=lr, weight_decay=weight_decay, betas=betas, eps=eps, process_group=process_group,
                         engine=e)

    def _fwd_bwd(self, *inputs, on_boundary=None) -> torch.Tensor:
        frames, augmented, spec = inputs
        out, tape = self.engine.forward(frames, augmented, spec, training=True, with_ce=True)
        self.grad.zero_()
        self.engine.backward(tape, (out["dlogits"], out["dwA"]), self.grad, on_boundary)
        return out["losses"]

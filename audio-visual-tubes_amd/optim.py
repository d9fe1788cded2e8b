"""Fused Adam over an AVENet's flat parameter buffer (libavt ``avt_adam_step``).

Drop-in for ``torch.optim.Adam(model.parameters(), lr, weight_decay=wd)`` as used at
train_hardway_1frame.py:116/134 (betas (0.9, 0.999), eps 1e-8, coupled L2 decay, amsgrad off).
Parameters whose ``.grad`` is None are skipped, exactly like torch.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ._lib import call
from .trunk import P, stream_ptr


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("avt Adam: amsgrad is not used by the reference")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or not p.is_cuda:
                    raise TypeError("avt Adam: fp32 GPU parameters only")
                st: Dict = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad
                if g.stride() != p.stride():
                    g = torch.empty_like(p).copy_(g)  # match p's memory order (layout plumbing only)
                for t in (p, g, st["exp_avg"], st["exp_avg_sq"]):
                    if not _dense(t):
                        raise RuntimeError("avt Adam: non-dense parameter/grad layout")
                call("avt_adam_step", P(p), P(g), P(st["exp_avg"]), P(st["exp_avg_sq"]), p.numel(), 1.0, group["lr"],
                     b1, b2, group["eps"], group["weight_decay"], st["step"], stream_ptr())
        return loss


def _dense(t: torch.Tensor) -> bool:
    """True if t covers a contiguous block of memory in some dim order (e.g. channels_last)."""
    return t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last)


class FlatAdam:
    """Adam state for the trainable region of a FlatStore.  The step count AND the hyper-parameters
    live on the device (``avt_adam_step_dev`` reads them at every launch), so a step captured into
    a HIP graph follows later changes: ``opt.lr = x`` / ``set_lr(x)`` (a MultiStepLR schedule,
    train_hardway_1frame.py:118) or a restored checkpoint (checkpoint.load_flat_adam_state_dict)
    takes effect in the next replay.  The setters are stream-ordered device writes (no host sync)."""

    _HYPER = ("lr", "beta1", "beta2", "eps", "wd")

    def __init__(self, flat, lr=1e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4):
        self.flat = flat
        n = flat.n_train
        dev = flat.flat.device
        self.exp_avg = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(n, device=dev, dtype=torch.float32)
        self.t_dev = torch.zeros(1, device=dev, dtype=torch.int32)
        self._coef = torch.zeros(8, device=dev, dtype=torch.float32)  # AVT_ADAM_COEF_FLOATS
        self._host = {"lr": float(lr), "beta1": float(betas[0]), "beta2": float(betas[1]), "eps": float(eps),
                      "wd": float(weight_decay)}
        self.initial_lr = None  # set by the first scheduler, saved in checkpoints (torch's group 'initial_lr')
        self._hyper = torch.tensor([self._host[k] for k in self._HYPER], device=dev, dtype=torch.float32)

    def _set(self, key: str, value: float):
        self._host[key] = float(value)
        # a (stream-ordered) H2D copy: every later launch, graph replays included, reads the new value
        self._hyper[self._HYPER.index(key)] = float(value)

    @property
    def lr(self) -> float:
        return self._host["lr"]

    @lr.setter
    def lr(self, v: float):
        self._set("lr", v)

    def set_lr(self, v: float):
        self._set("lr", v)

    @property
    def betas(self):
        return (self._host["beta1"], self._host["beta2"])

    @betas.setter
    def betas(self, v):
        self._set("beta1", v[0])
        self._set("beta2", v[1])

    @property
    def eps(self) -> float:
        return self._host["eps"]

    @eps.setter
    def eps(self, v: float):
        self._set("eps", v)

    @property
    def wd(self) -> float:
        return self._host["wd"]

    @wd.setter
    def wd(self, v: float):
        self._set("wd", v)

    @property
    def t(self) -> int:
        """Steps taken (host read: synchronises)."""
        return int(self.t_dev.item())

    def step(self, gflat: torch.Tensor, grad_scale: float = 1.0):
        call("avt_adam_step_dev", P(self.flat.flat), P(gflat), P(self.exp_avg), P(self.exp_avg_sq),
             self.flat.n_train, grad_scale, P(self._hyper), P(self.t_dev), P(self._coef), stream_ptr())

    # step() in parts: prep() once per step (advances the step counter), then apply() over regions that
    # together cover [0, n_train) exactly once -- the same update, element for element
    def prep(self):
        call("avt_adam_prep_dev", P(self._hyper), P(self.t_dev), P(self._coef), stream_ptr())

    def apply(self, gflat: torch.Tensor, lo: int, hi: int, grad_scale: float = 1.0):
        if lo % 4 or (hi % 4 and hi != self.flat.n_train) or not 0 <= lo <= hi <= self.flat.n_train:
            raise ValueError(f"FlatAdam.apply: region [{lo}, {hi}) is not 16-byte aligned inside the flat buffer")
        call("avt_adam_apply_dev", P(self.flat.flat[lo:]), P(gflat[lo:]), P(self.exp_avg[lo:]),
             P(self.exp_avg_sq[lo:]), hi - lo, grad_scale, P(self._coef), stream_ptr())


class FlatMultiStepLR:
    """torch.optim.lr_scheduler.MultiStepLR (train_hardway_1frame.py:118: milestones [60,100,150,180],
    gamma 0.1, stepped once per epoch at :138) for a FlatAdam: lr = base_lr * gamma^(number of
    milestones <= epoch).  Writes the device hyper-parameter, so captured step graphs follow.

    base_lr is the optimizer's lr for a fresh schedule (last_epoch = -1; recorded as opt.initial_lr,
    like torch's group 'initial_lr').  Resuming (last_epoch = e >= 0: the constructor's step moves to
    epoch e+1, as torch's does) takes base_lr from the argument, else opt.initial_lr (restored with the
    checkpoint), else infers it from the optimizer's current lr -- the restored lr of epoch e+1 -- so
    the restored lr is kept and the decay never applied twice; later epochs follow the uninterrupted
    schedule (torch's chainable form multiplies the restored lr at each later milestone: the same)."""

    def __init__(self, opt: FlatAdam, milestones, gamma: float = 0.1, last_epoch: int = -1,
                 base_lr: Optional[float] = None):
        self.opt = opt
        self.milestones = sorted(int(m) for m in milestones)
        self.gamma = float(gamma)
        if base_lr is None:
            if last_epoch == -1:
                base_lr = opt.lr
            elif getattr(opt, "initial_lr", None) is not None:
                base_lr = opt.initial_lr
            else:
                base_lr = opt.lr / self.gamma ** self._decays(last_epoch + 1)
        self.base_lr = float(base_lr)
        if getattr(opt, "initial_lr", None) is None:
            opt.initial_lr = self.base_lr
        self.last_epoch = last_epoch
        self.step()

    def _decays(self, epoch: int) -> int:
        return sum(1 for m in self.milestones if m <= epoch)

    def get_last_lr(self):
        return [self.opt.lr]

    def step(self):
        self.last_epoch += 1
        lr = self.base_lr * self.gamma ** self._decays(self.last_epoch)
        if lr != self.opt.lr:
            self.opt.set_lr(lr)

    def state_dict(self):
        return {"milestones": self.milestones, "gamma": self.gamma, "base_lr": self.base_lr,
                "last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.milestones, self.gamma = list(sd["milestones"]), float(sd["gamma"])
        self.base_lr, self.last_epoch = float(sd["base_lr"]), int(sd["last_epoch"])
        k = sum(1 for m in self.milestones if m <= self.last_epoch)
        self.opt.set_lr(self.base_lr * self.gamma ** k)

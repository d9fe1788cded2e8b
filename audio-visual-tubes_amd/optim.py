"""Fused Adam over an AVENet's flat parameter buffer (libavt ``avt_adam_step``).

Drop-in for ``torch.optim.Adam(model.parameters(), lr, weight_decay=wd)`` as used at
train_hardway_1frame.py:116/134 (betas (0.9, 0.999), eps 1e-8, coupled L2 decay, amsgrad off).
Parameters whose ``.grad`` is None are skipped, exactly like torch.
"""
from __future__ import annotations

from typing import Dict

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
    """Adam state for the trainable region of a FlatStore.  The step count lives on the device
    (``avt_adam_step_dev``), so a step is replayable from a captured HIP graph."""

    def __init__(self, flat, lr=1e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4):
        self.flat = flat
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        n = flat.n_train
        dev = flat.flat.device
        self.exp_avg = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(n, device=dev, dtype=torch.float32)
        self.t_dev = torch.zeros(1, device=dev, dtype=torch.int32)
        self._coef = torch.zeros(2, device=dev, dtype=torch.float32)

    @property
    def t(self) -> int:
        """Steps taken (host read: synchronises)."""
        return int(self.t_dev.item())

    def step(self, gflat: torch.Tensor, grad_scale: float = 1.0):
        call("avt_adam_step_dev", P(self.flat.flat), P(gflat), P(self.exp_avg), P(self.exp_avg_sq),
             self.flat.n_train, grad_scale, self.lr, self.betas[0], self.betas[1], self.eps, self.wd, P(self.t_dev),
             P(self._coef), stream_ptr())

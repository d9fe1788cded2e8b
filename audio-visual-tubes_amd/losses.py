"""Drop-in for the loss the reference's 16-frame step imports from losses.py (train_hardway.py:110:
``criterion2 = PropagationLoss()``), computed by libavt (``avt_propagation_loss``, HIP).

``PropagationLoss()(heatmap)`` with heatmap [b, t, h, w] = mean over (clip, frame pair, pixel) of
|heatmap[:, s+1] - heatmap[:, s]| (losses.py:16-23).  Its gradient is produced in the same launch
and scaled by the upstream gradient in backward.
"""
from __future__ import annotations

import torch
from torch import nn

from ._lib import call
from .trunk import P, stream_ptr


class _PropagationLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, heatmap: torch.Tensor):
        if not heatmap.is_cuda:
            raise RuntimeError("avt: PropagationLoss runs on the GPU (no CPU path)")
        if heatmap.dim() != 4:
            raise ValueError(f"avt: PropagationLoss expects [b, t, h, w], got {tuple(heatmap.shape)}")
        b, t, h, w = heatmap.shape
        if t < 2:
            raise ValueError("avt: PropagationLoss needs t >= 2 (the reference's mean over an empty diff is NaN)")
        x = heatmap.detach().contiguous().float()
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        dx = torch.empty_like(x) if heatmap.requires_grad else None
        call("avt_propagation_loss", P(x), b, t, h * w, P(loss), P(dx), stream_ptr())
        ctx.save_for_backward(dx)
        ctx.in_dtype = heatmap.dtype
        return loss.to(heatmap.dtype)

    @staticmethod
    def backward(ctx, g):
        (dx,) = ctx.saved_tensors
        return (dx * g).to(ctx.in_dtype)


class PropagationLoss(nn.Module):
    """losses.py:16-23."""

    def forward(self, heatmap: torch.Tensor) -> torch.Tensor:
        return _PropagationLossFn.apply(heatmap)

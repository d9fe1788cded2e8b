"""Drop-ins for the reference's losses.py, computed by libavt (HIP); each gradient is produced in the
forward launch and scaled by the upstream gradient in backward.

* ``PropagationLoss()(heatmap)`` (losses.py:16-23; train_hardway.py:110 ``criterion2``), heatmap
  [b, t, h, w]: mean over (clip, frame pair, pixel) of |heatmap[:, s+1] - heatmap[:, s]|.
* ``NPRatio()(heatmap)`` (losses.py:7-14; train_3D.py:113, 135 ``criterion2``), heatmap [b, t, h, w]:
  mean over (clip, frame pair) of |sum_hw heatmap[:, s+1] - sum_hw heatmap[:, s]|.
* ``FlipLoss()(heatmap, flipped_heatmap)`` (losses.py:25-36): nn.L1Loss()(flipped_heatmap,
  RandomHorizontalFlip(p=1)(heatmap)), the flip along the last dimension.

Each runs on a multi-block grid (no size limit): gradients elementwise, the loss as per-block partial
sums that one block adds in a fixed order (deterministic, run to run).
"""
from __future__ import annotations

import torch
from torch import nn

from ._lib import call, query
from .trunk import P, stream_ptr


def _workspace(x: torch.Tensor, rows: int = 0) -> torch.Tensor:
    """Scratch of the multi-block loss kernels (per-block partial sums, NPRatio's row sums)."""
    return torch.empty(int(query("avt_loss_workspace_floats", x.numel(), rows)), device=x.device, dtype=torch.float32)


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
        call("avt_propagation_loss", P(x), b, t, h * w, P(loss), P(dx), P(_workspace(x)), stream_ptr())
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


class _NPRatioFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, heatmap: torch.Tensor):
        if not heatmap.is_cuda:
            raise RuntimeError("avt: NPRatio runs on the GPU (no CPU path)")
        if heatmap.dim() != 4:
            raise ValueError(f"avt: NPRatio expects [b, t, h, w], got {tuple(heatmap.shape)}")
        b, t, h, w = heatmap.shape
        if t < 2:
            raise ValueError("avt: NPRatio needs t >= 2 (the reference's mean over an empty diff is NaN)")
        x = heatmap.detach().contiguous().float()
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        dx = torch.empty_like(x) if heatmap.requires_grad else None
        call("avt_npratio_loss", P(x), b, t, h * w, P(loss), P(dx), P(_workspace(x, b * t)), stream_ptr())
        ctx.save_for_backward(dx)
        ctx.in_dtype = heatmap.dtype
        return loss.to(heatmap.dtype)

    @staticmethod
    def backward(ctx, g):
        (dx,) = ctx.saved_tensors
        return (dx * g).to(ctx.in_dtype)


class NPRatio(nn.Module):
    """losses.py:7-14 (Negative / Positive Ratio Loss)."""

    def forward(self, heatmap: torch.Tensor) -> torch.Tensor:
        return _NPRatioFn.apply(heatmap)


class _FlipLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, heatmap: torch.Tensor, flipped: torch.Tensor):
        if not heatmap.is_cuda or not flipped.is_cuda:
            raise RuntimeError("avt: FlipLoss runs on the GPU (no CPU path)")
        if heatmap.shape != flipped.shape or heatmap.dim() < 1:
            raise ValueError(f"avt: FlipLoss needs two tensors of one shape, got {tuple(heatmap.shape)} and "
                             f"{tuple(flipped.shape)}")
        x = heatmap.detach().contiguous().float()
        y = flipped.detach().contiguous().float()
        W = x.shape[-1]
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        dx = torch.empty_like(x) if heatmap.requires_grad else None
        dy = torch.empty_like(y) if flipped.requires_grad else None
        call("avt_flip_l1_loss", P(x), P(y), x.numel() // W, W, P(loss), P(dx), P(dy), P(_workspace(x)), stream_ptr())
        ctx.save_for_backward(dx, dy)
        ctx.dtypes = (heatmap.dtype, flipped.dtype)
        return loss.to(flipped.dtype)

    @staticmethod
    def backward(ctx, g):
        dx, dy = ctx.saved_tensors
        return (None if dx is None else (dx * g).to(ctx.dtypes[0]),
                None if dy is None else (dy * g).to(ctx.dtypes[1]))


class FlipLoss(nn.Module):
    """losses.py:25-36: L1 between flipped_heatmap and the horizontally flipped heatmap."""

    def forward(self, heatmap: torch.Tensor, flipped_heatmap: torch.Tensor) -> torch.Tensor:
        return _FlipLossFn.apply(heatmap, flipped_heatmap)

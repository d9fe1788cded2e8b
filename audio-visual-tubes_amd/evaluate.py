"""Localisation evaluation of the reference's test loops on libavt (HIP), batched over heatmaps.

The reference evaluates one heatmap at a time on the host (train_hardway_1frame.py:187-216,
train_hardway.py test loop, test.py:85-172): cv2 resize 14x14 -> 224x224, normalise, median-binarise,
``utils.Evaluator.cal_CIOU(pred, gt, 0.5)``, then cIoU@0.5 and AUC over the test set, and mTC over
consecutive frames.  Here the per-map work runs in one launch for the whole batch of heatmaps
(``avt_localize_ciou``: one block per map, exact median by radix select) straight from the model's
``A`` on the device; the 21-point AUC of the resulting cIoU vector is host arithmetic on N numbers,
as in the reference.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import call
from .trunk import P, stream_ptr

GT_SIZE = 224


def localize(A: torch.Tensor, gt: Optional[torch.Tensor] = None, size: int = GT_SIZE,
             return_maps: bool = False) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """A: heatmaps [N,1,h,w] (AVENet's first output) or [N,h,w] on the GPU; gt: [N,size,size] maps.
    Returns (stats [N,3] fp64 = (cIoU, intersection, denominator) or None without gt,
             binary prediction maps [N,size,size] uint8 if return_maps)."""
    if not A.is_cuda:
        raise RuntimeError("avt: localize runs on the GPU (no CPU path)")
    if A.dim() == 4:
        if A.shape[1] != 1:
            raise ValueError(f"avt: heatmaps must be [N,1,h,w], got {tuple(A.shape)}")
        A = A[:, 0]
    if A.dim() != 3:
        raise ValueError(f"avt: heatmaps must be [N,h,w], got {tuple(A.shape)}")
    N, h, w = A.shape
    if gt is None and not return_maps:
        raise ValueError("avt: localize needs gt maps or return_maps=True")
    A = A.detach().contiguous().float()
    stats = maps = None
    if gt is not None:
        if tuple(gt.shape) != (N, size, size):
            raise ValueError(f"avt: gt must be [{N},{size},{size}], got {tuple(gt.shape)}")
        gt = gt.to(A.device).contiguous().float()
        stats = torch.empty(N, 3, device=A.device, dtype=torch.float64)
    if return_maps:
        maps = torch.empty(N, size, size, device=A.device, dtype=torch.uint8)
    call("avt_localize_ciou", P(A), N, h, w, size, P(gt), P(stats), P(maps), stream_ptr())
    return stats, maps


def mtc(pred_maps: torch.Tensor) -> float:
    """utils.mTC (utils.py:311-318): mean cIoU(pred_i, pred_{i+1}, 0.5) over consecutive frames,
    from ``localize(..., return_maps=True)`` maps [T,S,S] of one clip."""
    if pred_maps.shape[0] < 2:
        raise ValueError("avt: mTC needs at least two frames")
    p = pred_maps.contiguous()
    T = p.shape[0]
    out = torch.empty(T - 1, device=p.device, dtype=torch.float64)
    call("avt_pair_ciou", P(p), T, p[0].numel(), P(out), stream_ptr())
    return float(out.sum().item() / (T - 1))


def auc_from_cious(cious: Sequence[float]) -> float:
    """utils.Evaluator.cal_AUC (utils.py:216-225): trapezoid area under the fraction of maps with
    cIoU >= 0.05 i, i = 0..20 (sklearn.metrics.auc of a monotonic x is the trapezoid rule)."""
    c = np.asarray(cious, dtype=np.float64)
    x = np.array([0.05 * i for i in range(21)])
    y = np.array([np.sum(c >= 0.05 * i) / len(c) for i in range(21)])
    return float(np.sum((x[1:] - x[:-1]) * (y[1:] + y[:-1]) / 2))


class Evaluator:
    """utils.Evaluator (utils.py:203-231): accumulates cIoUs; ``cal_CIOU(infer, gtmap, thres)`` on
    [S,S] maps (numpy or tensors), ``add`` for a localize() batch, ``cal_AUC``, ``final`` (cIoU@0.5)."""

    def __init__(self):
        self.ciou = []

    def cal_CIOU(self, infer, gtmap, thres=0.01):
        infer = torch.as_tensor(infer)
        gtmap = torch.as_tensor(gtmap, device=infer.device).double()
        infer_map = (infer >= thres).double()
        inter = float((infer_map * gtmap).sum())
        denom = float(gtmap.sum() + (infer_map * (gtmap == 0)).sum())
        ciou = inter / denom
        self.ciou.append(ciou)
        return ciou, inter, denom

    def add(self, stats: torch.Tensor):
        self.ciou.extend(stats[:, 0].tolist())

    def cal_AUC(self):
        return auc_from_cious(self.ciou)

    def final(self):
        return float(np.mean(np.array(self.ciou) >= 0.5))

    def clear(self):
        self.ciou = []


def gt_map_flickr(bboxs, size: int = GT_SIZE) -> np.ndarray:
    """utils.testset_gt flickr branch (utils.py:243-263) from the parsed XML boxes [xmin, ymin, xmax,
    ymax] (annotation frame 256 px): boxes scaled to 224, summed, halved, clipped at 1."""
    gt = np.zeros([size, size])
    for b in bboxs:
        x0, y0, x1, y1 = [int(size * int(v) / 256) for v in b]
        gt[y0:y1, x0:x1] += 1
    gt /= 2
    gt[gt > 1] = 1
    return gt


def gt_map_vggss(bboxs, size: int = GT_SIZE) -> np.ndarray:
    """utils.testset_gt vggss branch (utils.py:264-273) from normalised boxes [xmin, ymin, xmax, ymax]."""
    gt = np.zeros([size, size])
    for b in bboxs:
        x0, y0, x1, y1 = [int(size * max(x, 0)) for x in b]
        gt[y0:y1, x0:x1] += 1
    gt[gt > 0] = 1
    return gt


@torch.no_grad()
def evaluate_hardway(model, batches, gt_maps) -> Tuple[float, float]:
    """The test_hardway loop (train_hardway_1frame.py:187-216): eval-mode forward of each (image,
    spec) batch, localisation of every heatmap against its gt map.  ``batches`` yields (image, spec)
    GPU tensors; ``gt_maps`` yields the matching [B,224,224] maps.  Returns (cIoU@0.5, AUC)."""
    was_training = model.training
    model.eval()
    ev = Evaluator()
    try:
        for (image, spec), gt in zip(batches, gt_maps):
            A = model(image.float(), spec.float())[0]
            stats, _ = localize(A, torch.as_tensor(gt))
            ev.add(stats)
    finally:
        model.train(was_training)
    return ev.final(), ev.cal_AUC()

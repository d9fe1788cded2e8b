"""CPU restatement of the reference's localisation evaluation — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module (as the checker of ``avt_localize_ciou`` / ``avt_pair_ciou``
and ``avt_amd.evaluate``).  What it restates (reference file:line):

  * the per-map test protocol of train_hardway_1frame.py:195-206 (same in 150-164, 227-240 and
    train_hardway.py's test loop; test.py:97-130 with the layer4-activation map):
        heatmap_now = cv2.resize(heatmap[i, 0], (224, 224), interpolation=cv2.INTER_LINEAR)
        heatmap_now = normalize_img(-heatmap_now);  pred = 1 - heatmap_now
        threshold = np.sort(pred.flatten())[int(224 * 224 / 2)]
        pred[pred > threshold] = 1;  pred[pred < 1] = 0
        ciou = Evaluator().cal_CIOU(pred, gt_map, 0.5)
  * utils.Evaluator.cal_CIOU / cal_AUC / final (utils.py:203-231), normalize_img (234-239),
    testset_gt's box rasterisation (241-274), mTC (311-318).

cv2 is not importable in this image, so ``cv2.resize(INTER_LINEAR)`` is restated from
OpenCV's published algorithm for float images (half-pixel centres fx = (x+0.5)*src/dst - 0.5,
floor, edge clamp with zero weight; horizontal pass then vertical, fp32 products and sums).
Parity of that resize with OpenCV itself is therefore UNPINNED (its SIMD path may contract the
products into FMAs: last-bit differences that can move a pixel across the median); it is checked
against torch's independent bilinear (align_corners=False) implementation.  sklearn.metrics.auc
(the reference's own call) is used directly.
"""
from __future__ import annotations

import numpy as np


def _coef(src: int, dst: int):
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * (src / dst) - 0.5).astype(np.float32)
    i = np.floor(f).astype(np.int64)
    f = (f - i.astype(np.float32)).astype(np.float32)
    lo = i < 0
    f[lo], i[lo] = 0.0, 0
    hi = i >= src - 1
    f[hi], i[hi] = 0.0, src - 1
    return i, (np.float32(1.0) - f).astype(np.float32), f


def cv2_resize_linear(m: np.ndarray, size: int = 224) -> np.ndarray:
    """cv2.resize(m, (size, size), interpolation=cv2.INTER_LINEAR) for a 2-D float32 map."""
    m = np.asarray(m, dtype=np.float32)
    h, w = m.shape
    sy, ay0, ay1 = _coef(h, size)
    sx, ax0, ax1 = _coef(w, size)
    sy1, sx1 = np.minimum(sy + 1, h - 1), np.minimum(sx + 1, w - 1)
    rows = m[:, sx] * ax0[None, :] + m[:, sx1] * ax1[None, :]   # horizontal pass, [h, size] fp32
    return (rows[sy, :] * ay0[:, None] + rows[sy1, :] * ay1[:, None]).astype(np.float32)


def normalize_img(value, vmax=None, vmin=None):
    """utils.py:234-239."""
    vmin = value.min() if vmin is None else vmin
    vmax = value.max() if vmax is None else vmax
    if not (vmax - vmin) == 0:
        value = (value - vmin) / (vmax - vmin)
    return value


def binarize(heatmap: np.ndarray, size: int = 224) -> np.ndarray:
    """train_hardway_1frame.py:198-204: resize, normalise, 1 - ., median threshold, binarise."""
    heatmap_now = normalize_img(-cv2_resize_linear(heatmap, size))
    pred = 1 - heatmap_now
    threshold = np.sort(pred.flatten())[int(pred.shape[0] * pred.shape[1] / 2)]
    pred[pred > threshold] = 1
    pred[pred < 1] = 0
    return pred


def cal_ciou(infer, gtmap, thres=0.01):
    """utils.Evaluator.cal_CIOU (utils.py:209-214) -> (ciou, intersection, denominator)."""
    infer_map = np.zeros(gtmap.shape)
    infer_map[infer >= thres] = 1
    inter = np.sum(infer_map * gtmap)
    denom = np.sum(gtmap) + np.sum(infer_map * (gtmap == 0))
    return inter / denom, inter, denom


def cal_auc(cious):
    """utils.Evaluator.cal_AUC (utils.py:216-225)."""
    from sklearn.metrics import auc

    results = [np.sum(np.array(cious) >= 0.05 * i) / len(cious) for i in range(21)]
    return auc([0.05 * i for i in range(21)], results)


def mtc(preds):
    """utils.mTC (utils.py:311-318): mean cIoU of consecutive binarised maps."""
    c = [cal_ciou(preds[i], preds[i + 1], 0.5)[0] for i in range(len(preds) - 1)]
    return float(np.sum(c) / (len(preds) - 1))


def gt_map_flickr(bboxs, size=224):
    """testset_gt flickr branch (utils.py:243-263) from parsed XML boxes [xmin, ymin, xmax, ymax] in
    the annotation's 256-pixel frame."""
    gt_map = np.zeros([size, size])
    for b in bboxs:
        item = [int(size * int(v) / 256) for v in b]
        temp = np.zeros([size, size])
        temp[item[1]:item[3], item[0]:item[2]] = 1
        gt_map += temp
    gt_map /= 2
    gt_map[gt_map > 1] = 1
    return gt_map


def gt_map_vggss(bboxs, size=224):
    """testset_gt vggss branch (utils.py:264-273) from normalised boxes [xmin, ymin, xmax, ymax]."""
    gt_map = np.zeros([size, size])
    for b in bboxs:
        xmin, ymin, xmax, ymax = [int(size * max(x, 0)) for x in b]
        temp = np.zeros([size, size])
        temp[ymin:ymax, xmin:xmax] = 1
        gt_map += temp
    gt_map[gt_map > 0] = 1
    return gt_map

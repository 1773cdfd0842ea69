"""ORACLE — test infrastructure only.  Pairwise box costs restated from boxmot/utils/iou.py.

Every function keeps the reference's NumPy operation order (it decides the last bit of each
float64 cost, and the HIP kernels are checked bit-exact against these).
"""
import numpy as np


def _overlap(a, b):
    """Shared intersection terms of iou.py:13-19 / :39-45 / :77-83 / :120-126."""
    a = a[:, None, :]
    b = b[None, :, :]
    iw = np.maximum(0.0, np.minimum(a[..., 2], b[..., 2]) - np.maximum(a[..., 0], b[..., 0]))
    ih = np.maximum(0.0, np.minimum(a[..., 3], b[..., 3]) - np.maximum(a[..., 1], b[..., 1]))
    inter = iw * ih
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    return a, b, inter, inter / (area_a + area_b - inter)


def iou_batch(a, b):
    """iou.py:6-25."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return _overlap(a, b)[3]


def giou_batch(a, b):
    """iou.py:28-62 (incl. the enclosure assertion at :58)."""
    a, b, inter, iou = _overlap(np.asarray(a, np.float64), np.asarray(b, np.float64))
    ew = np.maximum(a[..., 2], b[..., 2]) - np.minimum(a[..., 0], b[..., 0])
    eh = np.maximum(a[..., 3], b[..., 3]) - np.minimum(a[..., 1], b[..., 1])
    assert (ew > 0).all() and (eh > 0).all()
    enc = ew * eh
    g = iou - (enc - inter) / enc
    return (g + 1.0) / 2.0


def _centre_terms(a, b):
    cxa = (a[..., 0] + a[..., 2]) / 2.0
    cya = (a[..., 1] + a[..., 3]) / 2.0
    cxb = (b[..., 0] + b[..., 2]) / 2.0
    cyb = (b[..., 1] + b[..., 3]) / 2.0
    inner = (cxa - cxb) ** 2 + (cya - cyb) ** 2
    ex = np.maximum(a[..., 2], b[..., 2]) - np.minimum(a[..., 0], b[..., 0])
    ey = np.maximum(a[..., 3], b[..., 3]) - np.minimum(a[..., 1], b[..., 1])
    outer = ex ** 2 + ey ** 2
    return inner, outer


def diou_batch(a, b):
    """iou.py:65-105."""
    a, b, inter, iou = _overlap(np.asarray(a, np.float64), np.asarray(b, np.float64))
    inner, outer = _centre_terms(a, b)
    return (iou - inner / outer + 1) / 2.0


def ciou_batch(a, b):
    """iou.py:108-161 (+1 px on both heights, :152-155)."""
    a, b, inter, iou = _overlap(np.asarray(a, np.float64), np.asarray(b, np.float64))
    inner, outer = _centre_terms(a, b)
    wa = a[..., 2] - a[..., 0]
    ha = a[..., 3] - a[..., 1] + 1.0
    wb = b[..., 2] - b[..., 0]
    hb = b[..., 3] - b[..., 1] + 1.0
    at = np.arctan(wb / hb) - np.arctan(wa / ha)
    v = (4 / (np.pi ** 2)) * (at ** 2)
    alpha = v / ((1 - iou) + v)
    return (iou - inner / outer - alpha * v + 1) / 2.0


def centroid_batch(a, b, w, h):
    """iou.py:164-188."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    ca = np.stack(((a[..., 0] + a[..., 2]) / 2, (a[..., 1] + a[..., 3]) / 2), axis=-1)[:, None]
    cb = np.stack(((b[..., 0] + b[..., 2]) / 2, (b[..., 1] + b[..., 3]) / 2), axis=-1)[None]
    dist = np.sqrt(np.sum((ca - cb) ** 2, axis=-1))
    return 1 - dist / np.sqrt(w ** 2 + h ** 2)


def iou_distance(a_boxes, b_boxes):
    """matching.py:94-119: 1 - IoU, float32 zeros when either side is empty."""
    if len(a_boxes) == 0 or len(b_boxes) == 0:
        return np.zeros((len(a_boxes), len(b_boxes)), dtype=np.float32)
    return 1 - iou_batch(np.asarray(a_boxes), np.asarray(b_boxes))


def fuse_score(cost, scores):
    """matching.py:213-221: 1 - (1 - cost) * score_j."""
    if cost.size == 0:
        return cost
    sim = 1 - cost
    return 1 - sim * np.asarray(scores, dtype=np.float64)[None, :]

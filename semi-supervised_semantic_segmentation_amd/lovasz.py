"""Lovász-softmax helpers — drop-in for reference lovasz.py (Berman 2018, MIT).

Device work (sort + scan + dot) runs in ssseg_lovasz_*; the small host helpers keep the reference's
semantics: lovasz_grad (lovasz.py:19-31), iou_binary / iou (:34-73, the mIoU of BASELINE's parity
report), mean (:235-253).
"""
from itertools import filterfalse as ifilterfalse

import numpy as np
import torch

from ssseg import ops


def lovasz_grad(gt_sorted):
    gts = gt_sorted.sum()
    intersection = gts - gt_sorted.float().cumsum(0)
    union = gts + (1 - gt_sorted).float().cumsum(0)
    jaccard = 1. - intersection / union
    if len(gt_sorted) > 1:
        jaccard[1:] = jaccard[1:] - jaccard[:-1].clone()
    return jaccard


def iou_binary(preds, labels, EMPTY=1., ignore=None, per_image=True):
    if not per_image:
        preds, labels = (preds,), (labels,)
    ious = []
    for pred, label in zip(preds, labels):
        inter = ((label == 1) & (pred == 1)).sum()
        union = ((label == 1) | ((pred == 1) & (label != ignore))).sum()
        ious.append(EMPTY if not union else float(inter) / float(union))
    return 100 * mean(ious)


def iou(preds, labels, C, EMPTY=1., ignore=None, per_image=False):
    if not per_image:
        preds, labels = (preds,), (labels,)
    per = []
    for pred, label in zip(preds, labels):
        row = []
        for c in range(C):
            if c == ignore:
                continue
            inter = ((label == c) & (pred == c)).sum()
            union = ((label == c) | ((pred == c) & (label != ignore))).sum()
            row.append(EMPTY if not union else float(inter) / float(union))
        per.append(row)
    return 100 * np.array([mean(col) for col in zip(*per)])


def lovasz_softmax(probas, labels, classes='present', per_image=False, ignore=None):
    """lovasz.py:155-170 for the configuration the hot path uses (binary logits [B,2,H,W], classes=[1],
    per_image=True): dispatched to the device kernel.  Other configurations are not implemented."""
    if not (per_image and list(classes) == [1] and probas.dim() == 4 and probas.shape[1] == 2):
        raise NotImplementedError('lovasz_softmax: only the binary per-image configuration of losses.py:249')
    target = torch.stack([(labels == 0), (labels == 1)], 1).to(probas.dtype)
    return ops.lovasz_binary(probas, target, valid_weighted=False)


def isnan(x):
    return x != x


def mean(values, ignore_nan=False, empty=0):
    it = iter(values)
    if ignore_nan:
        it = ifilterfalse(isnan, it)
    try:
        n = 1
        acc = next(it)
    except StopIteration:
        if empty == 'raise':
            raise ValueError('Empty mean')
        return empty
    for n, v in enumerate(it, 2):
        acc += v
    return acc if n == 1 else acc / n

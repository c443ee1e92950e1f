"""Losses — drop-in for the hot-path part of reference losses.py, on the MI355X kernels.

  CalculateLoss                           losses.py:8-22   (bilinear resize of each prediction + weighted sum)
  DenseBinaryCrossEntropyLossWithLogits   losses.py:41-48  (reduction='mean')
  binary_lovasz_loss_with_logits          losses.py:239-250
Out of scope (not in the hot path / BASELINE configs): Focal, OHEM, Dice, NormalizedFocal, entropy,
RMILoss (losses.py:51-230, 271-592) — importing them raises NotImplementedError.
"""
import torch
import torch.nn as nn

from ssseg import ops


class CalculateLoss:
    def __init__(self, losses):
        # losses: list of {'loss_fn': callable(prediction, target), 'weight': [w per prediction]}
        self.losses = losses

    def __call__(self, predictions_list, target):
        total = None
        size = (target.size(2), target.size(3))
        for idx, prediction in enumerate(predictions_list):
            prediction = ops.interpolate_bilinear(prediction, size, align_corners=False)
            for spec in self.losses:
                term, w = spec['loss_fn'](prediction, target), float(spec['weight'][idx])
                # total + term * w on the device (ssseg_axpby): same fp32 arithmetic as the reference's
                total = ops.scale(term, w) if total is None else ops.add_scaled(total, term, w)
        return total if total is not None else 0


class DenseBinaryCrossEntropyLossWithLogits(nn.Module):
    def __init__(self, reduction='mean'):
        super().__init__()
        if reduction != 'mean':
            raise NotImplementedError('only reduction="mean" has a kernel (the hot-path configuration)')
        self.reduction = reduction

    def forward(self, input, target):
        return ops.bce_with_logits_mean(input, target)


def binary_lovasz_loss_with_logits(input, target):
    """losses.py:239-250: per-image binary Lovász-softmax on raw logits (class 1), sum(loss*valid)/(sum valid + 0.001)."""
    return ops.lovasz_binary(input, target)


def _out_of_scope(name):
    def f(*a, **k):
        raise NotImplementedError(f'losses.{name} is outside the MI355X hot path (SURVEY §2.1 row 3)')
    return f


for _n in ('DenseCrossEntropyLossWithLogits', 'OhemCrossEntropy', 'FocalLoss', 'DiceWithLogitsLoss', 'RMILoss',
           'NormalizedFocalLossSigmoid', 'binary_entropy_loss', 'entropy_loss', 'log_dice_loss'):
    globals()[_n] = _out_of_scope(_n)

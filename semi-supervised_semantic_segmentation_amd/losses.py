"""Losses — drop-in for the hot-path part of reference losses.py, on the MI355X kernels.

  CalculateLoss                           losses.py:8-22   (bilinear resize of each prediction + weighted sum)
  DenseBinaryCrossEntropyLossWithLogits   losses.py:41-48  (reduction='mean')
  binary_lovasz_loss_with_logits          losses.py:239-250
  RMILoss                                 losses.py:271-592 (the default-config loss, configs/default_config.py:147;
                                          sigmoid form, rmi_pool 'avg' / 'none', rmi_radius 1-3)
Out of scope (not in the hot path / BASELINE configs): Focal, OHEM, Dice, NormalizedFocal, entropy
(losses.py:51-230) — calling them raises NotImplementedError.
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


class RMILoss(nn.Module):
    """Region mutual information loss (losses.py:271-592), forward = forward_sigmoid (losses.py:480-518).

    Same constructor and checks as the reference (:286-311).  The device kernels (csrc/rmi.hip) cover the pools the
    reference's configs use ('avg', and 'none') and rmi_radius 1-3 (D = radius^2 <= 9; the default config uses 3);
    'max' / 'interpolation' pooling and larger radii raise NotImplementedError here rather than run elsewhere."""

    _CLIP_MIN = 1e-6    # losses.py:281-283
    _CLIP_MAX = 1.0
    _POS_ALPHA = 5e-4
    _IS_SUM = 1

    def __init__(self, num_classes=21, rmi_radius=3, rmi_pool='avg', rmi_pool_size=3, rmi_pool_stride=3):
        super().__init__()
        self.num_classes = num_classes
        assert rmi_radius in [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
        self.rmi_radius = rmi_radius
        assert rmi_pool in ['max', 'avg', 'interpolation', 'none']
        self.rmi_pool = rmi_pool
        assert rmi_pool_size == rmi_pool_stride
        self.rmi_pool_size = rmi_pool_size
        self.rmi_pool_stride = rmi_pool_stride
        self.half_d = rmi_radius * rmi_radius
        self.d = 2 * self.half_d
        self.kernel_padding = rmi_pool_size // 2
        self.ignore_index = 255
        if rmi_radius > 3:
            raise NotImplementedError(f'RMILoss: rmi_radius={rmi_radius} (kernels cover 1-3, D <= 9)')
        if rmi_pool_stride > 1 and rmi_pool in ('max', 'interpolation'):
            raise NotImplementedError(f'RMILoss: rmi_pool={rmi_pool!r} (kernels cover avg and none)')

    def pool_params(self):
        """(k, s, pad) of losses.py:529-538; (1, 1, 0) when the reference skips the pooling."""
        if self.rmi_pool_stride <= 1 or self.rmi_pool == 'none':
            return 1, 1, 0
        return self.rmi_pool_size, self.rmi_pool_stride, self.kernel_padding

    def forward(self, logits_4D, labels_4D):
        return ops.rmi_loss(logits_4D, labels_4D, self.num_classes, self.rmi_radius, *self.pool_params())


def _out_of_scope(name):
    def f(*a, **k):
        raise NotImplementedError(f'losses.{name} is outside the MI355X hot path (SURVEY §2.1 row 3)')
    return f


for _n in ('DenseCrossEntropyLossWithLogits', 'OhemCrossEntropy', 'FocalLoss', 'DiceWithLogitsLoss',
           'NormalizedFocalLossSigmoid', 'binary_entropy_loss', 'entropy_loss', 'log_dice_loss'):
    globals()[_n] = _out_of_scope(_n)

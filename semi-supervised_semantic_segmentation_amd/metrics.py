"""metrics.dice_metric (reference metrics.py:1-7) — validation only (not the train hot path)."""


def dice_metric(input, target):
    smooth = 1.
    intersection = (input * target).sum(dim=(1, 2, 3))
    cardinality = (input + target).sum(dim=(1, 2, 3))
    return (2. * intersection + smooth) / (cardinality + smooth)

"""reversible_augmentations (reference :5-49) wraps kornia rotate/resize; train.py imports it but never
calls it.  kornia is not available, so the classes keep the API and raise when used."""


class Rotate:
    def __init__(self, max_angle):
        self.max_angle = max_angle

    def apply(self, inputs):
        raise NotImplementedError('kornia-based reversible augmentations are outside the MI355X hot path')

    reverse = apply


class Rescale:
    def __init__(self, min_scale, max_scale):
        self.min_scale, self.max_scale = min_scale, max_scale

    def apply(self, inputs):
        raise NotImplementedError('kornia-based reversible augmentations are outside the MI355X hot path')

    reverse = apply

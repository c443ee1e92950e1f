"""Host-side augmentations with the albumentations call convention used by the reference datasets
(`aug(image=HxWx3 uint8, mask=HxWxC uint8) -> {'image': ..., 'mask': ...}`, reference data/dataset.py:71-74,
unsupervised_dataset.py:20-21).  albumentations / cv2 are absent in this image, so this is a numpy + PIL
restatement of the deterministic part of the reference pipelines (configs/default_config.py:179-252):
LongestMaxSize, PadIfNeeded (constant border), HorizontalFlip and ToFloat, composed by Compose.  Resizing goes
through PIL's bilinear filter (cv2.INTER_LINEAR differs by rounding), so outputs are not bit-identical with
the reference's loader; the photometric / geometric train augmentations (Rotate, RandomResizedCrop, colour,
blur, noise, distortions) are not restated."""
import random

import numpy as np
from PIL import Image


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, **data):
        for t in self.transforms:
            data = t(**data)
        return data


def _resize(a, h, w, resample):
    if a.ndim == 3 and a.shape[2] not in (1, 3, 4):
        return np.stack([_resize(a[..., i], h, w, resample) for i in range(a.shape[2])], axis=2)
    squeeze = a.ndim == 3 and a.shape[2] == 1
    img = Image.fromarray(a[..., 0] if squeeze else a)
    out = np.asarray(img.resize((w, h), resample=resample))
    return out[..., None] if squeeze else out


class LongestMaxSize:
    """Scale so that max(H, W) == max_size (aspect kept; image bilinear, mask nearest like albumentations)."""

    def __init__(self, max_size=1024, always_apply=True, p=1.0):
        self.max_size = max_size

    def __call__(self, image, mask=None, **kw):
        h, w = image.shape[:2]
        s = self.max_size / float(max(h, w))
        nh, nw = int(round(h * s)), int(round(w * s))
        out = dict(kw, image=_resize(image, nh, nw, Image.BILINEAR))
        if mask is not None:
            out['mask'] = _resize(mask, nh, nw, Image.NEAREST)
        return out


class PadIfNeeded:
    """Constant (0) padding to at least min_height x min_width, split top/bottom and left/right as
    albumentations does (the odd pixel goes to the bottom / right)."""

    def __init__(self, min_height=1024, min_width=1024, border_mode=0, value=0, always_apply=True, p=1.0):
        self.min_height, self.min_width, self.value = min_height, min_width, value

    def _pad(self, a, top, bottom, left, right):
        pad = [(top, bottom), (left, right)] + [(0, 0)] * (a.ndim - 2)
        return np.pad(a, pad, mode='constant', constant_values=self.value)

    def __call__(self, image, mask=None, **kw):
        h, w = image.shape[:2]
        dh, dw = max(self.min_height - h, 0), max(self.min_width - w, 0)
        top, left = dh // 2, dw // 2
        out = dict(kw, image=self._pad(image, top, dh - top, left, dw - left))
        if mask is not None:
            out['mask'] = self._pad(mask, top, dh - top, left, dw - left)
        return out


class HorizontalFlip:
    def __init__(self, p=0.5, rng=None):
        # default: the module-level `random` (albumentations' convention), which torch reseeds in every
        # DataLoader worker, so forked workers do not replay one flip sequence
        self.p, self.rng = p, rng or random

    def __call__(self, image, mask=None, **kw):
        flip = self.rng.random() < self.p
        out = dict(kw, image=image[:, ::-1].copy() if flip else image)
        if mask is not None:
            out['mask'] = mask[:, ::-1].copy() if flip else mask
        return out


class ToFloat:
    """image / max_value as float32 (albumentations ToFloat, max_value=255 for uint8); the mask is untouched."""

    def __init__(self, max_value=255.0, always_apply=True, p=1.0):
        self.max_value = max_value

    def __call__(self, image, **kw):
        return dict(kw, image=image.astype(np.float32) / np.float32(self.max_value))

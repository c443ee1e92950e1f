"""Synthetic labeled / unlabeled segmentation datasets for the BASELINE configs: images
U[0,1) and 2-channel one-hot masks of smoothed-noise blobs.  The reference's SkinSegDataset needs
cv2 + albumentations (absent here)."""
import math

import torch
import torch.nn.functional as F


class SyntheticSegDataset(torch.utils.data.Dataset):
    def __init__(self, length=64, size=512, seed=0, with_masks=True, blob_sigma=16.0, fg_fraction=0.4, uint8=False):
        self.length, self.size, self.seed = length, size, seed
        self.with_masks, self.sigma, self.fg = with_masks, blob_sigma, fg_fraction
        # uint8: the image as the reference's host loader leaves it before ToFloat (LongestMaxSize + PadIfNeeded
        # output, data/dataset.py:70-72), for the device augmentation pipeline (data.device_augment)
        self.uint8 = uint8

    def __len__(self):
        return self.length

    def _blobs(self, g):
        k = int(2 * round(3 * self.sigma) + 1)
        x = torch.arange(k, dtype=torch.float32) - k // 2
        w = torch.exp(-x * x / (2 * self.sigma ** 2))
        w = (w / w.sum()).view(1, 1, k, 1)
        n = torch.randn(1, 1, self.size, self.size, generator=g)
        f = F.conv2d(F.conv2d(n, w, padding=(k // 2, 0)), w.transpose(2, 3), padding=(0, k // 2))
        thr = torch.quantile(f.flatten(), 1 - self.fg)
        return (f > thr).float()[0]

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        out = {'image': torch.rand(3, self.size, self.size, generator=g)}
        if self.uint8:
            out['image'] = (out['image'] * 255).round().to(torch.uint8)
        if self.with_masks:
            fg = self._blobs(g)
            out['semantic_mask'] = torch.cat([1 - fg, fg], 0)
        return out

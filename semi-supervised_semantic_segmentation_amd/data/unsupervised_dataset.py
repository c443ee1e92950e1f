"""UnsupervisedImagesDataset — drop-in for reference data/unsupervised_dataset.py:10-31 (every *.jp*g of
the given directories; PIL decoding instead of cv2, see data/dataset.py)."""
import os
from glob import glob

import numpy as np
import torch

from data.dataset import read_rgb


class UnsupervisedImagesDataset(torch.utils.data.Dataset):
    def __init__(self, dataset_dirs, augmentations=None):
        self.filenames = []
        for dataset_dir in dataset_dirs:
            self.filenames.extend(glob(os.path.join(dataset_dir, '*.jp*g')))
        self.augmentations = augmentations

    def __getitem__(self, item):
        image = self.augmentations(image=read_rgb(self.filenames[item]))['image']
        return {'image': torch.from_numpy(np.ascontiguousarray(np.transpose(image, axes=(2, 0, 1))))}

    def __len__(self):
        return len(self.filenames)

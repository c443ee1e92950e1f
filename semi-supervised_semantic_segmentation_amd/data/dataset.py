"""SkinSegDataset — drop-in for reference data/dataset.py:24-90 (same constructor, same sample dict).

Directory layout as in the reference: `<dataset_dir>/part_config.json` (a list of partitions, each a list of
sample names) and `<dataset_dir>/<name>/image.jpg` with one `<anything>_<class>.png` mask per class
(class in {background, skin}).  The soft 2-channel mask is assembled exactly as the reference does
(dataset.py:55-68: clip, background = 1 - max, normalise, quantise to uint8), augmented with the
albumentations call convention (data/transforms.py) and returned as float32 / 255.  Decoding uses PIL
instead of cv2 (absent here); JPEG decoders can differ by a few levels per pixel.
"""
import json
import os
from glob import glob

import numpy as np
import torch
from PIL import Image


def read_rgb(path):
    with Image.open(path) as im:
        return np.asarray(im.convert('RGB'))


def read_gray(path):
    with Image.open(path) as im:
        return np.asarray(im.convert('L'))


def assemble_semantic_mask(mask_files, class2idx, shape):
    """reference data/dataset.py:55-68 -> HxWxC uint8."""
    semantic_mask = np.zeros(shape=(len(class2idx), shape[0], shape[1]), dtype=np.float32)
    for file_path in mask_files:
        mask = read_gray(file_path).astype(np.float32)
        mask /= 255.
        class_name = os.path.splitext(os.path.basename(file_path))[0].split('_')[1]
        semantic_mask[class2idx[class_name]] += mask
    semantic_mask = np.clip(semantic_mask, 0., 1.)
    semantic_mask[0] = np.ones_like(semantic_mask[0]) - np.max(semantic_mask, axis=0, keepdims=False)
    semantic_mask /= np.sum(semantic_mask, axis=0, keepdims=True)
    semantic_mask = (semantic_mask * 255).astype(np.uint8)
    return np.transpose(semantic_mask, axes=(1, 2, 0))


class SkinSegDataset(torch.utils.data.Dataset):
    def __init__(self, dataset_dir, augmentations=None, partition=None):
        self.class2idx = {'background': 0, 'skin': 1}
        if partition is None:
            raise ValueError('Partition should be integer and not None')
        with open(os.path.join(dataset_dir, 'part_config.json')) as part_f:
            partitions = json.load(part_f)
        whitelist = []
        if isinstance(partition, int):
            whitelist.extend(partitions[partition])
        elif isinstance(partition, (list, tuple)):
            for part_idx in partition:
                whitelist.extend(partitions[part_idx])
        filenames = glob(os.path.join(dataset_dir, '*', 'image.jpg'))
        if whitelist:
            keep = set(whitelist)
            filenames = [f for f in filenames if os.path.splitext(os.path.basename(os.path.dirname(f)))[0] in keep]
        self.filenames = filenames
        self.dataset_dir = dataset_dir
        self.augmentations = augmentations

    def __getitem__(self, item):
        image_filename = self.filenames[item]
        image = read_rgb(image_filename)
        mask_files = glob(os.path.join(os.path.dirname(image_filename), '*.png'))
        semantic_mask = assemble_semantic_mask(mask_files, self.class2idx, image.shape[:2])
        augmented = self.augmentations(image=image, mask=semantic_mask)
        image, semantic_mask = augmented['image'], augmented['mask']
        image = torch.from_numpy(np.ascontiguousarray(np.transpose(image, axes=(2, 0, 1))))
        semantic_mask = np.transpose(semantic_mask, axes=(2, 0, 1)).astype(np.float32) / 255
        return {'image': image, 'semantic_mask': torch.from_numpy(np.ascontiguousarray(semantic_mask)),
                'filename': image_filename}

    def __len__(self):
        return len(self.filenames)

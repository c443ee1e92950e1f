"""CPU tests of the input pipeline drop-ins (reference data/dataset.py:24-90, unsupervised_dataset.py:10-31):
partition filtering, soft-mask assembly, augmentation call convention, sample dict layout.  The reference
loaders need cv2 + albumentations (absent), so the expected masks are restated from dataset.py:55-68
here; parity with the reference loader itself is unpinned."""
import json
import os

import numpy as np
import torch
from PIL import Image

from data import transforms as T
from data.dataset import SkinSegDataset
from data.unsupervised_dataset import UnsupervisedImagesDataset


def _write_sample(root, name, h, w, rng, skin=True):
    d = os.path.join(root, name)
    os.makedirs(d)
    Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(os.path.join(d, 'image.jpg'), quality=95)
    m = np.zeros((h, w), np.uint8)
    if skin:
        m[h // 4:h // 2, w // 3:] = 255
        m[0, 0] = 128
    Image.fromarray(m).save(os.path.join(d, '0_skin.png'))
    return m


def test_skinseg_partitions_mask_and_sample_layout(tmp_path):
    rng = np.random.default_rng(0)
    root = str(tmp_path)
    masks = {n: _write_sample(root, n, 30, 41, rng, skin=(n != 'c')) for n in ('a', 'b', 'c')}
    with open(os.path.join(root, 'part_config.json'), 'w') as f:
        json.dump([['a'], ['b', 'c']], f)
    aug = T.Compose([T.ToFloat()])
    ds0 = SkinSegDataset(root, augmentations=aug, partition=0)
    ds1 = SkinSegDataset(root, augmentations=aug, partition=1)
    dsall = SkinSegDataset(root, augmentations=aug, partition=[0, 1])
    assert len(ds0) == 1 and len(ds1) == 2 and len(dsall) == 3
    for ds in (ds0, ds1):
        for i in range(len(ds)):
            s = ds[i]
            name = os.path.basename(os.path.dirname(s['filename']))
            assert s['image'].shape == (3, 30, 41) and s['image'].dtype == torch.float32
            assert 0.0 <= float(s['image'].min()) and float(s['image'].max()) <= 1.0
            assert s['semantic_mask'].shape == (2, 30, 41)
            # dataset.py:55-68 restated: skin = m/255, bg = 1 - skin, normalise, quantise to uint8, /255
            skin = masks[name].astype(np.float32) / 255.
            sm = np.stack([1 - skin, skin])
            sm /= sm.sum(0, keepdims=True)
            exp = (sm * 255).astype(np.uint8).astype(np.float32) / 255
            np.testing.assert_array_equal(s['semantic_mask'].numpy(), exp)


def test_transforms_longest_max_size_pad_flip():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (20, 50, 3), dtype=np.uint8)
    mask = rng.integers(0, 256, (20, 50, 2), dtype=np.uint8)
    out = T.Compose([T.LongestMaxSize(max_size=100), T.PadIfNeeded(min_height=64, min_width=64),
                     T.HorizontalFlip(p=1.0), T.ToFloat()])(image=img, mask=mask)
    assert out['image'].shape == (64, 100, 3) and out['image'].dtype == np.float32
    assert out['mask'].shape == (64, 100, 2) and out['mask'].dtype == np.uint8
    # 40 rows of content padded 12 top / 12 bottom with zeros
    assert not out['image'][:12].any() and not out['image'][52:].any() and out['image'][12:52].any()
    # nearest-resized mask keeps the label set
    assert set(np.unique(out['mask'])) <= set(np.unique(mask))


def test_unsupervised_dataset(tmp_path):
    rng = np.random.default_rng(2)
    for d in ('u1', 'u2'):
        os.makedirs(tmp_path / d)
        for k in range(2):
            Image.fromarray(rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)).save(str(tmp_path / d / f'{k}.jpg'))
    ds = UnsupervisedImagesDataset([str(tmp_path / 'u1'), str(tmp_path / 'u2')],
                                   augmentations=T.Compose([T.PadIfNeeded(32, 32), T.ToFloat()]))
    assert len(ds) == 4
    s = ds[3]
    assert set(s) == {'image'} and s['image'].shape == (3, 32, 32) and s['image'].dtype == torch.float32

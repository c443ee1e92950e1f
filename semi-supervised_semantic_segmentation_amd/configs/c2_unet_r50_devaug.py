"""Config C2 with the reference's train-time augmentation pipelines on the device (default_config.py:179-212 as
data.device_augment.DeviceAugment): the datasets deliver uint8 images as the host-only transforms leave them
(LongestMaxSize + PadIfNeeded, data/dataset.py:70-72; synthetic stand-ins here, 640x640 before the 512 crop) and
train.train augments every labelled and unlabelled batch on the device before the step."""
from functools import partial

from c2_unet_r50 import common, model, train, val  # noqa: F401  (the rest of C2 unchanged; fromfile puts configs/ on the path)
from data.device_augment import DeviceAugment
from data.synthetic import SyntheticSegDataset

common = dict(common, output_dir='runs/c2_unet_r50_devaug')
train = dict(train)
train['dataset'] = partial(SyntheticSegDataset, length=160, size=640, seed=1, uint8=True)
train['unsupervised_dataset'] = partial(SyntheticSegDataset, length=320, size=640, seed=3, with_masks=False, uint8=True)
train['device_augmentations'] = partial(DeviceAugment, train['crop_size'])

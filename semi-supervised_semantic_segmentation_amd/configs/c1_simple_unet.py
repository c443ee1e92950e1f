"""BASELINE config C1: SimpleUNet(num_blocks 7, first 32, max 256) on 64x64 synthetic masks, supervised, bs 2.
The reference runs this on the CPU (plumbing); here it runs on the MI355X kernels (fp32 compute), and the
CPU execution of the same path is the oracle (oracle/train_ref.py)."""
from functools import partial

import torch

import losses
from data.synthetic import SyntheticSegDataset
from models.adapters import ListOutput
from models.simple_unet import UNet

common = dict(world_size=1, use_cpu=False, workers=1, output_dir='runs/c1_simple_unet', num_classes=2, image_size=64,
              compute_dtype='fp32')
model = dict(model_fn=lambda: ListOutput(UNet(2, num_blocks=7, first_channels=32, max_width=256)))
train = dict(print_freq=10, batch_size_per_worker=2, virtual_batch_size_multiplier=1, num_dataloader_workers=0,
             crop_size=64, gradient_clip_value=5.0, use_semi_supervised=False, mask_proportion_range=(0.45, 0.55),
             sigma_range=(8, 32), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=0.97,
             pretrained_checkpoint_path='')
train['base_lr'] = 0.01
train['loss'] = losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'),
                                       'weight': [0.5]}])
train['min_lr'] = train['base_lr'] * 0.001
train['optimizer'] = partial(torch.optim.SGD, lr=train['base_lr'], momentum=0.9, weight_decay=0.0005)
train['lr_scheduler'] = partial(torch.optim.lr_scheduler.CosineAnnealingWarmRestarts, T_0=300, T_mult=2,
                                eta_min=train['base_lr'] * 0.01, last_epoch=-1)
train['dataset'] = partial(SyntheticSegDataset, length=16, size=64, seed=1, blob_sigma=4.0)
train['unsupervised_dataset'] = partial(SyntheticSegDataset, length=16, size=64, seed=3, with_masks=False)
val = dict(batch_size_per_worker=2, num_dataloader_workers=0,
           dataset=partial(SyntheticSegDataset, length=4, size=64, seed=2, blob_sigma=4.0))

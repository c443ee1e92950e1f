"""BASELINE config C5: FC-HarDNet(n_classes=2) 512x512 + Discriminator(5 layers, 64 -> 512 channels), fp16, DDP on
8 GPUs.  The discriminator is built exactly as the reference config names it (default_config.py:116-120); the
reference trainer never calls it, so its adversarial use here is build-defined
(train.adversarial_terms / discriminator_step, after Hung et al. 2018): weight 0.01 on the student's
BCE(D(sigmoid(logits)), 1), a discriminator SGD step per training step.  fp16 compute runs with dynamic loss
scaling (ssseg.amp)."""
from functools import partial

import torch

import losses
from data.synthetic import SyntheticSegDataset
from models.adapters import ListOutput
from models.discriminator import Discriminator
from models.hardnet import HarDNet

common = dict(world_size=8, use_cpu=False, workers=8, output_dir='runs/c5_hardnet_disc', num_classes=2,
              image_size=512, compute_dtype='fp16')
model = dict(model_fn=lambda: ListOutput(HarDNet(n_classes=2)),
             discriminator=partial(Discriminator, num_layers=5, initial_channels=64, max_depth=512, out_channels=1))
train = dict(print_freq=10, batch_size_per_worker=16, virtual_batch_size_multiplier=1, num_dataloader_workers=2,
             crop_size=512, gradient_clip_value=5.0, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
             sigma_range=(8, 32), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=0.97,
             pretrained_checkpoint_path='')
train['base_lr'] = 0.0001 * train['virtual_batch_size_multiplier'] / 4 * 9
train['loss'] = losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'),
                                       'weight': [0.5]}])
train['min_lr'] = train['base_lr'] * 0.001
train['optimizer'] = partial(torch.optim.SGD, lr=train['base_lr'], momentum=0.9, weight_decay=0.0005)
train['adversarial_loss_weight'] = 0.01
train['discriminator_optimizer'] = partial(torch.optim.SGD, lr=train['base_lr'], momentum=0.9)
train['lr_scheduler'] = partial(torch.optim.lr_scheduler.CosineAnnealingWarmRestarts, T_0=300, T_mult=2,
                                eta_min=train['base_lr'] * 0.01, last_epoch=-1)
train['dataset'] = partial(SyntheticSegDataset, length=1280, size=512, seed=1)
train['unsupervised_dataset'] = partial(SyntheticSegDataset, length=2560, size=512, seed=3, with_masks=False)
val = dict(batch_size_per_worker=16, num_dataloader_workers=2,
           dataset=partial(SyntheticSegDataset, length=128, size=512, seed=2))

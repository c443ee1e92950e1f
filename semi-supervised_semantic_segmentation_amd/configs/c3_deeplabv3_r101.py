"""BASELINE config C3: DeepLabV3-ResNet101 (output stride 8) 512x512, Lovász-softmax supervised loss + MSE
consistency (mean teacher + CowMix), bs 16/GPU, DDP over RCCL on 8 GPUs.  The reference runs fp32; this config
uses the bf16 throughput mode (compute_dtype='fp32' gives the parity mode)."""
from functools import partial

import torch

import losses
from data.synthetic import SyntheticSegDataset
from models.adapters import ListOutput
from models.deeplabv3 import deeplabv3_resnet101

common = dict(world_size=8, use_cpu=False, workers=8, output_dir='runs/c3_deeplabv3_r101', num_classes=2,
              image_size=512, compute_dtype='bf16')
model = dict(model_fn=lambda: ListOutput(deeplabv3_resnet101(2)))
train = dict(print_freq=10, batch_size_per_worker=16, virtual_batch_size_multiplier=1, num_dataloader_workers=2,
             crop_size=512, gradient_clip_value=5.0, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
             sigma_range=(8, 32), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=0.97,
             pretrained_checkpoint_path='')
train['base_lr'] = 0.0001 * train['virtual_batch_size_multiplier'] / 4 * 9
train['loss'] = losses.CalculateLoss([{'loss_fn': losses.binary_lovasz_loss_with_logits, 'weight': [1.0]}])
train['min_lr'] = train['base_lr'] * 0.001
train['optimizer'] = partial(torch.optim.SGD, lr=train['base_lr'], momentum=0.9, weight_decay=0.0005)
train['lr_scheduler'] = partial(torch.optim.lr_scheduler.CosineAnnealingWarmRestarts, T_0=300, T_mult=2,
                                eta_min=train['base_lr'] * 0.01, last_epoch=-1)
train['dataset'] = partial(SyntheticSegDataset, length=1280, size=512, seed=1)
train['unsupervised_dataset'] = partial(SyntheticSegDataset, length=2560, size=512, seed=3, with_masks=False)
val = dict(batch_size_per_worker=16, num_dataloader_workers=2,
           dataset=partial(SyntheticSegDataset, length=128, size=512, seed=2))

"""BASELINE config C4: MultiscaleAttention(HRNet-W32 small, 480 feature channels, 2 scales) on 1024x1024, mean
teacher + CowMix, DDP over RCCL on 8 GPUs — the reference's default model (configs/default_config.py:115).
The reference's default loss (RMILoss, fp64 Cholesky) is outside the hot path; BCE is used as in C2."""
from functools import partial

import torch

import losses
from data.synthetic import SyntheticSegDataset
from models.higher_hrnet import POSE_HIGHER_RESOLUTION_NET, get_pose_net
from models.multiscale_attention import MultiscaleAttention

common = dict(world_size=8, use_cpu=False, workers=8, output_dir='runs/c4_msa_hrnet', num_classes=2, image_size=1024,
              compute_dtype='bf16')
model = dict(model_fn=partial(MultiscaleAttention, model_fn=partial(get_pose_net, cfg=POSE_HIGHER_RESOLUTION_NET),
                              num_feature_channels=32 + 64 + 128 + 256, num_scales=2))
train = dict(print_freq=9, batch_size_per_worker=16, virtual_batch_size_multiplier=1, num_dataloader_workers=2,
             crop_size=1024, gradient_clip_value=5.0, use_semi_supervised=True, mask_proportion_range=(0.45, 0.55),
             sigma_range=(8, 32), consistency_loss_weight=10, ema_model_alpha=0.99, confidence_threshold=0.97,
             pretrained_checkpoint_path='')
train['base_lr'] = 0.0001 * train['virtual_batch_size_multiplier'] / 4 * 9
train['loss'] = losses.CalculateLoss([{'loss_fn': losses.DenseBinaryCrossEntropyLossWithLogits(reduction='mean'),
                                       'weight': [0.5]}])
train['min_lr'] = train['base_lr'] * 0.001
train['optimizer'] = partial(torch.optim.SGD, lr=train['base_lr'], momentum=0.9, weight_decay=0.0005)
train['lr_scheduler'] = partial(torch.optim.lr_scheduler.CosineAnnealingWarmRestarts, T_0=300, T_mult=2,
                                eta_min=train['base_lr'] * 0.01, last_epoch=-1)
train['dataset'] = partial(SyntheticSegDataset, length=1280, size=1024, seed=1)
train['unsupervised_dataset'] = partial(SyntheticSegDataset, length=2560, size=1024, seed=3, with_masks=False)
val = dict(batch_size_per_worker=8, num_dataloader_workers=2,
           dataset=partial(SyntheticSegDataset, length=64, size=1024, seed=2))

"""Output adapter: train.py expects `features, pred_maps = model(x)` with `pred_maps` a list of NCHW
logits (reference train.py:47,70,91).  Single-tensor models (UNet, SimpleUNet, HarDNet, DeepLabV3)
are wrapped at the config `model_fn` level; constructors stay untouched."""
import torch.nn as nn


class ListOutput(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.model = model

    @property
    def ssseg_batched_eval(self):
        return getattr(self.model, 'ssseg_batched_eval', False)

    def forward(self, x):
        y = self.model(x)
        return [y], [y]

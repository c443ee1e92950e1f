"""Hierarchical multi-scale attention — drop-in for reference models/multiscale_attention.py:7-65
(same constructor `MultiscaleAttention(model_fn, num_feature_channels, num_scales)`, module tree and
parameter names).

The base model runs at 1/2^(s-1) ... 1/1 of the input (bilinear downsample of the NCHW image,
align_corners=False; the 1/1 "downsample" is PyTorch's identity copy and is skipped).  The attention head
(ConvBNRelu x2 + Conv1x1) runs on the low-resolution features on the conv engine; its logit and the
running output are bilinearly resized to the high-resolution logits, and
`out*sigmoid(a) + hi*(1-sigmoid(a))` is one fused kernel (ssseg_att_blend) forward and backward.
Returns `(features, [out_logits])` like the reference.
"""
from typing import List

import torch.nn as nn

from ssseg import nn as snn
from ssseg import ops

from .higher_hrnet import ConvBN, ConvBNRelu  # noqa: F401  (reference import surface)


class MultiscaleAttention(nn.Module):
    def __init__(self, model_fn, num_feature_channels, num_scales):
        super().__init__()
        self.model = model_fn()
        self.attention_head = nn.Sequential(
            ConvBNRelu(num_feature_channels, num_feature_channels // 2, kernel_size=3, stride=1, padding=1),
            ConvBNRelu(num_feature_channels // 2, num_feature_channels // 4, kernel_size=3, stride=1, padding=1),
            snn.Conv2d(num_feature_channels // 4, 1, kernel_size=1, stride=1, padding=0, head=True))
        self.num_scales = num_scales

    def downsample(self, input, factor):
        if factor == 1:
            return input
        return ops.interpolate_bilinear(input, (input.size(2) // factor, input.size(3) // factor),
                                        align_corners=False)

    def upsample_to(self, input, target_size: List[int]):
        if tuple(input.shape[2:4]) == tuple(target_size):
            return input
        return ops.interpolate_bilinear(input, target_size, align_corners=False)

    def forward(self, input):
        features = []
        low_res_features, low = self.model(self.downsample(input, factor=2 ** (self.num_scales - 1)))
        low_res_features = low_res_features[0]
        out_logits = low[0]
        features.append(low_res_features)
        scale_idx = self.num_scales - 2
        while scale_idx >= 0:
            hi_feats, hi = self.model(self.downsample(input, factor=2 ** scale_idx))
            high_res_features, high_res_logits = hi_feats[0], hi[0]
            h0, h1, conv = self.attention_head
            att = conv(h1(h0(low_res_features)))
            size = (high_res_logits.shape[2], high_res_logits.shape[3])
            att = self.upsample_to(att, size)
            out_logits = self.upsample_to(out_logits, size)
            out_logits = ops.att_blend(out_logits, high_res_logits, att)
            low_res_features = high_res_features
            features.append(low_res_features)
            scale_idx -= 1
        return features, [out_logits]

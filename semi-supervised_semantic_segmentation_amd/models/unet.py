"""UNet decoder over an endpoint encoder — drop-in for reference models/unet.py.

Constructor signatures and submodule names follow the reference (ConvBlock unet.py:4-14, UpBlock
unet.py:16-50, _center_crop unet.py:52-60, UNet unet.py:63-102), so reference state_dicts load.  The
forward runs on the native kernels: ConvTranspose2d(4,2,1)+bias+ReLU in one epilogue, bilinear
x2 (align_corners=True) + 1x1 conv with a fused ReLU, the concat read part by part by conv3_0 (virtual concat,
ssseg_vcat; one copy where the parts do not qualify), Conv+BN+ReLU blocks.
The input may be an NCHW image batch (converted once to NHWC) and the logits come back fp32.
"""
import os

import torch.nn as nn

from ssseg import nn as snn
from ._common import ConvBlock, center_crop as _center_crop  # noqa: F401  (reference names)

# the decoder blocks' outputs marked single-use (their consumer conv carries conv3_1's BN backward); 0: A/B off
_DEC_SINGLE_USE = os.environ.get('SSSEG_UNET_SINGLE_USE', '1') != '0'


class UpBlock(nn.Module):
    def __init__(self, in_channels, skip_in_channels, out_channels, shrink=True, norm_layer=nn.BatchNorm2d,
                 train_upsampling=False):
        super().__init__()
        self.train_upsampling = train_upsampling
        if train_upsampling:
            self.upsampler = nn.Sequential(snn.ConvTranspose2d(in_channels, out_channels, kernel_size=4, stride=2,
                                                               padding=1), nn.ReLU())
        else:
            self.upsampler = nn.Sequential(snn.Upsample(scale_factor=2, mode='bilinear', align_corners=True),
                                           snn.Conv2d(in_channels, out_channels, 1, bias=False), nn.ReLU())
        self.out_channels = out_channels
        self.skip_channels = skip_in_channels
        self.conv3_0 = ConvBlock(out_channels + skip_in_channels, out_channels, 3, norm_layer=norm_layer)
        self.conv3_1 = ConvBlock(out_channels, out_channels // 2 if shrink else out_channels, 3, norm_layer=norm_layer)

    def _upsample(self, x):
        if self.train_upsampling:
            return self.upsampler[0].forward_relu(x)
        return self.upsampler[1].forward_relu(self.upsampler[0](x))

    def forward(self, x, skip, single_use=False):
        """single_use: the caller guarantees the block's output feeds exactly one conv (UNet: the next block's
        upsampler or the 1x1 head), whose input gradient then carries conv3_1's BN backward (snn.conv_bn_act)."""
        x = self._upsample(x)
        # conv3_0 is the concat's only consumer: it reads [x | skip] part by part (virtual concat, no copy)
        x = snn.cat_crop(x, skip, self.out_channels, self.skip_channels, lazy=True)
        return self.conv3_1(self.conv3_0(x, single_use=True), single_use=single_use)


class UNet(nn.Module):
    # eval forward is per-sample and accepts an NHWC activation batch (train.train_step batches the teacher)
    ssseg_batched_eval = True

    def __init__(self, num_classes, encoder, max_width, norm_layer=nn.BatchNorm2d, train_upsampling=False):
        super().__init__()
        self.encoder = encoder
        self.num_classes = num_classes
        depths = list(encoder.endpoint_depths)
        self.decoder = nn.ModuleList()
        ch_in = depths[-1]
        for level in range(len(encoder.endpoints) - 2, -1, -1):
            width = min(min(depths) * 2 ** level, max_width)
            self.decoder.append(UpBlock(ch_in, depths[level], width, shrink=False, norm_layer=norm_layer,
                                        train_upsampling=train_upsampling))
            ch_in = width
        self.final_block = snn.Conv2d(ch_in, num_classes, 1, bias=False, head=True)

    def forward(self, x):
        feats = self.encoder(snn.to_act(x))
        y = feats[-1]
        for i, block in enumerate(self.decoder):
            # (each block's output feeds only the next block's upsampler conv / the head conv)
            y = block(y, feats[len(feats) - 2 - i], single_use=_DEC_SINGLE_USE)
        return self.final_block(y)

    def get_params_with_layerwise_lr(self, encoder_lr, decoder_lr, classifier_lr):
        return [{'params': self.encoder.parameters(), 'lr': encoder_lr},
                {'params': self.decoder.parameters(), 'lr': decoder_lr},
                {'params': self.final_block.parameters(), 'lr': classifier_lr}]

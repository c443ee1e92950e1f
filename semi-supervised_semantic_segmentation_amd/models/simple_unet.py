"""Plain UNet — drop-in for reference models/simple_unet.py (UNet simple_unet.py:5-56, UpBlock :59-95,
DownBlock :98-107, ConvBlock :110-120), same constructor signatures and submodule names, forward on
the native kernels (MaxPool2d(2,2,ceil_mode) -> DownBlocks; ConvT/bilinear upsampler + BN + ReLU)."""
import torch.nn as nn

from ssseg import nn as snn
from ._common import ConvBlock, norm_factory, center_crop as _center_crop  # noqa: F401


class DownBlock(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=3, norm_layer=nn.BatchNorm2d):
        super().__init__()
        self.down_block = nn.Sequential(ConvBlock(in_channels, out_channels, kernel_size, norm_layer),
                                        ConvBlock(out_channels, out_channels, kernel_size, norm_layer))

    def forward(self, x):
        return self.down_block[1](self.down_block[0](x))


class UpBlock(nn.Module):
    def __init__(self, in_channels, out_channels, shrink=True, norm_layer=nn.BatchNorm2d, train_upsampling=False):
        super().__init__()
        norm = norm_factory(norm_layer)
        self.train_upsampling = train_upsampling
        if train_upsampling:
            self.upsampler = nn.Sequential(snn.ConvTranspose2d(in_channels, out_channels, kernel_size=4, stride=2,
                                                               padding=1), norm(out_channels), nn.ReLU())
        else:
            self.upsampler = nn.Sequential(snn.Upsample(scale_factor=2, mode='bilinear', align_corners=True),
                                           snn.Conv2d(in_channels, out_channels, 1, bias=False), norm(out_channels),
                                           nn.ReLU())
        self.out_channels = out_channels
        self.conv3_0 = ConvBlock(2 * out_channels, out_channels, 3, norm_layer=norm_layer)
        self.conv3_1 = ConvBlock(out_channels, out_channels // 2 if shrink else out_channels, 3, norm_layer=norm_layer)

    def forward(self, x, skip):
        if self.train_upsampling:
            conv, bn, _ = self.upsampler
            x = snn.conv_bn_act(conv, x, bn, relu=True)
        else:
            up, conv, bn, _ = self.upsampler
            x = snn.conv_bn_act(conv, up(x), bn, relu=True)
        x = snn.cat_crop(x, skip, self.out_channels, self.out_channels)
        return self.conv3_1(self.conv3_0(x))


class UNet(nn.Module):
    ssseg_batched_eval = True   # per-sample eval forward on an NHWC activation batch (batched teacher)

    def __init__(self, num_classes, num_blocks, first_channels=32, max_width=256, norm_layer=nn.BatchNorm2d,
                 train_upsampling=True):
        super().__init__()
        self.num_blocks = num_blocks
        widths = [min(first_channels * 2 ** i, max_width) for i in range(num_blocks + 1)]
        self.encoder = nn.ModuleList()
        ch = 3
        for i, w in enumerate(widths):
            head = snn.MaxPool2d(2, 2, ceil_mode=True) if i else nn.Identity()
            self.encoder.append(nn.Sequential(head, DownBlock(ch, w, norm_layer=norm_layer)))
            ch = w
        self.decoder = nn.ModuleList()
        for i in range(num_blocks - 1, -1, -1):
            width = first_channels * 2 ** i
            out = min(width, max_width)
            shrink = i > 0 and width <= max_width
            self.decoder.append(UpBlock(ch, out, shrink=shrink, norm_layer=norm_layer,
                                        train_upsampling=train_upsampling))
            ch = out // 2 if shrink else out
        self.final_block = nn.Sequential(DownBlock(ch, ch, kernel_size=3, norm_layer=norm_layer),
                                         snn.Conv2d(ch, num_classes, 1, bias=False, head=True))
        self.feature_channels = num_classes

    def get_feature_channels(self):
        return self.feature_channels

    def forward(self, x):
        x = snn.to_act(x)
        skips = []
        for stage in self.encoder:
            x = stage[1](stage[0](x))
            skips.append(x)
        for i, block in enumerate(self.decoder):
            x = block(x, skips[len(skips) - 2 - i])
        return self.final_block[1](self.final_block[0](x))

"""ResNet-50 encoder with the endpoint protocol of the reference's encoders (`endpoints` ModuleList +
`endpoint_depths`, reference models/encoders/mobilenetv2.py:113-131,180-184), which the reference's
UNet (models/unet.py:63-95) consumes.  NEW relative to the reference ("UNet-ResNet50"
does not exist there): torchvision v1.5 Bottleneck layout (stride on the 3x3), random init.

Endpoints: 0 stem conv7x7/s2+BN+ReLU (/2, 64) · 1 maxpool3x3/s2 + layer1 (/4, 256) · 2 layer2 (/8, 512)
· 3 layer3 (/16, 1024) · 4 layer4 (/32, 2048).  Bottleneck: bn3 + residual add + ReLU in one pass.
"""
import torch.nn as nn

from ssseg import nn as snn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, width, stride=1, downsample=None):
        super().__init__()
        self.conv1 = snn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = snn.BatchNorm2d(width)
        self.conv2 = snn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = snn.BatchNorm2d(width)
        self.conv3 = snn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = snn.BatchNorm2d(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is not None:
            # x feeds conv1 and the projection shortcut: their input gradients meet in one dgrad epilogue
            snn.mark_join(x)
            conv, bn = self.downsample
            shortcut = snn.conv_bn_act(conv, x, bn, relu=False)
        else:
            shortcut = x
        # identity shortcut: its gradient is added in conv1's dgrad epilogue (snn.GradHandoff)
        h = snn.GradHandoff() if self.downsample is None else None
        y = snn.conv_bn_act(self.conv1, x, self.bn1, grad_in=h, single_use=True)
        y = snn.conv_bn_act(self.conv2, y, self.bn2, single_use=True)
        return snn.conv_bn_act(self.conv3, y, self.bn3, relu=True, residual=shortcut, grad_out=h)


class Stem(nn.Sequential):
    def __init__(self):
        super().__init__(snn.Conv2d(3, 64, 7, 2, 3, bias=False), snn.BatchNorm2d(64), nn.ReLU(inplace=True))

    def forward(self, x):
        return snn.conv_bn_act(self[0], x, self[1], relu=True)


class Stage(nn.Sequential):
    def forward(self, x):
        for m in self:
            x = m(x)
        return x


class ResNetEncoder(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3)):
        super().__init__()
        self.endpoint_depths = [64, 256, 512, 1024, 2048]
        stages = [Stem()]
        inplanes = 64
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            stride = 1 if i == 0 else 2
            down = nn.Sequential(snn.Conv2d(inplanes, width * 4, 1, stride, bias=False), snn.BatchNorm2d(width * 4))
            blocks = [Bottleneck(inplanes, width, stride, down)]
            inplanes = width * 4
            blocks += [Bottleneck(inplanes, width) for _ in range(n - 1)]
            if i == 0:
                blocks = [snn.MaxPool2d(3, 2, 1)] + blocks
            stages.append(Stage(*blocks))
        self.endpoints = nn.ModuleList(stages)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')

    def forward(self, x):
        outs = []
        for i, ep in enumerate(self.endpoints):
            x = ep(x)
            if i + 1 < len(self.endpoints):
                # an endpoint feeds the next stage and (in the UNet) the decoder concat: one joined gradient
                snn.mark_join(x)
            outs.append(x)
        return outs


def resnet50_encoder():
    return ResNetEncoder((3, 4, 6, 3))

"""DeepLabV3 / FCN over dilated ResNets — drop-in for reference models/deeplabv3.py:8-108
(`deeplabv3_resnet101(num_classes)`, `deeplabv3_resnet50(num_classes)`, `fcn_resnet50(num_classes)`).

The reference builds these from torchvision (v0.5.0 hub tag, deeplabv3.py:9) and swaps the last classifier
conv for `num_classes` outputs, deletes the aux head and overrides forward with a bilinear
(align_corners=False) resize of the logits to the input size (deeplabv3.py:28-36).  torchvision is not
available here and the hub weights need a download, so the architecture is restated from torchvision's
published layout with the same module tree and parameter names (a torchvision state_dict loads):
  backbone  ResNet (v1.5 Bottleneck, stride on the 3x3) with replace_stride_with_dilation=[F, T, T]
            (output stride 8: layer3 dilation 2, layer4 dilation 4; the first block of a dilated layer
            keeps the previous dilation), avgpool/fc dropped;
  classifier DeepLabHead = ASPP(2048, rates 12/24/36: 1x1, three dilated 3x3, image pooling; 1x1
            projection + BN + ReLU + Dropout(0.5)) -> Conv3x3(256) + BN + ReLU -> Conv1x1(num_classes);
            FCNHead = Conv3x3(512) + BN + ReLU + Dropout(0.1) -> Conv1x1(num_classes).
Weights are random (kaiming fan_out for the backbone like torchvision); `pretrained` weights need the
network and are refused.  Parity against the reference is therefore unpinned; the oracle
(oracle/models_ref.py) restates the same layout in plain torch and the GPU tests compare against it.

Forward on the ssseg kernels: dilated convs are the implicit-GEMM engine's dilation; every Conv+BN(+ReLU)
is one conv_bn_act; the image-pooling branch is a global-average-pool kernel, a 1x1 conv and a bilinear
broadcast back to the feature size; the five ASPP branches are concatenated by cat_n.
"""
import torch.nn as nn

from ssseg import nn as snn
from ssseg import ops


class Bottleneck(nn.Module):
    """torchvision Bottleneck (v1.5): 1x1 -> 3x3(stride, dilation) -> 1x1 (x4), residual add + ReLU."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = snn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = snn.BatchNorm2d(planes)
        self.conv2 = snn.Conv2d(planes, planes, 3, stride, padding=dilation, dilation=dilation, bias=False)
        self.bn2 = snn.BatchNorm2d(planes)
        self.conv3 = snn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = snn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if self.downsample is not None:
            conv, bn = self.downsample
            identity = snn.conv_bn_act(conv, x, bn, relu=False)
        else:
            identity = x
        out = snn.conv_bn_act(self.conv1, x, self.bn1, single_use=True)
        out = snn.conv_bn_act(self.conv2, out, self.bn2, single_use=True)
        return snn.conv_bn_act(self.conv3, out, self.bn3, relu=True, residual=identity)


class Layer(nn.Sequential):
    def forward(self, x):
        for m in self:
            x = m(x)
        return x


class ResNetBackbone(nn.Module):
    """torchvision ResNet trunk as IntermediateLayerGetter keeps it (conv1 .. layer4; avgpool/fc dropped)."""

    def __init__(self, layers, replace_stride_with_dilation=(False, True, True)):
        super().__init__()
        self.inplanes, self.dilation = 64, 1
        self.conv1 = snn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = snn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = snn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2, dilate=replace_stride_with_dilation[0])
        self.layer3 = self._make_layer(256, layers[2], stride=2, dilate=replace_stride_with_dilation[1])
        self.layer4 = self._make_layer(512, layers[3], stride=2, dilate=replace_stride_with_dilation[2])
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1, dilate=False):
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(snn.Conv2d(self.inplanes, planes * 4, 1, stride, bias=False),
                                       snn.BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample, previous_dilation)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes, dilation=self.dilation))
        return Layer(*layers)

    def forward(self, x):
        x = snn.conv_bn_act(self.conv1, snn.to_act(x), self.bn1, relu=True)
        x = self.maxpool(x)
        x = self.layer3(self.layer2(self.layer1(x)))
        return {'out': self.layer4(x)}


class ConvBNReLU(nn.Sequential):
    def forward(self, x):
        return snn.conv_bn_act(self[0], x, self[1], relu=True)


class ASPPConv(ConvBNReLU):
    def __init__(self, in_channels, out_channels, dilation):
        super().__init__(snn.Conv2d(in_channels, out_channels, 3, padding=dilation, dilation=dilation, bias=False),
                         snn.BatchNorm2d(out_channels), nn.ReLU())


class ASPPPooling(nn.Sequential):
    def __init__(self, in_channels, out_channels):
        super().__init__(snn.AdaptiveAvgPool2d(1), snn.Conv2d(in_channels, out_channels, 1, bias=False),
                         snn.BatchNorm2d(out_channels), nn.ReLU())

    def forward(self, x):
        size = (x.shape[2], x.shape[3])
        y = snn.conv_bn_act(self[1], snn.global_avgpool(x), self[2], relu=True)
        return snn.resize_act(y, size, align_corners=False)


class Project(nn.Sequential):
    def forward(self, x):
        return self[3](snn.conv_bn_act(self[0], x, self[1], relu=True))


class ASPP(nn.Module):
    def __init__(self, in_channels, atrous_rates, out_channels=256):
        super().__init__()
        modules = [ConvBNReLU(snn.Conv2d(in_channels, out_channels, 1, bias=False), snn.BatchNorm2d(out_channels),
                              nn.ReLU())]
        for rate in atrous_rates:
            modules.append(ASPPConv(in_channels, out_channels, rate))
        modules.append(ASPPPooling(in_channels, out_channels))
        self.convs = nn.ModuleList(modules)
        self.out_channels = out_channels
        self.project = Project(snn.Conv2d(len(self.convs) * out_channels, out_channels, 1, bias=False),
                               snn.BatchNorm2d(out_channels), nn.ReLU(), snn.Dropout(0.5))

    def forward(self, x):
        res = [conv(x) for conv in self.convs]
        return self.project(snn.cat_n(res, [self.out_channels] * len(res)))


class DeepLabHead(nn.Sequential):
    def __init__(self, in_channels, num_classes):
        super().__init__(ASPP(in_channels, [12, 24, 36]), snn.Conv2d(256, 256, 3, padding=1, bias=False),
                         snn.BatchNorm2d(256), nn.ReLU(), snn.Conv2d(256, num_classes, 1, head=True))

    def forward(self, x):
        return self[4](snn.conv_bn_act(self[1], self[0](x), self[2], relu=True))


class FCNHead(nn.Sequential):
    def __init__(self, in_channels, channels):
        inter = in_channels // 4
        super().__init__(snn.Conv2d(in_channels, inter, 3, padding=1, bias=False), snn.BatchNorm2d(inter), nn.ReLU(),
                         snn.Dropout(0.1), snn.Conv2d(inter, channels, 1, head=True))

    def forward(self, x):
        return self[4](self[3](snn.conv_bn_act(self[0], x, self[1], relu=True)))


class SegmentationModel(nn.Module):
    """torchvision _SimpleSegmentationModel with the reference's custom_forward (deeplabv3.py:28-36)."""

    def __init__(self, backbone, classifier):
        super().__init__()
        self.backbone = backbone
        self.classifier = classifier

    def forward(self, x):
        input_shape = x.shape[-2:]
        features = self.backbone(x)
        y = self.classifier(features['out'])
        return ops.interpolate_bilinear(y, input_shape, align_corners=False)


def _get_params_with_layerwise_lr(model, base_lr):
    """deeplabv3.py:15-24: frozen backbone (lr 0), decoder and last layer at base_lr."""
    last = list(model.classifier[-1].parameters())
    last_ids = {id(p) for p in last}
    decoder = [p for p in model.classifier.parameters() if id(p) not in last_ids]
    return [{'params': model.backbone.parameters(), 'lr': 0}, {'params': decoder, 'lr': base_lr},
            {'params': last, 'lr': base_lr}]


def _finish(model):
    model.get_params_with_layerwise_lr = _get_params_with_layerwise_lr   # unbound, as deeplabv3.py:26
    return model


def deeplabv3_resnet101(num_classes, pretrained=False):
    if pretrained:
        raise RuntimeError('deeplabv3_resnet101: pretrained torchvision weights need a download; load a local '
                           'state_dict instead (the parameter names are torchvision\'s)')
    return _finish(SegmentationModel(ResNetBackbone([3, 4, 23, 3]), DeepLabHead(2048, num_classes)))


def deeplabv3_resnet50(num_classes):
    return _finish(SegmentationModel(ResNetBackbone([3, 4, 6, 3]), DeepLabHead(2048, num_classes)))


def fcn_resnet50(num_classes):
    return _finish(SegmentationModel(ResNetBackbone([3, 4, 6, 3]), FCNHead(2048, num_classes)))

"""MobileNetV2 encoder — drop-in for reference models/encoders/mobilenetv2.py (same constructor, same
module tree and parameter names, same `endpoints` / `endpoint_depths` protocol used by models.unet.UNet).

Compute runs on the ssseg engine: ConvBNReLU = conv -> BN -> ReLU6 as one `conv_bn_act` (folded into
the conv epilogue for eval BN), the 3x3 depthwise convs on ssseg_dwconv_*, the InvertedResidual skip
add fused into the projection BN (`residual=`).  `pretrained=True` needs a download (mobilenetv2.py:9,
175-178) and is refused offline.
"""
from torch import nn

from ssseg import nn as snn

__all__ = ['MobileNetV2', 'mobilenet_v2']


def _make_divisible(v, divisor, min_value=None):
    """mobilenetv2.py:12-28 (TF slim rule): round to a multiple of divisor, never below 90 % of v."""
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNReLU(nn.Sequential):
    """mobilenetv2.py:31-39: Conv(groups) -> BN -> ReLU6."""

    def __init__(self, in_planes, out_planes, kernel_size=3, stride=1, groups=1):
        padding = (kernel_size - 1) // 2
        super().__init__(
            snn.Conv2d(in_planes, out_planes, kernel_size, stride, padding, groups=groups, bias=False),
            snn.BatchNorm2d(out_planes),
            nn.ReLU6(inplace=True))

    def forward(self, x):
        return snn.conv_bn_act(self[0], x, self[1], relu=snn.ACT_RELU6)


class InvertedResidual(nn.Module):
    """mobilenetv2.py:42-68: [1x1 expand] -> 3x3 depthwise -> 1x1 project + BN (+ identity)."""

    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        self.stride = stride
        assert stride in [1, 2]
        hidden_dim = int(round(inp * expand_ratio))
        self.use_res_connect = self.stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNReLU(inp, hidden_dim, kernel_size=1))
        layers.extend([
            ConvBNReLU(hidden_dim, hidden_dim, stride=stride, groups=hidden_dim),
            snn.Conv2d(hidden_dim, oup, 1, 1, 0, bias=False),
            snn.BatchNorm2d(oup),
        ])
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        *pre, proj, bn = self.conv
        y = x
        for m in pre:
            y = m(y)
        return snn.conv_bn_act(proj, y, bn, relu=False, residual=x if self.use_res_connect else None)


class MobileNetV2(nn.Module):
    """mobilenetv2.py:72-162 without the classifier (the encoder deletes it, :185-188)."""

    def __init__(self, num_classes=1000, width_mult=1.0, inverted_residual_setting=None, round_nearest=8):
        super().__init__()
        block = InvertedResidual
        input_channel = 32
        last_channel = 1280
        self.width_mult = width_mult
        self.round_nearest = round_nearest
        if inverted_residual_setting is None:
            inverted_residual_setting = [
                [1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
                [6, 320, 1, 1]]
        self.inverted_residual_setting = inverted_residual_setting
        if len(inverted_residual_setting) == 0 or len(inverted_residual_setting[0]) != 4:
            raise ValueError('inverted_residual_setting should be non-empty or a 4-element list, got '
                             f'{inverted_residual_setting}')
        input_channel = _make_divisible(input_channel * width_mult, round_nearest)
        self.input_channel = input_channel
        self.last_channel = _make_divisible(last_channel * max(1.0, width_mult), round_nearest)
        features = [ConvBNReLU(3, input_channel, stride=2)]
        layer_idx = 0
        self.endpoint_indicies = [0]
        self.endpoint_depths = []
        for t, c, n, s in inverted_residual_setting:
            output_channel = _make_divisible(c * width_mult, round_nearest)
            for i in range(n):
                layer_idx += 1
                stride = s if i == 0 else 1
                if stride != 1:
                    self.endpoint_indicies.append(layer_idx)
                    self.endpoint_depths.append(input_channel)
                features.append(block(input_channel, output_channel, stride, expand_ratio=t))
                input_channel = output_channel
        self.endpoint_indicies.append(layer_idx + 1)
        self.endpoint_depths.append(input_channel)
        features.append(ConvBNReLU(input_channel, self.last_channel, kernel_size=1))
        self.features = nn.Sequential(*features)
        for m in self.modules():                                   # mobilenetv2.py:145-155
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out')
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        output_tensors = []
        for module in self.endpoints:
            x = module(x)
            output_tensors.append(x)
        return output_tensors


def mobilenet_v2(pretrained=False, progress=True, **kwargs):
    """mobilenetv2.py:165-188: the encoder exposes `endpoints` (feature slices) and drops the classifier."""
    if pretrained:
        raise RuntimeError('mobilenet_v2(pretrained=True) downloads ImageNet weights; no network here — '
                           'load a local state_dict instead')
    model = MobileNetV2(**kwargs)
    model.endpoints = nn.ModuleList()
    for i in range(len(model.endpoint_indicies) - 1):
        b, e = model.endpoint_indicies[i], model.endpoint_indicies[i + 1]
        model.endpoints.append(nn.Sequential(*model.features[b:e]))
    del model.features
    return model

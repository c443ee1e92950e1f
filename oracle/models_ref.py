"""Oracle: the segmentation networks as plain torch.nn (CPU, fp32).  TEST INFRASTRUCTURE ONLY.

Parameter names match the reference module trees so that state_dicts move freely between the
reference, this oracle and the HIP product:

  SimpleUNet     <- reference/models/simple_unet.py:5-131   (pinned by G6 model_simple_unet_*)
  UNet           <- reference/models/unet.py:4-95           (pinned by G6 model_unet_mbv2_*)
  mobilenet_v2   <- reference/models/encoders/mobilenetv2.py:22-188 (endpoint protocol :113-131,180-184)
  resnet50_encoder  NEW (the reference has no ResNet-50 encoder): torchvision v1.5
                 Bottleneck layout (stride on the 3x3) exposing the same `endpoints` /
                 `endpoint_depths` protocol.  Parity unpinned against the reference; its decoder
                 semantics are pinned through the MobileNetV2 UNet fixture.
  ListOutput     the `(features, [logits])` adapter train.py:47,70,91 needs
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _conv_bn_relu(cin, cout, k, norm=nn.BatchNorm2d):
    return nn.Sequential(nn.Conv2d(cin, cout, k, padding=k // 2, bias=False),
                         norm(cout) if norm is not None else nn.Identity(), nn.ReLU())


class ConvBlock(nn.Module):                                  # unet.py:4-14, simple_unet.py:110-120
    def __init__(self, cin, cout, k, norm_layer=nn.BatchNorm2d):
        super().__init__()
        self.conv_block = _conv_bn_relu(cin, cout, k, norm_layer)

    def forward(self, x):
        return self.conv_block(x)


def center_crop(t, hw):                                      # unet.py:52-60
    dh, dw = (t.shape[2] - hw[0]) // 2, (t.shape[3] - hw[1]) // 2
    return t[:, :, dh:dh + hw[0], dw:dw + hw[1]]


def _match(x, skip):                                         # unet.py:40-43 (compares dim 2 only)
    if skip.shape[2] > x.shape[2]:
        skip = center_crop(skip, x.shape[2:])
    elif skip.shape[2] < x.shape[2]:
        x = center_crop(x, skip.shape[2:])
    return torch.cat((x, skip), 1)


# ---------------------------------------------------------------------------------------------
# SimpleUNet (simple_unet.py)
# ---------------------------------------------------------------------------------------------
class SimpleDownBlock(nn.Module):                            # simple_unet.py:98-107
    def __init__(self, cin, cout, kernel_size=3, norm_layer=nn.BatchNorm2d):
        super().__init__()
        self.down_block = nn.Sequential(ConvBlock(cin, cout, kernel_size, norm_layer),
                                        ConvBlock(cout, cout, kernel_size, norm_layer))

    def forward(self, x):
        return self.down_block(x)


class SimpleUpBlock(nn.Module):                              # simple_unet.py:59-95
    def __init__(self, cin, cout, shrink=True, norm_layer=nn.BatchNorm2d, train_upsampling=False):
        super().__init__()
        if train_upsampling:
            self.upsampler = nn.Sequential(nn.ConvTranspose2d(cin, cout, 4, 2, 1), norm_layer(cout), nn.ReLU())
        else:
            self.upsampler = nn.Sequential(nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True),
                                           nn.Conv2d(cin, cout, 1, bias=False), norm_layer(cout), nn.ReLU())
        self.conv3_0 = ConvBlock(2 * cout, cout, 3, norm_layer)
        self.conv3_1 = ConvBlock(cout, cout // 2 if shrink else cout, 3, norm_layer)

    def forward(self, x, skip):
        return self.conv3_1(self.conv3_0(_match(self.upsampler(x), skip)))


class SimpleUNet(nn.Module):                                 # simple_unet.py:5-56
    def __init__(self, num_classes, num_blocks, first_channels=32, max_width=256,
                 norm_layer=nn.BatchNorm2d, train_upsampling=True):
        super().__init__()
        self.num_blocks = num_blocks
        widths = [min(first_channels * 2 ** i, max_width) for i in range(num_blocks + 1)]
        self.encoder = nn.ModuleList()
        prev = 3
        for i, w in enumerate(widths):
            pool = nn.MaxPool2d(2, 2, ceil_mode=True) if i > 0 else nn.Identity()
            self.encoder.append(nn.Sequential(pool, SimpleDownBlock(prev, w, norm_layer=norm_layer)))
            prev = w
        self.decoder = nn.ModuleList()
        for i in reversed(range(num_blocks)):
            bw = first_channels * 2 ** i
            ch = min(bw, max_width)
            shrink = i > 0 and bw <= max_width
            self.decoder.append(SimpleUpBlock(prev, ch, shrink, norm_layer, train_upsampling))
            prev = ch // 2 if shrink else ch
        self.final_block = nn.Sequential(SimpleDownBlock(prev, prev, 3, norm_layer),
                                         nn.Conv2d(prev, num_classes, 1, bias=False))
        self.feature_channels = num_classes

    def forward(self, x):
        skips = []
        for blk in self.encoder:
            x = blk(x)
            skips.append(x)
        for i, blk in enumerate(self.decoder):
            x = blk(x, skips[-i - 2])
        return self.final_block(x)


# ---------------------------------------------------------------------------------------------
# UNet over an endpoint encoder (unet.py)
# ---------------------------------------------------------------------------------------------
class UpBlock(nn.Module):                                    # unet.py:16-50
    def __init__(self, cin, skip_ch, cout, shrink=True, norm_layer=nn.BatchNorm2d, train_upsampling=False):
        super().__init__()
        if train_upsampling:
            self.upsampler = nn.Sequential(nn.ConvTranspose2d(cin, cout, 4, 2, 1), nn.ReLU())
        else:
            self.upsampler = nn.Sequential(nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True),
                                           nn.Conv2d(cin, cout, 1, bias=False), nn.ReLU())
        self.conv3_0 = ConvBlock(cout + skip_ch, cout, 3, norm_layer)
        self.conv3_1 = ConvBlock(cout, cout // 2 if shrink else cout, 3, norm_layer)

    def forward(self, x, skip):
        return self.conv3_1(self.conv3_0(_match(self.upsampler(x), skip)))


class UNet(nn.Module):                                       # unet.py:63-95
    def __init__(self, num_classes, encoder, max_width, norm_layer=nn.BatchNorm2d, train_upsampling=False):
        super().__init__()
        self.encoder = encoder
        self.num_classes = num_classes
        depths = list(encoder.endpoint_depths)
        self.decoder = nn.ModuleList()
        prev = depths[-1]
        for i in reversed(range(len(encoder.endpoints) - 1)):
            ch = min(min(depths) * 2 ** i, max_width)
            self.decoder.append(UpBlock(prev, depths[i], ch, False, norm_layer, train_upsampling))
            prev = ch
        self.final_block = nn.Conv2d(prev, num_classes, 1, bias=False)

    def forward(self, x):
        feats = []
        for ep in self.encoder.endpoints:
            x = ep(x)
            feats.append(x)
        x = feats[-1]
        for i, blk in enumerate(self.decoder):
            x = blk(x, feats[-i - 2])
        return self.final_block(x)


# ---------------------------------------------------------------------------------------------
# MobileNetV2 encoder (mobilenetv2.py)
# ---------------------------------------------------------------------------------------------
def _make_divisible(v, divisor, min_value=None):             # mobilenetv2.py:12-28
    min_value = divisor if min_value is None else min_value
    nv = max(min_value, int(v + divisor / 2) // divisor * divisor)
    return nv + divisor if nv < 0.9 * v else nv


class ConvBNReLU(nn.Sequential):                             # mobilenetv2.py:31-39
    def __init__(self, cin, cout, kernel_size=3, stride=1, groups=1):
        super().__init__(nn.Conv2d(cin, cout, kernel_size, stride, (kernel_size - 1) // 2, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU6(inplace=True))


class InvertedResidual(nn.Module):                           # mobilenetv2.py:42-68
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = [ConvBNReLU(inp, hidden, kernel_size=1)] if expand_ratio != 1 else []
        layers += [ConvBNReLU(hidden, hidden, stride=stride, groups=hidden),
                   nn.Conv2d(hidden, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        y = self.conv(x)
        return x + y if self.use_res_connect else y


class MobileNetV2Encoder(nn.Module):                         # mobilenetv2.py:72-162, 165-188
    SETTING = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
               [6, 320, 1, 1]]

    def __init__(self, width_mult=1.0, round_nearest=8):
        super().__init__()
        cin = _make_divisible(32 * width_mult, round_nearest)
        last = _make_divisible(1280 * max(1.0, width_mult), round_nearest)
        feats = [ConvBNReLU(3, cin, stride=2)]
        starts, depths = [0], []
        for t, c, n, s in self.SETTING:
            cout = _make_divisible(c * width_mult, round_nearest)
            for i in range(n):
                stride = s if i == 0 else 1
                if stride != 1:
                    starts.append(len(feats))
                    depths.append(cin)
                feats.append(InvertedResidual(cin, cout, stride, t))
                cin = cout
        starts.append(len(feats))
        depths.append(cin)
        feats.append(ConvBNReLU(cin, last, kernel_size=1))   # dropped with `features` (mobilenetv2.py:187)
        self.endpoint_depths = depths
        self.endpoints = nn.ModuleList(nn.Sequential(*feats[a:b]) for a, b in zip(starts[:-1], starts[1:]))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out')
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        outs = []
        for ep in self.endpoints:
            x = ep(x)
            outs.append(x)
        return outs


def mobilenet_v2(pretrained=False, progress=True, **kwargs):
    if pretrained:
        raise RuntimeError('pretrained weights need a network download; not available')
    return MobileNetV2Encoder(**kwargs)


# ---------------------------------------------------------------------------------------------
# ResNet-50 encoder (NEW; parity unpinned against the reference)
# ---------------------------------------------------------------------------------------------
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idn = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        return self.relu(self.bn3(self.conv3(y)) + idn)


class ResNet50Encoder(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3)):
        super().__init__()
        self.endpoint_depths = [64, 256, 512, 1024, 2048]
        stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True))
        stages = []
        cin = 64
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            stride = 1 if i == 0 else 2
            down = nn.Sequential(nn.Conv2d(cin, width * 4, 1, stride, bias=False), nn.BatchNorm2d(width * 4))
            blocks = [Bottleneck(cin, width, stride, down)]
            cin = width * 4
            blocks += [Bottleneck(cin, width) for _ in range(n - 1)]
            stages.append(nn.Sequential(*blocks))
        stages[0] = nn.Sequential(nn.MaxPool2d(3, 2, 1), *stages[0])
        self.endpoints = nn.ModuleList([stem] + stages)

    def forward(self, x):
        outs = []
        for ep in self.endpoints:
            x = ep(x)
            outs.append(x)
        return outs


def resnet50_encoder():
    return ResNet50Encoder()


class Discriminator(nn.Module):                                 # discriminator.py:6-28
    def __init__(self, num_layers, in_channels=2, initial_channels=64, max_depth=512, out_channels=1):
        super().__init__()
        layers = []
        cin, cout = in_channels, initial_channels
        for _ in range(num_layers):
            layers.append(nn.Sequential(nn.Conv2d(cin, cout, 4, 2, 1), nn.LeakyReLU(0.2)))
            cin, cout = cout, min(cout * 2, max_depth)
        layers.append(nn.Sequential(nn.Conv2d(cin, out_channels, 1, bias=False)))
        self.net = nn.Sequential(*layers)

    def forward(self, x):
        return self.net(x)


class ListOutput(nn.Module):
    """(features, [logits]) adapter."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, x):
        y = self.model(x)
        return [y], [y]


def load_state(module, arrays, prefix):
    """Load a fixture's '<prefix>name' arrays into module (strict)."""
    sd = {k[len(prefix):]: torch.from_numpy(arrays[k].copy()) for k in arrays.files if k.startswith(prefix)}
    module.load_state_dict(sd, strict=True)
    return module


# ---------------------------------------------------------------------------------------------
# DeepLabV3 / FCN over dilated ResNets (deeplabv3.py:8-108 -> torchvision v0.5.0 layout, restated;
# torchvision is absent here: parity against the reference unpinned)
# ---------------------------------------------------------------------------------------------
class TVBottleneck(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, padding=dilation, dilation=dilation, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idn = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        return self.relu(self.bn3(self.conv3(y)) + idn)


class DilatedResNet(nn.Module):
    def __init__(self, layers, dilate=(False, True, True)):
        super().__init__()
        self.inplanes, self.dilation = 64, 1
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._layer(64, layers[0])
        self.layer2 = self._layer(128, layers[1], 2, dilate[0])
        self.layer3 = self._layer(256, layers[2], 2, dilate[1])
        self.layer4 = self._layer(512, layers[3], 2, dilate[2])

    def _layer(self, planes, blocks, stride=1, dilate=False):
        prev = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride, bias=False), nn.BatchNorm2d(planes * 4))
        layers = [TVBottleneck(self.inplanes, planes, stride, down, prev)]
        self.inplanes = planes * 4
        layers += [TVBottleneck(self.inplanes, planes, dilation=self.dilation) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        return {'out': self.layer4(self.layer3(self.layer2(self.layer1(x))))}


class ASPPPooling(nn.Sequential):
    def __init__(self, cin, cout):
        super().__init__(nn.AdaptiveAvgPool2d(1), nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU())

    def forward(self, x):
        size = x.shape[-2:]
        for m in self:
            x = m(x)
        return F.interpolate(x, size=size, mode='bilinear', align_corners=False)


class ASPP(nn.Module):
    def __init__(self, cin, rates, cout=256):
        super().__init__()
        mods = [nn.Sequential(nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU())]
        for r in rates:
            mods.append(nn.Sequential(nn.Conv2d(cin, cout, 3, padding=r, dilation=r, bias=False), nn.BatchNorm2d(cout),
                                      nn.ReLU()))
        mods.append(ASPPPooling(cin, cout))
        self.convs = nn.ModuleList(mods)
        self.project = nn.Sequential(nn.Conv2d(len(mods) * cout, cout, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(),
                                     nn.Dropout(0.5))

    def forward(self, x):
        return self.project(torch.cat([c(x) for c in self.convs], 1))


def deeplab_head(cin, num_classes):
    return nn.Sequential(ASPP(cin, [12, 24, 36]), nn.Conv2d(256, 256, 3, padding=1, bias=False), nn.BatchNorm2d(256),
                         nn.ReLU(), nn.Conv2d(256, num_classes, 1))


def fcn_head(cin, num_classes):
    return nn.Sequential(nn.Conv2d(cin, cin // 4, 3, padding=1, bias=False), nn.BatchNorm2d(cin // 4), nn.ReLU(),
                         nn.Dropout(0.1), nn.Conv2d(cin // 4, num_classes, 1))


class SegModel(nn.Module):
    def __init__(self, backbone, classifier):
        super().__init__()
        self.backbone = backbone
        self.classifier = classifier

    def forward(self, x):                                    # deeplabv3.py:28-36
        y = self.classifier(self.backbone(x)['out'])
        return F.interpolate(y, size=x.shape[-2:], mode='bilinear', align_corners=False)


def deeplabv3_resnet101(num_classes):
    return SegModel(DilatedResNet([3, 4, 23, 3]), deeplab_head(2048, num_classes))


def deeplabv3_resnet50(num_classes):
    return SegModel(DilatedResNet([3, 4, 6, 3]), deeplab_head(2048, num_classes))


def fcn_resnet50(num_classes):
    return SegModel(DilatedResNet([3, 4, 6, 3]), fcn_head(2048, num_classes))

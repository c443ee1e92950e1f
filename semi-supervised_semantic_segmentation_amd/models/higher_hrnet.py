"""HRNet-W32 "small" segmentation net — drop-in for the live part of reference models/higher_hrnet.py
(config :75-121, BasicBlock :154-187, BottleneckBlock :190-236, ConvBNRelu :239-253, ConvBN :256-268,
HighResolutionModule :286-333, Stage :342-366, TransitionFuse :369-486, HighResolutionMultiscaleAggregator
:1020-1034, Stem :1188-1214, HigherResolutionNet :1217-1330, init_weights :1339-1354, get_pose_net
:1524-1527).  Same constructors, module tree and parameter names (reference state_dicts load strictly) and
the same construction / init order (the same seed gives the same weights).  The unused variants of the
reference file (ImprovedTransitionFuse*, HigherDecoder*, OCR, PixelwiseAttention: :489-1017, :1036-1185,
:1405-1521) are not rebuilt.

Forward on the ssseg kernels: every Conv+BN(+ReLU) is one `conv_bn_act` (eval BN folded into the conv
epilogue); BasicBlock / Bottleneck's `skip_add.add_relu` is the conv epilogue's residual + ReLU; the
TransitionFuse branch sums (add ... add_relu) are one n-ary `add_act` pass per output branch, after the
low-resolution branches are bilinearly resized (align_corners=False) on the activation layout; the
multi-resolution aggregator is resize + one `cat_n`.  Returns `([features], [logits])` like the reference
(features: the 480-channel /4 activation; logits: fp32 NCHW at /4).
"""
import logging
import os
from typing import List

import torch
import torch.nn as nn

from ssseg import nn as snn

logger = logging.getLogger(__name__)


class CN(dict):
    """Stand-in for yacs.config.CfgNode (higher_hrnet.py:23): a dict with attribute access."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = v


# small net (higher_hrnet.py:75-121)
POSE_HIGHER_RESOLUTION_NET = CN()
POSE_HIGHER_RESOLUTION_NET.PRETRAINED_LAYERS = ['*']
POSE_HIGHER_RESOLUTION_NET.STEM_INPLANES = 64
POSE_HIGHER_RESOLUTION_NET.FINAL_CONV_KERNEL = 1
POSE_HIGHER_RESOLUTION_NET.NUM_JOINTS = 2
POSE_HIGHER_RESOLUTION_NET.TAG_PER_JOINT = True
for _name, _mods, _branches, _blocks, _chans, _block in (
        ('STAGE1', 1, 1, [2], [64], 'BOTTLENECK'),
        ('STAGE2', 1, 2, [2, 2], [32, 64], 'BASIC'),
        ('STAGE3', 4, 3, [2, 2, 2], [32, 64, 128], 'BASIC'),
        ('STAGE4', 3, 4, [2, 2, 2, 2], [32, 64, 128, 256], 'BASIC')):
    _st = CN()
    _st.NUM_MODULES, _st.NUM_BRANCHES, _st.NUM_BLOCKS, _st.NUM_CHANNELS = _mods, _branches, _blocks, _chans
    _st.BLOCK, _st.FUSE_METHOD = _block, 'SUM'
    POSE_HIGHER_RESOLUTION_NET[_name] = _st
POSE_HIGHER_RESOLUTION_NET.LOSS = CN(WITH_AE_LOSS=[False, False, False])
POSE_HIGHER_RESOLUTION_NET.OCR = CN(DROPOUT=0.05, KEY_CHANNELS=48, MID_CHANNELS=96, SCALE=1)

BN_MOMENTUM = 0.1


def conv3x3(in_planes, out_planes, stride=1):
    return snn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


def _shortcut_grad(downsample, x):
    """The residual block's shortcut gradient route (as models/encoders/resnet.py): identity -> a GradHandoff the
    block's last BN backward fills and its first conv's dgrad adds in its epilogue; a projection (a module of ssseg
    convs) -> x's consumers joined (snn.mark_join), returns None."""
    if isinstance(downsample, nn.Identity):
        return snn.GradHandoff()
    snn.mark_join(x)
    return None


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = snn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = snn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.downsample = downsample if downsample is not None else nn.Identity()
        self.stride = stride

    def forward(self, x):
        # x feeds conv1 and the shortcut: an identity shortcut's gradient is added in conv1's dgrad epilogue
        # (snn.GradHandoff), a projection shortcut's meets conv1's through a join -- no separate autograd add
        h = _shortcut_grad(self.downsample, x)
        residual = self.downsample(x)
        # (no single_use on the branch blocks: with their 32-64 channels the consumer-epilogue BN backward measured
        # slower on C4, 188.3 vs 186.5 ms per graph step)
        out = snn.conv_bn_act(self.conv1, x, self.bn1, relu=True, grad_in=h)
        return snn.conv_bn_act(self.conv2, out, self.bn2, relu=True, residual=residual,
                               grad_out=h)   # skip_add.add_relu


class BottleneckBlock(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = snn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = snn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = snn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = snn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv3 = snn.Conv2d(planes, planes * self.expansion, kernel_size=1, bias=False)
        self.bn3 = snn.BatchNorm2d(planes * self.expansion, momentum=BN_MOMENTUM)
        self.downsample = downsample if downsample is not None else nn.Identity()
        self.stride = stride

    def forward(self, x):
        h = _shortcut_grad(self.downsample, x)
        residual = self.downsample(x)
        out = snn.conv_bn_act(self.conv1, x, self.bn1, relu=True, grad_in=h)
        out = snn.conv_bn_act(self.conv2, out, self.bn2, relu=True)
        return snn.conv_bn_act(self.conv3, out, self.bn3, relu=True, residual=residual, grad_out=h)


class ConvBNRelu(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1):
        super().__init__()
        self.conv = snn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False)
        self.bn = snn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(True)

    def forward(self, input):
        return snn.conv_bn_act(self.conv, input, self.bn, relu=True)


class ConvBN(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1):
        super().__init__()
        self.conv = snn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False)
        self.bn = snn.BatchNorm2d(out_channels)

    def forward(self, input):
        return snn.conv_bn_act(self.conv, input, self.bn, relu=False)


class Stack(nn.Sequential):
    """nn.Sequential whose forward chains the ssseg blocks (keeps the reference's integer child names)."""

    def forward(self, x):
        for m in self:
            x = m(x)
        return x


class TransitionFuse(nn.Module):
    """higher_hrnet.py:369-486.  Output branch i = sum_j f_ij(input_j) (+ReLU on the last add when there
    is more than one input branch): j > i ConvBN 1x1 then bilinear up, j == i identity / ConvBN 1x1,
    j < i a chain of strided 3x3 ConvBN(ReLU)."""

    def __init__(self, num_in_channels, num_out_channels):
        super().__init__()
        self.num_in_branches = len(num_in_channels)
        self.num_out_branches = len(num_out_channels)
        fuse_layers = []
        for i in range(len(num_out_channels)):
            fuse_layer = []
            for j in range(len(num_in_channels)):
                if j > i:
                    fuse_layer.append(ConvBN(num_in_channels[j], num_out_channels[i], kernel_size=1, stride=1,
                                             padding=0))
                elif j == i:
                    if num_in_channels[j] == num_out_channels[i]:
                        fuse_layer.append(nn.Identity())
                    else:
                        fuse_layer.append(ConvBN(num_in_channels[j], num_out_channels[i], kernel_size=1, stride=1,
                                                 padding=0))
                else:
                    conv3x3s = []
                    for k in range(j, i):
                        if k == i - 1:
                            conv3x3s.append(ConvBN(num_in_channels[k], num_out_channels[k + 1], kernel_size=3,
                                                   stride=2, padding=1))
                        else:
                            conv3x3s.append(ConvBNRelu(num_in_channels[k], num_in_channels[k + 1], kernel_size=3,
                                                       stride=2, padding=1))
                    fuse_layer.append(Stack(*conv3x3s))
            fuse_layers.append(nn.ModuleList(fuse_layer))
        self.fuse_layers = nn.ModuleList(fuse_layers)

    def forward(self, input: List[torch.Tensor]):
        if len(self.fuse_layers) > 1:
            # input j feeds every output branch: its conv consumers' input gradients meet in one join (the last one
            # adds the others' in its dgrad epilogue) instead of one autograd add per extra consumer; an identity
            # consumer (j == i) still reaches x_j through autograd's own accumulation
            for t in input:
                snn.mark_join(t)
        output = []
        for i, scale_fuse_layers in enumerate(self.fuse_layers):
            tensors = []
            for j, fuse_layer in enumerate(scale_fuse_layers):
                t = fuse_layer(input[j])
                if i < j:     # smaller scale: resize to branch i (higher_hrnet.py:453-457)
                    t = snn.resize_act(t, (input[i].shape[2], input[i].shape[3]), align_corners=False)
                tensors.append(t)
            # y = t0 (+ t1 ...), add_relu on the last addition (higher_hrnet.py:475-485)
            output.append(snn.add_act(tensors, act=self.num_in_branches > 1))
        return output


class HighResolutionModule(nn.Module):
    def __init__(self, num_in_channels, num_out_channels, num_blocks, block, fuse_method):
        super().__init__()
        self.num_in_channels = num_in_channels
        self.num_out_channels = num_out_channels
        self.fuse_method = fuse_method
        self.num_branches = len(num_out_channels)
        self.fuse_module = TransitionFuse(num_in_channels, num_out_channels)
        self.branches = self._make_branches(self.num_branches, block, num_blocks, num_out_channels)

    def _make_one_branch(self, block, num_blocks, num_channels):
        num_in_channels = num_channels * block.expansion
        return Stack(*[block(num_in_channels, num_channels) for _ in range(num_blocks)])

    def _make_branches(self, num_branches, block, num_blocks, num_channels):
        return nn.ModuleList([self._make_one_branch(block, num_blocks[b], num_channels[b] // block.expansion)
                              for b in range(num_branches)])

    def forward(self, x: List[torch.Tensor]):
        x = self.fuse_module(x)
        return [branch(x[b]) for b, branch in enumerate(self.branches)]


blocks_dict = {'BASIC': BasicBlock, 'BOTTLENECK': BottleneckBlock}


class Stage(nn.Module):
    def __init__(self, num_in_channels, num_out_channels, num_modules, num_blocks, block, fuse_method):
        super().__init__()
        modules = []
        for _ in range(num_modules):
            modules.append(HighResolutionModule(num_in_channels, num_out_channels, num_blocks, block, fuse_method))
            num_in_channels = num_out_channels
        self.num_out_channels = [c * block.expansion for c in num_out_channels]
        self.mods = nn.ModuleList(modules)

    def forward(self, input: List[torch.Tensor]):
        x = input
        for module in self.mods:
            x = module(x)
        return x


class HighResolutionMultiscaleAggregator(nn.Module):
    """higher_hrnet.py:1020-1034: resize every branch to branch 0 (bilinear, align_corners=False), concat."""

    def forward(self, input: List[torch.Tensor]):
        tgt = (input[0].shape[2], input[0].shape[3])
        # the resizes write straight into their channel slices of the concat (snn.resize_cat)
        return snn.resize_cat(input, [t.shape[1] for t in input], tgt, align_corners=False)


class Stem(nn.Module):
    def __init__(self, num_in_channels=3, num_out_channels=64):
        super().__init__()
        self.conv1 = snn.Conv2d(num_in_channels, num_out_channels, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn1 = snn.BatchNorm2d(num_out_channels, momentum=BN_MOMENTUM)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = snn.Conv2d(num_out_channels, num_out_channels, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn2 = snn.BatchNorm2d(num_out_channels, momentum=BN_MOMENTUM)
        self.relu2 = nn.ReLU(inplace=True)

    def forward(self, input):
        x = snn.conv_bn_act(self.conv1, input, self.bn1, relu=True)
        return snn.conv_bn_act(self.conv2, x, self.bn2, relu=True)


class HigherResolutionNet(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        stem_num_channels = cfg['STEM_INPLANES']
        self.stem = Stem(num_in_channels=3, num_out_channels=stem_num_channels)

        def stage_args(name):
            c = cfg[name]
            block = blocks_dict[c['BLOCK']]
            return c, block, [ch * block.expansion for ch in c['NUM_CHANNELS']]

        self.stage1_cfg, block, num_channels = stage_args('STAGE1')
        self.stage1 = Stage([stem_num_channels], num_channels, self.stage1_cfg['NUM_MODULES'],
                            self.stage1_cfg['NUM_BLOCKS'], block, self.stage1_cfg['FUSE_METHOD'])
        self.stage2_cfg, block, num_channels = stage_args('STAGE2')
        # the reference hard-codes 64 * 4 input channels here (higher_hrnet.py:1253-1254)
        self.stage2 = Stage([64 * 4], num_channels, self.stage2_cfg['NUM_MODULES'], self.stage2_cfg['NUM_BLOCKS'],
                            block, self.stage2_cfg['FUSE_METHOD'])
        pre_stage_channels = num_channels
        self.stage3_cfg, block, num_channels = stage_args('STAGE3')
        self.stage3 = Stage(pre_stage_channels, num_channels, self.stage3_cfg['NUM_MODULES'],
                            self.stage3_cfg['NUM_BLOCKS'], block, self.stage3_cfg['FUSE_METHOD'])
        pre_stage_channels = num_channels
        self.stage4_cfg, block, num_channels = stage_args('STAGE4')
        self.stage4 = Stage(pre_stage_channels, num_channels, self.stage4_cfg['NUM_MODULES'],
                            self.stage4_cfg['NUM_BLOCKS'], block, self.stage4_cfg['FUSE_METHOD'])
        pre_stage_channels = num_channels
        num_final_channels = sum(pre_stage_channels)
        self.multires_aggregation = HighResolutionMultiscaleAggregator()
        self.cls_head = nn.Sequential(
            ConvBNRelu(num_final_channels, num_final_channels // 2, kernel_size=3, stride=1, padding=1),
            ConvBNRelu(num_final_channels // 2, num_final_channels // 4, kernel_size=3, stride=1, padding=1),
            snn.Conv2d(num_final_channels // 4, cfg.NUM_JOINTS, kernel_size=1, stride=1, padding=0, bias=True,
                       head=True))

    def forward(self, x):
        x = self.stem(snn.to_act(x))
        y_list = [x]
        y_list = self.stage1(y_list)
        y_list = self.stage2(y_list)
        y_list = self.stage3(y_list)
        y_list = self.stage4(y_list)
        features = self.multires_aggregation(y_list)
        h0, h1, conv = self.cls_head
        logits = conv(h1(h0(features)))
        return [features], [logits]

    def init_weights(self, pretrained='', verbose=True):
        """higher_hrnet.py:1339-1378: N(0, 0.001) conv weights, zero biases, unit BN; optional checkpoint."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, std=0.001)
                for name, _ in m.named_parameters():
                    if name in ['bias']:
                        nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.ConvTranspose2d):
                nn.init.normal_(m.weight, std=0.001)
                for name, _ in m.named_parameters():
                    if name in ['bias']:
                        nn.init.constant_(m.bias, 0)
        if os.path.isfile(pretrained):
            state = torch.load(pretrained, map_location='cpu', weights_only=True)
            names = set(n for n, _ in self.named_parameters()) | set(n for n, _ in self.named_buffers())
            self.load_state_dict({k: v for k, v in state.items() if k in names}, strict=False)


def get_pose_net(cfg):
    model = HigherResolutionNet(cfg)
    model.init_weights('', verbose=False)
    return model

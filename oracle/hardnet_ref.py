"""Oracle: FC-HarDNet (reference models/hardnet.py:100-212) as plain torch.nn on the CPU.  TEST INFRASTRUCTURE ONLY.

A restatement of the reference network's arithmetic for the C5 parity tests (the fp16 compute mode checked against this
network's fp64 and fp16 runs): parameter names, shapes and the construction order of every layer follow the reference
module tree, so the same seed gives the same weights (pinned by golden G6b, tests/golden/model2_hardnet.npz, whose
weight SHA and outputs tests/test_oracle_golden.py checks) and state_dicts move freely between the reference, this
oracle and the HIP product (models/hardnet.py).

  harmonic links   hardnet.py:21-37   layer k (1-based) reads layers k - 2^i for every 2^i dividing k; its width is
                                      growth * grmul^(#links - 1), rounded to an even count
  HarDBlock        hardnet.py:44-83   output = concat of layer 0 if keepBase, every odd layer and the last one
  TransitionUp     hardnet.py:86-101  bilinear (align_corners=True) to the skip's size, then concat [up, skip]
  HarDNet          hardnet.py:104-212 stem (3 ConvLayers, two stride-2), 6 encoder blocks with 1x1 transitions and 2x2
                                      average pools, 5 decoder stages (up + concat + 1x1 halving + HarDBlock), 1x1 head,
                                      bilinear (align_corners=True) back to the input size
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class ConvLayer(nn.Sequential):                                  # hardnet.py:6-17 (conv-BN-ReLU, no bias)
    def __init__(self, cin, cout, kernel=3, stride=1):
        super().__init__()
        self.add_module('conv', nn.Conv2d(cin, cout, kernel, stride, kernel // 2, bias=False))
        self.add_module('norm', nn.BatchNorm2d(cout))
        self.add_module('relu', nn.ReLU())


def harmonic_link(k, base, growth, grmul):
    """(out channels, in channels, source layers) of layer k of a block whose layer 0 has `base` channels."""
    if k == 0:
        return base, 0, []
    srcs = [k - 2 ** i for i in range(10) if k % 2 ** i == 0]
    width = growth * grmul ** (len(srcs) - 1)
    width = int(int(width + 1) / 2) * 2
    return width, sum(harmonic_link(s, base, growth, grmul)[0] for s in srcs), srcs


class HarDBlock(nn.Module):                                      # hardnet.py:20-83
    def __init__(self, cin, growth, grmul, n_layers, keep_base=False):
        super().__init__()
        self.keep_base = keep_base
        self.links = []
        self.out_channels = 0
        mods = []
        for k in range(1, n_layers + 1):
            cout, lin, srcs = harmonic_link(k, cin, growth, grmul)
            self.links.append(srcs)
            mods.append(ConvLayer(lin, cout))
            if k % 2 == 1 or k == n_layers:
                self.out_channels += cout
        self.layers = nn.ModuleList(mods)

    def forward(self, x):
        outs = [x]
        for srcs, layer in zip(self.links, self.layers):
            inp = torch.cat([outs[s] for s in srcs], 1) if len(srcs) > 1 else outs[srcs[0]]
            outs.append(layer(inp))
        last = len(outs) - 1
        keep = [t for i, t in enumerate(outs) if (i == 0 and self.keep_base) or i == last or i % 2 == 1]
        return torch.cat(keep, 1)


class TransitionUp(nn.Module):                                   # hardnet.py:86-101 (no parameters)
    def forward(self, x, skip):
        up = F.interpolate(x, size=skip.shape[2:4], mode='bilinear', align_corners=True)
        return torch.cat([up, skip], 1)


class HarDNet(nn.Module):                                        # hardnet.py:104-212 (HarDNet-68 channel tables)
    STEM = (48, 50, 56, 64)
    WIDTHS = (64, 96, 160, 224, 320, 480)
    GROWTH = (10, 12, 14, 16, 20, 22)
    DEPTHS = (4, 4, 8, 8, 8, 8)
    GRMUL = 1.7

    def __init__(self, n_classes=19):
        super().__init__()
        s = self.STEM
        self.base = nn.ModuleList([ConvLayer(3, s[0], 3, 2), ConvLayer(s[0], s[1], 3), ConvLayer(s[1], s[2], 3, 2),
                                   ConvLayer(s[2], s[3], 3)])
        self.shortcut_layers, skips, ch = [], [], s[3]
        nb = len(self.DEPTHS)
        for i in range(nb):
            blk = HarDBlock(ch, self.GROWTH[i], self.GRMUL, self.DEPTHS[i])
            skips.append(blk.out_channels)
            self.base.append(blk)
            if i < nb - 1:
                self.shortcut_layers.append(len(self.base) - 1)
            self.base.append(ConvLayer(blk.out_channels, self.WIDTHS[i], 1))
            ch = self.WIDTHS[i]
            if i < nb - 1:
                self.base.append(nn.AvgPool2d(2, 2))
        self.n_blocks = nb - 1
        self.transUpBlocks, self.denseBlocksUp, self.conv1x1_up = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        prev = ch
        for i in reversed(range(self.n_blocks)):
            self.transUpBlocks.append(TransitionUp())
            half = (prev + skips[i]) // 2
            self.conv1x1_up.append(ConvLayer(prev + skips[i], half, 1))
            blk = HarDBlock(half, self.GROWTH[i], self.GRMUL, self.DEPTHS[i])
            self.denseBlocksUp.append(blk)
            prev = blk.out_channels
        self.finalConv = nn.Conv2d(prev, n_classes, 1, 1, 0, bias=True)

    def forward(self, x):
        hw = x.shape[2:4]
        skips = []
        for i, m in enumerate(self.base):
            x = m(x)
            if i in self.shortcut_layers:
                skips.append(x)
        for up, squeeze, blk in zip(self.transUpBlocks, self.conv1x1_up, self.denseBlocksUp):
            x = blk(squeeze(up(x, skips.pop())))
        return F.interpolate(self.finalConv(x), size=hw, mode='bilinear', align_corners=True)

"""FC-HarDNet — drop-in for reference models/hardnet.py (ConvLayer :6-17, HarDBlock :20-79, TransitionUp
:82-97, HarDNet :100-212): same constructor (`n_classes`), module tree and parameter names, so reference
state_dicts load strictly.

Forward on the ssseg kernels: ConvLayer = conv -> BN -> ReLU as one `conv_bn_act` (folded into the conv
epilogue for eval BN); the harmonic-dense links and the up-path concatenations are `cat_n` (one gather launch per
concat, real channel counts packed densely — HarDNet's widths are even but not multiples of the MFMA vector; the
backward is one split launch that also sums the gradients of layer outputs read by several consumers); AvgPool2d(2, 2) and the align_corners=True bilinear resizes run on their own kernels.  The output is
fp32 NCHW logits at the input resolution (hardnet.py:207-212).
"""
import torch.nn as nn

from ssseg import nn as snn
from ssseg import ops


class ConvLayer(nn.Sequential):
    """hardnet.py:6-17: Conv(k, stride, pad k//2, no bias) -> BN -> ReLU (`dropout` unused, as in the ref)."""

    def __init__(self, in_channels, out_channels, kernel=3, stride=1, dropout=0.1):
        super().__init__()
        self.add_module('conv', snn.Conv2d(in_channels, out_channels, kernel_size=kernel, stride=stride,
                                           padding=kernel // 2, bias=False))
        self.add_module('norm', snn.BatchNorm2d(out_channels))
        self.add_module('relu', nn.ReLU(inplace=True))
        self.out_channels = out_channels

    def forward(self, x):
        return snn.conv_bn_act(self.conv, x, self.norm, relu=True)


class HarDBlock(nn.Module):
    def get_link(self, layer, base_ch, growth_rate, grmul):
        """hardnet.py:21-38: layer l links to l - 2^i for every 2^i dividing l; width grows by grmul per link."""
        if layer == 0:
            return base_ch, 0, []
        out_channels = growth_rate
        link = []
        for i in range(10):
            dv = 2 ** i
            if layer % dv == 0:
                link.append(layer - dv)
                if i > 0:
                    out_channels *= grmul
        out_channels = int(int(out_channels + 1) / 2) * 2
        in_channels = 0
        for i in link:
            ch, _, _ = self.get_link(i, base_ch, growth_rate, grmul)
            in_channels += ch
        return out_channels, in_channels, link

    def get_out_ch(self):
        return self.out_channels

    def __init__(self, in_channels, growth_rate, grmul, n_layers, keepBase=False, residual_out=False):
        super().__init__()
        self.keepBase = keepBase
        self.links = []
        self.layer_channels = [in_channels]   # real width of layers_[i] (hardnet.py:60)
        layers_ = []
        self.out_channels = 0
        for i in range(n_layers):
            outch, inch, link = self.get_link(i + 1, in_channels, growth_rate, grmul)
            self.links.append(link)
            layers_.append(ConvLayer(inch, outch))
            self.layer_channels.append(outch)
            if (i % 2 == 0) or (i == n_layers - 1):
                self.out_channels += outch
        self.layers = nn.ModuleList(layers_)

    def forward(self, x):
        # every layer output feeds the next layer and up to three later link concats (+ the block's output concat):
        # their input gradients are summed inside the consumers' kernels (snn.GradJoin), not by separate adds
        layers_ = [snn.mark_join(x)]
        for layer in range(len(self.layers)):
            link = self.links[layer]
            x = snn.cat_n([layers_[i] for i in link], [self.layer_channels[i] for i in link])
            layers_.append(snn.mark_join(self.layers[layer](x)))
        t = len(layers_)
        keep = [i for i in range(t) if (i == 0 and self.keepBase) or (i == t - 1) or (i % 2 == 1)]
        return snn.cat_n([layers_[i] for i in keep], [self.layer_channels[i] for i in keep])


class TransitionUp(nn.Module):
    """hardnet.py:82-97: bilinear (align_corners=True) resize to the skip's size, then concat."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.in_channels = in_channels

    def forward(self, x, skip, concat=True, skip_channels=None):
        out = snn.resize_act(x, (skip.size(2), skip.size(3)), align_corners=True)
        if concat:
            out = snn.cat_n([out, skip], [self.in_channels, skip_channels if skip_channels is not None
                                          else skip.shape[1]])
        return out


class HarDNet(nn.Module):
    def __init__(self, n_classes=19):
        super().__init__()
        first_ch = [48, 50, 56, 64]
        ch_list = [64, 96, 160, 224, 320, 480]
        grmul = 1.7
        gr = [10, 12, 14, 16, 20, 22]
        n_layers = [4, 4, 8, 8, 8, 8]
        blks = len(n_layers)
        self.shortcut_layers = []
        self.base = nn.ModuleList([])
        self.base.append(ConvLayer(in_channels=3, out_channels=first_ch[0], kernel=3, stride=2))
        self.base.append(ConvLayer(first_ch[0], first_ch[1], kernel=3))
        self.base.append(ConvLayer(first_ch[1], first_ch[2], kernel=3, stride=2))
        self.base.append(ConvLayer(first_ch[2], first_ch[3], kernel=3))
        skip_connection_channel_counts = []
        ch = first_ch[3]
        for i in range(blks):
            blk = HarDBlock(ch, gr[i], grmul, n_layers[i])
            ch = blk.get_out_ch()
            skip_connection_channel_counts.append(ch)
            self.base.append(blk)
            if i < blks - 1:
                self.shortcut_layers.append(len(self.base) - 1)
            self.base.append(ConvLayer(ch, ch_list[i], kernel=1))
            ch = ch_list[i]
            if i < blks - 1:
                self.base.append(snn.AvgPool2d(kernel_size=2, stride=2))
        self.skip_channels = skip_connection_channel_counts
        prev_block_channels = ch
        n_blocks = blks - 1
        self.n_blocks = n_blocks
        self.transUpBlocks = nn.ModuleList([])
        self.denseBlocksUp = nn.ModuleList([])
        self.conv1x1_up = nn.ModuleList([])
        for i in range(n_blocks - 1, -1, -1):
            self.transUpBlocks.append(TransitionUp(prev_block_channels, prev_block_channels))
            cur_channels_count = prev_block_channels + skip_connection_channel_counts[i]
            self.conv1x1_up.append(ConvLayer(cur_channels_count, cur_channels_count // 2, kernel=1))
            cur_channels_count = cur_channels_count // 2
            blk = HarDBlock(cur_channels_count, gr[i], grmul, n_layers[i])
            self.denseBlocksUp.append(blk)
            prev_block_channels = blk.get_out_ch()
            cur_channels_count = prev_block_channels
        self.finalConv = snn.Conv2d(in_channels=cur_channels_count, out_channels=n_classes, kernel_size=1, stride=1,
                                    padding=0, bias=True, head=True)

    def forward(self, x):
        size_in = x.size()
        x = snn.to_act(x)
        skip_connections = []
        for i in range(len(self.base)):
            x = self.base[i](x)
            if i in self.shortcut_layers:
                skip_connections.append(x)
        out = x
        for i in range(self.n_blocks):
            skip = skip_connections.pop()
            out = self.transUpBlocks[i](out, skip, True, skip_channels=self.skip_channels[self.n_blocks - 1 - i])
            out = self.conv1x1_up[i](out)
            out = self.denseBlocksUp[i](out)
        out = self.finalConv(out)
        return ops.interpolate_bilinear(out, (size_in[2], size_in[3]), align_corners=True)

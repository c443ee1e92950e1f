"""Discriminators — drop-in for reference models/discriminator.py (same constructors, module tree and
parameter names, so reference state_dicts load).

Compute runs on the ssseg engine: every Conv4x4/s2 + LeakyReLU(0.2) pair is one implicit-GEMM launch
with the activation in the epilogue (discriminator.py:14-17, 36-48); the strided conv's input gradient
uses the engine's output-phase decomposition.  The final 1x1 conv is a "head" (fp32 output, real channel
count visible, NCHW-indexable view), like every model's logits.  The input is the 2-channel prediction map
(NCHW fp32) — converted once to the NHWC compute layout.  The reference trainer never calls these modules
(SURVEY §8a row a8); their adversarial use is build-defined (config C5).
"""
import torch.nn as nn

from ssseg import nn as snn

LEAKY = ('leaky', 0.2)


class Discriminator(nn.Module):
    """discriminator.py:6-28: num_layers x [Conv4x4/s2/p1 + LeakyReLU(0.2)], then Conv1x1 (no bias)."""

    def __init__(self, num_layers, in_channels=2, initial_channels=64, max_depth=512, out_channels=1):
        super().__init__()
        layers = nn.ModuleList()
        pred_channels = in_channels
        next_channels = initial_channels
        for _ in range(num_layers):
            layers.append(nn.Sequential(
                snn.Conv2d(pred_channels, next_channels, kernel_size=4, stride=2, padding=1),
                nn.LeakyReLU(0.2, inplace=True)))
            pred_channels = next_channels
            next_channels = min(next_channels * 2, max_depth)
        layers.append(nn.Sequential(snn.Conv2d(pred_channels, out_channels, kernel_size=1, bias=False, head=True)))
        self.net = nn.Sequential(*layers)

    def forward(self, input):
        x = snn.to_act(input)
        for block in self.net:
            conv = block[0]
            # each LeakyReLU output feeds only the next conv: its backward runs inside that conv's input gradient
            x = conv.forward_act(x, LEAKY, single_use=True) if len(block) > 1 else conv(x)
        return x


class MultiscaleFeatureDiscriminator(nn.Module):
    """discriminator.py:31-60: stem Conv4x4/s2 on inputs[0], then per scale cat(out, inputs[i+1]) ->
    Conv4x4/s2 + LeakyReLU, classifier Conv1x1 (bias)."""

    def __init__(self, in_channels=[48, 48 * 2, 48 * 4, 48 * 8], out_channels=[64, 128, 256, 512, 1]):
        super().__init__()
        self.in_channels, self.out_channels = list(in_channels), list(out_channels)
        self.layers = nn.ModuleList()
        self.stem = nn.Sequential(
            snn.Conv2d(in_channels[0], out_channels[0], kernel_size=4, stride=2, padding=1),
            nn.LeakyReLU(0.2, inplace=True))
        for i in range(1, len(out_channels) - 1):
            self.layers.append(nn.Sequential(
                snn.Conv2d(in_channels[i] + out_channels[i - 1], out_channels[i], kernel_size=4, stride=2, padding=1),
                nn.LeakyReLU(0.2, inplace=True)))
        self.classifier = snn.Conv2d(out_channels[-2], out_channels[-1], kernel_size=1, bias=True, head=True)

    def forward(self, inputs):
        out = self.stem[0].forward_act(snn.to_act(inputs[0]), LEAKY)
        for idx, layer in enumerate(self.layers):
            feat = snn.to_act(inputs[idx + 1])
            out = snn.cat_n([out, feat], [self.out_channels[idx], self.in_channels[idx + 1]])
            out = layer[0].forward_act(out, LEAKY)
        return self.classifier(out)

"""Shared pieces of the drop-in model files: norm-layer mapping and the fused Conv+BN+ReLU block."""
import torch.nn as nn

from ssseg import nn as snn


def norm_factory(norm_layer):
    """Map the reference's `norm_layer` argument onto the native BatchNorm2d (SyncBN across ranks)."""
    if norm_layer is None:
        return None
    if norm_layer in (nn.BatchNorm2d, nn.SyncBatchNorm, snn.BatchNorm2d):
        return snn.BatchNorm2d
    raise NotImplementedError(f'norm_layer {norm_layer!r} has no MI355X kernel')


class ConvBlock(nn.Module):
    """Conv(k, pad k//2, no bias) -> BN -> ReLU (unet.py:4-14, simple_unet.py:110-120).

    Same submodule names as the reference (conv_block.0/1/2); forward fuses BN+ReLU into one pass
    (or ReLU into the conv epilogue when norm_layer is None)."""

    def __init__(self, in_channels, out_channels, kernel_size, norm_layer=nn.BatchNorm2d):
        super().__init__()
        norm = norm_factory(norm_layer)
        self.conv_block = nn.Sequential(
            snn.Conv2d(in_channels, out_channels, kernel_size, padding=kernel_size // 2, bias=False),
            norm(out_channels) if norm is not None else nn.Identity(),
            nn.ReLU(),
        )

    def forward(self, x, single_use=False):
        """single_use: the output feeds exactly one conv (UpBlock conv3_0 -> conv3_1; snn.conv_bn_act)."""
        conv, norm, _ = self.conv_block
        if isinstance(norm, nn.Identity):
            return conv.forward_relu(x)
        return snn.conv_bn_act(conv, x, norm, relu=True, single_use=single_use)


def center_crop(tensor, target_size):
    """_center_crop (unet.py:52-60): slice the centre target_size window (plain tensor view)."""
    _, _, h, w = tensor.size()
    top, left = (h - target_size[0]) // 2, (w - target_size[1]) // 2
    return tensor[:, :, top:top + target_size[0], left:left + target_size[1]]

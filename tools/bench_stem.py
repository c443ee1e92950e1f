"""Stem conv (ResNet-50 7x7/s2/p3, 3 -> 64 channels, 512^2 images) device time per launch: the training forward with
fused BN statistics, the folded eval forward (teacher: bs 32) and the differentiated eval forward (raw accumulator
kept), HIP events over 20 launches each, plus an output hash (A/B bit-identity).

    python tools/bench_stem.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import nn as snn  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3, out


def main():
    snn.set_compute_dtype(torch.bfloat16)
    dev = torch.device('cuda')
    torch.manual_seed(0)
    conv = snn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    bn = snn.BatchNorm2d(64).to(dev)
    for n in (16, 32):
        x = snn.to_act(torch.rand(n, 3, 512, 512, device=dev))
        bn.train()
        with torch.no_grad():
            us, y = timed(lambda: snn.conv_bn_act(conv, x, bn, relu=True))
        print(f'bs{n} train fwd + BN stats + apply  {us:8.1f} us  hash {float(y.float().sum()):.6e}')
        bn.eval()
        with torch.no_grad():
            us, y = timed(lambda: snn.conv_bn_act(conv, x, bn, relu=True))
        print(f'bs{n} eval folded fwd             {us:8.1f} us  hash {float(y.float().sum()):.6e}')
        xg = x.detach().requires_grad_(True)
        us, y = timed(lambda: snn.conv_bn_act(conv, xg, bn, relu=True))
        print(f'bs{n} eval fwd, raw copy kept     {us:8.1f} us  hash {float(y.detach().float().sum()):.6e}')


if __name__ == '__main__':
    main()

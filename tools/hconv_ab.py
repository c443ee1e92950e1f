"""A/B of the halo-tiled 3x3 forward kernel (engine variant 24, conv_hconv3.hip) vs the best of the other variants
(the autotuner's choice with knob 11 = -1, which removes variant 24) on the C2 step's 3x3 stride-1 geometries:
forward and input-gradient launches, HIP events, bitwise comparison of the outputs.

    python tools/hconv_ab.py [--reps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402
from ssseg import nn as snn  # noqa: E402

# (cin, cout, hw, batch) -- forward batches 16 (student) and 32 (teacher), input gradients at 16
LAYERS = [(128, 64, 256, 16), (64, 64, 256, 16), (384, 128, 128, 16), (64, 64, 128, 16), (128, 128, 128, 16),
          (640, 128, 64, 16), (128, 128, 64, 16), (64, 64, 128, 32), (128, 64, 256, 32)]


def timeit(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    tot = {}
    for cin, cout, hw, b in LAYERS:
        conv = snn.Conv2d(cin, cout, 3, 1, 1, bias=False).to(dev)
        conv.weight.requires_grad_(False)
        x = snn.to_act(torch.randn(b, cin, hw, hw, device=dev)).requires_grad_(True)
        flops = 2.0 * b * hw * hw * cin * cout * 9
        res, outs = [], {}
        for name, knobs in (('other', ((11, -1), (4, 0))), ('halo', ((11, 0), (4, 24)))):
            for k, v in knobs:
                N.call('ssseg_set_knob', k, v)
            y = conv(x)
            gy = torch.ones_like(y)
            fwd = timeit(lambda: conv(x), a.reps)
            bwd = timeit(lambda: torch.autograd.grad(conv(x), x, gy), a.reps) - fwd
            outs[name] = (conv(x).detach().clone(), torch.autograd.grad(conv(x), x, gy)[0].clone())
            tot[name] = tot.get(name, 0.0) + fwd + bwd
            res.append(f'{name}: fwd {fwd:7.1f} us {flops / fwd / 1e6:6.0f} TF/s dgrad {bwd:7.1f} us '
                       f'{flops / bwd / 1e6:6.0f} TF/s')
        same = torch.equal(outs['halo'][0], outs['other'][0]) and torch.equal(outs['halo'][1], outs['other'][1])
        print(f'{cin:4d}->{cout:<4d} @{b}x{hw}x{hw}: ' + ' | '.join(res) + f' | bitwise {same}', flush=True)
    N.call('ssseg_set_knob', 4, 0)
    N.call('ssseg_set_knob', 11, 0)
    print('total us: ' + ', '.join(f'{k} {v:.1f}' for k, v in tot.items()))


if __name__ == '__main__':
    main()

"""A/B of the halo-tiled 3x3 weight gradient (knob 11 = 0) vs the split-K LDS-DMA kernel (knob 11 = -1) on the C2
step's 3x3 stride-1 geometries (batch 32 = the merged supervised + consistency launch), HIP events per launch (incl.
the slab reduce), and the max relative deviation between the two (summation order only).

    python tools/halo_ab.py [--batch 32] [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402
from ssseg import nn as snn  # noqa: E402

LAYERS = [(128, 64, 256), (384, 128, 128), (64, 64, 256), (128, 128, 64), (64, 64, 128), (640, 128, 64),
          (128, 128, 128), (256, 256, 32), (512, 512, 16), (1152, 128, 32)]


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
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layers", type=int, default=len(LAYERS))
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    tot = {0: 0.0, -1: 0.0}
    for cin, cout, hw in LAYERS[:a.layers]:
        conv = snn.Conv2d(cin, cout, 3, 1, 1, bias=False).to(dev)
        x = snn.to_act(torch.randn(a.batch, cin, hw, hw, device=dev))
        gy = snn.to_act(torch.randn(a.batch, cout, hw, hw, device=dev))
        flops = 2.0 * a.batch * hw * hw * cin * cout * 9
        out, res = {}, []
        for knob in (0, -1):
            N.call('ssseg_set_knob', 11, knob)

            def run():
                conv.weight.grad = None
                conv._ssseg_wgrad(x, gy, bias_grad=False, want=(True, False))
            us = timeit(run, a.reps)
            out[knob] = conv.weight.grad.detach().clone()
            tot[knob] += us
            res.append(f'{"halo" if knob == 0 else "splitK"} {us:8.1f} us {flops / us / 1e6:7.1f} TF/s')
        d = float((out[0] - out[-1]).abs().max() / out[-1].abs().max())
        print(f'{cin:5d}->{cout:<5d} @{a.batch}x{hw}x{hw}: ' + ' | '.join(res) + f' | rel diff {d:.1e}', flush=True)
    N.call('ssseg_set_knob', 11, 0)
    print(f'total: halo {tot[0]:.1f} us, split-K {tot[-1]:.1f} us')


if __name__ == '__main__':
    main()

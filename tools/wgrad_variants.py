"""Weight-gradient LDS-DMA configs (knob 9, WGRAD_CFGS in conv_wgrad.hip) x split scales (knob 10) on the C2
step's weight-gradient geometries (batch 32 = the merged supervised + consistency launch).  Prints us per launch
(incl. the slab reduce) and the max relative deviation of dW from the static plan's (summation order only).

    python tools/wgrad_variants.py [--batch 32] [--cfgs 1,2,...] [--scales 50,100,200] > gpurun_out/wgv.txt
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402
from ssseg import nn as snn  # noqa: E402

# (cin, cout, k, hw) at 512x512 input, the C2 step's largest weight gradients first (profiles/r2j_conv_layers.txt)
LAYERS = [(128, 64, 3, 256), (384, 128, 3, 128), (256, 256, 3, 32), (64, 64, 3, 256), (128, 128, 3, 64),
          (64, 64, 3, 128), (64, 256, 1, 128), (256, 1024, 1, 32), (640, 128, 3, 64), (1024, 256, 1, 32),
          (128, 512, 1, 64), (512, 512, 3, 16), (1152, 128, 3, 32), (2048, 512, 1, 16), (512, 2048, 1, 16)]
CFG_C = {1: 64, 2: 128, 3: 64, 4: 128, 5: 128, 6: 128, 7: 128, 8: 64, 9: 256, 10: 128, 11: 64, 12: 128, 13: 64, 19: 128, 20: 64,
         14: 64, 15: 64, 16: 64, 17: 128, 18: 128}


def timeit(fn, reps=5):
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
    ap.add_argument('--cfgs', default='0,1,3,4,5,6,14,15,16,17,18')
    ap.add_argument('--scales', default='100,70,50,35,25')
    ap.add_argument('--layers', type=int, default=len(LAYERS))
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    cfgs = [int(c) for c in a.cfgs.split(',')]
    scales = [int(s) for s in a.scales.split(',')]
    best_tot = base_tot = 0.0
    for cin, cout, k, hw in LAYERS[:a.layers]:
        conv = snn.Conv2d(cin, cout, k, 1, k // 2, bias=False).to(dev)
        x = snn.to_act(torch.randn(a.batch, cin, hw, hw, device=dev))
        gy = snn.to_act(torch.randn(a.batch, cout, hw, hw, device=dev))
        flops = 2.0 * a.batch * hw * hw * cin * cout * k * k
        res = []
        ref = None
        for c in cfgs:
            if c and cin % CFG_C[c]:
                continue
            for sc in scales:
                if c == 0 and sc != 100:
                    continue
                N.call('ssseg_set_knob', 9, c)
                N.call('ssseg_set_knob', 10, sc)

                def run():
                    conv.weight.grad = None
                    conv._ssseg_wgrad(x, gy, bias_grad=False)
                us = timeit(run)
                g = conv.weight.grad.detach().clone()
                if ref is None:
                    ref = g
                dev_ = float((g - ref).abs().max() / (ref.abs().max() + 1e-30))
                res.append((us, c, sc, dev_))
        N.call('ssseg_set_knob', 9, 0)
        N.call('ssseg_set_knob', 10, 100)
        base = res[0][0]
        best = min(res)
        best_tot += best[0]
        base_tot += base
        line = ' '.join(f'{c}/{sc}:{us:.0f}' + ('!' if d > 1e-4 else '') for us, c, sc, d in res)
        print(f'{cin:5d}->{cout:5d} k{k} @{a.batch}x{hw:3d}: static {base:8.1f} us ({flops / base / 1e6:6.1f} TF/s)  '
              f'best cfg {best[1]} x{best[2]}% {best[0]:8.1f} us ({flops / best[0] / 1e6:6.1f} TF/s) | {line}',
              flush=True)
    print(f'total static {base_tot:.1f} us, best {best_tot:.1f} us')


if __name__ == '__main__':
    main()

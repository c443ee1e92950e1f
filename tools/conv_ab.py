"""Time one conv layer's forward and forward+backward (dgrad + wgrad) on the engine, after autotuning, for several
channel shapes -- e.g. a general-k layer (C % 64 != 0) against the same layer with its channels padded to 64.

    python tools/conv_ab.py 480,240,3,256 512,256,3,256 [--batch 16] [--reps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import nn as snn  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('layers', nargs='+', help='cin,cout,k,hw')
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    for spec in a.layers:
        cin, cout, k, hw = (int(v) for v in spec.split(','))
        conv = snn.Conv2d(cin, cout, k, 1, k // 2, bias=False).to(dev)
        x = snn.to_act(torch.randn(a.batch, cin, hw, hw, device=dev)).requires_grad_(True)
        gy = None

        def fwd():
            with torch.no_grad():
                conv(x)

        def fwdbwd():
            nonlocal gy
            y = conv(x)
            if gy is None:
                gy = torch.randn_like(y)
            y.backward(gy)
            x.grad = None
            conv.weight.grad = None

        tf = timed(fwd, a.reps)
        tb = timed(fwdbwd, a.reps)
        gf = 2.0 * a.batch * hw * hw * cin * cout * k * k / 1e9
        print(f'{cin}->{cout} k{k} @{a.batch}x{hw}^2: fwd {tf:.3f} ms ({gf / tf:.0f} TF/s), fwd+bwd {tb:.3f} ms '
              f'({3 * gf / tb:.0f} TF/s)', flush=True)


if __name__ == '__main__':
    main()

"""Run ONE conv layer's forward / dgrad / wgrad launch REPS times (for rocprofv3 --pmc passes on a single kernel).

    python tools/one_layer.py --kind wgrad --cin 128 --cout 64 --k 3 --hw 256 --batch 32 [--reps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import nn as snn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kind', default='wgrad', choices=['fwd', 'dgrad', 'wgrad'])
    ap.add_argument('--cin', type=int, default=128)
    ap.add_argument('--cout', type=int, default=64)
    ap.add_argument('--k', type=int, default=3)
    ap.add_argument('--stride', type=int, default=1)
    ap.add_argument('--hw', type=int, default=256)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--variant', type=int, default=0, help='forced LDS-DMA config (knob 4; 0 = autotune)')
    ap.add_argument('--wvariant', type=int, default=0, help='forced weight-gradient config (knob 9)')
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    from ssseg import native as N
    N.lib().ssseg_set_knob(4, a.variant)
    N.lib().ssseg_set_knob(9, a.wvariant)
    conv = snn.Conv2d(a.cin, a.cout, a.k, a.stride, a.k // 2, bias=False).to(dev)
    x = snn.to_act(torch.randn(a.batch, a.cin, a.hw, a.hw, device=dev))
    with torch.no_grad():
        y = conv(x)
    gy = snn.to_act(torch.randn(y.shape[0], a.cout, y.shape[2], y.shape[3], device=dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.reps + 1):
        if r == 1:
            e0.record()
        if a.kind == 'wgrad':
            conv._ssseg_wgrad(x, gy, bias_grad=False)
        elif a.kind == 'dgrad':
            conv._ssseg_dgrad(gy, x.shape)
        else:
            with torch.no_grad():
                conv(x)
    e1.record()
    torch.cuda.synchronize()
    print(f'v{a.variant}/{a.wvariant} {a.kind} {a.cin}->{a.cout} k{a.k} s{a.stride} @{a.batch}x{a.hw}^2: {e0.elapsed_time(e1) / a.reps * 1e3:.1f} us')


if __name__ == '__main__':
    main()

"""Weight-gradient cost at batch 2B vs two launches at batch B (does merging the supervised and the consistency
backward's weight gradients into one launch pay?).  For each C2 layer geometry: time ssseg_conv_wgrad at
batch B twice (accumulate) and once at batch 2B.

    python tools/bench_wgrad_batch.py [--batch 16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402
from ssseg import nn as snn  # noqa: E402

LAYERS = [(128, 64, 3, 256), (64, 64, 3, 256), (384, 128, 3, 128), (64, 64, 3, 128), (128, 128, 3, 64),
          (256, 256, 3, 32), (512, 512, 3, 16), (64, 256, 1, 128), (256, 1024, 1, 32), (1024, 256, 1, 32),
          (512, 2048, 1, 16), (2048, 512, 1, 16), (1152, 128, 3, 32), (640, 128, 3, 64)]


def timeit(fn, reps=10):
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
    ap.add_argument('--batch', type=int, default=16)
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    tot1 = tot2 = 0.0
    for cin, cout, k, hw in LAYERS:
        conv = snn.Conv2d(cin, cout, k, 1, k // 2, bias=False).to(dev)
        res = {}
        for n in (a.batch, 2 * a.batch):
            x = snn.to_act(torch.randn(n, cin, hw, hw, device=dev))
            gy = snn.to_act(torch.randn(n, cout, hw, hw, device=dev))
            res[n] = timeit(lambda: conv._ssseg_wgrad(x, gy, bias_grad=False))
        two, one = 2 * res[a.batch], res[2 * a.batch]
        tot1 += two
        tot2 += one
        print(f'{cin:5d}->{cout:5d} k{k} @{hw:3d}: 2 x B{a.batch} {two:8.1f} us   1 x B{2 * a.batch} {one:8.1f} us  '
              f'({one / two:.2f})', flush=True)
    print(f'total: {tot1:.1f} us -> {tot2:.1f} us ({tot2 / tot1:.2f})')


if __name__ == '__main__':
    main()

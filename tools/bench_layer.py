"""Time ONE conv layer's forward under every engine variant (knob 4) and compare with a plain write of the
same output bytes (torch fill_), so memory-bound layers can be priced against their floor.

    python tools/bench_layer.py [--cin 64 --cout 256 --k 1 --stride 1 --hw 128 --batch 16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402
from ssseg import nn as snn  # noqa: E402


def timeit(fn, reps=20):
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
    ap.add_argument('--cin', type=int, default=64)
    ap.add_argument('--cout', type=int, default=256)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--stride', type=int, default=1)
    ap.add_argument('--hw', type=int, default=128)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--rotate', type=int, default=1, help='keep this many outputs alive (>1: cold-cache writes)')
    a = ap.parse_args()
    import collections
    keep = collections.deque(maxlen=a.rotate)
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    conv = snn.Conv2d(a.cin, a.cout, a.k, a.stride, a.k // 2, bias=False).to(dev)
    x = snn.to_act(torch.randn(a.batch, a.cin, a.hw, a.hw, device=dev))
    with torch.no_grad():
        y = conv(x)
    out_bytes = y.numel() * 2
    in_bytes = x.numel() * 2
    flops = 2.0 * y.shape[0] * y.shape[2] * y.shape[3] * a.cout * a.cin * a.k * a.k
    fill = torch.empty_like(y)
    fills = [torch.empty_like(y) for _ in range(a.rotate)]
    it = iter(range(1 << 30))
    t = timeit(lambda: fills[next(it) % a.rotate].fill_(1.0))
    print(f'layer {a.cin}->{a.cout} k{a.k} s{a.stride} @{a.batch}x{a.hw}^2: out {out_bytes / 1e6:.1f} MB in '
          f'{in_bytes / 1e6:.1f} MB, {flops / 1e9:.1f} GFLOP; torch fill of the output: {t:.1f} us '
          f'({out_bytes / t / 1e3:.0f} GB/s)')
    src = torch.empty(y.numel() // 2 + x.numel() // 2 * 0, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    t = timeit(lambda: dst.copy_(src))
    print(f'torch copy of {src.numel() * 4 / 1e6:.1f} MB: {t:.1f} us ({2 * src.numel() * 4 / t / 1e3:.0f} GB/s)')
    if a.k == 1 and a.stride == 1:
        xm = torch.randn(x.numel() // a.cin, a.cin, device=dev, dtype=torch.bfloat16)
        wm = torch.randn(a.cin, a.cout, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(xm, wm))
        print(f'torch.mm (hipBLASLt) same GEMM: {t:.1f} us  {(in_bytes + out_bytes) / t / 1e3:6.0f} GB/s')
    for v in [11] + list(range(1, 11)) + list(range(12, 18)):
        N.call('ssseg_set_knob', 4, v)
        with torch.no_grad():
            t = timeit(lambda: keep.append(conv(x)))
        print(f'variant {v:2d}: {t:8.1f} us  {(in_bytes + out_bytes) / t / 1e3:6.0f} GB/s  {flops / t / 1e6:6.0f} TF')
    N.call('ssseg_set_knob', 4, 0)


if __name__ == '__main__':
    main()

"""Bandwidth of the BatchNorm kernels at UNet-R50 shapes (bf16 NHWC), HIP events, one process.

    python tools/bench_bn.py [--knob ID:VAL,...]

Prints, per (P, C) shape and kernel, microseconds and algorithmic GB/s (bytes each kernel must move).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402

SHAPES = [(16 * 256 * 256, 64), (16 * 128 * 128, 256), (16 * 64 * 64, 512), (16 * 32 * 32, 1024), (16 * 16 * 16, 2048)]


def timeit(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--knob', default='')
    a = ap.parse_args()
    dev = torch.device('cuda')
    for kv in filter(None, a.knob.split(',')):
        k, v = kv.split(':')
        N.call('ssseg_set_knob', int(k), int(v))
    s = N.stream()
    bf = N.BF16 if hasattr(N, 'BF16') else 1
    for P, C in SHAPES:
        x = torch.randn(P, C, device=dev).bfloat16()
        dy = torch.randn(P, C, device=dev).bfloat16()
        r = torch.randn(P, C, device=dev).bfloat16()
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x)
        mean = torch.zeros(C, device=dev)
        inv = torch.ones(C, device=dev)
        g = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        sums = torch.zeros(2 * C, device=dev, dtype=torch.float64)
        nb = N.lib().ssseg_bn_workspace_bytes(C)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        p = N.dev_ptr
        e = P * C
        rows = []
        t = timeit(lambda: N.call('ssseg_bn_stats', p(x), P, C, C, bf, p(sums), p(ws), nb, s))
        rows.append(('stats', t, 2 * e))
        t = timeit(lambda: N.call('ssseg_bn_apply', p(x), p(r), p(y), P, C, C, C, C, p(mean), p(inv), p(g), p(b), 1,
                                  bf, s))
        rows.append(('apply+res', t, 6 * e))
        t = timeit(lambda: N.call('ssseg_bn_apply', p(x), None, p(y), P, C, C, C, C, p(mean), p(inv), p(g), p(b), 1,
                                  bf, s))
        rows.append(('apply', t, 4 * e))
        t = timeit(lambda: N.call('ssseg_bn_bwd_reduce', p(dy), p(x), p(r), P, C, C, C, C, p(mean), p(inv), p(g),
                                  p(b), 1, bf, p(sums), p(ws), nb, s))
        rows.append(('bwd_reduce+res', t, 6 * e))
        t = timeit(lambda: N.call('ssseg_bn_bwd_reduce', p(dy), p(x), None, P, C, C, C, C, p(mean), p(inv), p(g),
                                  p(b), 1, bf, p(sums), p(ws), nb, s))
        rows.append(('bwd_reduce', t, 4 * e))
        t = timeit(lambda: N.call('ssseg_bn_bwd_apply', p(dy), p(x), p(r), p(dx), p(dres), P, C, C, C, C, C, p(mean),
                                  p(inv), p(g), p(b), 1, 1, p(sums), float(P), bf, s))
        rows.append(('bwd_apply+res', t, 10 * e))
        t = timeit(lambda: N.call('ssseg_bn_eval_bwd', p(dy), p(y), p(x), p(dx), None, P, C, C, p(g), p(mean), p(inv),
                                  1, bf, p(sums), p(ws), nb, s))
        rows.append(('eval_bwd', t, 8 * e))
        t = timeit(lambda: N.call('ssseg_nhwc_copy', p(x), p(y), 16, P // 16, 1, C, C, C, 0, 0, 0, 0, bf, s)
                   if False else y.copy_(x))
        rows.append(('torch copy', t, 4 * e))
        for name, us, by in rows:
            print(f'P={P:8d} C={C:5d} {name:15s} {us:8.1f} us {by / us / 1e3:7.0f} GB/s')


if __name__ == '__main__':
    main()

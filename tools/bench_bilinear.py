"""Device time of the fp32 logits resizes (ssseg_bilinear_fwd / _bwd: NHWC logits with a padded pixel stride -> NCHW
at the image size, train.py:71,74,93 / losses.py:18) and a hash of the results, for A/B runs of the per-pixel kernels
(SSSEG_BIL_PIX=0 turns them off; run both and compare the hashes: they must be equal).

    python tools/bench_bilinear.py [--n 16 --c 2 --ldc 8 --hin 256 --hout 512]
"""
import argparse
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..',
                                'semi-supervised_semantic_segmentation_amd'))


def main():
    from ssseg import native as N
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=16)
    ap.add_argument('--c', type=int, default=2)
    ap.add_argument('--ldc', type=int, default=8)
    ap.add_argument('--hin', type=int, default=256)
    ap.add_argument('--hout', type=int, default=512)
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    g = torch.Generator().manual_seed(0)
    base = torch.randn(a.n, a.ldc, a.hin, a.hin, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    x = base[:, :a.c]
    y = torch.empty(a.n, a.c, a.hout, a.hout, device=dev)
    gy = torch.randn(a.n, a.c, a.hout, a.hout, generator=g).to(dev)
    gxb = torch.zeros_like(base)
    gx = gxb[:, :a.c]
    st = N.stream()

    def fwd():
        N.call('ssseg_bilinear_fwd', N.dev_ptr(x), N.dev_ptr(y), a.n, a.c, a.hin, a.hin, a.hout, a.hout,
               N.strides4(x), N.strides4(y), 0, N.F32, st)

    def bwd():
        N.call('ssseg_bilinear_bwd', N.dev_ptr(gy), N.dev_ptr(gx), a.n, a.c, a.hin, a.hin, a.hout, a.hout,
               N.strides4(gy), N.strides4(gx), 0, N.F32, st)

    res = {}
    for name, fn in (('fwd', fwd), ('bwd', bwd)):
        for _ in range(3):
            fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = []
        for _ in range(a.reps):
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
        ts.sort()
        res[name] = ts[len(ts) // 2]
    torch.cuda.synchronize()
    h = hashlib.sha256(y.cpu().numpy().tobytes() + gx.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"pix={os.environ.get('SSSEG_BIL_PIX', '1')} fwd {res['fwd']:.1f} us  bwd {res['bwd']:.1f} us  hash {h}")


if __name__ == '__main__':
    main()

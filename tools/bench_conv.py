"""Per-layer conv-engine timing on the C2 model (UNet-R50 512x512, bs16, bf16): one forward + backward,
HIP events around every conv launch, interleaved over kernel variants (ssseg_set_knob) in ONE process.

    python tools/bench_conv.py [--knobs 3:-1,3:0/4:0,3:0/4:6] [--rounds 3] [--batch 16] [--size 512] [--top 25]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--knobs', default='0:1')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--top', type=int, default=25)
    args = ap.parse_args()
    from models import unet
    from models.encoders import resnet
    from ssseg import native as N
    from ssseg import nn as snn
    snn.set_compute_dtype(torch.bfloat16)
    dev = torch.device('cuda')
    torch.manual_seed(0)
    model = unet.UNet(2, resnet.resnet50_encoder(), 128, train_upsampling=True).to(dev)
    x = torch.rand(args.batch, 3, args.size, args.size, device=dev)
    gy = torch.randn(args.batch, 2, args.size // 2, args.size // 2, device=dev)
    # a variant is one or more knob settings joined by '/': e.g. 3:-1,3:0/4:0,3:0/4:6
    variants = [tuple(tuple(int(v) for v in kv.split(':')) for kv in var.split('/')) for var in args.knobs.split(',')]

    def run():
        y = model(x)
        y.backward(gy)

    for _ in range(2):
        run()
    res = {v: collections.defaultdict(list) for v in variants}
    tot = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            for kid, kval in v:
                N.call('ssseg_set_knob', kid, kval)
            run()
            torch.cuda.synchronize()
            rows = snn.probe(True)
            run()
            snn.probe(False)
            torch.cuda.synchronize()
            t = 0.0
            per = collections.defaultdict(lambda: [0.0, 0.0])
            for e0, e1, fl, kind, tag in rows:
                ms = e0.elapsed_time(e1)
                per[(kind, tag)][0] += ms
                per[(kind, tag)][1] += fl
                t += ms
            for k, (ms, fl) in per.items():
                res[v][k].append((ms, fl))
            tot[v].append(t)
    for v in variants:
        ts = sorted(tot[v])
        print(f'knob {v}: conv engine fwd+bwd median {ts[len(ts) // 2]:.2f} ms (min {ts[0]:.2f})')
    base = variants[0]
    keys = sorted(res[base], key=lambda k: -min(m for m, _ in res[base][k]))
    print(f"{'kind':6s} {'layer':45s} " + ' '.join(f'{str(v):>16s}' for v in variants))
    for k in keys[:args.top]:
        cells = []
        for v in variants:
            ms = min(m for m, _ in res[v][k])
            fl = res[v][k][0][1]
            cells.append(f'{ms:7.3f}ms {fl / ms / 1e9:5.0f}TF')
        print(f'{k[0]:6s} {k[1]:45s} ' + ' '.join(f'{c:>16s}' for c in cells))


if __name__ == '__main__':
    main()

"""Per-layer conv-engine breakdown of one FULL C2 training step (the bench.py workload: supervised pass,
two teacher passes, the eval-mode consistency pass and both backwards), from the live HIP-event probe
bench.py's roofline uses: for every (kind, layer geometry) the summed duration, flops and TF/s, sorted by
time.  Shows which layers hold the step's conv time.

    python tools/layer_report.py [--batch 16] [--size 512] [--top 50] > gpurun_out/layers.txt
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
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--top', type=int, default=50)
    a = ap.parse_args()
    import bench
    import train
    from ssseg import nn as snn
    dev = torch.device('cuda', 0)
    snn.set_compute_dtype(torch.bfloat16)
    model, teacher, opt, cfg = bench.build(a.batch, a.size, dev)
    data = bench.synthetic_batches(2, a.batch, a.size, dev, 0)
    model.train()
    opt.zero_grad()
    for s in range(3):
        img, mask, ua, ub = data[s % 2]
        train.train_step(model, teacher, opt, img, mask, ua, ub, 30, s, cfg)
    torch.cuda.synchronize()
    rows = snn.probe(True)
    img, mask, ua, ub = data[1]
    train.train_step(model, teacher, opt, img, mask, ua, ub, 30, 3, cfg)
    snn.probe(False)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    by_kind = collections.defaultdict(lambda: [0.0, 0.0])
    for e0, e1, fl, kind, tag in rows:
        ms = e0.elapsed_time(e1)
        r = agg[(kind, tag)]
        r[0] += ms
        r[1] += fl
        r[2] += 1
        by_kind[kind][0] += ms
        by_kind[kind][1] += fl
    tot_ms = sum(v[0] for v in agg.values())
    tot_fl = sum(v[1] for v in agg.values())
    print(f'conv engine: {tot_ms:.3f} ms, {tot_fl / 1e9:.1f} GFLOP, {tot_fl / tot_ms / 1e9:.1f} TF/s, {len(rows)} calls')
    for k, (ms, fl) in sorted(by_kind.items(), key=lambda kv: -kv[1][0]):
        print(f'  {k:6s} {ms:8.3f} ms  {fl / 1e9:8.1f} GFLOP  {fl / ms / 1e9:7.1f} TF/s')
    print(f'{"ms":>8s} {"pct":>6s} {"calls":>5s} {"GFLOP":>8s} {"TF/s":>7s}  kind   layer')
    for (kind, tag), (ms, fl, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f'{ms:8.3f} {100 * ms / tot_ms:6.2f} {n:5d} {fl / 1e9:8.1f} {fl / ms / 1e9:7.1f}  {kind:6s} {tag}')


if __name__ == '__main__':
    main()

"""A/B of the fused BatchNorm statistics epilogue: one conv forward with and without `stats` (StatRows partial rows,
the training pass's conv -> BN), per LDS-DMA config (knob 4), on the layers named on the command line.

    python tools/stats_ab.py 64,256,1,128 128,512,1,64 [--batch 16] [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd'))

import torch  # noqa: E402

from ssseg import native as N  # noqa: E402
from ssseg import nn as snn  # noqa: E402

CFGS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 26, 27]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('layers', nargs='+', help='cin,cout,k,hw')
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--sdbg', default='0', help='comma list of knob-12 values (fused-statistics experiment switch: '
                    '1 no sums, 2 no tile_stats, 4 no row write, 8 no shuffles); --tune runs the stats launch per value')
    ap.add_argument('--tune', action='store_true',
                    help='print the autotuner\'s own per-config event timings (SSSEG_TUNE_LOG=1 must be set) for the plain '
                         'and the statistics launch of each layer instead of the Python-timed loop')
    a = ap.parse_args()
    dev = torch.device('cuda')
    snn.set_compute_dtype(torch.bfloat16)
    for spec in a.layers:
        cin, cout, k, hw = (int(v) for v in spec.split(','))
        conv = snn.Conv2d(cin, cout, k, 1, k // 2, bias=False).to(dev)
        x = snn.to_act(torch.randn(a.batch, cin, hw, hw, device=dev))
        cap = conv.stat_rows_cap(a.batch, hw, hw)
        if a.tune:
            for st, dbg in [(False, 0)] + [(True, int(v)) for v in a.sdbg.split(',')]:
                N.lib().ssseg_set_knob(6, 1)   # clear the variant cache: the next launch tunes (and logs)
                N.lib().ssseg_set_knob(12, dbg)
                print(f'{cin}->{cout} k{k} @{a.batch}x{hw}^2 stats={st} sdbg={dbg}', file=sys.stderr, flush=True)
                with torch.no_grad():
                    conv._ssseg_forward(x, False, stats=snn.StatRows(cout, cap, dev) if st else None)
                torch.cuda.synchronize()
            N.lib().ssseg_set_knob(12, 0)
            continue
        line = []
        for v in CFGS:
            N.lib().ssseg_set_knob(4, v)
            res = []
            for st in (False, True):
                def run():
                    stats = snn.StatRows(cout, cap, dev) if st else None
                    with torch.no_grad():
                        conv._ssseg_forward(x, False, stats=stats)
                try:
                    run()
                except RuntimeError:
                    res.append(float('nan'))
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run()
                e1.record()
                torch.cuda.synchronize()
                res.append(e0.elapsed_time(e1) / a.reps * 1e3)
            line.append(f'{v}:{res[0]:.0f}/{res[1]:.0f}')
        N.lib().ssseg_set_knob(4, 0)
        print(f'{cin}->{cout} k{k} @{a.batch}x{hw}^2 (plain/stats us): ' + ' '.join(line), flush=True)


if __name__ == '__main__':
    main()

"""Device occupancy of the last N steps of a rocprofv3 kernel trace (csv) of bench.py: wall span per step, the union of
the kernels' [start, end) intervals (busy), idle = span - busy, and the time with two or more kernels in flight (the
side-stream overlap of train.train_step).  Steps are delimited by sgd_kernel launches.

    python tools/trace_busy.py gpurun_out/r6_gtrace/g_kernel_trace.csv [--steps 7]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, default=7)
    ap.add_argument('--skip-last', type=int, default=0, help='steps at the end to leave out (e.g. bench.py\'s eager_n1 '
                    'steps after the graph-replayed ones)')
    a = ap.parse_args()
    rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'])
                  for r in csv.DictReader(open(a.trace)))
    sgd = sorted(e for s, e, n in rows if 'sgd_kernel' in n)
    end = len(sgd) - 1 - a.skip_last
    t0, t1 = sgd[end - a.steps], sgd[end]
    sel = [(s, e) for s, e, _ in rows if s >= t0 and e <= t1]
    ev = sorted([(s, 1) for s, _ in sel] + [(e, -1) for _, e in sel])
    busy = multi = 0
    depth, last = 0, t0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    span = t1 - t0
    ksum = sum(e - s for s, e in sel)
    n = a.steps
    print(f'{n} steps: span {span / n / 1e6:.3f} ms/step, busy {busy / n / 1e6:.3f}, idle {(span - busy) / n / 1e6:.3f}, '
          f'>= 2 kernels in flight {multi / n / 1e6:.3f}, kernel-time sum {ksum / n / 1e6:.3f} ms/step, '
          f'{len(sel) / n:.0f} launches/step')


if __name__ == '__main__':
    main()

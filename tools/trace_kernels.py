"""Per-kernel (function name, template arguments dropped) time per step over the last N timed steps (delimited by
sgd_kernel launches) of a rocprofv3 --output-format csv kernel trace of bench.py.

    python tools/trace_kernels.py gpurun_out/btrace/b_kernel_trace.csv [--steps 7]
"""
import argparse
import collections
import csv
import re


def base(name):
    n = name.replace('(anonymous namespace)::', '')
    n = n.split('(')[0]
    n = re.sub(r'^void ', '', n)
    return re.sub(r'<.*', '', n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, default=7)
    ap.add_argument('--skip-last', type=int, default=0, help="steps at the end to leave out (bench.py's eager_n1 steps)")
    a = ap.parse_args()
    rows = [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in csv.DictReader(open(a.trace))]
    sgd = sorted(s for n, s, e in rows if 'sgd_kernel' in n)
    end = len(sgd) - 1 - a.skip_last
    t0, t1 = sgd[end - a.steps], sgd[end]
    sel = [(n, s, e) for n, s, e in rows if t0 < s <= t1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in sel:
        agg[base(n)][0] += 1
        agg[base(n)][1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    span = (max(e for _, _, e in sel) - min(s for _, s, _ in sel)) / 1e6
    print(f'steps {a.steps}: span {span / a.steps:.3f} ms/step, kernel time {tot / a.steps / 1e3:.3f} ms/step')
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f'{c / a.steps:7.1f}/step {t / a.steps:9.1f} us/step {t / c:7.1f} us avg  {k}')


if __name__ == '__main__':
    main()

"""Per-family kernel time per step of the last N timed steps (delimited by sgd_kernel launches) from a rocprofv3
--output-format csv kernel trace of bench.py.

    python tools/trace_families.py gpurun_out/btrace/b_kernel_trace.csv [--steps 20]
"""
import argparse
import collections
import csv

FAMILIES = ['igemm_glds', 'hconv3', 'igemm_kernel', 'wgrad_halo3', 'wgrad_glds', 'wgrad_kernel', 'wgrad_reduce',
            'bn_bwd_apply', 'bn_eval_bwd', 'bn_partial_final', 'bn_partial_rows', 'bn_partial_kernel', 'bn_apply',
            'bn_fold', 'bn_finalize', 'stem', 'weight_pack', 'phase_zero', 'splitk', 'cowmix', 'lovasz', 'bilinear',
            'sgd', 'ema', 'maxpool', 'nhwc', 'bce', 'cons', 'sq_']


def family(n):
    n = n.replace('(anonymous namespace)::', '')
    for k in FAMILIES:
        if k in n:
            return k
    return n[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, default=20)
    a = ap.parse_args()
    rows = [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in csv.DictReader(open(a.trace))]
    sgd = [s for n, s, e in rows if 'sgd_kernel' in n]
    t0 = sgd[-(a.steps + 1)]
    sel = [(n, s, e) for n, s, e in rows if s > t0]
    span = (max(e for _, _, e in sel) - min(s for _, s, _ in sel)) / 1e6
    fam = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in sel:
        f = family(n)
        fam[f][0] += 1
        fam[f][1] += (e - s) / 1e6
    tot = sum(v[1] for v in fam.values())
    print(f'steps {a.steps}: span {span / a.steps:.3f} ms/step, kernel time {tot / a.steps:.3f} ms/step')
    conv = sum(v[1] for k, v in fam.items() if k in ('igemm_glds', 'hconv3', 'igemm_kernel', 'wgrad_halo3', 'wgrad_glds',
                                                      'wgrad_kernel', 'wgrad_reduce', 'stem'))
    bn = sum(v[1] for k, v in fam.items() if k.startswith('bn_'))
    print(f'conv engine {conv / a.steps:.3f} ms/step, BN family {bn / a.steps:.3f} ms/step')
    for k, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f'{k:50s} {c / a.steps:7.1f}/step {t / a.steps:8.3f} ms/step')


if __name__ == '__main__':
    main()

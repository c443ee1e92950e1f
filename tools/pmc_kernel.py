"""Aggregate a rocprofv3 --pmc counter CSV per kernel (name prefix): dispatches and counter sums / per dispatch.

    rocprofv3 --pmc <counters> -d gpurun_out/pmcX -o p --output-format csv -- python <program>
    python tools/pmc_kernel.py gpurun_out/pmcX [name-substring ...]
"""
import collections
import csv
import glob
import sys


def main(d, subs):
    f = glob.glob(f'{d}/**/*counter_collection.csv', recursive=True)[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        e = disp.setdefault(int(r['Dispatch_Id']), {'name': r['Kernel_Name']})
        e[r['Counter_Name']] = e.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    agg = collections.defaultdict(collections.Counter)
    for e in disp.values():
        n = e['name'].replace('(anonymous namespace)::', '')
        key = (n[:n.find('(')] if '(' in n else n).replace('void ', '')[:90]
        if subs and not any(s in key for s in subs):
            continue
        agg[key]['dispatches'] += 1
        for k, v in e.items():
            if k != 'name':
                agg[key][k] += v
    for k, c in agg.items():
        n = c['dispatches']
        print(k, f'dispatches {n}')
        for ck in sorted(c):
            if ck != 'dispatches':
                print(f'   {ck:32s} {c[ck] / n:16.1f} per dispatch')
        w = c.get('SQ_WAVE_CYCLES', 0)
        if w:
            print('   shares of wave cycles: wait %.1f%% issue-stall %.1f%% active %.1f%% lds-issue %.1f%%' % tuple(
                100 * c.get(x, 0) / w for x in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY',
                                                 'SQ_WAIT_INST_LDS')))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])

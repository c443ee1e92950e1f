"""Per-kernel instruction / stall anatomy of ONE C2 training step from a rocprofv3 SQ-counter pass over
tools/pmc_step.py (the dispatches between its two marker launches):

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \\
        SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d gpurun_out/pmcs -o p --output-format csv -- python tools/pmc_step.py
    python tools/pmc_anatomy.py gpurun_out/pmcs > profiles/<name>.txt

Columns: launches, waves, VALU / SALU / VMEM instructions per wave, and the share of wave cycles parked in
s_waitcnt / barrier (wait%), stalled at issue (issue%) and issuing (act%); wc% = share of the step's wave cycles.
"""
import collections
import csv
import glob
import sys


def main(d):
    f = glob.glob(f'{d}/*counter_collection.csv')[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        e = disp.setdefault(int(r['Dispatch_Id']), {'name': r['Kernel_Name']})
        e[r['Counter_Name']] = e.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    ids = sorted(disp)
    marks = [i for i in ids if 'cast_kernel' in disp[i]['name']]
    lo, hi = marks[-2], marks[-1]
    agg = collections.defaultdict(collections.Counter)
    for i in ids:
        if lo < i < hi:
            n = disp[i]['name']
            n = n.replace('(anonymous namespace)::', '')
            key = (n[:n.find('(')] if '(' in n else n).replace('void ', '')[:78]
            c = agg[key]
            c['launches'] += 1
            for k, v in disp[i].items():
                if k != 'name':
                    c[k] += v
    tot = sum(c['SQ_WAVE_CYCLES'] for c in agg.values()) or 1
    print(f"{'kernel':78s} {'n':>4s} {'waves':>8s} {'VALU/w':>7s} {'SALU/w':>7s} {'VMEM/w':>6s} "
          f"{'wait%':>6s} {'issue%':>6s} {'act%':>5s} {'wc%':>5s}")
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES']):
        w = c['SQ_WAVES'] or 1
        wc = c['SQ_WAVE_CYCLES'] or 1
        print(f"{k:78s} {c['launches']:4d} {w:8.0f} {c['SQ_INSTS_VALU'] / w:7.0f} {c['SQ_INSTS_SALU'] / w:7.0f} "
              f"{c['SQ_INSTS_VMEM'] / w:6.0f} {100 * c['SQ_WAIT_ANY'] / wc:6.1f} {100 * c['SQ_WAIT_INST_ANY'] / wc:6.1f} "
              f"{100 * c['SQ_ACTIVE_INST_ANY'] / wc:5.1f} {100 * wc / tot:5.1f}")


if __name__ == '__main__':
    main(sys.argv[1])

"""Summarise tools/pmc_layer.sh output: per forced variant, the median over the conv-engine dispatches of each
counter, and the derived wave-state shares (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES).

    python tools/pmc_layer.py gpurun_out/pmcl > profiles/<name>.txt
"""
import collections
import csv
import glob
import os
import statistics
import sys

KERNELS = ('igemm_glds_kernel', 'igemm_kernel', 'wgrad_glds_kernel', 'wgrad_kernel')


def main(d):
    for vdir in sorted(glob.glob(os.path.join(d, 'v*')), key=lambda p: int(p.rsplit('v', 1)[1]) if p.rsplit('v', 1)[1].isdigit() else 0):
        if not os.path.isdir(vdir):
            continue
        files = glob.glob(os.path.join(vdir, '**', '*counter_collection.csv'), recursive=True)
        if not files:
            continue
        disp = collections.defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(files[0])):
            if not any(k in r['Kernel_Name'] for k in KERNELS):
                continue
            i = int(r['Dispatch_Id'])
            names[i] = r['Kernel_Name']
            disp[i][r['Counter_Name']] = disp[i].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
        if not disp:
            continue
        ids = sorted(disp)[1:] or sorted(disp)   # drop the first (warm-up) dispatch
        med = {c: statistics.median(disp[i].get(c, 0.0) for i in ids) for c in disp[ids[0]]}
        log = [l for l in open(vdir + '.log').read().splitlines() if l.startswith('v')]
        print(f'== {os.path.basename(vdir)}: {log[-1] if log else ""}')
        print(f'   kernel {names[ids[0]][:110]}')
        wc = med.get('SQ_WAVE_CYCLES')
        for c, v in sorted(med.items()):
            extra = f'  ({100 * v / wc:5.1f} % of wave cycles)' if wc and c.startswith(('SQ_WAIT', 'SQ_ACTIVE')) else ''
            print(f'   {c:32s} {v:16.0f}{extra}')
        if med.get('TCP_TCC_READ_REQ'):
            gui = med.get('GRBM_GUI_ACTIVE', 0) / 8 or 1
            print(f'   -> L2 read latency {med.get("TCP_TCC_READ_REQ_LATENCY", 0) / med["TCP_TCC_READ_REQ"]:.0f} cyc, '
                  f'TD busy {100 * med.get("TD_TD_BUSY", 0) / 256 / gui:.0f} %, TA busy '
                  f'{100 * med.get("TA_TA_BUSY", 0) / 256 / gui:.0f} %, TCP pending-stall '
                  f'{100 * med.get("TCP_PENDING_STALL_CYCLES", 0) / 256 / gui:.0f} % of {gui:.0f} cycles')


if __name__ == '__main__':
    main(sys.argv[1])

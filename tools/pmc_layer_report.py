"""Per-config PMC anatomy of one conv layer from the three rocprofv3 --pmc passes of tools/r6_pmc_layers.sh (each pass ran
tools/one_layer.py with the autotuner on, so every candidate config of the geometry was dispatched 6x): per config,
cycles per dispatch, MFMA utilisation, wave-cycle shares (waiting / issue-stalled / issuing), texture-path busy, L2
request latency and hit rate, LDS bank conflicts.

    python tools/pmc_layer_report.py gpurun_out/pmcl6_k3fwd > profiles/r6_pmc_layer_k3fwd.txt
"""
import collections
import csv
import glob
import sys

CUS, SIMDS, XCDS, CLK = 256, 1024, 8, 2.4e9


def load(d):
    f = glob.glob(f'{d}/**/*counter_collection.csv', recursive=True)[0]
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        e = disp.setdefault(int(r['Dispatch_Id']), {'name': r['Kernel_Name']})
        e[r['Counter_Name']] = e.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    agg = collections.defaultdict(collections.Counter)
    for e in disp.values():
        n = e['name'].replace('(anonymous namespace)::', '').replace('void ', '')
        key = n[:n.find('(')] if '(' in n else n
        if not any(s in key for s in ('igemm', 'hconv3', 'pw_kernel')):
            continue
        agg[key]['n'] += 1
        for k, v in e.items():
            if k != 'name':
                agg[key][k] += v
    return {k: {c: v / a['n'] for c, v in a.items() if c != 'n'} | {'n': a['n']} for k, a in agg.items()}


def main(base):
    p = [load(f'{base}_p{i}') for i in (1, 2, 3)]
    head = open(f'{base}_p1.log').read().strip().splitlines()
    print(f'# {base}: ' + ' | '.join(ln for ln in head if ln.startswith('v')))
    print('%-70s %7s %6s %6s %6s %6s %6s %6s %7s %6s %8s' % (
        'config', 'us', 'mfma', 'wait', 'istall', 'active', 'TA', 'TD', 'L2lat', 'L2hit', 'ldsconf'))
    rows = []
    for k in p[0]:
        a, b, c = p[0].get(k, {}), p[1].get(k, {}), p[2].get(k, {})
        cyc = c.get('GRBM_GUI_ACTIVE', b.get('GRBM_GUI_ACTIVE', 0)) / XCDS
        if not cyc:
            continue
        w = a.get('SQ_WAVE_CYCLES', 0) or 1
        mfma = a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (SIMDS * cyc)
        lat = b.get('TCP_TCC_READ_REQ_LATENCY', 0) / max(1.0, b.get('TCP_TCC_READ_REQ', 0))
        hit = c.get('TCC_HIT_sum', 0) / max(1.0, c.get('TCC_HIT_sum', 0) + c.get('TCC_MISS_sum', 0))
        conf = c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1.0, c.get('SQ_LDS_IDX_ACTIVE', 0))
        rows.append((cyc / CLK * 1e6, k, mfma, a.get('SQ_WAIT_ANY', 0) / w, a.get('SQ_WAIT_INST_ANY', 0) / w,
                     a.get('SQ_ACTIVE_INST_ANY', 0) / w, b.get('TA_TA_BUSY', 0) / (CUS * cyc),
                     b.get('TD_TD_BUSY', 0) / (CUS * cyc), lat, hit, conf))
    for r in sorted(rows):
        print('%-70s %7.1f %6.3f %6.2f %6.2f %6.2f %6.2f %6.2f %7.0f %6.2f %8.3f' % ((r[1][:70],) + (r[0],) + r[2:]))
    print('(us: GRBM_GUI_ACTIVE / 8 XCDs at 2.4 GHz per dispatch, serialised by the PMC collection, so longer than the '
          'tuned launch; mfma = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles); wait / istall / active = shares of '
          'SQ_WAVE_CYCLES; TA / TD = busy per CU; L2lat = TCP->TCC read latency in cycles; ldsconf = bank-conflict '
          'cycles / LDS-array cycles)')


if __name__ == '__main__':
    main(sys.argv[1])

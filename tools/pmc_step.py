"""HBM traffic of the conv engine over ONE C2 training step, from rocprofv3 PMC counters.

Run mode: the bench.py workload (UNet-R50 512x512 bs16 bf16 semi-supervised step), 3 warm-up steps (the
per-geometry autotune runs there), then one step bracketed by two marker launches (a 256-thread
ssseg_cast of 8 floats) so the dispatches of exactly that step can be cut out of the counter trace:

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- python tools/pmc_step.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- python tools/pmc_step.py

    rocprofv3 --kernel-trace -d gpurun_out/pmc_t -o t --output-format csv -- python tools/pmc_step.py

Parse mode (CPU):  python tools/pmc_step.py --parse gpurun_out/pmc_f gpurun_out/pmc_w [--trace gpurun_out/pmc_t]
                   > profiles/<name>.json
With --trace, every kernel family of the step (not only the conv engine) is listed with its bytes, device time
and achieved HBM bandwidth (corrected bytes / time).

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters).  Per MI355X_MICROARCH.md §HBM, gfx950's
FETCH_SIZE reports half of the bytes of wide (16 B/lane) streaming reads, which is how every conv-engine
kernel reads (buffer_load ... lds dwordx4 / global_load_dwordx4), so the corrected read traffic is 2x the
counter; WRITE_SIZE is exact for 16-byte stores.  Both are reported raw and corrected.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONV_KERNELS = ('igemm_kernel', 'igemm_glds_kernel', 'hconv3_kernel', 'hconv3s_kernel', 'pw_kernel', 'wgrad_halo3_kernel', 'wgrad_kernel',
                'wgrad_glds_kernel', 'wgrad_reduce_kernel',
                'wgrad_reduce_wide_kernel', 'splitk_finalize_kernel', 'slab_finalize_kernel', 'phase_zero_kernel')


def run():
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'semi-supervised_semantic_segmentation_amd')]
    import torch
    import bench
    import train
    from ssseg import native as N
    from ssseg import nn as snn
    dev = torch.device('cuda', 0)
    snn.set_compute_dtype(torch.bfloat16)
    model, teacher, opt, cfg = bench.build(16, 512, dev)
    data = bench.synthetic_batches(2, 16, 512, dev, 0)
    model.train()
    opt.zero_grad()
    for s in range(4):
        img, mask, ua, ub = data[s % 2]
        if s == 3:
            torch.cuda.synchronize()
            src = torch.zeros(8, device=dev)
            dst = torch.empty(8, dtype=torch.bfloat16, device=dev)
            N.call('ssseg_cast', N.dev_ptr(src), N.dev_ptr(dst), 8, N.F32, N.BF16, N.stream())
        train.train_step(model, teacher, opt, img, mask, ua, ub, 30, s, cfg)
    N.call('ssseg_cast', N.dev_ptr(src), N.dev_ptr(dst), 8, N.F32, N.BF16, N.stream())
    torch.cuda.synchronize()
    print('pmc_step: done')


def _rows(d):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no counter_collection.csv under {d}')
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    key = 'Dispatch_Id' if 'Dispatch_Id' in rows[0] else 'Correlation_Id'
    rows.sort(key=lambda r: int(r[key]))
    return rows


def _rows_named(d, pattern):
    files = glob.glob(os.path.join(d, '**', pattern), recursive=True)
    if not files:
        raise SystemExit(f'no {pattern} under {d}')
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    key = 'Dispatch_Id' if 'Dispatch_Id' in rows[0] else 'Correlation_Id'
    rows.sort(key=lambda r: int(r[key]))
    return rows


def _family(name):
    name = name.replace('(anonymous namespace)::', '').replace('void ', '').strip()
    if not name.startswith('at::'):
        name = name.split('(')[0].split('<')[0]
    else:
        name = name.split('(')[0]
    for k in CONV_KERNELS:
        if k in name:
            return k
    return name[:90]


def _step_rows(rows):
    marks = [i for i, r in enumerate(rows) if 'cast_kernel' in r['Kernel_Name']
             and int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0) <= 256]
    if len(marks) < 2:
        raise SystemExit('markers not found')
    return rows[marks[-2] + 1:marks[-1]]


def _all_sums(d):
    per = collections.defaultdict(lambda: [0.0, 0])
    for r in _step_rows(_rows(d)):
        fam = _family(r['Kernel_Name'])
        per[fam][0] += float(r['Counter_Value'])
        per[fam][1] += 1
    return per


def _trace_sums(d):
    per = collections.defaultdict(lambda: [0.0, 0])
    for r in _step_rows(_rows_named(d, '*kernel_trace.csv')):
        fam = _family(r['Kernel_Name'])
        per[fam][0] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-3   # us
        per[fam][1] += 1
    return per


def _step_sums(d):
    rows = _rows(d)
    marks = [i for i, r in enumerate(rows) if 'cast_kernel' in r['Kernel_Name'] and int(r.get('Grid_Size', 0)) <= 256]
    if len(marks) < 2:
        raise SystemExit(f'{d}: markers not found')
    a, b = marks[-2], marks[-1]
    per = collections.defaultdict(lambda: [0.0, 0])
    total, launches = 0.0, 0
    for r in rows[a + 1:b]:
        name = r['Kernel_Name']
        fam = next((k for k in CONV_KERNELS if k in name), None)
        if fam is None:
            continue
        v = float(r['Counter_Value'])
        per[fam][0] += v
        per[fam][1] += 1
        total += v
        launches += 1
    return total, launches, {k: v for k, v in per.items()}, rows[0].get('Counter_Name', '?')


def parse(fetch_dir, write_dir, trace_dir=None):
    f_kb, n_f, f_per, _ = _step_sums(fetch_dir)
    w_kb, n_w, w_per, _ = _step_sums(write_dir)
    fetch, write = f_kb * 1024.0, w_kb * 1024.0
    out = {
        'what': 'conv-engine HBM traffic of one C2 training step (UNet-R50 512x512 bs16 bf16), rocprofv3 PMC',
        'kernel_launches': n_f,
        'fetch_bytes_raw': fetch, 'fetch_bytes_corrected_x2': 2 * fetch, 'write_bytes': write,
        'traffic_bytes': 2 * fetch + write,
        'per_kernel_family': {k: {'fetch_kb_raw': f_per.get(k, [0, 0])[0], 'write_kb': w_per.get(k, [0, 0])[0],
                                  'launches': f_per.get(k, [0, 0])[1]} for k in sorted(set(f_per) | set(w_per))},
        'correction': 'FETCH_SIZE x2 for 16 B/lane streaming reads on gfx950 (MI355X_MICROARCH.md §HBM)',
    }
    if trace_dir:
        fa, wa, ta = _all_sums(fetch_dir), _all_sums(write_dir), _trace_sums(trace_dir)
        fams = []
        for k in sorted(ta, key=lambda k: -ta[k][0]):
            us = ta[k][0]
            byt = 2 * fa.get(k, [0, 0])[0] * 1024 + wa.get(k, [0, 0])[0] * 1024
            fams.append({'kernel': k, 'launches': ta[k][1], 'time_us': round(us, 1),
                         'fetch_bytes_corrected_x2': 2 * fa.get(k, [0, 0])[0] * 1024,
                         'write_bytes': wa.get(k, [0, 0])[0] * 1024,
                         'achieved_GBps': round(byt / (us * 1e3), 1) if us > 0 else None})
        out['all_kernels_step_time_us'] = round(sum(v[0] for v in ta.values()), 1)
        out['all_kernels'] = fams
    print(json.dumps(out, indent=1))


# MFMA 16x16x32 (bf16 / f16): 16 x 16 x 32 multiply-adds = 16384 flop per instruction, 16 cycles of one SIMD
# (MI355X_MICROARCH.md, instruction table); SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over the SIMDs,
# GRBM_GUI_ACTIVE the GPU-busy cycles summed over the 8 XCDs (so / 8 = elapsed cycles), 256 CUs x 4 SIMDs
SIMDS = 1024


def parse_mfma(mfma_dir, trace_dir, flops_json=None):
    """MFMA utilisation per kernel family of one C2 step: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8),
    i.e. the fraction of SIMD-cycles the matrix cores were busy while the family's kernels ran, next to the
    family's device time; with flops_json (tools/layer_report.py --json) the conv families' flop-derived fraction of
    the 2.5 PF dense peak too."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    rows = _rows(mfma_dir)
    key = 'Dispatch_Id' if 'Dispatch_Id' in rows[0] else 'Correlation_Id'
    # several counters per dispatch (one row each): the step lies between the last two marker DISPATCHES
    marks = sorted({int(r[key]) for r in rows if 'cast_kernel' in r['Kernel_Name']
                    and int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0) <= 256})
    if len(marks) < 2:
        raise SystemExit('markers not found')
    lo, hi = marks[-2], marks[-1]
    for r in (r for r in rows if lo < int(r[key]) < hi):
        fam = _family(r['Kernel_Name'])
        per[fam][r['Counter_Name']] += float(r['Counter_Value'])
    ta = _trace_sums(trace_dir) if trace_dir else {}
    fams = []
    tot = collections.defaultdict(float)
    conv = collections.defaultdict(float)
    for k in sorted(per, key=lambda k: -per[k].get('GRBM_GUI_ACTIVE', 0)):
        c = per[k]
        busy, act = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0), c.get('GRBM_GUI_ACTIVE', 0.0)
        row = {'kernel': k, 'mfma_busy_cycles': busy, 'gpu_active_cycles_sum8': act,
               'sq_busy_cycles': c.get('SQ_BUSY_CYCLES', 0.0),
               'mfma_util': round(busy / (SIMDS * act / 8), 4) if act else None,
               'implied_mfma_instructions': round(busy / 16)}
        if k in ta:
            row['time_us'] = round(ta[k][0], 1)
            row['launches'] = ta[k][1]
            row['implied_clock_GHz'] = round(act / 8 / (ta[k][0] * 1e3), 3) if ta[k][0] else None
        fams.append(row)
        for key in ('mfma_busy_cycles', 'gpu_active_cycles_sum8'):
            tot[key] += row[key]
            if k in CONV_KERNELS:
                conv[key] += row[key]
    out = {
        'what': 'MFMA utilisation per kernel family of one C2 training step (UNet-R50 512x512 bs16 bf16), rocprofv3 '
                '--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (one pass)',
        'definition': 'mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); '
                      'implied_mfma_instructions = busy cycles / 16 (16x16x32 bf16: 16 cycles per SIMD)',
        'conv_engine': {'mfma_util': round(conv['mfma_busy_cycles'] / (SIMDS * conv['gpu_active_cycles_sum8'] / 8), 4)
                        if conv['gpu_active_cycles_sum8'] else None,
                        'implied_gflop': round(conv['mfma_busy_cycles'] / 16 * 16384 / 1e9, 1),
                        'time_us': round(sum(ta[k][0] for k in ta if k in CONV_KERNELS), 1) if ta else None},
        'whole_step': {'mfma_util': round(tot['mfma_busy_cycles'] / (SIMDS * tot['gpu_active_cycles_sum8'] / 8), 4)
                       if tot['gpu_active_cycles_sum8'] else None},
        'families': fams,
    }
    ce = out['conv_engine']
    if ce['time_us']:
        ce['implied_TFLOPs'] = round(ce['implied_gflop'] * 1e9 / (ce['time_us'] * 1e-6) / 1e12, 1)
        ce['implied_frac_of_2p5PF'] = round(ce['implied_TFLOPs'] / 2500.0, 4)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--parse', nargs=2, metavar=('FETCH_DIR', 'WRITE_DIR'))
    ap.add_argument('--mfma', default=None, metavar='MFMA_DIR')
    ap.add_argument('--trace', default=None)
    a = ap.parse_args()
    if a.mfma:
        parse_mfma(a.mfma, a.trace)
    elif a.parse:
        parse(*a.parse, trace_dir=a.trace)
    else:
        run()

"""Do two HIP streams run concurrently on MI355X?  Stream A gets a long chain of large GEMMs, stream B a chain of small
ones; B waits for an event recorded after A's first GEMM (case 'event'), waits for nothing ('free'), or runs on a
high-priority stream ('prio').  Run under rocprofv3 --kernel-trace and read the trace with --analyze: when B's first
kernel starts relative to A's chain.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/so -o so -- python tools/stream_overlap.py
    python tools/stream_overlap.py --analyze gpurun_out/so/so_kernel_trace.csv
"""
import argparse
import csv
import sys


def run():
    import torch
    dev = torch.device('cuda:0')
    a_big = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    b_small = torch.randn(512, 512, device=dev, dtype=torch.bfloat16)
    main = torch.cuda.current_stream()
    for case in ('event', 'free', 'prio', 'event', 'free', 'prio'):
        side = torch.cuda.Stream(priority=-1) if case == 'prio' else torch.cuda.Stream()
        torch.cuda.synchronize()
        # marker kernels: a fill names the case in the trace (its size encodes the case)
        torch.empty({'event': 1, 'free': 2, 'prio': 3}[case] * 1024 * 1024, device=dev).fill_(0)
        torch.cuda.synchronize()
        x = a_big @ a_big
        ev = torch.cuda.Event()
        ev.record(main)
        for _ in range(40):
            x = a_big @ a_big
        if case != 'free':
            side.wait_event(ev)
        with torch.cuda.stream(side):
            y = b_small
            for _ in range(40):
                y = (y @ b_small) * 1e-3
        torch.cuda.synchronize()
        print(case, float(x[0, 0]), float(y[0, 0]), flush=True)


def timing():
    """Without a profiler: wall time of chain A alone, chain B alone and both issued on two streams (B free)."""
    import time
    import torch
    dev = torch.device('cuda:0')
    a_big = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    b_small = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def chain_a():
        x = a_big
        for _ in range(40):
            x = a_big @ a_big
        return x

    def chain_b():
        with torch.cuda.stream(side):
            y = b_small
            for _ in range(400):
                y = (y @ b_small) * 1e-3
        return y

    def clock(fn):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2e7))   # hold the device while the host enqueues
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for rep in range(3):
        ta = clock(chain_a)
        tb = clock(lambda: (side.wait_stream(main), chain_b()))
        tab = clock(lambda: (side.wait_stream(main), chain_a(), chain_b()))
        print(f'rep {rep}: A {ta:.2f} ms, B {tb:.2f} ms, A+B on two streams {tab:.2f} ms '
              f'(serial would be {ta + tb:.2f})', flush=True)


def analyze(path):
    rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r['Queue_Id'],
                   int(r['Grid_Size_X'])) for r in csv.DictReader(open(path)))
    marks = [i for i, r in enumerate(rows) if 'fill' in r[2].lower() or 'FillFunctor' in r[2]]
    for mi, i in enumerate(marks):
        j = marks[mi + 1] if mi + 1 < len(marks) else len(rows)
        seg = rows[i + 1:j]
        if not seg:
            continue
        t0 = seg[0][0]
        qs = sorted({r[3] for r in seg})
        print(f'case marker grid {rows[i][4]}: queues {qs}')
        for q in qs:
            ks = [r for r in seg if r[3] == q]
            print(f'   q{q}: {len(ks)} kernels, first start {(ks[0][0] - t0) / 1e3:8.1f} us, last end '
                  f'{(ks[-1][1] - t0) / 1e3:8.1f} us, {ks[0][2][:40]}')


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--analyze')
    ap.add_argument('--timing', action='store_true')
    a = ap.parse_args()
    if a.timing:
        timing()
    elif a.analyze:
        analyze(a.analyze)
    else:
        run()
        sys.exit(0)

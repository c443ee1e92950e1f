"""Per-kernel summary (pct, total_us, calls, avg_us, name) from a rocprofv3 rocpd database
(`rocprofv3 --kernel-trace --stats -d DIR -o run -- ...` writes DIR/run_results.db) or from the csv kernel
trace (`--output-format csv`: DIR/run_kernel_trace.csv).

    python tools/prof_summary.py DB [--tail-ms MS] [--header TEXT] > profiles/rN_kernel_stats.tsv

--tail-ms keeps only dispatches that start in the last MS milliseconds of the trace (the timed steps;
drops warm-up and one-time autotuning launches).
"""
import argparse
import sqlite3


def summary_csv(path, tail_ms=None):
    """Same summary from a rocprofv3 `--output-format csv` kernel trace (DIR/<o>_kernel_trace.csv)."""
    import csv
    with open(path) as fh:
        rows = [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in csv.DictReader(fh)]
    t0 = max(e for _, _, e in rows) - int(tail_ms * 1e6) if tail_ms else 0
    agg = {}
    for name, s, e in rows:
        if s >= t0:
            n, ns = agg.get(name, (0, 0))
            agg[name] = (n + 1, ns + e - s)
    total = sum(ns for _, ns in agg.values()) or 1
    out = [(100.0 * ns / total, ns / 1e3, n, ns / 1e3 / n, name) for name, (n, ns) in agg.items()]
    return sorted(out, key=lambda r: -r[1])


def summary(db, tail_ms=None):
    if db.endswith('.csv'):
        return summary_csv(db, tail_ms)
    c = sqlite3.connect(db)
    t0 = 0
    if tail_ms:
        (tmax,) = c.execute('select max(end) from rocpd_kernel_dispatch').fetchone()
        t0 = tmax - int(tail_ms * 1e6)
    rows = c.execute("""
        select s.kernel_name, count(*), sum(d.end - d.start)
        from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
        where d.start >= ? group by s.kernel_name order by 3 desc""", (t0,)).fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(100.0 * ns / total, ns / 1e3, n, ns / 1e3 / n, name) for name, n, ns in rows]


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--tail-ms', type=float, default=None)
    ap.add_argument('--header', default=None)
    a = ap.parse_args()
    if a.header:
        print('# ' + a.header)
    print('# columns: pct, total_us, calls, avg_us, kernel')
    for pct, tot, n, avg, name in summary(a.db, a.tail_ms):
        print(f'{pct:7.3f}\t{tot:12.1f}\t{n:6d}\t{avg:10.2f}\t{name}')

"""Per-kernel summary (pct, total_us, calls, avg_us, name) from a rocprofv3 rocpd database
(`rocprofv3 --kernel-trace --stats -d DIR -o run -- ...` writes DIR/run_results.db).

    python tools/prof_summary.py gpurun_out/prof3/run_results.db [header comment] > profiles/rN_kernel_stats.tsv
"""
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    rows = c.execute("""
        select s.kernel_name, count(*), sum(d.end - d.start)
        from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
        group by s.kernel_name order by 3 desc""").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(100.0 * ns / total, ns / 1e3, n, ns / 1e3 / n, name) for name, n, ns in rows]


if __name__ == '__main__':
    if len(sys.argv) > 2:
        print('# ' + sys.argv[2])
    print('# columns: pct, total_us, calls, avg_us, kernel')
    for pct, tot, n, avg, name in summary(sys.argv[1]):
        print(f'{pct:7.3f}\t{tot:12.1f}\t{n:6d}\t{avg:10.2f}\t{name}')

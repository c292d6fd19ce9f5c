"""Summarise a rocprofv3 rocpd database (kernel trace) into a CSV like
`rocprofv3 --stats`: per kernel name calls, total/avg/min/max ns, percentage.

    python tools/rocpd_summary.py gpurun_out/prof_r01/run_results.db > profiles/r01/kernel_stats.csv
"""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage")
    for name, n, s, a, mn, mx in rows:
        print(f'"{name}",{n},{s},{a:.1f},{mn},{mx},{100.0 * s / tot:.3f}')


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise a rocprofv3 rocpd database (``-d DIR -o run`` -> DIR/run_results.db).

    python tools/prof_summary.py stats gpurun_out/prof_r01/trace/run_results.db > profiles/r01_kernel_stats.csv
    python tools/prof_summary.py pmc   gpurun_out/prof_r01/fetch/run_results.db > profiles/r01_pmc_fetch.csv

``stats``: one row per kernel name — calls, total/avg/min/max duration (ns) and share of GPU time,
the same figures rocprofv3 --stats writes to kernel_stats.csv.
``pmc``: one row per (kernel, counter) — dispatches and the mean/min/max counter value per dispatch.
"""
import csv
import re
import sqlite3
import sys


def short(name):
    m = re.match(r"(?:void )?(?:cacto::)?([\w:<>\-, ]+?)\(", name)
    return m.group(1) if m else name[:80]


def stats(db):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                       "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "percent"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([short(name), n, int(tot), round(avg, 1), int(mn), int(mx), round(100.0 * tot / total, 2)])


def pmc(db):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select kernel_name, counter_name, count(*), avg(value), min(value), max(value), avg(duration) "
                       "from counters_collection group by kernel_name, counter_name").fetchall()
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "counter", "dispatches", "mean", "min", "max", "avg_duration_ns"])
    for name, ctr, n, avg, mn, mx, dur in rows:
        w.writerow([short(name), ctr, n, round(avg, 3), round(mn, 3), round(mx, 3), round(dur, 1)])


if __name__ == "__main__":
    {"stats": stats, "pmc": pmc}[sys.argv[1]](sys.argv[2])

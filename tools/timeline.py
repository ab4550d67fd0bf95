"""Print a window of the kernel timeline from a rocprofv3 rocpd database (start/end relative, us).

    python tools/timeline.py DB [filter-substring] [count] [skip-from-end]
"""
import re
import sqlite3
import sys

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "k_"
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 24
back = int(sys.argv[4]) if len(sys.argv) > 4 else 200
cur = sqlite3.connect(db).cursor()
rows = [r for r in cur.execute("select name, start, end, queue_id, stream_id from kernels order by start").fetchall()
        if flt in r[0]]
sel = rows[-back:-back + cnt] if back > cnt else rows[-cnt:]
t0 = sel[0][1]
for name, s, e, q, stm in sel:
    m = re.match(r"(?:void )?(?:cacto::)?([\w:<>\-, ]+?)\(", name)
    print("%9.1f %9.1f %7.1f  q%-3s s%-3s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, stm,
                                              m.group(1) if m else name[:60]))
